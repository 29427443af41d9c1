/* ORACLE / TEST INFRASTRUCTURE: C twin of oracle/coders_ref.py's rANS restatement
 * (compressai==1.2.4 BufferedRansEncoder / RansDecoder: rans64, 16-bit precision, 4-bit bypass;
 * called from the reference at model/compression.py:199-206,255-262 and utils/ckbd.py:76-115).
 * Used only by the CPU baseline leg of bench.py and by tests; the product coder is
 * rdeic_amd/csrc/coders.cpp. Checked against the Python restatement and the golden bitstreams. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PREC 16
#define BYP 4
#define BYP_MAX ((1 << BYP) - 1)
#define RL (1ull << 31)

typedef struct { uint32_t start, freq; int bypass; } sym_t;

/* Encodes n symbols; writes the stream into out (cap bytes). Returns bytes written or -1. */
int64_t oracle_rans_encode(const int32_t *symbols, const int32_t *indexes, int64_t n,
                           const int32_t *cdf, int64_t cdf_stride, const int32_t *lens,
                           const int32_t *offs, uint8_t *out, int64_t cap) {
  int64_t cap_syms = n * 4 + 64, ns = 0;
  sym_t *s = (sym_t *)malloc(sizeof(sym_t) * cap_syms);
  if (!s) return -1;
  for (int64_t i = 0; i < n; i++) {
    const int32_t ci = indexes[i];
    const int32_t *c = cdf + ci * cdf_stride;
    const int32_t maxv = lens[ci] - 2;
    int32_t v = symbols[i] - offs[ci];
    uint32_t raw = 0;
    if (v < 0) { raw = (uint32_t)(-2 * v - 1); v = maxv; }
    else if (v >= maxv) { raw = (uint32_t)(2 * (v - maxv)); v = maxv; }
    if (ns + 24 > cap_syms) { cap_syms *= 2; s = (sym_t *)realloc(s, sizeof(sym_t) * cap_syms); }
    s[ns++] = (sym_t){(uint32_t)c[v] & 0xFFFF, (uint32_t)(c[v + 1] - c[v]) & 0xFFFF, 0};
    if (v == maxv) {
      int nb = 0;
      while (nb < 8 && (raw >> (nb * BYP)) != 0) nb++;
      int w = nb;
      while (w >= BYP_MAX) { s[ns++] = (sym_t){BYP_MAX, BYP_MAX + 1, 1}; w -= BYP_MAX; }
      s[ns++] = (sym_t){(uint32_t)w, (uint32_t)w + 1, 1};
      for (int j = 0; j < nb; j++) {
        uint32_t nib = (raw >> (j * BYP)) & BYP_MAX;
        s[ns++] = (sym_t){nib, nib + 1, 1};
      }
    }
  }
  /* encode in reverse; words collected back to front */
  int64_t wcap = ns + 4, nw = 0;
  uint32_t *words = (uint32_t *)malloc(sizeof(uint32_t) * wcap);
  uint64_t x = RL;
  for (int64_t i = ns - 1; i >= 0; i--) {
    uint64_t freq = s[i].bypass ? (1u << (PREC - BYP)) : s[i].freq;
    uint64_t xmax = ((RL >> PREC) << 32) * freq;
    if (x >= xmax) { words[nw++] = (uint32_t)x; x >>= 32; }
    if (s[i].bypass) x = (x << BYP) | s[i].start;
    else x = ((x / freq) << PREC) + (x % freq) + s[i].start;
  }
  words[nw++] = (uint32_t)(x >> 32);
  words[nw++] = (uint32_t)x;
  free(s);
  if (nw * 4 > cap) { free(words); return -1; }
  for (int64_t i = 0; i < nw; i++) memcpy(out + 4 * i, &words[nw - 1 - i], 4);
  free(words);
  return nw * 4;
}

typedef struct { uint64_t x; const uint32_t *p, *end; } dec_t;

int64_t oracle_rans_dec_state_size(void) { return sizeof(dec_t); }

int oracle_rans_dec_init(void *st, const uint8_t *data, int64_t nbytes) {
  dec_t *d = (dec_t *)st;
  if (nbytes % 4 || nbytes < 8) return -1;
  d->p = (const uint32_t *)data;
  d->end = d->p + nbytes / 4;
  d->x = (uint64_t)d->p[0] | ((uint64_t)d->p[1] << 32);
  d->p += 2;
  return 0;
}

static int rd(dec_t *d, uint32_t *w) {
  if (d->p >= d->end) return -1;
  *w = *d->p++;
  return 0;
}

static int get_bits(dec_t *d, int n, uint32_t *v) {
  *v = (uint32_t)(d->x & ((1u << n) - 1));
  d->x >>= n;
  if (d->x < RL) { uint32_t w; if (rd(d, &w)) return -1; d->x = (d->x << 32) | w; }
  return 0;
}

/* Decodes n symbols continuing the stream in st. Returns 0, or -1 on an exhausted stream. */
int oracle_rans_decode(void *st, const int32_t *indexes, int64_t n, const int32_t *cdf,
                       int64_t cdf_stride, const int32_t *lens, const int32_t *offs, int32_t *out) {
  dec_t *d = (dec_t *)st;
  const uint64_t mask = (1u << PREC) - 1;
  for (int64_t i = 0; i < n; i++) {
    const int32_t ci = indexes[i];
    const int32_t *c = cdf + ci * cdf_stride;
    const int32_t maxv = lens[ci] - 2;
    uint32_t cum = (uint32_t)(d->x & mask);
    int32_t s = 0;
    while ((uint32_t)c[s + 1] <= cum) s++;
    uint64_t start = (uint32_t)c[s], freq = (uint32_t)(c[s + 1] - c[s]);
    uint64_t x = freq * (d->x >> PREC) + (d->x & mask) - start;
    if (x < RL) { uint32_t w; if (rd(d, &w)) return -1; x = (x << 32) | w; }
    d->x = x;
    int32_t v = s;
    if (v == maxv) {
      uint32_t b, nb;
      if (get_bits(d, BYP, &b)) return -1;
      nb = b;
      while (b == BYP_MAX) { if (get_bits(d, BYP, &b)) return -1; nb += b; }
      uint32_t raw = 0;
      for (uint32_t j = 0; j < nb; j++) {
        if (get_bits(d, BYP, &b)) return -1;
        raw |= b << (j * BYP);
      }
      v = (int32_t)(raw >> 1);
      if (raw & 1) v = -v - 1;
      else v += maxv;
    }
    out[i] = v + offs[ci];
  }
  return 0;
}
