// Host entropy coders of the RDEIC bitstream, bit-compatible with the reference's
// third-party natives (absent from the reference tree, restated from their published
// algorithms; see DESIGN.md "Oracle"):
//
//  * compressai 1.2.4 rANS  — BufferedRansEncoder::encode_with_indexes / flush and
//    RansDecoder::set_stream / decode_stream (called at model/compression.py:166,205-206,
//    230-231 and utils/ckbd.py:103,112): ryg_rans 64-bit state, L = 2^31, 32-bit words,
//    16-bit quantised CDFs, out-of-range values escaped through 4-bit "bypass" symbols.
//  * compressai pmf_to_quantized_cdf (GaussianConditional.update, compression.py:275-280).
//  * torchac 0.9.3 — 32-bit low/high binary arithmetic coder with pending (E3) bits, MSB-first
//    bit packing, for the uniform 16384-symbol hyper-latent CDF (utils/ckbd.py:117-141).
//
// Differences by design: every export is reentrant (no global state) so images are coded on
// independent host threads, and decoders bound every read — a truncated or corrupt stream
// returns -EBADMSG instead of reading past the buffer (the reference treats any decompress
// exception as a decode failure, experiments/run_robustness.py:277-297).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cmath>
#include <new>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../../include/rdeic_hip.h"

#define RDEIC_OK 0
#define RDEIC_EINVAL (-22)
#define RDEIC_ENOSPC (-28)
#define RDEIC_EBADMSG (-74)

namespace {

constexpr int kPrecision = 16;
constexpr uint32_t kBypassBits = 4;
constexpr uint32_t kBypassMax = (1u << kBypassBits) - 1;
constexpr uint64_t kRansL = 1ull << 31;

struct RansSym {
  uint16_t start;
  uint16_t range;
  bool bypass;
};

// ---- encoder --------------------------------------------------------------
int rans_encode_impl(const int32_t* sym, const int32_t* idx, size_t n, const int32_t* cdf, int32_t cdf_ld,
                     const int32_t* cdf_len, const int32_t* offset, int32_t levels, uint8_t* out, size_t cap,
                     size_t* out_len, std::vector<RansSym>& syms, std::vector<uint32_t>& words) {
  syms.clear();
  syms.reserve(n + 16);
  for (size_t i = 0; i < n; ++i) {
    const int32_t ci = idx[i];
    if (ci < 0 || ci >= levels) return RDEIC_EINVAL;
    const int32_t* row = cdf + (size_t)ci * cdf_ld;
    const int32_t max_value = cdf_len[ci] - 2;
    if (max_value < 0 || max_value + 1 >= cdf_ld) return RDEIC_EINVAL;
    int32_t value = sym[i] - offset[ci];
    uint32_t raw = 0;
    if (value < 0) {
      raw = (uint32_t)(-2 * (int64_t)value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw = (uint32_t)(2 * (int64_t)(value - max_value));
      value = max_value;
    }
    syms.push_back({(uint16_t)row[value], (uint16_t)(row[value + 1] - row[value]), false});
    if (value == max_value) {
      int32_t nb = 0;
      while (nb < 8 && (raw >> (nb * kBypassBits)) != 0) ++nb;
      int32_t v = nb;
      while (v >= (int32_t)kBypassMax) {
        syms.push_back({(uint16_t)kBypassMax, (uint16_t)(kBypassMax + 1), true});
        v -= kBypassMax;
      }
      syms.push_back({(uint16_t)v, (uint16_t)(v + 1), true});
      for (int32_t j = 0; j < nb; ++j) {
        uint32_t nib = (raw >> (j * kBypassBits)) & kBypassMax;
        syms.push_back({(uint16_t)nib, (uint16_t)(nib + 1), true});
      }
    }
  }
  // flush: encode in reverse into a word buffer filled from the end
  words.assign(syms.size() + 2, 0u);
  size_t wp = words.size();
  uint64_t x = kRansL;
  for (size_t k = syms.size(); k-- > 0;) {
    const RansSym& s = syms[k];
    if (!s.bypass) {
      const uint64_t freq = s.range;
      const uint64_t x_max = ((kRansL >> kPrecision) << 32) * freq;
      if (x >= x_max) {
        words[--wp] = (uint32_t)x;
        x >>= 32;
      }
      x = ((x / freq) << kPrecision) + (x % freq) + s.start;
    } else {
      const uint64_t freq = 1ull << (kPrecision - kBypassBits);
      const uint64_t x_max = ((kRansL >> kPrecision) << 32) * freq;
      if (x >= x_max) {
        words[--wp] = (uint32_t)x;
        x >>= 32;
      }
      x = (x << kBypassBits) | s.start;
    }
  }
  words[--wp] = (uint32_t)(x >> 32);
  words[--wp] = (uint32_t)x;
  // after the two decrements, words[wp] = low half, words[wp+1] = high half
  const size_t nbytes = (words.size() - wp) * 4;
  *out_len = nbytes;
  if (nbytes > cap) return RDEIC_ENOSPC;
  memcpy(out, words.data() + wp, nbytes);
  return RDEIC_OK;
}

// ---- encoder on precomputed symbol tables ------------------------------------
// One entry per (cdf row, value): the rANS put x' = (x / freq) << 16 + x % freq + start done
// without a 64-bit division, as q = mulhi(x, rcp) >> shift (Alverson's exact reciprocal, the
// form of ryg_rans' Rans64EncSymbolInit), x' = x + bias + q * (2^16 - freq). For freq = 1 the
// reciprocal is 2^64 - 1 with shift 0 (q = x - 1) and bias = start + 2^16 - 1. Exact for every
// x < 2^63 (the encoder never holds more: x < freq << 47 before each put), so the bytes equal
// rans_encode_impl's; tests/test_coders.py checks both the quotients and whole streams.
struct EncSym {
  uint64_t rcp;
  uint32_t bias;
  uint16_t freq;   // 1..65535 (a zero-width bin is never coded)
  uint8_t shift;
  uint8_t pad;
};

struct EncTables {
  std::vector<EncSym> sym;         // row ci's entries at row_off[ci] .. row_off[ci] + cdf_len[ci] - 2
  std::vector<int32_t> row_off, max_value, offset;
  int32_t levels = 0;
};

EncSym make_enc_sym(uint32_t start, uint32_t freq) {
  EncSym s{};
  s.freq = (uint16_t)freq;
  if (freq < 2) {
    s.rcp = ~0ull;
    s.shift = 0;
    s.bias = start + (1u << kPrecision) - 1;
  } else {
    uint32_t sh = 0;
    while (freq > (1u << sh)) ++sh;  // ceil(log2 freq)
    const unsigned __int128 num = ((unsigned __int128)1 << (sh + 63)) + (freq - 1);
    s.rcp = (uint64_t)(num / freq);
    s.shift = (uint8_t)(sh - 1);
    s.bias = start;
  }
  return s;
}

inline uint64_t enc_quot(uint64_t x, const EncSym& s) {
  return (uint64_t)(((unsigned __int128)x * s.rcp) >> 64) >> s.shift;
}

// Words are written from the end of a per-thread buffer; it grows (keeping the tail) if a
// stream ever needs more than the initial estimate.
struct WordSink {
  std::vector<uint32_t>& buf;
  size_t wp;
  explicit WordSink(std::vector<uint32_t>& b) : buf(b), wp(b.size()) {}
  void emit(uint32_t w) {
    if (wp == 0) grow();
    buf[--wp] = w;
  }
  void grow() {
    const size_t old = buf.size(), add = std::max<size_t>(old, 1024);
    std::vector<uint32_t> nb(old + add);
    memcpy(nb.data() + add, buf.data(), old * sizeof(uint32_t));
    buf.swap(nb);
    wp += add;
  }
};

inline void enc_put(uint64_t& x, WordSink& ws, const EncSym& s) {
  if ((x >> 47) >= s.freq) {  // x >= x_max = ((L >> 16) << 32) * freq = freq << 47
    ws.emit((uint32_t)x);
    x >>= 32;
  }
  x = x + s.bias + enc_quot(x, s) * ((1u << kPrecision) - s.freq);
}

inline void enc_put_bits(uint64_t& x, WordSink& ws, uint32_t v) {
  if ((x >> 59) != 0) {  // bypass freq 2^12: x_max = 2^12 << 47
    ws.emit((uint32_t)x);
    x >>= 32;
  }
  x = (x << kBypassBits) | v;
}

// Same stream as rans_encode_impl in ONE reverse pass over the symbols: for symbol i the puts of
// its bypass nibbles (last first), then of its nibble count (the remainder, then the 15s), then
// of the symbol itself — exactly the reversed order of BufferedRansEncoder's list.
int rans_encode_tab_impl(const EncTables& T, const int32_t* sym, const int32_t* idx, size_t n, uint8_t* out,
                         size_t cap, size_t* out_len, std::vector<uint32_t>& buf) {
  if (buf.size() < n / 2 + 256) buf.assign(n / 2 + 256, 0u);
  WordSink ws(buf);
  uint64_t x = kRansL;
  for (size_t i = n; i-- > 0;) {
    const int32_t ci = idx[i];
    if (ci < 0 || ci >= T.levels) return RDEIC_EINVAL;
    const int32_t max_value = T.max_value[ci];
    int32_t value = sym[i] - T.offset[ci];
    if (value < 0 || value >= max_value) {
      const uint32_t raw = value < 0 ? (uint32_t)(-2 * (int64_t)value - 1) : (uint32_t)(2 * (int64_t)(value - max_value));
      int32_t nb = 0;
      while (nb < 8 && (raw >> (nb * kBypassBits)) != 0) ++nb;
      for (int32_t j = nb; j-- > 0;) enc_put_bits(x, ws, (raw >> (j * kBypassBits)) & kBypassMax);
      enc_put_bits(x, ws, (uint32_t)(nb % (int32_t)kBypassMax));
      for (int32_t v = nb / (int32_t)kBypassMax; v-- > 0;) enc_put_bits(x, ws, kBypassMax);
      value = max_value;
    }
    enc_put(x, ws, T.sym[(size_t)T.row_off[ci] + value]);
  }
  ws.emit((uint32_t)(x >> 32));
  ws.emit((uint32_t)x);
  const size_t nbytes = (ws.buf.size() - ws.wp) * 4;
  *out_len = nbytes;
  if (nbytes > cap) return RDEIC_ENOSPC;
  memcpy(out, ws.buf.data() + ws.wp, nbytes);
  return RDEIC_OK;
}

// ---- decoder --------------------------------------------------------------
struct RansDecoder {
  std::vector<uint32_t> words;
  size_t pos = 0;
  uint64_t x = 0;
  bool bad = false;

  bool read_word(uint32_t& w) {
    if (pos >= words.size()) { bad = true; return false; }
    w = words[pos++];
    return true;
  }
  uint32_t get_bits(uint32_t nbits) {
    uint32_t v = (uint32_t)(x & ((1u << nbits) - 1));
    x >>= nbits;
    if (x < kRansL) {
      uint32_t w;
      if (read_word(w)) x = (x << 32) | w;
    }
    return v;
  }
};

int rans_decode_impl(RansDecoder* d, const int32_t* idx, size_t n, const int32_t* cdf, int32_t cdf_ld,
                     const int32_t* cdf_len, const int32_t* offset, int32_t levels, int32_t* out) {
  if (d->bad) return RDEIC_EBADMSG;
  for (size_t i = 0; i < n; ++i) {
    const int32_t ci = idx[i];
    if (ci < 0 || ci >= levels) return RDEIC_EINVAL;
    const int32_t* row = cdf + (size_t)ci * cdf_ld;
    const int32_t len = cdf_len[ci];
    const int32_t max_value = len - 2;
    if (max_value < 0 || len > cdf_ld) return RDEIC_EINVAL;
    const uint32_t cum = (uint32_t)(d->x & ((1u << kPrecision) - 1));
    // first entry > cum, minus one (rows are strictly increasing; row[len-1] = 2^16 > cum)
    const int32_t* it = std::upper_bound(row, row + len, (int32_t)cum);
    int32_t s = (int32_t)(it - row) - 1;
    if (s < 0 || s >= len - 1) return RDEIC_EBADMSG;
    const uint64_t start = (uint32_t)row[s], freq = (uint32_t)(row[s + 1] - row[s]);
    uint64_t x = d->x;
    x = freq * (x >> kPrecision) + (x & ((1u << kPrecision) - 1)) - start;
    if (x < kRansL) {
      uint32_t w;
      if (!d->read_word(w)) return RDEIC_EBADMSG;
      x = (x << 32) | w;
    }
    d->x = x;
    int32_t value = s;
    if (value == max_value) {
      int32_t v = (int32_t)d->get_bits(kBypassBits);
      int32_t nb = v;
      while (v == (int32_t)kBypassMax) {
        if (d->bad || nb > 8) return RDEIC_EBADMSG;
        v = (int32_t)d->get_bits(kBypassBits);
        nb += v;
      }
      if (nb > 8) return RDEIC_EBADMSG;
      uint32_t raw = 0;
      for (int32_t j = 0; j < nb; ++j) {
        uint32_t nib = d->get_bits(kBypassBits);
        raw |= nib << (j * kBypassBits);
      }
      if (d->bad) return RDEIC_EBADMSG;
      value = (int32_t)(raw >> 1);
      if (raw & 1)
        value = -value - 1;
      else
        value += max_value;
    }
    out[i] = value + offset[ci];
  }
  return d->bad ? RDEIC_EBADMSG : RDEIC_OK;
}

// Persistent host worker pool: the decoder is called once per checkerboard stage (20x per
// batch), so spawning threads per call would cost more than the decode of a small stage.
// One job runs at a time (callers serialise on job_mu); the caller thread works too.
class WorkerPool {
 public:
  // one pool per calling thread: codec sessions on different host threads (bench.py --streams)
  // code their images concurrently instead of queueing on one job lock
  static WorkerPool& get() {
    thread_local WorkerPool* p = new WorkerPool();  // intentionally leaked: workers outlive thread dtors
    return *p;
  }
  void run(int32_t count, int32_t threads, const std::function<void(int32_t)>& f) {
    std::lock_guard<std::mutex> job(job_mu_);
    int32_t helpers = std::max(0, std::min(threads, count) - 1);
    while ((int32_t)workers_.size() < helpers) {
      const int32_t id = (int32_t)workers_.size();
      try {
        workers_.reserve(workers_.size() + 1);
        std::thread(&WorkerPool::loop, this, id).detach();
      } catch (...) {
        helpers = (int32_t)workers_.size();  // out of threads: run with what exists
        break;
      }
      workers_.push_back(id);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &f;
      count_ = count;
      next_.store(0);
      helpers_ = helpers;
      active_ = helpers;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const int32_t i = next_.fetch_add(1);
      if (i >= count_) break;
      (*fn_)(i);
    }
  }
  void loop(int32_t id) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= helpers_) continue;  // not needed for this job
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }

  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<int32_t> workers_;
  const std::function<void(int32_t)>* fn_ = nullptr;
  std::atomic<int32_t> next_{0};
  int32_t count_ = 0, active_ = 0, helpers_ = 0;
  uint64_t gen_ = 0;
};

// Every extern "C" body runs under guard(): no C++ exception may cross the C ABI (ctypes would
// see std::terminate -> SIGABRT). Allocation failure maps to -ENOSPC, anything else to -EINVAL.
template <typename F>
int guard(F&& f) noexcept {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return RDEIC_ENOSPC;
  } catch (...) {
    return RDEIC_EINVAL;
  }
}

// f(i) must not throw (callers catch inside); thread creation failure degrades to running the
// remaining items on the calling thread.
template <typename F>
void parallel_for(int32_t count, int32_t threads, F&& f) {
  if (threads <= 1 || count <= 1) {
    for (int32_t i = 0; i < count; ++i) f(i);
    return;
  }
  const std::function<void(int32_t)> fn = f;
  WorkerPool::get().run(count, threads, fn);
}

// ---- torchac-compatible arithmetic coder ------------------------------------
struct BitWriter {
  uint8_t* out;
  size_t cap;
  size_t len = 0;
  uint8_t cache = 0;
  int count = 0;
  bool overflow = false;
  void put(int bit) {
    cache = (uint8_t)((cache << 1) | (bit & 1));
    if (++count == 8) {
      if (len < cap) out[len] = cache; else overflow = true;
      ++len;
      count = 0;
      cache = 0;
    }
  }
  void put_with_pending(int bit, uint64_t& pending) {
    put(bit);
    while (pending > 0) { put(!bit); --pending; }
  }
  void flush() {
    while (count > 0) put(0);
  }
};

struct BitReader {
  const uint8_t* in;
  size_t n;
  size_t ptr = 0;
  uint8_t cache = 0;
  int cached = 0;
  void get(uint32_t& value) {
    if (cached == 0) {
      if (ptr == n) { value <<= 1; return; }  // torchac shifts in zeros past the end
      cache = in[ptr++];
      cached = 8;
    }
    value = (value << 1) | ((cache >> (cached - 1)) & 1);
    --cached;
  }
};

inline uint16_t binsearch_u16(const uint16_t* cdf, uint16_t target, uint16_t max_sym) {
  uint16_t left = 0, right = (uint16_t)(max_sym + 1);
  while (left + 1 < right) {
    const uint16_t m = (uint16_t)((left + right) / 2);
    const uint16_t v = cdf[m];
    if (v < target) left = m;
    else if (v > target) right = m;
    else return m;
  }
  return left;
}

}  // namespace

extern "C" {

int rdeic_version(void) { return 1; }

// number of entry points declared in include/rdeic_hip.h (checked by tests/test_abi.py)
int rdeic_abi_count(void) { return 93; }

static int pmf_to_quantized_cdf_impl(const float* pmf, int32_t n, int32_t precision, uint32_t* cdf_out) {
  if (!pmf || !cdf_out || n <= 0 || precision <= 0 || precision > 24) return RDEIC_EINVAL;
  for (int32_t i = 0; i < n; ++i)
    if (!(pmf[i] >= 0.f) || !std::isfinite(pmf[i])) return RDEIC_EINVAL;
  const uint32_t one = 1u << precision;
  std::vector<uint32_t> cdf((size_t)n + 1);
  cdf[0] = 0;
  for (int32_t i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)std::round(pmf[i] * (float)one);
  uint64_t total = 0;
  for (uint32_t v : cdf) total += v;
  if (total == 0) return RDEIC_EINVAL;
  for (auto& v : cdf) v = (uint32_t)(((uint64_t)one * v) / total);
  for (size_t i = 1; i < cdf.size(); ++i) cdf[i] += cdf[i - 1];
  cdf.back() = one;
  const int32_t m = (int32_t)cdf.size();
  for (int32_t i = 0; i < m - 1; ++i) {
    if (cdf[i] == cdf[i + 1]) {
      uint32_t best_freq = ~0u;
      int32_t best = -1;
      for (int32_t j = 0; j < m - 1; ++j) {
        const uint32_t f = cdf[j + 1] - cdf[j];
        if (f > 1 && f < best_freq) { best_freq = f; best = j; }
      }
      if (best < 0) return RDEIC_EINVAL;
      if (best < i) {
        for (int32_t j = best + 1; j <= i; ++j) cdf[j]--;
      } else {
        for (int32_t j = i + 1; j <= best; ++j) cdf[j]++;
      }
    }
  }
  memcpy(cdf_out, cdf.data(), cdf.size() * sizeof(uint32_t));
  return RDEIC_OK;
}

int rdeic_pmf_to_quantized_cdf(const float* pmf, int32_t n, int32_t precision, uint32_t* cdf_out) {
  return guard([&] { return pmf_to_quantized_cdf_impl(pmf, n, precision, cdf_out); });
}

static int build_gaussian_tables_impl(const float* pmf, const int32_t* pmf_len, int32_t levels, int32_t pmf_ld,
                                      int32_t* cdf, int32_t cdf_ld, int32_t* cdf_len) {
  if (!pmf || !pmf_len || !cdf || !cdf_len || levels <= 0) return RDEIC_EINVAL;
  std::vector<float> row;
  std::vector<uint32_t> q;
  for (int32_t i = 0; i < levels; ++i) {
    const int32_t L = pmf_len[i];
    if (L <= 0 || L + 1 > pmf_ld || L + 2 > cdf_ld) return RDEIC_EINVAL;
    // pmf row: L probabilities followed by the tail mass at column L
    row.assign(pmf + (size_t)i * pmf_ld, pmf + (size_t)i * pmf_ld + L + 1);
    q.assign((size_t)L + 2, 0u);
    int rc = pmf_to_quantized_cdf_impl(row.data(), L + 1, kPrecision, q.data());
    if (rc) return rc;
    int32_t* out = cdf + (size_t)i * cdf_ld;
    for (int32_t j = 0; j < cdf_ld; ++j) out[j] = j < L + 2 ? (int32_t)q[j] : 0;
    cdf_len[i] = L + 2;
  }
  return RDEIC_OK;
}

int rdeic_build_gaussian_tables(const float* pmf, const int32_t* pmf_len, int32_t levels, int32_t pmf_ld, int32_t* cdf,
                                int32_t cdf_ld, int32_t* cdf_len, void* reserved) {
  (void)reserved;
  return guard([&] { return build_gaussian_tables_impl(pmf, pmf_len, levels, pmf_ld, cdf, cdf_ld, cdf_len); });
}

int rdeic_rans_encode(const int32_t* sym, const int32_t* idx, size_t n, const int32_t* cdf, int32_t cdf_ld,
                      const int32_t* cdf_len, const int32_t* offset, int32_t levels, uint8_t* out, size_t cap,
                      size_t* out_len) {
  if ((!sym || !idx) && n) return RDEIC_EINVAL;
  if (!cdf || !cdf_len || !offset || !out || !out_len || levels <= 0) return RDEIC_EINVAL;
  return guard([&] {
    std::vector<RansSym> syms;
    std::vector<uint32_t> words;
    return rans_encode_impl(sym, idx, n, cdf, cdf_ld, cdf_len, offset, levels, out, cap, out_len, syms, words);
  });
}

int rdeic_rans_encode_batch(int32_t count, const int32_t* sym, const int32_t* idx, size_t n_per, size_t stride,
                            const int32_t* cdf, int32_t cdf_ld, const int32_t* cdf_len, const int32_t* offset,
                            int32_t levels, uint8_t* out, size_t cap_per, size_t* out_len, int32_t threads) {
  if (count <= 0 || !sym || !idx || !out || !out_len) return RDEIC_EINVAL;
  return guard([&] {
    std::vector<int> rc(count, 0);
    parallel_for(count, threads, [&](int32_t i) {
      rc[i] = guard([&] {
        std::vector<RansSym> syms;
        std::vector<uint32_t> words;
        return rans_encode_impl(sym + i * stride, idx + i * stride, n_per, cdf, cdf_ld, cdf_len, offset, levels,
                                out + i * cap_per, cap_per, &out_len[i], syms, words);
      });
    });
    for (int v : rc)
      if (v) return v;
    return (int)RDEIC_OK;
  });
}

void* rdeic_rans_enc_tables_create(const int32_t* cdf, int32_t cdf_ld, const int32_t* cdf_len, const int32_t* offset,
                                   int32_t levels) {
  if (!cdf || !cdf_len || !offset || levels <= 0 || cdf_ld < 2) return nullptr;
  EncTables* T = new (std::nothrow) EncTables();
  if (!T) return nullptr;
  try {
    T->levels = levels;
    T->row_off.resize(levels);
    T->max_value.resize(levels);
    T->offset.assign(offset, offset + levels);
    size_t total = 0;
    for (int32_t ci = 0; ci < levels; ++ci) {
      const int32_t len = cdf_len[ci];
      if (len < 2 || len > cdf_ld) throw std::invalid_argument("cdf_len");
      T->row_off[ci] = (int32_t)total;
      T->max_value[ci] = len - 2;
      total += (size_t)len - 1;
    }
    T->sym.resize(total);
    for (int32_t ci = 0; ci < levels; ++ci) {
      const int32_t* row = cdf + (size_t)ci * cdf_ld;
      for (int32_t v = 0; v <= T->max_value[ci]; ++v) {
        const int32_t start = row[v], freq = row[v + 1] - row[v];
        if (start < 0 || freq <= 0 || start + freq > (1 << kPrecision)) throw std::invalid_argument("cdf row");
        T->sym[(size_t)T->row_off[ci] + v] = make_enc_sym((uint32_t)start, (uint32_t)freq);
      }
    }
  } catch (...) {
    delete T;
    return nullptr;
  }
  return T;
}

void rdeic_rans_enc_tables_destroy(void* tables) { delete (EncTables*)tables; }

int rdeic_rans_encode_batch_t(const void* tables, int32_t count, const int32_t* sym, const int32_t* idx, size_t n_per,
                              size_t stride, uint8_t* out, size_t cap_per, size_t* out_len, int32_t threads) {
  if (!tables || count <= 0 || ((!sym || !idx) && n_per) || !out || !out_len) return RDEIC_EINVAL;
  const EncTables& T = *(const EncTables*)tables;
  return guard([&] {
    std::vector<int> rc(count, 0);
    parallel_for(count, threads, [&](int32_t i) {
      rc[i] = guard([&] {
        thread_local std::vector<uint32_t> buf;
        return rans_encode_tab_impl(T, sym + i * stride, idx + i * stride, n_per, out + i * cap_per, cap_per,
                                    &out_len[i], buf);
      });
    });
    for (int v : rc)
      if (v) return v;
    return (int)RDEIC_OK;
  });
}

int rdeic_rans_enc_quotient(const void* tables, int32_t row, int32_t value, uint64_t x, uint64_t* q) {
  if (!tables || !q) return RDEIC_EINVAL;
  const EncTables& T = *(const EncTables*)tables;
  if (row < 0 || row >= T.levels || value < 0 || value > T.max_value[row]) return RDEIC_EINVAL;
  const EncSym& s = T.sym[(size_t)T.row_off[row] + value];
  *q = s.freq < 2 ? x : enc_quot(x, s);  // freq 1 stores q = x - 1 with bias + 2^16 - 1; report x / 1
  return RDEIC_OK;
}

void* rdeic_rans_dec_open(const uint8_t* data, size_t len) {
  if (!data && len) return nullptr;
  RansDecoder* d = new (std::nothrow) RansDecoder();
  if (!d) return nullptr;
  const size_t nw = len / 4;
  try {
    d->words.resize(nw);
  } catch (...) {
    delete d;
    return nullptr;
  }
  if (nw) memcpy(d->words.data(), data, nw * 4);
  if (len % 4 != 0 || nw < 2) {
    d->bad = true;
    return d;
  }
  d->x = (uint64_t)d->words[0] | ((uint64_t)d->words[1] << 32);
  d->pos = 2;
  return d;
}

int rdeic_rans_decode(void* handle, const int32_t* idx, size_t n, const int32_t* cdf, int32_t cdf_ld,
                      const int32_t* cdf_len, const int32_t* offset, int32_t levels, int32_t* out) {
  if (!handle || (!idx && n) || (!out && n) || !cdf || !cdf_len || !offset) return RDEIC_EINVAL;
  return guard([&] { return rans_decode_impl((RansDecoder*)handle, idx, n, cdf, cdf_ld, cdf_len, offset, levels, out); });
}

int rdeic_rans_decode_batch(int32_t count, void** handles, const int32_t* idx, size_t n_per, size_t stride,
                            const int32_t* cdf, int32_t cdf_ld, const int32_t* cdf_len, const int32_t* offset,
                            int32_t levels, int32_t* out, int32_t threads) {
  if (count <= 0 || !handles || !idx || !out) return RDEIC_EINVAL;
  return guard([&] {
    std::vector<int> rc(count, 0);
    parallel_for(count, threads, [&](int32_t i) {
      rc[i] = handles[i] ? guard([&] {
        return rans_decode_impl((RansDecoder*)handles[i], idx + i * stride, n_per, cdf, cdf_ld, cdf_len, offset,
                                levels, out + i * stride);
      })
                         : (int)RDEIC_EINVAL;
    });
    for (int v : rc)
      if (v) return v;
    return (int)RDEIC_OK;
  });
}

void rdeic_rans_dec_close(void* handle) { delete (RansDecoder*)handle; }

int rdeic_ac_uniform_cdf(int32_t codebook_size, int16_t* cdf_row) {
  // compute_cdf_uniform_prob (utils/ckbd.py:117-128): float32 cumsum of 1/K, last = 1.0;
  // torchac _convert_to_int_and_normalize: round(cdf * (2^16 - (Lp-1))) as int16, + arange(Lp).
  if (codebook_size <= 0 || codebook_size > 32768 || !cdf_row) return RDEIC_EINVAL;
  const int32_t lp = codebook_size + 1;
  const float p = 1.0f / (float)codebook_size;
  float acc = 0.f;
  const float maxv = 65536.0f - (float)(lp - 1);
  for (int32_t k = 0; k < lp; ++k) {
    float c = (k == lp - 1) ? 1.0f : acc;
    float v = std::nearbyint(c * maxv);
    int32_t iv = (int32_t)v;
    cdf_row[k] = (int16_t)(uint16_t)((uint32_t)(iv + k) & 0xFFFFu);
    acc += p;
  }
  return RDEIC_OK;
}

int rdeic_ac_encode(const int16_t* sym, size_t n, const int16_t* cdf_row, int32_t lp, uint8_t* out, size_t cap,
                    size_t* out_len) {
  if ((!sym && n) || !cdf_row || lp < 2 || !out || !out_len) return RDEIC_EINVAL;
  const uint16_t* cdf = (const uint16_t*)cdf_row;
  const int32_t max_symbol = lp - 2;
  BitWriter bw{out, cap};
  uint32_t low = 0, high = 0xFFFFFFFFu;
  uint64_t pending = 0;
  for (size_t i = 0; i < n; ++i) {
    const int32_t s = sym[i];
    if (s < 0 || s > max_symbol) return RDEIC_EINVAL;
    const uint64_t span = (uint64_t)high - (uint64_t)low + 1;
    const uint32_t c_low = cdf[s];
    const uint32_t c_high = s == max_symbol ? 0x10000u : cdf[s + 1];
    high = (low - 1) + (uint32_t)((span * c_high) >> kPrecision);
    low = low + (uint32_t)((span * c_low) >> kPrecision);
    for (;;) {
      if (high < 0x80000000u) {
        bw.put_with_pending(0, pending);
        low <<= 1;
        high = (high << 1) | 1;
      } else if (low >= 0x80000000u) {
        bw.put_with_pending(1, pending);
        low <<= 1;
        high = (high << 1) | 1;
      } else if (low >= 0x40000000u && high < 0xC0000000u) {
        ++pending;
        low = (low << 1) & 0x7FFFFFFFu;
        high = (high << 1) | 0x80000001u;
      } else {
        break;
      }
    }
  }
  pending += 1;
  bw.put_with_pending(low < 0x40000000u ? 0 : 1, pending);
  bw.flush();
  *out_len = bw.len;
  return bw.overflow ? RDEIC_ENOSPC : RDEIC_OK;
}

int rdeic_ac_decode(const uint8_t* data, size_t len, size_t n, const int16_t* cdf_row, int32_t lp, int16_t* out) {
  if ((!data && len) || !cdf_row || lp < 2 || (!out && n)) return RDEIC_EINVAL;
  if (n == 0) return RDEIC_OK;
  const uint16_t* cdf = (const uint16_t*)cdf_row;
  const uint16_t max_symbol = (uint16_t)(lp - 2);
  BitReader br{data, len};
  uint32_t low = 0, high = 0xFFFFFFFFu, value = 0;
  for (int i = 0; i < 32; ++i) br.get(value);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t span = (uint64_t)high - (uint64_t)low + 1;
    const uint16_t count = (uint16_t)((((uint64_t)value - (uint64_t)low + 1) * 0x10000u - 1) / span);
    const uint16_t s = binsearch_u16(cdf, count, max_symbol);
    out[i] = (int16_t)s;
    if (i == n - 1) break;
    const uint32_t c_low = cdf[s];
    const uint32_t c_high = s == max_symbol ? 0x10000u : cdf[s + 1];
    high = (low - 1) + (uint32_t)((span * c_high) >> kPrecision);
    low = low + (uint32_t)((span * c_low) >> kPrecision);
    for (;;) {
      if (low >= 0x80000000u || high < 0x80000000u) {
        low <<= 1;
        high = (high << 1) | 1;
        br.get(value);
      } else if (low >= 0x40000000u && high < 0xC0000000u) {
        low = (low << 1) & 0x7FFFFFFFu;
        high = (high << 1) | 0x80000001u;
        value -= 0x40000000u;
        br.get(value);  // get() shifts value left and appends the next bit
      } else {
        break;
      }
    }
  }
  return RDEIC_OK;
}

}  // extern "C"
