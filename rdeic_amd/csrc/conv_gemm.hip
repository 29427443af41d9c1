// Implicit-GEMM convolution / linear for gfx950 (MFMA), NHWC activations.
//
// GEMM view: M = n*ho*wo output pixels, N = cout, K = kh*kw*cin.
//   A[m, k] is gathered on the fly from NHWC input(s) (k = (ky, kx, ci), ci fastest)
//   B[k, n] = packed weight [cout][wld] (K-contiguous rows)
// Both operands are K-major in LDS, so an MFMA fragment (8 consecutive k of one
// row for bf16 16x16x32, 1 element for f32 16x16x4) is one ds_read per lane.
//
// Fusions (all optional, selected per launch):
//   prologue : two-segment channel concat (UNet skip concat, control-branch input),
//              nearest x2 upsample (UNet/VAE Upsample), stride / asymmetric pad
//              (UNet / VAE Downsample), GroupNorm affine + SiLU on the gathered values
//   epilogue : bias, per-(image, cout) timestep-embedding add, activation
//              (leaky_relu / gelu / silu), residual add, PixelShuffle(2) store.
//
// Accumulation order over K is fixed (k-tiles in order, fixed MFMA), independent of
// tile shape or batch size, so results are batch-invariant — a requirement of the
// entropy model (encoder and decoder must recompute identical means / scales).
//
// Replaces: every nn.Conv2d / nn.Linear on the RDEIC hot path (see include/rdeic_hip.h).
#include "common.h"
#include "../../include/rdeic_hip.h"
#include "prof.h"

namespace {

struct ConvArgs {
  const char* in0; const char* in1;
  int c0, c1, ld0, ld1;
  int n, h, w, up2;
  const char* weight; int wld;
  const float* bias;
  int cout, kh, kw, stride, pad_t, pad_l, ho, wo;
  const float* gn_ab; int gn_silu;
  const float* emb; int emb_ld;
  int act; float act_param;
  const char* res; int res_ld;
  char* out; int out_ld, out_mode;
  int out_f32;
  int M, cin, ktot, nk;
  long in_bs, w_bs, out_bs;  // batched-GEMM strides (elements), blockIdx.z
  int batch;
  int epi_vec;               // 1: LDS-staged vector epilogue where eligible
  int splits, kper;          // split-K: blockIdx.z = split, k-steps [z*kper, (z+1)*kper), raw fp32 partial out
  float* gn_part;            // fused GroupNorm statistics of the output (see epilogue_vec), or NULL
  int gn_row0;               // absolute output row of this launch's row 0 (image-group launches)
  int gn_hw;                 // pixels per image of the GroupNorm those statistics feed
  const float* ln_rows;      // folded LayerNorm: [M][2] (mean, rstd) of the raw input rows, or NULL
  const float* ln_cs;        // ... and the column sums of the packed (gamma-scaled) bf16 weight
  float* sk_ws;              // split-K folded into the producer (LDS-DMA path): raw fp32 partial slabs ...
  int* sk_cnt;               // ... and one arrival counter per output tile (zero before, left zero after)
};

// Folded LayerNorm (rdeic_conv_desc.ln_rows): LN(x) W = rstd (x W' - mean colsum(W')) with W' = diag(gamma) W
// and beta W in the bias; applied to the raw accumulator before everything else of the epilogue.
__device__ __forceinline__ float ln_fold(const ConvArgs& a, int m, int n, float v) {
  const float2 ms = reinterpret_cast<const float2*>(a.ln_rows)[m];
  return ms.y * (v - ms.x * a.ln_cs[n]);
}

int g_conv_path = 2;  // 0: 128-tiles with the fused GroupNorm prologue only, 2 (default): big-tile auto choice
int g_epi_vec = 1;    // LDS-staged vector epilogue (rdeic_set_conv_option(0, v))
int g_swz = 1;        // swizzled 128-B LDS rows where they win (1) / padded 144-B rows everywhere (0) (option 3)
int g_force_tile = -1;  // >= 0: force launch_plain_auto's candidate (rdeic_set_conv_option(4, i)), tuning only
int g_dma = 1;        // LDS-DMA path for cin % 64 == 0 (rdeic_set_conv_option(5, v))
int g_pf2 = 0;        // 2-deep register prefetch in the plain path (rdeic_set_conv_option(2, v)); measured neutral, off

constexpr int ROWB = 144;  // fp32 tiles: LDS bytes per row, 128 B of k-data + 16 B pad (bank spread)

// bf16 tiles use unpadded 128-byte rows with the 16-byte chunks XOR-swizzled by row bits 1 and 3:
// chunk c of row r lives in slot c ^ key(r); every ds_read_b128 lane group of the 16x16x32
// fragment reads (rows r..r+15, one chunk column) then covers all 64 banks once, and a row's
// 8 chunks written by 8 lanes still cover 32 banks. Rows a lane touches differ by multiples of
// 16, so key(r) is a per-lane constant on both sides.
template <typename T, bool SWZ = true> __host__ __device__ constexpr int tile_rowb() { return (sizeof(T) == 2 && SWZ) ? 128 : ROWB; }
template <typename T, bool SWZ = true> __device__ __forceinline__ int chunk_key(int r) {
  if constexpr (sizeof(T) == 2 && SWZ) return (((r >> 3) & 1) << 1) | (((r >> 1) & 1) << 2);
  return 0;
}
// dynamic LDS of conv_kernel: the double-buffered tiles, or the vector epilogue's half tile
template <typename T, int BM, int BN, bool SWZ = true> __host__ __device__ constexpr int conv_lds_bytes() {
  return (2 * (BM + BN) * tile_rowb<T, SWZ>() > (BM / 2) * (BN + 4) * 4 || sizeof(T) != 2)
             ? 2 * (BM + BN) * tile_rowb<T, SWZ>()
             : (BM / 2) * (BN + 4) * 4;
}

template <typename T> struct MmaTraits;
template <> struct MmaTraits<bf16> {
  static constexpr int BK = 64;   // k per tile (128 B per row)
  static constexpr int EPC = 8;   // elements per 16-byte chunk
};
template <> struct MmaTraits<float> {
  static constexpr int BK = 32;
  static constexpr int EPC = 4;
};

__device__ __forceinline__ float apply_act(float v, int act, float p) {
  if (act == 1) return v >= 0.f ? v : v * p;
  if (act == 2) return gelu_f(v);
  if (act == 3) return silu_f(v);
  return v;
}

// Load 16 bytes (one chunk) from global, or zeros.
__device__ __forceinline__ uint4 ld16(const char* p) { return *reinterpret_cast<const uint4*>(p); }

template <typename T>
__device__ __forceinline__ uint4 gn_apply_chunk(uint4 raw, const float* ab, int silu) {
  constexpr int E = MmaTraits<T>::EPC;
  T v[E];
  *reinterpret_cast<uint4*>(v) = raw;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float x = to_f32(v[e]);
    x = x * ab[2 * e] + ab[2 * e + 1];
    if (silu) x = silu_f(x);
    v[e] = from_f32<T>(x);
  }
  return *reinterpret_cast<uint4*>(v);
}

// Vectorised epilogue through LDS (bf16 activations; out_mode 0): the accumulators of half the
// tile rows at a time are parked in LDS as fp32, then re-read row-contiguous 8 at a time so the
// bias / emb / activation / residual are applied per 8-wide chunk and the residual load and the
// output store are 16-byte coalesced vectors. Same fp32 operation order as the scalar epilogue
// ((acc + bias) + emb -> act -> + res -> round), so results are bit-identical to it.
// Needs BM/2 * (BN + 4) * 4 bytes of LDS; the caller has finished with its k-loop buffers.
__host__ __device__ __forceinline__ bool epi_vec_ok(const ConvArgs& a) {
  if (a.out_mode == 2) return (a.cout % 8) == 0 && (a.out_ld % 4) == 0 && ((uintptr_t)a.out % 8) == 0;
  return a.out_mode == 0 && (a.cout % 8) == 0 && (a.out_ld % 8) == 0 && ((uintptr_t)a.out % 16) == 0 &&
         (!a.res || ((a.res_ld % 8) == 0 && ((uintptr_t)a.res % 16) == 0));
}

// Tile row -> output row (GEMM m) of the vector epilogue: the GEMM kernels' tiles are BM consecutive
// rows from m0; the halo conv's tiles are image blocks whose 64-row wave rows are each contiguous.
struct RowsFrom {
  int m0;
  __device__ __forceinline__ int operator()(int r) const { return m0 + r; }
};

template <int BM, int BN, int WGM, int WGN, int NT, int P = 2, class RowMap = RowsFrom, bool PF = true>
__device__ __forceinline__ void epilogue_vec(const f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16], const ConvArgs& a,
                                             int m0, int n0, int wm, int wn, int lane, int tid, char* lds,
                                             RowMap rmap = RowMap{0}) {
  if constexpr (__is_same(RowMap, RowsFrom)) rmap.m0 = m0;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int HM = TM / P;                    // fragment rows per pass
  constexpr int PR = BM / P;                    // tile rows per pass
  constexpr int SDW = BN + 4;                   // LDS row stride in dwords (bank spread)
  constexpr int CPR = BN / 8;                   // 8-wide chunks per row
  static_assert(TM % P == 0, "P passes");
  const int lr = lane & 15, lq = lane >> 4;
  float* L = reinterpret_cast<float*>(lds);
  const int hw_o = a.ho * a.wo;
  const bool of32 = a.out_f32;
  // Fused GroupNorm statistics (a.gn_part): per output channel and absolute 64-row block, the sum
  // and the sum of squares of the values as stored (bf16-rounded), in a CANONICAL order that does
  // not depend on the tile: four 16-row groups, each summed sequentially in row order (fmaf for the
  // squares), combined as ((g0 + g1) + g2) + g3 — exactly what gn_rows_partial_kernel computes, so
  // the statistics (and every GroupNorm after them) are identical for every tile and batch size.
  // Each pass writes its stored values back over its parked accumulators; thread (b, j) then scans
  // column j of 64-row block b in LDS (NU such pairs per thread when the tile has more pairs than
  // threads). Needs WTM in {32, 64} (a wave-row block inside one 64-row block); the host enables it
  // only for such tiles (stats_tile_ok).
  const bool st = a.gn_part != nullptr;
  constexpr int NU = ((BM / 64) * BN + NT - 1) / NT;  // (64-row block, channel) pairs per thread
  float sg[NU][4], qg[NU][4];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) sg[u][g] = qg[u][g] = 0.f;
  // The per-chunk global operands (residual rows, LayerNorm row statistics, bias, LayerNorm column sums)
  // are loaded at the top of each pass, before the accumulators are parked, behind raw barriers (no
  // vmcnt(0) drain): their latency overlaps the park instead of being exposed once per chunk in a chain
  // (r05: the loads inside the chunk loop made the epilogue 19.5k cycles of a 38k-cycle 256x256 linear tile,
  // tools/dma_stamps.hip). Loaded values and the arithmetic order are unchanged: outputs are bit-identical.
  constexpr int NCH = (PR * CPR + NT - 1) / NT;  // chunks per thread per pass
  constexpr int NPF = !PF ? 0 : NCH < 2 ? NCH : 2;  // of them prefetched (register budget; PF off: none)
  constexpr bool HOIST = PF && (NT % CPR) == 0;   // every chunk of a thread has the same 8 channels
  auto bar = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  float4 bh[2] = {float4{0.f, 0.f, 0.f, 0.f}, float4{0.f, 0.f, 0.f, 0.f}}, chh[2] = {bh[0], bh[0]};
  if constexpr (HOIST) {  // bias / LayerNorm column sums of this thread's channels, once
    const int nn = n0 + (tid % CPR) * 8;
    if (nn < a.cout) {
      if (a.bias) {
        bh[0] = *reinterpret_cast<const float4*>(a.bias + nn);
        bh[1] = *reinterpret_cast<const float4*>(a.bias + nn + 4);
      }
      if (a.ln_rows) {
        chh[0] = *reinterpret_cast<const float4*>(a.ln_cs + nn);
        chh[1] = *reinterpret_cast<const float4*>(a.ln_cs + nn + 4);
      }
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    uint4 rpf[NPF > 0 ? NPF : 1];    // bf16 residual chunk
    float2 lpf[NPF > 0 ? NPF : 1];   // LayerNorm (mean, rstd) of the chunk's row
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int c = tid + k * NT;
      const int pr = c / CPR, cc = c - pr * CPR;
      const int wmr = pr / (WTM / P), wr = pr - wmr * (WTM / P);
      const int m = rmap(wmr * WTM + p * (WTM / P) + wr);
      const int nn = n0 + cc * 8;
      const bool ok = c < PR * CPR && m < a.M && nn < a.cout;
      rpf[k] = uint4{0u, 0u, 0u, 0u};
      lpf[k] = float2{0.f, 0.f};
      if (ok) {
        if (a.res && !of32 && a.out_mode != 2)
          rpf[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.res) + (long)m * a.res_ld + nn);
        if (a.ln_rows) lpf[k] = reinterpret_cast<const float2*>(a.ln_rows)[m];
      }
    }
    bar();  // the previous pass's LDS readers are done
#pragma unroll
    for (int ii = 0; ii < HM; ++ii)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = wm * (WTM / P) + ii * 16 + lq * 4 + r;
#pragma unroll
        for (int j = 0; j < TN; ++j) L[pr * SDW + wn * WTN + j * 16 + lr] = acc[p * HM + ii][j][r];
      }
    bar();
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = tid + k * NT;
      if (c >= PR * CPR) continue;
      const int pr = c / CPR, cc = c - pr * CPR;
      // pass-local row pr -> wave row block wm' = pr / (WTM/P), row within = pr % (WTM/P)
      const int wmr = pr / (WTM / P), wr = pr - wmr * (WTM / P);
      const int m = rmap(wmr * WTM + p * (WTM / P) + wr);
      const int nn = n0 + cc * 8;
      if (m >= a.M || nn >= a.cout) continue;
      float v[8];
      const float4 x0 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8 + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      if (a.ln_rows) {
        const float2 ms = k < NPF ? lpf[k < NPF ? k : 0] : reinterpret_cast<const float2*>(a.ln_rows)[m];
        float4 c0 = chh[0], c1 = chh[1];
        if constexpr (!HOIST) {
          c0 = *reinterpret_cast<const float4*>(a.ln_cs + nn);
          c1 = *reinterpret_cast<const float4*>(a.ln_cs + nn + 4);
        }
        const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        // v = rstd * (v - mean * colsum), two columns per packed fma / mul
        const f32x2 nm = {-ms.x, -ms.x}, rs = {ms.y, ms.y};
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 r = rs * pk_fma(nm, f32x2{cs[e], cs[e + 1]}, f32x2{v[e], v[e + 1]});
          v[e] = r.x;
          v[e + 1] = r.y;
        }
      }
      if (a.bias) {
        float4 b0 = bh[0], b1 = bh[1];
        if constexpr (!HOIST) {
          b0 = *reinterpret_cast<const float4*>(a.bias + nn);
          b1 = *reinterpret_cast<const float4*>(a.bias + nn + 4);
        }
        const float bs[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 r = f32x2{v[e], v[e + 1]} + f32x2{bs[e], bs[e + 1]};
          v[e] = r.x;
          v[e + 1] = r.y;
        }
      }
      if (a.emb) {
        const float* em = a.emb + (long)(m / hw_o) * a.emb_ld + nn;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += em[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], a.act, a.act_param);
      if (a.out_mode == 2) {
        // fused GEGLU (attention.py:49-56): the packed weight interleaves 4 value rows with their 4
        // gate rows, so this chunk is (x0..x3, g0..g3) of output channels nn/2 .. nn/2+3. Both halves
        // are rounded to bf16 first, as the unfused projection + rdeic_geglu see them.
        bf16 gv[4];
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 xv = {to_f32(from_f32<bf16>(v[e])), to_f32(from_f32<bf16>(v[e + 1]))};
          const f32x2 gt = {to_f32(from_f32<bf16>(v[4 + e])), to_f32(from_f32<bf16>(v[5 + e]))};
          const f32x2 r = xv * gelu_fast2(gt);
          gv[e] = from_f32<bf16>(r.x);
          gv[e + 1] = from_f32<bf16>(r.y);
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(a.out) + (long)m * a.out_ld + (nn >> 1)) =
            *reinterpret_cast<uint2*>(gv);
        continue;
      }
      if (a.res) {
        if (of32) {
          const float4 r0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.res) + (long)m * a.res_ld + nn);
          const float4 r1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.res) + (long)m * a.res_ld + nn + 4);
          v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w; v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
        } else {
          bf16 rv[8];
          *reinterpret_cast<uint4*>(rv) =
              k < NPF ? rpf[k < NPF ? k : 0]
                      : *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.res) + (long)m * a.res_ld + nn);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += to_f32(rv[e]);
        }
      }
      if (of32) {
        float* o = reinterpret_cast<float*>(a.out) + (long)m * a.out_ld + nn;
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
        if (st) {  // stored values back over the parked accumulators, for the statistics scan
          *reinterpret_cast<float4*>(L + pr * SDW + cc * 8) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(L + pr * SDW + cc * 8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      } else {
        bf16 ov[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[e] = from_f32<bf16>(v[e]);
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(a.out) + (long)m * a.out_ld + nn) = *reinterpret_cast<uint4*>(ov);
        if (st) {
          *reinterpret_cast<float4*>(L + pr * SDW + cc * 8) =
              make_float4(to_f32(ov[0]), to_f32(ov[1]), to_f32(ov[2]), to_f32(ov[3]));
          *reinterpret_cast<float4*>(L + pr * SDW + cc * 8 + 4) =
              make_float4(to_f32(ov[4]), to_f32(ov[5]), to_f32(ov[6]), to_f32(ov[7]));
        }
      }
    }
    if constexpr ((WTM == 32 || WTM == 64) && (WTM / P) % 16 == 0) {
      if (st) {
        bar();  // LDS-only: the stored values written back (the global stores stay in flight)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
        const int b = (tid + u * NT) / BN, j = (tid + u * NT) % BN;
        if (b < BM / 64) {
          constexpr int WPB = 64 / WTM;  // wave-row blocks per 64-row block
#pragma unroll
          for (int w = 0; w < WPB; ++w) {
            const int wmr = b * WPB + w;
#pragma unroll
            for (int k = 0; k < (WTM / P) / 16; ++k) {
              const int off = w * WTM + p * (WTM / P) + k * 16;  // row offset inside the 64-row block
              const float* col = L + (wmr * (WTM / P) + k * 16) * SDW + j;
              const int nv = a.M - (rmap(b * 64) + off);  // valid rows of this 16-row group
              float s1 = 0.f, s2 = 0.f;
              if (nv >= 16) {  // all 16 loads issued before the (row-ordered) sums
                float y[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) y[r] = col[r * SDW];
#pragma unroll
                for (int r = 0; r < 16; ++r) { s1 += y[r]; s2 = fmaf(y[r], y[r], s2); }
              } else {
                for (int r = 0; r < nv; ++r) { const float y = col[r * SDW]; s1 += y; s2 = fmaf(y, y, s2); }
              }
              sg[u][off >> 4] = s1;
              qg[u][off >> 4] = s2;
            }
          }
        }
        }
      }
    }
  }
  if constexpr ((WTM == 32 || WTM == 64) && (WTM / P) % 16 == 0) {
    if (st) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int b = (tid + u * NT) / BN, j = (tid + u * NT) % BN;
        const int nn = n0 + j;
        if (b < BM / 64 && nn < a.cout && rmap(b * 64) < a.M) {  // blocks past M are not in the buffer
          float* pp = a.gn_part + 4 + ((long)((a.gn_row0 + rmap(b * 64)) / 64) * a.cout + nn) * 2;
          pp[0] = ((sg[u][0] + sg[u][1]) + sg[u][2]) + sg[u][3];
          pp[1] = ((qg[u][0] + qg[u][1]) + qg[u][2]) + qg[u][3];
        }
      }
      if (tid == 0 && rmap(0) == 0 && n0 == 0) reinterpret_cast<int*>(a.gn_part)[0] = 64;  // rows per partial
    }
  }
}

// the compile-time conditions under which epilogue_vec computes fused statistics (mirrors its
// `if constexpr`): a wave-row block inside one 64-row block, 16-row groups per pass, one thread per
// (64-row block, channel)
template <int BM, int BN, int WGM, int NT, int P>
constexpr bool stats_tile_ok() {
  constexpr int WTM = BM / WGM;
  return (WTM == 32 || WTM == 64) && (WTM / P) % 16 == 0;
}

// GNP: compile the GroupNorm+SiLU gather prologue in (false = plain gather, fewer VGPRs / VALU).
template <typename T, int BM, int BN, int WGM, int WGN, bool VEC, bool GNP = true, bool PF2 = false, bool SWZ = true>
__global__ __launch_bounds__(WGM * WGN * 64) void conv_kernel(ConvArgs a) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int BK = MmaTraits<T>::BK;
  constexpr int EPC = MmaTraits<T>::EPC;
  constexpr int ES = sizeof(T);
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RPI = NT / 8;                  // tile rows covered per load instruction (8 chunks per row)
  constexpr int AR = BM / RPI;                 // A chunks per thread
  constexpr int BR = (BN + RPI - 1) / RPI;     // B chunks per thread
  static_assert(TM >= 1 && TN >= 1 && AR >= 1 && BM % RPI == 0, "tile");

  extern __shared__ __attribute__((aligned(16))) char lds[];
  // buffer b: A tile at lds + b*(BM+BN)*RB, B tile right after it
  constexpr int RB = tile_rowb<T, SWZ>();
#define AS(b) (lds + (b) * (BM + BN) * RB)
#define BS(b) (lds + (b) * (BM + BN) * RB + BM * RB)

  int kt_begin = 0, kt_end = a.nk;
  if (a.splits > 1) {
    const int z = blockIdx.z;
    kt_begin = min(a.nk, z * a.kper);
    kt_end = min(a.nk, kt_begin + a.kper);
    a.out += (long)z * a.M * a.out_ld * 4;  // this split's fp32 partial slab
  } else if (gridDim.z > 1) {
    const long z = blockIdx.z;
    a.in0 += z * a.in_bs * ES; a.in1 += z * a.in_bs * ES;
    a.weight += z * a.w_bs * ES;
    a.out += z * a.out_bs * (((sizeof(T) == 4) || a.out_f32) ? 4 : ES);
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kc = tid & 7;   // chunk column this thread gathers (same every k-tile)
  const int hw_o = a.ho * a.wo;
  const int hin = a.up2 ? 2 * a.h : a.h, win = a.up2 ? 2 * a.w : a.w;

  // per-row gather state (rows fixed across the K loop)
  int r_img[AR], r_iy[AR], r_ix[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    int m = m0 + (tid >> 3) + RPI * i;
    if (m < a.M) {
      int img = m / hw_o, rem = m - img * hw_o;
      int oy = rem / a.wo, ox = rem - oy * a.wo;
      r_img[i] = img;
      r_iy[i] = oy * a.stride - a.pad_t;
      r_ix[i] = ox * a.stride - a.pad_l;
    } else {
      r_img[i] = -1; r_iy[i] = 0; r_ix[i] = 0;
    }
  }

  uint4 areg[AR];
  uint4 breg[BR];
  int a_c[AR];  // channel of chunk start per row (for the GN prologue), -1 = zero chunk

  auto gather_a = [&](int kt, uint4 (&areg)[AR]) {
    const int k0 = kt * BK + kc * EPC;
    if constexpr (VEC) {
      bool kval = k0 < a.ktot;
      int tap = kval ? k0 / a.cin : 0;
      int c = k0 - tap * a.cin;
      int ky = tap / a.kw, kx = tap - ky * a.kw;
      const char* base; int ld, cs;
      if (c < a.c0) { base = a.in0; ld = a.ld0; cs = c; } else { base = a.in1; ld = a.ld1; cs = c - a.c0; }
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        int iy = r_iy[i] + ky, ix = r_ix[i] + kx;
        bool ok = kval && r_img[i] >= 0 && iy >= 0 && iy < hin && ix >= 0 && ix < win;
        if (ok) {
          if (a.up2) { iy >>= 1; ix >>= 1; }
          long pix = ((long)r_img[i] * a.h + iy) * a.w + ix;
          areg[i] = ld16(base + (pix * ld + cs) * ES);
          a_c[i] = c;
        } else {
          areg[i] = make_uint4(0, 0, 0, 0);
          a_c[i] = -1;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        T v[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          int k = k0 + e;
          float x = 0.f;
          if (k < a.ktot && r_img[i] >= 0) {
            int tap = k / a.cin, c = k - tap * a.cin;
            int ky = tap / a.kw, kx = tap - ky * a.kw;
            int iy = r_iy[i] + ky, ix = r_ix[i] + kx;
            if (iy >= 0 && iy < hin && ix >= 0 && ix < win) {
              if (a.up2) { iy >>= 1; ix >>= 1; }
              long pix = ((long)r_img[i] * a.h + iy) * a.w + ix;
              const T* src = (c < a.c0) ? reinterpret_cast<const T*>(a.in0) + pix * a.ld0 + c
                                        : reinterpret_cast<const T*>(a.in1) + pix * a.ld1 + (c - a.c0);
              x = to_f32(*src);
              if (GNP && a.gn_ab) {
                const float* ab = a.gn_ab + ((long)r_img[i] * a.cin + c) * 2;
                x = x * ab[0] + ab[1];
                if (a.gn_silu) x = silu_f(x);
              }
            }
          }
          v[e] = from_f32<T>(x);
        }
        areg[i] = *reinterpret_cast<uint4*>(v);
        a_c[i] = -1;  // prologue already applied
      }
    }
  };

  auto gather_b = [&](int kt, uint4 (&breg)[BR]) {
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      int cid = tid + NT * i;
      int row = cid >> 3, ch = cid & 7;
      if (row < BN) {
        int nn = n0 + row;
        if (nn < a.cout)
          breg[i] = ld16(a.weight + ((long)nn * a.wld + kt * BK + ch * EPC) * ES);
        else
          breg[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };

  auto store_tiles = [&](int buf, const uint4 (&areg)[AR], const uint4 (&breg)[BR]) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      uint4 v = areg[i];
      if constexpr (VEC) {
        if (GNP && a.gn_ab && a_c[i] >= 0)
          v = gn_apply_chunk<T>(v, a.gn_ab + ((long)r_img[i] * a.cin + a_c[i]) * 2, a.gn_silu);
      }
      int row = (tid >> 3) + RPI * i;
      *reinterpret_cast<uint4*>(AS(buf) + row * RB + (kc ^ chunk_key<T, SWZ>(row)) * 16) = v;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      int cid = tid + NT * i;
      int row = cid >> 3, ch = cid & 7;
      if (row < BN) *reinterpret_cast<uint4*>(BS(buf) + row * RB + (ch ^ chunk_key<T, SWZ>(row)) * 16) = breg[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lrow = lane & 15, lq = lane >> 4;

  auto compute = [&](int cur) {
    const char* Ab = AS(cur) + (wm * WTM + lrow) * RB;
    const char* Bb = BS(cur) + (wn * WTN + lrow) * RB;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int so = ((s * 4 + lq) ^ chunk_key<T, SWZ>(lrow)) * 16;  // swizzled fragment chunk
        if constexpr (TM * TN > 16) {
          // big wave tiles: hold the B fragments, stream A fragments one at a time (register budget)
          bf16x8 bfv[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(Bb + j * 16 * RB + so);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(Ab + i * 16 * RB + so);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
          }
        } else {
          bf16x8 af[TM], bfv[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(Ab + i * 16 * RB + so);
#pragma unroll
          for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(Bb + j * 16 * RB + so);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        float af[TM], bfv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const float*>(Ab + i * 16 * RB + (s * 4 + lq) * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const float*>(Bb + j * 16 * RB + (s * 4 + lq) * 4);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  if constexpr (PF2) {
    // two register sets: tile j lives in set j & 1; the load of tile k+2 is in flight while
    // tile k is computed and tile k+1 (loaded one step earlier) is written to LDS.
    uint4 ary[AR], bry[BR];
    gather_a(0, areg); gather_b(0, breg);
    store_tiles(0, areg, breg);
    if (a.nk > 1) { gather_a(1, ary); gather_b(1, bry); }
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < a.nk; kt += 2) {
      if (kt + 2 < a.nk) { gather_a(kt + 2, areg); gather_b(kt + 2, breg); }
      compute(0);
      store_tiles(1, ary, bry);
      __syncthreads();
      if (kt + 3 < a.nk) { gather_a(kt + 3, ary); gather_b(kt + 3, bry); }
      compute(1);
      if (kt + 2 < a.nk) store_tiles(0, areg, breg);
      __syncthreads();
    }
    if (kt < a.nk) compute(0);
  } else {
    if (kt_begin < kt_end) {
      gather_a(kt_begin, areg);
      gather_b(kt_begin, breg);
      store_tiles(0, areg, breg);
    }
    __syncthreads();
    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const int cur = (kt - kt_begin) & 1;
      if (kt + 1 < kt_end) { gather_a(kt + 1, areg); gather_b(kt + 1, breg); }
      compute(cur);
      if (kt + 1 < kt_end) store_tiles(cur ^ 1, areg, breg);
      __syncthreads();
    }
  }

#undef AS
#undef BS
  if constexpr (sizeof(T) == 2 && TM % 2 == 0 && (BM / 2) * (BN + 4) * 4 <= conv_lds_bytes<T, BM, BN, SWZ>()) {
    if (a.epi_vec && epi_vec_ok(a)) {
      epilogue_vec<BM, BN, WGM, WGN, NT, 2, RowsFrom, false>(acc, a, m0, n0, wm, wn, lane, tid, lds);
      return;
    }
  }
  // ---------------- epilogue: C[m][n], lane holds col n = lane&15, rows 4*lq + r
  const bool of32 = (sizeof(T) == 4) || a.out_f32;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WTM + i * 16 + lq * 4 + r;
      if (m >= a.M) continue;
      const int img = m / hw_o;
      long opix = m;
      int oy = 0, ox = 0;
      if (a.out_mode == 1) { int rem = m - img * hw_o; oy = rem / a.wo; ox = rem - oy * a.wo; }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nn = n0 + wn * WTN + j * 16 + lrow;
        if (nn >= a.cout) continue;
        float v = acc[i][j][r];
        if (a.ln_rows) v = ln_fold(a, m, nn, v);
        if (a.bias) v += a.bias[nn];
        if (a.emb) v += a.emb[(long)img * a.emb_ld + nn];
        v = apply_act(v, a.act, a.act_param);
        long oidx;
        if (a.out_mode == 1) {
          int c = nn >> 2, dy = (nn >> 1) & 1, dx = nn & 1;
          long p = ((long)img * (2 * a.ho) + (2 * oy + dy)) * (2 * a.wo) + (2 * ox + dx);
          oidx = p * a.out_ld + c;
          if (a.res) {
            long ridx = p * a.res_ld + c;
            v += of32 ? reinterpret_cast<const float*>(a.res)[ridx] : to_f32(reinterpret_cast<const T*>(a.res)[ridx]);
          }
        } else {
          oidx = opix * a.out_ld + nn;
          if (a.res) {
            long ridx = opix * a.res_ld + nn;
            v += of32 ? reinterpret_cast<const float*>(a.res)[ridx] : to_f32(reinterpret_cast<const T*>(a.res)[ridx]);
          }
        }
        if (of32) reinterpret_cast<float*>(a.out)[oidx] = v;
        else reinterpret_cast<T*>(a.out)[oidx] = from_f32<T>(v);
      }
    }
  }
}

template <typename T, int BM, int BN, int WGM, int WGN>
int launch_cfg(const ConvArgs& a, bool vec, hipStream_t s) {
  dim3 grid(cdiv(a.M, BM), cdiv(a.cout, BN), a.batch);
  size_t lds = conv_lds_bytes<T, BM, BN>();
  if (vec)
    hipLaunchKernelGGL((conv_kernel<T, BM, BN, WGM, WGN, true>), grid, dim3(WGM * WGN * 64), lds, s, a);
  else
    hipLaunchKernelGGL((conv_kernel<T, BM, BN, WGM, WGN, false>), grid, dim3(WGM * WGN * 64), lds, s, a);
  return launch_status();
}

// register-staged, no GN prologue (bf16, 16-byte gathers): the big-tile main path
template <int BM, int BN, int WGM, int WGN>
int launch_plain(ConvArgs a, hipStream_t s, bool* fused) {
  if (a.gn_part) {  // statistics in conv_kernel's vector epilogue (P = 2) where the tile allows
    constexpr int TM = BM / WGM / 16;
    constexpr bool swz = WGM * WGN <= 8;
    constexpr bool fits = TM % 2 == 0 && (BM / 2) * (BN + 4) * 4 <= conv_lds_bytes<bf16, BM, BN, swz>();
    const bool ok = fits && stats_tile_ok<BM, BN, WGM, WGM * WGN * 64, 2>() && g_swz && a.epi_vec && epi_vec_ok(a) &&
                    a.gn_hw > 0 && a.gn_hw % 64 == 0 && a.batch == 1 && a.splits <= 1 && a.out_mode == 0;
    if (!ok) a.gn_part = nullptr;
    if (fused) *fused = ok;
  }
  dim3 grid(cdiv(a.M, BM), cdiv(a.cout, BN), a.batch);
  // measured A/B (one process, bit-identical results): the swizzled 128-B rows win on the
  // 4- and 8-wave tiles (+3-6 %) and lose on the 16-wave 256x256 tile (-16 %), which keeps the
  // padded 144-B rows
  constexpr bool SWZ_OK = (WGM * WGN <= 8);
  if (!g_swz || !SWZ_OK) {
    constexpr int lds0 = conv_lds_bytes<bf16, BM, BN, false>();
    hipLaunchKernelGGL((conv_kernel<bf16, BM, BN, WGM, WGN, true, false, false, false>), grid, dim3(WGM * WGN * 64),
                       lds0, s, a);
    return launch_status();
  }
  size_t lds = conv_lds_bytes<bf16, BM, BN>();
  // 2-deep register prefetch where the register budget allows it (<= 8 waves per block)
  constexpr bool PF = (WGM * WGN <= 8);
  if (PF && g_pf2)
    hipLaunchKernelGGL((conv_kernel<bf16, BM, BN, WGM, WGN, true, false, PF>), grid, dim3(WGM * WGN * 64), lds, s, a);
  else
    hipLaunchKernelGGL((conv_kernel<bf16, BM, BN, WGM, WGN, true, false, false>), grid, dim3(WGM * WGN * 64), lds, s,
                       a);
  return launch_status();
}

// Tile choice for the plain path: maximise (useful fraction of the padded tile grid) x (CU fill)
// x (operand reuse of the tile); the accumulation order does not depend on the choice.
int launch_plain_auto(const ConvArgs& a, hipStream_t s, int tile = -1, bool* fused = nullptr) {
  struct Cand { int bm, bn; float reuse; };
  const Cand cands[] = {{256, 256, 1.0f}, {256, 128, 0.86f}, {128, 256, 0.86f}, {128, 128, 0.72f}, {64, 128, 0.55f},
                        {128, 64, 0.55f}};
  int best = 3;
  float best_score = -1.f;
  for (int i = 0; i < 6; ++i) {
    const long tm = cdiv(a.M, cands[i].bm), tn = cdiv(a.cout, cands[i].bn);
    const float useful = (float)a.M * a.cout / ((float)tm * cands[i].bm * tn * cands[i].bn);
    const float blocks = (float)tm * tn * a.batch;
    const float fill = blocks >= 256.f ? 1.f : blocks / 256.f;
    const float score = useful * fill * cands[i].reuse;
    if (score > best_score + 1e-6f) { best_score = score; best = i; }
  }
  if (g_force_tile >= 0 && g_force_tile < 11) best = g_force_tile;
  if (tile >= 0 && tile < 11 && tile != 5) best = tile;
  switch (best) {
    case 0: return launch_plain<256, 256, 4, 4>(a, s, fused);
    case 1: return launch_plain<256, 128, 4, 2>(a, s, fused);
    case 2: return launch_plain<128, 256, 2, 4>(a, s, fused);
    case 3: return launch_plain<128, 128, 2, 2>(a, s, fused);
    case 4: return launch_plain<64, 128, 2, 2>(a, s, fused);
    case 6: return launch_plain<256, 128, 4, 4>(a, s, fused);
    case 7: return launch_plain<128, 256, 4, 4>(a, s, fused);
    case 8: return launch_plain<128, 128, 2, 4>(a, s, fused);
    case 9: return launch_plain<128, 128, 4, 4>(a, s, fused);
    case 10: return launch_plain<64, 128, 2, 4>(a, s, fused);
    default: return launch_plain<128, 64, 2, 2>(a, s, fused);
  }
}

// ============================================================================================
// Tiny-cout direct 3x3 conv (cout <= 4; the VAE decoder's conv_out 128 -> 3 with GroupNorm +
// SiLU on its input). An MFMA tile would compute 16 columns for 3 useful ones and re-apply GN on
// every gathered element, so this is a VALU (bf16 dot2) kernel instead: a 256-thread block owns a 16x16
// output patch; per 32-channel chunk the 18x18 input halo is staged once into LDS (GN affine +
// SiLU applied there, rounded to bf16 exactly like the materialised GN path), the chunk's
// weights go to LDS as fp32, and each thread accumulates its pixel's COUT outputs in fp32.
// HBM traffic ~= one read of the input (+ halo) and one write of the output.
// ============================================================================================
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

template <int COUT>
__global__ __launch_bounds__(256) void conv3x3_smallc_kernel(ConvArgs a) {
  constexpr int CC = 32, PS = 40;  // channels per chunk; LDS pixel stride in bf16 (80 B: bank spread)
  __shared__ __attribute__((aligned(16))) bf16 xs[18 * 18 * PS];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int img = blockIdx.z;
  const int oy0 = blockIdx.y * 16, ox0 = blockIdx.x * 16;
  const int cin = a.c0;
  float acc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
  const bf16* in = reinterpret_cast<const bf16*>(a.in0);
  for (int c0 = 0; c0 < cin; c0 += CC) {
    __syncthreads();
    // stage 18x18 pixels x 32 channels = 1296 chunks of 8 channels
    for (int q = tid; q < 18 * 18 * (CC / 8); q += 256) {
      const int p = q >> 2, ch = (q & 3) * 8;
      const int py = p / 18, px = p - py * 18;
      const int iy = oy0 + py - 1, ix = ox0 + px - 1;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (iy >= 0 && iy < a.h && ix >= 0 && ix < a.w && c0 + ch < cin) {
        v = *reinterpret_cast<const uint4*>(in + (((long)img * a.h + iy) * a.w + ix) * a.ld0 + c0 + ch);
        if (a.gn_ab) v = gn_apply_chunk<bf16>(v, a.gn_ab + ((long)img * cin + c0 + ch) * 2, a.gn_silu);
      }
      *reinterpret_cast<uint4*>(xs + p * PS + ch) = v;
    }
    __syncthreads();
    // weights are wave-uniform: scalar loads of the packed bf16 rows (k = (ky*3+kx)*cin + ci)
    const bf16* wp = reinterpret_cast<const bf16*>(a.weight);
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - ky * 3;
      const bf16* xp = xs + ((ty + ky) * 18 + tx + kx) * PS;
#pragma unroll
      for (int c8 = 0; c8 < CC; c8 += 8) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xp + c8);
        bf16x8 wv[COUT];
#pragma unroll
        for (int o = 0; o < COUT; ++o)
          wv[o] = *reinterpret_cast<const bf16x8*>(wp + (long)o * a.wld + t * cin + c0 + c8);
        // v_dot2_f32_bf16: two bf16 products summed into the fp32 accumulator per instruction,
        // no bf16 -> fp32 conversions (they were 4 of every 7 VALU ops of the fmaf form)
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const bf16x2 x2 = {xv[e], xv[e + 1]};
#pragma unroll
          for (int o = 0; o < COUT; ++o) {
            const bf16x2 w2 = {wv[o][e], wv[o][e + 1]};
            acc[o] = __builtin_amdgcn_fdot2_f32_bf16(x2, w2, acc[o], false);
          }
        }
      }
    }
  }
  const int oy = oy0 + ty, ox = ox0 + tx;
  if (oy >= a.ho || ox >= a.wo) return;
  const long m = ((long)img * a.ho + oy) * a.wo + ox;
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
    if (o >= a.cout) break;
    float v = acc[o];
    if (a.bias) v += a.bias[o];
    v = apply_act(v, a.act, a.act_param);
    if (a.res) v += a.out_f32 ? reinterpret_cast<const float*>(a.res)[m * a.res_ld + o]
                              : to_f32(reinterpret_cast<const bf16*>(a.res)[m * a.res_ld + o]);
    if (a.out_f32) reinterpret_cast<float*>(a.out)[m * a.out_ld + o] = v;
    else reinterpret_cast<bf16*>(a.out)[m * a.out_ld + o] = from_f32<bf16>(v);
  }
}

int launch_smallc(const ConvArgs& a, hipStream_t s) {
  dim3 grid(cdiv(a.wo, 16), cdiv(a.ho, 16), a.n);
  switch (a.cout) {
    case 1: hipLaunchKernelGGL(conv3x3_smallc_kernel<1>, grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(conv3x3_smallc_kernel<2>, grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL(conv3x3_smallc_kernel<3>, grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(conv3x3_smallc_kernel<4>, grid, dim3(256), 0, s, a); break;
  }
  return launch_status();
}

// Deterministic split-K reduction + epilogue of one 8-channel chunk: out = act(sum_z part[z] + bias + emb)
// + res, the splits summed in index order in fp32 (16-byte loads / stores); st (optional) receives the
// stored values as fp32 (the fused GroupNorm statistics of the split-K fold).
__device__ __forceinline__ void splitk_reduce_chunk(const ConvArgs& a, const float* __restrict__ part, int m, int nn,
                                                    float* st = nullptr) {
  const long slab = (long)a.M * a.cout;
  float v[8];
  {
    const float4 x0 = *reinterpret_cast<const float4*>(part + (long)m * a.cout + nn);
    const float4 x1 = *reinterpret_cast<const float4*>(part + (long)m * a.cout + nn + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
  }
  for (int z = 1; z < a.splits; ++z) {
    const float* pz = part + z * slab + (long)m * a.cout + nn;
    const float4 x0 = *reinterpret_cast<const float4*>(pz), x1 = *reinterpret_cast<const float4*>(pz + 4);
    v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w; v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
  }
  const int hw_o = a.ho * a.wo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (a.ln_rows) v[e] = ln_fold(a, m, nn + e, v[e]);
    if (a.bias) v[e] += a.bias[nn + e];
    if (a.emb) v[e] += a.emb[(long)(m / hw_o) * a.emb_ld + nn + e];
    v[e] = apply_act(v[e], a.act, a.act_param);
    if (a.res) v[e] += a.out_f32 ? reinterpret_cast<const float*>(a.res)[(long)m * a.res_ld + nn + e]
                                 : to_f32(reinterpret_cast<const bf16*>(a.res)[(long)m * a.res_ld + nn + e]);
  }
  if (a.out_f32) {
    float* o = reinterpret_cast<float*>(a.out) + (long)m * a.out_ld + nn;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = v[e];
    if (st) {
#pragma unroll
      for (int e = 0; e < 8; ++e) st[e] = v[e];
    }
  } else {
    bf16 ov[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] = from_f32<bf16>(v[e]);
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(a.out) + (long)m * a.out_ld + nn) = *reinterpret_cast<uint4*>(ov);
    if (st) {
#pragma unroll
      for (int e = 0; e < 8; ++e) st[e] = to_f32(ov[e]);
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(ConvArgs a, const float* __restrict__ part) {
  const int cp = a.cout >> 3;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)a.M * cp) return;
  const int m = (int)(i / cp), nn = (int)(i - (long)m * cp) * 8;
  splitk_reduce_chunk(a, part, m, nn);
}

// The split-K reduction folded into the producer (stream-K "fixup"): every split block of an output tile
// writes its raw fp32 partial slab, then counts itself in; the LAST block to arrive sums the tile's slabs in
// split order (splitk_reduce_chunk: the same arithmetic as the reduce kernel, so outputs are bit-identical)
// and, when the output feeds a GroupNorm, writes its canonical statistics (per channel and 64-row block,
// four 16-row groups summed sequentially, ((g0 + g1) + g2) + g3: gn_rows_partial_kernel's order). No
// separate reduce / statistics launches. lds: >= BM / 16 * BN * 8 bytes, free.
template <int BM, int BN, int NT>
__device__ __forceinline__ void splitk_fold(const ConvArgs& a, int tile, int m0, int n0, int tid, char* lds) {
  __threadfence();  // this block's partial slab is visible device-wide before it counts itself in
  __syncthreads();
  int* flag = reinterpret_cast<int*>(lds);
  if (tid == 0) *flag = atomicAdd(a.sk_cnt + tile, 1) == a.splits - 1;
  __syncthreads();
  if (!*flag) return;
  __threadfence();  // acquire: the other splits' slabs
  constexpr int CPR = BN / 8, G = BM / 16;
  if (!a.gn_part) {
    for (int c = tid; c < BM * CPR; c += NT) {
      const int m = m0 + c / CPR, nn = n0 + (c % CPR) * 8;
      if (m < a.M && nn < a.cout) splitk_reduce_chunk(a, a.sk_ws, m, nn);
    }
  } else {
    __syncthreads();  // every thread has read the flag before the statistics reuse the LDS
    float* red = reinterpret_cast<float*>(lds);  // [G][BN][2]
    for (int w = tid; w < G * CPR; w += NT) {
      const int g = w / CPR, cc = w % CPR, nn = n0 + cc * 8;
      float s1[8], s2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 16 * g + r;
        if (m < a.M && nn < a.cout) {
          float y[8];
          splitk_reduce_chunk(a, a.sk_ws, m, nn, y);
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += y[e]; s2[e] = fmaf(y[e], y[e], s2[e]); }
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(g * BN + cc * 8 + e) * 2] = s1[e];
        red[(g * BN + cc * 8 + e) * 2 + 1] = s2[e];
      }
    }
    __syncthreads();
    for (int w = tid; w < (BM / 64) * BN; w += NT) {
      const int b = w / BN, j = w % BN, nn = n0 + j;
      if (m0 + 64 * b >= a.M || nn >= a.cout) continue;
      const float* q = red + ((4 * b) * BN + j) * 2;
      float* pp = a.gn_part + 4 + ((long)((a.gn_row0 + m0 + 64 * b) / 64) * a.cout + nn) * 2;
      pp[0] = ((q[0] + q[2 * BN]) + q[4 * BN]) + q[6 * BN];
      pp[1] = ((q[1] + q[2 * BN + 1]) + q[4 * BN + 1]) + q[6 * BN + 1];
    }
    if (tid == 0 && m0 == 0 && n0 == 0) reinterpret_cast<int*>(a.gn_part)[0] = 64;  // rows per partial
  }
  if (tid == 0) a.sk_cnt[tile] = 0;  // every split has arrived: reset for the next launch
}


// ============================================================================================
// bf16 main path for cin % 64 == 0 (every UNet / VAE / compressor conv and linear but the
// 4+256-channel control input and the 224-channel context conv): LDS-DMA implicit GEMM.
//
// * A k-tile (64 consecutive k) never straddles a filter tap or a concat segment, so the im2col
//   gather address of a tile row is  pixel(row, tap) * ld + channel-block * 64 + chunk * 8:
//   the per-row part is recomputed only when the tap (or segment) changes, the channel block
//   goes into the wave-uniform soffset, and padding / image borders / M and N tails use the
//   buffer descriptor's range check (voffset = 0x80000000 reads zeros). The main loop issues
//   no address VALU at all; the register-staged kernel spent ~11 VALU per MFMA there.
// * buffer_load_dwordx4 ... lds moves each 16-byte chunk HBM/L2 -> LDS without VGPRs or
//   ds_write. One wave-instruction fills 8 LDS rows of 128 B (lane-linear); the XOR swizzle of
//   the 16-byte chunks (chunk c of row r at slot c ^ key(r)) is applied on the SOURCE side, so
//   the MFMA fragment reads (ds_read_b128) stay conflict-free.
// * S-deep LDS ring, one raw s_barrier per k-tile, counted vmcnt: S-2 tiles stay in flight
//   across the barrier (no vmcnt(0) inside the loop).
// * Blocks are remapped XCD-aware: each XCD owns a contiguous run of tile ids (N fastest), so
//   neighbouring M tiles (shared input halo) and all N tiles of an M panel share one L2.
// k order: tiles in ascending k, two 16x16x32 MFMAs per tile in ascending k (identical to
// conv_kernel), so results are bit-identical to every other bf16 path.
// ============================================================================================
constexpr unsigned kOOB = 0x80000000u;  // voffset that reads zeros (buffers are < 2 GiB)
// split-K workspace layout (rdeic_conv2d_splitk): SK_CNT int32 tile counters (zero, left zero), then the
// fp32 partial slabs
constexpr int SK_CNT = 4096;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int dma_key(int r) { return (((r >> 3) & 1) << 1) | (((r >> 1) & 1) << 2); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// one 16-byte-per-lane LDS-DMA wave-instruction: lane l's chunk lands at lds_dst + 16 * l
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_dst, unsigned voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)lds_dst, 16, (int)voff, soff, 0, 0);
}

// Per-element epilogue straight from the accumulators (tails, PixelShuffle stores, fp32 outputs
// the vector epilogue does not take).
template <int TM, int TN, int WTM, int WTN>
__device__ __forceinline__ void epilogue_scalar(const f32x4 (&acc)[TM][TN], const ConvArgs& a, int m0, int n0, int wm,
                                                int wn, int lane) {
  if (a.out_mode == 2) return;  // unreachable: the host admits GEGLU only where the vector epilogue runs
  const int lrow = lane & 15, lq = lane >> 4;
  const int hw_o = a.ho * a.wo;
  const bool of32 = a.out_f32;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WTM + i * 16 + lq * 4 + r;
      if (m >= a.M) continue;
      const int img = m / hw_o;
      int oy = 0, ox = 0;
      if (a.out_mode == 1) { const int rem = m - img * hw_o; oy = rem / a.wo; ox = rem - oy * a.wo; }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nn = n0 + wn * WTN + j * 16 + lrow;
        if (nn >= a.cout) continue;
        float v = acc[i][j][r];
        if (a.ln_rows) v = ln_fold(a, m, nn, v);
        if (a.bias) v += a.bias[nn];
        if (a.emb) v += a.emb[(long)img * a.emb_ld + nn];
        v = apply_act(v, a.act, a.act_param);
        long oidx, ridx;
        if (a.out_mode == 1) {
          const int c = nn >> 2, dy = (nn >> 1) & 1, dx = nn & 1;
          const long p = ((long)img * (2 * a.ho) + (2 * oy + dy)) * (2 * a.wo) + (2 * ox + dx);
          oidx = p * a.out_ld + c;
          ridx = p * a.res_ld + c;
        } else {
          oidx = (long)m * a.out_ld + nn;
          ridx = (long)m * a.res_ld + nn;
        }
        if (a.res) v += of32 ? reinterpret_cast<const float*>(a.res)[ridx] : to_f32(reinterpret_cast<const bf16*>(a.res)[ridx]);
        if (of32) reinterpret_cast<float*>(a.out)[oidx] = v;
        else reinterpret_cast<bf16*>(a.out)[oidx] = from_f32<bf16>(v);
      }
    }
  }
}

#ifdef RDEIC_HALO_STAMPS
// diagnostic build only (tools/halo_stamps.hip, tools/dma_stamps.hip): per-block shader-clock stamps, 8 u64 per block,
// written by thread 0 with ordinary vector stores into a buffer nothing else reads
__device__ unsigned long long* g_halo_stamps;
#define HALO_STAMP(k)                                                                      \
  do {                                                                                     \
    if (threadIdx.x == 0) g_halo_stamps[(long)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define HALO_STAMP(k) do {} while (0)
#endif

// KB: k per LDS k-tile, 64 (128-byte rows, two 16x16x32 MFMA k-steps per tile) or 32 (64-byte rows, one
// k-step: half the ring bytes, so 256x128 tiles run two blocks per CU, r05). The MFMA sequence over k is the
// same either way, so results are bit-identical across KB.
__device__ __forceinline__ int dma_key32(int r) { return (4 - ((r >> 2) & 3)) & 3; }  // 64-byte rows: slot = chunk ^ key

template <int BM, int BN, int WGM, int WGN, int S, int EP, int KB = 64>
__device__ __forceinline__ void conv_dma_body(ConvArgs a, int tiles_n, unsigned bytes0, unsigned bytes1,
                                              unsigned bytesw) {
  static_assert(KB == 64 || KB == 32, "k-tile depth");
  constexpr int NW = WGM * WGN, NT = NW * 64;
  constexpr int RB = KB * 2;                 // LDS bytes per tile row
  constexpr int RPI = 1024 / RB;             // rows per LDS-DMA wave-instruction (1 KB)
  constexpr int LPR = RB / 16;               // lanes per row
  constexpr int KSUB = KB / 32;              // 16x16x32 k-steps per tile
  constexpr int A_BYTES = BM * RB, STAGE = (BM + BN) * RB;
  constexpr int AI = BM / NW / RPI, BI = BN / NW / RPI;
  constexpr int PER = AI + BI;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(AI >= 1 && BI >= 1 && AI * RPI * NW == BM && BI * RPI * NW == BN, "tile / wave split");
  static_assert(S >= 2 && S <= 4 && PER * (S - 2) <= 63, "ring");

  extern __shared__ __attribute__((aligned(16))) char lds[];
  HALO_STAMP(0);

  const int nkt = a.nk * (64 / KB);  // a.nk counts 64-deep k-tiles
  int kt_begin = 0, kt_end = nkt;
  if (a.splits > 1) {  // split-K: blockIdx.z = k-range, raw fp32 partial sums into slab z
    const int z = blockIdx.z;
    kt_begin = min(nkt, z * a.kper);
    kt_end = min(nkt, kt_begin + a.kper);
    if (!a.sk_cnt) a.out += (long)z * a.M * a.out_ld * 4;  // (the folded form writes a.sk_ws, below)
  } else if (gridDim.z > 1) {
    const long z = blockIdx.z;
    a.in0 += z * a.in_bs * 2; a.in1 += z * a.in_bs * 2;
    a.weight += z * a.w_bs * 2;
    a.out += z * a.out_bs * (a.out_f32 ? 4 : 2);
  }
  // XCD-aware bijective remap: blocks with equal blockIdx.x % 8 share an XCD
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int mt = wgid / tiles_n, nt = wgid - mt * tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave - (wave / WGN) * WGN;
  const int g = lane / LPR, sl = lane % LPR;
  // logical chunk of this lane's slot (128-byte rows: for rows with bit3 = 0; 64-byte rows: every row)
  const int ce = KB == 64 ? sl ^ (((g >> 1) & 1) << 2) : sl ^ dma_key32(g);
  const int hw_o = a.ho * a.wo;
  const int hin = a.up2 ? 2 * a.h : a.h, win = a.up2 ? 2 * a.w : a.w;

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in1, (short)0, (int)bytes1, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);

  // A rows of this lane: r = (wave*AI + j)*RPI + g
  int r_img[AI], r_iy[AI], r_ix[AI], pix[AI];
  unsigned voa[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int m = m0 + (wave * AI + j) * RPI + g;
    if (m < a.M) {
      const int img = m / hw_o, rem = m - img * hw_o;
      const int oy = rem / a.wo, ox = rem - oy * a.wo;
      r_img[j] = img;
      r_iy[j] = oy * a.stride - a.pad_t;
      r_ix[j] = ox * a.stride - a.pad_l;
    } else {
      r_img[j] = -1; r_iy[j] = 0; r_ix[j] = 0;
    }
  }
  unsigned vob[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int nn = n0 + (wave * BI + j) * RPI + g;
    const int ch = KB == 64 ? ce ^ (((wave * BI + j) & 1) << 1) : ce;
    vob[j] = nn < a.cout ? (unsigned)nn * (unsigned)(a.wld * 2) + ch * 16 : kOOB;
  }

  // issue cursor (wave-uniform): filter tap, concat segment, 64-channel block within the segment
  const int nb0 = a.c0 / KB, nb1 = a.c1 / KB;  // k-tiles per concat segment and tap
  int i_tap = kt_begin / (nb0 + nb1), i_seg = 0, i_cb = kt_begin - i_tap * (nb0 + nb1);
  if (i_cb >= nb0) { i_seg = 1; i_cb -= nb0; }
  auto set_rows = [&]() {  // pixel of every A row for tap i_tap (-1 = zero padding)
    const int ky = i_tap / a.kw, kx = i_tap - (i_tap / a.kw) * a.kw;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      int iy = r_iy[j] + ky, ix = r_ix[j] + kx;
      const bool ok = r_img[j] >= 0 && (unsigned)iy < (unsigned)hin && (unsigned)ix < (unsigned)win;
      if (a.up2) { iy >>= 1; ix >>= 1; }
      pix[j] = ok ? (r_img[j] * a.h + iy) * a.w + ix : -1;
    }
  };
  auto set_voff = [&]() {  // byte offsets for the current segment
    const unsigned ldb = (unsigned)(i_seg ? a.ld1 : a.ld0) * 2u;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int ch = KB == 64 ? ce ^ (((wave * AI + j) & 1) << 1) : ce;
      voa[j] = pix[j] >= 0 ? (unsigned)pix[j] * ldb + ch * 16 : kOOB;
    }
  };
  set_rows();
  set_voff();

  auto issue = [&](int kt, int slot) {
    char* sb = lds + slot * STAGE;
    const __amdgpu_buffer_rsrc_t rsa = i_seg ? rs1 : rs0;
    const int soa = i_cb * RB;
#pragma unroll
    for (int j = 0; j < AI; ++j)
      dma16(rsa, sb + (wave * AI + j) * 1024, voa[j], soa);
#pragma unroll
    for (int j = 0; j < BI; ++j) dma16(rsw, sb + A_BYTES + (wave * BI + j) * 1024, vob[j], kt * RB);
    // advance the cursor
    if (++i_cb == (i_seg ? nb1 : nb0)) {
      i_cb = 0;
      if (i_seg == 0 && nb1 > 0) {
        i_seg = 1;
      } else {
        i_seg = 0;
        ++i_tap;
        if (i_tap < a.kh * a.kw) set_rows();
      }
      set_voff();
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lrow = lane & 15, lq = lane >> 4;
  const int rkey = KB == 64 ? dma_key(lrow) : dma_key32(lrow);
  const int nk = kt_end - kt_begin;

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(kt_begin + s, s);
  HALO_STAMP(1);

  for (int t = 0; t < nk; ++t) {
    if constexpr (S == 2) {
      wait_vm<0>();
    } else if constexpr (S == 3) {
      if (t + 1 < nk) wait_vm<PER>(); else wait_vm<0>();
    } else {
      if (t + 2 < nk) wait_vm<2 * PER>(); else if (t + 1 < nk) wait_vm<PER>(); else wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (t + S - 1 < nk) issue(kt_begin + t + S - 1, (t + S - 1) % S);
    const int cur = t % S;
    const char* Ab = lds + cur * STAGE + (wm * WTM + lrow) * RB;
    const char* Bb = lds + cur * STAGE + A_BYTES + (wn * WTN + lrow) * RB;
#pragma unroll
    for (int s = 0; s < KSUB; ++s) {
      const int so = ((s * 4 + lq) ^ rkey) * 16;
      bf16x8 bfv[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(Bb + j * 16 * RB + so);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(Ab + i * 16 * RB + so);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  HALO_STAMP(2);
  // split-K folded into the producer: partial slab, then the last split reduces (the split launches run the
  // heuristic's 4- and 8-wave tiles, launch_dma_auto(tile -1); compiled only there: register budget)
  if constexpr (WGM * WGN <= 8) if (a.splits > 1 && a.sk_cnt) {
    ConvArgs p = a;
    p.out = reinterpret_cast<char*>(a.sk_ws + (long)blockIdx.z * a.M * a.cout);
    p.out_ld = a.cout; p.out_f32 = 1; p.out_mode = 0;
    p.bias = nullptr; p.emb = nullptr; p.act = 0; p.res = nullptr; p.gn_part = nullptr; p.ln_rows = nullptr;
    bool done = false;
    if constexpr (TM % EP == 0 && (BM / EP) * (BN + 4) * 4 <= S * STAGE) {
      if (p.epi_vec && epi_vec_ok(p)) {
        epilogue_vec<BM, BN, WGM, WGN, NT, EP>(acc, p, m0, n0, wm, wn, lane, tid, lds);
        done = true;
      }
    }
    if (!done) epilogue_scalar<TM, TN, WTM, WTN>(acc, p, m0, n0, wm, wn, lane);
    splitk_fold<BM, BN, NT>(a, wgid, m0, n0, tid, lds);
    HALO_STAMP(3);
    return;
  }
  if constexpr (TM % EP == 0 && (BM / EP) * (BN + 4) * 4 <= S * STAGE) {
    if ((a.epi_vec || a.out_mode == 2) && epi_vec_ok(a)) {
      epilogue_vec<BM, BN, WGM, WGN, NT, EP>(acc, a, m0, n0, wm, wn, lane, tid, lds);
      HALO_STAMP(3);
      return;
    }
  }
  epilogue_scalar<TM, TN, WTM, WTN>(acc, a, m0, n0, wm, wn, lane);
  HALO_STAMP(3);
}

// Kernel entry points. Residency: 1024-thread blocks need <= 80 SGPRs for two blocks per CU (the
// hardware admits floor(800 / (ceil(sgpr / 16) * 16 + 16)) waves per SIMD; MI355X_MICROARCH.md
// "Residency"), so the 16-wave 128x128 tile (64 KB of LDS: two blocks fit) is built with its
// SGPR budget capped; the others keep the compiler's allocation.
template <int BM, int BN, int WGM, int WGN, int S, int EP, int KB = 64>
__global__ __launch_bounds__(WGM * WGN * 64) void conv_dma_kernel(ConvArgs a, int tiles_n, unsigned bytes0,
                                                                  unsigned bytes1, unsigned bytesw) {
  conv_dma_body<BM, BN, WGM, WGN, S, EP, KB>(a, tiles_n, bytes0, bytes1, bytesw);
}

template <int BM, int BN, int WGM, int WGN, int S, int EP, int KB = 64>
__global__ __launch_bounds__(WGM * WGN * 64) __attribute__((amdgpu_num_sgpr(80))) void conv_dma_kernel_2pc(
    ConvArgs a, int tiles_n, unsigned bytes0, unsigned bytes1, unsigned bytesw) {
  conv_dma_body<BM, BN, WGM, WGN, S, EP, KB>(a, tiles_n, bytes0, bytes1, bytesw);
}

// two 8-wave blocks per CU (the 32-deep k-tile form): 4 waves per SIMD, <= 128 VGPRs
template <int BM, int BN, int WGM, int WGN, int S, int EP, int KB>
__global__ __launch_bounds__(WGM * WGN * 64) __attribute__((amdgpu_waves_per_eu(4, 4))) void conv_dma_kernel_2b(
    ConvArgs a, int tiles_n, unsigned bytes0, unsigned bytes1, unsigned bytesw) {
  conv_dma_body<BM, BN, WGM, WGN, S, EP, KB>(a, tiles_n, bytes0, bytes1, bytesw);
}

// DMA-path eligibility: bf16, 16-byte-aligned 64-channel blocks, every buffer < 2 GiB.
bool dma_ok(const rdeic_conv_desc* d, const ConvArgs& a, unsigned& b0, unsigned& b1, unsigned& bw) {
  if (d->dtype != 1 || d->gn_ab || (d->c0 % 64) || (d->c1 % 64) || (d->ld0 % 8) || ((uintptr_t)d->in0 % 16)) return false;
  if (d->c1 && ((d->ld1 % 8) || ((uintptr_t)d->in1 % 16))) return false;
  if (d->wld % 64 || a.ktot % 64) return false;
  const long pix = (long)d->n * d->h * d->w;
  const long e0 = ((pix - 1) * d->ld0 + d->c0) * 2 + (a.batch - 1) * d->in_bs * 2;
  const long e1 = d->c1 ? ((pix - 1) * d->ld1 + d->c1) * 2 : 16;
  const long ew = (long)d->cout * d->wld * 2 + (a.batch - 1) * d->w_bs * 2;
  if (e0 >= (1l << 31) || e1 >= (1l << 31) || ew >= (1l << 31)) return false;
  if (a.batch > 1 && (d->in_bs % 8 || d->w_bs % 8)) return false;
  // batched operands are addressed from the per-z base: the descriptor covers one slice
  b0 = (unsigned)(((pix - 1) * d->ld0 + d->c0) * 2);
  b1 = (unsigned)e1;
  bw = (unsigned)((long)d->cout * d->wld * 2);
  return true;
}

// Whether the kernel's vector epilogue runs for these arguments (the compile-time part mirrors the
// `if constexpr` in conv_dma_kernel).
template <int BM, int BN, int WGM, int WGN, int S, int EP, int KB = 64>
bool dma_vec_epilogue(const ConvArgs& a) {
  constexpr int TM = BM / WGM / 16;
  constexpr bool fits = TM % EP == 0 && (BM / EP) * (BN + 4) * 4 <= S * (BM + BN) * KB * 2;
  return fits && (a.epi_vec || a.out_mode == 2) && epi_vec_ok(a);
}

// gn_hw: pixels per image of the GroupNorm the statistics feed; the 64-row partial blocks must not
// straddle two images, and the epilogue must be the vector one with a statistics-capable tile.
template <int BM, int BN, int WGM, int WGN, int S, int EP, int KB = 64>
int launch_dma(ConvArgs a, unsigned b0, unsigned b1, unsigned bw, hipStream_t s, int gn_hw, bool* fused) {
  if (a.gn_part) {
    const bool ok = a.splits > 1 && a.sk_cnt  // the split-K fold's last block writes them
                        ? a.batch == 1 && a.out_mode == 0 && gn_hw > 0 && gn_hw % 64 == 0 && BM % 64 == 0
                        : a.splits <= 1 && a.batch == 1 && a.out_mode == 0 && gn_hw > 0 && gn_hw % 64 == 0 &&
                              stats_tile_ok<BM, BN, WGM, WGM * WGN * 64, EP>() &&
                              dma_vec_epilogue<BM, BN, WGM, WGN, S, EP, KB>(a);
    if (!ok) a.gn_part = nullptr;
    if (fused) *fused = ok;
  }
  const int tn = cdiv(a.cout, BN);
  const long tiles = (long)cdiv(a.M, BM) * tn;
  dim3 grid((unsigned)tiles, 1, a.splits > 1 ? a.splits : a.batch);
  constexpr int lds = S * (BM + BN) * KB * 2;
  if constexpr (WGM * WGN == 16 && lds <= 80 * 1024)
    hipLaunchKernelGGL((conv_dma_kernel_2pc<BM, BN, WGM, WGN, S, EP, KB>), grid, dim3(WGM * WGN * 64), lds, s, a, tn,
                       b0, b1, bw);
  else if constexpr (KB == 32 && WGM * WGN == 8 && lds <= 80 * 1024)
    hipLaunchKernelGGL((conv_dma_kernel_2b<BM, BN, WGM, WGN, S, EP, KB>), grid, dim3(WGM * WGN * 64), lds, s, a, tn,
                       b0, b1, bw);
  else
    hipLaunchKernelGGL((conv_dma_kernel<BM, BN, WGM, WGN, S, EP, KB>), grid, dim3(WGM * WGN * 64), lds, s, a, tn, b0,
                       b1, bw);
  return launch_status();
}

// DMA tiles (ids 20..39; BMxBN/waves, S = ring depth):
//   20 256x256/8 S2, 21 256x128/8 S3, 22 128x256/8 S3, 23 128x128/4 S3, 24 128x128/4 S2,
//   25 128x128/8 S2, 26 64x128/4 S3, 27 128x128/8 S3, 28 256x128/8 S2, 29 128x256/8 S2,
//   30 64x128/4 S2, 31 128x64/4 S2, 32 256x256/16 S2, 33 256x128/16 S2, 34 128x128/16 S2,
//   35 512x128/16 S2 (64x64 per wave at cout = 128: the whole 160 KB of LDS, one block per CU),
//   36 64x128/8 S2 (32x32 per wave: twice the waves of tile 30 on grids of ~256 tiles),
//   37 128x160/4 S2 and 38 64x160/4 S2 (N = 320 layers: two N tiles, no padded columns),
//   39 256x128/8 S3 with 32-deep k-tiles (72 KB: two blocks per CU, so one block's epilogue overlaps the
//   other's k-loop; for the short-K transformer linears, r05)
// (r05: 128x320/8 S2, 64 x 80 per wave, the whole N = 320 in one tile so the 64^2 3x3 convs gather their im2col
//  A rows once instead of once per 160-wide N tile of tile 37: equal to tile 37 there (778 / 776, 1049 / 1031,
//  1120 / 1120 TF), slower on the 1280-channel levels: profiles/r05_tile_128x320.jsonl; the 4.9x PMC
//  re-read of tile 37 is absorbed by the L2 / MALL, not a bound)
// (r05: 256x256/16 S4 with 32-deep k-tiles, tile 32's 128 KB as four slots, ran 2-5% slower than tile 32 on
//  every linear and 3x3 conv shape: profiles/r05_tile_s4_kb32.jsonl)
// (r04: 16-wave S3 / S4 rings for the short-K linears, 256x128 S3, 128x256 S3, 128x128 S4, were
//  slower than these S2 tiles on every transformer linear: profiles/r04_linear_tiles.jsonl)
// Measured (tools/dma_bench.py, one MI355X): 32 is best where a 256x256 grid fills the chip
// without padding waste (1.19-1.27 PF on the VAE 512-channel layers), 25 on the rest with >= 256
// 128x128 tiles, the 4-wave 64x128 tile when even that grid cannot fill the chip; 34 often wins
// on short-K linears (the committed per-shape table rdeic_amd/conv_tiles.json picks, measured by
// tools/tune_tiles.py; shapes missing from it use this heuristic).
int launch_dma_auto(const ConvArgs& a, unsigned b0, unsigned b1, unsigned bw, hipStream_t s, int tile,
                    int gn_hw = 0, bool* fused = nullptr) {
  if (tile < 20 || tile > 39) {
    const long zb = a.splits > 1 ? a.splits : a.batch;
    const long t128 = (long)cdiv(a.M, 128) * cdiv(a.cout, 128) * zb;
    const long t256 = (long)cdiv(a.M, 256) * cdiv(a.cout, 256) * zb;
    const float useful256 = (float)a.M * a.cout / ((float)cdiv(a.M, 256) * 256 * cdiv(a.cout, 256) * 256);
    tile = (t256 >= 256 && useful256 >= 0.9f) ? 32 : t128 >= 256 ? 25 : 26;
  }
  switch (tile) {
    case 20: return launch_dma<256, 256, 2, 4, 2, 4>(a, b0, b1, bw, s, gn_hw, fused);
    case 21: return launch_dma<256, 128, 4, 2, 3, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 22: return launch_dma<128, 256, 2, 4, 3, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 24: return launch_dma<128, 128, 2, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 25: return launch_dma<128, 128, 2, 4, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 26: return launch_dma<64, 128, 2, 2, 3, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 27: return launch_dma<128, 128, 2, 4, 3, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 28: return launch_dma<256, 128, 4, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 29: return launch_dma<128, 256, 2, 4, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 30: return launch_dma<64, 128, 2, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 31: return launch_dma<128, 64, 2, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 32: return launch_dma<256, 256, 4, 4, 2, 4>(a, b0, b1, bw, s, gn_hw, fused);
    case 33: return launch_dma<256, 128, 4, 4, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 34: return launch_dma<128, 128, 4, 4, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 35: return launch_dma<512, 128, 8, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 36: return launch_dma<64, 128, 2, 4, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 37: return launch_dma<128, 160, 2, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 38: return launch_dma<64, 160, 2, 2, 2, 2>(a, b0, b1, bw, s, gn_hw, fused);
    case 39: return launch_dma<256, 128, 4, 2, 3, 2, 32>(a, b0, b1, bw, s, gn_hw, fused);
    default: return launch_dma<128, 128, 2, 2, 3, 2>(a, b0, b1, bw, s, gn_hw, fused);
  }
}

int make_args(const rdeic_conv_desc* d, ConvArgs& a, bool& vec);

// Images are independent in a conv, so a launch whose buffers exceed the 2 GiB reach of a
// 32-bit buffer offset runs the DMA kernel over groups of images (same per-pixel arithmetic,
// bit-identical). Returns -1 when the DMA path does not apply.
int dma_grouped(const rdeic_conv_desc* d, int tile, int splits, float* ws, hipStream_t s, bool* fused = nullptr) {
  ConvArgs a;
  bool vec = false;
  if (make_args(d, a, vec) != RDEIC_OK || !vec) return -1;
  unsigned b0, b1, bw;
  if (dma_ok(d, a, b0, b1, bw)) {
    if (splits > 1) {  // folded split-K: the real epilogue stays in the arguments, partial slabs after the counters
      a.splits = splits; a.kper = (a.nk + splits - 1) / splits;
      a.sk_cnt = reinterpret_cast<int*>(ws);
      a.sk_ws = ws + SK_CNT;
      // the fold is compiled into the 4- and 8-wave tiles only (conv_dma_body): 128x128 / 8 waves when the
      // split grid fills the chip, else 64x128 / 4 waves (the heuristic's small-grid choices)
      tile = (long)cdiv(a.M, 128) * cdiv(a.cout, 128) * splits >= 256 ? 25 : 26;
    }
    return launch_dma_auto(a, b0, b1, bw, s, tile, d->gn_hw, fused);
  }
  if (splits > 1 || d->batch > 1 || d->n <= 1) return -1;
  // per-image sizes (bytes); pick the largest image group that fits
  const long ipix = (long)d->h * d->w;
  const long per0 = ipix * d->ld0 * 2, per1 = d->c1 ? ipix * d->ld1 * 2 : 0;
  const long per = per0 > per1 ? per0 : per1;
  const int g = (int)(((1l << 31) - 1) / per);
  if (g < 1) return -1;
  rdeic_conv_desc e = *d;
  const int osz = (d->out_f32 || d->dtype == 0) ? 4 : 2;
  const long opix = d->out_mode == 1 ? 4l * d->ho * d->wo : (long)d->ho * d->wo;
  for (int i0 = 0; i0 < d->n; i0 += g) {
    e.n = d->n - i0 < g ? d->n - i0 : g;
    e.in0 = (const char*)d->in0 + i0 * per0;
    e.in1 = d->in1 ? (const char*)d->in1 + i0 * per1 : nullptr;
    e.out = (char*)d->out + i0 * opix * d->out_ld * osz;
    e.res = d->res ? (const char*)d->res + i0 * opix * d->res_ld * osz : nullptr;
    e.emb = d->emb ? d->emb + (long)i0 * d->emb_ld : nullptr;
    e.ln_rows = d->ln_rows ? d->ln_rows + 2l * i0 * d->ho * d->wo : nullptr;
    ConvArgs ea;
    if (make_args(&e, ea, vec) != RDEIC_OK || !vec || !dma_ok(&e, ea, b0, b1, bw)) return -1;
    ea.gn_row0 = i0 * d->ho * d->wo;
    bool f = false;
    const int rc = launch_dma_auto(ea, b0, b1, bw, s, tile, d->gn_hw, &f);
    if (rc != RDEIC_OK) return rc;
    if (fused) *fused = (i0 == 0 ? f : (*fused && f));
  }
  return RDEIC_OK;  // *fused false if any group could not fuse: the caller recomputes the statistics
}

// ============================================================================================
// 3x3 / stride-1 / pad-1 conv on a halo strip, with the input GroupNorm affine (+ SiLU) applied
// ONCE per element in LDS: the VAE ResnetBlock's norm -> nonlinearity -> conv
// (ldm/modules/diffusionmodules/model.py:131-151, Normalize + nonlinearity + conv1 / conv2).
//
// The im2col path (conv_dma_kernel) re-stages every input element for each of the 9 taps, so a
// GroupNorm + SiLU fused into its staging costs 9x the VALU of the element-wise pass and loses to
// materialising silu(a x + b) in HBM (one read + one write of the activation). Here a tile is an
// image block of TR x TC = 4 x 64 output pixels x 128 output channels; per 32-channel block the
// (TR + 2) x (TC + 2) halo of the RAW input is DMA'd to LDS once (buffer_load ... lds, 25 x 1 KB
// pieces, zeros outside the image from the descriptor's range check), transformed in place
// (x * a + b, then x * rcp(1 + e^-x): exactly the bf16 values rdeic_groupnorm_apply writes; halo
// pixels outside the image stay zero = the conv's zero padding of the normalised tensor) and then
// read by all 9 taps. The 32-channel weight slice of each tap streams through a 3-deep ring.
// Per step (tap) a wave (one output row, 64 channels) issues 16 v_mfma_f32_16x16x32_bf16.
// LDS 78 KB -> two blocks per CU, so one block's epilogue overlaps the other's main loop.
// Swizzle: 16-byte chunk q of halo pixel / weight row s lives at slot q ^ (((s >> 2) & 1) << 1),
// conflict-free for every ds_read_b128 lane group at any pixel offset (tap shift).
// k order: 32-channel block major, tap minor — fixed per shape (deterministic, batch-invariant),
// not the im2col kernels' (tap, 64-channel) order, so results differ from them by fp32 rounding.
// The epilogue is epilogue_vec (bias / residual / GroupNorm statistics of the output) with the
// tile's 64-pixel wave rows mapped to their image rows.
// ============================================================================================
namespace halo {
constexpr int TR = 4, TC = 64;            // output rows / columns per tile
constexpr int HR = TR + 2, HC = TC + 2;   // halo rows / columns
constexpr int HPIX = HR * HC;             // 396 halo pixels
constexpr int NPIECE = (HPIX * 4 + 63) / 64;  // 1 KB DMA pieces per halo (25)
constexpr int HBYTES = NPIECE * 1024;     // one halo buffer (the last piece's tail slots read zeros)
constexpr int BN = 128, NW = 8, NT = NW * 64;
constexpr int BBYTES = BN * 64;           // one tap's 32-channel weight slice
constexpr int NB = 3;                     // weight ring depth
constexpr int AB_MAX = 512;               // input channels whose GroupNorm affine fits the LDS table
constexpr int LDS = 2 * HBYTES + NB * BBYTES + AB_MAX * 8;
static_assert(LDS <= 80 * 1024, "two blocks per CU");
static_assert((TR * TC / 2) * (BN + 4) * 4 <= LDS, "epilogue parking (two passes)");
__device__ __forceinline__ int sw(int s) { return ((s >> 2) & 1) << 1; }

struct Rows {  // tile row r (wave row r / 64, column r % 64) -> output pixel
  int base, W;
  __device__ __forceinline__ int operator()(int r) const { return base + (r >> 6) * W + (r & 63); }
};

// Epilogue LDS plan (four passes of 64 tile rows: one 16-row fragment per wave row): a parked pass
// (64 x (BN + 4) fp32) and two 16 KB residual buffers. Pass 0's residual is DMA'd during the main loop's
// last taps into the halo buffer the last channel block does not read, so the layout depends on the
// parity of the channel-block count.
constexpr int PK_BYTES = 64 * (BN + 4) * 4;  // 33,792
constexpr int RES_BYTES = 64 * BN * 2;       // 16,384: 64 pixels x 128 bf16
constexpr int RING_END = 2 * HBYTES + NB * BBYTES;
static_assert(HBYTES + PK_BYTES + RES_BYTES <= RING_END, "epilogue plan, even channel blocks");
static_assert(HBYTES + RES_BYTES + PK_BYTES <= RING_END, "epilogue plan, odd channel blocks");
static_assert(RES_BYTES <= HBYTES, "pass-0 residual in the free halo buffer");
__device__ __forceinline__ int res_off(int parity, int p) {  // residual buffer of pass p
  return ((p & 1) == 0) ? (parity ? HBYTES : 0) : (parity ? 0 : HBYTES + PK_BYTES);
}
__device__ __forceinline__ int park_off(int parity) { return parity ? HBYTES + RES_BYTES : HBYTES; }
}  // namespace halo

// The halo conv's epilogue for bf16 outputs without emb / activation (every VAE ResnetBlock conv):
// out = (acc + bias) + residual, rounded to bf16, in four passes of 64 tile rows. Per pass: the
// accumulators of fragment row p are parked in LDS; the residual rows of the pass are already in LDS
// (LDS-DMA issued one pass ahead, so its HBM latency overlaps the previous pass instead of stalling
// every chunk); each thread keeps the bias of its 8 channels in registers and handles 2 chunks
// (16-byte LDS reads, residual read, one 16-byte store each). Arithmetic and rounding are epilogue_vec's,
// so outputs are bit-identical to it. Fused GroupNorm statistics (a.gn_part) keep the canonical order:
// pass p is 16-row group p of every 64-row block (one wave row), summed by a column scan of the stored
// values, and ((g0 + g1) + g2) + g3 at the end.
// The residual rows of epilogue pass p (NW x 8 pixels x 128 channels) by LDS-DMA: this wave's pieces
// q = wave, wave + NW; lane i of piece q brings pass row 4q + i / 16 (wave row (4q + i / 16) / 16, pixel
// p * 16 + (4q + i / 16) % 16 of it), channels n0 + 8 (i % 16) .. + 7. Offsets are recomputed at each use
// (not kept live).
template <int NW>
__device__ __forceinline__ void halo_res_dma(__amdgpu_buffer_rsrc_t rsr, char* dst, int base, int W, int res_ld,
                                             int n0, int wave, int lane, int p) {
  int l = lane;
  asm volatile("" : "+v"(l));  // keep the offsets here, not hoisted into the main loop's live set
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int pr = 4 * (wave + NW * k) + (l >> 4);
    const unsigned vo = (unsigned)(base + (pr >> 4) * W + (pr & 15)) * (unsigned)(res_ld * 2) + (unsigned)((l & 15) * 16);
    dma16(rsr, dst + (wave + NW * k) * 1024, vo, p * 16 * res_ld * 2 + n0 * 2);
  }
}

// The halo convs' epilogue for bf16 outputs without emb / activation (every VAE ResnetBlock conv):
// out = (acc + bias) + residual, rounded to bf16, in four passes (one 16-row fragment per wave row, NW x 8
// tile rows). Per pass: the accumulators of fragment row p are parked in LDS (park); the residual rows of
// the pass are already in LDS (r0 / r1 alternate; LDS-DMA issued one pass ahead, right after the barrier that
// frees its buffer, so its latency overlaps the previous pass and this pass's park; pass 0's is issued by the
// caller during its last taps); each thread keeps the bias of its 8 channels in registers and handles 2 chunks (16-byte LDS reads,
// residual read, one 16-byte store each). Arithmetic and rounding are epilogue_vec's, so outputs are
// bit-identical to it. Fused GroupNorm statistics (a.gn_part) keep the canonical order: pass p is 16-row
// group p of every 64-row block (one wave row), summed by a column scan of the stored values, and
// ((g0 + g1) + g2) + g3 at the end.
template <int NW, bool RES>
__device__ __forceinline__ void halo_epilogue(const f32x4 (&acc)[4][4], const ConvArgs& a, int n0, int wm, int wn,
                                              int tid, char* lds, int base, int W, int park, int r0, int r1,
                                              __amdgpu_buffer_rsrc_t rsr, int wave) {
  constexpr int BN = 128, SDW = BN + 4, NT = NW * 64;
  // laundered: every address below is derived after the main loop (hoisted, they would sit in the
  // 128-VGPR main loop's live set and spill)
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int lr = lane & 15, lq = lane >> 4;
  float* const L = reinterpret_cast<float*>(lds + park);
  constexpr bool has_res = RES;  // a.res != nullptr, a compile-time split (no branch around the residual loads,
                                 // whose vmcnt scoreboard the compiler would otherwise merge over both paths)
  const bool st = a.gn_part != nullptr;
  const int cc = tid & 15;  // this thread's 8 channels n0 + 8 cc (NT % 16 == 0: the same in every chunk)
  const int nn = n0 + cc * 8;
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = 0.f;
  if (a.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + nn), b1 = *reinterpret_cast<const float4*>(a.bias + nn + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w; bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  float sg[4], qg[4];
  // LDS-only barriers (__syncthreads() would also drain vmcnt(0): the previous pass's output stores and the
  // next pass's residual loads). The residual of pass 0 is in LDS (r0, LDS-DMA'd by the caller during its
  // last taps); passes 1-3 load theirs into registers one pass ahead (an LDS-DMA here would make the compiler
  // drain vmcnt(0) before the next LDS read, i.e. wait out the prefetch at once).
  auto bar = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto res_rows = [&](int p, uint4 (&dst)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = (tid >> 4) + (NT / 16) * k;
      const long m = base + (pr >> 4) * W + p * 16 + (pr & 15);
      // a buffer load through the residual's descriptor (a plain load here compiled to flat_load, which counts
      // in lgkmcnt too, so every LDS barrier would wait for it)
      typedef unsigned u4v __attribute__((ext_vector_type(4)));
      const u4v r = __builtin_amdgcn_raw_buffer_load_b128(rsr, (unsigned)(m * a.res_ld + nn) * 2u, 0, 0);
      dst[k] = uint4{r.x, r.y, r.z, r.w};
    }
  };
  uint4 rbuf[2][2];  // [pass & 1][chunk]: pass p reads rbuf[p & 1], pass p + 1's rows load into the other
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    bar();  // p = 0: the main loop's LDS reads are done; else: the previous pass's readers are
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(wm * 16 + lq * 4 + r) * SDW + wn * 64 + j * 16 + lr] = acc[p][j][r];
    if (has_res && p == 0) wait_vm<0>();  // this wave's pass-0 residual pieces (nothing else is in flight)
    bar();
    // consumed one pass later; pass 0 issues pass 1's after its LDS residual reads (the compiler drains
    // vmcnt(0) before the first read of LDS-DMA'd data)
    if (has_res && p > 0 && p + 1 < 4) res_rows(p + 1, rbuf[(p + 1) & 1]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = (tid >> 4) + (NT / 16) * k;  // pass row: wave row pr / 16, row p * 16 + pr % 16 of it
      const long m = base + (pr >> 4) * W + p * 16 + (pr & 15);
      const float4 x0 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8 + 4);
      float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias[e];
      if (has_res) {
        bf16x8 rv;
        if (p == 0) rv = *reinterpret_cast<const bf16x8*>(lds + r0 + pr * 256 + cc * 16);
        else *reinterpret_cast<uint4*>(&rv) = rbuf[p & 1][k];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
      }
      bf16x8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.out) + m * a.out_ld + nn) = ov;
      if (st) {
        *reinterpret_cast<float4*>(L + pr * SDW + cc * 8) = make_float4((float)ov[0], (float)ov[1], (float)ov[2], (float)ov[3]);
        *reinterpret_cast<float4*>(L + pr * SDW + cc * 8 + 4) = make_float4((float)ov[4], (float)ov[5], (float)ov[6], (float)ov[7]);
      }
    }
    if (has_res && p == 0) res_rows(1, rbuf[1]);
    if (st) {  // column scan: thread (wave row b, channel j), the 16 rows of group p, in row order
      bar();
      const int b = tid >> 7, j = tid & 127;
      const float* col = L + (b * 16) * SDW + j;
      float y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) y[r] = col[r * SDW];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s1 += y[r]; s2 = fmaf(y[r], y[r], s2); }
      sg[p] = s1;
      qg[p] = s2;
    }
  }
  if (st) {
    const int b = tid >> 7, j = tid & 127;
    float* pp = a.gn_part + 4 + ((long)((a.gn_row0 + base + b * W) / 64) * a.cout + n0 + j) * 2;
    pp[0] = ((sg[0] + sg[1]) + sg[2]) + sg[3];
    pp[1] = ((qg[0] + qg[1]) + qg[2]) + qg[3];
    if (tid == 0 && base == 0 && n0 == 0) reinterpret_cast<int*>(a.gn_part)[0] = 64;  // rows per partial
  }
}

// GN: 0 plain conv, 1 GroupNorm affine on the input, 2 affine + SiLU (compile-time: no per-element branch);
// FE: the fast epilogue (halo_epilogue: bf16 out, no emb / activation), else epilogue_vec
template <int GN, bool FE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void conv3x3_halo_kernel(ConvArgs a, int tiles_x, int tiles_y, unsigned bytes0,
                                                               unsigned bytesw) {
  using namespace halo;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const hbuf = lds;
  char* const bbuf = lds + 2 * HBYTES;
  float* const abl = reinterpret_cast<float*>(lds + 2 * HBYTES + NB * BBYTES);
  HALO_STAMP(0);
#ifdef RDEIC_HALO_STAMPS
  if (threadIdx.x == 0) {
    g_halo_stamps[(long)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    g_halo_stamps[(long)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  const int tn = a.cout / BN;
  // XCD-aware bijective remap (as conv_dma_body): an XCD owns a contiguous run of tile ids, the N
  // tiles of one image block adjacent (they share its halo through L2)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
  const int nt = wgid % tn;
  int sp = wgid / tn;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * TC, n0 = nt * BN;
  const int H = a.h, W = a.w, cin = a.c0;
  const int ncb = cin >> 5, U = ncb * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wave = (output row, 64-channel half)

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);

  // halo pieces of this wave: w, w + 8, w + 16 and (wave 0) 24; the other waves repeat piece w + 16
  // as their 4th (same bytes to the same slots), so every wave issues 4 and vmcnt stays uniform
  unsigned hvo[4];
  int hpo[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = (wave + 8 * k < NPIECE) ? wave + 8 * k : wave + 16;
    const int sl = p * 16 + (lane >> 2), ph = lane & 3;
    hpo[k] = p * 1024;
    hvo[k] = kOOB;
    if (sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        hvo[k] = (unsigned)((img * H + iy) * W + ix) * (unsigned)(a.ld0 * 2) + (unsigned)((ph ^ sw(sl)) * 16);
    }
  }
  // residual pieces of the epilogue (halo_epilogue): this wave's pieces q = wave, wave + 8 of every pass;
  // lane i of piece q brings pass row 4q + i / 16 (wave row (4q + i / 16) / 16), chunk i % 16
  const bool res_dma = FE && a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res_dma ? a.res : a.in0), (short)0, res_dma ? (int)((long)(img * H + H) * W * a.res_ld * 2) : 0, 0x00020000);
  const int parity = (cin >> 5) & 1;
  // weight rows of this wave: n = 16 wave + lane / 4, chunk lane % 4
  unsigned bvo;
  {
    const int n = wave * 16 + (lane >> 2), ph = lane & 3;
    bvo = (n0 + n < a.cout) ? (unsigned)(n0 + n) * (unsigned)(a.wld * 2) + (unsigned)((ph ^ sw(n)) * 16) : kOOB;
  }
  auto issue_halo = [&](int cb) {
    char* dst = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int k = 0; k < 4; ++k) dma16(rs0, dst + hpo[k], hvo[k], cb * 64);
  };
  auto issue_b = [&](int u) {
    const int cb = u / 9, t = u - (u / 9) * 9;
    dma16(rsw, bbuf + (u % NB) * BBYTES + wave * 1024, bvo, (t * cin + cb * 32) * 2);
  };
  // The in-place GroupNorm (+ SiLU) of a halo: every wave transforms exactly the chunks its own
  // DMA pieces brought in (one 16-byte chunk per lane per piece; the duplicate 4th piece of waves
  // 1..7 is skipped), right after its own counted vmcnt: no barrier between landing and transform.
  // Pixels outside the image (the conv's zero padding of the normalised tensor) stay zero.
  // per piece k: bit k = this lane's chunk is inside the image (transform it), bits 4 + 2k: its
  // logical channel chunk (one VGPR for all four pieces)
  unsigned hinfo = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = (wave + 8 * k < NPIECE) ? wave + 8 * k : -1;
    const int sl = (p < 0 ? 0 : p) * 16 + (lane >> 2);
    if (p >= 0 && hvo[k] != kOOB) hinfo |= 1u << k;
    hinfo |= (unsigned)((lane & 3) ^ sw(sl)) << (4 + 2 * k);
  }
  // piece k of this wave's halo pieces (one 16-byte chunk per lane), transformed in place
  auto transform_piece = [&](int cb, int k) {
    if (!(hinfo & (1u << k))) return;
    char* hb = hbuf + (cb & 1) * HBYTES + lane * 16 + hpo[k];
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(hb);
    const int ch = (hinfo >> (4 + 2 * k)) & 3;
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb * 32 + ch * 8) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];  // (a, b) of the chunk's 8 channels
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = __builtin_fmaf((float)v[e], av[e], bv[e]);
      if constexpr (GN == 2) x *= __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      o[e] = (bf16)x;
    }
    *reinterpret_cast<bf16x8*>(hb) = o;
  };
  auto transform = [&](int cb) {
#pragma unroll
    for (int k = 0; k < 4; ++k) transform_piece(cb, k);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier releases readers
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: the image's GroupNorm (a, b) table (cin x 8 bytes, <= 4 KB) comes by LDS-DMA together with
  // the first halo and weight slices, so their latencies overlap. Each wave issues ONE table piece (waves
  // past the table's pieces repeat piece 0: same bytes to the same slots), keeping vmcnt uniform.
  if constexpr (GN != 0) {
    const int tbytes = cin * 8, tp = wave < (tbytes + 1023) / 1024 ? wave : 0;
    const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.gn_ab + (long)img * cin * 2), (short)0, tbytes, 0x00020000);
    dma16(rst, reinterpret_cast<char*>(abl) + tp * 1024, (unsigned)(tp * 1024 + lane * 16), 0);
  }
  issue_halo(0);
  issue_b(0);
  issue_b(1);
  wait_vm<2>();  // the table piece and this wave's halo pieces
  if constexpr (GN != 0) {
    __syncthreads();  // every wave's table piece has landed
    transform(0);
  }

  HALO_STAMP(1);
  const int lr = lane & 15, lq = lane >> 4;
  const int bsw = (lq ^ sw(lr)) * 16;  // weight rows n = 64 wn + 16 j + lr share sw(lr)
  // A fragment i of a tap reads halo slots s0 + 16 i + lr: adding 16 leaves bits 0..3 (and so the
  // swizzle) unchanged, so one lane address per tap serves all four fragments (immediate offsets)
  // taps unrolled: ring slot (u % 3 = t % 3, 9 taps per block), filter offset, waits and the next
  // loads are compile-time per tap; the only runtime branch is "is there a next channel block"
  for (int cb = 0; cb < ncb; ++cb) {
    const bool more = cb + 1 < ncb;
    const char* hb = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // this tap's weights (and at tap 2 the next halo); younger ops allowed in flight: the next tap's
      // weights and, at tap 1, the next halo's 4 pieces issued at tap 0
      if (t == 1) {
        if (more) wait_vm<5>(); else wait_vm<1>();
      } else if (t < 8 || more) {
        wait_vm<1>();
      } else if (res_dma) {
        wait_vm<2>();  // younger: the epilogue's pass-0 residual pieces (issued at tap 7)
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      if (t + 2 < 9) {
        dma16(rsw, bbuf + ((t + 2) % NB) * BBYTES + wave * 1024, bvo, ((t + 2) * cin + cb * 32) * 2);
      } else if (more) {
        dma16(rsw, bbuf + ((t + 2) % NB) * BBYTES + wave * 1024, bvo, ((t + 2 - 9) * cin + (cb + 1) * 32) * 2);
      }
      if (t == 0 && more) issue_halo(cb + 1);
      if (t == 7 && !more && res_dma)  // pass 0's residual rows into the halo buffer the last block does not read
        halo_res_dma<NW>(rsr, lds + halo::res_off(parity, 0), (img * H + oy0) * W + ox0, W, a.res_ld, n0, wave, lane, 0);
      const char* bb = bbuf + (t % NB) * BBYTES + (wn * 64 + lr) * 64 + bsw;
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bfv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(bb + j * 16 * 64);
      // per-tap lane address, recomputed each tap from a laundered base (the compiler would otherwise
      // hoist all 9 taps' addresses out of the channel-block loop and spill)
      int lb = wm * HC + lr;
      asm volatile("" : "+v"(lb));
      const int sl = lb + ky * HC + kx;
      const char* ab = hb + sl * 64 + ((lq ^ sw(sl)) << 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ab + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
      }
      // the next block's halo (own pieces landed at tap 2's wait) is transformed one piece per tap over
      // taps 2..5, AFTER this tap's MFMAs are issued, so its VALU runs beside the matrix pipe instead of
      // delaying the next barrier; the block reads it from its tap 0 on (several barriers later)
      if constexpr (GN != 0)
        if (t >= 2 && t < 6 && more) {
          transform_piece(cb + 1, t - 2);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier
        }
    }
  }
  HALO_STAMP(2);
  if constexpr (FE) {
    if (a.res)
      halo_epilogue<NW, true>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(parity),
                              res_off(parity, 0), res_off(parity, 1), rsr, wave);
    else
      halo_epilogue<NW, false>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(parity),
                               res_off(parity, 0), res_off(parity, 1), rsr, wave);
  } else {
    epilogue_vec<TR * TC, BN, 4, 2, NT, 2, Rows, false>(acc, a, 0, n0, wm, wn, lane, tid, lds,
                                                        Rows{(img * H + oy0) * W + ox0, W});
  }
  HALO_STAMP(3);
}

// ============================================================================================
// The 8-row halo conv (r04): one 1024-thread block per CU computes 8 x 64 output pixels x 128 channels
// (16 waves: 8 output rows x 2 channel halves of 64, the same 64 x 64 wave tile as conv3x3_halo_kernel).
// Against the 4-row kernel (two 512-thread blocks per CU) it trades the second co-resident block for
// depth: the whole 160 KB of LDS holds a 10 x 66-pixel halo double buffer (1.29 halo pixels per output
// pixel instead of 1.55) and an 8-slot weight ring fed 6 taps ahead (the 4-row kernel's 3-slot ring,
// 2 taps ahead, left the main loop waiting on ~1.1 us LDS-DMA landings, tools/halo_stamps.hip, r04).
// Roles are split so every wave's vmcnt counts only its own stream: waves 0..7 stream the weight slices
// (1 KB = 16 rows each), waves 8..15 the halo pieces (6 each, duplicates for the 42 pieces) and the
// GroupNorm table, and transform the pieces they loaded (affine + SiLU in place). Same MFMA order as
// the 4-row kernel (channel block major, tap minor), so both give bit-identical outputs.
// ============================================================================================
namespace halo8 {
constexpr int TR = 8, TC = 64;
constexpr int HR = TR + 2, HC = TC + 2;            // 10 x 66 halo pixels
constexpr int HPIX = HR * HC;                      // 660
constexpr int NPIECE = (HPIX * 4 + 63) / 64;       // 42 pieces of 1 KB
constexpr int HBYTES = NPIECE * 1024;              // 43,008
constexpr int BN = 128, NW = 16, NT = NW * 64;
constexpr int BBYTES = BN * 64;                    // one tap's 32-channel weight slice
constexpr int NB = 8, LEAD = 6;                    // weight ring: slice u + LEAD issued at tap u
constexpr int PPW = 6;                             // halo pieces per halo wave (8 waves x 6 >= 42)
constexpr int AB_MAX = 512;
constexpr int TABLE = 2 * HBYTES + NB * BBYTES;    // 151,552
constexpr int LDS = TABLE + AB_MAX * 8;            // 155,648
static_assert(LDS <= 160 * 1024, "one block per CU");
static_assert(NB >= LEAD + 1, "a slot is reused only after every wave passed the barrier of its last reader");
// epilogue (halo_epilogue<16>): park 128 rows x 132 fp32, two 32 KB residual pass buffers; pass 0's
// residual lands in the halo buffer the last channel block does not read (index = ncb & 1)
constexpr int PK = 128 * (BN + 4) * 4, RB = 128 * BN * 2;
static_assert(RB <= HBYTES && HBYTES + RB + PK <= LDS && HBYTES + PK + RB <= LDS, "epilogue plan");
__device__ __forceinline__ int res_off(int f, int p) { return ((p & 1) == 0) ? (f ? HBYTES : 0) : (f ? 0 : HBYTES + PK); }
__device__ __forceinline__ int park_off(int f) { return f ? HBYTES + RB : HBYTES; }
__device__ __forceinline__ int sw(int s) { return ((s >> 2) & 1) << 1; }
}  // namespace halo8

// vmcnt(n) for a wave-uniform runtime n in [0, 7]
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    default: wait_vm<7>(); break;
  }
}

template <int GN>
__global__ __launch_bounds__(1024) void conv3x3_halo8_kernel(ConvArgs a, int tiles_x, int tiles_y, unsigned bytes0,
                                                            unsigned bytesw) {
  using namespace halo8;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const hbuf = lds;
  char* const bbuf = lds + 2 * HBYTES;
  float* const abl = reinterpret_cast<float*>(lds + TABLE);
  HALO_STAMP(0);
#ifdef RDEIC_HALO_STAMPS
  if (threadIdx.x == 0) {
    g_halo_stamps[(long)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    g_halo_stamps[(long)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  const int tn = a.cout / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;  // XCD-aware bijective remap (as conv3x3_halo_kernel)
  const int xcd = orig & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
  const int nt = wgid % tn;
  int sp = wgid / tn;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * TC, n0 = nt * BN;
  const int H = a.h, W = a.w, cin = a.c0;
  const int ncb = cin >> 5, U = ncb * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wave = (output row, 64-channel half)
  const bool wload = wave < 8;              // weight-stream wave; else halo-stream wave
  const int hw = wave - 8;

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);
  const bool res_dma = a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res_dma ? a.res : a.in0), (short)0, res_dma ? (int)((long)(img * H + H) * W * a.res_ld * 2) : 0, 0x00020000);
  const int f = ncb & 1;  // the halo buffer the last channel block does not read

  // halo waves: pieces hw + 8 k (k < 6; past the 42 pieces, piece hw + 32 again: same bytes, same slots).
  // A piece's source offset (or out-of-image zeros) is recomputed at each issue from a laundered lane id
  // (six live offsets would push the 128-VGPR loop into scratch).
  auto hpiece = [&](int k) { return hw + 8 * k < NPIECE ? hw + 8 * k : hw + 32; };  // wave-uniform
  auto halo_voff = [&](int k, int ln) {
    const int p = hpiece(k);
    const int sl = p * 16 + (ln >> 2), ph = ln & 3;
    unsigned vo = kOOB;
    if (sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        vo = (unsigned)((img * H + iy) * W + ix) * (unsigned)(a.ld0 * 2) + (unsigned)((ph ^ sw(sl)) * 16);
    }
    return vo;
  };
  auto hpo = [&](int k) { return hpiece(k) * 1024; };
  // The GroupNorm transform is balanced over all 16 waves: wave w transforms pieces w + 16 k (k < 3,
  // < 42) whoever loaded them (r04: -3.5% against transforming by the loader). tinfo: per k a valid bit
  // (bit k: a real piece inside the image) and the lane's logical channel chunk (bits 8 + 2k).
  unsigned tinfo = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int p = wave + 16 * k;
    const int sl = p * 16 + (lane >> 2), ph = lane & 3;
    bool in = false;
    if (p < NPIECE && sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    }
    if (in) tinfo |= 1u << k;
    tinfo |= (unsigned)(ph ^ sw(sl)) << (8 + 2 * k);
  }
  // halo waves: all six pieces of block cb (prologue), or half of them (main loop, k in [k0, k1))
  auto issue_halo = [&](int cb, int k0, int k1) {
    char* dst = hbuf + (cb & 1) * HBYTES;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int k = k0; k < k1; ++k) dma16(rs0, dst + hpo(k), halo_voff(k, ln), cb * 64);
  };
  // weight waves: rows n = 16 wave + lane / 4, chunk lane % 4 of every tap slice
  unsigned bvo = kOOB;
  if (wload) {
    const int n = wave * 16 + (lane >> 2), ph = lane & 3;
    bvo = (n0 + n < a.cout) ? (unsigned)(n0 + n) * (unsigned)(a.wld * 2) + (unsigned)((ph ^ sw(n)) * 16) : kOOB;
  }
  auto issue_b = [&](int u) {
    const int cb = u / 9, t = u - (u / 9) * 9;
    dma16(rsw, bbuf + (u % NB) * BBYTES + wave * 1024, bvo, (t * cin + cb * 32) * 2);
  };
  // piece wave + 16 k of block cb, in place (out-of-image chunks stay zero: the conv's padding of the
  // normalised tensor). info and lane are laundered so their derived offsets are recomputed here instead of
  // hoisted out of the channel-block loop, where hipcc kept them in scratch; every reload was an
  // s_waitcnt vmcnt(0) that drained the weight ring's in-flight LDS-DMA (r04)
  auto transform_piece = [&](int cb, int k) {
    unsigned info = tinfo;
    int ln = lane;
    asm volatile("" : "+v"(info), "+v"(ln));
    if (!(info & (1u << k))) return;
    char* pc = hbuf + (cb & 1) * HBYTES + ln * 16 + (wave + 16 * k) * 1024;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(pc);
    const int ch = (info >> (8 + 2 * k)) & 3;
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb * 32 + ch * 8) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = __builtin_fmaf((float)v[e], av[e], bv[e]);
      if constexpr (GN == 2) x *= __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      o[e] = (bf16)x;
    }
    *reinterpret_cast<bf16x8*>(pc) = o;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: halo waves bring the table (one piece each; waves past its pieces repeat piece 0) and
  // block 0's halo; weight waves the first LEAD slices
  if (wload) {
    const int n0s = U < LEAD ? U : LEAD;
    for (int u = 0; u < n0s; ++u) issue_b(u);
  } else {
    if constexpr (GN != 0) {
      const int tbytes = cin * 8, tp = hw < (tbytes + 1023) / 1024 ? hw : 0;
      const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.gn_ab + (long)img * cin * 2), (short)0, tbytes, 0x00020000);
      dma16(rst, reinterpret_cast<char*>(abl) + tp * 1024, (unsigned)(tp * 1024 + lane * 16), 0);
    }
    issue_halo(0, 0, PPW);
    wait_vm<0>();
  }
  if constexpr (GN != 0) {
    __syncthreads();  // every table piece and every halo piece of block 0 has landed
#pragma unroll 1
    for (int k = 0; k < 3; ++k) transform_piece(0, k);  // one piece at a time (register budget)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier releases readers
  }

  HALO_STAMP(1);
  const int lr = lane & 15, lq = lane >> 4;
  const int bsw = (lq ^ sw(lr)) * 16;
  // Schedule (r04, each step measured): one barrier per two taps, every wait and weight
  // DMA issue at even taps; the next halo issued in two halves at taps 0 and 2, waited for at tap 4 and
  // transformed at taps 4..6 after each tap's MFMAs.
  for (int cb = 0; cb < ncb; ++cb) {
    const bool more = cb + 1 < ncb;
    const char* hb = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int u = cb * 9 + t;
      const bool BAR = t % 2 == 0;  // t is unrolled: a compile-time value
      if (wload && BAR) {  // slices u and (t < 8) u + 1 landed; issued so far: up to u + 5
        if (u + 6 < U) {
          t < 8 ? wait_vm<4>() : wait_vm<5>();  // steady state: a compile-time count, no branch chain
        } else {
          const int issued = u + 5 < U - 1 ? u + 5 : U - 1;
          const int need = (t < 8 && u + 1 < U) ? u + 1 : u;
          wait_vm_rt(issued - need);
        }
      }
      if (!wload && more && t == 4) wait_vm<0>();  // this wave's six pieces of the next block have landed
      if (BAR) __builtin_amdgcn_s_barrier();
      if (wload) {
        if (BAR) {  // slices u + 6 and (t < 8) u + 7: slots last read at taps u - 2 and u - 1
          if (u + LEAD < U) issue_b(u + LEAD);
          if (t < 8 && u + LEAD + 1 < U) issue_b(u + LEAD + 1);
        }
      } else if (t == 0 && more) {  // the next halo's six pieces in two halves, so no barrier waits on six
        issue_halo(cb + 1, 0, PPW / 2);
      } else if (t == 2 && more) {
        issue_halo(cb + 1, PPW / 2, PPW);
      }
      // pass 0's residual rows (32 KB) into the halo buffer the last channel block does not read, issued by the
      // halo waves at the last block's tap 0 (they load nothing else in it): nine taps of lead for the HBM
      // latency the epilogue's first pass used to wait on (issued at tap 8: +8.6k cycles per block, r05 stamps)
      if (t == 0 && !more && res_dma && !wload) {
        int l = lane;
        asm volatile("" : "+v"(l));
        const int base = (img * H + oy0) * W + ox0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = hw + 8 * k, pr = 4 * q + (l >> 4);
          const unsigned vo = (unsigned)(base + (pr >> 4) * W + (pr & 15)) * (unsigned)(a.res_ld * 2) + (unsigned)((l & 15) * 16);
          dma16(rsr, lds + res_off(f, 0) + q * 1024, vo, n0 * 2);
        }
      }
      const char* bb = bbuf + (u % NB) * BBYTES + (wn * 64 + lr) * 64 + bsw;
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bfv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(bb + j * 16 * 64);
      int lb = wm * HC + lr;
      asm volatile("" : "+v"(lb));
      const int sl = lb + ky * HC + kx;
      const char* ab = hb + sl * 64 + ((lq ^ sw(sl)) << 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ab + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
      }
      // the next block's transform: pieces wave + 16 k, k = 0..2, by every wave at taps 4..6 (the loaders'
      // tap-4 wait and barrier made them visible), after this tap's MFMAs in program order
      if constexpr (GN != 0)
        if (t >= 4 && t < 7 && more) {
          transform_piece(cb + 1, t - 4);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier
        }
    }
  }
  HALO_STAMP(2);
  if (a.res)
    halo_epilogue<NW, true>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(f), res_off(f, 0),
                            res_off(f, 1), rsr, wave);
  else
    halo_epilogue<NW, false>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(f), res_off(f, 0),
                             res_off(f, 1), rsr, wave);
  HALO_STAMP(3);
}

// ============================================================================================
// The 256-channel halo conv (r05): one 1024-thread block per CU computes 4 x 64 output pixels x 256
// channels (16 waves: 4 output rows x 4 channel quarters of 64, the same 64 x 64 wave tile and MFMA order
// as the 4- and 8-row kernels, so outputs and statistics are bit-identical to them). Against halo8 (8 x 64
// pixels x 128 channels) it stages and transforms 396 halo pixels per channel block instead of 660 for the
// same MFMA work: the GroupNorm + SiLU transform per output falls by 40% on the cout >= 256 layers, at the
// price of twice the weight bytes per tap (16 KB slices through a 6-slot ring fed 4 taps ahead).
// Roles as in halo8: waves 0..7 stream the weight slices (2 KB = 32 rows each), waves 8..15 the halo
// pieces (4 each: 25 pieces plus duplicates) and the GroupNorm table; all 16 waves transform.
// ============================================================================================
namespace halo256 {
constexpr int TR = 4, TC = 64;
constexpr int HR = TR + 2, HC = TC + 2;            // 6 x 66 halo pixels
constexpr int HPIX = HR * HC;                      // 396
constexpr int NPIECE = (HPIX * 4 + 63) / 64;       // 25 pieces of 1 KB
constexpr int HBYTES = NPIECE * 1024;              // 25,600
constexpr int BN = 256, NW = 16, NT = NW * 64;
constexpr int BBYTES = BN * 64;                    // one tap's 32-channel weight slice: 16 KB
constexpr int NB = 6, LEAD = 4;                    // weight ring: slices u + 4 (and u + 5) issued at even tap u
constexpr int PPW = 4;                             // halo pieces per halo wave (8 waves x 4 >= 25)
constexpr int AB_MAX = 512;
constexpr int RING = 2 * HBYTES;                   // 51,200
constexpr int TABLE = RING + NB * BBYTES;          // 149,504
constexpr int LDS = TABLE + AB_MAX * 8;            // 153,600
static_assert(LDS <= 160 * 1024, "one block per CU");
static_assert(NB >= LEAD + 2, "slot of u + LEAD + 1 was last read at tap u - 1 (one barrier per two taps)");
// epilogue: four passes of 64 tile rows (one 16-row fragment per wave row) x 256 channels: a parked pass
// (64 x 260 fp32) and two 32 KB residual buffers; pass 0's residual is DMA'd at the last tap into two ring
// slots the last taps do not read (r0), the other two regions are placed around it
constexpr int SDW = BN + 4;
constexpr int PK = 64 * SDW * 4;                   // 66,560
constexpr int RB = 64 * BN * 2;                    // 32,768
static_assert(RB == 2 * BBYTES, "pass-0 residual = two ring slots");
__device__ __forceinline__ int sw(int s) { return ((s >> 2) & 1) << 1; }
// the first of two adjacent ring slots free at the last tap (slot s = (U - 1) % NB is being read; the
// barrier of that tap released every slot read before it)
__host__ __device__ constexpr int r0_slot(int s) { return s <= NB - 3 ? s + 1 : 0; }
__host__ __device__ constexpr bool plan_ok(int s) {  // park / r0 / r1 disjoint and inside the LDS
  const int r0 = RING + r0_slot(s) * BBYTES;
  const int park = r0 >= PK ? 0 : r0 + RB;
  const int r1 = park == 0 ? (r0 >= PK + RB ? PK : r0 + RB) : 0;
  auto dis = [](int a, int la, int b, int lb) { return a + la <= b || b + lb <= a; };
  return r0 + RB <= LDS && park + PK <= LDS && r1 + RB <= LDS && dis(r0, RB, park, PK) && dis(r0, RB, r1, RB) &&
         dis(park, PK, r1, RB) && dis(r0, RB, RING + s * BBYTES, BBYTES);
}
static_assert(plan_ok(0) && plan_ok(1) && plan_ok(2) && plan_ok(3) && plan_ok(4) && plan_ok(5), "epilogue plan");
}  // namespace halo256

// Epilogue of the 256-channel halo conv (halo_epilogue's arithmetic and statistics order for a 256-wide
// tile: out = (acc + bias) + residual, bf16; fused GroupNorm partials per (64-row block, channel) as
// ((g0 + g1) + g2) + g3 of column scans in row order). park / r0 / r1: LDS offsets of the parked pass and
// the residual buffers of even / odd passes; pass 0's residual is already in flight into r0.
__device__ __forceinline__ void halo256_res_dma(__amdgpu_buffer_rsrc_t rsr, char* dst, int base, int W, int res_ld,
                                                int n0, int wave, int lane, int p) {
  // pass rows: 64 (wave row pr / 16, pixel p * 16 + pr % 16) x 512 B; piece q (this wave's wave and
  // wave + 16) = rows 2q, 2q + 1; lane i: row 2q + i / 32, chunk i % 32
  int l = lane;
  asm volatile("" : "+v"(l));
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = wave + 16 * k;
    const int pr = 2 * q + (l >> 5);
    const unsigned vo = (unsigned)(base + (pr >> 4) * W + (pr & 15)) * (unsigned)(res_ld * 2) + (unsigned)((l & 31) * 16);
    dma16(rsr, dst + q * 1024, vo, p * 16 * res_ld * 2 + n0 * 2);
  }
}

__device__ __forceinline__ void halo256_epilogue(const f32x4 (&acc)[4][4], const ConvArgs& a, int n0, int wm, int wn,
                                                 int tid, char* lds, int base, int W, int park, int r0, int r1,
                                                 __amdgpu_buffer_rsrc_t rsr, int wave) {
  using halo256::SDW;
  asm volatile("" : "+v"(tid));  // addresses derived after the main loop (not hoisted into its live set)
  const int lane = tid & 63;
  const int lr = lane & 15, lq = lane >> 4;
  float* const L = reinterpret_cast<float*>(lds + park);
  const bool has_res = a.res != nullptr;
  const bool st = a.gn_part != nullptr;
  const int cc = tid & 31;  // this thread's 8 channels n0 + 8 cc in every chunk
  const int nn = n0 + cc * 8;
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = 0.f;
  if (a.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + nn), b1 = *reinterpret_cast<const float4*>(a.bias + nn + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w; bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  float sg[4], qg[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    __syncthreads();  // p = 0: the main loop's LDS reads are done; else: the previous pass's readers are
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(wm * 16 + lq * 4 + r) * SDW + wn * 64 + j * 16 + lr] = acc[p][j][r];
    if (has_res) {  // this wave's residual pieces of pass p (younger: the 2 stores of pass p - 1)
      if (p == 0) wait_vm<0>(); else wait_vm<2>();
    }
    __syncthreads();
    if (has_res && p + 1 < 4)  // the next pass's residual into the buffer pass p - 1 read
      halo256_res_dma(rsr, lds + ((p + 1) & 1 ? r1 : r0), base, W, a.res_ld, n0, wave, lane, p + 1);
    const char* R = lds + (p & 1 ? r1 : r0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = (tid >> 5) + 32 * k;  // pass row: wave row pr / 16, pixel p * 16 + pr % 16 of it
      const long m = base + (pr >> 4) * W + p * 16 + (pr & 15);
      const float4 x0 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8 + 4);
      float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias[e];
      if (has_res) {
        const bf16x8 rv = *reinterpret_cast<const bf16x8*>(R + pr * 512 + cc * 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
      }
      bf16x8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.out) + m * a.out_ld + nn) = ov;
      if (st) {
        *reinterpret_cast<float4*>(L + pr * SDW + cc * 8) = make_float4((float)ov[0], (float)ov[1], (float)ov[2], (float)ov[3]);
        *reinterpret_cast<float4*>(L + pr * SDW + cc * 8 + 4) = make_float4((float)ov[4], (float)ov[5], (float)ov[6], (float)ov[7]);
      }
    }
    if (st) {  // column scan: thread (wave row b, channel j), the 16 rows of group p, in row order
      __syncthreads();
      const int b = tid >> 8, j = tid & 255;
      const float* col = L + (b * 16) * SDW + j;
      float y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) y[r] = col[r * SDW];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s1 += y[r]; s2 = fmaf(y[r], y[r], s2); }
      sg[p] = s1;
      qg[p] = s2;
    }
  }
  if (st) {
    const int b = tid >> 8, j = tid & 255;
    float* pp = a.gn_part + 4 + ((long)((a.gn_row0 + base + b * W) / 64) * a.cout + n0 + j) * 2;
    pp[0] = ((sg[0] + sg[1]) + sg[2]) + sg[3];
    pp[1] = ((qg[0] + qg[1]) + qg[2]) + qg[3];
    if (tid == 0 && base == 0 && n0 == 0) reinterpret_cast<int*>(a.gn_part)[0] = 64;  // rows per partial
  }
}

template <int GN>
__global__ __launch_bounds__(1024) void conv3x3_halo256_kernel(ConvArgs a, int tiles_x, int tiles_y, unsigned bytes0,
                                                              unsigned bytesw) {
  using namespace halo256;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const hbuf = lds;
  char* const bbuf = lds + RING;
  float* const abl = reinterpret_cast<float*>(lds + TABLE);
  HALO_STAMP(0);
#ifdef RDEIC_HALO_STAMPS
  if (threadIdx.x == 0) {
    g_halo_stamps[(long)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    g_halo_stamps[(long)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  const int tn = a.cout / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;  // XCD-aware bijective remap (as conv3x3_halo_kernel)
  const int xcd = orig & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
  const int nt = wgid % tn;
  int sp = wgid / tn;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * TC, n0 = nt * BN;
  const int H = a.h, W = a.w, cin = a.c0;
  const int ncb = cin >> 5, U = ncb * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // wave = (output row, 64-channel quarter)
  const bool wload = wave < 8;              // weight-stream wave; else halo-stream wave
  const int hw = wave - 8;

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);
  const bool res_dma = a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res_dma ? a.res : a.in0), (short)0, res_dma ? (int)((long)(img * H + H) * W * a.res_ld * 2) : 0, 0x00020000);
  // epilogue LDS plan: r0 = two ring slots free at the last tap; the parked pass and r1 around it
  const int r0 = RING + r0_slot((U - 1) % NB) * BBYTES;
  const int park = r0 >= PK ? 0 : r0 + RB;  // below r0 when it fits (r0 at ring slot >= 1), else right after it
  const int r1 = park == 0 ? (r0 >= PK + RB ? PK : r0 + RB) : 0;

  // halo waves: pieces hw + 8 k (k < 4; past the 25 pieces, piece hw + 16 again: same bytes, same slots);
  // offsets recomputed at each issue from a laundered lane id
  auto hpiece = [&](int k) { return hw + 8 * k < NPIECE ? hw + 8 * k : hw + 16; };  // wave-uniform
  auto halo_voff = [&](int k, int ln) {
    const int p = hpiece(k);
    const int sl = p * 16 + (ln >> 2), ph = ln & 3;
    unsigned vo = kOOB;
    if (sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        vo = (unsigned)((img * H + iy) * W + ix) * (unsigned)(a.ld0 * 2) + (unsigned)((ph ^ sw(sl)) * 16);
    }
    return vo;
  };
  auto issue_halo = [&](int cb, int k0, int k1) {
    char* dst = hbuf + (cb & 1) * HBYTES;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int k = k0; k < k1; ++k) dma16(rs0, dst + hpiece(k) * 1024, halo_voff(k, ln), cb * 64);
  };
  // transform: wave w takes pieces w + 16 k (k < 2, < 25) whoever loaded them; tinfo: per k a valid bit
  // (a real piece inside the image) and the lane's logical channel chunk (bits 8 + 2k)
  unsigned tinfo = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = wave + 16 * k;
    const int sl = p * 16 + (lane >> 2), ph = lane & 3;
    bool in = false;
    if (p < NPIECE && sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    }
    if (in) tinfo |= 1u << k;
    tinfo |= (unsigned)(ph ^ sw(sl)) << (8 + 2 * k);
  }
  // weight waves: rows n = 32 wave + 16 k + lane / 4 (k = 0, 1), chunk lane % 4 of every tap slice
  unsigned bvo0 = kOOB, bvo1 = kOOB;
  if (wload) {
    const int na = wave * 32 + (lane >> 2), nb = na + 16, ph = lane & 3;
    bvo0 = (n0 + na < a.cout) ? (unsigned)(n0 + na) * (unsigned)(a.wld * 2) + (unsigned)((ph ^ sw(na)) * 16) : kOOB;
    bvo1 = (n0 + nb < a.cout) ? (unsigned)(n0 + nb) * (unsigned)(a.wld * 2) + (unsigned)((ph ^ sw(nb)) * 16) : kOOB;
  }
  auto issue_b = [&](int u) {
    const int cb = u / 9, t = u - (u / 9) * 9;
    char* dst = bbuf + (u % NB) * BBYTES + wave * 2048;
    dma16(rsw, dst, bvo0, (t * cin + cb * 32) * 2);
    dma16(rsw, dst + 1024, bvo1, (t * cin + cb * 32) * 2);
  };
  auto transform_piece = [&](int cb, int k) {
    unsigned info = tinfo;
    int ln = lane;
    asm volatile("" : "+v"(info), "+v"(ln));
    if (!(info & (1u << k))) return;
    char* pc = hbuf + (cb & 1) * HBYTES + ln * 16 + (wave + 16 * k) * 1024;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(pc);
    const int ch = (info >> (8 + 2 * k)) & 3;
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb * 32 + ch * 8) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = __builtin_fmaf((float)v[e], av[e], bv[e]);
      if constexpr (GN == 2) x *= __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      o[e] = (bf16)x;
    }
    *reinterpret_cast<bf16x8*>(pc) = o;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: halo waves bring the table (one piece each; waves past its pieces repeat piece 0) and
  // block 0's halo; weight waves the first LEAD slices
  if (wload) {
    const int n0s = U < LEAD ? U : LEAD;
    for (int u = 0; u < n0s; ++u) issue_b(u);
  } else {
    if constexpr (GN != 0) {
      const int tbytes = cin * 8, tp = hw < (tbytes + 1023) / 1024 ? hw : 0;
      const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.gn_ab + (long)img * cin * 2), (short)0, tbytes, 0x00020000);
      dma16(rst, reinterpret_cast<char*>(abl) + tp * 1024, (unsigned)(tp * 1024 + lane * 16), 0);
    }
    issue_halo(0, 0, PPW);
    wait_vm<0>();
  }
  if constexpr (GN != 0) {
    __syncthreads();  // every table piece and every halo piece of block 0 has landed
#pragma unroll 1
    for (int k = 0; k < 2; ++k) transform_piece(0, k);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier releases readers
  }

  HALO_STAMP(1);
  const int lr = lane & 15, lq = lane >> 4;
  const int bsw = (lq ^ sw(lr)) * 16;
  // Schedule (halo8's): one barrier per two taps, every wait and weight DMA issue at even taps; the next
  // halo issued in two halves at taps 0 and 2, waited for at tap 4 and transformed at taps 4 and 5 after
  // each tap's MFMAs; pass 0's residual rows DMA'd at the last tap into two free ring slots.
  for (int cb = 0; cb < ncb; ++cb) {
    const bool more = cb + 1 < ncb;
    const char* hb = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int u = cb * 9 + t;
      const bool BAR = t % 2 == 0;  // t is unrolled: a compile-time value
      if (wload && BAR) {  // slices u and (t < 8) u + 1 landed; issued so far: up to u + 3 (2 DMAs each)
        if (u + LEAD + 1 < U) {
          t < 8 ? wait_vm<4>() : wait_vm<6>();  // steady state: a compile-time count
        } else {
          const int issued = u + LEAD - 1 < U - 1 ? u + LEAD - 1 : U - 1;
          const int need = (t < 8 && u + 1 < U) ? u + 1 : u;
          wait_vm_rt(2 * (issued - need));
        }
      }
      if (!wload && more && t == 4) wait_vm<0>();  // this wave's pieces of the next block have landed
      if (BAR) __builtin_amdgcn_s_barrier();
      if (wload) {
        if (BAR) {  // slices u + 4 and (t < 8) u + 5: slots last read at taps u - 2 and u - 1
          if (u + LEAD < U) issue_b(u + LEAD);
          if (t < 8 && u + LEAD + 1 < U) issue_b(u + LEAD + 1);
        }
      } else if (t == 0 && more) {  // the next halo's pieces in two halves
        issue_halo(cb + 1, 0, PPW / 2);
      } else if (t == 2 && more) {
        issue_halo(cb + 1, PPW / 2, PPW);
      }
      if (t == 8 && !more && res_dma)  // pass 0's residual rows into the two ring slots the last taps do not read
        halo256_res_dma(rsr, lds + r0, (img * H + oy0) * W + ox0, W, a.res_ld, n0, wave, lane, 0);
      // per-tap lane addresses from laundered bases (hoisted over the 9 unrolled taps, with the ring slot
      // not a multiple of 9 taps, hipcc kept 15 of them in scratch and reloaded them in the loop)
      int bl = (wn * 64 + lr) * 64 + bsw;
      int lb = wm * HC + lr;
      asm volatile("" : "+v"(bl), "+v"(lb));
      const char* bb = bbuf + (u % NB) * BBYTES + bl;
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bfv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(bb + j * 16 * 64);
      const int sl = lb + ky * HC + kx;
      const char* ab = hb + sl * 64 + ((lq ^ sw(sl)) << 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ab + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
      }
      if constexpr (GN != 0)
        if (t >= 4 && t < 6 && more) {
          transform_piece(cb + 1, t - 4);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier
        }
    }
  }
  HALO_STAMP(2);
  halo256_epilogue(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park, r0, r1, rsr, wave);
  HALO_STAMP(3);
}

// the 256-channel halo conv where it applies (rdeic_set_conv_option(10, v)); off by default: measured 2-3%
// slower than halo8 on every VAE cout >= 256 shape and -0.6% on the bench (profiles/r05_halo256_ab.txt)
// ============================================================================================
// Persistent short-K linear (r05, option 12): the transformer's 1x1 projections with K = 320..1280 (GEGLU
// 320 -> 2560 etc., LayerNorm-folded q/k/v). In the per-tile kernels their fixed cost is the epilogue
// (26k of 42k cycles of a 256x256 GEGLU tile, tools/dma_stamps.hip), which no MFMA work overlaps. Here one
// 512-thread block per CU walks its tiles (256 x 128, 8 waves of 64 x 64, 32-deep k-tiles through a 3-slot
// LDS-DMA ring that runs on across tile boundaries). At the end of a tile's k-loop the accumulators get the
// LayerNorm fold and the bias, are rounded to bf16 and parked in LDS; during the NEXT tile's k-loop every
// thread turns one parked 8-column chunk per k-tile into output (GEGLU x * gelu(g) or a plain copy) and
// stores it, so the epilogue's VALU and stores run beside that tile's MFMAs. Same MFMA sequence over k and
// the same fp32 epilogue arithmetic as the LDS-DMA tiles (LN fold, + bias, round to bf16; GEGLU on the bf16
// halves): outputs are bit-identical to tile 32 (test_kernels_gpu.py::test_linear_persistent_bit_identical).
// ============================================================================================
namespace lp {
constexpr int BM = 256, BN = 128, WGN = 2, NW = 8, NT = NW * 64;
constexpr int KB = 32, RB = KB * 2, RPI = 1024 / RB, LPR = RB / 16, S = 3;
constexpr int A_BYTES = BM * RB, STAGE = (BM + BN) * RB, RING = S * STAGE;
constexpr int AI = BM / NW / RPI, BI = BN / NW / RPI, PER = AI + BI;
constexpr int WTM = 64, WTN = 64, TM = WTM / 16, TN = WTN / 16;
constexpr int PROW = BN * 2 + 16;  // parked bf16 row (+16 B: bank spread of the chunk reads)
constexpr int CPR = BN / 8;        // 8-column chunks per row
constexpr int NCHUNK = BM * CPR / NT;
constexpr int PARK = BM * PROW;
// per-tile epilogue operands, LDS-DMA'd with the tile's first k-tile (two buffers: the next tile's arrive before
// this one parks): LayerNorm (mean, rstd) of the 256 rows, column sums and bias of the 128 columns
constexpr int EPI = BM * 8 + BN * 4 * 2;
constexpr int LDS = RING + PARK + 2 * EPI;
static_assert(AI * RPI * NW == BM && BI * RPI * NW == BN && NCHUNK * NT == BM * CPR, "tile split");
static_assert(BM * 8 == 2 * 1024 && BN * 4 * 2 == 1024, "epilogue operands: 3 LDS-DMA wave-instructions");
static_assert(LDS <= 160 * 1024, "one block per CU");
}  // namespace lp

// Every vector-memory op of this kernel is counted (wave-uniform): the k-tile and epilogue-operand LDS-DMAs and
// the output stores (buffer stores, issued whole-wave, out-of-range lanes discarded by the descriptor), so the
// wait for ring slot gi is exactly "all but the ops issued after it" (vmcnt returns in issue order).
template <bool GEGLU>
__global__ __launch_bounds__(lp::NT) void linear_persist_kernel(ConvArgs a, int tiles_n, int ntiles, unsigned bytes0,
                                                                unsigned bytesw, unsigned bytes_out) {
  using namespace lp;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const park = lds + RING;
  char* const epi = park + PARK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave - (wave / WGN) * WGN;
  const int g = lane / LPR, sl = lane % LPR;
  const int ce = sl ^ dma_key32(g);
  // XCD-aware block order (as conv_dma_body): an XCD's blocks take consecutive tile ids, so they share A rows
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int my_tiles = wgid < ntiles ? (ntiles - 1 - wgid) / nwg + 1 : 0;
  const int nk = a.c0 / KB;
  const int total = my_tiles * nk;
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);
  const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc((void*)a.out, (short)0, (int)bytes_out, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.ln_rows, (short)0, a.ln_rows ? (int)(a.M * 8u) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.ln_cs, (short)0, a.ln_rows ? (int)(a.cout * 4u) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bias, (short)0, a.bias ? (int)(a.cout * 4u) : 0, 0x00020000);
  const unsigned lda = (unsigned)a.ld0 * 2u, ldw = (unsigned)a.wld * 2u;

  int issued = 0;  // vector-memory ops this wave has issued
  int mark[S];     // issued count right after ring slot s's k-tile was issued
  auto issue = [&](int gi) {  // block-local k-iteration gi -> (tile, k-tile) into ring slot gi % S
    const int lt = gi / nk, kt = gi - lt * nk;
    const int tile = wgid + lt * nwg;
    const int mt = tile / tiles_n, nt = tile - mt * tiles_n;
    char* sb = lds + (gi % S) * STAGE;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int m = mt * BM + (wave * AI + j) * RPI + g;
      dma16(rs0, sb + (wave * AI + j) * 1024, m < a.M ? (unsigned)m * lda + ce * 16 : kOOB, kt * RB);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int nn = nt * BN + (wave * BI + j) * RPI + g;
      dma16(rsw, sb + A_BYTES + (wave * BI + j) * 1024, nn < a.cout ? (unsigned)nn * ldw + ce * 16 : kOOB, kt * RB);
    }
    issued += PER;
    if (kt == 0 && wave < 4) {  // the tile's epilogue operands into epi buffer lt & 1, one op on waves 0..3
      char* eb = epi + (lt & 1) * EPI;
      if (wave < 2) {  // LayerNorm rows: 16 B per lane = rows 2 l, 2 l + 1
        const int m = mt * BM + wave * 128 + 2 * lane;
        const unsigned vo = (unsigned)(mt * BM + wave * 128) * 8u + lane * 16;
        dma16(rsl, eb + wave * 1024, m < a.M ? vo : kOOB, 0);
      } else {  // wave 2 lanes 0-31: column sums at eb + 2048; wave 3 lanes 32-63: bias at eb + 2560 (4 columns a lane)
        const int nn = nt * BN + (lane & 31) * 4;
        const unsigned vo = nn < a.cout ? (unsigned)nn * 4u : kOOB;
        if (wave == 2) {
          if (lane < 32) dma16(rsc, eb + 2048, vo, 0);
        } else {
          if (lane >= 32) dma16(rsb, eb + 2048, vo, 0);
        }
      }
      ++issued;
    }
    mark[gi % S] = issued;
  };

  const int lr = lane & 15, lq = lane >> 4;
  const int rkey = dma_key32(lr);
  const int so = (lq ^ rkey) * 16;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one parked chunk (row pr, columns cc*8 .. +7) of tile ptile -> output (a buffer store, issued by the whole wave)
  auto chunk = [&](int ptile, int c) {
    const int id = tid + c * NT;
    const int pr = id / CPR, cc = id - pr * CPR;
    const int mt = ptile / tiles_n, nt = ptile - mt * tiles_n;
    const int m = mt * BM + pr, nn = nt * BN + cc * 8;
    const bool ok = m < a.M && nn < a.cout;
    const uint4 raw = *reinterpret_cast<const uint4*>(park + pr * PROW + cc * 16);
    if constexpr (GEGLU) {
      bf16 hv[8];
      *reinterpret_cast<uint4*>(hv) = raw;
      bf16 gv[4];
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const f32x2 r = f32x2{to_f32(hv[e]), to_f32(hv[e + 1])} * gelu_fast2(f32x2{to_f32(hv[4 + e]), to_f32(hv[5 + e])});
        gv[e] = from_f32<bf16>(r.x);
        gv[e + 1] = from_f32<bf16>(r.y);
      }
      typedef unsigned u2 __attribute__((ext_vector_type(2)));
      const uint2 gw = *reinterpret_cast<uint2*>(gv);
      __builtin_amdgcn_raw_buffer_store_b64(u2{gw.x, gw.y}, rso,
                                            ok ? (unsigned)((long)m * a.out_ld + (nn >> 1)) * 2u : kOOB, 0, 0);
    } else {
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(u4{raw.x, raw.y, raw.z, raw.w}, rso,
                                             ok ? (unsigned)((long)m * a.out_ld + nn) * 2u : kOOB, 0, 0);
    }
    ++issued;
  };

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < total) issue(s);

  int kt = 0, lt = 0, ptile = -1;
  for (int gi = 0; gi < total; ++gi) {
    wait_vm_rt(issued - mark[gi % S]);  // at most a store + the next slot's PER + 1 ops (<= 5) follow slot gi
    __builtin_amdgcn_s_barrier();
    // the previous tile's epilogue, one chunk per k-tile (nk >= NCHUNK), beside this tile's MFMAs
    if (ptile >= 0 && kt < NCHUNK) chunk(ptile, kt);
    if (gi + S - 1 < total) issue(gi + S - 1);
    const char* Ab = lds + (gi % S) * STAGE + (wm * WTM + lr) * RB + so;
    const char* Bb = lds + (gi % S) * STAGE + A_BYTES + (wn * WTN + lr) * RB + so;
    bf16x8 bfv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(Bb + j * 16 * RB);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(Ab + i * 16 * RB);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
    }
    if (++kt == nk) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every parked chunk read
      // park: LayerNorm fold, bias, round to bf16 (the vector epilogue's order: rstd (acc - mean colsum) + bias);
      // the epilogue operands landed with this tile's first k-tile, long waited for
      const char* eb = epi + (lt & 1) * EPI;
      float csum[TN], bia[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 16 + lr;
        csum[j] = *reinterpret_cast<const float*>(eb + 2048 + col * 4);
        bia[j] = *reinterpret_cast<const float*>(eb + 2560 + col * 4);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pr0 = wm * WTM + i * 16 + lq * 4;
        float2 lnr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) lnr[r] = *reinterpret_cast<const float2*>(eb + (pr0 + r) * 8);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float v = acc[i][j][r];
            if (a.ln_rows) v = lnr[r].y * __builtin_fmaf(-lnr[r].x, csum[j], v);
            if (a.bias) v += bia[j];
            *reinterpret_cast<bf16*>(park + (pr0 + r) * PROW + (wn * WTN + j * 16 + lr) * 2) = from_f32<bf16>(v);
            acc[i][j][r] = 0.f;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // parked before the next barrier
      ptile = wgid + lt * nwg;
      ++lt;
      kt = 0;
    }
  }
  if (ptile >= 0) {
    __builtin_amdgcn_s_barrier();
    for (int c = 0; c < NCHUNK; ++c) chunk(ptile, c);
  }
}

// persistent short-K linear (rdeic_set_conv_option(12, v)): 0 off (default), 1 where no tile is named
// (rdeic_conv2d, tile -1), 2 also over a named tile 20..39 (the tile table's picks); tile 40 names it explicitly.
// Off: measured slower than the LDS-DMA tiles on every transformer projection (r05, tools/lp_bench.py,
// profiles/r05_lpersist.jsonl: 262 vs 252 us on the 65536 x 320 -> 2560 GEGLU, 1.4-1.7x slower at K >= 640).
// Its k-loop alone (no output) took 225 us there: a 3-slot ring of 32-deep k-tiles keeps ~1k MFMA cycles in
// flight per SIMD, under the L2 -> LDS latency, and the park buffer leaves no LDS for a deeper ring.
int g_lpersist = 0;

// eligibility: bf16 1x1 stride-1 projection, one input segment, K a multiple of 32, no residual / emb / act /
// GroupNorm (input or statistics), output plain (mode 0, 16-byte rows) or GEGLU (mode 2)
bool lp_ok(const rdeic_conv_desc* d, const ConvArgs& a, unsigned& b0, unsigned& bw, unsigned& bo) {
  if (d->dtype != 1 || d->kh != 1 || d->kw != 1 || d->stride != 1 || d->pad_t || d->pad_l || d->up2 ||
      d->c1 || a.batch > 1 || d->gn_ab || d->gn_part || d->res || d->emb || d->act || d->out_f32)
    return false;
  if (d->out_mode == 2) {
    if (d->out_ld % 4 || ((uintptr_t)d->out) % 8) return false;
  } else if (d->out_mode != 0 || d->out_ld % 8 || ((uintptr_t)d->out) % 16) {
    return false;
  }
  if (d->c0 % lp::KB || d->c0 < 8 * lp::KB || d->ld0 % 8 || ((uintptr_t)d->in0) % 16 || d->cout % 8 || d->wld % 64)
    return false;
  if (a.M < 2048) return false;
  const long e0 = ((long)(a.M - 1) * d->ld0 + d->c0) * 2, ew = (long)d->cout * d->wld * 2;
  const long eo = ((long)(a.M - 1) * d->out_ld + (d->out_mode == 2 ? d->cout / 2 : d->cout)) * 2;
  if (e0 >= (1l << 31) || ew >= (1l << 31) || eo >= (1l << 31)) return false;
  b0 = (unsigned)e0;
  bw = (unsigned)ew;
  bo = (unsigned)eo;
  return true;
}

int launch_lpersist(const ConvArgs& a, unsigned b0, unsigned bw, unsigned bo, hipStream_t s) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  const int tn = cdiv(a.cout, lp::BN);
  const int ntiles = cdiv(a.M, lp::BM) * tn;
  const int blocks = ntiles < cus ? ntiles : cus;
  rdeic_count_launch(RDEIC_COUNT_LPERSIST);
  if (a.out_mode == 2)
    hipLaunchKernelGGL(linear_persist_kernel<true>, dim3(blocks), dim3(lp::NT), lp::LDS, s, a, tn, ntiles, b0, bw, bo);
  else
    hipLaunchKernelGGL(linear_persist_kernel<false>, dim3(blocks), dim3(lp::NT), lp::LDS, s, a, tn, ntiles, b0, bw, bo);
  return launch_status();
}

int g_halo256 = 0;

int g_halo8 = 1;  // the 8-row halo conv where it applies (rdeic_set_conv_option(9, v))
// split-K reduction folded into the producer (rdeic_set_conv_option(11, v)); off by default: the last split
// of a tile reduces it alone, so the reduction runs on one block per output tile (80 on the UNet's 8x8
// level) instead of the reduce kernel's hundreds, and the fold's tiles are restricted to the 4- / 8-wave
// ones; measured r05: bench 149.0 -> 133.2 img/s, fine-tune 19.0 -> 14.3 img/s (gpurun_out/r05f)
int g_sk_fold = 0;

int g_halo = 1;  // 3x3 halo conv: 0 off, 1 for GroupNorm-input convs (default), 2 for every eligible conv

bool halo_ok(const rdeic_conv_desc* d, const ConvArgs& a) {
  return d->dtype == 1 && d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad_t == 1 && d->pad_l == 1 && !d->up2 &&
         d->c1 == 0 && d->c0 % 32 == 0 && d->c0 <= halo::AB_MAX && d->cout % halo::BN == 0 && d->ho == d->h &&
         d->wo == d->w && d->h % halo::TR == 0 && d->w % halo::TC == 0 && a.batch == 1 && d->out_mode == 0 &&
         d->ld0 % 8 == 0 && ((uintptr_t)d->in0 % 16) == 0 && d->wld % 64 == 0 && epi_vec_ok(a) && a.epi_vec;
}

// The halo conv over image groups whose input stays inside a 32-bit buffer offset.
int launch_halo(const rdeic_conv_desc* d, ConvArgs a, hipStream_t s, bool* fused) {
  using namespace halo;
  const long ipix = (long)d->h * d->w;
  const long per = ipix * d->ld0 * 2;
  const int g = (int)(((1l << 31) - 1) / per);
  if (g < 1 || (long)d->cout * d->wld * 2 >= (1l << 31)) return -1;
  const bool stats = a.gn_part != nullptr && d->gn_hw == ipix;
  if (fused) *fused = stats;
  if (!stats) a.gn_part = nullptr;
  const int osz = a.out_f32 ? 4 : 2;
  for (int i0 = 0; i0 < d->n; i0 += g) {
    ConvArgs e = a;
    e.n = d->n - i0 < g ? d->n - i0 : g;
    e.M = e.n * d->ho * d->wo;
    e.in0 = a.in0 + i0 * per;
    e.out = a.out + i0 * ipix * d->out_ld * osz;
    e.res = a.res ? a.res + i0 * ipix * d->res_ld * osz : nullptr;
    e.emb = a.emb ? a.emb + (long)i0 * a.emb_ld : nullptr;
    e.gn_ab = a.gn_ab ? a.gn_ab + (long)i0 * d->c0 * 2 : nullptr;
    e.gn_row0 = i0 * (int)ipix;
    const unsigned b0 = (unsigned)(((e.n * ipix - 1) * d->ld0 + d->c0) * 2);
    const unsigned bw = (unsigned)((long)d->cout * d->wld * 2);
    rdeic_count_launch(RDEIC_COUNT_HALO_CONV);
    const bool fe = !e.out_f32 && !e.emb && e.act == 0;
    const int gm = e.gn_ab ? (e.gn_silu ? 2 : 1) : 0;
    if (g_halo256 && fe && d->cout % halo256::BN == 0) {  // 4 x 64 pixels x 256 channels, one block per CU
      rdeic_count_launch(RDEIC_COUNT_HALO256);
      const int txw = d->w / halo256::TC, tyw = d->h / halo256::TR;
      const dim3 gw((unsigned)((long)e.n * tyw * txw * (d->cout / halo256::BN))), bw2(halo256::NT);
      if (gm == 2) hipLaunchKernelGGL((conv3x3_halo256_kernel<2>), gw, bw2, halo256::LDS, s, e, txw, tyw, b0, bw);
      else if (gm == 1) hipLaunchKernelGGL((conv3x3_halo256_kernel<1>), gw, bw2, halo256::LDS, s, e, txw, tyw, b0, bw);
      else hipLaunchKernelGGL((conv3x3_halo256_kernel<0>), gw, bw2, halo256::LDS, s, e, txw, tyw, b0, bw);
      const int rc = launch_status();
      if (rc != RDEIC_OK) return rc;
      continue;
    }
    if (g_halo8 && fe && d->h % halo8::TR == 0) {  // the 8-row, one-block-per-CU form
      const int tx8 = d->w / halo8::TC, ty8 = d->h / halo8::TR;
      const dim3 g8((unsigned)((long)e.n * ty8 * tx8 * (d->cout / halo8::BN))), b8(halo8::NT);
      if (gm == 2) hipLaunchKernelGGL((conv3x3_halo8_kernel<2>), g8, b8, halo8::LDS, s, e, tx8, ty8, b0, bw);
      else if (gm == 1) hipLaunchKernelGGL((conv3x3_halo8_kernel<1>), g8, b8, halo8::LDS, s, e, tx8, ty8, b0, bw);
      else hipLaunchKernelGGL((conv3x3_halo8_kernel<0>), g8, b8, halo8::LDS, s, e, tx8, ty8, b0, bw);
      const int rc = launch_status();
      if (rc != RDEIC_OK) return rc;
      continue;
    }
    const int tx = d->w / TC, ty = d->h / TR;
    const long tiles = (long)e.n * ty * tx * (d->cout / BN);
    const dim3 g((unsigned)tiles), b(NT);
    if (gm == 2 && fe) hipLaunchKernelGGL((conv3x3_halo_kernel<2, true>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (gm == 2) hipLaunchKernelGGL((conv3x3_halo_kernel<2, false>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (gm == 1 && fe) hipLaunchKernelGGL((conv3x3_halo_kernel<1, true>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (gm == 1) hipLaunchKernelGGL((conv3x3_halo_kernel<1, false>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (fe) hipLaunchKernelGGL((conv3x3_halo_kernel<0, true>), g, b, LDS, s, e, tx, ty, b0, bw);
    else hipLaunchKernelGGL((conv3x3_halo_kernel<0, false>), g, b, LDS, s, e, tx, ty, b0, bw);
    const int rc = launch_status();
    if (rc != RDEIC_OK) return rc;
  }
  return RDEIC_OK;
}

}  // namespace

namespace {
// descriptor -> kernel arguments (validation shared by rdeic_conv2d / rdeic_conv2d_splitk)
int make_args(const rdeic_conv_desc* d, ConvArgs& a, bool& vec) {
  a.sk_ws = nullptr;
  a.sk_cnt = nullptr;
  if (!d || !d->in0 || !d->weight || !d->out) return RDEIC_EINVAL;
  if (d->c0 <= 0 || d->c1 < 0 || (d->c1 > 0 && !d->in1) || d->cout <= 0 || d->kh <= 0 || d->kw <= 0 ||
      d->stride <= 0 || d->n <= 0 || d->ho <= 0 || d->wo <= 0)
    return RDEIC_EINVAL;
  if (d->dtype != 0 && d->dtype != 1) return RDEIC_EINVAL;
  a.in0 = (const char*)d->in0; a.in1 = (const char*)(d->in1 ? d->in1 : d->in0);
  a.c0 = d->c0; a.c1 = d->c1; a.ld0 = d->ld0; a.ld1 = d->c1 ? d->ld1 : d->ld0;
  a.n = d->n; a.h = d->h; a.w = d->w; a.up2 = d->up2;
  a.weight = (const char*)d->weight; a.wld = d->wld; a.bias = d->bias;
  a.cout = d->cout; a.kh = d->kh; a.kw = d->kw; a.stride = d->stride; a.pad_t = d->pad_t; a.pad_l = d->pad_l;
  a.ho = d->ho; a.wo = d->wo;
  a.gn_ab = d->gn_ab; a.gn_silu = d->gn_silu;
  a.emb = d->emb; a.emb_ld = d->emb_ld;
  a.act = d->act; a.act_param = d->act_param;
  a.res = (const char*)d->res; a.res_ld = d->res_ld;
  a.out = (char*)d->out; a.out_ld = d->out_ld; a.out_mode = d->out_mode;
  a.out_f32 = d->out_f32;
  a.epi_vec = g_epi_vec;
  a.splits = 1; a.kper = 0;
  a.gn_part = d->gn_part; a.gn_row0 = 0; a.gn_hw = d->gn_hw;
  a.ln_rows = d->ln_rows; a.ln_cs = d->ln_colsum;
  if ((d->ln_rows != nullptr) != (d->ln_colsum != nullptr)) return RDEIC_EINVAL;
  if (d->ln_rows && (d->dtype != 1 || d->batch > 1 || d->out_mode == 1 || d->gn_ab || ((uintptr_t)d->ln_colsum) % 16))
    return RDEIC_EINVAL;
  a.M = d->n * d->ho * d->wo;
  a.batch = d->batch > 1 ? d->batch : 1;
  a.in_bs = d->in_bs; a.w_bs = d->w_bs; a.out_bs = d->out_bs;
  if (a.batch > 1 && (d->res || d->emb || d->out_mode)) return RDEIC_EINVAL;
  a.cin = d->c0 + d->c1;
  a.ktot = d->kh * d->kw * a.cin;
  const int BK = d->dtype == 1 ? 64 : 32;
  if (d->wld < a.ktot || d->wld % 64 != 0) return RDEIC_EINVAL;
  a.nk = (a.ktot + BK - 1) / BK;
  if (d->out_mode < 0 || d->out_mode > 2) return RDEIC_EINVAL;
  if (d->out_mode == 1 && (d->cout % 4 != 0)) return RDEIC_EINVAL;
  if (d->out_mode == 2 && (d->dtype != 1 || d->cout % 8 || d->res || d->emb || d->act || d->out_f32 || d->gn_ab ||
                           a.batch > 1 || d->out_ld % 4 || ((uintptr_t)d->out) % 8))
    return RDEIC_EINVAL;
  const int epc = d->dtype == 1 ? 8 : 4;
  vec = (d->c0 % epc == 0) && (d->ld0 % epc == 0) && (((uintptr_t)d->in0) % 16 == 0);
  if (d->c1) vec = vec && (d->c1 % epc == 0) && (d->ld1 % epc == 0) && (((uintptr_t)d->in1) % 16 == 0);
  if (((uintptr_t)d->weight) % 16 != 0) return RDEIC_EINVAL;
  return RDEIC_OK;
}
}  // namespace

static int conv2d_run(const rdeic_conv_desc* d, void* stream, bool* fused) {
  ConvArgs a;
  bool vec = false;
  const int rc = make_args(d, a, vec);
  if (rc != RDEIC_OK) return rc;
  float* const part = a.gn_part;
  a.gn_part = nullptr;  // statistics fuse into the LDS-DMA (dma_grouped reads d) and big-tile register paths
  hipStream_t s = (hipStream_t)stream;
  {
    unsigned lb0 = 0, lbw = 0, lbo = 0;
    if (vec && g_lpersist && lp_ok(d, a, lb0, lbw, lbo)) return launch_lpersist(a, lb0, lbw, lbo, s);
  }
  if (d->out_mode == 2) {  // fused GEGLU exists in the LDS-DMA kernel's vector epilogue only
    const int rc2 = vec ? dma_grouped(d, -1, 1, nullptr, s) : -1;
    return rc2 == -1 ? RDEIC_EINVAL : rc2;
  }

  if (vec && g_halo && (d->gn_ab || g_halo == 2) && halo_ok(d, a)) {
    a.gn_part = part;
    const int rc2 = launch_halo(d, a, s, fused);
    if (rc2 != -1) return rc2;
    a.gn_part = nullptr;
  }
  if (d->dtype == 1 && vec && d->cout <= 4 && d->c0 % 32 == 0 && d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad_t == 1 &&
      d->pad_l == 1 && !d->up2 && !d->c1 && d->out_mode == 0 && a.batch == 1 && d->ho == d->h && d->wo == d->w &&
      g_conv_path != 0)
    return launch_smallc(a, s);
  if (d->dtype == 1 && vec && !d->gn_ab && d->cout > 32 && g_conv_path != 0) {
    if (g_dma) {
      const int rc2 = dma_grouped(d, -1, 1, nullptr, s, fused);
      if (rc2 != -1) return rc2;
    }
    a.gn_part = part;
    return launch_plain_auto(a, s, -1, fused);
  }
  if (d->dtype == 1) {
    if (d->cout <= 16) return launch_cfg<bf16, 128, 16, 4, 1>(a, vec, s);
    if (d->cout <= 32) return launch_cfg<bf16, 128, 32, 4, 1>(a, vec, s);
    if (d->cout % 128 != 0 && d->cout % 64 == 0) return launch_cfg<bf16, 128, 64, 2, 2>(a, vec, s);
    if (a.M <= 4096) return launch_cfg<bf16, 64, 128, 2, 2>(a, vec, s);
    return launch_cfg<bf16, 128, 128, 2, 2>(a, vec, s);
  } else {
    if (d->cout <= 16) return launch_cfg<float, 64, 16, 4, 1>(a, vec, s);
    // 128x128 tiles (64x64 per wave: 4096 MFMA cycles per k-tile hide the single-stage prefetch)
    // where their grid still fills the chip; same k order as 64x64, so bit-identical
    if (d->cout >= 128 && (long)cdiv(a.M, 128) * cdiv(a.cout, 128) * a.batch >= 512)
      return launch_cfg<float, 128, 128, 2, 2>(a, vec, s);
    return launch_cfg<float, 64, 64, 2, 2>(a, vec, s);
  }
}

// Explicit tile choice for the big-tile path (autotuning by the caller; every tile gives
// bit-identical results). tile -1 = the built-in heuristic. Shapes outside the big-tile path
// (GN prologue, cout <= 32, fp32, unaligned) ignore it and run exactly as rdeic_conv2d.
static int conv2d_tile_run(const rdeic_conv_desc* d, int32_t tile, void* stream, bool* fused) {
  ConvArgs a;
  bool vec = false;
  const int rc = make_args(d, a, vec);
  if (rc != RDEIC_OK) return rc;
  {  // the persistent short-K linear takes its shapes whatever the table's tile (tile 40 = it, when eligible)
    unsigned lb0 = 0, lbw = 0, lbo = 0;
    if (vec && (tile == 40 || (tile < 20 && g_lpersist) || g_lpersist == 2) && lp_ok(d, a, lb0, lbw, lbo))
      return launch_lpersist(a, lb0, lbw, lbo, (hipStream_t)stream);
  }
  if (d->out_mode == 2) {
    const int rc2 = vec ? dma_grouped(d, tile >= 20 ? tile : -1, 1, nullptr, (hipStream_t)stream) : -1;
    return rc2 == -1 ? RDEIC_EINVAL : rc2;
  }
  if (d->dtype == 1 && vec && !d->gn_ab && d->cout > 32 && g_conv_path != 0) {
    if (tile >= 20) {
      const int rc2 = dma_grouped(d, tile, 1, nullptr, (hipStream_t)stream, fused);
      if (rc2 != -1) return rc2;
      tile = -1;
    }
    return launch_plain_auto(a, (hipStream_t)stream, tile, fused);
  }
  return conv2d_run(d, stream, fused);
}

static double conv_flops(const rdeic_conv_desc* d) {
  if (!d) return 0.0;
  const double b = d->batch > 1 ? d->batch : 1;
  return 2.0 * b * d->n * d->ho * d->wo * d->cout * (double)d->kh * d->kw * (d->c0 + d->c1);
}

// algorithmic HBM bytes of one launch: every input element once (an upsampled input at its stored size),
// the packed weight once, the output, the residual (RDEIC_PROF_CONV_BYTES)
static double conv_bytes(const rdeic_conv_desc* d) {
  if (!d) return 0.0;
  const double b = d->batch > 1 ? d->batch : 1;
  const double es = d->dtype == 1 ? 2.0 : 4.0, os = (d->dtype == 0 || d->out_f32) ? 4.0 : 2.0;
  const double in = b * d->n * (double)d->h * d->w * (d->c0 + d->c1) * es;
  const double w = (double)(d->batch > 1 ? b : 1) * d->cout * d->wld * es;
  double outc = d->out_mode == 2 ? d->cout / 2.0 : (double)d->cout;
  const double out = b * d->n * (d->out_mode == 1 ? 4.0 : 1.0) * d->ho * d->wo * (d->out_mode == 1 ? outc / 4 : outc) * os;
  return in + w + out + (d->res ? out : 0.0);
}

// d->gn_part: the output's GroupNorm statistics in the partial format of rdeic_groupnorm_parts_ab,
// fused into the epilogue where the launch allows it, else by a separate pass over the output.
static int conv2d_impl(const rdeic_conv_desc* d, int32_t tile, void* stream) {
  if (d && d->gn_part &&
      (d->gn_hw <= 0 || d->gn_hw % 64 || d->batch > 1 || d->out_mode != 0 || (long)d->n * d->ho * d->wo % d->gn_hw))
    return RDEIC_EINVAL;
  bool fused = false;
  int rc;
  {
    rdeic_prof_add_bytes(conv_bytes(d));
    ProfScope ps((hipStream_t)stream, RDEIC_PROF_CONV, conv_flops(d));
    rc = tile == -2 ? conv2d_run(d, stream, &fused) : conv2d_tile_run(d, tile, stream, &fused);
  }
  if (rc != RDEIC_OK || !d->gn_part || fused) return rc;
  const long rows = (long)d->n * d->ho * d->wo;
  return gn_rows_partial(d->out, rows, d->cout, d->out_ld, d->gn_hw, d->gn_part,
                         (d->out_f32 || d->dtype == 0) ? 0 : 1, (hipStream_t)stream);
}

// Split-K variant (small-M, large-K layers): `splits` k-ranges computed into a caller-provided
// fp32 workspace of splits * M * cout floats, then reduced in split order (deterministic) with
// the bias / emb / activation / residual epilogue. bf16 or fp32, 16-byte gathers, no GN prologue,
// out_mode 0, batch 1, cout % 8 == 0. The k-order differs from rdeic_conv2d (not bit-identical
// to it), so callers that need batch invariance must not use it.
static int conv2d_splitk_impl(const rdeic_conv_desc* d, int32_t splits, float* ws, size_t ws_floats,
                              void* stream, bool* stats_done) {
  ConvArgs a;
  bool vec = false;
  const int rc = make_args(d, a, vec);
  if (rc != RDEIC_OK) return rc;
  if (!vec || d->gn_ab || d->out_mode != 0 || a.batch != 1 || d->cout % 8 || splits < 2 || !ws ||
      (d->out_ld % 8) || ((uintptr_t)d->out % 16) || ((uintptr_t)ws % 16))
    return RDEIC_EINVAL;
  if (ws_floats < (size_t)SK_CNT + (size_t)splits * a.M * a.cout) return RDEIC_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  float* const part = ws + SK_CNT;  // the first SK_CNT words are the folded form's tile counters
  if (d->dtype == 0) {  // fp32: 64x64 register-staged partial tiles, fp32 output from the reduction
    ConvArgs p = a;
    p.bias = nullptr; p.emb = nullptr; p.act = 0; p.res = nullptr; p.gn_part = nullptr; p.ln_rows = nullptr;
    p.out = (char*)part; p.out_ld = a.cout; p.out_f32 = 0;
    p.splits = splits;
    p.kper = (a.nk + splits - 1) / splits;
    dim3 grid(cdiv(a.M, 64), cdiv(a.cout, 64), splits);
    constexpr int lds = conv_lds_bytes<float, 64, 64>();
    hipLaunchKernelGGL((conv_kernel<float, 64, 64, 2, 2, true, false, false, true>), grid, dim3(256), lds, s, p);
    a.splits = splits;
    a.out_f32 = 1;  // the reduction's output (and residual) type: fp32
    const long chunks = (long)a.M * (a.cout / 8);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, a,
                       (const float*)part);
    return launch_status();
  }
  // LDS-DMA path: the reduction (and the output's GroupNorm statistics) folded into the producing launch's
  // last split per tile (splitk_fold) when the tile counters fit
  if (g_dma && g_sk_fold && (long)cdiv(a.M, 64) * cdiv(a.cout, 128) <= SK_CNT) {
    bool fused = false;
    if (dma_grouped(d, -1, splits, ws, s, &fused) == RDEIC_OK) {
      if (stats_done) *stats_done = d->gn_part && fused;
      return launch_status();
    }
  }
  if (g_dma && !g_sk_fold) {  // the unfolded LDS-DMA form (A/B and tests): partial launch, then the reduce kernel
    rdeic_conv_desc e = *d;
    e.bias = nullptr; e.emb = nullptr; e.act = 0; e.res = nullptr; e.gn_part = nullptr; e.ln_rows = nullptr;
    e.out = part; e.out_ld = d->cout; e.out_f32 = 1;
    ConvArgs pa;
    bool pv = false;
    unsigned b0, b1, bw;
    if (make_args(&e, pa, pv) == RDEIC_OK && pv && dma_ok(&e, pa, b0, b1, bw)) {
      pa.splits = splits; pa.kper = (pa.nk + splits - 1) / splits;
      if (launch_dma_auto(pa, b0, b1, bw, s, -1) == RDEIC_OK) {
        a.splits = splits;
        const long chunks = (long)a.M * (a.cout / 8);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, a,
                           (const float*)part);
        return launch_status();
      }
    }
  }
  ConvArgs p = a;  // partial pass: raw sums into the workspace
  p.bias = nullptr; p.emb = nullptr; p.act = 0; p.res = nullptr; p.gn_part = nullptr; p.ln_rows = nullptr;
  p.out = (char*)part; p.out_ld = a.cout; p.out_f32 = 1;
  p.splits = splits;
  p.kper = (a.nk + splits - 1) / splits;
  dim3 grid(cdiv(a.M, 128), cdiv(a.cout, 128), splits);
  constexpr int lds = conv_lds_bytes<bf16, 128, 128>();
  hipLaunchKernelGGL((conv_kernel<bf16, 128, 128, 2, 2, true, false, false, true>), grid, dim3(256), lds, s, p);
  a.splits = splits;
  const long chunks = (long)a.M * (a.cout / 8);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, a,
                     (const float*)part);
  return launch_status();
}

// algorithmic FLOPs of one launch (2 per MAC), for the launch profiler

extern "C" int rdeic_conv2d(const rdeic_conv_desc* d, void* stream) { return conv2d_impl(d, -2, stream); }

extern "C" int rdeic_conv2d_tile(const rdeic_conv_desc* d, int32_t tile, void* stream) {
  return conv2d_impl(d, tile, stream);
}

extern "C" int rdeic_conv2d_splitk(const rdeic_conv_desc* d, int32_t splits, float* ws, size_t ws_floats,
                                   void* stream) {
  if (d && d->gn_part && (d->gn_hw <= 0 || d->gn_hw % 64 || (long)d->n * d->ho * d->wo % d->gn_hw))
    return RDEIC_EINVAL;
  int rc;
  bool stats_done = false;
  {
    rdeic_prof_add_bytes(conv_bytes(d));
    ProfScope ps((hipStream_t)stream, RDEIC_PROF_CONV, conv_flops(d));
    rc = conv2d_splitk_impl(d, splits, ws, ws_floats, stream, &stats_done);
  }
  if (rc == RDEIC_OK) rdeic_count_launch(RDEIC_COUNT_SPLITK);
  if (rc != RDEIC_OK || !d->gn_part || stats_done) return rc;  // statistics of the reduced output: stand-alone pass
  return gn_rows_partial(d->out, (long)d->n * d->ho * d->wo, d->cout, d->out_ld, d->gn_hw, d->gn_part,
                         d->out_f32 ? 0 : 1, (hipStream_t)stream);
}

extern "C" int rdeic_set_conv_path(int32_t path) {
  int prev = g_conv_path;
  g_conv_path = path;
  return prev;
}

extern int rdeic_g_attn64;
extern int rdeic_g_attn512;

extern "C" int rdeic_set_conv_option(int32_t key, int32_t value) {
  if (key == 0) { int prev = g_epi_vec; g_epi_vec = value; return prev; }
  if (key == 1) { int prev = rdeic_g_attn64; rdeic_g_attn64 = value; return prev; }
  if (key == 2) { int prev = g_pf2; g_pf2 = value; return prev; }
  if (key == 3) { int prev = g_swz; g_swz = value; return prev; }
  if (key == 4) { int prev = g_force_tile; g_force_tile = value; return prev; }
  if (key == 5) { int prev = g_dma; g_dma = value; return prev; }
  if (key == 6) { int prev = g_halo; g_halo = value; return prev; }
  if (key == 8) { int prev = rdeic_g_attn512; rdeic_g_attn512 = value; return prev; }
  if (key == 9) { int prev = g_halo8; g_halo8 = value; return prev; }
  if (key == 10) { int prev = g_halo256; g_halo256 = value; return prev; }
  if (key == 11) { int prev = g_sk_fold; g_sk_fold = value; return prev; }
  if (key == 12) { int prev = g_lpersist; g_lpersist = value; return prev; }
  return RDEIC_EINVAL;
}
