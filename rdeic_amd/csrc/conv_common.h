// Shared definitions of the convolution / linear kernels (conv_gemm.hip: register-staged tiles, the tiny-cout
// kernel, split-K reduce, dispatch and the C ABI; conv_dma.hip: the LDS-DMA implicit GEMM; conv_halo.hip: the
// GroupNorm-fused 3x3 halo convs; conv_edge.hip: the VAE edge convs). Kernel arguments, the fused epilogues and
// the LDS-DMA / wait helpers live here so the translation units compile in parallel.
#pragma once
#include "common.h"
#include "../../include/rdeic_hip.h"
#include "prof.h"

namespace rdeic_conv {

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
};

// Folded LayerNorm (rdeic_conv_desc.ln_rows): LN(x) W = rstd (x W' - mean colsum(W')) with W' = diag(gamma) W
// and beta W in the bias; applied to the raw accumulator before everything else of the epilogue.
__device__ __forceinline__ float ln_fold(const ConvArgs& a, int m, int n, float v) {
  const float2 ms = reinterpret_cast<const float2*>(a.ln_rows)[m];
  return ms.y * (v - ms.x * a.ln_cs[n]);
}

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

// Fused GEGLU epilogue (out_mode 2, attention.py:49-56): the packed weight interleaves 4 value rows with their 4
// gate rows, so two adjacent 8-column chunks (x0..x3, g0..g3, x4..x7, g4..g7) are 8 consecutive outputs. Each
// thread takes such chunk PAIRS and writes one 16-byte store per pair, where epilogue_vec writes one 8-byte store
// per chunk: half the store instructions for the same bytes (a tile's epilogue is bound by the CU's
// store-instruction rate, MI355X_MICROARCH.md). Per element the arithmetic is epilogue_vec's (LayerNorm fold,
// bias, bf16 rounding of both halves, x * gelu(g)), so outputs are bit-identical to it. Needs cout % 16 == 0.
template <int BM, int BN, int WGM, int WGN, int NT, int P>
__device__ __forceinline__ void epilogue_geglu(const f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16], const ConvArgs& a,
                                               int m0, int n0, int wm, int wn, int lane, int tid, char* lds) {
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int HM = TM / P;        // fragment rows per pass
  constexpr int PR = BM / P;        // tile rows per pass
  constexpr int SDW = BN + 4;       // LDS row stride in dwords
  constexpr int DPR = BN / 16;      // chunk pairs per row
  constexpr int ND = (PR * DPR + NT - 1) / NT;
  constexpr int NPF = ND < 2 ? ND : 2;      // LayerNorm row statistics prefetched per pass (as epilogue_vec)
  constexpr bool HOIST = (NT % DPR) == 0;  // every pair of a thread has the same 16 columns
  static_assert(TM % P == 0 && BN % 16 == 0, "P passes, chunk pairs");
  const int lr = lane & 15, lq = lane >> 4;
  float* L = reinterpret_cast<float*>(lds);
  auto bar = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto row_of = [&](int d, int p) {
    const int pr = d / DPR;
    const int wmr = pr / (WTM / P), wr = pr - wmr * (WTM / P);
    return m0 + wmr * WTM + p * (WTM / P) + wr;
  };
  // bias / LayerNorm column sums of this thread's 16 columns, once (loaded before the first park)
  float4 bh[4], chh[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bh[q] = chh[q] = float4{0.f, 0.f, 0.f, 0.f};
  if constexpr (HOIST) {
    const int nn = n0 + (tid % DPR) * 16;
    if (nn < a.cout) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (a.bias) bh[q] = *reinterpret_cast<const float4*>(a.bias + nn + 4 * q);
        if (a.ln_rows) chh[q] = *reinterpret_cast<const float4*>(a.ln_cs + nn + 4 * q);
      }
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    float2 lpf[NPF];
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int d = tid + k * NT;
      const int m = row_of(d, p);
      lpf[k] = float2{0.f, 0.f};
      if (a.ln_rows && d < PR * DPR && m < a.M) lpf[k] = reinterpret_cast<const float2*>(a.ln_rows)[m];
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
    for (int k = 0; k < ND; ++k) {
      const int d = tid + k * NT;
      if (d >= PR * DPR) continue;
      const int pr = d / DPR, cq = d - pr * DPR;
      const int m = row_of(d, p);
      const int nn = n0 + cq * 16;
      if (m >= a.M || nn >= a.cout) continue;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(L + pr * SDW + cq * 16 + 4 * q);
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
      if (a.ln_rows) {  // v = rstd * (v - mean * colsum), two columns per packed fma / mul
        const float2 ms = k < NPF ? lpf[k < NPF ? k : 0] : reinterpret_cast<const float2*>(a.ln_rows)[m];
        const f32x2 nm = {-ms.x, -ms.x}, rs = {ms.y, ms.y};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 c = HOIST ? chh[q] : *reinterpret_cast<const float4*>(a.ln_cs + nn + 4 * q);
          const float cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2 r = rs * pk_fma(nm, f32x2{cs[e], cs[e + 1]}, f32x2{v[4 * q + e], v[4 * q + e + 1]});
            v[4 * q + e] = r.x;
            v[4 * q + e + 1] = r.y;
          }
        }
      }
      if (a.bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 b = HOIST ? bh[q] : *reinterpret_cast<const float4*>(a.bias + nn + 4 * q);
          const f32x2 r0 = f32x2{v[4 * q], v[4 * q + 1]} + f32x2{b.x, b.y};
          const f32x2 r1 = f32x2{v[4 * q + 2], v[4 * q + 3]} + f32x2{b.z, b.w};
          v[4 * q] = r0.x; v[4 * q + 1] = r0.y; v[4 * q + 2] = r1.x; v[4 * q + 3] = r1.y;
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = apply_act(v[e], a.act, a.act_param);
      bf16 gv[8];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f32x2 xv = {to_f32(from_f32<bf16>(v[8 * h + e])), to_f32(from_f32<bf16>(v[8 * h + e + 1]))};
          const f32x2 gt = {to_f32(from_f32<bf16>(v[8 * h + 4 + e])), to_f32(from_f32<bf16>(v[8 * h + 5 + e]))};
          const f32x2 r = xv * gelu_fast2(gt);
          gv[4 * h + e] = from_f32<bf16>(r.x);
          gv[4 * h + e + 1] = from_f32<bf16>(r.y);
        }
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(a.out) + (long)m * a.out_ld + (nn >> 1)) =
          *reinterpret_cast<uint4*>(gv);
    }
  }
}

constexpr unsigned kOOB = 0x80000000u;  // voffset that reads zeros (buffers are < 2 GiB)

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

// process-wide switches (rdeic_set_conv_option / rdeic_set_conv_path), defined in conv_gemm.hip
extern int g_conv_path, g_epi_vec, g_swz, g_force_tile, g_dma, g_halo, g_halo8, g_edge;

// cross-unit entry points
int make_args(const rdeic_conv_desc* d, ConvArgs& a, bool& vec);                                     // conv_gemm.hip
bool dma_ok(const rdeic_conv_desc* d, const ConvArgs& a, unsigned& b0, unsigned& b1, unsigned& bw);  // conv_dma.hip
int launch_dma_auto(const ConvArgs& a, unsigned b0, unsigned b1, unsigned bw, hipStream_t s, int tile,
                    int gn_hw = 0, bool* fused = nullptr);
int dma_grouped(const rdeic_conv_desc* d, int tile, hipStream_t s, bool* fused = nullptr);
bool halo_ok(const rdeic_conv_desc* d, const ConvArgs& a);                                          // conv_halo.hip
int launch_halo(const rdeic_conv_desc* d, ConvArgs a, hipStream_t s, bool* fused);
int launch_edge(const rdeic_conv_desc* d, const ConvArgs& a, hipStream_t s, bool* fused);  // conv_edge.hip
}  // namespace rdeic_conv
