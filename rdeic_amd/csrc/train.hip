// Backward and optimizer kernels of the adapter fine-tune step (config 5, SURVEY.md §8f rank 1:
// model/rdeic.py:763-881 p_losses / configure_optimizers, model/compression.py:52-149 Compression.forward,
// model/compression_modules.py:228-307 VectorQuantiser.forward) on gfx950.
//
//   * strided batched GEMM on MFMA (weight gradients, attention backward, VQ distances): every operand
//     addressed by (batch, row, col) strides, so no transposed copies are ever materialised;
//   * conv backward helpers: flipped / transposed weight packing (input gradients run on the forward
//     implicit-GEMM conv), im2col for the weight-gradient GEMM, stride-2 zero insertion, nearest-up
//     sum pooling, pixel unshuffle, split-K reduction into the torch weight layout;
//   * deterministic column sums (bias / timestep-embedding gradients), activation forward/backward;
//   * GroupNorm(+SiLU) training forward (mean / rstd kept) and backward, LayerNorm backward,
//     row-softmax backward, GEGLU backward;
//   * the checkerboard entropy model's training forward / backward (compressai GaussianConditional
//     "noise" likelihood with LowerBound semantics, quantize_ste), the VQ codebook step
//     (commitment + contrastive loss, dead-code re-initialisation) and AdamW.
// Every reduction runs in a fixed order (no atomics): a step is bit-reproducible run to run.
#include "common.h"
#include "../../include/rdeic_hip.h"
#include "prof.h"

// the optimizer / loss arithmetic follows torch's separate roundings: no fma contraction
#pragma clang fp contract(off)

namespace {

inline int grid_1d(long total, int per = 256) { return (int)std::min<long>((total + per - 1) / per, 65536L); }

template <typename T> __device__ __forceinline__ float ldf(const T* p, long i) { return to_f32(p[i]); }

// ------------------------------------------------------------------------------------------------
// Strided batched GEMM: C[z] = alpha * A[z] B[z] (+ beta * C[z]), A[z] m x k, B[z] k x n, fp32 MFMA
// accumulate. A(i, kk) = a[z-offset + i*a_sm + kk*a_sk], B(kk, j) = b[z-offset + kk*b_sk + j*b_sn],
// C(i, j) = c[z-offset + i*c_sm + j]. Batch z = z1 * nb2 + z2 with two stride pairs (images x heads).
// ksplit > 0: z1 indexes a k-range of that length instead (split-K into separate C planes, c_bs1).
// Tiles 64x64x32, 4 waves of 32x32; the staging mapping follows whichever operand dim is contiguous.
struct GemmArgs {
  const void* a;
  long a_bs1, a_bs2, a_sm, a_sk;
  const void* b;
  long b_bs1, b_bs2, b_sk, b_sn;
  void* c;
  long c_bs1, c_bs2, c_sm;
  int nb2, m, n, k, ksplit, c_f32;
  float alpha, beta;
  float* rsum;  // optional row sums of A (see rdeic_gemm_desc)
  long rsum_bs;
};

constexpr int GBK = 32;

// Operand images in LDS. An operand whose k stride is 1 ("KC") is staged as rows of the tile's
// m (or n) index with k contiguous, [TB][GBK + pad], and read as 8 consecutive k per lane. Any
// other operand ("MN": m / n contiguous in memory, or generic strides) is staged as rows of k,
// [GBK][TB], with one 16-byte write per 8 elements; bf16 lanes then read it with the gfx950
// transposed read ds_read_b64_tr_b16 (two per 16x16x32 fragment, delivering the same k -> lane
// mapping as the KC image, so both images give bit-identical products). The bf16 MN image has no
// pad: its 32-byte slots are XOR-swizzled by the row (mn_swz) so that the eight rows one 32-lane
// half reads (k = 8lg + q, lg = 0/1, q = 0..3) land on eight different bank groups. fp32 MN images
// are read one element per lane (16x16x4 f32 operand) with a 16-float pad.
template <int TB>
__device__ __forceinline__ int mn_swz(int k) {
  return TB == 128 ? ((k & 3) | (((k >> 3) & 1) << 2)) : (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}
template <typename T, int TB>
__device__ __forceinline__ int mn_off(int k, int m) {  // element offset of (k, m) in an MN image
  if constexpr (sizeof(T) == 2) return k * TB + ((((m >> 4) ^ mn_swz<TB>(k))) << 4) + (m & 15);
  else return k * (TB + 16) + m;
}

typedef short short4v __attribute__((ext_vector_type(4)));

// the 8 k values (8lg .. 8lg+7) of row `r` of an MN bf16 image for this lane, as one MFMA operand
template <int TB>
__device__ __forceinline__ bf16x8 mn_frag(const bf16* S, int r0, int lane) {
  const int lg = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int m = r0 + 4 * p;
  const int k0 = 8 * lg + q;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(S + mn_off<bf16, TB>(k0, m)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(S + mn_off<bf16, TB>(k0 + 4, m)));
  // one shuffle + bit cast (element-wise __bf16 inserts were packed wrongly by this compiler)
  typedef short short8v __attribute__((ext_vector_type(8)));
  const short8v r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// TB x TB tile (64 or 128), 4 waves of (TB/2)^2; each thread stages TB/64 groups of 8 elements per
// operand. AKC / BKC: the operand's k stride is 1 (KC image), else MN image (see above).
template <typename T, int TB, bool AKC, bool BKC>
__global__ __launch_bounds__(256) void gemm_strided_kernel(GemmArgs g) {
  constexpr int PAD = sizeof(T) == 2 ? 8 : 4;
  constexpr int G = TB / 64, TF = TB / 32;  // staging groups per thread, 16x16 fragments per wave dim
  constexpr int KC_ELEMS = TB * (GBK + PAD);
  constexpr int MN_ELEMS = sizeof(T) == 2 ? GBK * TB : GBK * (TB + 16);
  constexpr int A_ELEMS = AKC ? KC_ELEMS : MN_ELEMS, B_ELEMS = BKC ? KC_ELEMS : MN_ELEMS;
  __shared__ __attribute__((aligned(16))) T As[A_ELEMS];
  __shared__ __attribute__((aligned(16))) T Bs[B_ELEMS];
  const int z = blockIdx.z, z1 = z / g.nb2, z2 = z - z1 * g.nb2;
  const T* A = (const T*)g.a + z2 * g.a_bs2;
  const T* B = (const T*)g.b + z2 * g.b_bs2;
  long klen = g.k;
  if (g.ksplit > 0) {
    const long k0 = (long)z1 * g.ksplit;
    klen = min((long)g.ksplit, (long)g.k - k0);
    A += k0 * g.a_sk;
    B += k0 * g.b_sk;
  } else {
    A += z1 * g.a_bs1;
    B += z1 * g.b_bs1;
  }
  const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
  // staging coordinates of group 0 (group q adds 64 rows of m / n)
  const int ar = AKC ? (tid >> 2) : ((tid & 7) * 8), ak = AKC ? ((tid & 3) * 8) : (tid >> 3);
  const int br = BKC ? (tid >> 2) : ((tid & 7) * 8), bk = BKC ? ((tid & 3) * 8) : (tid >> 3);
  T ra[G][8], rb[G][8];
  // the 8 elements of a group are contiguous in memory when the staged dimension has stride 1
  // (k for KC, else m / n): one (bf16) or two (fp32) 16-byte loads when aligned and in bounds,
  // element loads otherwise
  const bool a_vec = AKC || g.a_sm == 1, b_vec = BKC || g.b_sn == 1;
  auto load8 = [&](const T* base, long step, bool contiguous, int valid, T (&r)[8]) {
    if (contiguous && valid == 8 && ((uintptr_t)base & 15) == 0) {
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(r) = *reinterpret_cast<const uint4*>(base);
      } else {
        reinterpret_cast<uint4*>(r)[0] = reinterpret_cast<const uint4*>(base)[0];
        reinterpret_cast<uint4*>(r)[1] = reinterpret_cast<const uint4*>(base)[1];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = e < valid ? base[e * step] : from_f32<T>(0.f);
    }
  };
  auto load = [&](long k0) {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int arq = ar + 64 * q, brq = br + 64 * q;
      const long kk = k0 + ak, kb = k0 + bk;
      if constexpr (AKC) {
        const int valid = (m0 + arq < g.m) ? (int)max(0L, min(8L, klen - kk)) : 0;
        load8(A + (long)(m0 + arq) * g.a_sm + kk, 1, true, valid, ra[q]);
      } else {
        const int valid = kk < klen ? max(0, min(8, g.m - (m0 + arq))) : 0;
        load8(A + (long)(m0 + arq) * g.a_sm + kk * g.a_sk, g.a_sm, a_vec, valid, ra[q]);
      }
      if constexpr (BKC) {
        const int valid = (n0 + brq < g.n) ? (int)max(0L, min(8L, klen - kb)) : 0;
        load8(B + kb + (long)(n0 + brq) * g.b_sn, 1, true, valid, rb[q]);
      } else {
        const int valid = kb < klen ? max(0, min(8, g.n - (n0 + brq))) : 0;
        load8(B + kb * g.b_sk + (long)(n0 + brq) * g.b_sn, g.b_sn, b_vec, valid, rb[q]);
      }
    }
  };
  auto store16 = [&](T* dst, const T (&r)[8]) {
    if constexpr (sizeof(T) == 2) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(r);
    else { reinterpret_cast<uint4*>(dst)[0] = reinterpret_cast<const uint4*>(r)[0];
           reinterpret_cast<uint4*>(dst)[1] = reinterpret_cast<const uint4*>(r)[1]; }
  };
  auto store = [&](T* S, bool kc, int r0, int k0s, const T (&r)[8]) {
    if (kc) store16(S + r0 * (GBK + PAD) + k0s, r);
    else store16(S + mn_off<T, TB>(k0s, r0), r);
  };
  f32x4 acc[TF][TF];
#pragma unroll
  for (int i = 0; i < TF; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = (wave >> 1) * (TB / 2), wn = (wave & 1) * (TB / 2);
  // row sums of A (bias gradient): the n-column-0 blocks' left waves run one extra MFMA per A
  // fragment against a ones operand
  const bool rs = g.rsum != nullptr && blockIdx.x == 0 && (wave & 1) == 0;
  f32x4 racc[TF];
#pragma unroll
  for (int i = 0; i < TF; ++i) racc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0);
  for (long k0 = 0; k0 < klen; k0 += GBK) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < G; ++q) {
      store(As, AKC, ar + 64 * q, ak, ra[q]);
      store(Bs, BKC, br + 64 * q, bk, rb[q]);
    }
    __syncthreads();
    if (k0 + GBK < klen) load(k0 + GBK);
    if constexpr (sizeof(T) == 2) {
      bf16x8 af[TF], bfr[TF];
#pragma unroll
      for (int i = 0; i < TF; ++i)
        af[i] = AKC ? *reinterpret_cast<const bf16x8*>(&As[(wm + 16 * i + lr) * (GBK + PAD) + 8 * lg])
                    : mn_frag<TB>(As, wm + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < TF; ++j)
        bfr[j] = BKC ? *reinterpret_cast<const bf16x8*>(&Bs[(wn + 16 * j + lr) * (GBK + PAD) + 8 * lg])
                     : mn_frag<TB>(Bs, wn + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (rs) {
        bf16x8 ones;
#pragma unroll
        for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
#pragma unroll
        for (int i = 0; i < TF; ++i) racc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, racc[i], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < GBK / 4; ++s) {
        float af[TF], bfr[TF];
#pragma unroll
        for (int i = 0; i < TF; ++i)
          af[i] = AKC ? As[(wm + 16 * i + lr) * (GBK + PAD) + 4 * s + lg] : As[mn_off<T, TB>(4 * s + lg, wm + 16 * i + lr)];
#pragma unroll
        for (int j = 0; j < TF; ++j)
          bfr[j] = BKC ? Bs[(wn + 16 * j + lr) * (GBK + PAD) + 4 * s + lg] : Bs[mn_off<T, TB>(4 * s + lg, wn + 16 * j + lr)];
#pragma unroll
        for (int i = 0; i < TF; ++i)
#pragma unroll
          for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if (rs) {
#pragma unroll
          for (int i = 0; i < TF; ++i) racc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], 1.0f, racc[i], 0, 0, 0);
        }
      }
    }
  }
  if (rs && lr == 0) {  // every column of racc holds the row sum; lanes of column 0 write 4 rows each
    float* rp = g.rsum + (long)z1 * g.rsum_bs;
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = m0 + wm + 16 * i + 4 * lg + r;
        if (mm < g.m) rp[mm] = racc[i][r];
      }
  }
  const long coff = z1 * g.c_bs1 + z2 * g.c_bs2;
#pragma unroll
  for (int i = 0; i < TF; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = m0 + wm + 16 * i + 4 * lg + r, nn = n0 + wn + 16 * j + lr;
        if (mm >= g.m || nn >= g.n) continue;
        const long ci = coff + (long)mm * g.c_sm + nn;
        float v = g.alpha * acc[i][j][r];
        if (g.c_f32) {
          float* cp = (float*)g.c;
          if (g.beta != 0.f) v += g.beta * cp[ci];
          cp[ci] = v;
        } else {
          T* cp = (T*)g.c;
          if (g.beta != 0.f) v += g.beta * to_f32(cp[ci]);
          cp[ci] = from_f32<T>(v);
        }
      }
}

template <typename T, int TB>
void launch_gemm(const GemmArgs& g, dim3 grid, hipStream_t s) {
  const bool akc = g.a_sk == 1, bkc = g.b_sk == 1;
  if (akc && bkc) hipLaunchKernelGGL((gemm_strided_kernel<T, TB, true, true>), grid, dim3(256), 0, s, g);
  else if (akc) hipLaunchKernelGGL((gemm_strided_kernel<T, TB, true, false>), grid, dim3(256), 0, s, g);
  else if (bkc) hipLaunchKernelGGL((gemm_strided_kernel<T, TB, false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_strided_kernel<T, TB, false, false>), grid, dim3(256), 0, s, g);
}

// ------------------------------------------------------------------------------------------------
// conv backward helpers
// dgrad weight: out[ci][(ky*kw + kx)*cout + co] = w[co][ci][kh-1-ky][kw-1-kx] (zero tail to wld):
// the input gradient is then the forward conv of dy with pad kh-1-pad.
template <typename T>
__global__ void pack_dgrad_kernel(const float* __restrict__ w, int cout, int cin, int kh, int kw, T* __restrict__ out,
                                  int wld) {
  const long total = (long)cin * wld;
  const int K = kh * kw * cout;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int ci = (int)(i / wld), kk = (int)(i - (long)ci * wld);
    float v = 0.f;
    if (kk < K) {
      const int tap = kk / cout, co = kk - tap * cout;
      const int ky = tap / kw, kx = tap - ky * kw;
      v = w[(((long)co * cin + ci) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)];
    }
    out[i] = from_f32<T>(v);
  }
}

// all trainable layers' forward / input-gradient packings in one launch (rdeic_pack_batch): one
// workgroup per output row; the row's sources are read coalesced into LDS, then written in the
// packed k order (LDS reads at stride kh*kw: conflict-free for the odd 1x1 / 3x3 / 5x5 filters)
constexpr int PACK_ROW_MAX = 36864;  // floats of LDS per row (144 KB)
template <typename T>
__global__ __launch_bounds__(256) void pack_batch_kernel(const rdeic_pack_job* __restrict__ jobs, int njobs) {
  extern __shared__ float srow[];
  const long r = blockIdx.x;
  int lo = 0, hi = njobs - 1;  // last job with start <= r
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].start <= r) lo = mid; else hi = mid - 1;
  }
  const rdeic_pack_job j = jobs[lo];
  const int row = (int)(r - j.start), khw = j.kh * j.kw, t = threadIdx.x;
  T* out = reinterpret_cast<T*>(j.out) + (long)row * j.wld;
  if (j.mode == 0) {  // row = co: w[co][ci][tap] contiguous -> out[(tap, ci)]
    const int K = j.cin * khw;
    const float* src = j.w + (long)row * K;
    for (int i = t; i < K; i += 256) srow[i] = src[i];
    __syncthreads();
    for (int k = t; k < j.wld; k += 256) {
      float v = 0.f;
      if (k < K) { const int tap = k / j.cin, ci = k - tap * j.cin; v = srow[ci * khw + tap]; }
      out[k] = from_f32<T>(v);
    }
  } else {  // row = ci: w[co][ci][tap] for every co -> out[(flipped tap, co)]
    const int K = j.cout * khw;
    for (int i = t; i < K; i += 256) {
      const int co = i / khw, tap = i - co * khw;
      srow[i] = j.w[((long)co * j.cin + row) * khw + tap];
    }
    __syncthreads();
    for (int k = t; k < j.wld; k += 256) {
      float v = 0.f;
      if (k < K) {
        const int tap = k / j.cout, co = k - tap * j.cout;
        const int ky = tap / j.kw, kx = tap - ky * j.kw;
        v = srow[co * khw + (j.kh - 1 - ky) * j.kw + (j.kw - 1 - kx)];
      }
      out[k] = from_f32<T>(v);
    }
  }
}

// out[p][(ky*kw + kx)*c + ci] = x at the tap's input pixel (zero outside; up2: nearest-upsampled input)
template <typename T>
__global__ void im2col_kernel(const T* __restrict__ x, int n, int h, int w, int c, int ld, int kh, int kw, int stride,
                              int pad_t, int pad_l, int ho, int wo, int up2, T* __restrict__ out, long out_ld) {
  const int K = kh * kw * c;
  const long total = (long)n * ho * wo * K;
  const int hi = up2 ? 2 * h : h, wi = up2 ? 2 * w : w;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long p = i / K;
    const int kk = (int)(i - p * K);
    const int tap = kk / c, ci = kk - tap * c;
    const int ky = tap / kw, kx = tap - ky * kw;
    const int img = (int)(p / ((long)ho * wo));
    const int rem = (int)(p - (long)img * ho * wo);
    const int oy = rem / wo, ox = rem - oy * wo;
    const int iy = oy * stride - pad_t + ky, ix = ox * stride - pad_l + kx;
    T v = from_f32<T>(0.f);
    if (iy >= 0 && iy < hi && ix >= 0 && ix < wi) {
      const int sy = up2 ? iy >> 1 : iy, sx = up2 ? ix >> 1 : ix;
      v = x[(((long)img * h + sy) * w + sx) * ld + ci];
    }
    out[p * out_ld + kk] = v;
  }
}

// dst [n][2h][2w][c]: src at even positions, zero elsewhere (input gradient of a stride-2 conv)
template <typename T>
__global__ void zero_insert2_kernel(const T* __restrict__ src, int n, int h, int w, int c, int ld, T* __restrict__ dst,
                                    int dld) {
  const long total = (long)n * 4 * h * w * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int img = (int)(pix / (4L * h * w));
    const int rem = (int)(pix - (long)img * 4 * h * w);
    const int y = rem / (2 * w), x = rem - y * 2 * w;
    T v = from_f32<T>(0.f);
    if (!(y & 1) && !(x & 1)) v = src[(((long)img * h + (y >> 1)) * w + (x >> 1)) * ld + ch];
    dst[pix * dld + ch] = v;
  }
}

// dst[n][h][w][c] = sum of the 2x2 block of src [n][2h][2w][c] (nearest-upsample backward)
template <typename T>
__global__ void sum_pool2_kernel(const T* __restrict__ src, int n, int h, int w, int c, int ld, T* __restrict__ dst,
                                 int dld) {
  const long total = (long)n * h * w * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int img = (int)(pix / ((long)h * w));
    const int rem = (int)(pix - (long)img * h * w);
    const int y = rem / w, x = rem - y * w;
    const T* s = src + (((long)img * 2 * h + 2 * y) * 2 * w + 2 * x) * ld + ch;
    const float v = (to_f32(s[0]) + to_f32(s[ld])) + (to_f32(s[(long)2 * w * ld]) + to_f32(s[(long)2 * w * ld + ld]));
    dst[pix * dld + ch] = from_f32<T>(v);
  }
}

// dst [n][h][w][4c], dst[.., 4*cc + 2*i + j] = src[n][2y+i][2x+j][cc]  (PixelShuffle(2) backward)
template <typename T>
__global__ void pixel_unshuffle2_kernel(const T* __restrict__ src, int n, int h, int w, int c, int ld,
                                        T* __restrict__ dst, int dld) {
  const long total = (long)n * h * w * 4 * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / (4 * c);
    const int ch4 = (int)(i - pix * 4 * c);
    const int cc = ch4 >> 2, ii = (ch4 >> 1) & 1, jj = ch4 & 1;
    const int img = (int)(pix / ((long)h * w));
    const int rem = (int)(pix - (long)img * h * w);
    const int y = rem / w, x = rem - y * w;
    dst[pix * dld + ch4] = src[(((long)img * 2 * h + 2 * y + ii) * 2 * w + 2 * x + jj) * ld + cc];
  }
}

// dw[co][ci][ky][kx] (+)= sum_s part[s][co][(ky*kw + kx)*cin + ci]
__global__ void wgrad_finalize_kernel(const float* __restrict__ part, int splits, int cout, int cin, int kh, int kw,
                                      float* __restrict__ dw, int accumulate, const float* __restrict__ rpart,
                                      float* __restrict__ db) {
  const int K = kh * kw * cin;
  const long total = (long)cout * K;
  if (db && blockIdx.x == 0) {  // bias gradient: the GEMM's row-sum planes, summed in split order
    for (int co = threadIdx.x; co < cout; co += 256) {
      float s = 0.f;
      for (int sp = 0; sp < splits; ++sp) s += rpart[(long)sp * cout + co];
      db[co] = accumulate ? db[co] + s : s;
    }
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int co = (int)(i / K), kk = (int)(i - (long)co * K);
    float s = 0.f;
    for (int sp = 0; sp < splits; ++sp) s += part[(long)sp * total + i];
    const int tap = kk / cin, ci = kk - tap * cin;
    const int ky = tap / kw, kx = tap - ky * kw;
    float* d = dw + (((long)co * cin + ci) * kh + ky) * kw + kx;
    *d = accumulate ? *d + s : s;
  }
}

// column sums: stage 1 per (group, row chunk), stage 2 over chunks in order
// Rows per stage-1 block: 32 (B=1 training shapes: enough blocks to fill the chip), growing with
// the row count so that stage 2 sums at most 256 partials per column.
inline long cs_rows(long rows_per_group) {
  long r = 32;
  while ((rows_per_group + r - 1) / r > 256) r *= 2;
  return r;
}
template <typename T>
__global__ void col_sum_partial_kernel(const T* __restrict__ x, long rows_per_group, int c, int ld, int nchunk,
                                       long rpc, float* __restrict__ ws) {
  const int grp = blockIdx.z, chunk = blockIdx.y, ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= c) return;
  const long r0 = (long)chunk * rpc, r1 = min(rows_per_group, r0 + rpc);
  const T* xp = x + ((long)grp * rows_per_group) * ld + ch;
  float s = 0.f;
  long r = r0;
  for (; r + 8 <= r1; r += 8) {  // 8 loads in flight, then the row-ordered adds
    float y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) y[u] = to_f32(xp[(r + u) * ld]);
#pragma unroll
    for (int u = 0; u < 8; ++u) s += y[u];
  }
  for (; r < r1; ++r) s += to_f32(xp[r * ld]);
  ws[((long)grp * nchunk + chunk) * c + ch] = s;
}

__global__ void col_sum_final_kernel(const float* __restrict__ ws, int groups, int nchunk, int c,
                                     float* __restrict__ out, int accumulate) {
  const long total = (long)groups * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int grp = (int)(i / c), ch = (int)(i - (long)grp * c);
    const float* w = ws + (long)grp * nchunk * c + ch;
    float s = 0.f;
    int q = 0;
    for (; q + 8 <= nchunk; q += 8) {
      float y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) y[u] = w[(long)(q + u) * c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += y[u];
    }
    for (; q < nchunk; ++q) s += w[(long)q * c];
    out[i] = accumulate ? out[i] + s : s;
  }
}

// activations: 1 leaky (slope), 2 exact GELU, 3 SiLU
__device__ __forceinline__ float act_f(float z, int act, float slope) {
  if (act == 1) return z > 0.f ? z : z * slope;
  if (act == 2) return gelu_f(z);
  if (act == 3) return z / (1.f + expf(-z));
  return z;
}
__device__ __forceinline__ float act_df(float z, int act, float slope) {
  if (act == 1) return z > 0.f ? 1.f : slope;
  if (act == 2) return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * expf(-0.5f * z * z);
  if (act == 3) {
    const float s = 1.f / (1.f + expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  return 1.f;
}

// rows x c views with row strides (a contiguous tensor is rows = numel / c, ld = c)
template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ z, long rows, int c, int ldz, const T* __restrict__ res, int ldr,
                               int act, float slope, T* __restrict__ out, int ldo) {
  const long total = rows * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / c;
    const int j = (int)(i - r * c);
    float v = act_f(to_f32(z[r * ldz + j]), act, slope);
    if (res) v += to_f32(res[r * ldr + j]);
    out[r * ldo + j] = from_f32<T>(v);
  }
}

template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ dy, int ldy, const T* __restrict__ z, int ldz, long rows, int c,
                               int act, float slope, T* __restrict__ dz, int lddz) {
  const long total = rows * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / c;
    const int j = (int)(i - r * c);
    dz[r * lddz + j] = from_f32<T>(to_f32(dy[r * ldy + j]) * act_df(to_f32(z[r * ldz + j]), act, slope));
  }
}

// ------------------------------------------------------------------------------------------------
// GroupNorm (training). Partials per (image, pixel chunk, channel) in fp64:
//   MODE 0 (forward):  (sum x, sum x^2)
//   MODE 1 (backward): (sum dY, sum dY * xhat), dY = dy * silu'(gamma*xhat + beta) (or dy)
constexpr int GNT_CHUNK = 32;  // pixels per partial (grid = chunks x images x 256-channel blocks)
template <typename T, int MODE>
__global__ __launch_bounds__(256) void gnt_partial_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ dy,
                                                          int ldy, int hw, int c, int groups, int nchunk,
                                                          const float* __restrict__ mr, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, int silu,
                                                          double* __restrict__ part) {
  const int img = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * GNT_CHUNK, p1 = min(hw, p0 + GNT_CHUNK);
  const int cpg = c / groups;
  {
    const int ch = blockIdx.z * 256 + threadIdx.x;
    if (ch >= c) return;
    double s1 = 0.0, s2 = 0.0;
    float mean = 0.f, rstd = 0.f, ga = 1.f, be = 0.f;
    if (MODE == 1) {
      const int g = ch / cpg;
      mean = mr[((long)img * groups + g) * 2];
      rstd = mr[((long)img * groups + g) * 2 + 1];
      ga = gamma ? gamma[ch] : 1.f;
      be = beta ? beta[ch] : 0.f;
    }
    for (int p = p0; p < p1; ++p) {
      const long pix = (long)img * hw + p;
      const float xv = to_f32(x[pix * ldx + ch]);
      if (MODE == 0) {
        s1 += xv;
        s2 += (double)xv * xv;
      } else {
        const float xh = (xv - mean) * rstd;
        float d = to_f32(dy[pix * ldy + ch]);
        if (silu) {
          const float u = ga * xh + be;
          const float s = 1.f / (1.f + expf(-u));
          d *= s * (1.f + u * (1.f - s));
        }
        s1 += d;
        s2 += (double)d * xh;
      }
    }
    double* o = part + (((long)img * nchunk + chunk) * c + ch) * 2;
    o[0] = s1;
    o[1] = s2;
  }
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  const double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// forward finalize per (group, image): mean, var (biased), rstd -> mr[img][g] and ab[img][c]
__global__ __launch_bounds__(256) void gnt_fwd_finalize_kernel(const double* __restrict__ part, int hw, int c,
                                                               int groups, int nchunk, float eps,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float* __restrict__ mr,
                                                               float* __restrict__ ab) {
  const int g = blockIdx.x, img = blockIdx.y, t = threadIdx.x;
  const int cpg = c / groups;
  __shared__ double red[4];
  double s1 = 0.0, s2 = 0.0;
  for (int i = t; i < nchunk * cpg; i += 256) {
    const int q = i / cpg, j = i - q * cpg;
    const double* e = part + (((long)img * nchunk + q) * c + g * cpg + j) * 2;
    s1 += e[0];
    s2 += e[1];
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  const double N = (double)hw * cpg;
  const double mean = s1 / N;
  const double var = fmax(s2 / N - mean * mean, 0.0);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float mf = (float)mean;
  if (t == 0) {
    mr[((long)img * groups + g) * 2] = mf;
    mr[((long)img * groups + g) * 2 + 1] = rstd;
  }
  for (int j = t; j < cpg; j += 256) {
    const int ch = g * cpg + j;
    const float ga = gamma ? gamma[ch] : 1.f, be = beta ? beta[ch] : 0.f;
    const float av = ga * rstd;
    ab[((long)img * c + ch) * 2] = av;
    ab[((long)img * c + ch) * 2 + 1] = be - mf * av;
  }
}

// backward finalize per (group, image): per-channel A = sum dY, B = sum dY*xhat -> nc[img][c];
// coef[img][g] = (sum_c gamma A / N, sum_c gamma B / N)
__global__ __launch_bounds__(256) void gnt_bwd_finalize_kernel(const double* __restrict__ part, int hw, int c,
                                                               int groups, int nchunk, const float* __restrict__ gamma,
                                                               double* __restrict__ nc, float* __restrict__ coef) {
  const int g = blockIdx.x, img = blockIdx.y, t = threadIdx.x;
  const int cpg = c / groups;
  __shared__ double red[4];
  double ga_s = 0.0, gb_s = 0.0;
  for (int j = t; j < cpg; j += 256) {
    const int ch = g * cpg + j;
    double a = 0.0, b = 0.0;
    for (int q = 0; q < nchunk; ++q) {
      const double* e = part + (((long)img * nchunk + q) * c + ch) * 2;
      a += e[0];
      b += e[1];
    }
    nc[((long)img * c + ch) * 2] = a;
    nc[((long)img * c + ch) * 2 + 1] = b;
    const double ga = gamma ? gamma[ch] : 1.0;
    ga_s += ga * a;
    gb_s += ga * b;
  }
  ga_s = block_sum_d(ga_s, red);
  gb_s = block_sum_d(gb_s, red);
  if (t == 0) {
    const double N = (double)hw * cpg;
    coef[((long)img * groups + g) * 2] = (float)(ga_s / N);
    coef[((long)img * groups + g) * 2 + 1] = (float)(gb_s / N);
  }
}

// dx = rstd * (gamma*dY - mean(gamma dY) - xhat * mean(gamma dY xhat))
template <typename T>
__global__ void gnt_bwd_dx_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ dy, int ldy, int n, int hw,
                                  int c, int groups, const float* __restrict__ mr, const float* __restrict__ coef,
                                  const float* __restrict__ gamma, const float* __restrict__ beta, int silu,
                                  T* __restrict__ dx, int lddx, const T* __restrict__ dres, int ldr) {
  const long total = (long)n * hw * c;
  const int cpg = c / groups;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int img = (int)(pix / hw), g = ch / cpg;
    const long gi = ((long)img * groups + g) * 2;
    const float mean = mr[gi], rstd = mr[gi + 1];
    const float ga = gamma ? gamma[ch] : 1.f, be = beta ? beta[ch] : 0.f;
    const float xh = (to_f32(x[pix * ldx + ch]) - mean) * rstd;
    float d = to_f32(dy[pix * ldy + ch]);
    if (silu) {
      const float u = ga * xh + be;
      const float s = 1.f / (1.f + expf(-u));
      d *= s * (1.f + u * (1.f - s));
    }
    const float v = rstd * (ga * d - coef[gi] - xh * coef[gi + 1]);
    // dres: a second gradient of x (a residual path), added as autograd would add the two tensors: each
    // rounded to T first, then summed in fp32 and rounded again
    dx[pix * lddx + ch] = dres ? from_f32<T>(to_f32(from_f32<T>(v)) + to_f32(dres[pix * ldr + ch])) : from_f32<T>(v);
  }
}

__global__ void gnt_param_grad_kernel(const double* __restrict__ nc, int n, int c, float* __restrict__ dgamma,
                                      float* __restrict__ dbeta, int accumulate) {
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= c) return;
  double a = 0.0, b = 0.0;
  for (int img = 0; img < n; ++img) {
    a += nc[((long)img * c + ch) * 2];
    b += nc[((long)img * c + ch) * 2 + 1];
  }
  if (dgamma) dgamma[ch] = accumulate ? dgamma[ch] + (float)b : (float)b;
  if (dbeta) dbeta[ch] = accumulate ? dbeta[ch] + (float)a : (float)a;
}

// ------------------------------------------------------------------------------------------------
// LayerNorm backward, one wave per row (c <= 2048): dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma.
// dgb_part (optional): per-wave partial (sum dy*xhat, sum dy) [waves][c][2], reduced by col sums.
template <typename T>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ x, int ldx, long rows, int c,
                                                            const float* __restrict__ gamma, float eps,
                                                            const T* __restrict__ dy, int ldy, T* __restrict__ dx,
                                                            int lddx, float* __restrict__ dgb_part,
                                                            const T* __restrict__ dres, int ldr) {
  constexpr int MAXJ = 32;
  const int lane = threadIdx.x & 63;
  const long wv = blockIdx.x * 4L + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  const int nj = (c + 63) / 64;
  float pg[MAXJ], pb[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) { pg[j] = 0.f; pb[j] = 0.f; }
  for (long r = wv; r < rows; r += nw) {
    float xv[MAXJ], gv[MAXJ];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int col = lane + 64 * j;
      xv[j] = (j < nj && col < c) ? to_f32(x[r * ldx + col]) : 0.f;
      s += xv[j];
    }
    const float mean = warp_sum(s) / c;
    float v2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int col = lane + 64 * j;
      if (j < nj && col < c) {
        const float d = xv[j] - mean;
        v2 += d * d;
      }
    }
    const float rstd = rsqrtf(warp_sum(v2) / c + eps);
    float m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int col = lane + 64 * j;
      gv[j] = 0.f;
      if (j < nj && col < c) {
        const float d = to_f32(dy[r * ldy + col]);
        const float xh = (xv[j] - mean) * rstd;
        xv[j] = xh;
        gv[j] = d * gamma[col];
        m1 += gv[j];
        m2 += gv[j] * xh;
        pg[j] += d * xh;
        pb[j] += d;
      }
    }
    m1 = warp_sum(m1) / c;
    m2 = warp_sum(m2) / c;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int col = lane + 64 * j;
      if (j < nj && col < c) {
        const float v = rstd * (gv[j] - m1 - xv[j] * m2);  // + dres as autograd's add of the two T tensors
        dx[r * lddx + col] = dres ? from_f32<T>(to_f32(from_f32<T>(v)) + to_f32(dres[r * ldr + col])) : from_f32<T>(v);
      }
    }
  }
  if (dgb_part) {
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int col = lane + 64 * j;
      if (j < nj && col < c) {
        dgb_part[(wv * c + col) * 2] = pg[j];
        dgb_part[(wv * c + col) * 2 + 1] = pb[j];
      }
    }
  }
}

// LayerNorm (dgamma, dbeta): the per-wave partials [nwaves][c][2] summed in 32-wave chunks (stage 1,
// grid over chunks x channel blocks), then over the chunks in order (stage 2)
constexpr int LN_CHUNK = 32;
__global__ void ln_param_partial_kernel(const float* __restrict__ part, long nwaves, int c2, float* __restrict__ ws) {
  const int col = blockIdx.x * 256 + threadIdx.x, chunk = blockIdx.y;
  if (col >= c2) return;
  const long w0 = (long)chunk * LN_CHUNK, w1 = min(nwaves, w0 + LN_CHUNK);
  float sacc = 0.f;
  for (long w = w0; w < w1; ++w) sacc += part[w * c2 + col];
  ws[(long)chunk * c2 + col] = sacc;
}

__global__ void ln_param_grad_kernel(const float* __restrict__ ws, int nchunk, int c, float* __restrict__ dgamma,
                                     float* __restrict__ dbeta, int accumulate) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= c) return;
  float g = 0.f, b = 0.f;
  for (int q = 0; q < nchunk; ++q) {
    g += ws[(long)q * 2 * c + 2 * col];
    b += ws[(long)q * 2 * c + 2 * col + 1];
  }
  dgamma[col] = accumulate ? dgamma[col] + g : g;
  dbeta[col] = accumulate ? dbeta[col] + b : b;
}

// softmax backward per row: ds = p * (dp - sum(p*dp)) * scale   (p: T, dp: fp32 [rows][L])
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ p, const float* __restrict__ dp,
                                                          long rows, int L, float scale, T* __restrict__ ds) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* pr = p + row * L;
  const float* dr = dp + row * L;
  float s = 0.f;
  for (int j = lane; j < L; j += 64) s += to_f32(pr[j]) * dr[j];
  s = warp_sum(s);
  T* o = ds + row * L;
  for (int j = lane; j < L; j += 64) o[j] = from_f32<T>(to_f32(pr[j]) * (dr[j] - s) * scale);
}

// GEGLU backward: x = [a | g] (value, gate), out = a * gelu(g)
template <typename T>
__global__ void geglu_bwd_kernel(const T* __restrict__ x, int ldx, long rows, int c, const T* __restrict__ dy, int ldy,
                                 T* __restrict__ dx, int lddx) {
  const long total = rows * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / c;
    const int j = (int)(i - r * c);
    const float a = to_f32(x[r * ldx + j]), g = to_f32(x[r * ldx + c + j]);
    const float d = to_f32(dy[r * ldy + j]);
    dx[r * lddx + j] = from_f32<T>(d * gelu_f(g));
    dx[r * lddx + c + j] = from_f32<T>(d * a * act_df(g, 2, 0.f));
  }
}

// ------------------------------------------------------------------------------------------------
// Checkerboard entropy model, training mode (model/compression.py:80-139, utils/ckbd.py:27-45).
// Anchor positions: (row + col) odd. Params tensors hold [scales (c) | means (c)] per pixel.
__device__ __forceinline__ bool is_anchor(int y, int x) { return ((y + x) & 1) != 0; }

__device__ __forceinline__ float std_cum(float u) { return 0.5f * erfcf(-0.70710678118654752f * u); }
__device__ __forceinline__ float std_pdf(float u) { return 0.39894228040143268f * expf(-0.5f * u * u); }

// GaussianConditional._likelihood with LowerBound(0.11) on the scale (before the 1e-9 likelihood bound)
__device__ __forceinline__ float gauss_lik(float x, float sigma, float mu) {
  const float s = fmaxf(sigma, 0.11f);
  const float v = fabsf(x - mu);
  return std_cum((0.5f - v) / s) - std_cum((-0.5f - v) / s);
}

// anchor_hat = anchor ? round(y - mu_a) + mu_a : 0
template <typename T>
__global__ void ckbd_anchor_fwd_kernel(const T* __restrict__ y, int ldy, const T* __restrict__ pa, int ldpa, int n,
                                       int h, int w, int c, T* __restrict__ out, int ldo) {
  const long total = (long)n * h * w * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int rem = (int)(pix % ((long)h * w)), yy = rem / w, xx = rem - yy * w;
    float v = 0.f;
    if (is_anchor(yy, xx)) {
      const float mu = to_f32(pa[pix * ldpa + c + ch]);
      v = rintf(to_f32(y[pix * ldy + ch]) - mu) + mu;
    }
    out[pix * ldo + ch] = from_f32<T>(v);
  }
}

// out = x at anchor (which = 1) or non-anchor (which = 0) positions, 0 elsewhere (ckbd_anchor /
// ckbd_nonanchor, utils/ckbd.py:33-45): the straight-through gradient of a masked slice
template <typename T>
__global__ void ckbd_mask_kernel(const T* __restrict__ x, int ldx, int n, int h, int w, int c, int which,
                                 T* __restrict__ out, int ldo) {
  const long total = (long)n * h * w * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int rem = (int)(pix % ((long)h * w)), yy = rem / w, xx = rem - yy * w;
    out[pix * ldo + ch] = is_anchor(yy, xx) == (which != 0) ? x[pix * ldx + ch] : from_f32<T>(0.f);
  }
}

// likelihoods of the whole slice (noise mode, and dequantize mode for q_bpp) summed as ln(lik) per
// block; nonanchor_hat = nonanchor ? round(y - mu_n) + mu_n : 0
template <typename T>
__global__ __launch_bounds__(256) void ckbd_lik_fwd_kernel(const T* __restrict__ y, int ldy, const T* __restrict__ pa,
                                                           int ldpa, const T* __restrict__ pn, int ldpn,
                                                           const float* __restrict__ noise, int n, int h, int w, int c,
                                                           T* __restrict__ nonanchor_hat, int ldo,
                                                           double* __restrict__ part) {
  const long total = (long)n * h * w * c;
  double s_lik = 0.0, s_q = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int rem = (int)(pix % ((long)h * w)), yy = rem / w, xx = rem - yy * w;
    const bool an = is_anchor(yy, xx);
    const T* pp = an ? pa + pix * ldpa : pn + pix * ldpn;
    const float sigma = to_f32(pp[ch]), mu = to_f32(pp[c + ch]);
    const float yv = to_f32(y[pix * ldy + ch]);
    const float lik = fmaxf(gauss_lik(yv + noise[i], sigma, mu), 1e-9f);
    const float qv = rintf(yv - mu) + mu;
    const float ql = fmaxf(gauss_lik(qv, sigma, mu), 1e-9f);
    s_lik += (double)logf(lik);
    s_q += (double)logf(ql);
    nonanchor_hat[pix * ldo + ch] = from_f32<T>(an ? 0.f : qv);
  }
  __shared__ double red[4];
  s_lik = block_sum_d(s_lik, red);
  s_q = block_sum_d(s_q, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2] = s_lik;
    part[blockIdx.x * 2 + 1] = s_q;
  }
}

__global__ void sum_pairs_kernel(const double* __restrict__ part, int nblk, float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double a = 0.0, b = 0.0;
  for (int i = 0; i < nblk; ++i) { a += part[2 * i]; b += part[2 * i + 1]; }
  out[0] = (float)a;
  out[1] = (float)b;
}

// backward of S = sum ln(lik) (g = dL/dS, a device scalar) and of nonanchor_hat (STE):
//   dy = mask_n * d_nonanchor + g/lik * dlik/dx;  dpa / dpn = (dscale, dmean) at their own positions
template <typename T>
__global__ void ckbd_lik_bwd_kernel(const T* __restrict__ y, int ldy, const T* __restrict__ pa, int ldpa,
                                    const T* __restrict__ pn, int ldpn, const float* __restrict__ noise, int n, int h,
                                    int w, int c, const float* __restrict__ gS, const T* __restrict__ dnon, int ldd,
                                    T* __restrict__ dy, int lddy, T* __restrict__ dpa, int lddpa, T* __restrict__ dpn,
                                    int lddpn) {
  const long total = (long)n * h * w * c;
  const float G = gS[0];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / c;
    const int ch = (int)(i - pix * c);
    const int rem = (int)(pix % ((long)h * w)), yy = rem / w, xx = rem - yy * w;
    const bool an = is_anchor(yy, xx);
    const T* pp = an ? pa + pix * ldpa : pn + pix * ldpn;
    const float sigma = to_f32(pp[ch]), mu = to_f32(pp[c + ch]);
    const float xn = to_f32(y[pix * ldy + ch]) + noise[i];
    const float s = fmaxf(sigma, 0.11f);
    const float diff = xn - mu;
    const float v = fabsf(diff);
    const float u1 = (0.5f - v) / s, u2 = (-0.5f - v) / s;
    const float lik_raw = std_cum(u1) - std_cum(u2);
    const float lik = fmaxf(lik_raw, 1e-9f);
    float g = G / lik;                                         // d ln(lik_b) / d lik_b
    if (!(lik_raw >= 1e-9f || g < 0.f)) g = 0.f;               // LowerBound(1e-9) backward
    const float p1 = std_pdf(u1), p2 = std_pdf(u2);
    const float dv = g * (p2 - p1) / s;                        // d lik / d v
    float dsig = g * (u2 * p2 - u1 * p1) / s;                  // d lik / d s
    if (!(sigma >= 0.11f || dsig < 0.f)) dsig = 0.f;           // LowerBound(0.11) backward
    const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
    float dyv = dv * sg;
    if (!an && dnon) dyv += to_f32(dnon[pix * ldd + ch]);
    dy[pix * lddy + ch] = from_f32<T>(dyv);
    T* da = dpa + pix * lddpa;
    T* dn = dpn + pix * lddpn;
    da[ch] = from_f32<T>(an ? dsig : 0.f);
    da[c + ch] = from_f32<T>(an ? -dv * sg : 0.f);
    dn[ch] = from_f32<T>(an ? 0.f : dsig);
    dn[c + ch] = from_f32<T>(an ? 0.f : -dv * sg);
  }
}

// ------------------------------------------------------------------------------------------------
// VQ codebook step (VectorQuantiser.forward, training, anchor 'closest', contrastive loss), one block
// per code e. d[p][e] = (-|z_p|^2 - |E_e|^2) + 2 z_p.E_e. The column is sorted ascending (bitonic,
// LDS); pos = mean of the top max(1, P/K) distances, neg = the P/2 smallest; CE(target 0) over
// [pos, neg] / 0.07. Writes: per-code (CE_e, sum_{idx_p = e} |E_e - z_p|^2), the re-initialised
// codebook row and embed_prob (in place), and dE_unit[e] = d(emb_loss)/dE_e with the upstream
// gradient 1 (the -|E|^2 term uses the re-initialised row, as the reference's in-place .data
// update makes autograd do).
constexpr int VQ_PMAX = 4096;
__global__ __launch_bounds__(256) void vq_code_kernel(const float* __restrict__ dot, const float* __restrict__ zn,
                                                      const float* __restrict__ en, const float* __restrict__ z,
                                                      const int* __restrict__ idx, int P, int K, int D,
                                                      float* __restrict__ E, float* __restrict__ embed_prob,
                                                      float beta, float decay, float temp,
                                                      float* __restrict__ code_out, float* __restrict__ dE_unit) {
  const int e = blockIdx.x, t = threadIdx.x;
  __shared__ float sv[VQ_PMAX];
  __shared__ int si[VQ_PMAX];
  __shared__ float gcol[VQ_PMAX];
  __shared__ float Eold[512];
  __shared__ float red[4];
  __shared__ float cred[4];
  int NP = 1;
  while (NP < P) NP <<= 1;
  const float ene = en[e];
  for (int p = t; p < NP; p += 256) {
    if (p < P) {
      sv[p] = (-zn[p] - ene) + 2.f * dot[(long)p * K + e];
      si[p] = p;
    } else {
      sv[p] = INFINITY;
      si[p] = 0x7fffffff;
    }
    gcol[p] = 0.f;
  }
  for (int d = t; d < D; d += 256) Eold[d] = E[(long)e * D + d];
  __syncthreads();
  // bitonic sort ascending by (value, index)
  for (int k = 2; k <= NP; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < NP; i += 256) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const float a = sv[i], b = sv[l];
          const int ia = si[i], ib = si[l];
          const bool gt = (a > b) || (a == b && ia > ib);
          if (gt == up) {
            sv[i] = b; sv[l] = a;
            si[i] = ib; si[l] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  const int npos = max(1, P / K), nneg = P / 2;
  // cross entropy over [pos, neg_0 .. neg_{nneg-1}] / temp, target 0 (thread 0: nneg <= 2048 terms)
  if (t == 0) {
    float pos = 0.f;
    for (int q = P - npos; q < P; ++q) pos += sv[q];
    pos = pos / (float)npos;
    const float l0 = pos / temp;
    float mx = l0;
    for (int q = 0; q < nneg; ++q) mx = fmaxf(mx, sv[q] / temp);
    float se = expf(l0 - mx);
    for (int q = 0; q < nneg; ++q) se += expf(sv[q] / temp - mx);
    const float lse = mx + logf(se);
    code_out[(long)e * 2] = lse - l0;
    // d CE_e / d logit_j = softmax_j - [j == 0]; mean over the K codes; logits = dis / temp
    const float sc = 1.f / ((float)K * temp);
    const float g0 = (expf(l0 - lse) - 1.f) * sc / (float)npos;
    for (int q = P - npos; q < P; ++q) gcol[si[q]] += g0;
    for (int q = 0; q < nneg; ++q) gcol[si[q]] += expf(sv[q] / temp - lse) * sc;
  }
  int cnt = 0;
  for (int p = t; p < P; p += 256) cnt += idx[p] == e;
  const float cw = warp_sum((float)cnt);  // exact: integer counts << 2^24
  if ((t & 63) == 0) cred[t >> 6] = cw;
  __syncthreads();
  // embed_prob EMA, decay, re-initialisation from the closest point (sorted last)
  const float avg = ((cred[0] + cred[1]) + (cred[2] + cred[3])) / (float)P;
  const float ep = embed_prob[e] * decay + avg * (1.f - decay);
  const float dcy = expf(-(ep * (float)K * 10.f) / (1.f - decay) - 1e-3f);
  const int pclose = si[P - 1];
  float gsum = 0.f;
  for (int p = 0; p < P; ++p) gsum += gcol[p];  // every thread, same order
  const float numel = (float)P * (float)D;
  float sq = 0.f;
  for (int d = t; d < D; d += 256) {
    const float eo = Eold[d];
    const float en_ = eo * (1.f - dcy) + z[(long)pclose * D + d] * dcy;
    float gd = -2.f * en_ * gsum;
    for (int p = 0; p < P; ++p) {
      const float gp = gcol[p];
      if (gp != 0.f) gd += gp * 2.f * z[(long)p * D + d];
      if (idx[p] == e) {
        const float df = eo - z[(long)p * D + d];
        gd += 2.f * df / numel;
        sq += df * df;
      }
    }
    dE_unit[(long)e * D + d] = gd;
    E[(long)e * D + d] = en_;
  }
  sq = warp_sum(sq);
  if ((t & 63) == 0) red[t >> 6] = sq;
  __syncthreads();
  if (t == 0) {
    code_out[(long)e * 2 + 1] = (red[0] + red[1]) + (red[2] + red[3]);
    embed_prob[e] = ep;
  }
}

// emb_loss = beta*mse + mse + mean_e CE_e, mse = sum_e sq_e / numel (one thread, fixed order)
__global__ __launch_bounds__(256) void vq_loss_kernel(const float* __restrict__ code_out, int K, float numel,
                                                      float beta, float* __restrict__ out) {
  __shared__ double red[4];
  double ce = 0.0, sq = 0.0;
  for (int e = threadIdx.x; e < K; e += 256) { ce += code_out[2 * e]; sq += code_out[2 * e + 1]; }
  ce = block_sum_d(ce, red);
  sq = block_sum_d(sq, red);
  if (threadIdx.x != 0) return;
  const float mse = (float)(sq / numel);
  out[0] = (beta * mse + mse) + (float)(ce / K);
  out[1] = mse;
  out[2] = (float)(ce / K);
}

// dz = dzq (straight-through) + g * beta * 2 (z - zq) / numel
template <typename T>
__global__ void vq_z_grad_kernel(const float* __restrict__ z, const float* __restrict__ zq, const T* __restrict__ dzq,
                                 long count, const float* __restrict__ gL, float coef, T* __restrict__ dz) {
  const float g = gL[0] * coef;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < count; i += (long)gridDim.x * 256)
    dz[i] = from_f32<T>((dzq ? to_f32(dzq[i]) : 0.f) + g * (z[i] - zq[i]));
}

// y (+)= s[0] * x
__global__ void scale_dev_kernel(const float* __restrict__ x, long count, const float* __restrict__ s,
                                 float* __restrict__ y, int accumulate) {
  const float a = s[0];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < count; i += (long)gridDim.x * 256)
    y[i] = accumulate ? y[i] + a * x[i] : a * x[i];
}

// torch.optim.AdamW single-tensor update, in its op order (torch/optim/adamw.py)
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long count, float c_wd, float one_m_b1, float b2, float one_m_b2,
                             float bc2_sqrt, float neg_step, float eps) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < count; i += (long)gridDim.x * 256) {
    const float gi = g[i];
    const float pi = p[i] * c_wd;
    const float mi = m[i] + one_m_b1 * (gi - m[i]);
    const float vi = v[i] * b2 + one_m_b2 * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi + neg_step * mi / denom;
  }
}

// as adamw_kernel, with the step-dependent scalars (-lr / bias_correction1, sqrt(bias_correction2))
// read from device memory: a captured hipGraph replays the same launch every step
__global__ void adamw_dev_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                 float* __restrict__ v, long count, float c_wd, float one_m_b1, float b2,
                                 float one_m_b2, const float* __restrict__ sc, float eps) {
  const float neg_step = sc[0], bc2_sqrt = sc[1];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < count; i += (long)gridDim.x * 256) {
    const float gi = g[i];
    const float pi = p[i] * c_wd;
    const float mi = m[i] + one_m_b1 * (gi - m[i]);
    const float vi = v[i] * b2 + one_m_b2 * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi + neg_step * mi / denom;
  }
}

}  // namespace

// ================================================================================================
extern "C" int rdeic_gemm_strided(const rdeic_gemm_desc* d, void* stream) {
  if (!d || !d->a || !d->b || !d->c || d->m <= 0 || d->n <= 0 || d->k <= 0 || d->batch <= 0 || d->nb2 <= 0 ||
      d->batch % d->nb2 || d->ksplit < 0)
    return RDEIC_EINVAL;
  if (d->ksplit > 0 && (long)(d->batch / d->nb2) * d->ksplit < d->k) return RDEIC_EINVAL;
  GemmArgs g;
  g.a = d->a; g.a_bs1 = d->a_bs1; g.a_bs2 = d->a_bs2; g.a_sm = d->a_sm; g.a_sk = d->a_sk;
  g.b = d->b; g.b_bs1 = d->b_bs1; g.b_bs2 = d->b_bs2; g.b_sk = d->b_sk; g.b_sn = d->b_sn;
  g.c = d->c; g.c_bs1 = d->c_bs1; g.c_bs2 = d->c_bs2; g.c_sm = d->c_sm;
  g.nb2 = d->nb2; g.m = d->m; g.n = d->n; g.k = d->k; g.ksplit = d->ksplit; g.c_f32 = d->c_f32;
  g.alpha = d->alpha; g.beta = d->beta;
  g.rsum = d->rsum; g.rsum_bs = d->rsum_bs;
  if (d->batch > 65535 || (d->rsum && d->nb2 != 1)) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const double flops = 2.0 * d->m * d->n * (d->ksplit > 0 ? (double)d->k : (double)d->k * (d->batch / d->nb2)) * d->nb2;
  ProfScope ps(s, RDEIC_PROF_GEMM, flops);
  // 128x128 tiles where their grid still has ~a workgroup per CU, else 64x64
  const long t128 = (long)((d->n + 127) / 128) * ((d->m + 127) / 128) * d->batch;
  if (d->m >= 128 && d->n >= 128 && t128 >= 200) {
    dim3 grid((d->n + 127) / 128, (d->m + 127) / 128, d->batch);
    if (d->dtype == 1) launch_gemm<bf16, 128>(g, grid, s);
    else launch_gemm<float, 128>(g, grid, s);
  } else {
    dim3 grid((d->n + 63) / 64, (d->m + 63) / 64, d->batch);
    if (d->dtype == 1) launch_gemm<bf16, 64>(g, grid, s);
    else launch_gemm<float, 64>(g, grid, s);
  }
  return launch_status();
}

extern "C" int rdeic_pack_conv_weight_dgrad(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                                            void* out, int32_t wld, int32_t to_bf16, void* stream) {
  if (!w || !out || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || wld < kh * kw * cout || wld % 64) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d((long)cin * wld);
  if (to_bf16)
    hipLaunchKernelGGL(pack_dgrad_kernel<bf16>, dim3(g), dim3(256), 0, s, w, cout, cin, kh, kw, (bf16*)out, wld);
  else
    hipLaunchKernelGGL(pack_dgrad_kernel<float>, dim3(g), dim3(256), 0, s, w, cout, cin, kh, kw, (float*)out, wld);
  return launch_status();
}

extern "C" int rdeic_pack_batch(const rdeic_pack_job* jobs, int32_t njobs, int64_t total, int32_t row_floats,
                                int32_t to_bf16, void* stream) {
  if (!jobs || njobs <= 0 || total <= 0 || total > 0x7fffffffL || row_floats <= 0 || row_floats > PACK_ROW_MAX)
    return RDEIC_EINVAL;
  const size_t lds = (size_t)row_floats * sizeof(float);
  if (to_bf16)
    hipLaunchKernelGGL(pack_batch_kernel<bf16>, dim3((unsigned)total), dim3(256), lds, (hipStream_t)stream, jobs, njobs);
  else
    hipLaunchKernelGGL(pack_batch_kernel<float>, dim3((unsigned)total), dim3(256), lds, (hipStream_t)stream, jobs, njobs);
  return launch_status();
}

extern "C" int rdeic_im2col(const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ld, int32_t kh,
                            int32_t kw, int32_t stride, int32_t pad_t, int32_t pad_l, int32_t ho, int32_t wo,
                            int32_t up2, void* out, int64_t out_ld, int32_t dtype, void* stream) {
  if (!x || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || ld < c || ho <= 0 || wo <= 0 || out_ld < (int64_t)kh * kw * c)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d((long)n * ho * wo * kh * kw * c);
  if (dtype == 1)
    hipLaunchKernelGGL(im2col_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)x, n, h, w, c, ld, kh, kw, stride,
                       pad_t, pad_l, ho, wo, up2, (bf16*)out, (long)out_ld);
  else
    hipLaunchKernelGGL(im2col_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, n, h, w, c, ld, kh, kw, stride,
                       pad_t, pad_l, ho, wo, up2, (float*)out, (long)out_ld);
  return launch_status();
}

#define RDEIC_LAYOUT_OP(NAME, KERNEL, OUTPIX)                                                                      \
  extern "C" int NAME(const void* src, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ld, void* dst,        \
                      int32_t dst_ld, int32_t dtype, void* stream) {                                              \
    if (!src || !dst || n <= 0 || h <= 0 || w <= 0 || c <= 0 || ld < c) return RDEIC_EINVAL;                      \
    hipStream_t s = (hipStream_t)stream;                                                                          \
    const int g = grid_1d((long)n * h * w * c * (OUTPIX));                                                        \
    if (dtype == 1)                                                                                                \
      hipLaunchKernelGGL(KERNEL<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)src, n, h, w, c, ld, (bf16*)dst,   \
                         dst_ld);                                                                                  \
    else                                                                                                           \
      hipLaunchKernelGGL(KERNEL<float>, dim3(g), dim3(256), 0, s, (const float*)src, n, h, w, c, ld, (float*)dst, \
                         dst_ld);                                                                                  \
    return launch_status();                                                                                        \
  }
// h, w: the SMALL grid in all three (zero_insert2: src size; sum_pool2 / pixel_unshuffle2: dst size)
RDEIC_LAYOUT_OP(rdeic_zero_insert2, zero_insert2_kernel, 4)
RDEIC_LAYOUT_OP(rdeic_sum_pool2, sum_pool2_kernel, 1)
RDEIC_LAYOUT_OP(rdeic_pixel_unshuffle2, pixel_unshuffle2_kernel, 4)
#undef RDEIC_LAYOUT_OP

extern "C" int rdeic_wgrad_finalize(const float* part, int32_t splits, int32_t cout, int32_t cin, int32_t kh,
                                    int32_t kw, float* dw, int32_t accumulate, const float* rpart, float* db,
                                    void* stream) {
  if (!part || !dw || splits <= 0 || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || (db && !rpart))
    return RDEIC_EINVAL;
  hipLaunchKernelGGL(wgrad_finalize_kernel, dim3(grid_1d((long)cout * kh * kw * cin)), dim3(256), 0,
                     (hipStream_t)stream, part, splits, cout, cin, kh, kw, dw, accumulate, rpart, db);
  return launch_status();
}

extern "C" size_t rdeic_col_sum_ws_floats(int64_t rows, int32_t c, int32_t groups) {
  if (rows <= 0 || c <= 0 || groups <= 0 || rows % groups) return 0;
  const long rpg = rows / groups;
  const long rpc = cs_rows(rpg);
  return (size_t)groups * ((rpg + rpc - 1) / rpc) * c;
}

extern "C" int rdeic_col_sum(const void* x, int64_t rows, int32_t c, int32_t ld, int32_t groups, float* out,
                             int32_t accumulate, float* ws, size_t ws_floats, int32_t dtype, void* stream) {
  if (!x || !out || !ws || rows <= 0 || c <= 0 || ld < c || groups <= 0 || rows % groups) return RDEIC_EINVAL;
  if (ws_floats < rdeic_col_sum_ws_floats(rows, c, groups)) return RDEIC_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  const long rpg = rows / groups;
  const long rpc = cs_rows(rpg);
  const int nchunk = (int)((rpg + rpc - 1) / rpc);
  if (nchunk > 65535 || groups > 65535) return RDEIC_EINVAL;
  dim3 grid((c + 255) / 256, nchunk, groups);
  if (dtype == 1)
    hipLaunchKernelGGL(col_sum_partial_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, rpg, c, ld, nchunk, rpc, ws);
  else
    hipLaunchKernelGGL(col_sum_partial_kernel<float>, grid, dim3(256), 0, s, (const float*)x, rpg, c, ld, nchunk, rpc, ws);
  hipLaunchKernelGGL(col_sum_final_kernel, dim3(grid_1d((long)groups * c)), dim3(256), 0, s, ws, groups, nchunk, c, out,
                     accumulate);
  return launch_status();
}

extern "C" int rdeic_act_fwd(const void* z, int64_t rows, int32_t c, int32_t ldz, const void* res, int32_t ldr,
                             int32_t act, float slope, void* out, int32_t ldo, int32_t dtype, void* stream) {
  if (!z || !out || rows <= 0 || c <= 0 || act < 0 || act > 3) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d(rows * c);
  if (dtype == 1)
    hipLaunchKernelGGL(act_fwd_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)z, (long)rows, c, ldz,
                       (const bf16*)res, ldr, act, slope, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(act_fwd_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)z, (long)rows, c, ldz,
                       (const float*)res, ldr, act, slope, (float*)out, ldo);
  return launch_status();
}

extern "C" int rdeic_act_bwd(const void* dy, int32_t ldy, const void* z, int32_t ldz, int64_t rows, int32_t c,
                             int32_t act, float slope, void* dz, int32_t lddz, int32_t dtype, void* stream) {
  if (!dy || !z || !dz || rows <= 0 || c <= 0 || act < 0 || act > 3) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d(rows * c);
  if (dtype == 1)
    hipLaunchKernelGGL(act_bwd_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)dy, ldy, (const bf16*)z, ldz,
                       (long)rows, c, act, slope, (bf16*)dz, lddz);
  else
    hipLaunchKernelGGL(act_bwd_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)dy, ldy, (const float*)z, ldz,
                       (long)rows, c, act, slope, (float*)dz, lddz);
  return launch_status();
}

extern "C" size_t rdeic_gn_train_ws_doubles(int32_t n, int32_t hw, int32_t c) {
  if (n <= 0 || hw <= 0 || c <= 0) return 0;
  const long nchunk = (hw + GNT_CHUNK - 1) / GNT_CHUNK;
  return (size_t)n * nchunk * c * 2 + (size_t)n * c * 2;
}

extern "C" int rdeic_gn_train_fwd(const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t c, int32_t groups,
                                  float eps, const float* gamma, const float* beta, float* mr, float* ab, double* ws,
                                  int32_t dtype, void* stream) {
  if (!x || !mr || !ab || !ws || n <= 0 || hw <= 0 || c <= 0 || groups <= 0 || c % groups) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int nchunk = (hw + GNT_CHUNK - 1) / GNT_CHUNK;
  if (dtype == 1)
    hipLaunchKernelGGL((gnt_partial_kernel<bf16, 0>), dim3(nchunk, n, (c + 255) / 256), dim3(256), 0, s, (const bf16*)x, ldx,
                       (const bf16*)nullptr, 0, hw, c, groups, nchunk, nullptr, nullptr, nullptr, 0, ws);
  else
    hipLaunchKernelGGL((gnt_partial_kernel<float, 0>), dim3(nchunk, n, (c + 255) / 256), dim3(256), 0, s, (const float*)x, ldx,
                       (const float*)nullptr, 0, hw, c, groups, nchunk, nullptr, nullptr, nullptr, 0, ws);
  hipLaunchKernelGGL(gnt_fwd_finalize_kernel, dim3(groups, n), dim3(256), 0, s, ws, hw, c, groups, nchunk, eps, gamma,
                     beta, mr, ab);
  return launch_status();
}

extern "C" int rdeic_gn_train_bwd(const void* x, int32_t ldx, const void* dy, int32_t ldy, int32_t n, int32_t hw,
                                  int32_t c, int32_t groups, const float* mr, const float* gamma, const float* beta,
                                  int32_t silu, void* dx, int32_t lddx, float* dgamma, float* dbeta,
                                  int32_t accumulate, double* ws, float* coef, int32_t dtype, void* stream) {
  return rdeic_gn_train_bwd_res(x, ldx, dy, ldy, n, hw, c, groups, mr, gamma, beta, silu, nullptr, 0, dx, lddx, dgamma,
                                dbeta, accumulate, ws, coef, dtype, stream);
}

extern "C" int rdeic_gn_train_bwd_res(const void* x, int32_t ldx, const void* dy, int32_t ldy, int32_t n, int32_t hw,
                                      int32_t c, int32_t groups, const float* mr, const float* gamma, const float* beta,
                                      int32_t silu, const void* dres, int32_t ldr, void* dx, int32_t lddx,
                                      float* dgamma, float* dbeta, int32_t accumulate, double* ws, float* coef,
                                      int32_t dtype, void* stream) {
  if (!x || !dy || !dx || !mr || !ws || !coef || n <= 0 || hw <= 0 || c <= 0 || groups <= 0 || c % groups)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int nchunk = (hw + GNT_CHUNK - 1) / GNT_CHUNK;
  double* part = ws;
  double* nc = ws + (size_t)n * nchunk * c * 2;
  if (dtype == 1)
    hipLaunchKernelGGL((gnt_partial_kernel<bf16, 1>), dim3(nchunk, n, (c + 255) / 256), dim3(256), 0, s, (const bf16*)x, ldx,
                       (const bf16*)dy, ldy, hw, c, groups, nchunk, mr, gamma, beta, silu, part);
  else
    hipLaunchKernelGGL((gnt_partial_kernel<float, 1>), dim3(nchunk, n, (c + 255) / 256), dim3(256), 0, s, (const float*)x, ldx,
                       (const float*)dy, ldy, hw, c, groups, nchunk, mr, gamma, beta, silu, part);
  hipLaunchKernelGGL(gnt_bwd_finalize_kernel, dim3(groups, n), dim3(256), 0, s, part, hw, c, groups, nchunk, gamma, nc,
                     coef);
  const int g = grid_1d((long)n * hw * c);
  if (dtype == 1)
    hipLaunchKernelGGL(gnt_bwd_dx_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)x, ldx, (const bf16*)dy, ldy,
                       n, hw, c, groups, mr, coef, gamma, beta, silu, (bf16*)dx, lddx, (const bf16*)dres, ldr);
  else
    hipLaunchKernelGGL(gnt_bwd_dx_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, ldx, (const float*)dy,
                       ldy, n, hw, c, groups, mr, coef, gamma, beta, silu, (float*)dx, lddx, (const float*)dres, ldr);
  if (dgamma || dbeta)
    hipLaunchKernelGGL(gnt_param_grad_kernel, dim3((c + 255) / 256), dim3(256), 0, s, nc, n, c, dgamma, dbeta,
                       accumulate);
  return launch_status();
}

static long ln_bwd_blocks(long rows) { return std::min<long>((rows + 3) / 4, 256); }

extern "C" size_t rdeic_layernorm_bwd_ws_floats(int64_t rows, int32_t c) {
  if (rows <= 0 || c <= 0) return 0;
  const long nw = ln_bwd_blocks(rows) * 4;
  return (size_t)nw * c * 2 + (size_t)((nw + LN_CHUNK - 1) / LN_CHUNK) * c * 2;
}

extern "C" int rdeic_layernorm_bwd(const void* x, int32_t ldx, int64_t rows, int32_t c, const float* gamma, float eps,
                                   const void* dy, int32_t ldy, void* dx, int32_t lddx, float* dgamma, float* dbeta,
                                   int32_t accumulate, float* ws, size_t ws_floats, int32_t dtype, void* stream) {
  return rdeic_layernorm_bwd_res(x, ldx, rows, c, gamma, eps, dy, ldy, nullptr, 0, dx, lddx, dgamma, dbeta, accumulate,
                                 ws, ws_floats, dtype, stream);
}

extern "C" int rdeic_layernorm_bwd_res(const void* x, int32_t ldx, int64_t rows, int32_t c, const float* gamma,
                                       float eps, const void* dy, int32_t ldy, const void* dres, int32_t ldr, void* dx,
                                       int32_t lddx, float* dgamma, float* dbeta, int32_t accumulate, float* ws,
                                       size_t ws_floats, int32_t dtype, void* stream) {
  if (!x || !dy || !dx || !gamma || rows <= 0 || c <= 0 || c > 2048) return RDEIC_EINVAL;
  const bool pg = dgamma && dbeta;
  if (pg && (!ws || ws_floats < rdeic_layernorm_bwd_ws_floats(rows, c))) return RDEIC_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (int)ln_bwd_blocks(rows);
  if (dtype == 1)
    hipLaunchKernelGGL(layernorm_bwd_kernel<bf16>, dim3(blocks), dim3(256), 0, s, (const bf16*)x, ldx, (long)rows, c,
                       gamma, eps, (const bf16*)dy, ldy, (bf16*)dx, lddx, pg ? ws : nullptr, (const bf16*)dres, ldr);
  else
    hipLaunchKernelGGL(layernorm_bwd_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, ldx, (long)rows, c,
                       gamma, eps, (const float*)dy, ldy, (float*)dx, lddx, pg ? ws : nullptr, (const float*)dres, ldr);
  if (pg) {
    const long nw = (long)blocks * 4;
    const int nchunk = (int)((nw + LN_CHUNK - 1) / LN_CHUNK);
    float* ws2 = ws + nw * c * 2;
    hipLaunchKernelGGL(ln_param_partial_kernel, dim3((2 * c + 255) / 256, nchunk), dim3(256), 0, s, ws, nw, 2 * c, ws2);
    hipLaunchKernelGGL(ln_param_grad_kernel, dim3((c + 255) / 256), dim3(256), 0, s, ws2, nchunk, c, dgamma, dbeta,
                       accumulate);
  }
  return launch_status();
}

extern "C" int rdeic_softmax_bwd_rows(const void* p, const float* dp, int64_t rows, int32_t cols, float scale, void* ds,
                                      int32_t dtype, void* stream) {
  if (!p || !dp || !ds || rows <= 0 || cols <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_bwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)p, dp, (long)rows, cols, scale,
                       (bf16*)ds);
  else
    hipLaunchKernelGGL(softmax_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)p, dp, (long)rows, cols, scale,
                       (float*)ds);
  return launch_status();
}

extern "C" int rdeic_geglu_bwd(const void* x, int32_t ldx, int64_t rows, int32_t c, const void* dy, int32_t ldy,
                               void* dx, int32_t lddx, int32_t dtype, void* stream) {
  if (!x || !dy || !dx || rows <= 0 || c <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d(rows * c);
  if (dtype == 1)
    hipLaunchKernelGGL(geglu_bwd_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)x, ldx, (long)rows, c,
                       (const bf16*)dy, ldy, (bf16*)dx, lddx);
  else
    hipLaunchKernelGGL(geglu_bwd_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, ldx, (long)rows, c,
                       (const float*)dy, ldy, (float*)dx, lddx);
  return launch_status();
}

extern "C" int rdeic_ckbd_train_anchor(const void* y, int32_t ldy, const void* pa, int32_t ldpa, int32_t n, int32_t h,
                                       int32_t w, int32_t c, void* out, int32_t ldo, int32_t dtype, void* stream) {
  if (!y || !pa || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0 || ldpa < 2 * c) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d((long)n * h * w * c);
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_anchor_fwd_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)y, ldy, (const bf16*)pa,
                       ldpa, n, h, w, c, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(ckbd_anchor_fwd_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)y, ldy,
                       (const float*)pa, ldpa, n, h, w, c, (float*)out, ldo);
  return launch_status();
}

extern "C" int rdeic_ckbd_mask(const void* x, int32_t ldx, int32_t n, int32_t h, int32_t w, int32_t c, int32_t which,
                               void* out, int32_t ldo, int32_t dtype, void* stream) {
  if (!x || !out || n <= 0 || h <= 0 || w <= 0 || c <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d((long)n * h * w * c);
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_mask_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)x, ldx, n, h, w, c, which,
                       (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(ckbd_mask_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, ldx, n, h, w, c, which,
                       (float*)out, ldo);
  return launch_status();
}

extern "C" size_t rdeic_ckbd_train_ws_doubles(int32_t n, int32_t h, int32_t w, int32_t c) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0) return 0;
  return (size_t)grid_1d((long)n * h * w * c) * 2;
}

extern "C" int rdeic_ckbd_train_lik(const void* y, int32_t ldy, const void* pa, int32_t ldpa, const void* pn,
                                    int32_t ldpn, const float* noise, int32_t n, int32_t h, int32_t w, int32_t c,
                                    void* nonanchor_hat, int32_t ldo, double* ws, float* out2, int32_t dtype,
                                    void* stream) {
  if (!y || !pa || !pn || !noise || !nonanchor_hat || !ws || !out2 || n <= 0 || h <= 0 || w <= 0 || c <= 0 ||
      ldpa < 2 * c || ldpn < 2 * c)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d((long)n * h * w * c);
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_lik_fwd_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)y, ldy, (const bf16*)pa, ldpa,
                       (const bf16*)pn, ldpn, noise, n, h, w, c, (bf16*)nonanchor_hat, ldo, ws);
  else
    hipLaunchKernelGGL(ckbd_lik_fwd_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)y, ldy, (const float*)pa,
                       ldpa, (const float*)pn, ldpn, noise, n, h, w, c, (float*)nonanchor_hat, ldo, ws);
  hipLaunchKernelGGL(sum_pairs_kernel, dim3(1), dim3(64), 0, s, ws, g, out2);
  return launch_status();
}

extern "C" int rdeic_ckbd_train_lik_bwd(const void* y, int32_t ldy, const void* pa, int32_t ldpa, const void* pn,
                                        int32_t ldpn, const float* noise, int32_t n, int32_t h, int32_t w, int32_t c,
                                        const float* g_sum, const void* d_nonanchor, int32_t ldd, void* dy,
                                        int32_t lddy, void* dpa, int32_t lddpa, void* dpn, int32_t lddpn,
                                        int32_t dtype, void* stream) {
  if (!y || !pa || !pn || !noise || !g_sum || !dy || !dpa || !dpn || n <= 0 || h <= 0 || w <= 0 || c <= 0)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d((long)n * h * w * c);
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_lik_bwd_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)y, ldy, (const bf16*)pa, ldpa,
                       (const bf16*)pn, ldpn, noise, n, h, w, c, g_sum, (const bf16*)d_nonanchor, ldd, (bf16*)dy,
                       lddy, (bf16*)dpa, lddpa, (bf16*)dpn, lddpn);
  else
    hipLaunchKernelGGL(ckbd_lik_bwd_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)y, ldy, (const float*)pa,
                       ldpa, (const float*)pn, ldpn, noise, n, h, w, c, g_sum, (const float*)d_nonanchor, ldd,
                       (float*)dy, lddy, (float*)dpa, lddpa, (float*)dpn, lddpn);
  return launch_status();
}

extern "C" int rdeic_vq_train(const float* dot, const float* zn, const float* en, const float* z, const int32_t* idx,
                              int32_t P, int32_t K, int32_t D, float* E, float* embed_prob, float beta, float decay,
                              float temp, float* code_out, float* dE_unit, float* loss3, void* stream) {
  if (!dot || !zn || !en || !z || !idx || !E || !embed_prob || !code_out || !dE_unit || !loss3 || P <= 0 ||
      P > VQ_PMAX || K <= 0 || D <= 0 || D > 512)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(vq_code_kernel, dim3(K), dim3(256), 0, s, dot, zn, en, z, idx, P, K, D, E, embed_prob, beta, decay,
                     temp, code_out, dE_unit);
  hipLaunchKernelGGL(vq_loss_kernel, dim3(1), dim3(256), 0, s, code_out, K, (float)P * (float)D, beta, loss3);
  return launch_status();
}

extern "C" int rdeic_vq_z_grad(const float* z, const float* zq, const void* dzq, int64_t count, const float* g_loss,
                               float coef, void* dz, int32_t dtype, void* stream) {
  if (!z || !zq || !g_loss || !dz || count <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_1d(count);
  if (dtype == 1)
    hipLaunchKernelGGL(vq_z_grad_kernel<bf16>, dim3(g), dim3(256), 0, s, z, zq, (const bf16*)dzq, (long)count, g_loss,
                       coef, (bf16*)dz);
  else
    hipLaunchKernelGGL(vq_z_grad_kernel<float>, dim3(g), dim3(256), 0, s, z, zq, (const float*)dzq, (long)count,
                       g_loss, coef, (float*)dz);
  return launch_status();
}

extern "C" int rdeic_scale_dev(const float* x, int64_t count, const float* s, float* y, int32_t accumulate,
                               void* stream) {
  if (!x || !s || !y || count <= 0) return RDEIC_EINVAL;
  hipLaunchKernelGGL(scale_dev_kernel, dim3(grid_1d(count)), dim3(256), 0, (hipStream_t)stream, x, (long)count, s, y,
                     accumulate);
  return launch_status();
}

extern "C" int rdeic_adamw(float* p, const float* g, float* m, float* v, int64_t count, float lr, float beta1,
                           float beta2, float eps, float weight_decay, int32_t step, void* stream) {
  if (!p || !g || !m || !v || count <= 0 || step <= 0) return RDEIC_EINVAL;
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_1d(count)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (long)count,
                     (float)(1.0 - (double)lr * weight_decay), (float)(1.0 - (double)beta1), beta2,
                     (float)(1.0 - (double)beta2), (float)sqrt(bc2), (float)(-(double)lr / bc1), eps);
  return launch_status();
}

extern "C" int rdeic_adamw_dev(float* p, const float* g, float* m, float* v, int64_t count, float lr, float beta1,
                               float beta2, float eps, float weight_decay, const float* step_scalars, void* stream) {
  if (!p || !g || !m || !v || !step_scalars || count <= 0) return RDEIC_EINVAL;
  hipLaunchKernelGGL(adamw_dev_kernel, dim3(grid_1d(count)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (long)count,
                     (float)(1.0 - (double)lr * weight_decay), (float)(1.0 - (double)beta1), beta2,
                     (float)(1.0 - (double)beta2), step_scalars, eps);
  return launch_status();
}
