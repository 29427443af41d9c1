// GroupNorm statistics / apply and LayerNorm over NHWC activations (gfx950).
//
// GroupNorm is split in two so that the normalisation itself can be fused into the
// consumer's loads (the implicit-GEMM conv prologue applies y = silu?(x*a + b)):
//   pass 1  per (image, pixel-chunk) block: per-channel shifted sums  S1=sum(x-K), S2=sum((x-K)^2)
//           with K = x[img, pixel 0, ch] (shifted data keeps the fp32 variance well conditioned)
//   pass 2  per (image, group): combine chunks in a fixed order -> mean, rstd -> per-channel a, b
// The input may be a two-segment channel concatenation (the UNet decoder's torch.cat of the
// running activation and the skip), whose groups can straddle the segment boundary: pass 1
// runs per segment into one per-channel partial buffer, pass 2 is segment-agnostic.
// Both passes are deterministic (fixed reduction order, no atomics).
//
// Replaces GroupNorm32 (ldm/modules/diffusionmodules/util.py:224-226, eps 1e-5, fp32),
// GroupNorm_leq32 (model/rdeic.py:480-482), Normalize (attention.py:96-97 / model.py:48-49, eps 1e-6)
// and nn.LayerNorm (attention.py:265-267).
#include <cstdlib>
#include "common.h"
#include "../../include/rdeic_hip.h"
#include "prof.h"

namespace {

constexpr int GN_CHUNK_MAX = 512;  // pixels per pass-1 block (fp32; bf16 adapts, gn_chunk)

// Pass-1 pixels per block: 512, halved for bf16 (down to 32) while an image has fewer than 64
// chunks, so the 64x64 .. 8x8 UNet levels still launch enough blocks to fill the chip. It depends
// on hw and dtype only, never on the batch, so the statistics stay batch-invariant; the fp32
// (parity) path keeps 512.
inline int gn_chunk(int hw, int esize) {
  int ch = GN_CHUNK_MAX;
  if (esize == 2)
    while (ch > 32 && hw / ch < 64) ch >>= 1;
  return ch;
}

template <typename T>
__device__ __forceinline__ float load_seg(const T* x0, int c0, int ld0, const T* x1, int ld1, long img_pix, int ch) {
  return ch < c0 ? to_f32(x0[img_pix * ld0 + ch]) : to_f32(x1[img_pix * ld1 + (ch - c0)]);
}

// One segment: channels [coff, coff + cs) of the logical c-channel tensor.
template <typename T>
__global__ __launch_bounds__(256) void gn_partial_kernel(const T* __restrict__ x, int hw, int cs, int ld, int coff,
                                                         int c, int nchunk, int pix_per, float* __restrict__ part) {
  const int img = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * pix_per;
  const int p1 = min(hw, p0 + pix_per);
  const T* xi = x + (long)img * hw * ld;
  int PL = 1;  // pixel lanes when the segment width divides 256
  if (cs < 256 && 256 % cs == 0) PL = 256 / cs;
  __shared__ float red[2][256];
  const int t = threadIdx.x;
  if (PL > 1) {
    const int ch0 = t % cs, pl = t / cs;
    const float K = to_f32(xi[ch0]);
    float s1 = 0.f, s2 = 0.f;
    // 16 loads in flight per thread, then the pixel-ordered sums (same order as one at a time)
    for (int p = p0 + pl; p < p1; p += 16 * PL) {
      float y[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) y[u] = p + u * PL < p1 ? to_f32(xi[(long)(p + u * PL) * ld + ch0]) : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (p + u * PL >= p1) break;
        float v = y[u] - K;
        s1 += v;
        s2 += v * v;
      }
    }
    red[0][t] = s1;
    red[1][t] = s2;
    __syncthreads();
    if (pl == 0) {
      for (int q = 1; q < PL; ++q) { s1 += red[0][t + q * cs]; s2 += red[1][t + q * cs]; }
      float* o = part + (((long)img * nchunk + chunk) * c + coff + ch0) * 2;
      o[0] = s1;
      o[1] = s2;
    }
  } else {
    for (int ch0 = t; ch0 < cs; ch0 += 256) {
      const float K = to_f32(xi[ch0]);
      float s1 = 0.f, s2 = 0.f;
      for (int p = p0; p < p1; p += 16) {
        float y[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) y[u] = p + u < p1 ? to_f32(xi[(long)(p + u) * ld + ch0]) : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (p + u >= p1) break;
          float v = y[u] - K;
          s1 += v;
          s2 += v * v;
        }
      }
      float* o = part + (((long)img * nchunk + chunk) * c + coff + ch0) * 2;
      o[0] = s1;
      o[1] = s2;
    }
  }
}

// 16-byte vectorised pass 1 for bf16 (segment width a multiple of 8, at most 2048 channels):
// thread = one 8-channel chunk of pixels pl, pl+PL, ...; pixel lanes reduced in a fixed order.
template <int U>
__global__ __launch_bounds__(256) void gn_partial_vec_kernel(const bf16* __restrict__ x, int hw, int cs, int ld,
                                                             int coff, int c, int nchunk, int pix_per,
                                                             float* __restrict__ part) {
  const int img = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * pix_per;
  const int p1 = min(hw, p0 + pix_per);
  const bf16* xi = x + (long)img * hw * ld;
  const int cp = cs >> 3;
  const int PL = 256 / cp;
  const int t = threadIdx.x;
  const int q = t % cp, pl = t / cp;
  const bool active = pl < PL;
  float s1[8], s2[8], K[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; K[e] = 0.f; }
  if (active) {
    bf16x8 k = *reinterpret_cast<const bf16x8*>(xi + q * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) K[e] = (float)k[e];
    // U independent 16-byte loads in flight per thread; accumulation stays in pixel order
    int p = p0 + pl;
    const bf16* xq = xi + q * 8;
    for (; p + (U - 1) * PL < p1; p += U * PL) {
      bf16x8 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const bf16x8*>(xq + (long)(p + u * PL) * ld);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float d = (float)v[u][e] - K[e];
          s1[e] += d;
          s2[e] += d * d;
        }
    }
    for (; p < p1; p += PL) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(xq + (long)p * ld);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = (float)v[e] - K[e];
        s1[e] += d;
        s2[e] += d * d;
      }
    }
  }
  __shared__ float red[256 * 16];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[e * 256 + t] = s1[e]; red[(8 + e) * 256 + t] = s2[e]; }  // SoA: no bank conflicts
  __syncthreads();
  if (active && pl == 0) {
    for (int l = 1; l < PL; ++l) {
      const float* r = red + l * cp + q;
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] += r[e * 256]; s2[e] += r[(8 + e) * 256]; }
    }
    float* o = part + (((long)img * nchunk + chunk) * c + coff + q * 8) * 2;
#pragma unroll
    for (int e = 0; e < 8; ++e) { o[2 * e] = s1[e]; o[2 * e + 1] = s2[e]; }
  }
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// pass 2, one 256-thread block per (group, image): the (chunk, channel) partials of the group are
// spread over all threads (fixed assignment, fixed tree order -> deterministic). With K_ch the
// per-channel shift, S1_ch = sum_q s1[q][ch], S2_ch likewise:
//   mean = (sum_ch S1_ch + cnt * sum_ch K_ch) / N
//   M2   = sum_ch S2_ch + 2 sum_ch d_ch S1_ch + cnt sum_ch d_ch^2,   d_ch = K_ch - mean
template <typename T>
__global__ __launch_bounds__(256) void gn_finalize_kernel(const T* __restrict__ x0, int c0, int ld0,
                                                          const T* __restrict__ x1, int ld1, int hw, int c, int groups,
                                                          int nchunk, const float* __restrict__ part, float eps,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ ab) {
  const int img = blockIdx.y, g = blockIdx.x;
  const int cpg = c / groups;
  const int t = threadIdx.x;
  const float cnt = (float)hw;
  __shared__ float Ks[512];
  __shared__ float red[4];
  for (int j = t; j < cpg; j += 256) Ks[j] = load_seg(x0, c0, ld0, x1, ld1, (long)img * hw, g * cpg + j);
  __syncthreads();
  const int pairs = nchunk * cpg;
  const float* pb = part + ((long)img * nchunk * c + g * cpg) * 2;
  float a1 = 0.f, ks = 0.f;
  for (int i = t; i < pairs; i += 256) {
    const int q = i / cpg, j = i - q * cpg;
    a1 += pb[((long)q * c + j) * 2];
  }
  for (int j = t; j < cpg; j += 256) ks += Ks[j];
  const float n_el = cnt * (float)cpg;
  const float mean = (block_sum256(a1, red) + cnt * block_sum256(ks, red)) / n_el;
  float a2 = 0.f, dd = 0.f;
  for (int i = t; i < pairs; i += 256) {
    const int q = i / cpg, j = i - q * cpg;
    const float* pp = pb + ((long)q * c + j) * 2;
    a2 += pp[1] + 2.f * (Ks[j] - mean) * pp[0];
  }
  for (int j = t; j < cpg; j += 256) {
    const float d = Ks[j] - mean;
    dd += d * d;
  }
  const float m2 = block_sum256(a2, red) + cnt * block_sum256(dd, red);
  const float var = fmaxf(m2 / n_el, 0.f);
  const float rstd = rsqrtf(var + eps);
  for (int j = t; j < cpg; j += 256) {
    const int ch = g * cpg + j;
    const float ga = gamma ? gamma[ch] : 1.f, be = beta ? beta[ch] : 0.f;
    const float av = ga * rstd;
    ab[((long)img * c + ch) * 2 + 0] = av;
    ab[((long)img * c + ch) * 2 + 1] = be - mean * av;
  }
}

// y = silu?(x*a + b) * out_mul; ab rows have ab_c channels per image (ab points at channel 0 of x)
template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x, int n, int hw, int c, int ld,
                                                       const float* __restrict__ ab, int ab_c, int silu,
                                                       float out_mul, T* __restrict__ y, int yld) {
  long total = (long)n * hw * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    long pix = i / c;
    int ch = (int)(i - pix * c);
    int img = (int)(pix / hw);
    const float* p = ab + ((long)img * ab_c + ch) * 2;
    float v = to_f32(x[pix * ld + ch]) * p[0] + p[1];
    if (silu) v = silu_f(v);
    y[pix * yld + ch] = from_f32<T>(v * out_mul);
  }
}

// 16-byte vectorised variant: one thread = 8 bf16 channels of one pixel (c, ld, yld multiples of 8);
// grid (x, image), 32-bit indexing inside an image, U chunks per thread for loads in flight. When
// 256 % (c / 8) == 0 (every VAE / compressor width: 128, 256, 512) a thread's U chunks share one
// channel group, so its 64 bytes of (a, b) are loaded once instead of U times (the per-chunk table
// reads were 4x the x traffic through L1 / TA).
constexpr int GN_APPLY_LDS_C = 2560;  // widest non-uniform GroupNorm input (the UNet's 2560-channel concat)

template <bool UNIFORM, int U>
__global__ __launch_bounds__(256) void gn_apply_vec_kernel(const bf16* __restrict__ x, int n, int hw, int c, int ld,
                                                           const float* __restrict__ ab, int ab_c, int silu,
                                                           float out_mul, bf16* __restrict__ y, int yld) {
  const int cp = c >> 3;
  const int img = blockIdx.y;
  const int total = hw * cp;
  const bf16* xi = x + (long)img * hw * ld;
  bf16* yi = y + (long)img * hw * yld;
  const float* abi = ab + (long)img * ab_c * 2;
  const int base = blockIdx.x * (256 * U) + threadIdx.x;
  bf16x8 v[U];
  int pix[U], ch[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = base + u * 256;
    pix[u] = i / cp;
    ch[u] = (i - pix[u] * cp) * 8;
    if (i < total) v[u] = *reinterpret_cast<const bf16x8*>(xi + (long)pix[u] * ld + ch[u]);
  }
  float4 sab[4];
  // non-uniform widths (the UNet's 320 ... 2560 channels): the image's (a, b) table goes to LDS once
  // per block (<= 20 KB), behind the x loads already in flight, so the per-chunk table reads are
  // LDS reads instead of 4x the x traffic through the vector cache
  __shared__ __attribute__((aligned(16))) float lab[UNIFORM ? 4 : 2 * GN_APPLY_LDS_C];
  if (UNIFORM) {
    const float4* p = reinterpret_cast<const float4*>(abi + ch[0] * 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) sab[q] = p[q];
  } else {
    for (int i = threadIdx.x; i < cp * 4; i += 256)
      reinterpret_cast<float4*>(lab)[i] = reinterpret_cast<const float4*>(abi)[i];
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (base + u * 256 >= total) break;
    const float4* p = reinterpret_cast<const float4*>(lab + ch[u] * 2);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 s = UNIFORM ? sab[q] : p[q];  // (a, b) of channels ch+2q, ch+2q+1
      float v0 = (float)v[u][2 * q] * s.x + s.y;
      float v1 = (float)v[u][2 * q + 1] * s.z + s.w;
      if (silu) {  // x * rcp(1 + e^-x): v_rcp instead of the IEEE divide sequence (bf16 output)
        v0 *= __builtin_amdgcn_rcpf(1.0f + __expf(-v0));
        v1 *= __builtin_amdgcn_rcpf(1.0f + __expf(-v1));
      }
      o[2 * q] = (bf16)(v0 * out_mul);
      o[2 * q + 1] = (bf16)(v1 * out_mul);
    }
    *reinterpret_cast<bf16x8*>(yi + (long)pix[u] * yld + ch[u]) = o;
  }
}

// LayerNorm, bf16, c % 8 == 0, c <= 2048: one wave per row, the row held in registers (one HBM
// read), 4 rows per 256-thread block.
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const bf16* __restrict__ x, int rows, int c, int ld,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            bf16* __restrict__ y, int yld) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int cp = c >> 3;
  const bf16* xr = x + (long)row * ld;
  bf16x8 v[4];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = lane + u * 64;
    if (k < cp) {
      v[u] = *reinterpret_cast<const bf16x8*>(xr + k * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)v[u][e];
    }
  }
  s = warp_sum(s);
  const float mean = s / c;
  float v2 = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = lane + u * 64;
    if (k < cp) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)v[u][e] - mean;
        v2 += d * d;
      }
    }
  }
  v2 = warp_sum(v2);
  const float rstd = rsqrtf(v2 / c + eps);
  bf16* yr = y + (long)row * yld;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = lane + u * 64;
    if (k < cp) {
      const float4 g0 = *reinterpret_cast<const float4*>(gamma + k * 8), g1 = *reinterpret_cast<const float4*>(gamma + k * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(beta + k * 8), b1 = *reinterpret_cast<const float4*>(beta + k * 8 + 4);
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)(((float)v[u][e] - mean) * rstd * gg[e] + bb[e]);
      *reinterpret_cast<bf16x8*>(yr + k * 8) = o;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(64) void layernorm_kernel(const T* __restrict__ x, int rows, int c, int ld,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps, T* __restrict__ y,
                                                       int yld) {
  const int row = blockIdx.x;
  const int lane = threadIdx.x;
  const T* xr = x + (long)row * ld;
  float s = 0.f;
  for (int j = lane; j < c; j += 64) s += to_f32(xr[j]);
  s = warp_sum(s);
  const float mean = s / c;
  float v2 = 0.f;
  for (int j = lane; j < c; j += 64) {
    float d = to_f32(xr[j]) - mean;
    v2 += d * d;
  }
  v2 = warp_sum(v2);
  const float rstd = rsqrtf(v2 / c + eps);
  T* yr = y + (long)row * yld;
  for (int j = lane; j < c; j += 64) {
    float d = (to_f32(xr[j]) - mean) * rstd;
    yr[j] = from_f32<T>(d * gamma[j] + beta[j]);
  }
}

template <typename T>
int gn_stats(const void* x0, int32_t c0, int32_t ld0, const void* x1, int32_t c1, int32_t ld1, int32_t n, int32_t hw,
             int32_t groups, float eps, const float* gamma, const float* beta, float* ab, float* ws, hipStream_t s) {
  const int c = c0 + c1;
  const int pix_per = gn_chunk(hw, (int)sizeof(T));
  const int nchunk = (hw + pix_per - 1) / pix_per;
  auto seg = [&](const void* xs, int cs, int ld, int coff) {
    const bool vec = sizeof(T) == 2 && cs % 8 == 0 && cs <= 2048 && ld % 8 == 0 && ((uintptr_t)xs) % 16 == 0;
    // 8 loads in flight per thread (A/B on the bench: stats 7.12 -> 6.93 ms/step vs 4); env override for A/B
    static const int unroll = getenv("RDEIC_GN_UNROLL") ? atoi(getenv("RDEIC_GN_UNROLL")) : 8;
    if (vec && unroll == 8)
      hipLaunchKernelGGL(gn_partial_vec_kernel<8>, dim3(nchunk, n), dim3(256), 0, s, (const bf16*)xs, hw, cs, ld, coff,
                         c, nchunk, pix_per, ws);
    else if (vec)
      hipLaunchKernelGGL(gn_partial_vec_kernel<4>, dim3(nchunk, n), dim3(256), 0, s, (const bf16*)xs, hw, cs, ld, coff,
                         c, nchunk, pix_per, ws);
    else
      hipLaunchKernelGGL(gn_partial_kernel<T>, dim3(nchunk, n), dim3(256), 0, s, (const T*)xs, hw, cs, ld, coff, c,
                         nchunk, pix_per, ws);
  };
  seg(x0, c0, ld0, 0);
  if (c1 > 0) seg(x1, c1, ld1, c0);
  hipLaunchKernelGGL(gn_finalize_kernel<T>, dim3(groups, n), dim3(256), 0, s, (const T*)x0, c0, ld0,
                     (const T*)(x1 ? x1 : x0), c1 > 0 ? ld1 : ld0, hw, c, groups, nchunk, ws, eps, gamma, beta, ab);
  return launch_status();
}

// ---- GroupNorm from per-row-block partial sums (the conv epilogue's fused statistics) ----------
// Partial format: a 16-byte header whose first int32 is R = 64 (rows per partial), then
// [rows / 64][c][2] fp32 (sum, sum of squares) of the tensor's stored values over each 64-row
// block, in the canonical order ((g0 + g1) + g2) + g3 of four 16-row groups summed sequentially
// (fmaf for the squares). The conv epilogue writes the same numbers (conv_gemm.hip, epilogue_vec);
// this kernel is its stand-alone fallback. 64 divides the image's pixel count (no straddling).
template <typename T>
__global__ __launch_bounds__(256) void gn_rows_partial_kernel(const T* __restrict__ x, long rows, int c, int ld,
                                                              float* __restrict__ part) {
  const int blk = blockIdx.x, ch = blockIdx.y * 256 + threadIdx.x;
  if (blk == 0 && ch == 0) reinterpret_cast<int*>(part)[0] = 64;
  if (ch >= c) return;
  const T* xp = x + (long)blk * 64 * ld + ch;
  float sg[4], qg[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const long nv = rows - ((long)blk * 64 + g * 16);  // valid rows of this 16-row group
    float s1 = 0.f, s2 = 0.f;
    if (nv >= 16) {  // 16 loads in flight, then the row-ordered sums
      float y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) y[r] = to_f32(xp[(long)(g * 16 + r) * ld]);
#pragma unroll
      for (int r = 0; r < 16; ++r) { s1 += y[r]; s2 = fmaf(y[r], y[r], s2); }
    } else {
      for (int r = 0; r < nv; ++r) {
        const float v = to_f32(xp[(long)(g * 16 + r) * ld]);
        s1 += v;
        s2 = fmaf(v, v, s2);
      }
    }
    sg[g] = s1;
    qg[g] = s2;
  }
  float* o = part + 4 + ((long)blk * c + ch) * 2;
  o[0] = ((sg[0] + sg[1]) + sg[2]) + sg[3];
  o[1] = ((qg[0] + qg[1]) + qg[2]) + qg[3];
}

__device__ __forceinline__ double block_sum256_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// One 256-thread block per (group, image). Channels [0, c0) come from p0, [c0, c0 + c1) from p1
// (the UNet's skip concat); sums in fp64 in a fixed order (deterministic); var = E[x^2] - mean^2.
__global__ __launch_bounds__(256) void gn_finalize_parts_kernel(const float* __restrict__ p0, int c0,
                                                                const float* __restrict__ p1, int c1, int hw,
                                                                int groups, float eps, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                float* __restrict__ ab) {
  const int img = blockIdx.y, g = blockIdx.x, t = threadIdx.x;
  const int c = c0 + c1, cpg = c / groups, ga = g * cpg, gb = ga + cpg;
  __shared__ double red[4];
  double S = 0.0, Q = 0.0;
  for (int sgi = 0; sgi < 2; ++sgi) {
    const float* p = sgi ? p1 : p0;
    const int base = sgi ? c0 : 0, cs = sgi ? c1 : c0;
    const int lo = max(ga, base), hi = min(gb, base + cs);
    if (hi <= lo) continue;
    const int R = reinterpret_cast<const int*>(p)[0];
    const int T = hw / R, nch = hi - lo;
    const float* q = p + 4 + ((long)img * T * cs + (lo - base)) * 2;
    // thread t sums the row blocks t, t + 256, ...: each one's nch (sum, sum of squares) pairs are
    // contiguous, read as 16-byte vectors when the channel count and the alignment allow
    const bool vec = (nch & 1) == 0 && (cs & 1) == 0 && (((uintptr_t)q) & 15) == 0;
    for (int tt = t; tt < T; tt += 256) {
      const float* e = q + (long)tt * cs * 2;
      if (vec) {
        for (int j = 0; j < nch; j += 2) {
          const float4 v = *reinterpret_cast<const float4*>(e + 2 * j);
          S += (double)v.x;
          Q += (double)v.y;
          S += (double)v.z;
          Q += (double)v.w;
        }
      } else {
        for (int j = 0; j < nch; ++j) {
          S += (double)e[2 * j];
          Q += (double)e[2 * j + 1];
        }
      }
    }
  }
  S = block_sum256_d(S, red);
  Q = block_sum256_d(Q, red);
  const double N = (double)hw * cpg;
  const double mean = S / N;
  const float var = (float)fmax(Q / N - mean * mean, 0.0);
  const float rstd = rsqrtf(var + eps);
  const float mf = (float)mean;
  for (int j = t; j < cpg; j += 256) {
    const int ch = ga + j;
    const float gm = gamma ? gamma[ch] : 1.f, be = beta ? beta[ch] : 0.f;
    const float av = gm * rstd;
    ab[((long)img * c + ch) * 2 + 0] = av;
    ab[((long)img * c + ch) * 2 + 1] = be - mf * av;
  }
}

// GroupNorm finalize + apply in ONE launch for small images (hw <= 256 pixels: the UNet / control net's 16^2 and
// 8^2 levels, T = hw / 64 <= 4 partial row blocks per image), openaimodel.py:200-204 / 254-274 (in_layers /
// out_layers GroupNorm32 -> SiLU) and attention.py:250-266 (SpatialTransformer.norm). There the two-launch form
// (gn_finalize_parts, then gn_apply) is two ~10 us latency floors for a few hundred KB of data.
// Every block recomputes its image's (a, b) table from the T x c partials (<= 80 KB, L2-resident) instead of
// waiting for a finalize launch: lane tt of a T-lane segment sums row block tt's channel pairs of one group in
// fp64 in gn_finalize_parts_kernel's order, and a butterfly over the T lanes (xor offsets T/2 .. 1) gives the
// same number as that kernel's 256-thread reduction (its lanes >= T add exact zeros), so mean / rstd and the
// (a, b) table are bit-identical to the two-launch path; so is the apply arithmetic (gn_apply_vec_kernel's).
// Channels [0, c0) come from x0 / p0 and [c0, c0 + c1) from x1 / p1 (the UNet's skip concat); the output y holds
// all c0 + c1 channels. Block (0, img) also writes the table to ab (for any other consumer of it).
constexpr int GNPA_U = 8;  // 16-byte chunks per thread
__global__ __launch_bounds__(256) void gn_parts_apply_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                             const bf16* __restrict__ x0, int c0, int ld0,
                                                             const bf16* __restrict__ x1, int c1, int ld1, int hw,
                                                             int groups, float eps, const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int silu,
                                                             float* __restrict__ ab, bf16* __restrict__ y, int yld) {
  __shared__ __attribute__((aligned(16))) float lab[2 * GN_APPLY_LDS_C];
  __shared__ float gms[2 * 256];  // per group (mean as float, rstd)
  const int img = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = c0 + c1, cpg = c / groups;
  const int T = hw / 64;                 // partial row blocks per image: 1, 2 or 4
  const int gpw = 64 / T;                // groups per wave pass
  // x chunks first (their loads fly under the finalize)
  const int cp = c >> 3, total = hw * cp;
  const int base = blockIdx.x * (256 * GNPA_U) + t;
  bf16x8 v[GNPA_U];
  int pix[GNPA_U], ch[GNPA_U];
#pragma unroll
  for (int u = 0; u < GNPA_U; ++u) {
    const int i = base + u * 256;
    pix[u] = i / cp;
    ch[u] = (i - pix[u] * cp) * 8;
    if (i < total) {
      const bool s1 = ch[u] >= c0;
      v[u] = *reinterpret_cast<const bf16x8*>(s1 ? x1 + ((long)img * hw + pix[u]) * ld1 + (ch[u] - c0)
                                                  : x0 + ((long)img * hw + pix[u]) * ld0 + ch[u]);
    }
  }
  // finalize: wave w takes groups w * gpw + k * 4 * gpw + lane / T
  for (int gb = wave * gpw; gb < groups; gb += 4 * gpw) {
    const int g = gb + lane / T, tt = lane % T;
    double S = 0.0, Q = 0.0;
    if (g < groups) {
      const int ga = g * cpg, ge = ga + cpg;
      for (int sgi = 0; sgi < 2; ++sgi) {
        const float* p = sgi ? p1 : p0;
        const int sb = sgi ? c0 : 0, cs = sgi ? c1 : c0;
        const int lo = max(ga, sb), hi = min(ge, sb + cs);
        if (hi <= lo) continue;
        const float* e = p + 4 + (((long)img * T + tt) * cs + (lo - sb)) * 2;
        const int nch = hi - lo;
        int j = 0;
        for (; j + 8 <= nch; j += 8) {  // 8 loads in flight, then the adds in channel order
          float2 v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float2*>(e + 2 * (j + u));
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            S += (double)v[u].x;
            Q += (double)v[u].y;
          }
        }
        for (; j < nch; ++j) {
          S += (double)e[2 * j];
          Q += (double)e[2 * j + 1];
        }
      }
    }
    for (int o = T >> 1; o > 0; o >>= 1) {  // the 256-thread reduction restricted to its nonzero lanes
      S += __shfl_xor(S, o, 64);
      Q += __shfl_xor(Q, o, 64);
    }
    S = (S + 0.0) + (0.0 + 0.0);  // block_sum256_d's cross-wave combine, the other waves' sums being +0
    Q = (Q + 0.0) + (0.0 + 0.0);
    if (g < groups && tt == 0) {
      const double N = (double)hw * cpg;
      const double mean = S / N;
      const float var = (float)fmax(Q / N - mean * mean, 0.0);
      gms[2 * g] = (float)mean;
      gms[2 * g + 1] = rsqrtf(var + eps);
    }
  }
  __syncthreads();
  for (int j = t; j < c; j += 256) {
    const int g = j / cpg;
    const float mf = gms[2 * g], rstd = gms[2 * g + 1];
    const float gm = gamma ? gamma[j] : 1.f, be = beta ? beta[j] : 0.f;
    const float av = gm * rstd, bv = be - mf * av;
    lab[2 * j] = av;
    lab[2 * j + 1] = bv;
    if (blockIdx.x == 0) {
      ab[((long)img * c + j) * 2 + 0] = av;
      ab[((long)img * c + j) * 2 + 1] = bv;
    }
  }
  __syncthreads();
  bf16* yi = y + (long)img * hw * yld;
#pragma unroll
  for (int u = 0; u < GNPA_U; ++u) {
    if (base + u * 256 >= total) break;
    const float4* p = reinterpret_cast<const float4*>(lab + ch[u] * 2);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 s = p[q];  // (a, b) of channels ch+2q, ch+2q+1
      float v0 = (float)v[u][2 * q] * s.x + s.y;
      float v1 = (float)v[u][2 * q + 1] * s.z + s.w;
      if (silu) {  // x * rcp(1 + e^-x), as gn_apply_vec_kernel
        v0 *= __builtin_amdgcn_rcpf(1.0f + __expf(-v0));
        v1 *= __builtin_amdgcn_rcpf(1.0f + __expf(-v1));
      }
      o[2 * q] = (bf16)v0;
      o[2 * q + 1] = (bf16)v1;
    }
    *reinterpret_cast<bf16x8*>(yi + (long)pix[u] * yld + ch[u]) = o;
  }
}

}  // namespace

// stand-alone partials of a [rows][c] (pixel stride ld) tensor (declared in common.h for the conv
// launcher's fallback); hw (pixels per image) must be a multiple of 64
int gn_rows_partial(const void* x, long rows, int c, int ld, int hw, float* part, int dtype, hipStream_t s) {
  if (hw % 64 || rows % hw) return RDEIC_EINVAL;
  dim3 grid((unsigned)(rows / 64), (unsigned)((c + 255) / 256));
  if (dtype == 1)
    hipLaunchKernelGGL(gn_rows_partial_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, rows, c, ld, part);
  else
    hipLaunchKernelGGL(gn_rows_partial_kernel<float>, grid, dim3(256), 0, s, (const float*)x, rows, c, ld, part);
  return launch_status();
}

extern "C" size_t rdeic_groupnorm_parts_floats(int64_t rows, int32_t c, int32_t hw) {
  if (hw <= 0 || hw % 64 || rows <= 0 || c <= 0) return 0;  // 0: statistics cannot be fused for this shape
  return (size_t)(4 + (rows / 64) * c * 2);
}

extern "C" int rdeic_groupnorm_parts_ab(const float* p0, int32_t c0, const float* p1, int32_t c1, int32_t n,
                                        int32_t hw, int32_t groups, float eps, const float* gamma, const float* beta,
                                        float* ab, void* stream) {
  const int c = c0 + c1;
  if (!p0 || !ab || n <= 0 || hw <= 0 || hw % 64 || c0 <= 0 || c1 < 0 || (c1 > 0 && !p1) || groups <= 0 ||
      c % groups)
    return RDEIC_EINVAL;
  hipLaunchKernelGGL(gn_finalize_parts_kernel, dim3(groups, n), dim3(256), 0, (hipStream_t)stream, p0, c0,
                     p1 ? p1 : p0, c1, hw, groups, eps, gamma, beta, ab);
  return launch_status();
}

extern "C" int rdeic_groupnorm_parts_apply(const float* p0, int32_t c0, const float* p1, int32_t c1, const void* x0,
                                           int32_t ld0, const void* x1, int32_t ld1, int32_t n, int32_t hw,
                                           int32_t groups, float eps, const float* gamma, const float* beta,
                                           int32_t silu, float* ab, void* y, int32_t yld, void* stream) {
  const int c = c0 + c1;
  if (!p0 || !x0 || !ab || !y || n <= 0 || (hw != 64 && hw != 128 && hw != 256) || c0 <= 0 || c1 < 0 ||
      (c1 > 0 && (!p1 || !x1)) || groups <= 0 || groups > 256 || c % groups || c0 % 8 || c1 % 8 ||
      c > GN_APPLY_LDS_C || ld0 % 8 || (c1 && ld1 % 8) || yld % 8 || ((uintptr_t)x0) % 16 ||
      (c1 && ((uintptr_t)x1) % 16) || ((uintptr_t)y) % 16)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(s, RDEIC_PROF_GN_APPLY, 2.0 * n * hw * c * 2);
  rdeic_count_launch(RDEIC_COUNT_GN_PARTS_APPLY);
  const int blocks = (hw * (c / 8) + 256 * GNPA_U - 1) / (256 * GNPA_U);
  hipLaunchKernelGGL(gn_parts_apply_kernel, dim3(blocks, n), dim3(256), 0, s, p0, p1 ? p1 : p0, (const bf16*)x0, c0, ld0,
                     (const bf16*)(x1 ? x1 : x0), c1, c1 ? ld1 : ld0, hw, groups, eps, gamma, beta, silu, ab, (bf16*)y,
                     yld);
  return launch_status();
}

extern "C" size_t rdeic_groupnorm_ws_floats(int32_t n, int32_t hw, int32_t c) {
  const int pix_per = gn_chunk(hw, 2);  // the bf16 chunk is never larger than the fp32 one
  long nchunk = (hw + pix_per - 1) / pix_per;
  return (size_t)n * nchunk * c * 2;
}

extern "C" int rdeic_groupnorm_stats(const void* x0, int32_t c0, int32_t ld0, const void* x1, int32_t c1, int32_t ld1,
                                     int32_t n, int32_t hw, int32_t groups, float eps, const float* gamma,
                                     const float* beta, float* ab, float* ws, int32_t dtype, void* stream) {
  const int c = c0 + c1;
  if (!x0 || !ab || !ws || n <= 0 || hw <= 0 || c0 <= 0 || c1 < 0 || (c1 > 0 && !x1) || groups <= 0 ||
      c % groups != 0 || c / groups > 512)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(s, RDEIC_PROF_GN_STATS, (double)n * hw * c * (dtype == 1 ? 2 : 4));
  if (dtype == 1) return gn_stats<bf16>(x0, c0, ld0, x1, c1, ld1, n, hw, groups, eps, gamma, beta, ab, ws, s);
  return gn_stats<float>(x0, c0, ld0, x1, c1, ld1, n, hw, groups, eps, gamma, beta, ab, ws, s);
}

extern "C" int rdeic_groupnorm_apply(const void* x, int32_t n, int32_t hw, int32_t c, int32_t ld, const float* ab,
                                     int32_t ab_c, int32_t silu, float out_mul, void* y, int32_t yld, int32_t dtype,
                                     void* stream) {
  if (!x || !ab || !y || n <= 0 || hw <= 0 || c <= 0 || ab_c < c) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(s, RDEIC_PROF_GN_APPLY, 2.0 * n * hw * c * (dtype == 1 ? 2 : 4));
  rdeic_count_launch(RDEIC_COUNT_GN_APPLY);
  long total = (long)n * hw * c;
  if (dtype == 1 && c % 8 == 0 && ld % 8 == 0 && yld % 8 == 0 && ((uintptr_t)x) % 16 == 0 &&
      ((uintptr_t)y) % 16 == 0 && ((uintptr_t)ab) % 16 == 0 && (ab_c % 2) == 0 &&
      (256 % (c / 8) == 0 || c <= GN_APPLY_LDS_C)) {
    if ((long)hw * (c / 8) >= (1L << 31) - 2048) return RDEIC_EINVAL;
    if (256 % (c / 8) == 0) {
      const int blocks = (int)(((long)hw * (c / 8) + 2047) / 2048);
      hipLaunchKernelGGL((gn_apply_vec_kernel<true, 8>), dim3(blocks, n), dim3(256), 0, s, (const bf16*)x, n, hw, c, ld,
                         ab, ab_c, silu, out_mul, (bf16*)y, yld);
    } else {
      const int blocks = (int)(((long)hw * (c / 8) + 1023) / 1024);
      hipLaunchKernelGGL((gn_apply_vec_kernel<false, 4>), dim3(blocks, n), dim3(256), 0, s, (const bf16*)x, n, hw, c,
                         ld, ab, ab_c, silu, out_mul, (bf16*)y, yld);
    }
    return launch_status();
  }
  int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  if (dtype == 1)
    hipLaunchKernelGGL(gn_apply_kernel<bf16>, dim3(blocks), dim3(256), 0, s, (const bf16*)x, n, hw, c, ld, ab, ab_c,
                       silu, out_mul, (bf16*)y, yld);
  else
    hipLaunchKernelGGL(gn_apply_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, n, hw, c, ld, ab, ab_c,
                       silu, out_mul, (float*)y, yld);
  return launch_status();
}

// Row statistics of a LayerNorm whose affine is folded into the consuming linear
// (rdeic_conv_desc.ln_rows): 16 lanes per row, 4 rows per wave, each lane up to 16 chunks of 8 bf16 in
// registers (one HBM read), mean then the centred sum of squares (two passes over the registers, as
// rdeic_layernorm computes them), xor-shuffle sums inside the 16-lane group.
__global__ __launch_bounds__(256) void ln_rowstats_kernel(const bf16* __restrict__ x, int rows, int c, int ld, float eps,
                                                          float2* __restrict__ ms) {
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int l = threadIdx.x & 15;
  const int cp = c >> 3;
  const bool live = row < rows;
  const bf16* xr = x + (long)(live ? row : 0) * ld;
  bf16x8 v[16];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int k = l + u * 16;
    if (live && k < cp) {
      v[u] = *reinterpret_cast<const bf16x8*>(xr + k * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)v[u][e];
    }
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / c;
  float v2 = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int k = l + u * 16;
    if (live && k < cp) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)v[u][e] - mean;
        v2 += d * d;
      }
    }
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v2 += __shfl_xor(v2, o, 64);
  if (live && l == 0) ms[row] = make_float2(mean, rsqrtf(v2 / c + eps));
}

extern "C" int rdeic_layernorm_rowstats(const void* x, int32_t rows, int32_t c, int32_t ld, float eps, float* ms,
                                        void* stream) {
  if (!x || !ms || rows <= 0 || c <= 0 || c % 8 || c > 2048 || ld % 8 || ((uintptr_t)x) % 16 || ((uintptr_t)ms) % 8)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  rdeic_count_launch(RDEIC_COUNT_LN_FUSED);
  hipLaunchKernelGGL(ln_rowstats_kernel, dim3((rows + 15) / 16), dim3(256), 0, s, (const bf16*)x, rows, c, ld, eps,
                     reinterpret_cast<float2*>(ms));
  return launch_status();
}

extern "C" int rdeic_layernorm(const void* x, int32_t rows, int32_t c, int32_t ld, const float* gamma,
                               const float* beta, float eps, void* y, int32_t yld, int32_t dtype, void* stream) {
  if (!x || !y || !gamma || !beta || rows <= 0 || c <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  rdeic_count_launch(RDEIC_COUNT_LAYERNORM);
  if (dtype == 1 && c % 8 == 0 && c <= 2048 && ld % 8 == 0 && yld % 8 == 0 && ((uintptr_t)x) % 16 == 0 &&
      ((uintptr_t)y) % 16 == 0 && ((uintptr_t)gamma) % 16 == 0 && ((uintptr_t)beta) % 16 == 0)
    hipLaunchKernelGGL(layernorm_vec_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, (const bf16*)x, rows, c, ld, gamma,
                       beta, eps, (bf16*)y, yld);
  else if (dtype == 1)
    hipLaunchKernelGGL(layernorm_kernel<bf16>, dim3(rows), dim3(64), 0, s, (const bf16*)x, rows, c, ld, gamma, beta,
                       eps, (bf16*)y, yld);
  else
    hipLaunchKernelGGL(layernorm_kernel<float>, dim3(rows), dim3(64), 0, s, (const float*)x, rows, c, ld, gamma, beta,
                       eps, (float*)y, yld);
  return launch_status();
}
