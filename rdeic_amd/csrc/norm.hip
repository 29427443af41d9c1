// GroupNorm statistics / apply and LayerNorm over NHWC activations (gfx950).
//
// GroupNorm is split in two so that the normalisation itself can be fused into the
// consumer's loads (the implicit-GEMM conv prologue applies y = silu?(x*a + b)):
//   pass 1  per (image, pixel-chunk) block: per-channel shifted sums  S1=sum(x-K), S2=sum((x-K)^2)
//           with K = x[img, pixel 0, ch] (shifted data keeps the fp32 variance well conditioned)
//   pass 2  per (image, group): combine chunks in a fixed order -> mean, rstd -> per-channel a, b
// Both passes are deterministic (fixed reduction order, no atomics).
//
// Replaces GroupNorm32 (ldm/modules/diffusionmodules/util.py:224-226, eps 1e-5, fp32),
// GroupNorm_leq32 (model/rdeic.py:480-482), Normalize (attention.py:96-97 / model.py:48-49, eps 1e-6)
// and nn.LayerNorm (attention.py:265-267).
#include "common.h"
#include "../../include/rdeic_hip.h"

namespace {

constexpr int GN_CHUNK = 512;  // pixels per pass-1 block

template <typename T>
__global__ __launch_bounds__(256) void gn_partial_kernel(const T* __restrict__ x, int hw, int c, int ld, int nchunk,
                                                         float* __restrict__ part /*[n][nchunk][c][2]*/) {
  const int img = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * GN_CHUNK;
  const int p1 = min(hw, p0 + GN_CHUNK);
  const T* xi = x + (long)img * hw * ld;
  // pixel lanes: split the 256 threads into PL pixel lanes when c divides 256
  int PL = 1;
  if (c < 256 && 256 % c == 0) PL = 256 / c;
  __shared__ float red[2][256];
  const int t = threadIdx.x;
  const int pl = (PL > 1) ? t / c : 0;
  for (int ch0 = (PL > 1 ? t % c : t); ch0 < c; ch0 += (PL > 1 ? c : 256)) {
    const float K = to_f32(xi[ch0]);
    float s1 = 0.f, s2 = 0.f;
    for (int p = p0 + pl; p < p1; p += PL) {
      float v = to_f32(xi[(long)p * ld + ch0]) - K;
      s1 += v;
      s2 += v * v;
    }
    if (PL > 1) {
      red[0][t] = s1; red[1][t] = s2;
      __syncthreads();
      if (pl == 0) {
        for (int q = 1; q < PL; ++q) { s1 += red[0][t + q * c]; s2 += red[1][t + q * c]; }
        float* o = part + (((long)img * nchunk + chunk) * c + ch0) * 2;
        o[0] = s1; o[1] = s2;
      }
      __syncthreads();
    } else {
      float* o = part + (((long)img * nchunk + chunk) * c + ch0) * 2;
      o[0] = s1; o[1] = s2;
    }
    if (PL > 1) break;
  }
}

template <typename T>
__global__ __launch_bounds__(64) void gn_finalize_kernel(const T* __restrict__ x, int hw, int c, int ld, int groups,
                                                         int nchunk, const float* __restrict__ part, float eps,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ ab) {
  const int img = blockIdx.y, g = blockIdx.x;
  const int cpg = c / groups;
  const int lane = threadIdx.x;
  const T* xi = x + (long)img * hw * ld;
  // pass A: per-channel totals (lane owns channels lane, lane+64, ...) in fixed order
  double cnt = (double)hw;
  float s1c[8], s2c[8], Kc[8];  // cpg <= 512 -> up to 8 channels per lane
  int nmine = 0;
  for (int j = lane; j < cpg; j += 64, ++nmine) {
    int ch = g * cpg + j;
    float s1 = 0.f, s2 = 0.f;
    for (int q = 0; q < nchunk; ++q) {
      const float* pp = part + (((long)img * nchunk + q) * c + ch) * 2;
      s1 += pp[0];
      s2 += pp[1];
    }
    s1c[nmine] = s1; s2c[nmine] = s2; Kc[nmine] = to_f32(xi[ch]);
  }
  // group mean
  float tot = 0.f;
  for (int q = 0; q < nmine; ++q) tot += s1c[q] + (float)cnt * Kc[q];
  tot = warp_sum(tot);
  const float n_el = (float)(cnt * cpg);
  const float mean = tot / n_el;
  float m2 = 0.f;
  for (int q = 0; q < nmine; ++q) {
    float d = Kc[q] - mean;
    m2 += s2c[q] + 2.f * d * s1c[q] + (float)cnt * d * d;
  }
  m2 = warp_sum(m2);
  float var = fmaxf(m2 / n_el, 0.f);
  float rstd = rsqrtf(var + eps);
  for (int j = lane; j < cpg; j += 64) {
    int ch = g * cpg + j;
    float ga = gamma ? gamma[ch] : 1.f, be = beta ? beta[ch] : 0.f;
    float a = ga * rstd;
    ab[((long)img * c + ch) * 2 + 0] = a;
    ab[((long)img * c + ch) * 2 + 1] = be - mean * a;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x, int n, int hw, int c, int ld,
                                                       const float* __restrict__ ab, int silu, T* __restrict__ y,
                                                       int yld) {
  long total = (long)n * hw * c;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    long pix = i / c;
    int ch = (int)(i - pix * c);
    int img = (int)(pix / hw);
    const float* p = ab + ((long)img * c + ch) * 2;
    float v = to_f32(x[pix * ld + ch]) * p[0] + p[1];
    if (silu) v = silu_f(v);
    y[pix * yld + ch] = from_f32<T>(v);
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

}  // namespace

extern "C" size_t rdeic_groupnorm_ws_floats(int32_t n, int32_t hw, int32_t c) {
  long nchunk = (hw + GN_CHUNK - 1) / GN_CHUNK;
  return (size_t)n * nchunk * c * 2;
}

extern "C" int rdeic_groupnorm_stats(const void* x, int32_t n, int32_t hw, int32_t c, int32_t ld, int32_t groups,
                                     float eps, const float* gamma, const float* beta, float* ab, float* ws,
                                     int32_t dtype, void* stream) {
  if (!x || !ab || !ws || n <= 0 || hw <= 0 || c <= 0 || groups <= 0 || c % groups != 0 || c / groups > 512)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int nchunk = (hw + GN_CHUNK - 1) / GN_CHUNK;
  dim3 g1(nchunk, n), g2(groups, n);
  if (dtype == 1) {
    hipLaunchKernelGGL(gn_partial_kernel<bf16>, g1, dim3(256), 0, s, (const bf16*)x, hw, c, ld, nchunk, ws);
    hipLaunchKernelGGL(gn_finalize_kernel<bf16>, g2, dim3(64), 0, s, (const bf16*)x, hw, c, ld, groups, nchunk, ws,
                       eps, gamma, beta, ab);
  } else {
    hipLaunchKernelGGL(gn_partial_kernel<float>, g1, dim3(256), 0, s, (const float*)x, hw, c, ld, nchunk, ws);
    hipLaunchKernelGGL(gn_finalize_kernel<float>, g2, dim3(64), 0, s, (const float*)x, hw, c, ld, groups, nchunk,
                       ws, eps, gamma, beta, ab);
  }
  return launch_status();
}

extern "C" int rdeic_groupnorm_apply(const void* x, int32_t n, int32_t hw, int32_t c, int32_t ld, const float* ab,
                                     int32_t silu, void* y, int32_t yld, int32_t dtype, void* stream) {
  if (!x || !ab || !y || n <= 0 || hw <= 0 || c <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  long total = (long)n * hw * c;
  int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  if (dtype == 1)
    hipLaunchKernelGGL(gn_apply_kernel<bf16>, dim3(blocks), dim3(256), 0, s, (const bf16*)x, n, hw, c, ld, ab, silu,
                       (bf16*)y, yld);
  else
    hipLaunchKernelGGL(gn_apply_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, n, hw, c, ld, ab, silu,
                       (float*)y, yld);
  return launch_status();
}

extern "C" int rdeic_layernorm(const void* x, int32_t rows, int32_t c, int32_t ld, const float* gamma,
                               const float* beta, float eps, void* y, int32_t yld, int32_t dtype, void* stream) {
  if (!x || !y || !gamma || !beta || rows <= 0 || c <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1)
    hipLaunchKernelGGL(layernorm_kernel<bf16>, dim3(rows), dim3(64), 0, s, (const bf16*)x, rows, c, ld, gamma, beta,
                       eps, (bf16*)y, yld);
  else
    hipLaunchKernelGGL(layernorm_kernel<float>, dim3(rows), dim3(64), 0, s, (const float*)x, rows, c, ld, gamma, beta,
                       eps, (float*)y, yld);
  return launch_status();
}
