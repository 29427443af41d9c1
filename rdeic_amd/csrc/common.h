// Shared device helpers for the RDEIC MI355X (gfx950) kernels.
//
// Layout conventions used by every kernel in this library:
//   * activations are NHWC ("pixel-major, channel-contiguous"); a tensor is
//     addressed as base + pixel * ld + channel, where ld >= C lets a kernel
//     read or write a channel slice of a wider buffer (this is how the
//     reference's torch.cat / channel slicing is expressed without copies);
//   * conv / linear weights are packed once at load time as [Cout][KH][KW][Cin]
//     (K-contiguous), so both GEMM operands of the implicit-GEMM conv are
//     K-major and feed MFMA fragments with 16-byte loads;
//   * "dtype" 0 = fp32 parity mode, 1 = bf16 perf mode (fp32 accumulate).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RDEIC_OK 0
#define RDEIC_EINVAL (-22)
#define RDEIC_ENOSPC (-28)
#define RDEIC_EBADMSG (-74)
#define RDEIC_ELAUNCH (-5)

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
// exact-erf GELU (torch.nn.GELU / F.gelu default)
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// GELU with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 on erf): one rcp and one exp instead
// of the library erff's range split. For bf16 outputs only (the fused GEGLU projection epilogue);
// fp32 parity paths keep gelu_f.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, z, 1.0f));
  float p = __builtin_fmaf(1.061405429f, t, -1.453152027f);
  p = __builtin_fmaf(p, t, 1.421413741f);
  p = __builtin_fmaf(p, t, -0.284496736f);
  p = __builtin_fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = 1.0f - p * __expf(-z * z);  // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + copysignf(e, x));
}

// Two values at a time on the packed-f32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth of
// work per issue). For epilogues, which run with no MFMA in flight; beside MFMAs packed f32 is an anti-lever
// (MI355X_MICROARCH.md, constants table).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
// gelu_fast on a pair: the same A&S 7.1.26 erf, the polynomial and the affine steps packed, the rcp / exp scalar
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2 d = pk_fma(z, f32x2{0.3275911f, 0.3275911f}, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = pk_fma(f32x2{1.061405429f, 1.061405429f}, t, f32x2{-1.453152027f, -1.453152027f});
  p = pk_fma(p, t, f32x2{1.421413741f, 1.421413741f});
  p = pk_fma(p, t, f32x2{-0.284496736f, -0.284496736f});
  p = pk_fma(p, t, f32x2{0.254829592f, 0.254829592f});
  p *= t;
  const f32x2 a = z * z * -1.4426950408889634f;  // exp(-z^2) = exp2(-z^2 log2 e)
  const f32x2 ex = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  const f32x2 e = pk_fma(-p, ex, f32x2{1.0f, 1.0f});  // erf(|x| / sqrt 2)
  const f32x2 se = {__builtin_copysignf(e.x, x.x), __builtin_copysignf(e.y, x.y)};
  return (x * 0.5f) * (se + 1.0f);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? RDEIC_OK : RDEIC_ELAUNCH;
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// GroupNorm statistics of a [rows][c] tensor in the per-row-block partial format of
// rdeic_groupnorm_parts_ab (norm.hip): the conv launcher's fallback when its epilogue cannot fuse them.
int gn_rows_partial(const void* x, long rows, int c, int ld, int hw, float* part, int dtype, hipStream_t s);
