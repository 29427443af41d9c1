// Checkerboard Gaussian-conditional entropy-model kernels and the vector-quantiser
// nearest-code search (gfx950).
//
// Checkerboard (utils/ckbd.py:35-115): anchor = (even row, odd col) u (odd row, even col),
// non-anchor = the complement. A stage (slice, phase) touches the [n][c][hy][wy/2]
// "squeezed" lattice: squeezed (r, j) <-> full column 2j + 1 - (r&1) (anchor) or 2j + (r&1).
// Per squeezed element (compressai 1.2.4 GaussianConditional semantics):
//   sigma = max(scale, 0.11); index = L-1 - #{k < L-1 : sigma <= table[k]}   (build_indexes)
//   sym   = int(round_half_even(y - mean))                                     (quantize "symbols")
//   yhat  = sym + mean, scattered back to the full grid                        (ckbd_*_unsequeeze)
// Symbols / indexes land per image in the reference's list order: stage-major, then
// C-order over [c][hy][wy/2] (compress_anchor / compress_nonanchor .reshape(-1).tolist()).
#include "common.h"
#include "../../include/rdeic_hip.h"

// parity-sensitive scalar arithmetic: no fma contraction (matches the reference's separate roundings)
#pragma clang fp contract(off)

namespace {

__device__ __forceinline__ int squeezed_col(int r, int j, int phase) {
  // phase 0 = anchor: even rows take odd cols; phase 1 = non-anchor: even rows take even cols
  return phase == 0 ? 2 * j + 1 - (r & 1) : 2 * j + (r & 1);
}

__device__ __forceinline__ int build_index(float scale, const float* table, int levels, float bound) {
  float s = fmaxf(scale, bound);
  int idx = levels - 1;
  for (int k = 0; k < levels - 1; ++k) idx -= (s <= table[k]) ? 1 : 0;
  return idx;
}

template <typename T>
__global__ void ckbd_encode_kernel(const T* __restrict__ y, int yld, const T* __restrict__ params, int pld, int n,
                                   int hy, int wy, int c, int phase, const float* __restrict__ table, int levels,
                                   float bound, int32_t* __restrict__ sym, int32_t* __restrict__ idx, long img_stride,
                                   long off, T* __restrict__ yhat, int yhld, T* __restrict__ anchor_out, int ald) {
  const int wq = wy / 2;
  long total = (long)n * c * hy * wq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long rem = i;
    int j = (int)(rem % wq); rem /= wq;
    int r = (int)(rem % hy); rem /= hy;
    int ch = (int)(rem % c);
    int img = (int)(rem / c);
    int col = squeezed_col(r, j, phase);
    long pix = ((long)img * hy + r) * wy + col;
    float scale = to_f32(params[pix * pld + ch]);
    float mean = to_f32(params[pix * pld + c + ch]);
    float yv = to_f32(y[pix * yld + ch]);
    int s = (int)rintf(__fsub_rn(yv, mean));
    long o = (long)img * img_stride + off + ((long)ch * hy + r) * wq + j;
    sym[o] = s;
    idx[o] = build_index(scale, table, levels, bound);
    float yh = __fadd_rn((float)s, mean);
    yhat[pix * yhld + ch] = from_f32<T>(yh);
    if (anchor_out) {
      anchor_out[pix * ald + ch] = from_f32<T>(yh);
      long pix2 = ((long)img * hy + r) * wy + squeezed_col(r, j, 1 - phase);
      anchor_out[pix2 * ald + ch] = from_f32<T>(0.f);
    }
  }
}

template <typename T>
__global__ void ckbd_indexes_kernel(const T* __restrict__ params, int pld, int n, int hy, int wy, int c, int phase,
                                    const float* __restrict__ table, int levels, float bound, int32_t* __restrict__ idx,
                                    long img_stride, long off) {
  const int wq = wy / 2;
  long total = (long)n * c * hy * wq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long rem = i;
    int j = (int)(rem % wq); rem /= wq;
    int r = (int)(rem % hy); rem /= hy;
    int ch = (int)(rem % c);
    int img = (int)(rem / c);
    int col = squeezed_col(r, j, phase);
    long pix = ((long)img * hy + r) * wy + col;
    long o = (long)img * img_stride + off + ((long)ch * hy + r) * wq + j;
    idx[o] = build_index(to_f32(params[pix * pld + ch]), table, levels, bound);
  }
}

template <typename T>
__global__ void ckbd_dequant_kernel(const int32_t* __restrict__ sym, const T* __restrict__ params, int pld, int n,
                                    int hy, int wy, int c, int phase, long img_stride, long off, T* __restrict__ yhat,
                                    int yhld, T* __restrict__ anchor_out, int ald) {
  const int wq = wy / 2;
  long total = (long)n * c * hy * wq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long rem = i;
    int j = (int)(rem % wq); rem /= wq;
    int r = (int)(rem % hy); rem /= hy;
    int ch = (int)(rem % c);
    int img = (int)(rem / c);
    int col = squeezed_col(r, j, phase);
    long pix = ((long)img * hy + r) * wy + col;
    long o = (long)img * img_stride + off + ((long)ch * hy + r) * wq + j;
    float mean = to_f32(params[pix * pld + c + ch]);
    float yh = __fadd_rn((float)sym[o], mean);
    yhat[pix * yhld + ch] = from_f32<T>(yh);
    if (anchor_out) {
      anchor_out[pix * ald + ch] = from_f32<T>(yh);
      long pix2 = ((long)img * hy + r) * wy + squeezed_col(r, j, 1 - phase);
      anchor_out[pix2 * ald + ch] = from_f32<T>(0.f);
    }
  }
}

// d[r][j] = (zn[r] + en[j]) - 2 * dot[r][j]  (the reference's fp32 op order), first-min argmin per row.
__global__ __launch_bounds__(256) void vq_argmin_kernel(const float* __restrict__ dot, const float* __restrict__ zn,
                                                        const float* __restrict__ en, int rows, int ncode,
                                                        int32_t* __restrict__ idx) {
  const int r = blockIdx.x;
  const float* dr = dot + (long)r * ncode;
  float best = INFINITY;
  int bi = 0x7fffffff;
  const float z = zn[r];
  for (int j = threadIdx.x; j < ncode; j += 256) {
    float d = __fsub_rn(__fadd_rn(z, en[j]), __fmul_rn(2.0f, dr[j]));
    if (d < best || (d == best && j < bi)) { best = d; bi = j; }
  }
  __shared__ float sb[256];
  __shared__ int si[256];
  sb[threadIdx.x] = best; si[threadIdx.x] = bi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      float ob = sb[threadIdx.x + s]; int oi = si[threadIdx.x + s];
      if (ob < sb[threadIdx.x] || (ob == sb[threadIdx.x] && oi < si[threadIdx.x])) {
        sb[threadIdx.x] = ob; si[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) idx[r] = si[0];
}

template <typename TO>
__global__ void gather_rows_kernel(const float* __restrict__ table, int ldt, const int32_t* __restrict__ idx, int rows,
                                   int dim, TO* __restrict__ out, int ldo) {
  long total = (long)rows * dim;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int r = (int)(i / dim), d = (int)(i - (long)r * dim);
    out[(long)r * ldo + d] = from_f32<TO>(table[(long)idx[r] * ldt + d]);
  }
}

// out[r] = sum_d x[r][d]^2 in fp32, sequential in d (torch.sum(x**2, dim=1) order differs only in rounding)
template <typename T>
__global__ void row_sqnorm_kernel(const T* __restrict__ x, int rows, int dim, int ld, float* __restrict__ out) {
  int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int d = lane; d < dim; d += 64) {
    float v = to_f32(x[(long)r * ld + d]);
    s += v * v;
  }
  s = warp_sum(s);
  if (lane == 0) out[r] = s;
}

inline int grid_for(long total) { return (int)std::max<long>(1, std::min<long>((total + 255) / 256, 16384)); }

}  // namespace

extern "C" int rdeic_ckbd_encode(const void* y, int32_t yld, const void* params, int32_t pld, int32_t n, int32_t hy,
                                 int32_t wy, int32_t c, int32_t phase, const float* scale_table, int32_t levels,
                                 float scale_bound, int32_t* sym, int32_t* idx, int64_t img_stride, int64_t off,
                                 void* yhat, int32_t yhld, void* anchor_out, int32_t ald, int32_t dtype, void* stream) {
  if (!y || !params || !scale_table || !sym || !idx || !yhat || n <= 0 || hy <= 0 || wy <= 0 || (wy & 1) || c <= 0 ||
      (phase != 0 && phase != 1) || levels < 2)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int g = grid_for((long)n * c * hy * (wy / 2));
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_encode_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)y, yld, (const bf16*)params, pld,
                       n, hy, wy, c, phase, scale_table, levels, scale_bound, sym, idx, (long)img_stride, (long)off,
                       (bf16*)yhat, yhld, (bf16*)anchor_out, ald);
  else
    hipLaunchKernelGGL(ckbd_encode_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)y, yld, (const float*)params,
                       pld, n, hy, wy, c, phase, scale_table, levels, scale_bound, sym, idx, (long)img_stride,
                       (long)off, (float*)yhat, yhld, (float*)anchor_out, ald);
  return launch_status();
}

extern "C" int rdeic_ckbd_indexes(const void* params, int32_t pld, int32_t n, int32_t hy, int32_t wy, int32_t c,
                                  int32_t phase, const float* scale_table, int32_t levels, float scale_bound,
                                  int32_t* idx, int64_t img_stride, int64_t off, int32_t dtype, void* stream) {
  if (!params || !scale_table || !idx || n <= 0 || hy <= 0 || wy <= 0 || (wy & 1) || c <= 0 || levels < 2)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int g = grid_for((long)n * c * hy * (wy / 2));
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_indexes_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)params, pld, n, hy, wy, c,
                       phase, scale_table, levels, scale_bound, idx, (long)img_stride, (long)off);
  else
    hipLaunchKernelGGL(ckbd_indexes_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)params, pld, n, hy, wy, c,
                       phase, scale_table, levels, scale_bound, idx, (long)img_stride, (long)off);
  return launch_status();
}

extern "C" int rdeic_ckbd_dequant(const int32_t* sym, const void* params, int32_t pld, int32_t n, int32_t hy,
                                  int32_t wy, int32_t c, int32_t phase, int64_t img_stride, int64_t off, void* yhat,
                                  int32_t yhld, void* anchor_out, int32_t ald, int32_t dtype, void* stream) {
  if (!sym || !params || !yhat || n <= 0 || hy <= 0 || wy <= 0 || (wy & 1) || c <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int g = grid_for((long)n * c * hy * (wy / 2));
  if (dtype == 1)
    hipLaunchKernelGGL(ckbd_dequant_kernel<bf16>, dim3(g), dim3(256), 0, s, sym, (const bf16*)params, pld, n, hy, wy, c,
                       phase, (long)img_stride, (long)off, (bf16*)yhat, yhld, (bf16*)anchor_out, ald);
  else
    hipLaunchKernelGGL(ckbd_dequant_kernel<float>, dim3(g), dim3(256), 0, s, sym, (const float*)params, pld, n, hy, wy,
                       c, phase, (long)img_stride, (long)off, (float*)yhat, yhld, (float*)anchor_out, ald);
  return launch_status();
}

extern "C" int rdeic_vq_argmin(const float* dot, const float* zn, const float* en, int32_t rows, int32_t ncode,
                               int32_t* idx, void* stream) {
  if (!dot || !zn || !en || !idx || rows <= 0 || ncode <= 0) return RDEIC_EINVAL;
  hipLaunchKernelGGL(vq_argmin_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, dot, zn, en, rows, ncode, idx);
  return launch_status();
}

extern "C" int rdeic_gather_rows(const float* table, int32_t ld_table, const int32_t* idx, int32_t rows, int32_t dim,
                                 void* out, int32_t ld_out, int32_t dtype, void* stream) {
  if (!table || !idx || !out || rows <= 0 || dim <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int g = grid_for((long)rows * dim);
  if (dtype == 1)
    hipLaunchKernelGGL(gather_rows_kernel<bf16>, dim3(g), dim3(256), 0, s, table, ld_table, idx, rows, dim, (bf16*)out,
                       ld_out);
  else
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(g), dim3(256), 0, s, table, ld_table, idx, rows, dim,
                       (float*)out, ld_out);
  return launch_status();
}

extern "C" int rdeic_row_sqnorm(const void* x, int32_t rows, int32_t dim, int32_t ld, float* out, int32_t dtype,
                                void* stream) {
  if (!x || !out || rows <= 0 || dim <= 0) return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((rows + 3) / 4);
  if (dtype == 1)
    hipLaunchKernelGGL(row_sqnorm_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)x, rows, dim, ld, out);
  else
    hipLaunchKernelGGL(row_sqnorm_kernel<float>, g, dim3(256), 0, s, (const float*)x, rows, dim, ld, out);
  return launch_status();
}
