// Fused multi-head attention for gfx950: softmax(Q K^T * scale) V with online softmax.
//
// One workgroup = 4 waves = 64 query rows of one (batch, head); each wave owns 16 rows.
// Per 64-key tile: K tile [key][d] and V^T tile [d][key] are staged in LDS, S = Q K^T and
// O += P V run on MFMA (bf16 16x16x32 with fp32 accumulate, or exact-f32 16x16x4 in
// parity mode); the softmax runs in fp32 with a running max / sum per row (flash style),
// so the L x L score matrix is never materialised.
//
// The reference computes sim = einsum(q, k) * scale in fp32, softmax(dim=-1), then
// einsum(sim, v) (ldm/modules/attention.py:171-203); heads are read/written in place from
// the 'b n (h d)' projection layout, so no rearrange copies are needed.
//
// Head dims 16 / 32 / 64 (UNet base: 64, control branch: 16) use this kernel. The VAE's
// single-head d=512 AttnBlock (model.py:181-205) uses the materialised path
// (batched GEMM via rdeic_conv2d + rdeic_softmax_rows + GEMM), see rdeic_amd/ops.py.
#include "common.h"
#include "../../include/rdeic_hip.h"

namespace {

constexpr int QT = 64;   // query rows per block
constexpr int KT = 64;   // keys per tile

template <typename T> struct AT;
template <> struct AT<bf16> { static constexpr int KS = 32; };  // mfma k per instruction
template <> struct AT<float> { static constexpr int KS = 4; };

template <typename T, int DH>
__global__ __launch_bounds__(256) void attn_kernel(const T* __restrict__ q, int ldq, const T* __restrict__ k, int ldk,
                                                   const T* __restrict__ v, int ldv, T* __restrict__ o, int ldo,
                                                   int heads, int lq, int lk, float scale_log2, int kv_bcast) {
  constexpr int KS = AT<T>::KS;
  constexpr int DP = (DH < KS) ? KS : DH;           // padded head dim for the QK^T contraction
  constexpr int PADE = 16 / sizeof(T);
  constexpr int KROW = DP + PADE;                    // K tile row stride (elements)
  constexpr int VROW = KT + PADE;                    // V^T tile row stride
  constexpr int PROW = KT + PADE;                    // P tile row stride
  constexpr int NSUB = DP / KS;                      // MFMAs per 16x16 S tile
  constexpr int NDT = DH / 16;                       // O tiles per wave (d direction)
  constexpr int PSUB = KT / KS;                      // MFMAs per PV tile

  __shared__ __attribute__((aligned(16))) T Ks[KT * KROW];
  __shared__ __attribute__((aligned(16))) T Vt[DH * VROW];
  __shared__ __attribute__((aligned(16))) T Ps[4 * 16 * PROW];

  const int bh = blockIdx.y;
  const int b = bh / heads, h = bh - b * heads;
  const int q0 = blockIdx.x * QT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;

  const T* qb = q + (long)b * lq * ldq + h * DH;
  const long kvb = kv_bcast ? 0 : b;  // a single K/V batch (shared text context) serves every image
  const T* kb = k + kvb * lk * ldk + h * DH;
  const T* vb = v + kvb * lk * ldv + h * DH;

  // Q fragments in registers: lane holds Q[q0 + 16*wave + lr][s*KS + (bf16: 8*lg..+8 | f32: lg)]
  const int myq = q0 + wave * 16 + lr;
  typedef typename std::conditional<sizeof(T) == 2, bf16x8, float>::type frag_t;
  frag_t qf[NSUB];
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    if constexpr (sizeof(T) == 2) {
      bf16x8 z;
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = (bf16)0.f;
      int d0 = s * KS + 8 * lg;
      if (myq < lq && d0 < DH) z = *reinterpret_cast<const bf16x8*>(qb + (long)myq * ldq + d0);
      qf[s] = z;
    } else {
      int d0 = s * KS + lg;
      qf[s] = (myq < lq && d0 < DH) ? qb[(long)myq * ldq + d0] : 0.f;
    }
  }

  f32x4 oacc[NDT];
#pragma unroll
  for (int u = 0; u < NDT; ++u) oacc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_part[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m_run[i] = -INFINITY; l_part[i] = 0.f; }

  const int ntiles = (lk + KT - 1) / KT;
  constexpr int EPC = 16 / sizeof(T);
  constexpr int CPR = DH / EPC;                      // 16-byte chunks per K/V row
  for (int kt = 0; kt < ntiles; ++kt) {
    const int key0 = kt * KT;
    __syncthreads();
    // ---- stage K tile (row-major, zero-padded to DP) and V^T tile
    for (int cidx = tid; cidx < KT * CPR; cidx += 256) {
      int kr = cidx / CPR, ch = cidx - kr * CPR;
      int key = key0 + kr;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (key < lk) {
        kv = *reinterpret_cast<const uint4*>(kb + (long)key * ldk + ch * EPC);
        vv = *reinterpret_cast<const uint4*>(vb + (long)key * ldv + ch * EPC);
      }
      *reinterpret_cast<uint4*>(&Ks[kr * KROW + ch * EPC]) = kv;
      const T* ve = reinterpret_cast<const T*>(&vv);
#pragma unroll
      for (int e = 0; e < EPC; ++e) Vt[(ch * EPC + e) * VROW + kr] = ve[e];
    }
    if constexpr (DP > DH) {
      for (int idx = tid; idx < KT * (DP - DH); idx += 256) {
        int kr = idx / (DP - DH), dd = DH + idx % (DP - DH);
        Ks[kr * KROW + dd] = from_f32<T>(0.f);
      }
    }
    __syncthreads();

    // ---- S = Q K^T  (4 key sub-tiles of 16)
    f32x4 sacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        if constexpr (sizeof(T) == 2) {
          bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Ks[(16 * t + lr) * KROW + s * KS + 8 * lg]);
          sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], kf, sacc[t], 0, 0, 0);
        } else {
          float kf = Ks[(16 * t + lr) * KROW + s * KS + lg];
          sacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[s], kf, sacc[t], 0, 0, 0);
        }
      }
    }
    // ---- online softmax; lane holds S[row 4*lg+i][key 16t+lr]
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float sv = (key0 + 16 * t + lr < lk) ? sacc[t][i] * scale_log2 : -INFINITY;
        sacc[t][i] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      float mnew = fmaxf(m_run[i], mx);
      alpha[i] = exp2f(m_run[i] - mnew);
      m_run[i] = mnew;
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float p = exp2f(sacc[t][i] - mnew);
        ps += p;
        Ps[(wave * 16 + 4 * lg + i) * PROW + 16 * t + lr] = from_f32<T>(p);
      }
      l_part[i] = l_part[i] * alpha[i] + ps;
    }
#pragma unroll
    for (int u = 0; u < NDT; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) oacc[u][i] *= alpha[i];
    __syncthreads();
    // ---- O += P V
#pragma unroll
    for (int s = 0; s < PSUB; ++s) {
      frag_t pf;
      if constexpr (sizeof(T) == 2)
        pf = *reinterpret_cast<const bf16x8*>(&Ps[(wave * 16 + lr) * PROW + s * KS + 8 * lg]);
      else
        pf = Ps[(wave * 16 + lr) * PROW + s * KS + lg];
#pragma unroll
      for (int u = 0; u < NDT; ++u) {
        if constexpr (sizeof(T) == 2) {
          bf16x8 vf = *reinterpret_cast<const bf16x8*>(&Vt[(16 * u + lr) * VROW + s * KS + 8 * lg]);
          oacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, oacc[u], 0, 0, 0);
        } else {
          float vf = Vt[(16 * u + lr) * VROW + s * KS + lg];
          oacc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(pf, vf, oacc[u], 0, 0, 0);
        }
      }
    }
  }
  // ---- finalize: row sums across the 16 lanes of the row group
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float l = l_part[i];
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) l += __shfl_xor(l, off, 64);
    float inv = 1.f / l;
    int qrow = q0 + wave * 16 + 4 * lg + i;
    if (qrow < lq) {
      T* orow = o + ((long)b * lq + qrow) * ldo + h * DH;
#pragma unroll
      for (int u = 0; u < NDT; ++u) orow[16 * u + lr] = from_f32<T>(oacc[u][i] * inv);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ s, long rows, int cols, float scale,
                                                           T* __restrict__ p) {
  long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* sr = s + row * cols;
  float mx = -INFINITY;
  for (int j = lane; j < cols; j += 64) mx = fmaxf(mx, sr[j] * scale);
  mx = warp_max(mx);
  float sum = 0.f;
  for (int j = lane; j < cols; j += 64) sum += __expf(sr[j] * scale - mx);
  sum = warp_sum(sum);
  float inv = 1.f / sum;
  T* pr = p + row * cols;
  for (int j = lane; j < cols; j += 64) pr[j] = from_f32<T>(__expf(sr[j] * scale - mx) * inv);
}

template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ in, int rows, int cols, int ldin,
                                                        T* __restrict__ out, int ldout, long in_bs, long out_bs) {
  __shared__ T tile[32][33];
  const T* ib = in + blockIdx.z * in_bs;
  T* ob = out + blockIdx.z * out_bs;
  int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int yy = ty; yy < 32; yy += 8) {
    int r = r0 + yy, c = c0 + tx;
    if (r < rows && c < cols) tile[yy][tx] = ib[(long)r * ldin + c];
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    int c = c0 + yy, r = r0 + tx;
    if (r < rows && c < cols) ob[(long)c * ldout + r] = tile[tx][yy];
  }
}

template <typename T>
int launch_attn(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo, int batch,
                int heads, int lq, int lk, int dh, float scale, int kv_bcast, hipStream_t s) {
  dim3 grid((lq + QT - 1) / QT, batch * heads);
  float sl2 = scale * 1.4426950408889634f;
#define ATTN_CASE(D)                                                                                              \
  case D:                                                                                                         \
    hipLaunchKernelGGL((attn_kernel<T, D>), grid, dim3(256), 0, s, (const T*)q, ldq, (const T*)k, ldk, (const T*)v, \
                       ldv, (T*)o, ldo, heads, lq, lk, sl2, kv_bcast);                                                      \
    break;
  switch (dh) {
    ATTN_CASE(16)
    ATTN_CASE(32)
    ATTN_CASE(64)
    default: return RDEIC_EINVAL;
  }
#undef ATTN_CASE
  return launch_status();
}

}  // namespace

extern "C" int rdeic_attention(const void* q, int32_t ldq, const void* k, int32_t ldk, const void* v, int32_t ldv,
                               void* o, int32_t ldo, int32_t batch, int32_t heads, int32_t lq, int32_t lk, int32_t dh,
                               float scale, int32_t kv_bcast, int32_t dtype, void* stream) {
  if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || lq <= 0 || lk <= 0) return RDEIC_EINVAL;
  const int epc = dtype == 1 ? 8 : 4;
  if (ldq % epc || ldk % epc || ldv % epc || ((uintptr_t)k) % 16 || ((uintptr_t)v) % 16 || ((uintptr_t)q) % 16)
    return RDEIC_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) return launch_attn<bf16>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, dh, scale, kv_bcast, s);
  return launch_attn<float>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, dh, scale, kv_bcast, s);
}

extern "C" int rdeic_softmax_rows(const float* s, int64_t rows, int32_t cols, float scale, void* p, int32_t dtype,
                                  void* stream) {
  if (!s || !p || rows <= 0 || cols <= 0) return RDEIC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_rows_kernel<bf16>, grid, dim3(256), 0, st, s, (long)rows, cols, scale, (bf16*)p);
  else
    hipLaunchKernelGGL(softmax_rows_kernel<float>, grid, dim3(256), 0, st, s, (long)rows, cols, scale, (float*)p);
  return launch_status();
}

extern "C" int rdeic_transpose(const void* in, int32_t rows, int32_t cols, int32_t ldin, void* out, int32_t ldout,
                               int32_t batch, int64_t in_bs, int64_t out_bs, int32_t dtype, void* stream) {
  if (!in || !out || rows <= 0 || cols <= 0 || batch <= 0) return RDEIC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((cols + 31) / 32, (rows + 31) / 32, batch);
  if (dtype == 1)
    hipLaunchKernelGGL(transpose_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)in, rows, cols, ldin, (bf16*)out,
                       ldout, (long)in_bs, (long)out_bs);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, st, (const float*)in, rows, cols, ldin,
                       (float*)out, ldout, (long)in_bs, (long)out_bs);
  return launch_status();
}
