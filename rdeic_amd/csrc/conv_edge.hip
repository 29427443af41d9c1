// The VAE's two edge convolutions, written for the HBM roof instead of the MFMA one
// (ldm/modules/diffusionmodules/model.py:556 Encoder.conv_in, :681-683 Decoder norm_out -> swish -> conv_out).
// Both move ~1 GB per launch at 16 x 512^2 and do little arithmetic per byte:
//   * conv_in (3 -> 128 channels, input padded to 8, 3x3): 67 MB in, 1.07 GB of bf16 out (+ the GroupNorm
//     statistics of the output, which feed the first ResnetBlock's norm1): a STORE-bound kernel;
//   * norm_out + swish + conv_out (128 -> 3, fp32 out): 1.07 GB of bf16 in, 50 MB out: a READ-bound kernel
//     whose per-element GroupNorm + SiLU (2 transcendentals) is the VALU floor.
// The im2col tiles they ran on before staged every input element nine times and spent their time in the
// gather (conv_in: 1.6 TB/s) or in a per-block load -> sync -> VALU dot2 loop (conv_out: 1.3 TB/s).
#include "conv_common.h"

namespace rdeic_conv {

namespace {

// ============================================================================================
// conv_in: cin = 8 (3 real channels, zero-padded: rdeic_image_u8_to_nhwc), 3x3, stride 1, pad 1.
// GEMM view M = pixels, N = cout, K = 9 taps x 8 channels = 72, laid out as the LDS-DMA / register tiles'
// two 64-deep k-tiles (four 32-deep MFMA k-steps, the last all zero). An A-fragment lane of
// v_mfma_f32_16x16x32_bf16 holds 8 consecutive k = ONE tap's 8 channels of one pixel: a single 16-byte load
// from the NHWC input (zeros outside the image). B fragments (the packed weight, 32 KB) come straight from L2.
// No LDS staging, no im2col, no address VALU beyond one bounds check per tap. Tile: 128 pixels x 128 channels,
// 8 waves of 64 x 32 (one canonical 64-row GroupNorm block per wave row).
// The MFMA sequence over k is conv_kernel's (k-steps 0..3 in order, zero products included) and the epilogue
// IS epilogue_vec (bias, bf16 rounding, canonical statistics, 16-byte stores), so outputs and statistics are
// bit-identical to the register tile this replaces (test_edge_convs_gpu.py).
// ============================================================================================
constexpr int CI_BM = 128, CI_BN = 128, CI_WGM = 2, CI_WGN = 4, CI_NT = CI_WGM * CI_WGN * 64, CI_P = 4;
constexpr int CI_LDS = (CI_BM / CI_P) * (CI_BN + 4) * 4;  // epilogue_vec's parked pass (17 KB)

__global__ __launch_bounds__(CI_NT) void conv_in8_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int TM = CI_BM / CI_WGM / 16, TN = CI_BN / CI_WGN / 16;  // 4 x 2 fragments per wave
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / CI_WGN, wn = wave - (wave / CI_WGN) * CI_WGN;
  const int tn = (a.cout + CI_BN - 1) / CI_BN;
  const int mt = blockIdx.x / tn, nt = blockIdx.x - mt * tn;
  const int m0 = mt * CI_BM, n0 = nt * CI_BN;
  const int lr = lane & 15, lq = lane >> 4;
  const int hw = a.h * a.w;

  // B fragments of this wave's 32 columns, all four k-steps (k = 32 s + 8 lq)
  bf16x8 bfr[4][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (CI_BN / CI_WGN) + j * 16 + lr;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 v = {};
      if (n < a.cout) v = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.weight) + (long)n * a.wld + 32 * s + 8 * lq);
      bfr[s][j] = v;
    }
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int tap = 4 * s + lq;  // this lane's k-chunk in k-step s; taps >= 9 are the zero tail
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    bf16x8 af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * (CI_BM / CI_WGM) + i * 16 + lr;
      bf16x8 v = {};
      if (tap < 9 && m < a.M) {
        const int img = m / hw, rem = m - img * hw;
        const int iy = rem / a.w + ky - 1, ix = rem - (rem / a.w) * a.w + kx - 1;
        if ((unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w)
          v = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.in0) + ((long)(img * a.h + iy) * a.w + ix) * a.ld0);
      }
      af[i] = v;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[s][j], acc[i][j], 0, 0, 0);
  }
  epilogue_vec<CI_BM, CI_BN, CI_WGM, CI_WGN, CI_NT, CI_P>(acc, a, m0, n0, wm, wn, lane, tid, lds);
}

// ============================================================================================
// norm -> SiLU -> 3x3 conv to a few channels (cout <= 16; the decoder's conv_out 128 -> 3, fp32 output).
// A block owns TR x 64 output pixels (16 waves, one output row each). Per 32-channel block of the input, all
// 1024 threads load the (TR + 2) x 66 halo of the RAW input (16 bytes each, coalesced 64-byte pixel slices),
// apply the GroupNorm affine + SiLU ONCE per element in registers (rdeic_groupnorm_apply's formula:
// fma, then x * rcp(1 + e^-x), rounded to bf16) and write it to LDS; then every wave runs the 9 taps as
// 16x16x32 MFMAs with N = 16 (cout real columns, the rest zero weights) reading its A fragments from the halo.
// The transform is 1.16x the element count (halo rows / columns), the MFMA work ~10% of the VALU's, and two
// blocks (76 KB of LDS each) share a CU, so one block's transform runs beside the other's MFMAs and loads.
// k order: 32-channel block major, tap minor (as the halo convs); fp32 accumulation.
// ============================================================================================
constexpr int NR_TR = 16, NR_TC = 64, NR_HR = NR_TR + 2, NR_HC = NR_TC + 2, NR_HPIX = NR_HR * NR_HC;  // 1188
constexpr int NR_NT = 1024, NR_ITEMS = NR_HPIX * 4;  // 16-byte chunks per 32-channel halo (4752)
constexpr int NR_IPT = (NR_ITEMS + NR_NT - 1) / NR_NT;  // 5 per thread
constexpr int NR_LDS = NR_HPIX * 64;                      // 76,032 B of halo, then the (a, b) table
constexpr int NR_AB_MAX = 512;                            // input channels whose table fits
__device__ __forceinline__ int nr_sw(int s) { return ((s >> 2) & 1) << 1; }  // halo conv swizzle (conflict-free)

template <bool SILU>
__global__ __launch_bounds__(NR_NT) void conv3x3_gn_narrow_kernel(ConvArgs a, int tiles_x, int tiles_y) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* const abl = reinterpret_cast<float*>(lds + NR_LDS);  // the image's GroupNorm (a, b) table
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int sp = blockIdx.x;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * NR_TR, ox0 = tx * NR_TC;
  const int H = a.h, W = a.w, cin = a.c0;
  const int lr = lane & 15, lq = lane >> 4;
  const int q = tid & 3;  // this thread's 16-byte chunk of every halo pixel it loads (NR_NT % 4 == 0)
  const bf16* in = reinterpret_cast<const bf16*>(a.in0);
  // LDS-only barrier: __syncthreads() would also wait for the next channel block's loads in flight
  auto bar = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  for (int i = tid; i < cin / 2; i += NR_NT)
    reinterpret_cast<float4*>(abl)[i] = reinterpret_cast<const float4*>(a.gn_ab + (long)img * cin * 2)[i];
  uint4 raw[NR_IPT];
  auto load = [&](int cb) {  // the raw halo chunks of this thread (zeros outside the image)
#pragma unroll
    for (int k = 0; k < NR_IPT; ++k) {
      const int it = tid + k * NR_NT, hp = it >> 2;
      const int hr = hp / NR_HC, hc = hp - (hp / NR_HC) * NR_HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      raw[k] = uint4{0u, 0u, 0u, 0u};
      if (it < NR_ITEMS && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        raw[k] = *reinterpret_cast<const uint4*>(in + ((long)(img * H + iy) * W + ix) * a.ld0 + cb + 8 * q);
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  for (int cb = 0; cb < cin; cb += 32) {
    bar();  // cb = 0: the (a, b) table is in LDS; else the previous block's MFMA reads of the halo are done
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb + 8 * q) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
#pragma unroll
    for (int k = 0; k < NR_IPT; ++k) {
      const int it = tid + k * NR_NT, hp = it >> 2;
      if (it >= NR_ITEMS) continue;
      const int hr = hp / NR_HC, hc = hp - (hp / NR_HC) * NR_HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      bf16x8 o = {};
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {  // outside: the normalised tensor's zero pad
        bf16x8 v;
        *reinterpret_cast<uint4*>(&v) = raw[k];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = __builtin_fmaf((float)v[e], av[e], bv[e]);
          if constexpr (SILU) x *= __builtin_amdgcn_rcpf(1.0f + __expf(-x));
          o[e] = (bf16)x;
        }
      }
      *reinterpret_cast<bf16x8*>(lds + hp * 64 + ((q ^ nr_sw(hp)) << 4)) = o;
    }
    bar();
    if (cb + 32 < cin) load(cb + 32);  // the next block's loads fly under this block's MFMAs
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bfv = {};
      if (lr < a.cout)
        bfv = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(a.weight) + (long)lr * a.wld + t * cin + cb + 8 * lq);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hp = (wave + ky) * NR_HC + i * 16 + lr + kx;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(lds + hp * 64 + ((lq ^ nr_sw(hp)) << 4));
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv, acc[i], 0, 0, 0);
      }
    }
  }
  // lane: output channel lr, pixels ox0 + 16 i + 4 lq + r of row oy0 + wave
  if (lr >= a.cout) return;
  const float bias = a.bias ? a.bias[lr] : 0.f;
  const long row = (long)(img * H + oy0 + wave) * W + ox0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long m = row + i * 16 + lq * 4 + r;
      float v = apply_act(acc[i][r] + bias, a.act, a.act_param);
      if (a.res) v += a.out_f32 ? reinterpret_cast<const float*>(a.res)[m * a.res_ld + lr]
                                : to_f32(reinterpret_cast<const bf16*>(a.res)[m * a.res_ld + lr]);
      if (a.out_f32) reinterpret_cast<float*>(a.out)[m * a.out_ld + lr] = v;
      else reinterpret_cast<bf16*>(a.out)[m * a.out_ld + lr] = from_f32<bf16>(v);
    }
}

}  // namespace

int g_edge = 1;  // the edge kernels where they apply (rdeic_set_conv_option(10, v)): 1 on (default), 0 off

// Returns -1 when neither edge kernel takes the launch.
int launch_edge(const rdeic_conv_desc* d, const ConvArgs& a, hipStream_t s, bool* fused) {
  if (!g_edge || d->dtype != 1 || d->kh != 3 || d->kw != 3 || d->stride != 1 || d->pad_t != 1 || d->pad_l != 1 ||
      d->up2 || d->c1 || d->ho != d->h || d->wo != d->w || a.batch != 1 || d->out_mode != 0 || d->ld0 % 8 ||
      ((uintptr_t)d->in0) % 16 || ((uintptr_t)d->weight) % 16)
    return -1;
  // conv_in: 8 input channels, the vector epilogue (bf16 or fp32 output), statistics per image
  if (d->c0 == 8 && !d->gn_ab && d->wld >= 128 && d->cout >= 64 && epi_vec_ok(a) && a.epi_vec) {
    ConvArgs e = a;
    const bool stats = e.gn_part != nullptr && e.gn_hw > 0 && e.gn_hw % 64 == 0;
    if (!stats) e.gn_part = nullptr;
    if (fused) *fused = stats;
    rdeic_count_launch(RDEIC_COUNT_EDGE);
    const long blocks = (long)cdiv(e.M, CI_BM) * cdiv(e.cout, CI_BN);
    hipLaunchKernelGGL(conv_in8_kernel, dim3((unsigned)blocks), dim3(CI_NT), CI_LDS, s, e);
    return launch_status();
  }
  // norm -> (SiLU) -> conv to <= 16 channels
  if (d->gn_ab && d->cout <= 16 && d->c0 % 32 == 0 && d->c0 <= NR_AB_MAX && d->h % NR_TR == 0 && d->w % NR_TC == 0 &&
      !d->gn_part && !d->emb && ((uintptr_t)d->gn_ab) % 16 == 0) {
    rdeic_count_launch(RDEIC_COUNT_EDGE);
    const int cin_tab = d->c0 * 8;
    const int tx = d->w / NR_TC, ty = d->h / NR_TR;
    const dim3 g((unsigned)((long)d->n * ty * tx));
    if (d->gn_silu) hipLaunchKernelGGL(conv3x3_gn_narrow_kernel<true>, g, dim3(NR_NT), NR_LDS + cin_tab, s, a, tx, ty);
    else hipLaunchKernelGGL(conv3x3_gn_narrow_kernel<false>, g, dim3(NR_NT), NR_LDS + cin_tab, s, a, tx, ty);
    return launch_status();
  }
  return -1;
}

}  // namespace rdeic_conv
