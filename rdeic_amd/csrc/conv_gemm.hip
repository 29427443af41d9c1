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
#include "conv_common.h"

namespace rdeic_conv {

int g_conv_path = 2;    // 0: 128-tiles with the fused GroupNorm prologue only, 2 (default): big-tile auto choice
int g_epi_vec = 1;      // LDS-staged vector epilogue (rdeic_set_conv_option(0, v))
int g_swz = 1;          // swizzled 128-B LDS rows where they win (1) / padded 144-B rows everywhere (0) (option 3)
int g_force_tile = -1;  // >= 0: force launch_plain_auto's candidate (rdeic_set_conv_option(4, i)), tuning only
int g_dma = 1;          // LDS-DMA path for cin % 64 == 0 (rdeic_set_conv_option(5, v))
int g_halo = 1;         // 3x3 halo conv: 0 off, 1 for GroupNorm-input convs (default), 2 for every eligible conv
int g_halo8 = 1;        // the 8-row halo conv where it applies (rdeic_set_conv_option(9, v))

namespace {

// GNP: compile the GroupNorm+SiLU gather prologue in (false = plain gather, fewer VGPRs / VALU).
template <typename T, int BM, int BN, int WGM, int WGN, bool VEC, bool GNP = true, bool SWZ = true>
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
    hipLaunchKernelGGL((conv_kernel<bf16, BM, BN, WGM, WGN, true, false, false>), grid, dim3(WGM * WGN * 64),
                       lds0, s, a);
    return launch_status();
  }
  size_t lds = conv_lds_bytes<bf16, BM, BN>();
  hipLaunchKernelGGL((conv_kernel<bf16, BM, BN, WGM, WGN, true, false>), grid, dim3(WGM * WGN * 64), lds, s, a);
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

}  // namespace

// descriptor -> kernel arguments (validation shared by rdeic_conv2d / rdeic_conv2d_splitk)
int make_args(const rdeic_conv_desc* d, ConvArgs& a, bool& vec) {
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
}  // namespace rdeic_conv

using namespace rdeic_conv;

static int conv2d_run(const rdeic_conv_desc* d, void* stream, bool* fused) {
  ConvArgs a;
  bool vec = false;
  const int rc = make_args(d, a, vec);
  if (rc != RDEIC_OK) return rc;
  float* const part = a.gn_part;
  a.gn_part = nullptr;  // statistics fuse into the LDS-DMA (dma_grouped reads d) and big-tile register paths
  hipStream_t s = (hipStream_t)stream;
  {  // the VAE edge convs (conv_edge.hip): conv_in (8 input channels), norm -> SiLU -> conv to <= 16 channels
    ConvArgs e = a;
    e.gn_part = part;
    const int rc2 = launch_edge(d, e, s, fused);
    if (rc2 != -1) return rc2;
  }
  if (d->out_mode == 2) {  // fused GEGLU exists in the LDS-DMA kernel's vector epilogue only
    const int rc2 = vec ? dma_grouped(d, -1, s) : -1;
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
      const int rc2 = dma_grouped(d, -1, s, fused);
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
  if (vec) {  // the VAE edge convs take their shapes whatever the table's tile
    const int rc2 = launch_edge(d, a, (hipStream_t)stream, fused);
    if (rc2 != -1) return rc2;
  }
  if (d->out_mode == 2) {
    const int rc2 = vec ? dma_grouped(d, tile >= 20 ? tile : -1, (hipStream_t)stream) : -1;
    return rc2 == -1 ? RDEIC_EINVAL : rc2;
  }
  if (d->dtype == 1 && vec && !d->gn_ab && d->cout > 32 && g_conv_path != 0) {
    if (tile >= 20) {
      const int rc2 = dma_grouped(d, tile, (hipStream_t)stream, fused);
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
                              void* stream) {
  ConvArgs a;
  bool vec = false;
  const int rc = make_args(d, a, vec);
  if (rc != RDEIC_OK) return rc;
  if (!vec || d->gn_ab || d->out_mode != 0 || a.batch != 1 || d->cout % 8 || splits < 2 || !ws ||
      (d->out_ld % 8) || ((uintptr_t)d->out % 16) || ((uintptr_t)ws % 16))
    return RDEIC_EINVAL;
  if (ws_floats < (size_t)splits * a.M * a.cout) return RDEIC_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  float* const part = ws;
  if (d->dtype == 0) {  // fp32: 64x64 register-staged partial tiles, fp32 output from the reduction
    ConvArgs p = a;
    p.bias = nullptr; p.emb = nullptr; p.act = 0; p.res = nullptr; p.gn_part = nullptr; p.ln_rows = nullptr;
    p.out = (char*)part; p.out_ld = a.cout; p.out_f32 = 0;
    p.splits = splits;
    p.kper = (a.nk + splits - 1) / splits;
    dim3 grid(cdiv(a.M, 64), cdiv(a.cout, 64), splits);
    constexpr int lds = conv_lds_bytes<float, 64, 64>();
    hipLaunchKernelGGL((conv_kernel<float, 64, 64, 2, 2, true, false, true>), grid, dim3(256), lds, s, p);
    a.splits = splits;
    a.out_f32 = 1;  // the reduction's output (and residual) type: fp32
    const long chunks = (long)a.M * (a.cout / 8);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, a,
                       (const float*)part);
    return launch_status();
  }
  // LDS-DMA partial launch, then the reduce kernel. (r05: the reduction folded into the producer's last split
  // per tile measured -11% on the bench and -25% on the fine-tune step, one block per output tile reducing
  // instead of the reduce kernel's hundreds; removed in r06)
  if (g_dma) {
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
  hipLaunchKernelGGL((conv_kernel<bf16, 128, 128, 2, 2, true, false, true>), grid, dim3(256), lds, s, p);
  a.splits = splits;
  const long chunks = (long)a.M * (a.cout / 8);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, a,
                     (const float*)part);
  return launch_status();
}

extern "C" int rdeic_conv2d(const rdeic_conv_desc* d, void* stream) { return conv2d_impl(d, -2, stream); }

extern "C" int rdeic_conv2d_tile(const rdeic_conv_desc* d, int32_t tile, void* stream) {
  return conv2d_impl(d, tile, stream);
}

extern "C" int rdeic_conv2d_splitk(const rdeic_conv_desc* d, int32_t splits, float* ws, size_t ws_floats,
                                   void* stream) {
  if (d && d->gn_part && (d->gn_hw <= 0 || d->gn_hw % 64 || (long)d->n * d->ho * d->wo % d->gn_hw))
    return RDEIC_EINVAL;
  int rc;
  {
    rdeic_prof_add_bytes(conv_bytes(d));
    ProfScope ps((hipStream_t)stream, RDEIC_PROF_CONV, conv_flops(d));
    rc = conv2d_splitk_impl(d, splits, ws, ws_floats, stream);
  }
  if (rc == RDEIC_OK) rdeic_count_launch(RDEIC_COUNT_SPLITK);
  if (rc != RDEIC_OK || !d->gn_part) return rc;  // statistics of the reduced output: stand-alone pass
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
  if (key == 3) { int prev = g_swz; g_swz = value; return prev; }
  if (key == 4) { int prev = g_force_tile; g_force_tile = value; return prev; }
  if (key == 5) { int prev = g_dma; g_dma = value; return prev; }
  if (key == 6) { int prev = g_halo; g_halo = value; return prev; }
  if (key == 8) { int prev = rdeic_g_attn512; rdeic_g_attn512 = value; return prev; }
  if (key == 9) { int prev = g_halo8; g_halo8 = value; return prev; }
  if (key == 10) { int prev = g_edge; g_edge = value; return prev; }
  return RDEIC_EINVAL;
}
