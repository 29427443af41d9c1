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
// Replaces: the ATen conv / linear calls of every 64-channel-aligned layer (include/rdeic_hip.h).
// ============================================================================================
#include "conv_common.h"

namespace rdeic_conv {

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

// 64-deep k-tiles: 128-byte LDS rows, two 16x16x32 MFMA k-steps per tile.
// GEG: the fused-GEGLU instantiation (out_mode 2, epilogue_geglu); the others compile epilogue_vec only, so the
// GEGLU epilogue's registers never count against the plain tiles
template <int BM, int BN, int WGM, int WGN, int S, int EP, bool GEG = false>
__device__ __forceinline__ void conv_dma_body(ConvArgs a, int tiles_n, unsigned bytes0, unsigned bytes1,
                                              unsigned bytesw) {
  constexpr int KB = 64;
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

  int kt_begin = 0, kt_end = a.nk;
  if (a.splits > 1) {  // split-K: blockIdx.z = k-range, raw fp32 partial sums into slab z
    const int z = blockIdx.z;
    kt_begin = min(a.nk, z * a.kper);
    kt_end = min(a.nk, kt_begin + a.kper);
    a.out += (long)z * a.M * a.out_ld * 4;
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
  const int ce = sl ^ (((g >> 1) & 1) << 2);  // logical chunk of this lane's slot (rows with bit 3 = 0)
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
    const int ch = ce ^ (((wave * BI + j) & 1) << 1);
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
      const int ch = ce ^ (((wave * AI + j) & 1) << 1);
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
  const int rkey = dma_key(lrow);
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
  if constexpr (TM % EP == 0 && (BM / EP) * (BN + 4) * 4 <= S * STAGE) {
    if ((a.epi_vec || a.out_mode == 2) && epi_vec_ok(a)) {
      if constexpr (GEG) epilogue_geglu<BM, BN, WGM, WGN, NT, EP>(acc, a, m0, n0, wm, wn, lane, tid, lds);
      else epilogue_vec<BM, BN, WGM, WGN, NT, EP>(acc, a, m0, n0, wm, wn, lane, tid, lds);
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
template <int BM, int BN, int WGM, int WGN, int S, int EP, bool GEG = false>
__global__ __launch_bounds__(WGM * WGN * 64) void conv_dma_kernel(ConvArgs a, int tiles_n, unsigned bytes0,
                                                                  unsigned bytes1, unsigned bytesw) {
  conv_dma_body<BM, BN, WGM, WGN, S, EP, GEG>(a, tiles_n, bytes0, bytes1, bytesw);
}

template <int BM, int BN, int WGM, int WGN, int S, int EP, bool GEG = false>
__global__ __launch_bounds__(WGM * WGN * 64) __attribute__((amdgpu_num_sgpr(80))) void conv_dma_kernel_2pc(
    ConvArgs a, int tiles_n, unsigned bytes0, unsigned bytes1, unsigned bytesw) {
  conv_dma_body<BM, BN, WGM, WGN, S, EP, GEG>(a, tiles_n, bytes0, bytes1, bytesw);
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

namespace {
// Whether the kernel's vector epilogue runs for these arguments (the compile-time part mirrors the
// `if constexpr` in conv_dma_body).
template <int BM, int BN, int WGM, int WGN, int S, int EP>
bool dma_vec_epilogue(const ConvArgs& a) {
  constexpr int TM = BM / WGM / 16;
  constexpr bool fits = TM % EP == 0 && (BM / EP) * (BN + 4) * 4 <= S * (BM + BN) * 128;
  return fits && (a.epi_vec || a.out_mode == 2) && epi_vec_ok(a);
}

// gn_hw: pixels per image of the GroupNorm the statistics feed; the 64-row partial blocks must not
// straddle two images, and the epilogue must be the vector one with a statistics-capable tile.
template <int BM, int BN, int WGM, int WGN, int S, int EP>
int launch_dma(ConvArgs a, unsigned b0, unsigned b1, unsigned bw, hipStream_t s, int gn_hw, bool* fused) {
  if (a.gn_part) {
    const bool ok = a.splits <= 1 && a.batch == 1 && a.out_mode == 0 && gn_hw > 0 && gn_hw % 64 == 0 &&
                    stats_tile_ok<BM, BN, WGM, WGM * WGN * 64, EP>() && dma_vec_epilogue<BM, BN, WGM, WGN, S, EP>(a);
    if (!ok) a.gn_part = nullptr;
    if (fused) *fused = ok;
  }
  const int tn = cdiv(a.cout, BN);
  const long tiles = (long)cdiv(a.M, BM) * tn;
  dim3 grid((unsigned)tiles, 1, a.splits > 1 ? a.splits : a.batch);
  constexpr int lds = S * (BM + BN) * 128;
  // fused GEGLU with 16-byte chunk-pair stores (epilogue_geglu) where the vector epilogue runs
  const bool geg = a.out_mode == 2 && a.cout % 16 == 0 && a.out_ld % 8 == 0 && ((uintptr_t)a.out % 16) == 0 &&
                   dma_vec_epilogue<BM, BN, WGM, WGN, S, EP>(a);
  if constexpr (WGM * WGN == 16 && lds <= 80 * 1024) {
    // (no GEGLU instantiation here: its 76 VGPRs would leave one block per CU where the plain kernel's 63 fit two,
    // 217 -> 298 us on the 320-channel GEGLU, profiles/r06_geglu_lin_bench.txt)
    hipLaunchKernelGGL((conv_dma_kernel_2pc<BM, BN, WGM, WGN, S, EP>), grid, dim3(WGM * WGN * 64), lds, s, a, tn, b0,
                       b1, bw);
  } else {
    if (geg)
      hipLaunchKernelGGL((conv_dma_kernel<BM, BN, WGM, WGN, S, EP, true>), grid, dim3(WGM * WGN * 64), lds, s, a, tn,
                         b0, b1, bw);
    else
      hipLaunchKernelGGL((conv_dma_kernel<BM, BN, WGM, WGN, S, EP>), grid, dim3(WGM * WGN * 64), lds, s, a, tn, b0, b1,
                         bw);
  }
  return launch_status();
}
}  // namespace

// DMA tiles (ids 21..38; BMxBN/waves, S = ring depth):
//   21 256x128/8 S3, 22 128x256/8 S3, 23 128x128/4 S3, 24 128x128/4 S2,
//   25 128x128/8 S2, 26 64x128/4 S3, 27 128x128/8 S3, 28 256x128/8 S2, 29 128x256/8 S2,
//   30 64x128/4 S2, 31 128x64/4 S2, 32 256x256/16 S2, 33 256x128/16 S2, 34 128x128/16 S2,
//   35 512x128/16 S2 (64x64 per wave at cout = 128: the whole 160 KB of LDS, one block per CU),
//   36 64x128/8 S2 (32x32 per wave: twice the waves of tile 30 on grids of ~256 tiles),
//   37 128x160/4 S2 and 38 64x160/4 S2 (N = 320 layers: two N tiles, no padded columns)
// Removed after measurement (r06, git history and DESIGN.md keep the records): 20 256x256/8 (spilled 528 B per lane,
// never chosen), 39 256x128/8 with 32-deep k-tiles (r05: equal on the GEGLU, 3-20% slower elsewhere).
// (r05: 128x320/8 S2 equal to tile 37 on the N = 320 3x3 convs, slower on the 1280-channel levels; 256x256/16 S4
//  with 32-deep k-tiles 2-5% slower than tile 32; r04: 16-wave S3 / S4 rings slower on every transformer linear)
// Measured (tools/dma_bench.py, one MI355X): 32 is best where a 256x256 grid fills the chip
// without padding waste (1.19-1.27 PF on the VAE 512-channel layers), 25 on the rest with >= 256
// 128x128 tiles, the 4-wave 64x128 tile when even that grid cannot fill the chip; 34 often wins
// on short-K linears (the committed per-shape table rdeic_amd/conv_tiles.json picks, measured by
// tools/tune_tiles.py; shapes missing from it use this heuristic).
int launch_dma_auto(const ConvArgs& a, unsigned b0, unsigned b1, unsigned bw, hipStream_t s, int tile, int gn_hw,
                    bool* fused) {
  if (tile < 21 || tile > 38) {
    const long zb = a.splits > 1 ? a.splits : a.batch;
    const long t128 = (long)cdiv(a.M, 128) * cdiv(a.cout, 128) * zb;
    const long t256 = (long)cdiv(a.M, 256) * cdiv(a.cout, 256) * zb;
    const float useful256 = (float)a.M * a.cout / ((float)cdiv(a.M, 256) * 256 * cdiv(a.cout, 256) * 256);
    tile = (t256 >= 256 && useful256 >= 0.9f) ? 32 : t128 >= 256 ? 25 : 26;
  }
  switch (tile) {
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
    default: return launch_dma<128, 128, 2, 2, 3, 2>(a, b0, b1, bw, s, gn_hw, fused);  // 23
  }
}

// Images are independent in a conv, so a launch whose buffers exceed the 2 GiB reach of a
// 32-bit buffer offset runs the DMA kernel over groups of images (same per-pixel arithmetic,
// bit-identical). Returns -1 when the DMA path does not apply.
int dma_grouped(const rdeic_conv_desc* d, int tile, hipStream_t s, bool* fused) {
  ConvArgs a;
  bool vec = false;
  if (make_args(d, a, vec) != RDEIC_OK || !vec) return -1;
  unsigned b0, b1, bw;
  if (dma_ok(d, a, b0, b1, bw)) return launch_dma_auto(a, b0, b1, bw, s, tile, d->gn_hw, fused);
  if (d->batch > 1 || d->n <= 1) return -1;
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

}  // namespace rdeic_conv
