// The GroupNorm-fused 3x3 halo convolutions (VAE ResnetBlock convs, ldm/modules/diffusionmodules/model.py:131-151):
// the 4-row form (two 512-thread blocks per CU) and the 8-row form (one 1024-thread block per CU, the default).
#include "conv_common.h"

namespace rdeic_conv {

// ============================================================================================
// 3x3 / stride-1 / pad-1 conv on a halo strip, with the input GroupNorm affine (+ SiLU) applied
// ONCE per element in LDS: the VAE ResnetBlock's norm -> nonlinearity -> conv
// (ldm/modules/diffusionmodules/model.py:131-151, Normalize + nonlinearity + conv1 / conv2).
//
// The im2col path (conv_dma_kernel) re-stages every input element for each of the 9 taps, so a
// GroupNorm + SiLU fused into its staging costs 9x the VALU of the element-wise pass and loses to
// materialising silu(a x + b) in HBM (one read + one write of the activation). Here a tile is an
// image block of TR x TC = 4 x 64 output pixels x 128 output channels; per 32-channel block the
// (TR + 2) x (TC + 2) halo of the RAW input is DMA'd to LDS once (buffer_load ... lds, 25 x 1 KB
// pieces, zeros outside the image from the descriptor's range check), transformed in place
// (x * a + b, then x * rcp(1 + e^-x): exactly the bf16 values rdeic_groupnorm_apply writes; halo
// pixels outside the image stay zero = the conv's zero padding of the normalised tensor) and then
// read by all 9 taps. The 32-channel weight slice of each tap streams through a 3-deep ring.
// Per step (tap) a wave (one output row, 64 channels) issues 16 v_mfma_f32_16x16x32_bf16.
// LDS 78 KB -> two blocks per CU, so one block's epilogue overlaps the other's main loop.
// Swizzle: 16-byte chunk q of halo pixel / weight row s lives at slot q ^ (((s >> 2) & 1) << 1),
// conflict-free for every ds_read_b128 lane group at any pixel offset (tap shift).
// k order: 32-channel block major, tap minor — fixed per shape (deterministic, batch-invariant),
// not the im2col kernels' (tap, 64-channel) order, so results differ from them by fp32 rounding.
// The epilogue is epilogue_vec (bias / residual / GroupNorm statistics of the output) with the
// tile's 64-pixel wave rows mapped to their image rows.
// ============================================================================================
namespace halo {
constexpr int TR = 4, TC = 64;            // output rows / columns per tile
constexpr int HR = TR + 2, HC = TC + 2;   // halo rows / columns
constexpr int HPIX = HR * HC;             // 396 halo pixels
constexpr int NPIECE = (HPIX * 4 + 63) / 64;  // 1 KB DMA pieces per halo (25)
constexpr int HBYTES = NPIECE * 1024;     // one halo buffer (the last piece's tail slots read zeros)
constexpr int BN = 128, NW = 8, NT = NW * 64;
constexpr int BBYTES = BN * 64;           // one tap's 32-channel weight slice
constexpr int NB = 3;                     // weight ring depth
constexpr int AB_MAX = 512;               // input channels whose GroupNorm affine fits the LDS table
constexpr int LDS = 2 * HBYTES + NB * BBYTES + AB_MAX * 8;
static_assert(LDS <= 80 * 1024, "two blocks per CU");
static_assert((TR * TC / 2) * (BN + 4) * 4 <= LDS, "epilogue parking (two passes)");
__device__ __forceinline__ int sw(int s) { return ((s >> 2) & 1) << 1; }

struct Rows {  // tile row r (wave row r / 64, column r % 64) -> output pixel
  int base, W;
  __device__ __forceinline__ int operator()(int r) const { return base + (r >> 6) * W + (r & 63); }
};

// Epilogue LDS plan (four passes of 64 tile rows: one 16-row fragment per wave row): a parked pass
// (64 x (BN + 4) fp32) and two 16 KB residual buffers. Pass 0's residual is DMA'd during the main loop's
// last taps into the halo buffer the last channel block does not read, so the layout depends on the
// parity of the channel-block count.
constexpr int PK_BYTES = 64 * (BN + 4) * 4;  // 33,792
constexpr int RES_BYTES = 64 * BN * 2;       // 16,384: 64 pixels x 128 bf16
constexpr int RING_END = 2 * HBYTES + NB * BBYTES;
static_assert(HBYTES + PK_BYTES + RES_BYTES <= RING_END, "epilogue plan, even channel blocks");
static_assert(HBYTES + RES_BYTES + PK_BYTES <= RING_END, "epilogue plan, odd channel blocks");
static_assert(RES_BYTES <= HBYTES, "pass-0 residual in the free halo buffer");
__device__ __forceinline__ int res_off(int parity, int p) {  // residual buffer of pass p
  return ((p & 1) == 0) ? (parity ? HBYTES : 0) : (parity ? 0 : HBYTES + PK_BYTES);
}
__device__ __forceinline__ int park_off(int parity) { return parity ? HBYTES + RES_BYTES : HBYTES; }
}  // namespace halo

// Pass 0's residual rows (NW x 8 pixels x 128 channels) by LDS-DMA, issued by the 4-row kernel during its last
// taps: this wave's pieces q = wave, wave + NW; lane i of piece q brings pass row 4q + i / 16 (wave row (4q + i / 16) / 16, pixel
// p * 16 + (4q + i / 16) % 16 of it), channels n0 + 8 (i % 16) .. + 7. Offsets are recomputed at each use
// (not kept live).
template <int NW>
__device__ __forceinline__ void halo_res_dma(__amdgpu_buffer_rsrc_t rsr, char* dst, int base, int W, int res_ld,
                                             int n0, int wave, int lane, int p) {
  int l = lane;
  asm volatile("" : "+v"(l));  // keep the offsets here, not hoisted into the main loop's live set
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int pr = 4 * (wave + NW * k) + (l >> 4);
    const unsigned vo = (unsigned)(base + (pr >> 4) * W + (pr & 15)) * (unsigned)(res_ld * 2) + (unsigned)((l & 15) * 16);
    dma16(rsr, dst + (wave + NW * k) * 1024, vo, p * 16 * res_ld * 2 + n0 * 2);
  }
}

// The halo convs' epilogue for bf16 outputs without emb / activation (every VAE ResnetBlock conv):
// out = (acc + bias) + residual, rounded to bf16, in four passes (one 16-row fragment per wave row, NW x 8
// tile rows). Per pass: the accumulators of fragment row p are parked in LDS (park). Pass 0's residual rows
// are in LDS at r0 (LDS-DMA'd by the caller during its last taps); passes 1-3 buffer-load theirs into
// registers one pass ahead (rbuf), so only LDS-only barriers separate the passes (an LDS-DMA here would make
// the compiler drain vmcnt(0) before the next LDS read; r1 is not used). Each thread keeps the bias of its
// 8 channels in registers and handles 2 chunks (16-byte LDS reads, residual, one 16-byte store each).
// Arithmetic and rounding are epilogue_vec's, so outputs are bit-identical to it. Fused GroupNorm
// statistics (a.gn_part) keep the canonical order: pass p is 16-row group p of every 64-row block (one wave
// row), summed by a column scan of the stored values, and ((g0 + g1) + g2) + g3 at the end.
template <int NW, bool RES>
__device__ __forceinline__ void halo_epilogue(const f32x4 (&acc)[4][4], const ConvArgs& a, int n0, int wm, int wn,
                                              int tid, char* lds, int base, int W, int park, int r0, int r1,
                                              __amdgpu_buffer_rsrc_t rsr, int wave) {
  constexpr int BN = 128, SDW = BN + 4, NT = NW * 64;
  // laundered: every address below is derived after the main loop (hoisted, they would sit in the
  // 128-VGPR main loop's live set and spill)
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int lr = lane & 15, lq = lane >> 4;
  float* const L = reinterpret_cast<float*>(lds + park);
  constexpr bool has_res = RES;  // a.res != nullptr, a compile-time split (no branch around the residual loads,
                                 // whose vmcnt scoreboard the compiler would otherwise merge over both paths)
  const bool st = a.gn_part != nullptr;
  const int cc = tid & 15;  // this thread's 8 channels n0 + 8 cc (NT % 16 == 0: the same in every chunk)
  const int nn = n0 + cc * 8;
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = 0.f;
  if (a.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + nn), b1 = *reinterpret_cast<const float4*>(a.bias + nn + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w; bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  float sg[4], qg[4];
  // LDS-only barriers (__syncthreads() would also drain vmcnt(0): the previous pass's output stores and the
  // next pass's residual loads). The residual of pass 0 is in LDS (r0, LDS-DMA'd by the caller during its
  // last taps); passes 1-3 load theirs into registers one pass ahead (an LDS-DMA here would make the compiler
  // drain vmcnt(0) before the next LDS read, i.e. wait out the prefetch at once).
  auto bar = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  auto res_rows = [&](int p, uint4 (&dst)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = (tid >> 4) + (NT / 16) * k;
      const long m = base + (pr >> 4) * W + p * 16 + (pr & 15);
      // a buffer load through the residual's descriptor (a plain load here compiled to flat_load, which counts
      // in lgkmcnt too, so every LDS barrier would wait for it)
      typedef unsigned u4v __attribute__((ext_vector_type(4)));
      const u4v r = __builtin_amdgcn_raw_buffer_load_b128(rsr, (unsigned)(m * a.res_ld + nn) * 2u, 0, 0);
      dst[k] = uint4{r.x, r.y, r.z, r.w};
    }
  };
  uint4 rbuf[2][2];  // [pass & 1][chunk]: pass p reads rbuf[p & 1], pass p + 1's rows load into the other
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    bar();  // p = 0: the main loop's LDS reads are done; else: the previous pass's readers are
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) L[(wm * 16 + lq * 4 + r) * SDW + wn * 64 + j * 16 + lr] = acc[p][j][r];
    if (has_res && p == 0) wait_vm<0>();  // this wave's pass-0 residual pieces (nothing else is in flight)
    bar();
    // consumed one pass later; pass 0 issues pass 1's after its LDS residual reads (the compiler drains
    // vmcnt(0) before the first read of LDS-DMA'd data)
    if (has_res && p > 0 && p + 1 < 4) res_rows(p + 1, rbuf[(p + 1) & 1]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = (tid >> 4) + (NT / 16) * k;  // pass row: wave row pr / 16, row p * 16 + pr % 16 of it
      const long m = base + (pr >> 4) * W + p * 16 + (pr & 15);
      const float4 x0 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(L + pr * SDW + cc * 8 + 4);
      float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias[e];
      if (has_res) {
        bf16x8 rv;
        if (p == 0) rv = *reinterpret_cast<const bf16x8*>(lds + r0 + pr * 256 + cc * 16);
        else *reinterpret_cast<uint4*>(&rv) = rbuf[p & 1][k];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
      }
      bf16x8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.out) + m * a.out_ld + nn) = ov;
      if (st) {
        *reinterpret_cast<float4*>(L + pr * SDW + cc * 8) = make_float4((float)ov[0], (float)ov[1], (float)ov[2], (float)ov[3]);
        *reinterpret_cast<float4*>(L + pr * SDW + cc * 8 + 4) = make_float4((float)ov[4], (float)ov[5], (float)ov[6], (float)ov[7]);
      }
    }
    if (has_res && p == 0) res_rows(1, rbuf[1]);
    if (st) {  // column scan: thread (wave row b, channel j), the 16 rows of group p, in row order
      bar();
      const int b = tid >> 7, j = tid & 127;
      const float* col = L + (b * 16) * SDW + j;
      float y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) y[r] = col[r * SDW];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s1 += y[r]; s2 = fmaf(y[r], y[r], s2); }
      sg[p] = s1;
      qg[p] = s2;
    }
  }
  if (st) {
    const int b = tid >> 7, j = tid & 127;
    float* pp = a.gn_part + 4 + ((long)((a.gn_row0 + base + b * W) / 64) * a.cout + n0 + j) * 2;
    pp[0] = ((sg[0] + sg[1]) + sg[2]) + sg[3];
    pp[1] = ((qg[0] + qg[1]) + qg[2]) + qg[3];
    if (tid == 0 && base == 0 && n0 == 0) reinterpret_cast<int*>(a.gn_part)[0] = 64;  // rows per partial
  }
}

// GN: 0 plain conv, 1 GroupNorm affine on the input, 2 affine + SiLU (compile-time: no per-element branch);
// FE: the fast epilogue (halo_epilogue: bf16 out, no emb / activation), else epilogue_vec
template <int GN, bool FE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void conv3x3_halo_kernel(ConvArgs a, int tiles_x, int tiles_y, unsigned bytes0,
                                                               unsigned bytesw) {
  using namespace halo;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const hbuf = lds;
  char* const bbuf = lds + 2 * HBYTES;
  float* const abl = reinterpret_cast<float*>(lds + 2 * HBYTES + NB * BBYTES);
  HALO_STAMP(0);
#ifdef RDEIC_HALO_STAMPS
  if (threadIdx.x == 0) {
    g_halo_stamps[(long)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    g_halo_stamps[(long)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  const int tn = a.cout / BN;
  // XCD-aware bijective remap (as conv_dma_body): an XCD owns a contiguous run of tile ids, the N
  // tiles of one image block adjacent (they share its halo through L2)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
  const int nt = wgid % tn;
  int sp = wgid / tn;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * TC, n0 = nt * BN;
  const int H = a.h, W = a.w, cin = a.c0;
  const int ncb = cin >> 5, U = ncb * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wave = (output row, 64-channel half)

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);

  // halo pieces of this wave: w, w + 8, w + 16 and (wave 0) 24; the other waves repeat piece w + 16
  // as their 4th (same bytes to the same slots), so every wave issues 4 and vmcnt stays uniform
  unsigned hvo[4];
  int hpo[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = (wave + 8 * k < NPIECE) ? wave + 8 * k : wave + 16;
    const int sl = p * 16 + (lane >> 2), ph = lane & 3;
    hpo[k] = p * 1024;
    hvo[k] = kOOB;
    if (sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        hvo[k] = (unsigned)((img * H + iy) * W + ix) * (unsigned)(a.ld0 * 2) + (unsigned)((ph ^ sw(sl)) * 16);
    }
  }
  // residual pieces of the epilogue (halo_epilogue): this wave's pieces q = wave, wave + 8 of every pass;
  // lane i of piece q brings pass row 4q + i / 16 (wave row (4q + i / 16) / 16), chunk i % 16
  const bool res_dma = FE && a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res_dma ? a.res : a.in0), (short)0, res_dma ? (int)((long)(img * H + H) * W * a.res_ld * 2) : 0, 0x00020000);
  const int parity = (cin >> 5) & 1;
  // weight rows of this wave: n = 16 wave + lane / 4, chunk lane % 4
  unsigned bvo;
  {
    const int n = wave * 16 + (lane >> 2), ph = lane & 3;
    bvo = (n0 + n < a.cout) ? (unsigned)(n0 + n) * (unsigned)(a.wld * 2) + (unsigned)((ph ^ sw(n)) * 16) : kOOB;
  }
  auto issue_halo = [&](int cb) {
    char* dst = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int k = 0; k < 4; ++k) dma16(rs0, dst + hpo[k], hvo[k], cb * 64);
  };
  auto issue_b = [&](int u) {
    const int cb = u / 9, t = u - (u / 9) * 9;
    dma16(rsw, bbuf + (u % NB) * BBYTES + wave * 1024, bvo, (t * cin + cb * 32) * 2);
  };
  // The in-place GroupNorm (+ SiLU) of a halo: every wave transforms exactly the chunks its own
  // DMA pieces brought in (one 16-byte chunk per lane per piece; the duplicate 4th piece of waves
  // 1..7 is skipped), right after its own counted vmcnt: no barrier between landing and transform.
  // Pixels outside the image (the conv's zero padding of the normalised tensor) stay zero.
  // per piece k: bit k = this lane's chunk is inside the image (transform it), bits 4 + 2k: its
  // logical channel chunk (one VGPR for all four pieces)
  unsigned hinfo = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = (wave + 8 * k < NPIECE) ? wave + 8 * k : -1;
    const int sl = (p < 0 ? 0 : p) * 16 + (lane >> 2);
    if (p >= 0 && hvo[k] != kOOB) hinfo |= 1u << k;
    hinfo |= (unsigned)((lane & 3) ^ sw(sl)) << (4 + 2 * k);
  }
  // piece k of this wave's halo pieces (one 16-byte chunk per lane), transformed in place
  auto transform_piece = [&](int cb, int k) {
    if (!(hinfo & (1u << k))) return;
    char* hb = hbuf + (cb & 1) * HBYTES + lane * 16 + hpo[k];
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(hb);
    const int ch = (hinfo >> (4 + 2 * k)) & 3;
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb * 32 + ch * 8) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];  // (a, b) of the chunk's 8 channels
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = __builtin_fmaf((float)v[e], av[e], bv[e]);
      if constexpr (GN == 2) x *= __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      o[e] = (bf16)x;
    }
    *reinterpret_cast<bf16x8*>(hb) = o;
  };
  auto transform = [&](int cb) {
#pragma unroll
    for (int k = 0; k < 4; ++k) transform_piece(cb, k);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier releases readers
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: the image's GroupNorm (a, b) table (cin x 8 bytes, <= 4 KB) comes by LDS-DMA together with
  // the first halo and weight slices, so their latencies overlap. Each wave issues ONE table piece (waves
  // past the table's pieces repeat piece 0: same bytes to the same slots), keeping vmcnt uniform.
  if constexpr (GN != 0) {
    const int tbytes = cin * 8, tp = wave < (tbytes + 1023) / 1024 ? wave : 0;
    const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.gn_ab + (long)img * cin * 2), (short)0, tbytes, 0x00020000);
    dma16(rst, reinterpret_cast<char*>(abl) + tp * 1024, (unsigned)(tp * 1024 + lane * 16), 0);
  }
  issue_halo(0);
  issue_b(0);
  issue_b(1);
  wait_vm<2>();  // the table piece and this wave's halo pieces
  if constexpr (GN != 0) {
    __syncthreads();  // every wave's table piece has landed
    transform(0);
  }

  HALO_STAMP(1);
  const int lr = lane & 15, lq = lane >> 4;
  const int bsw = (lq ^ sw(lr)) * 16;  // weight rows n = 64 wn + 16 j + lr share sw(lr)
  // A fragment i of a tap reads halo slots s0 + 16 i + lr: adding 16 leaves bits 0..3 (and so the
  // swizzle) unchanged, so one lane address per tap serves all four fragments (immediate offsets)
  // taps unrolled: ring slot (u % 3 = t % 3, 9 taps per block), filter offset, waits and the next
  // loads are compile-time per tap; the only runtime branch is "is there a next channel block"
  for (int cb = 0; cb < ncb; ++cb) {
    const bool more = cb + 1 < ncb;
    const char* hb = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // this tap's weights (and at tap 2 the next halo); younger ops allowed in flight: the next tap's
      // weights and, at tap 1, the next halo's 4 pieces issued at tap 0
      if (t == 1) {
        if (more) wait_vm<5>(); else wait_vm<1>();
      } else if (t < 8 || more) {
        wait_vm<1>();
      } else if (res_dma) {
        wait_vm<2>();  // younger: the epilogue's pass-0 residual pieces (issued at tap 7)
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      if (t + 2 < 9) {
        dma16(rsw, bbuf + ((t + 2) % NB) * BBYTES + wave * 1024, bvo, ((t + 2) * cin + cb * 32) * 2);
      } else if (more) {
        dma16(rsw, bbuf + ((t + 2) % NB) * BBYTES + wave * 1024, bvo, ((t + 2 - 9) * cin + (cb + 1) * 32) * 2);
      }
      if (t == 0 && more) issue_halo(cb + 1);
      if (t == 7 && !more && res_dma)  // pass 0's residual rows into the halo buffer the last block does not read
        halo_res_dma<NW>(rsr, lds + halo::res_off(parity, 0), (img * H + oy0) * W + ox0, W, a.res_ld, n0, wave, lane, 0);
      const char* bb = bbuf + (t % NB) * BBYTES + (wn * 64 + lr) * 64 + bsw;
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bfv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(bb + j * 16 * 64);
      // per-tap lane address, recomputed each tap from a laundered base (the compiler would otherwise
      // hoist all 9 taps' addresses out of the channel-block loop and spill)
      int lb = wm * HC + lr;
      asm volatile("" : "+v"(lb));
      const int sl = lb + ky * HC + kx;
      const char* ab = hb + sl * 64 + ((lq ^ sw(sl)) << 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ab + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
      }
      // the next block's halo (own pieces landed at tap 2's wait) is transformed one piece per tap over
      // taps 2..5, AFTER this tap's MFMAs are issued, so its VALU runs beside the matrix pipe instead of
      // delaying the next barrier; the block reads it from its tap 0 on (several barriers later)
      if constexpr (GN != 0)
        if (t >= 2 && t < 6 && more) {
          transform_piece(cb + 1, t - 2);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier
        }
    }
  }
  HALO_STAMP(2);
  if constexpr (FE) {
    if (a.res)
      halo_epilogue<NW, true>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(parity),
                              res_off(parity, 0), res_off(parity, 1), rsr, wave);
    else
      halo_epilogue<NW, false>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(parity),
                               res_off(parity, 0), res_off(parity, 1), rsr, wave);
  } else {
    epilogue_vec<TR * TC, BN, 4, 2, NT, 2, Rows, false>(acc, a, 0, n0, wm, wn, lane, tid, lds,
                                                        Rows{(img * H + oy0) * W + ox0, W});
  }
  HALO_STAMP(3);
}

// ============================================================================================
// The 8-row halo conv (r04): one 1024-thread block per CU computes 8 x 64 output pixels x 128 channels
// (16 waves: 8 output rows x 2 channel halves of 64, the same 64 x 64 wave tile as conv3x3_halo_kernel).
// Against the 4-row kernel (two 512-thread blocks per CU) it trades the second co-resident block for
// depth: the whole 160 KB of LDS holds a 10 x 66-pixel halo double buffer (1.29 halo pixels per output
// pixel instead of 1.55) and an 8-slot weight ring fed 6 taps ahead (the 4-row kernel's 3-slot ring,
// 2 taps ahead, left the main loop waiting on ~1.1 us LDS-DMA landings, tools/halo_stamps.hip, r04).
// Roles are split so every wave's vmcnt counts only its own stream: waves 0..7 stream the weight slices
// (1 KB = 16 rows each), waves 8..15 the halo pieces (6 each, duplicates for the 42 pieces) and the
// GroupNorm table, and transform the pieces they loaded (affine + SiLU in place). Same MFMA order as
// the 4-row kernel (channel block major, tap minor), so both give bit-identical outputs.
// ============================================================================================
namespace halo8 {
constexpr int TR = 8, TC = 64;
constexpr int HR = TR + 2, HC = TC + 2;            // 10 x 66 halo pixels
constexpr int HPIX = HR * HC;                      // 660
constexpr int NPIECE = (HPIX * 4 + 63) / 64;       // 42 pieces of 1 KB
constexpr int HBYTES = NPIECE * 1024;              // 43,008
constexpr int BN = 128, NW = 16, NT = NW * 64;
constexpr int BBYTES = BN * 64;                    // one tap's 32-channel weight slice
constexpr int NB = 8, LEAD = 6;                    // weight ring: slice u + LEAD issued at tap u
constexpr int PPW = 6;                             // halo pieces per halo wave (8 waves x 6 >= 42)
constexpr int AB_MAX = 512;
constexpr int TABLE = 2 * HBYTES + NB * BBYTES;    // 151,552
constexpr int LDS = TABLE + AB_MAX * 8;            // 155,648
static_assert(LDS <= 160 * 1024, "one block per CU");
static_assert(NB >= LEAD + 1, "a slot is reused only after every wave passed the barrier of its last reader");
// epilogue (halo_epilogue<16>): park 128 rows x 132 fp32, two 32 KB residual pass buffers; pass 0's
// residual lands in the halo buffer the last channel block does not read (index = ncb & 1)
constexpr int PK = 128 * (BN + 4) * 4, RB = 128 * BN * 2;
static_assert(RB <= HBYTES && HBYTES + RB + PK <= LDS && HBYTES + PK + RB <= LDS, "epilogue plan");
__device__ __forceinline__ int res_off(int f, int p) { return ((p & 1) == 0) ? (f ? HBYTES : 0) : (f ? 0 : HBYTES + PK); }
__device__ __forceinline__ int park_off(int f) { return f ? HBYTES + RB : HBYTES; }
__device__ __forceinline__ int sw(int s) { return ((s >> 2) & 1) << 1; }
}  // namespace halo8

template <int GN>
__global__ __launch_bounds__(1024) void conv3x3_halo8_kernel(ConvArgs a, int tiles_x, int tiles_y, unsigned bytes0,
                                                            unsigned bytesw) {
  using namespace halo8;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const hbuf = lds;
  char* const bbuf = lds + 2 * HBYTES;
  float* const abl = reinterpret_cast<float*>(lds + TABLE);
  HALO_STAMP(0);
#ifdef RDEIC_HALO_STAMPS
  if (threadIdx.x == 0) {
    g_halo_stamps[(long)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    g_halo_stamps[(long)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  const int tn = a.cout / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;  // XCD-aware bijective remap (as conv3x3_halo_kernel)
  const int xcd = orig & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
  const int nt = wgid % tn;
  int sp = wgid / tn;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * TC, n0 = nt * BN;
  const int H = a.h, W = a.w, cin = a.c0;
  const int ncb = cin >> 5, U = ncb * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wave = (output row, 64-channel half)
  const bool wload = wave < 8;              // weight-stream wave; else halo-stream wave
  const int hw = wave - 8;

  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)bytes0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)a.weight, (short)0, (int)bytesw, 0x00020000);
  const bool res_dma = a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res_dma ? a.res : a.in0), (short)0, res_dma ? (int)((long)(img * H + H) * W * a.res_ld * 2) : 0, 0x00020000);
  const int f = ncb & 1;  // the halo buffer the last channel block does not read

  // halo waves: pieces hw + 8 k (k < 6; past the 42 pieces, piece hw + 32 again: same bytes, same slots).
  // A piece's source offset (or out-of-image zeros) is recomputed at each issue from a laundered lane id
  // (six live offsets would push the 128-VGPR loop into scratch).
  auto hpiece = [&](int k) { return hw + 8 * k < NPIECE ? hw + 8 * k : hw + 32; };  // wave-uniform
  auto halo_voff = [&](int k, int ln) {
    const int p = hpiece(k);
    const int sl = p * 16 + (ln >> 2), ph = ln & 3;
    unsigned vo = kOOB;
    if (sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        vo = (unsigned)((img * H + iy) * W + ix) * (unsigned)(a.ld0 * 2) + (unsigned)((ph ^ sw(sl)) * 16);
    }
    return vo;
  };
  auto hpo = [&](int k) { return hpiece(k) * 1024; };
  // The GroupNorm transform is balanced over all 16 waves: wave w transforms pieces w + 16 k (k < 3,
  // < 42) whoever loaded them (r04: -3.5% against transforming by the loader). tinfo: per k a valid bit
  // (bit k: a real piece inside the image) and the lane's logical channel chunk (bits 8 + 2k).
  unsigned tinfo = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int p = wave + 16 * k;
    const int sl = p * 16 + (lane >> 2), ph = lane & 3;
    bool in = false;
    if (p < NPIECE && sl < HPIX) {
      const int hr = sl / HC, hc = sl - (sl / HC) * HC;
      const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
      in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    }
    if (in) tinfo |= 1u << k;
    tinfo |= (unsigned)(ph ^ sw(sl)) << (8 + 2 * k);
  }
  // halo waves: all six pieces of block cb (prologue), or half of them (main loop, k in [k0, k1))
  auto issue_halo = [&](int cb, int k0, int k1) {
    char* dst = hbuf + (cb & 1) * HBYTES;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int k = k0; k < k1; ++k) dma16(rs0, dst + hpo(k), halo_voff(k, ln), cb * 64);
  };
  // weight waves: rows n = 16 wave + lane / 4, chunk lane % 4 of every tap slice
  unsigned bvo = kOOB;
  if (wload) {
    const int n = wave * 16 + (lane >> 2), ph = lane & 3;
    bvo = (n0 + n < a.cout) ? (unsigned)(n0 + n) * (unsigned)(a.wld * 2) + (unsigned)((ph ^ sw(n)) * 16) : kOOB;
  }
  auto issue_b = [&](int u) {
    const int cb = u / 9, t = u - (u / 9) * 9;
    dma16(rsw, bbuf + (u % NB) * BBYTES + wave * 1024, bvo, (t * cin + cb * 32) * 2);
  };
  // piece wave + 16 k of block cb, in place (out-of-image chunks stay zero: the conv's padding of the
  // normalised tensor). info and lane are laundered so their derived offsets are recomputed here instead of
  // hoisted out of the channel-block loop, where hipcc kept them in scratch; every reload was an
  // s_waitcnt vmcnt(0) that drained the weight ring's in-flight LDS-DMA (r04)
  auto transform_piece = [&](int cb, int k) {
    unsigned info = tinfo;
    int ln = lane;
    asm volatile("" : "+v"(info), "+v"(ln));
    if (!(info & (1u << k))) return;
    char* pc = hbuf + (cb & 1) * HBYTES + ln * 16 + (wave + 16 * k) * 1024;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(pc);
    const int ch = (info >> (8 + 2 * k)) & 3;
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb * 32 + ch * 8) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = __builtin_fmaf((float)v[e], av[e], bv[e]);
      if constexpr (GN == 2) x *= __builtin_amdgcn_rcpf(1.0f + __expf(-x));
      o[e] = (bf16)x;
    }
    *reinterpret_cast<bf16x8*>(pc) = o;
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: halo waves bring the table (one piece each; waves past its pieces repeat piece 0) and
  // block 0's halo; weight waves the first LEAD slices
  if (wload) {
    const int n0s = U < LEAD ? U : LEAD;
    for (int u = 0; u < n0s; ++u) issue_b(u);
  } else {
    if constexpr (GN != 0) {
      const int tbytes = cin * 8, tp = hw < (tbytes + 1023) / 1024 ? hw : 0;
      const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.gn_ab + (long)img * cin * 2), (short)0, tbytes, 0x00020000);
      dma16(rst, reinterpret_cast<char*>(abl) + tp * 1024, (unsigned)(tp * 1024 + lane * 16), 0);
    }
    issue_halo(0, 0, PPW);
    wait_vm<0>();
  }
  if constexpr (GN != 0) {
    __syncthreads();  // every table piece and every halo piece of block 0 has landed
#pragma unroll 1
    for (int k = 0; k < 3; ++k) transform_piece(0, k);  // one piece at a time (register budget)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier releases readers
  }

  HALO_STAMP(1);
  const int lr = lane & 15, lq = lane >> 4;
  const int bsw = (lq ^ sw(lr)) * 16;
  // Schedule (r04, each step measured): one barrier per two taps, every wait and weight
  // DMA issue at even taps; the next halo issued in two halves at taps 0 and 2, waited for at tap 4 and
  // transformed at taps 4..6 after each tap's MFMAs.
  for (int cb = 0; cb < ncb; ++cb) {
    const bool more = cb + 1 < ncb;
    const char* hb = hbuf + (cb & 1) * HBYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int u = cb * 9 + t;
      const bool BAR = t % 2 == 0;  // t is unrolled: a compile-time value
      if (wload && BAR) {  // slices u and (t < 8) u + 1 landed; issued so far: up to u + 5
        if (u + 6 < U) {
          t < 8 ? wait_vm<4>() : wait_vm<5>();  // steady state: a compile-time count, no branch chain
        } else {
          const int issued = u + 5 < U - 1 ? u + 5 : U - 1;
          const int need = (t < 8 && u + 1 < U) ? u + 1 : u;
          wait_vm_rt(issued - need);
        }
      }
      if (!wload && more && t == 4) wait_vm<0>();  // this wave's six pieces of the next block have landed
      if (BAR) __builtin_amdgcn_s_barrier();
      if (wload) {
        if (BAR) {  // slices u + 6 and (t < 8) u + 7: slots last read at taps u - 2 and u - 1
          if (u + LEAD < U) issue_b(u + LEAD);
          if (t < 8 && u + LEAD + 1 < U) issue_b(u + LEAD + 1);
        }
      } else if (t == 0 && more) {  // the next halo's six pieces in two halves, so no barrier waits on six
        issue_halo(cb + 1, 0, PPW / 2);
      } else if (t == 2 && more) {
        issue_halo(cb + 1, PPW / 2, PPW);
      }
      // pass 0's residual rows (32 KB) into the halo buffer the last channel block does not read, issued by the
      // halo waves at the last block's tap 0 (they load nothing else in it): nine taps of lead for the HBM
      // latency the epilogue's first pass used to wait on (issued at tap 8: +8.6k cycles per block, r05 stamps)
      if (t == 0 && !more && res_dma && !wload) {
        int l = lane;
        asm volatile("" : "+v"(l));
        const int base = (img * H + oy0) * W + ox0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = hw + 8 * k, pr = 4 * q + (l >> 4);
          const unsigned vo = (unsigned)(base + (pr >> 4) * W + (pr & 15)) * (unsigned)(a.res_ld * 2) + (unsigned)((l & 15) * 16);
          dma16(rsr, lds + res_off(f, 0) + q * 1024, vo, n0 * 2);
        }
      }
      const char* bb = bbuf + (u % NB) * BBYTES + (wn * 64 + lr) * 64 + bsw;
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bfv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfv[j] = *reinterpret_cast<const bf16x8*>(bb + j * 16 * 64);
      int lb = wm * HC + lr;
      asm volatile("" : "+v"(lb));
      const int sl = lb + ky * HC + kx;
      const char* ab = hb + sl * 64 + ((lq ^ sw(sl)) << 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ab + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[j], acc[i][j], 0, 0, 0);
      }
      // the next block's transform: pieces wave + 16 k, k = 0..2, by every wave at taps 4..6 (the loaders'
      // tap-4 wait and barrier made them visible), after this tap's MFMAs in program order
      if constexpr (GN != 0)
        if (t >= 4 && t < 7 && more) {
          transform_piece(cb + 1, t - 4);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // written before the next barrier
        }
    }
  }
  HALO_STAMP(2);
  if (a.res)
    halo_epilogue<NW, true>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(f), res_off(f, 0),
                            res_off(f, 1), rsr, wave);
  else
    halo_epilogue<NW, false>(acc, a, n0, wm, wn, tid, lds, (img * H + oy0) * W + ox0, W, park_off(f), res_off(f, 0),
                             res_off(f, 1), rsr, wave);
  HALO_STAMP(3);
}

bool halo_ok(const rdeic_conv_desc* d, const ConvArgs& a) {
  return d->dtype == 1 && d->kh == 3 && d->kw == 3 && d->stride == 1 && d->pad_t == 1 && d->pad_l == 1 && !d->up2 &&
         d->c1 == 0 && d->c0 % 32 == 0 && d->c0 <= halo::AB_MAX && d->cout % halo::BN == 0 && d->ho == d->h &&
         d->wo == d->w && d->h % halo::TR == 0 && d->w % halo::TC == 0 && a.batch == 1 && d->out_mode == 0 &&
         d->ld0 % 8 == 0 && ((uintptr_t)d->in0 % 16) == 0 && d->wld % 64 == 0 && epi_vec_ok(a) && a.epi_vec;
}

// The halo conv over image groups whose input stays inside a 32-bit buffer offset.
int launch_halo(const rdeic_conv_desc* d, ConvArgs a, hipStream_t s, bool* fused) {
  using namespace halo;
  const long ipix = (long)d->h * d->w;
  const long per = ipix * d->ld0 * 2;
  const int g = (int)(((1l << 31) - 1) / per);
  if (g < 1 || (long)d->cout * d->wld * 2 >= (1l << 31)) return -1;
  const bool stats = a.gn_part != nullptr && d->gn_hw == ipix;
  if (fused) *fused = stats;
  if (!stats) a.gn_part = nullptr;
  const int osz = a.out_f32 ? 4 : 2;
  for (int i0 = 0; i0 < d->n; i0 += g) {
    ConvArgs e = a;
    e.n = d->n - i0 < g ? d->n - i0 : g;
    e.M = e.n * d->ho * d->wo;
    e.in0 = a.in0 + i0 * per;
    e.out = a.out + i0 * ipix * d->out_ld * osz;
    e.res = a.res ? a.res + i0 * ipix * d->res_ld * osz : nullptr;
    e.emb = a.emb ? a.emb + (long)i0 * a.emb_ld : nullptr;
    e.gn_ab = a.gn_ab ? a.gn_ab + (long)i0 * d->c0 * 2 : nullptr;
    e.gn_row0 = i0 * (int)ipix;
    const unsigned b0 = (unsigned)(((e.n * ipix - 1) * d->ld0 + d->c0) * 2);
    const unsigned bw = (unsigned)((long)d->cout * d->wld * 2);
    rdeic_count_launch(RDEIC_COUNT_HALO_CONV);
    const bool fe = !e.out_f32 && !e.emb && e.act == 0;
    const int gm = e.gn_ab ? (e.gn_silu ? 2 : 1) : 0;
    if (g_halo8 && fe && d->h % halo8::TR == 0) {  // the 8-row, one-block-per-CU form
      const int tx8 = d->w / halo8::TC, ty8 = d->h / halo8::TR;
      const dim3 g8((unsigned)((long)e.n * ty8 * tx8 * (d->cout / halo8::BN))), b8(halo8::NT);
      if (gm == 2) hipLaunchKernelGGL((conv3x3_halo8_kernel<2>), g8, b8, halo8::LDS, s, e, tx8, ty8, b0, bw);
      else if (gm == 1) hipLaunchKernelGGL((conv3x3_halo8_kernel<1>), g8, b8, halo8::LDS, s, e, tx8, ty8, b0, bw);
      else hipLaunchKernelGGL((conv3x3_halo8_kernel<0>), g8, b8, halo8::LDS, s, e, tx8, ty8, b0, bw);
      const int rc = launch_status();
      if (rc != RDEIC_OK) return rc;
      continue;
    }
    const int tx = d->w / TC, ty = d->h / TR;
    const long tiles = (long)e.n * ty * tx * (d->cout / BN);
    const dim3 g((unsigned)tiles), b(NT);
    if (gm == 2 && fe) hipLaunchKernelGGL((conv3x3_halo_kernel<2, true>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (gm == 2) hipLaunchKernelGGL((conv3x3_halo_kernel<2, false>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (gm == 1 && fe) hipLaunchKernelGGL((conv3x3_halo_kernel<1, true>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (gm == 1) hipLaunchKernelGGL((conv3x3_halo_kernel<1, false>), g, b, LDS, s, e, tx, ty, b0, bw);
    else if (fe) hipLaunchKernelGGL((conv3x3_halo_kernel<0, true>), g, b, LDS, s, e, tx, ty, b0, bw);
    else hipLaunchKernelGGL((conv3x3_halo_kernel<0, false>), g, b, LDS, s, e, tx, ty, b0, bw);
    const int rc = launch_status();
    if (rc != RDEIC_OK) return rc;
  }
  return RDEIC_OK;
}

}  // namespace rdeic_conv
