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
// conv_in: cin = 8 (3 real channels, zero-padded: rdeic_image_u8_to_nhwc), 3x3, stride 1, pad 1, bias, bf16 out.
// GEMM view M = pixels, N = cout, K = 9 taps x 8 channels = 72: three 32-deep k-steps of
// v_mfma_f32_16x16x32_bf16, in which a pixel-fragment lane holds 8 consecutive k = ONE tap's 8 channels of one
// pixel (16 bytes). A block (4 waves, one per 32 output channels) walks 64-pixel tiles (one image row segment,
// persistent: tiles b, b + grid, ...):
//   * the tile's 3 x 66 halo pixels come by LDS-DMA, one 1 KB wave-instruction per wave, into a 4-deep ring issued
//     3 tiles ahead (no VGPRs held for the prefetch; the image pad and the k tail read zeros through the buffer
//     descriptor's range check); one barrier per tile;
//   * the MFMAs run transposed (weights as the A operand, pixels as B): a lane's result is 4 consecutive channels of
//     one pixel, parked in LDS with two dword writes per fragment. Each output element is the register tile's
//     32-term dot product over the same k-steps; the register tile's fourth k-step (all zero) adds +-0 products
//     to an accumulator that cannot be -0 (it starts at +0, and x + -0 = x, +0 + -0 = +0 in round-to-nearest), an
//     identity, so it is skipped and the outputs stay bit-identical;
//   * the epilogue is WAVE-PRIVATE (64 pixels = one canonical 64-row GroupNorm block x the wave's 32 channels): the
//     parked bf16 tile is stored as 16-byte row chunks (4 lanes per 64-byte pixel row slice) and scanned for the
//     GroupNorm partials: lane (channel pair, 16-row group g) sums its group's rows in order (fmaf for the squares,
//     packed over the pair), and ((g0 + g1) + g2) + g3 is taken across the four lane quarters: the canonical order
//     of epilogue_vec / gn_rows_partial, so the statistics are bit-identical too.
// Store-bound: 1.07 GB out per launch at 16 x 512^2 (a plain store kernel of the same pattern reaches 5.9 TB/s,
// tools/store_probe.hip).
// ============================================================================================
constexpr int CI_NT = 256;            // 4 waves: one 64-pixel block x 4 channel quarters of 32
constexpr int CI_ROWB = 68;           // LDS bytes per parked pixel row (32 bf16 + 4): conflict-free scans
constexpr int CI_WLDS = 64 * CI_ROWB; // per wave
constexpr int CJ_S = 4, CJ_STAGE = 4096;  // ring depth; 256 items per stage: 3 x 66 halo pixels, then zeros
constexpr int CJ_ZERO = 3 * 66;  // first zero item

template <bool STATS>
__global__ __launch_bounds__(CI_NT) __attribute__((amdgpu_waves_per_eu(4, 4))) void conv_in8_kernel(ConvArgs a, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = (wave & 3) * 32;  // this wave's 32 output channels
  char* const W = lds + CJ_S * CJ_STAGE + wave * CI_WLDS;
  const int lr = lane & 15, lq = lane >> 4;
  const int hw = a.h * a.w, grid = gridDim.x;
  const bf16* wt = reinterpret_cast<const bf16*>(a.weight);
  bf16* const out = reinterpret_cast<bf16*>(a.out);
  // waves past cout still load and sync (the ring is shared); they compute and store nothing
  const bool active = c0 < a.cout;

  bf16x8 wf[3][2];  // A operand: weight rows c0 + 16 j + lr, k = 32 s + 8 lq (k-step 2: k 64..71 in lq = 0 only)
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16x8 v = {};
      if (active && (s < 2 || lq == 0)) v = *reinterpret_cast<const bf16x8*>(wt + (long)(c0 + 16 * j + lr) * a.wld + 32 * s + 8 * lq);
      wf[s][j] = v;
    }
  f32x4 bias[2];  // channels c0 + 16 j + 4 lq + r
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = (active && a.bias) ? a.bias[c0 + 16 * j + 4 * lq + r] : 0.f;
  if (STATS && blockIdx.x == 0 && tid == 0) reinterpret_cast<int*>(a.gn_part)[0] = 64;  // rows per partial

  const __amdgpu_buffer_rsrc_t rsi = __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0,
                                                                      (int)((long)a.M * a.ld0 * 2), 0x00020000);
  const int item = wave * 64 + lane, hr = item / 66, hc = item - hr * 66;
  // the DMA of tile tt into ring slot `slot`; issued by every wave for every slot (tt past the end reads zeros),
  // so the count of younger vector-memory ops at each wait is a constant
  auto dma = [&](int tt, int slot) {
    const int m0 = tt * 64;  // 64 pixels of one image row (w % 64 == 0)
    const int img = __builtin_amdgcn_readfirstlane(m0 / hw), rem = __builtin_amdgcn_readfirstlane(m0 - img * hw);
    const int y0 = __builtin_amdgcn_readfirstlane(rem / a.w), x0 = __builtin_amdgcn_readfirstlane(rem - y0 * a.w);
    const int iy = y0 - 1 + hr, ix = x0 - 1 + hc;
    const bool ok = tt < ntiles && item < CJ_ZERO && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    dma16(rsi, lds + slot * CJ_STAGE + wave * 1024, ok ? (unsigned)(((img * a.h + iy) * a.w + ix) * a.ld0) * 2u : kOOB, 0);
  };
  // B fragment addresses: k-step s, lane tap 4 s + lq, pixel 16 i + lr -> halo item ky * 66 + kx + 16 i + lr;
  // taps 9..11 (k-step 2, lq > 0) read the zero items (no i stride: they stay inside the stage)
  int boff[3], bstr2;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int tap = 4 * s + lq, ky = tap / 3, kx = tap - (tap / 3) * 3;
    boff[s] = (tap < 9 ? ky * 66 + kx + lr : CJ_ZERO + lr) * 16;
  }
  bstr2 = lq == 0 ? 256 : 0;
  // vector-memory ops younger than DMA(k) at iteration k's wait (steady state): the DMAs of k+1 .. k+S-2 and the
  // stores of the S-1 iterations before k (4 row stores + the statistics store each)
  constexpr int NSTEADY = (CJ_S - 2) + (CJ_S - 1) * (4 + (STATS ? 1 : 0));
  static_assert(NSTEADY < 64, "vmcnt is 6 bits");

#pragma unroll
  for (int s = 0; s < CJ_S - 1; ++s) dma(blockIdx.x + s * grid, s);
  int k = 0;
  for (int t = blockIdx.x; t < ntiles; t += grid, ++k) {
    if (k < CJ_S - 1) wait_vm<0>();
    else if (active) wait_vm<NSTEADY>();
    else wait_vm<CJ_S - 2>();  // (a wave past cout issues no stores)
    __builtin_amdgcn_s_barrier();  // every wave's piece of tile t landed; slot (k - 1) % S is no longer read
    dma(t + (CJ_S - 1) * grid, (k + CJ_S - 1) % CJ_S);
    const char* st = lds + (k % CJ_S) * CJ_STAGE;
    const int m0 = t * 64;
    f32x4 acc[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // k-steps 0..2; the register tile's fourth (all-zero) step adds +-0 products to an accumulator that cannot be
    // -0 (it starts at +0, and x + -0 = x, +0 + -0 = +0 in round-to-nearest): an identity, skipped
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 pf = *reinterpret_cast<const bf16x8*>(st + boff[s] + (s == 2 ? i * bstr2 : i * 256));
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s][j], pf, acc[j][i], 0, 0, 0);
      }
    if (!active) continue;
    // (acc + bias) rounded to bf16, parked row-major: lane holds channels 16 j + 4 lq + 0..3 of pixel 16 i + lr
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        unsigned* dst = reinterpret_cast<unsigned*>(W + (16 * i + lr) * CI_ROWB + (16 * j + 4 * lq) * 2);
        const f32x4 v = acc[j][i] + bias[j];  // packed adds
        dst[0] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{v[0], v[1]}, bf16x2_t));
        dst[1] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{v[2], v[3]}, bf16x2_t));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS tile, written by all its lanes
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 4 lanes per pixel row of 64 bytes, 16 rows per instruction
      const int row = 16 * q + (lane >> 2), ch = lane & 3;
      const unsigned* src = reinterpret_cast<const unsigned*>(W + row * CI_ROWB + ch * 16);
      *reinterpret_cast<uint4*>(out + (long)(m0 + row) * a.out_ld + c0 + ch * 8) = uint4{src[0], src[1], src[2], src[3]};
    }
    if constexpr (STATS) {  // canonical 16-row groups, ((g0 + g1) + g2) + g3
      const int p2 = lane & 15, g = lane >> 4;
      f32x2 s1 = {0.f, 0.f}, s2 = {0.f, 0.f};  // the channel pair in packed-f32 ops (the same per-element order)
      unsigned w[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) w[r] = *reinterpret_cast<const unsigned*>(W + (16 * g + r) * CI_ROWB + p2 * 4);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const f32x2 y = {__uint_as_float(w[r] << 16), __uint_as_float(w[r] & 0xffff0000u)};
        s1 += y;
        s2 = __builtin_elementwise_fma(y, y, s2);
      }
      float t1[2], t2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        t1[e] = ((s1[e] + __shfl(s1[e], p2 + 16, 64)) + __shfl(s1[e], p2 + 32, 64)) + __shfl(s1[e], p2 + 48, 64);
        t2[e] = ((s2[e] + __shfl(s2[e], p2 + 16, 64)) + __shfl(s2[e], p2 + 32, 64)) + __shfl(s2[e], p2 + 48, 64);
      }
      if (g == 0) {
        float* pp = a.gn_part + 4 + ((long)((a.gn_row0 + m0) / 64) * a.cout + c0 + 2 * p2) * 2;
        *reinterpret_cast<float4*>(pp) = make_float4(t1[0], t2[0], t1[1], t2[1]);
      }
    }
  }
  wait_vm<0>();  // the tail DMAs (zeros past the last tile) land before the block's LDS is released
}

// ============================================================================================
// norm -> SiLU -> 3x3 conv to a few channels (cout <= 16; the decoder's conv_out 128 -> 3, fp32 output).
// A block owns TR x 64 output pixels (TR = 8 waves, one output row each; two 50 KB blocks per CU, so one block's
// transform runs beside the other's MFMAs: 16 rows per block measured 22% slower, 4 rows 5%, one raw block in
// flight instead of two 4%). Per 32-channel block of the input, the threads load the (TR + 2) x 66 halo of the RAW
// input (buffer loads, 16 bytes each: coalesced 64-byte pixel slices; zeros outside the image from the
// descriptor's range check), apply the GroupNorm affine + SiLU ONCE per element in registers (channel pairs in
// packed f32: z = -x log2(e) from the pre-scaled table, one v_exp for e^-x = 2^z, x / (1 + e^-x) as
// z * rcp(-log2(e) (1 + 2^z)); rounded to bf16) and write it to LDS; then every wave runs the
// 9 taps as 16x16x32 MFMAs with N = 16 (cout real columns, the rest zero weights) reading its A fragments from the
// halo and its B fragments from the weights staged in LDS (a global load there would wait, in-order vmcnt, behind
// the prefetched halo chunks). The raw chunks of the next two channel blocks are in flight (each reloaded right
// after its transform). The transform is (TR + 2) / TR x 66 / 64 of the element count.
// k order: 32-channel block major, tap minor (as the halo convs); fp32 accumulation.
// ============================================================================================
constexpr int NR_TC = 64, NR_HC = NR_TC + 2;
template <int TR> struct Narrow {
  static constexpr int NT = TR * 64, HPIX = (TR + 2) * NR_HC, ITEMS = HPIX * 4;  // 16-byte chunks per halo
  static constexpr int IPT = (ITEMS + NT - 1) / NT;
  static constexpr int LDS = HPIX * 64;  // halo (then the (a, b) table)
};
__device__ __forceinline__ int nr_sw(int s) { return ((s >> 2) & 1) << 1; }  // halo conv swizzle (conflict-free)

template <int TR, bool SILU>
__global__ __launch_bounds__(TR * 64) __attribute__((amdgpu_waves_per_eu(4, 4))) void conv3x3_gn_narrow_kernel(
    ConvArgs a, int tiles_x, int tiles_y) {
  using NR = Narrow<TR>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* const abl = reinterpret_cast<float*>(lds + NR::LDS);  // the image's GroupNorm (a, b) table
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int sp = blockIdx.x;
  const int tx = sp % tiles_x;
  sp /= tiles_x;
  const int ty = sp % tiles_y, img = sp / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * NR_TC;
  const int H = a.h, W = a.w, cin = a.c0;
  const int lr = lane & 15, lq = lane >> 4;
  const int q = tid & 3;  // this thread's 16-byte chunk of every halo pixel it loads (NT % 4 == 0)
  const bf16* in = reinterpret_cast<const bf16*>(a.in0);
  // LDS-only barrier: __syncthreads() would also wait for the channel blocks' loads in flight
  auto bar = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  constexpr float kNL2E = -1.4426950408889634f;  // -log2(e)
  for (int i = tid; i < cin / 2; i += NR::NT) {
    float4 v = reinterpret_cast<const float4*>(a.gn_ab + (long)img * cin * 2)[i];
    if constexpr (SILU) v = make_float4(v.x * kNL2E, v.y * kNL2E, v.z * kNL2E, v.w * kNL2E);  // gives z = -x log2(e)
    reinterpret_cast<float4*>(abl)[i] = v;
  }
  // the packed weights of the cout rows in LDS after the table: the MFMA phase then issues no global load, which
  // would wait (in-order vmcnt) behind the next blocks' raw chunks in flight
  char* const wl = lds + NR::LDS + cin * 8;
  const int wrow = 9 * cin;
  for (int i = tid; i < a.cout * wrow / 8; i += NR::NT) {
    const int r = i / (wrow / 8), c = i - r * (wrow / 8);
    reinterpret_cast<uint4*>(wl)[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.weight) + (long)r * a.wld + c * 8);
  }
  // per item: the chunk's byte offset in the input (kOOB: outside the image / past the halo: the buffer
  // descriptor's range check reads zeros, no branch) and its LDS slot, the same for every channel block
  const __amdgpu_buffer_rsrc_t rsi = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.in0, (short)0, (int)((long)a.n * H * W * a.ld0 * 2), 0x00020000);
  unsigned goff[NR::IPT];
  int loff[NR::IPT];
#pragma unroll
  for (int k = 0; k < NR::IPT; ++k) {
    const int it = tid + k * NR::NT, hp = it >> 2;
    const int hr = hp / NR_HC, hc = hp - (hp / NR_HC) * NR_HC;
    const int iy = oy0 - 1 + hr, ix = ox0 - 1 + hc;
    goff[k] = (it < NR::ITEMS && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                  ? (unsigned)(((img * H + iy) * W + ix) * a.ld0 + 8 * q) * 2u : kOOB;
    loff[k] = it < NR::ITEMS ? hp * 64 + ((q ^ nr_sw(hp)) << 4) : -1;
  }
  // raw chunks of two channel blocks in flight (the HBM latency is ~2 blocks of transform + MFMA)
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  u4v raw0[NR::IPT], raw1[NR::IPT];
  auto load = [&](u4v (&raw)[NR::IPT], int cb, int k) {
    if (cb < cin) raw[k] = __builtin_amdgcn_raw_buffer_load_b128(rsi, goff[k], cb * 2, 0);
  };
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one channel block: transform its raw chunks into the halo (reloading the registers with block cb + 64), then
  // the 9 taps
  auto step = [&](u4v (&raw)[NR::IPT], int cb) {
    bar();  // the (a, b) table is in LDS / the previous block's MFMA reads of the halo are done
    const float4* ab4 = reinterpret_cast<const float4*>(abl + (cb + 8 * q) * 2);
    const float4 t0 = ab4[0], t1 = ab4[1], t2 = ab4[2], t3 = ab4[3];
    const float av[8] = {t0.x, t0.z, t1.x, t1.z, t2.x, t2.z, t3.x, t3.z};
    const float bv[8] = {t0.y, t0.w, t1.y, t1.w, t2.y, t2.w, t3.y, t3.w};
#pragma unroll
    for (int k = 0; k < NR::IPT; ++k) {
      // a channel pair per packed-f32 op; computed for every chunk and zeroed outside the image (the normalised
      // tensor's zero pad) with a select, not a branch
      const unsigned w4[4] = {raw[k].x, raw[k].y, raw[k].z, raw[k].w};
      unsigned o4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // channels 2e, 2e + 1 of the chunk
        const f32x2 xin = {__uint_as_float(w4[e] << 16), __uint_as_float(w4[e] & 0xffff0000u)};
        f32x2 z = __builtin_elementwise_fma(xin, f32x2{av[2 * e], av[2 * e + 1]}, f32x2{bv[2 * e], bv[2 * e + 1]});
        if constexpr (SILU) {
          // the table is pre-scaled by -log2(e): z = -x log2(e), e^-x = 2^z (one v_exp), and
          // x / (1 + e^-x) = z / (-log2(e) (1 + 2^z)) (the last layer's fp32 output, no bit-parity partner)
          const f32x2 ex = {__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])};
          const f32x2 den = __builtin_elementwise_fma(ex, f32x2{kNL2E, kNL2E}, f32x2{kNL2E, kNL2E});
          z = z * f32x2{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
        }
        typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
        o4[e] = __builtin_bit_cast(unsigned, __builtin_convertvector(z, bf16x2_t));  // one v_cvt_pk_bf16_f32
      }
      const bool in_img = goff[k] != kOOB;
      const uint4 o = in_img ? uint4{o4[0], o4[1], o4[2], o4[3]} : uint4{0u, 0u, 0u, 0u};
      if (loff[k] >= 0) *reinterpret_cast<uint4*>(lds + loff[k]) = o;
      load(raw, cb + 64, k);  // two blocks ahead
    }
    bar();
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - (t / 3) * 3;
      // per-tap addresses from laundered bases (hoisted, the 36 fragment addresses would spill)
      int lb = wave * NR_HC + lr, wb = lr * wrow + cb + 8 * lq;
      asm volatile("" : "+v"(lb), "+v"(wb));
      bf16x8 bfv = {};
      if (lr < a.cout) bfv = *reinterpret_cast<const bf16x8*>(wl + (wb + t * cin) * 2);
      const int hp0 = lb + ky * NR_HC + kx;
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // + 16 i keeps the swizzle (bits 2 of the pixel index unchanged)
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(lds + (hp0 + 16 * i) * 64 + ((lq ^ nr_sw(hp0)) << 4));
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv, acc[i], 0, 0, 0);
      }
    }
  };
#pragma unroll
  for (int k = 0; k < NR::IPT; ++k) {
    load(raw0, 0, k);
    load(raw1, 32, k);
  }
  for (int cb = 0; cb < cin; cb += 64) {
    step(raw0, cb);
    if (cb + 32 < cin) step(raw1, cb + 32);
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

namespace {
int launch_narrow(const rdeic_conv_desc* d, const ConvArgs& a, hipStream_t s) {
  constexpr int TR = 8;
  const int lds = Narrow<TR>::LDS + d->c0 * 8 + d->cout * 9 * d->c0 * 2;
  if (!(d->gn_ab && d->cout <= 16 && d->c0 % 32 == 0 && d->h % TR == 0 && d->w % NR_TC == 0 && lds <= 160 * 1024 &&
        !d->gn_part && !d->emb && ((uintptr_t)d->gn_ab) % 16 == 0))
    return -1;
  rdeic_count_launch(RDEIC_COUNT_EDGE);
  const int tx = d->w / NR_TC, ty = d->h / TR;
  const dim3 g((unsigned)((long)d->n * ty * tx));
  if (d->gn_silu) hipLaunchKernelGGL((conv3x3_gn_narrow_kernel<TR, true>), g, dim3(TR * 64), lds, s, a, tx, ty);
  else hipLaunchKernelGGL((conv3x3_gn_narrow_kernel<TR, false>), g, dim3(TR * 64), lds, s, a, tx, ty);
  return launch_status();
}
}  // namespace

// Returns -1 when neither edge kernel takes the launch.
int launch_edge(const rdeic_conv_desc* d, const ConvArgs& a, hipStream_t s, bool* fused) {
  if (!g_edge || d->dtype != 1 || d->kh != 3 || d->kw != 3 || d->stride != 1 || d->pad_t != 1 || d->pad_l != 1 ||
      d->up2 || d->c1 || d->ho != d->h || d->wo != d->w || a.batch != 1 || d->out_mode != 0 || d->ld0 % 8 ||
      ((uintptr_t)d->in0) % 16 || ((uintptr_t)d->weight) % 16)
    return -1;
  // conv_in: 8 input channels, bias only, bf16 output, statistics per image (64-row blocks)
  if (d->c0 == 8 && !d->gn_ab && d->wld >= 128 && d->cout % 32 == 0 && d->cout <= 128 && d->w % 64 == 0 && !d->emb && !d->act && !d->res &&
      !d->out_f32 && !d->ln_rows && d->out_ld % 8 == 0 && ((uintptr_t)d->out) % 16 == 0) {
    ConvArgs e = a;
    const bool stats = e.gn_part != nullptr && e.gn_hw > 0 && e.gn_hw % 64 == 0;
    if (!stats) e.gn_part = nullptr;
    if (fused) *fused = stats;
    rdeic_count_launch(RDEIC_COUNT_EDGE);
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
    }
    const int ntiles = e.M / 64;  // w % 64 == 0
    const int lds = CJ_S * CJ_STAGE + 4 * CI_WLDS;
    const int blocks = ntiles < 4 * cus ? ntiles : 4 * cus;  // four 4-wave blocks per CU
    if (stats) hipLaunchKernelGGL(conv_in8_kernel<true>, dim3((unsigned)blocks), dim3(CI_NT), lds, s, e, ntiles);
    else hipLaunchKernelGGL(conv_in8_kernel<false>, dim3((unsigned)blocks), dim3(CI_NT), lds, s, e, ntiles);
    return launch_status();
  }
  // norm -> (SiLU) -> conv to <= 16 channels (table + weights in LDS beside the halo)
  return launch_narrow(d, a, s);
}

}  // namespace rdeic_conv
