// Diagnostic: where does conv3x3_halo_kernel spend its time? Compiles the conv sources (conv_gemm / conv_dma / conv_halo.hip) with per-block
// shader-clock stamps (RDEIC_HALO_STAMPS: kernel entry, main-loop start, main-loop end, epilogue end)
// and runs the halo conv on one layer shape with random operands, through the library's own dispatch
// (rdeic_conv2d). Prints the event-timed launch and the per-block phase split.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize tools/halo_stamps.hip -o tools/halo_stamps_cur
//   (self-contained: linking librdeic_hip.so let its registration of the same kernel names win, so the stamped
//   kernels never ran)
//   tools/halo_stamps N H W C COUT [res stats]
#define RDEIC_HALO_STAMPS 1
#include "../rdeic_amd/csrc/conv_gemm.hip"
#include "../rdeic_amd/csrc/conv_dma.hip"
#include "../rdeic_amd/csrc/conv_halo.hip"
#include "../rdeic_amd/csrc/conv_edge.hip"
#include "../rdeic_amd/csrc/prof.hip"
#include "../rdeic_amd/csrc/norm.hip"
#include "../rdeic_amd/csrc/attention.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void fill_bf16_k(bf16* p, long n, unsigned seed, float scale, float off) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (bf16)(((h & 0xFFFFFF) / 16777216.f - 0.5f) * scale + off);
  }
}
__global__ void fill_f32_k(float* p, long n, unsigned seed, float scale, float off) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = ((h & 0xFFFFFF) / 16777216.f - 0.5f) * scale + off;
  }
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[(size_t)(q * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 16, H = argc > 2 ? atoi(argv[2]) : 512, W = argc > 3 ? atoi(argv[3]) : 512;
  const int C = argc > 4 ? atoi(argv[4]) : 128, CO = argc > 5 ? atoi(argv[5]) : 128;
  const int use_res = argc > 6 ? atoi(argv[6]) : 1, use_stats = argc > 7 ? atoi(argv[7]) : 1;
  const long npx = (long)N * H * W;
  const int wld = (9 * C + 63) / 64 * 64;
  bf16 *x, *wt, *res, *out;
  float *bias, *ab, *part;
  CK(hipMalloc(&x, npx * C * 2));
  CK(hipMalloc(&wt, (long)CO * wld * 2));
  CK(hipMalloc(&res, npx * CO * 2));
  CK(hipMalloc(&out, npx * CO * 2));
  CK(hipMalloc(&bias, CO * 4));
  CK(hipMalloc(&ab, (long)N * C * 2 * 4));
  const long nparts = (npx / 64) * CO * 2 + 64;
  CK(hipMalloc(&part, nparts * 4));
  fill_bf16_k<<<4096, 256>>>(x, npx * C, 1, 4.f, 0.3f);
  fill_bf16_k<<<1024, 256>>>(wt, (long)CO * wld, 2, 0.1f, 0.f);
  fill_bf16_k<<<4096, 256>>>(res, npx * CO, 3, 2.f, 0.f);
  fill_f32_k<<<64, 256>>>(bias, CO, 4, 0.2f, 0.f);
  fill_f32_k<<<64, 256>>>(ab, (long)N * C * 2, 5, 1.f, 0.5f);
  // HALO4=1 in the environment: the 4-row kernel everywhere (option 9 off)
  const int h8 = getenv("HALO4") && atoi(getenv("HALO4")) ? 0 : 1;
  rdeic_set_conv_option(9, h8);
  const int trow = (h8 && H % 8 == 0) ? 8 : 4;
  const long tiles = (long)N * (H / trow) * (W / 64) * (CO / 128);
  unsigned long long* st;
  CK(hipMalloc(&st, tiles * 8 * 8));
  CK(hipMemset(st, 0, tiles * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_halo_stamps), &st, sizeof(st)));
  rdeic_conv_desc d{};
  d.in0 = x; d.c0 = C; d.ld0 = C; d.n = N; d.h = H; d.w = W;
  d.weight = wt; d.wld = wld; d.bias = bias; d.cout = CO; d.kh = 3; d.kw = 3; d.stride = 1; d.pad_t = 1; d.pad_l = 1;
  d.ho = H; d.wo = W; d.gn_ab = ab; d.gn_silu = 1; d.res = use_res ? res : nullptr; d.res_ld = CO;
  d.out = out; d.out_ld = CO; d.dtype = 1; d.batch = 1;
  if (use_stats) { d.gn_part = part; d.gn_hw = H * W; }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const long n0 = rdeic_launch_count(RDEIC_COUNT_HALO_CONV);
  for (int i = 0; i < 3; ++i)
    if (rdeic_conv2d(&d, s) != 0) { fprintf(stderr, "conv failed\n"); return 1; }
  CK(hipStreamSynchronize(s));
  if (rdeic_launch_count(RDEIC_COUNT_HALO_CONV) == n0) { fprintf(stderr, "halo kernel not taken\n"); return 1; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 10;
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) rdeic_conv2d(&d, s);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double flops = 2.0 * npx * CO * 9.0 * C;
  std::vector<unsigned long long> h(tiles * 8);
  CK(hipMemcpy(h.data(), st, tiles * 8 * 8, hipMemcpyDeviceToHost));  // stamps of the last launch
  unsigned long long t0 = ~0ull, t1 = 0;
  std::vector<double> pro, mainl, epi, tot;
  std::map<long, std::vector<std::pair<unsigned long long, unsigned long long>>> per_cu;
  for (long b = 0; b < tiles; ++b) {
    const unsigned long long* q = &h[b * 8];
    t0 = std::min(t0, q[0]);
    t1 = std::max(t1, q[3]);
    pro.push_back((double)(q[1] - q[0]));
    mainl.push_back((double)(q[2] - q[1]));
    epi.push_back((double)(q[3] - q[2]));
    tot.push_back((double)(q[3] - q[0]));
    const long hw = (long)q[5], xcc = (long)q[6];
    const long cu = (xcc & 0xF) * 4096 + ((hw >> 8) & 0xF) * 256 + ((hw >> 13) & 0x7) * 16 + ((hw >> 16) & 0x3);  // SE, SH, CU
    per_cu[cu].push_back({q[0], q[3]});
  }
  // busy fraction and mean blocks in flight per CU
  double conc = 0, span_sum = 0;
  for (auto& kv : per_cu) {
    unsigned long long a = ~0ull, z = 0;
    double busy = 0;
    for (auto& iv : kv.second) { a = std::min(a, iv.first); z = std::max(z, iv.second); busy += (double)(iv.second - iv.first); }
    conc += busy / (double)(z - a);
    span_sum += (double)(z - a);
  }
  // epilogue overlap: for each block, the share of its XCD's CUs whose blocks are in their epilogue at its
  // epilogue's midpoint (~1 when the CUs run in lockstep, ~epilogue/block when they are de-phased)
  std::map<long, std::vector<std::pair<unsigned long long, unsigned long long>>> epi_by_xcd;
  std::map<long, std::map<long, int>> cus_by_xcd;
  for (long b = 0; b < tiles; ++b) {
    const unsigned long long* q = &h[b * 8];
    const long xcc = (long)q[6] & 0xF, hw = (long)q[5];
    epi_by_xcd[xcc].push_back({q[2], q[3]});
    cus_by_xcd[xcc][((hw >> 8) & 0xF) * 256 + ((hw >> 13) & 0x7) * 16 + ((hw >> 16) & 0x3)] = 1;
  }
  double ov_sum = 0;
  long ov_n = 0;
  for (auto& kv : epi_by_xcd) {
    auto& v = kv.second;
    const double ncu = (double)cus_by_xcd[kv.first].size();
    for (size_t i = 0; i < v.size(); i += 7) {  // sampled
      const unsigned long long mid = v[i].first / 2 + v[i].second / 2;
      int c = 0;
      for (auto& e : v) c += (e.first <= mid && mid < e.second);
      ov_sum += c / ncu;
      ++ov_n;
    }
  }
  const double cyc_span = (double)(t1 - t0);
  const double clk_ghz = cyc_span / (ms * 1e6);
  // MFMA-bound floor per block: (9 taps x cin/32) x 16 MFMA x 16 cycles x waves per SIMD (2 or 4)
  const double floor_main = 9.0 * (C / 32) * 16 * 16 * (trow / 2);
  printf("{\"shape\": [%d, %d, %d, %d, %d], \"res\": %d, \"stats\": %d, \"ms\": %.4f, \"tflops\": %.1f, "
         "\"blocks\": %ld, \"cus_seen\": %zu, \"clock_ghz_est\": %.3f, \"blocks_in_flight_per_cu\": %.2f, "
         "\"cycles\": {\"prologue_med\": %.0f, \"main_med\": %.0f, \"main_p90\": %.0f, \"epilogue_med\": %.0f, "
         "\"epilogue_p90\": %.0f, \"block_med\": %.0f}, \"main_floor_cycles\": %.0f, \"tile_rows\": %d, \"epi_overlap\": %.3f}\n",
         N, H, W, C, CO, use_res, use_stats, ms, flops / (ms * 1e-3) / 1e12, tiles, per_cu.size(), clk_ghz,
         conc / per_cu.size(), pct(pro, .5), pct(mainl, .5), pct(mainl, .9), pct(epi, .5), pct(epi, .9), pct(tot, .5),
         floor_main, trow, ov_n ? ov_sum / ov_n : 0.0);
  return 0;
}
