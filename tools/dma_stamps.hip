// Diagnostic: where does an LDS-DMA conv tile (conv_dma_kernel) spend its time on a transformer linear?
// Compiles the conv sources (conv_gemm / conv_dma / conv_halo.hip) with per-block shader-clock stamps (RDEIC_HALO_STAMPS: entry, prologue DMA issued,
// k-loop end, epilogue end) and runs one 1x1 "conv" over M token rows through the library's own dispatch
// (rdeic_conv2d_tile), optionally with the fused GEGLU epilogue and a residual. Prints the event-timed
// launch and the per-block phase split (medians), plus the k-loop cycles per k-tile.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize tools/dma_stamps.hip -o tools/dma_stamps \
//         -Lrdeic_amd/lib -lrdeic_hip -Wl,-rpath,'$ORIGIN/../rdeic_amd/lib'
//   tools/dma_stamps M K N TILE [geglu res]
#define RDEIC_HALO_STAMPS 1
#include "../rdeic_amd/csrc/conv_gemm.hip"
#include "../rdeic_amd/csrc/conv_dma.hip"
#include "../rdeic_amd/csrc/conv_halo.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[(size_t)(q * (v.size() - 1))];
}

static const int BMS[] = {256, 128, 128, 128, 128, 64, 128, 256, 128, 64, 128, 256, 256, 128, 512, 64, 128, 64};  // tiles 21..38
static const int BNS[] = {128, 256, 128, 128, 128, 128, 128, 128, 256, 128, 64, 256, 128, 128, 128, 128, 160, 160};

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 65536, K = argc > 2 ? atoi(argv[2]) : 320, N = argc > 3 ? atoi(argv[3]) : 2560;
  const int tile = argc > 4 ? atoi(argv[4]) : 32;
  const int geglu = argc > 5 ? atoi(argv[5]) : 0, use_res = argc > 6 ? atoi(argv[6]) : 0;
  if (tile < 21 || tile > 38) { fprintf(stderr, "tile 21..38\n"); return 1; }
  const int wld = (K + 63) / 64 * 64;
  const int NO = geglu ? N / 2 : N;
  bf16 *x, *wt, *res = nullptr, *out;
  float* bias;
  CK(hipMalloc(&x, (long)M * K * 2));
  CK(hipMalloc(&wt, (long)N * wld * 2));
  CK(hipMalloc(&out, (long)M * NO * 2));
  CK(hipMalloc(&bias, N * 4));
  CK(hipMemset(bias, 0, N * 4));
  if (use_res) CK(hipMalloc(&res, (long)M * NO * 2));
  fill_bf16_k<<<4096, 256>>>(x, (long)M * K, 1, 2.f, 0.f);
  fill_bf16_k<<<1024, 256>>>(wt, (long)N * wld, 2, 0.1f, 0.f);
  if (use_res) fill_bf16_k<<<4096, 256>>>(res, (long)M * NO, 3, 1.f, 0.f);
  const int bm = BMS[tile - 21], bn = BNS[tile - 21];
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  unsigned long long* st;
  CK(hipMalloc(&st, tiles * 8 * 8));
  CK(hipMemset(st, 0, tiles * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_halo_stamps), &st, sizeof(st)));
  rdeic_conv_desc d{};
  d.in0 = x; d.c0 = K; d.ld0 = K; d.n = 1; d.h = M; d.w = 1;
  d.weight = wt; d.wld = wld; d.bias = bias; d.cout = N; d.kh = 1; d.kw = 1; d.stride = 1;
  d.ho = M; d.wo = 1; d.res = res; d.res_ld = NO; d.out = out; d.out_ld = NO; d.dtype = 1; d.batch = 1;
  d.out_mode = geglu ? 2 : 0;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int i = 0; i < 3; ++i)
    if (rdeic_conv2d_tile(&d, tile, s) != 0) { fprintf(stderr, "conv failed\n"); return 1; }
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 10;
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) rdeic_conv2d_tile(&d, tile, s);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double flops = 2.0 * M * (double)N * K;
  std::vector<unsigned long long> h(tiles * 8);
  CK(hipMemcpy(h.data(), st, tiles * 8 * 8, hipMemcpyDeviceToHost));  // stamps of the last launch
  unsigned long long t0 = ~0ull, t1 = 0;
  std::vector<double> pro, mainl, epi, tot;
  for (long b = 0; b < tiles; ++b) {
    const unsigned long long* q = &h[b * 8];
    if (!q[0]) continue;
    t0 = std::min(t0, q[0]);
    t1 = std::max(t1, q[3]);
    pro.push_back((double)(q[1] - q[0]));
    mainl.push_back((double)(q[2] - q[1]));
    epi.push_back((double)(q[3] - q[2]));
    tot.push_back((double)(q[3] - q[0]));
  }
  const int nk = wld / 64;
  printf("{\"shape\": [%d, %d, %d], \"tile\": %d, \"bm\": %d, \"bn\": %d, \"geglu\": %d, \"res\": %d, \"us\": %.2f, "
         "\"tflops\": %.1f, \"tiles\": %ld, \"span_cycles\": %.0f, \"cycles\": {\"issue_med\": %.0f, \"kloop_med\": %.0f, "
         "\"kloop_p90\": %.0f, \"kloop_per_ktile\": %.0f, \"epilogue_med\": %.0f, \"epilogue_p90\": %.0f, "
         "\"block_med\": %.0f}}\n",
         M, K, N, tile, bm, bn, geglu, use_res, ms * 1e3, flops / (ms * 1e-3) / 1e12, tiles, (double)(t1 - t0),
         pct(pro, .5), pct(mainl, .5), pct(mainl, .9), pct(mainl, .5) / nk, pct(epi, .5), pct(epi, .9), pct(tot, .5));
  return 0;
}
