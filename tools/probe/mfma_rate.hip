// Probe: MFMA issue rate of the halo8 main loop's shape without memory: 16 waves per CU (one 1024-thread block),
// each wave a 64 x 64 fp32 accumulator tile, operands in registers, per "tap" either 16 x v_mfma_f32_16x16x32_bf16
// (the shipped form) or 8 x v_mfma_f32_32x32x16_bf16 (same flops). Prints cycles per tap per SIMD against the
// 1024-cycle floor (4 waves x 256 MFMA cycles). With BAR=1 a raw s_barrier every two taps (halo8's cadence).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe/mfma_rate.hip -o tools/probe/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int FORM, int BAR>
__global__ __launch_bounds__(1024) void probe(float* out, int taps, unsigned long long* cyc) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) { a[i][e] = (__bf16)(0.001f * (lane + i + e)); b[i][e] = (__bf16)(0.002f * (lane - i + e)); }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  if constexpr (FORM == 0) {
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < taps; ++t) {
      if (BAR && (t & 1) == 0) __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  } else {
    f32x16 acc[2][2];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    for (int t = 0; t < taps; ++t) {
      if (BAR && (t & 1) == 0) __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2 * k + i], b[2 * k + j], acc[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) s += acc[i][j][0] + acc[i][j][15];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 1024 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int FORM, int BAR>
static void run(int taps) {
  const int blocks = 256;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 1024 * 4);
  hipMalloc(&cyc, blocks * 8);
  hipLaunchKernelGGL((probe<FORM, BAR>), dim3(blocks), dim3(1024), 0, 0, out, taps, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<FORM, BAR>), dim3(blocks), dim3(1024), 0, 0, out, taps, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[256];
  hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < blocks; ++i) mean += h[i];
  mean /= blocks;
  const double flops = (double)blocks * 16 * taps * 64.0 * 64 * 32 * 2;
  printf("{\"form\": \"%s\", \"barrier_every_2\": %d, \"taps\": %d, \"cycles_per_tap_per_simd\": %.1f, "
         "\"floor\": 1024, \"ms\": %.3f, \"tflops\": %.1f}\n",
         FORM == 0 ? "16x16x32" : "32x32x16", BAR, taps, mean / taps, ms, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
  hipFree(cyc);
}

int main(int argc, char** argv) {
  const int taps = argc > 1 ? atoi(argv[1]) : 2048;
  run<0, 0>(taps);
  run<1, 0>(taps);
  run<0, 1>(taps);
  run<1, 1>(taps);
  return 0;
}
