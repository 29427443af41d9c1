// Store-bandwidth probe for the conv_in epilogue's write pattern: 1.07 GB of bf16 [4M pixels x 128 ch] written
//   0: per wave 64 pixels x 32 channels (64-byte row slices, 256-byte stride: conv_in8_kernel's pattern)
//   1: per wave 16 pixels x 128 channels (whole 256-byte rows, 1 KB contiguous per instruction)
//   2: as 1 with nontemporal stores
//   3: as 0 with nontemporal stores
// persistent grid of 3 x CUs blocks of 256 threads, 64-pixel tiles. hipcc --offload-arch=gfx950 -O3 -o store_probe store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void store_kernel(uint4* out, int ntiles) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  const u4v v = u4v{(unsigned)lane, 1u, 2u, 3u};
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long m0 = (long)t * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      long idx;  // in uint4 units: a pixel row is 16 of them
      if (MODE == 0 || MODE == 3) {
        const int row = 16 * k + (lane >> 2), ch = lane & 3;
        idx = (m0 + row) * 16 + wave * 4 + ch;
      } else {
        const int row = wave * 16 + 4 * k + (lane >> 4), ch = lane & 15;
        idx = (m0 + row) * 16 + ch;
      }
      if (MODE >= 2) __builtin_nontemporal_store(v, reinterpret_cast<u4v*>(out) + idx);
      else reinterpret_cast<u4v*>(out)[idx] = v;
    }
  }
}

int main() {
  const long M = 16L * 512 * 512;
  const size_t bytes = M * 128 * 2;
  uint4* out;
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int ntiles = (int)(M / 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int grid_mul : {3, 8}) {
    for (int mode = 0; mode < 4; ++mode) {
      auto run = [&]() {
        const int g = grid_mul * cus;
        if (mode == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(g), dim3(256), 0, 0, out, ntiles);
        if (mode == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(g), dim3(256), 0, 0, out, ntiles);
        if (mode == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(g), dim3(256), 0, 0, out, ntiles);
        if (mode == 3) hipLaunchKernelGGL(store_kernel<3>, dim3(g), dim3(256), 0, 0, out, ntiles);
      };
      run();
      hipDeviceSynchronize();
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0, 0);
        for (int i = 0; i < 10; ++i) run();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms / 10 < best) best = ms / 10;
      }
      printf("{\"mode\": %d, \"grid\": %d, \"ms\": %.4f, \"TBps\": %.2f}\n", mode, grid_mul * cus, best, bytes / best / 1e9);
    }
  }
  hipFree(out);
  return 0;
}
