// Prints which LDS element each lane / element of ds_read_b64_tr_b16 returns when lane L
// supplies the address of the 4-element chunk L (element values = their LDS index).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short s[256];
  for (int i = threadIdx.x; i < 256; i += 64) s[i] = (short)i;
  __syncthreads();
  typedef __attribute__((address_space(3))) s4 ls4;
  s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ls4*)(s + 4 * threadIdx.x));
  for (int e = 0; e < 4; ++e) out[threadIdx.x * 4 + e] = r[e];
}
int main() {
  short* d; hipMalloc(&d, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) printf(" %3d(c%2d.%d)", h[4 * l + e], h[4 * l + e] / 4, h[4 * l + e] % 4);
    printf("\n");
  }
  return 0;
}
