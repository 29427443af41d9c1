/* ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
 * CPU twin of rdeic_fill_uniform (rdeic_amd/csrc/elementwise.hip): counter-based synthetic
 * weights so the reference modules (golden fixtures), the CPU oracle and the HIP path all
 * see bit-identical parameters without shipping a checkpoint:
 *   out[i] = float((splitmix64(seed + i) >> 40) - 2^23) * scale + offset   (two fp32 roundings) */
#include <stdint.h>

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_fill_uniform(float* out, int64_t n, uint64_t seed, float scale, float offset) {
  for (int64_t i = 0; i < n; ++i) {
    uint64_t r = splitmix64(seed + (uint64_t)i);
    volatile float u = (float)((int32_t)(r >> 40) - 8388608);
    volatile float m = u * scale; /* volatile: forbid contraction into an fma */
    out[i] = m + offset;
  }
}
