// Counter-based hashing used by the synthetic generators. Integer-only and
// exact in fp64, so the device generators and the numpy oracle
// (oracle/matrices.py) produce bit-identical matrices and right-hand sides.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace kr {

__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Uniform in [0,1) with 53 random bits: exactly representable.
__host__ __device__ inline double unit_uniform(uint64_t seed, uint64_t a, uint64_t b) {
  const uint64_t key =
      (seed * 0x9E3779B97F4A7C15ull) ^ (a * 0xC2B2AE3D27D4EB4Full) ^ (b * 0x165667B19E3779F9ull);
  return (double)(mix64(key) >> 11) * 0x1.0p-53;
}

// Synthetic right-hand side: b_i = 2u - 1 (exact).
__host__ __device__ inline double rhs_value(uint64_t seed, uint64_t i) {
  return 2.0 * unit_uniform(seed, i, 0xB5ull) - 1.0;
}

// Symmetric banded value of the pair (lo, lo + o): -u.
__host__ __device__ inline double band_value(uint64_t seed, uint64_t lo, uint64_t o) {
  return -unit_uniform(seed, lo, o);
}

}  // namespace kr
