// Dropout / GELU math shared by the standalone transformer epilogue kernels (dropout.hip)
// and the FFN GEMM epilogues of the implicit-GEMM kernel (conv_igemm_impl.h): the keep mask
// of element e is a counter-based hash of (seed, e / 8 chunk), so any kernel that knows an
// element's flat index regenerates the same mask.
#pragma once
#include "common.h"

namespace fdt {
namespace drop {

__device__ __forceinline__ uint64_t drop_hash(uint64_t i, uint64_t seed) {
  uint64_t x = i ^ seed;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// keep mask of the 8 elements [8c, 8c + 8): bit j set = element kept
__device__ __forceinline__ uint32_t keep8(long c, uint64_t seed, uint32_t thr) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t h = drop_hash((uint64_t)c * 4 + j, seed);
    m |= (uint32_t)((uint32_t)h >= thr) << (2 * j);
    m |= (uint32_t)((uint32_t)(h >> 32) >= thr) << (2 * j + 1);
  }
  return m;
}

__device__ __forceinline__ float gelu_erf(float a) { return 0.5f * a * (1.f + erff(a * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float a) {
  const float cdf = 0.5f * (1.f + erff(a * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * a * a);
  return cdf + a * pdf;
}

__device__ __forceinline__ uint64_t live_seed(uint64_t seed, const uint64_t* seed_ptr) {
  return seed_ptr != nullptr ? (seed ^ *seed_ptr) : seed;
}

}  // namespace drop
}  // namespace fdt
