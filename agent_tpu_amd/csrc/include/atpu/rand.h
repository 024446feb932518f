// Counter-based random init shared by the GPU kernel (kernels/rand_init.hip) and its CPU
// twin (runtime/rand_host.cpp): element i of stream `sid` under `seed` is a pure function
// of (seed, sid, i), so a model's random-init weights are built ON the GPU in well under a
// millisecond (no host randn of the whole pack, no H2D copy) and bit-identical to what the
// host builds for the fp32 oracle / HF-parity tests.
//
// Value: Irwin-Hall(4) of the four 16-bit lanes of splitmix64(seed, sid, i), centred and
// scaled to unit variance (support +-3.46 sigma; mean 0, variance 1, kurtosis -0.3): integer
// math, then ONE fp32 multiply by the caller's scale and a round-to-nearest-even cut to bf16
// on the float bits. Every step is exact or a single correctly rounded IEEE operation, so
// host and device agree bit for bit (no transcendentals, no contraction opportunity).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ATPU_HD __host__ __device__ __forceinline__
#else
#define ATPU_HD inline
#endif

namespace atpu {
namespace rnd {

ATPU_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// stream key of (seed, sid): mixed once per tensor
ATPU_HD uint64_t stream_key(uint64_t seed, uint64_t sid) {
  return splitmix64(splitmix64(seed * 0xD1B54A32D192ED03ull + 0x8CB92BA72F3D8DD7ull) ^ (sid * 0xABC98388FB8FAC03ull));
}

// centred Irwin-Hall(4) sum in [-131070, 131070] (integer; variance 4 * (65536^2 - 1) / 12)
ATPU_HD int32_t ih4(uint64_t key, uint64_t i) {
  const uint64_t h = splitmix64(key ^ (i * 0x9E3779B97F4A7C15ull));
  const int32_t s = (int32_t)(h & 0xFFFF) + (int32_t)((h >> 16) & 0xFFFF) + (int32_t)((h >> 32) & 0xFFFF) +
                    (int32_t)(h >> 48);
  return s - 131070;
}

// 1 / sqrt(4 * (65536^2 - 1) / 12): multiply ih4 by (std * kIh4Norm) for an N(0, std^2)-like value
constexpr double kIh4Norm = 2.6428997921303014e-05;

// fp32 -> bf16 bits, round to nearest even (finite inputs)
ATPU_HD uint16_t f2bf_rne(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

}  // namespace rnd
}  // namespace atpu
