// anx/rng.hpp — counter-based deterministic RNG shared bit-for-bit with the Python package
// (anx.utils.init). value(seed, stream, i) depends only on its arguments, so host, device and
// numpy implementations generate identical tensors in any order or in parallel.
#pragma once
#include <cstddef>
#include <cstdint>

namespace anx::rng {

enum Stream : uint64_t { kInput = 0, kW1 = 1, kB1 = 2, kW2 = 3, kB2 = 4, kExtra = 8 };

inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// Uniform float in [0, 1) with 24 random bits.
inline float uniform(uint64_t seed, uint64_t stream, uint64_t i) {
  const uint64_t key = (seed << 32) ^ (stream << 56) ^ i;
  return static_cast<float>(splitmix64(key) >> 40) * (1.0f / 16777216.0f);
}

}  // namespace anx::rng
