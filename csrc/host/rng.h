// Counter-based RNG shared by the host runtime and (bit-identically) the device sampler
// csrc/scenario.hip: splitmix64 finaliser, uniform floats with 24 random bits.
#pragma once
#include <stdint.h>

namespace mbh {

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

inline float u01(uint64_t key) { return (float)(mix64(key) >> 40) * (1.0f / 16777216.0f); }

// per-(seed, env, phase, round, agent) key of the parallel-RSA proposal (scenario.hip)
inline uint64_t rsa_key(uint64_t seed, int env, int phase, int round, int agent) {
  uint64_t key = mix64(seed ^ ((uint64_t)env << 1));
  key = mix64(key ^ ((uint64_t)phase << 7) ^ ((uint64_t)round << 9));
  return key ^ ((uint64_t)agent << 24);
}

}  // namespace mbh
