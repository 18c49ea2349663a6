// Host (CPU) scenario sampler: the same parallel random-sequential-adsorption process as the
// device kernel (csrc/scenario.hip) -- identical proposals (counter-based RNG) and identical
// acceptance rule, so for a given seed the CPU and GPU trainers see bit-identical scenarios.
// The device kernel tests every candidate against all N points (one workgroup per env); here a
// uniform grid of cell size >= r makes each round O(N), and environments run on a thread pool.
#pragma once
#include <stdint.h>

namespace mbh {

struct ScenarioSpec {
  int B, N, dim;          // envs, agents, 2 or 3
  int M;                  // static obstacle points per env (fixed conflict points), may be 0
  float L, r, spread;     // side length, min separation, goal offset half-width
  uint64_t seed;
  int max_rounds;
};

// S: (B, N, 2*dim) [p, v=0]; G: (B, N, dim); obs: (B, M, dim) or null; status: (B,) rounds used
// by the goal phase (>0) or -1 if max_rounds was hit. threads <= 0: hardware concurrency.
// Returns 0, or a negative code for invalid arguments.
int sample_scenarios(const ScenarioSpec& spec, const float* obs, float* S, float* G, int* status, int threads);

// Static point-set obstacles (B, n_obs * points, dim) from a counter-based seed:
// 2-D alternates circles (radius 0.1 + 0.2u) and axis-aligned rectangles (sides 0.2 + 0.4u),
// 3-D uses spheres (radius 0.1 + 0.2u); centres are uniform in [0, L]^dim. The unit shapes
// (points x dim: circle, unit-square rectangle boundary, Fibonacci sphere) are passed in so the
// point layout is exactly env.generate_obstacle_* of the reference-compatible API.
int sample_obstacles(float* out, int B, int n_obs, int points, int dim, float L, uint64_t seed,
                     const float* circle, const float* rect, const float* sphere);

// Minimum pairwise distance among the n points of one env (O(n) grid scan, diagnostic/tests).
float min_pair_distance(const float* p, int n, int dim, int stride, float L, float cutoff);

}  // namespace mbh
