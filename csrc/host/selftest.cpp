// Standalone self-test of the host runtime, built by tests/test_host_native.py with
// -fsanitize=address,undefined (sanitizers on the host-side native code).
// Exit code 0 = all invariants hold.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "rng.h"
#include "scenario_host.h"

static int fails = 0;
#define CHECK(c, ...)                        \
  do {                                       \
    if (!(c)) {                              \
      std::fprintf(stderr, __VA_ARGS__);     \
      std::fprintf(stderr, "\n");            \
      ++fails;                               \
    }                                        \
  } while (0)

static void run(int B, int N, int dim, int M, unsigned long long seed) {
  const float r = 0.07f, spread = 0.5f;
  const float L = dim == 2 ? std::sqrt(std::fmax(1.f, N / 8.f)) : std::cbrt(std::fmax(1.f, N / 8.f));
  std::vector<float> obs((size_t)B * M * dim), S((size_t)B * N * 2 * dim), G((size_t)B * N * dim);
  std::vector<float> S2(S.size()), G2(G.size());
  std::vector<int> st(B), st2(B);
  for (size_t q = 0; q < obs.size(); ++q) obs[q] = L * mbh::u01(seed * 977 + q);
  mbh::ScenarioSpec sp{B, N, dim, M, L, r, spread, seed, 256};
  CHECK(mbh::sample_scenarios(sp, M ? obs.data() : nullptr, S.data(), G.data(), st.data(), 4) == 0, "rc");
  CHECK(mbh::sample_scenarios(sp, M ? obs.data() : nullptr, S2.data(), G2.data(), st2.data(), 1) == 0, "rc1");
  CHECK(std::memcmp(S.data(), S2.data(), S.size() * 4) == 0 && std::memcmp(G.data(), G2.data(), G.size() * 4) == 0,
        "thread-count dependence (B=%d N=%d dim=%d)", B, N, dim);
  for (int b = 0; b < B; ++b) {
    CHECK(st[b] > 0, "env %d did not converge", b);
    const float* s = &S[(size_t)b * N * 2 * dim];
    const float* g = &G[(size_t)b * N * dim];
    const float ds = mbh::min_pair_distance(s, N, dim, 2 * dim, L, 1.f);
    const float dg = mbh::min_pair_distance(g, N, dim, dim, L + 1.f, 1.f);
    CHECK(N < 2 || ds > r, "starts too close: %g", ds);
    CHECK(N < 2 || dg > r, "goals too close: %g", dg);
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < dim; ++k) {
        const float p = s[i * 2 * dim + k];
        CHECK(p >= 0.f && p <= L, "start out of box");
        CHECK(s[i * 2 * dim + dim + k] == 0.f, "nonzero velocity");
        CHECK(std::fabs(g[i * dim + k] - p) <= spread + 1e-6f, "goal offset");
      }
    for (int q = 0; q < M; ++q)
      for (int i = 0; i < N; ++i) {
        float d2 = 0.f, e2 = 0.f;
        for (int k = 0; k < dim; ++k) {
          const float o = obs[((size_t)b * M + q) * dim + k];
          d2 += (s[i * 2 * dim + k] - o) * (s[i * 2 * dim + k] - o);
          e2 += (g[i * dim + k] - o) * (g[i * dim + k] - o);
        }
        CHECK(d2 > r * r && e2 > r * r, "obstacle conflict");
      }
  }
}

int main() {
  run(3, 1, 2, 0, 1);
  run(4, 8, 2, 0, 2);
  run(4, 300, 2, 0, 3);
  run(2, 1024, 2, 24, 4);
  run(3, 200, 3, 36, 5);
  run(2, 1024, 3, 96, 6);
  mbh::ScenarioSpec bad{0, 8, 2, 0, 1.f, 0.07f, 0.5f, 0, 256};
  CHECK(mbh::sample_scenarios(bad, nullptr, nullptr, nullptr, nullptr, 1) < 0, "bad args accepted");
  std::printf(fails ? "FAIL %d\n" : "OK\n", fails);
  return fails ? 1 : 0;
}
