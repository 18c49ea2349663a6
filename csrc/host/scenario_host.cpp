// Host scenario sampler (see scenario_host.h). Compiled with -ffp-contract=off, like the device
// kernel, so proposals and the distance tests round identically on both sides.
#include "scenario_host.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <thread>
#include <vector>

#include "rng.h"

namespace mbh {
namespace {

// Uniform grid over [lo, lo + n*cs)^dim with cell size cs >= r: every pair closer than r lies in
// the same or adjacent cells. Coordinates outside the box are clamped to the border cells
// (clamping never increases cell distance, so the +-1 neighbourhood stays exhaustive).
struct Grid {
  int dim = 2, n = 1;
  float lo = 0.f, inv = 1.f;
  std::vector<int> head, next, touched;

  void init(int dim_, float lo_, float hi_, float cs, int npts) {
    dim = dim_;
    lo = lo_;
    n = std::max(1, (int)std::ceil((hi_ - lo_) / cs));
    inv = (float)n / (hi_ - lo_);
    size_t cells = (size_t)n * n * (dim == 3 ? n : 1);
    head.assign(cells, -1);
    next.assign(npts, -1);
    touched.clear();
  }
  int coord(float x) const {
    int c = (int)std::floor((x - lo) * inv);
    return std::min(std::max(c, 0), n - 1);
  }
  size_t cell(const int* c) const {
    return dim == 3 ? ((size_t)c[2] * n + c[1]) * n + c[0] : (size_t)c[1] * n + c[0];
  }
  void insert(int id, const float* p) {
    int c[3] = {0, 0, 0};
    for (int k = 0; k < dim; ++k) c[k] = coord(p[k]);
    const size_t h = cell(c);
    if (head[h] < 0) touched.push_back((int)h);
    next[id] = head[h];
    head[h] = id;
  }
  void clear() {
    for (int h : touched) head[h] = -1;
    touched.clear();
  }
  // f(id) for every point in the 3^dim cells around p; stops early when f returns false
  template <class F>
  bool all_near(const float* p, F&& f) const {
    int c[3] = {0, 0, 0};
    for (int k = 0; k < dim; ++k) c[k] = coord(p[k]);
    const int zlo = dim == 3 ? std::max(c[2] - 1, 0) : 0, zhi = dim == 3 ? std::min(c[2] + 1, n - 1) : 0;
    for (int z = zlo; z <= zhi; ++z)
      for (int y = std::max(c[1] - 1, 0); y <= std::min(c[1] + 1, n - 1); ++y)
        for (int x = std::max(c[0] - 1, 0); x <= std::min(c[0] + 1, n - 1); ++x) {
          const int q[3] = {x, y, z};
          for (int id = head[cell(q)]; id >= 0; id = next[id])
            if (!f(id)) return false;
        }
    return true;
  }
};

inline float d2_to(const float* a, const float* b, int dim) {
  float s = 0.f;
  for (int k = 0; k < dim; ++k) {
    const float d = a[k] - b[k];
    s += d * d;
  }
  return s;
}

void sample_env(const ScenarioSpec& sp, int b, const float* obs, float* S, float* G, int* status) {
  const int N = sp.N, D = sp.dim, M = sp.M;
  const float r2 = sp.r * sp.r;
  std::vector<float> pos((size_t)N * D), cand((size_t)N * D), starts((size_t)N * D);
  std::vector<unsigned char> placed(N);
  std::vector<int> unplaced;
  unplaced.reserve(N);
  // ids: [0,N) placed points, [N,2N) this round's candidates, [2N,2N+M) obstacle points
  float lo = -sp.spread - sp.r, hi = sp.L + sp.spread + sp.r;
  const float cs = std::max(sp.r, (hi - lo) / (D == 3 ? 96.f : 1024.f));
  Grid fixed, grid;   // obstacles (per env), placed + candidates (per round)
  fixed.init(D, lo, hi, cs, std::max(M, 1));
  for (int q = 0; q < M; ++q) fixed.insert(q, obs + (size_t)q * D);
  grid.init(D, lo, hi, cs, 2 * N);
  int st = 0;
  for (int phase = 0; phase < 2; ++phase) {
    std::fill(placed.begin(), placed.end(), 0);
    grid.clear();
    int round = 0;
    for (; round < sp.max_rounds; ++round) {
      unplaced.clear();
      for (int i = 0; i < N; ++i) {
        if (placed[i]) continue;
        unplaced.push_back(i);
        const uint64_t key = rsa_key(sp.seed, b, phase, round, i);
        for (int k = 0; k < D; ++k) {
          const float u = u01((uint64_t)D * key + (uint64_t)k);
          cand[(size_t)i * D + k] = phase == 0 ? u * sp.L : starts[(size_t)i * D + k] + (u - 0.5f) * 2.f * sp.spread;
        }
      }
      // acceptance (scenario.hip): farther than r from the origin (2-D), every obstacle point,
      // every placed point and every lower-indexed candidate of this round
      for (int i : unplaced) grid.insert(N + i, &cand[(size_t)i * D]);
      std::vector<int> accepted;
      for (int i : unplaced) {
        const float* c = &cand[(size_t)i * D];
        bool ok = true;
        if (D == 2) ok = (c[0] * c[0] + c[1] * c[1]) > r2;
        if (ok && M) ok = fixed.all_near(c, [&](int q) { return d2_to(c, obs + (size_t)q * D, D) > r2; });
        if (ok)
          ok = grid.all_near(c, [&](int id) {
            if (id < N) return d2_to(c, &pos[(size_t)id * D], D) > r2;
            const int j = id - N;
            return j >= i || d2_to(c, &cand[(size_t)j * D], D) > r2;
          });
        if (ok) accepted.push_back(i);
      }
      // rebuild: placed points only (this round's candidates leave the grid)
      for (int i : accepted) {
        placed[i] = 1;
        for (int k = 0; k < D; ++k) pos[(size_t)i * D + k] = cand[(size_t)i * D + k];
      }
      grid.clear();
      for (int i = 0; i < N; ++i)
        if (placed[i]) grid.insert(i, &pos[(size_t)i * D]);
      if (accepted.size() == unplaced.size()) break;
    }
    if (round >= sp.max_rounds) {
      st = -1;
      for (int i = 0; i < N; ++i)
        if (!placed[i])
          for (int k = 0; k < D; ++k) pos[(size_t)i * D + k] = cand[(size_t)i * D + k];
    } else if (phase == 1 && st == 0) {
      st = round + 1;
    }
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < D; ++k) {
        const float p = pos[(size_t)i * D + k];
        if (phase == 0) {
          starts[(size_t)i * D + k] = p;
          S[(size_t)i * 2 * D + k] = p;
          S[(size_t)i * 2 * D + D + k] = 0.f;
        } else {
          G[(size_t)i * D + k] = p;
        }
      }
  }
  if (status) *status = st;
}

}  // namespace

int sample_scenarios(const ScenarioSpec& sp, const float* obs, float* S, float* G, int* status, int threads) {
  if (sp.B < 1 || sp.N < 1 || (sp.dim != 2 && sp.dim != 3) || sp.M < 0 || (sp.M > 0 && !obs) || !S || !G ||
      !(sp.r > 0.f) || !(sp.L > 0.f) || sp.max_rounds < 1)
    return -1;
  const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
  const int nt = std::min(sp.B, threads > 0 ? threads : hw);
  std::atomic<int> next_env{0};
  auto work = [&]() {
    for (int b = next_env++; b < sp.B; b = next_env++)
      sample_env(sp, b, obs ? obs + (size_t)b * sp.M * sp.dim : nullptr, S + (size_t)b * sp.N * 2 * sp.dim,
                 G + (size_t)b * sp.N * sp.dim, status ? status + b : nullptr);
  };
  if (nt <= 1) {
    work();
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(work);
    for (auto& t : pool) t.join();
  }
  return 0;
}

int sample_obstacles(float* out, int B, int n_obs, int points, int dim, float L, uint64_t seed,
                     const float* circle, const float* rect, const float* sphere) {
  if (B < 0 || n_obs < 0 || points < 1 || (dim != 2 && dim != 3) || !out) return -1;
  if (dim == 2 ? (!circle || !rect) : !sphere) return -1;
  const uint64_t base = mix64(seed ^ 0x6f62737461636c65ull);
  for (int b = 0; b < B; ++b)
    for (int o = 0; o < n_obs; ++o) {
      const uint64_t key = mix64(base ^ ((uint64_t)b << 20) ^ (uint64_t)o) * 8u;
      float c[3], sc[3];
      for (int k = 0; k < dim; ++k) c[k] = u01(key + k) * L;
      const float* tpl;
      if (dim == 3) {
        tpl = sphere;
        sc[0] = sc[1] = sc[2] = 0.1f + 0.2f * u01(key + 4);
      } else if (o % 2 == 0) {
        tpl = circle;
        sc[0] = sc[1] = 0.1f + 0.2f * u01(key + 4);
      } else {
        tpl = rect;
        sc[0] = 0.2f + 0.4f * u01(key + 4);
        sc[1] = 0.2f + 0.4f * u01(key + 5);
      }
      float* dst = out + ((size_t)b * n_obs + o) * points * dim;
      for (int q = 0; q < points; ++q)
        for (int k = 0; k < dim; ++k) dst[q * dim + k] = c[k] + tpl[q * dim + k] * sc[k];
    }
  return 0;
}

float min_pair_distance(const float* p, int n, int dim, int stride, float L, float cutoff) {
  Grid g;
  const float lo = -1.f, hi = L + 1.f;
  g.init(dim, lo, hi, std::max(cutoff, (hi - lo) / 1024.f), n);
  float best2 = cutoff * cutoff;
  for (int i = 0; i < n; ++i) {
    const float* a = p + (size_t)i * stride;
    g.all_near(a, [&](int j) {
      best2 = std::min(best2, d2_to(a, p + (size_t)j * stride, dim));
      return true;
    });
    g.insert(i, a);
  }
  return std::sqrt(best2);
}

}  // namespace mbh
