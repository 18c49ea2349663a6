// pybind11 module macbf_gnn_amd._host: the CPU-side native runtime (no HIP dependency).
// Arguments are host buffer addresses; shapes/dtypes are validated in macbf_gnn_amd/ops/host.py.
#include <pybind11/pybind11.h>

#include "scenario_host.h"

namespace py = pybind11;
typedef unsigned long long u64;

static int sample_scenarios(u64 S, u64 G, u64 obs, u64 status, int B, int N, int dim, int M, float L, float r,
                            float spread, u64 seed, int max_rounds, int threads) {
  mbh::ScenarioSpec sp{B, N, dim, M, L, r, spread, (uint64_t)seed, max_rounds};
  py::gil_scoped_release nogil;
  return mbh::sample_scenarios(sp, reinterpret_cast<const float*>(obs), reinterpret_cast<float*>(S),
                               reinterpret_cast<float*>(G), reinterpret_cast<int*>(status), threads);
}

static float min_pair_distance(u64 p, int n, int dim, int stride, float L, float cutoff) {
  py::gil_scoped_release nogil;
  return mbh::min_pair_distance(reinterpret_cast<const float*>(p), n, dim, stride, L, cutoff);
}

static int sample_obstacles(u64 out, int B, int n_obs, int points, int dim, float L, u64 seed, u64 circle,
                            u64 rect, u64 sphere) {
  py::gil_scoped_release nogil;
  return mbh::sample_obstacles(reinterpret_cast<float*>(out), B, n_obs, points, dim, L, (uint64_t)seed,
                               reinterpret_cast<const float*>(circle), reinterpret_cast<const float*>(rect),
                               reinterpret_cast<const float*>(sphere));
}

PYBIND11_MODULE(_host, m) {
  m.doc() = "macbf_gnn_amd host runtime (scenario sampler)";
  m.def("sample_scenarios", &sample_scenarios);
  m.def("sample_obstacles", &sample_obstacles);
  m.def("min_pair_distance", &min_pair_distance);
}
