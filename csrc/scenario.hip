// K11: on-device scenario sampler (reference core.py:45-71 is a sequential host rejection
// loop: 81 ms per env at N=1024, ~5 s per 64-env iteration).
//
// One workgroup per env runs *parallel* random sequential adsorption in rounds: every
// unplaced agent proposes a candidate (counter-based RNG keyed by seed/env/agent/round);
// a candidate is accepted if it is farther than r from every placed point, from every
// lower-indexed candidate of the same round, and from the origin (the reference's unfilled
// zero rows also exclude the origin). Starts are uniform in [0, L]^2, L = sqrt(max(1,N/8));
// goals are start + U(-0.5,0.5)^2 with the same separation rule among goals.
// Invariants (min pair distance > r, goal offsets in +-0.5, v = 0, density 8/unit^2) are
// tested against the host sampler. LDS: 25 B per agent (N <= ~6000); larger envs keep the same
// arrays in a per-env global workspace (a.ws) with a full-resolution cell grid: identical results
// (acceptance is order independent); its round barriers carry agent-scope fences (round_sync).
#include "common.h"
#include "args.h"
#include "state.h"

// no fp contraction: proposals and distance tests round exactly like the host runtime
// (csrc/host/scenario_host.cpp), which reproduces this sampler bit for bit on the CPU
#pragma clang fp contract(off)

namespace mb {


constexpr int SC_BLOCK = 1024;
constexpr size_t SC_LDS_MAX = 160 * 1024 - 64;

__host__ __device__ inline int sc_cells(int G, int D) { return D == 3 ? G * G * G : G * G; }

template <int D>
DEV float d2_to(const float* c, const float* q) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < D; ++k) { const float d = c[k] - q[k]; s += d * d; }
  return s;
}

// Cell grid over [lo, lo + G*cs)^D (cs >= r, coordinates clamped to the border cells, which
// never increases cell distance): every conflict of a candidate lies in its 3^D neighbourhood.
struct CellGrid {
  float lo, inv;
  int G;
  DEV int coord(float x) const { return min(max((int)floorf((x - lo) * inv), 0), G - 1); }
};

template <int D>
DEV int cell_of(const CellGrid& g, const float* p) {
  int c = g.coord(p[D - 1]);
#pragma unroll
  for (int k = D - 2; k >= 0; --k) c = c * g.G + g.coord(p[k]);
  return c;
}

// every id in the 3^D cells around p: f(id) -> false stops the scan
template <int D, class F>
DEV bool grid_all(const CellGrid& g, const int* head, const int* next, const float* p, F&& f) {
  int c[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < D; ++k) c[k] = g.coord(p[k]);
  const int zlo = D == 3 ? max(c[2] - 1, 0) : 0, zhi = D == 3 ? min(c[2] + 1, g.G - 1) : 0;
  for (int z = zlo; z <= zhi; ++z)
    for (int y = max(c[1] - 1, 0); y <= min(c[1] + 1, g.G - 1); ++y)
      for (int x = max(c[0] - 1, 0); x <= min(c[0] + 1, g.G - 1); ++x)
        for (int id = head[(z * g.G + y) * g.G + x]; id >= 0; id = next[id])
          if (!f(id)) return false;
  return true;
}

// D-dimensional variant: positions in [0, L]^D, goals start + U(-spread, spread)^D, and the
// optional static obstacle points (per env) as fixed conflict points of both phases. The
// origin exclusion of the reference's zero rows is kept for D = 2 (core.py:45-71).
// Each round rebuilds an LDS cell list of every agent's current point (placed position or
// this round's candidate; lists built with LDS atomics, whose order does not matter because
// acceptance needs *all* tests to pass), so a round is O(N) instead of O(N^2).
// Barrier of the round loop. With the arrays in a global workspace the cell heads are written
// by atomics (performed in L2) and read by plain loads, and every array is rewritten each round:
// a plain load may hit an L1 line left from an earlier round, and a stale head links into the
// previous round's list -- a cycle the cell walk never leaves. Agent-scope fences around the
// barrier publish this round's stores / atomics to L2 and drop the workgroup's L1 lines.
DEV void round_sync(bool global_ws) {
  if (global_ws) __threadfence();
  __syncthreads();
  if (global_ws) __threadfence();
}

template <int D>
__global__ __launch_bounds__(SC_BLOCK) void scenario_kernel(ScenArgs a, CellGrid grid) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* base = a.ws ? a.ws + (long)blockIdx.x * a.ws_env : smem;
  float* pos = reinterpret_cast<float*>(base);           // accepted points of this phase (N x D)
  float* cand = pos + a.N * D;                            // this round's candidates
  float* starts = cand + a.N * D;                         // phase-0 result (goal anchors)
  float* obs = starts + a.N * D;                          // M x D obstacle points
  int* next = reinterpret_cast<int*>(obs + a.M * D);      // N: cell-list links
  int* head = next + a.N;                                 // G^D: cell-list heads
  unsigned char* placed = reinterpret_cast<unsigned char*>(head + sc_cells(grid.G, D));
  __shared__ int n_unplaced;
  const int b = blockIdx.x;
  const float r2 = a.r * a.r;
  const int ncell = sc_cells(grid.G, D);
  const bool gws = a.ws != nullptr;
  for (int q = threadIdx.x; q < a.M * D; q += SC_BLOCK) obs[q] = a.obs[(long)b * a.M * D + q];
  int status = 0;
  for (int phase = 0; phase < 2; ++phase) {
    for (int i = threadIdx.x; i < a.N; i += SC_BLOCK) placed[i] = 0;
    round_sync(gws);
    int round = 0;
    for (; round < a.max_rounds; ++round) {
      for (int c = threadIdx.x; c < ncell; c += SC_BLOCK) head[c] = -1;
      for (int i = threadIdx.x; i < a.N; i += SC_BLOCK) {
        if (placed[i]) continue;
        unsigned long long key = a.seed;
        key = mix64(key ^ ((unsigned long long)b << 1));
        key = mix64(key ^ ((unsigned long long)phase << 7) ^ ((unsigned long long)round << 9));
        key = key ^ ((unsigned long long)i << 24);
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const float u = u01(D * key + k);
          cand[i * D + k] = (phase == 0) ? u * a.L : starts[i * D + k] + (u - 0.5f) * 2.f * a.spread;
        }
      }
      round_sync(gws);
      for (int i = threadIdx.x; i < a.N; i += SC_BLOCK) {
        const int c = cell_of<D>(grid, (placed[i] ? pos : cand) + i * D);
        next[i] = atomicExch(&head[c], i);
      }
      round_sync(gws);
      for (int i = threadIdx.x; i < a.N; i += SC_BLOCK) {
        if (placed[i]) continue;
        const float* c = cand + i * D;
        bool ok = true;
        if (D == 2) ok = (c[0] * c[0] + c[1] * c[1]) > r2;
        for (int q = 0; q < a.M && ok; ++q) ok = d2_to<D>(c, obs + q * D) > r2;
        // placed points and lower-indexed candidates of this round (placed[j] may turn 2
        // concurrently: still a candidate of this round, tested against cand either way)
        if (ok)
          ok = grid_all<D>(grid, head, next, c, [&](int j) {
            if (placed[j] == 1) return d2_to<D>(c, pos + j * D) > r2;
            return j >= i || d2_to<D>(c, cand + j * D) > r2;
          });
        if (ok) placed[i] = 2;
      }
      round_sync(gws);
      if (threadIdx.x == 0) n_unplaced = 0;
      round_sync(gws);
      int local = 0;
      for (int i = threadIdx.x; i < a.N; i += SC_BLOCK) {
        if (placed[i] == 2) {
          placed[i] = 1;
#pragma unroll
          for (int k = 0; k < D; ++k) pos[i * D + k] = cand[i * D + k];
        } else if (placed[i] == 0) ++local;
      }
      if (local) atomicAdd(&n_unplaced, local);
      round_sync(gws);
      if (n_unplaced == 0) break;
    }
    if (round >= a.max_rounds) {
      status = -1;   // flagged to the host; keep the last proposals so outputs are defined
      for (int i = threadIdx.x; i < a.N; i += SC_BLOCK)
        if (placed[i] == 0)
          for (int k = 0; k < D; ++k) pos[i * D + k] = cand[i * D + k];
      round_sync(gws);
    }
    else if (phase == 1 && status == 0) status = round + 1;
    for (int i = threadIdx.x; i < a.N; i += SC_BLOCK) {
      const float* p = pos + i * D;
      if (phase == 0) {
        float pp[D], vv[D];
#pragma unroll
        for (int k = 0; k < D; ++k) { pp[k] = p[k]; vv[k] = 0.f; starts[i * D + k] = p[k]; }
        store_rec<D>(a.S + (long)b * a.s_env * REC<D>, (unsigned)i, pp, vv);
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) a.G[((long)b * a.N + i) * D + k] = p[k];
      }
    }
    round_sync(gws);
  }
  if (threadIdx.x == 0 && a.status) a.status[b] = status;
}

}  // namespace mb

extern "C" int mb_scenario(const mb::ScenArgs* a, hipStream_t st) {
  using namespace mb;
  const int D = a->dim;
  if (D != 2 && D != 3) return -1;
  // fixed arrays, then as many grid cells (cell size >= r) as the remaining LDS holds
  const size_t base = (size_t)(3 * a->N + a->M) * D * 4 + (size_t)a->N * 4 + (size_t)a->N + 16;
  CellGrid g;
  g.lo = -a->spread - a->r;
  const float span = a->L + 2.f * (a->spread + a->r);
  int G = max(1, (int)floorf(span / a->r));
  size_t lds;
  if (a->ws) {
    // global workspace: full-resolution grid; a->ws_env must hold scenario_ws_bytes(N, M, D)
    if ((size_t)a->ws_env < base + 4 * (size_t)sc_cells(G, D)) return -3;
    lds = 0;
  } else {
    if (base + 4 * (size_t)sc_cells(1, D) > SC_LDS_MAX) return -2;
    const size_t room = (SC_LDS_MAX - base) / 4;
    while (G > 1 && (size_t)sc_cells(G, D) > room) --G;
    lds = base + 4 * (size_t)sc_cells(G, D);
  }
  g.G = G;
  g.inv = (float)G / span;
  if (D == 3) {
    (void)hipFuncSetAttribute((const void*)scenario_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(scenario_kernel<3>, dim3(a->B), dim3(SC_BLOCK), lds, st, *a, g);
  } else {
    (void)hipFuncSetAttribute((const void*)scenario_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(scenario_kernel<2>, dim3(a->B), dim3(SC_BLOCK), lds, st, *a, g);
  }
  return (int)hipGetLastError();
}
