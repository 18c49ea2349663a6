// Edge -> node record reductions shared by graph.hip (node_reduce / node_combine kernels) and
// the persistent small-scene BPTT kernel (ctrl.hip).
#pragma once
#include "args.h"
#include "common.h"
#include "state.h"

namespace mb {

// Both reductions below give each output node a 16-lane group: the K outgoing records of the
// node are one coalesced 16*K-byte segment (lane k reads slot k), the incoming edges are
// spread over the lanes (independent random 16-byte loads, L2-resident per step graph), and
// a fixed xor butterfly combines the lane partials -> deterministic, no atomics.
constexpr int RG = 16;             // lanes per node

DEV float grp_sum(float v) {
  static_assert(RG == 16, "16-lane groups");
  v += lane_xorf<8>(v);
  v += lane_xorf<4>(v);
  v += lane_xorf<2>(v);
  v += lane_xorf<1>(v);
  return v;
}

template <int R>
DEV void grp_sum(float4 (&g)[R]) {
#pragma unroll
  for (int q = 0; q < R; ++q) {
    g[q].x = grp_sum(g[q].x); g[q].y = grp_sum(g[q].y); g[q].z = grp_sum(g[q].z); g[q].w = grp_sum(g[q].w);
  }
}

template <int R, int SIGN>
DEV void acc_rec(float4 (&g)[R], const float4* src) {
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const float4 v = src[q];
    g[q].x += SIGN * v.x; g[q].y += SIGN * v.y; g[q].z += SIGN * v.z; g[q].w += SIGN * v.w;
  }
}
// the same from records already in registers
template <int R, int SIGN>
DEV void acc_rec_v(float4 (&g)[R], const float4 (&v)[R]) {
#pragma unroll
  for (int q = 0; q < R; ++q) {
    g[q].x += SIGN * v[q].x; g[q].y += SIGN * v[q].y; g[q].z += SIGN * v[q].z; g[q].w += SIGN * v[q].w;
  }
}

// One reverse-time step of the BPTT recursion (train.py:58-103 through autograd in the
// reference; hand-derived here):
//   G_t = dS_direct[t] + ego_t + sum_k dEc[i,k] - sum_in dEc[e]
//         + Euler adjoint of s_{t+1} = s_t + dt [v_t, a_t]  (if bptt)
// node = b*N + i, lane l of its 16-lane group (all 16 lanes call)
template <int D>
DEV void combine_node(const CombineArgs& a, long node, int l) {
#pragma clang fp contract(off)   // same arithmetic in every including file
  const int b = (int)(node / a.N), i = (int)(node % a.N);
  const int N = a.N, K = a.K;
  constexpr int R = REC<D>;
  float4 g[R];
#pragma unroll
  for (int q = 0; q < R; ++q) g[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  // the group leader's per-node records are requested before the edge gathers so that their
  // latency overlaps the gather + group reduction instead of following it
  float gp[D], gv[D], p[D], v[D], np_[D], nv[D];
#pragma unroll
  for (int q = 0; q < D; ++q) { gp[q] = gv[q] = p[q] = v[q] = np_[q] = nv[q] = 0.f; }
  if (l == 0) {
    load_rec<D>(a.dS + (long)b * a.ds_env * R, (unsigned)i, gp, gv);
    if (a.ego) load_rec<D>(a.ego + (long)b * N * R, (unsigned)i, p, v);
    if (a.Gn) load_rec<D>(a.Gn + (long)b * a.gn_env * R, (unsigned)i, np_, nv);
  }
  if (a.dEc) {
    const float4* dE = a.dEc + (long)b * N * K * R;
    for (int k = l; k < K; k += RG) acc_rec<R, 1>(g, dE + ((long)i * K + k) * R);
    const int* ptr = a.ptr + (long)b * a.ptr_env;
    const int* edges = a.edges + (long)b * a.edges_env;
    const int q0 = ptr[i], q1 = ptr[i + 1];
    for (int q = q0 + l; q < q1; q += RG) acc_rec<R, -1>(g, dE + (long)edges[q] * R);
    grp_sum<R>(g);
  }
  if (l != 0) return;
  if (a.ego) {
#pragma unroll
    for (int q = 0; q < D; ++q) { gp[q] += p[q]; gv[q] += v[q]; }
  }
  if (a.dEc) {
    // the reduced edge term, as a record
    float ep[D], ev[D];
    if (D == 2) { ep[0] = g[0].x; ep[1] = g[0].y; ev[0] = g[0].z; ev[1] = g[0].w; }
    else { ep[0] = g[0].x; ep[1] = g[0].y; ep[2] = g[0].z; ev[0] = g[R - 1].x; ev[1] = g[R - 1].y; ev[2] = g[R - 1].z; }
#pragma unroll
    for (int q = 0; q < D; ++q) { gp[q] += ep[q]; gv[q] += ev[q]; }
  }
  if (a.Gn) {
    // Euler adjoint of s_{t+1} = s_t + dt [v_t, a_t]: dp += G_p, dv += G_v + dt G_p
#pragma unroll
    for (int q = 0; q < D; ++q) { gp[q] += np_[q]; gv[q] += nv[q] + a.dt * np_[q]; }
  }
  store_rec<D>(a.Gout + (long)b * a.go_env * R, (unsigned)i, gp, gv);
}

}  // namespace mb
