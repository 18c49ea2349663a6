// Time-to-collision test shared by the scan kernels (scan.hip) and the persistent small-scene
// rollout (ctrl.hip): reference core.py:187-209 / 212-231. Include it after
// `#pragma clang fp contract(off)`: the decisions must match the PyTorch oracle bit for bit
// (separately rounded products, sums in coordinate order).
#pragma once
#include "common.h"

namespace mb {

// D-dimensional TTC test on relative position p and velocity v (sums in coordinate order)
template <int D>
DEV bool ttc_danger(const float (&p)[D], const float (&v)[D], float r2, float ttc) {
  float alpha = v[0] * v[0], pv = p[0] * v[0], pp = p[0] * p[0];
#pragma unroll
  for (int q = 1; q < D; ++q) { alpha = alpha + v[q] * v[q]; pv = pv + p[q] * v[q]; pp = pp + p[q] * p[q]; }
  float beta = 2.0f * pv;
  float gamma = pp - r2;
  float disc = beta * beta - (4.0f * alpha) * gamma;
  bool dist_d = gamma < 0.f;
  bool two_pos = (disc > 0.f) && (gamma > 0.f) && (beta < 0.f);
  float t2 = (2.0f * alpha) * ttc;
  float bt = beta + t2;
  bool lt = ((-beta) - t2 < 0.f) || (bt * bt < disc);
  return dist_d || (two_pos && lt);
}

// (d2, index) packed into one 64-bit key: d2 >= 0, so its IEEE bits order like the values and
// a single unsigned compare is the lexicographic (distance, lower index) order.
DEV uint64_t knn_key(float d2, unsigned j) { return ((uint64_t)__float_as_uint(d2) << 32) | j; }

}  // namespace mb
