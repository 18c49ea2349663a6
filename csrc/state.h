// D-dimensional double-integrator node records (D = 2: the reference; D = 3: config #5).
// A node record is REC<D> float4s: D = 2 -> (x, y, vx, vy); D = 3 -> (x, y, z, 0), (vx, vy, vz, 0).
// Buffer strides (s_env, s_step, ...) passed to the kernels are in RECORDS.
#pragma once
#include "common.h"

namespace mb {

template <int D> constexpr int REC = (D == 2) ? 1 : 2;

template <int D>
DEV void load_rec(const float4* base, unsigned i, float (&p)[D], float (&v)[D]) {
  if constexpr (D == 2) {
    const float4 a = base[i];
    p[0] = a.x; p[1] = a.y; v[0] = a.z; v[1] = a.w;
  } else {
    const float4 a = base[2 * i], b = base[2 * i + 1];
    p[0] = a.x; p[1] = a.y; p[2] = a.z;
    v[0] = b.x; v[1] = b.y; v[2] = b.z;
  }
}

// the same unpacking from records already in registers
template <int D>
DEV void load_rec_regs(const float4 (&r)[REC<D>], float (&p)[D], float (&v)[D]) {
  if constexpr (D == 2) {
    p[0] = r[0].x; p[1] = r[0].y; v[0] = r[0].z; v[1] = r[0].w;
  } else {
    p[0] = r[0].x; p[1] = r[0].y; p[2] = r[0].z;
    v[0] = r[1].x; v[1] = r[1].y; v[2] = r[1].z;
  }
}

template <int D>
DEV void store_rec(float4* base, unsigned i, const float (&p)[D], const float (&v)[D]) {
  if constexpr (D == 2) {
    base[i] = make_float4(p[0], p[1], v[0], v[1]);
  } else {
    base[2 * i] = make_float4(p[0], p[1], p[2], 0.f);
    base[2 * i + 1] = make_float4(v[0], v[1], v[2], 0.f);
  }
}

// sum_d x_d^2 in coordinate order (the oracle's order)
template <int D>
DEV float sqsum(const float (&x)[D]) {
  float s = x[0] * x[0];
#pragma unroll
  for (int q = 1; q < D; ++q) s = s + x[q] * x[q];
  return s;
}

}  // namespace mb
