// 16x16x32 building blocks shared by csrc/cbf16.h, csrc/ctrl16.h and csrc/node16.h
// (v_mfma_f32_16x16x32_bf16 / _f16; lane l: n = l & 15, g = l >> 4). x3 build: fp32-accurate
// split operands (hi + lo planes, three MFMAs per product); the 1-pass builds (bf16 / fp16, prec.h)
// carry only the hi plane -- the `l` members are never written or read and the lo-plane reads
// and stores compile away.
//   A (16x32): elem j = A[n][8g + j]   B (32x16): elem j = B[8g + j][n]   C: reg i = C[4g + i][n]
// A packed C tile (Pk4) is the B operand of the next layer with k(8g + j) = 32s + 16(j >> 2) + 4g +
// (j & 3) for the tile pair (2s, 2s + 1) (layout.kacc16); weights are packed to match.
#pragma once

// Workgroups per CU of the 8-wave CBF (cbf16.h) and edge (ctrl16.h) backward kernels: one (two
// waves per SIMD at <= 256 registers). The 1-pass builds fit two in LDS (<= 80 KiB each) but only
// at <= 128 registers: the CBF kernel then spills 96 registers, the edge kernel 6, and both run
// slower (bf16 headline 6.48 vs 6.25 ms, profiles/r4_k16/) -- CBF16_WGPC / E16_WGPC = 2 build
// that variant. The launch grids follow (mb_k16_wg_per_cu).
constexpr int CBF16_WGPC = 1;
constexpr int E16_WGPC = 1;

namespace mb {
namespace MB_PREC {

struct Pk4 { h16x4 h, l; };

DEV f32x4 mfma16(const h16x8& a, const h16x8& b, const f32x4& c) {
#if MB_FP16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}
// x3 product, small terms first (same order as mma()); one MFMA in the 1-pass builds
DEV f32x4 mma16(const Fr& a, const Fr& b, f32x4 c) {
  if constexpr (X3) {
    c = mfma16(a.l, b.h, c);
    c = mfma16(a.h, b.l, c);
  }
  return mfma16(a.h, b.h, c);
}
DEV f32x4 mma16_bx(const Fr& a, const h16x8& b, f32x4 c) {
  if constexpr (X3) c = mfma16(a.l, b, c);
  return mfma16(a.h, b, c);
}
DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
DEV f32x4 relu4(f32x4 c) {
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = relu_f(c[i]);
  return c;
}
DEV Pk4 to_pk4(const f32x4& c) {
  Pk4 p;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p.h[i] = (h16)c[i];
    if constexpr (X3) p.l[i] = (h16)(c[i] - (float)p.h[i]);
  }
  return p;
}
// B operand of K-step s from the packed tiles 2s (j < 4) and 2s + 1 (j >= 4)
DEV Fr pk4_fr(const Pk4& t0, const Pk4& t1) {
  Fr f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f.h[i] = t0.h[i]; f.h[4 + i] = t1.h[i];
    if constexpr (X3) { f.l[i] = t0.l[i]; f.l[4 + i] = t1.l[i]; }
  }
  return f;
}
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
// d *= relu'(pre) with H = relu(pre) packed (both planes of d masked by H's hi plane)
DEV void mask_pk4(Pk4& d, const Pk4& H) {
  const u32x2v m = __builtin_bit_cast(u32x2v, H.h);
  u32x2v dh = __builtin_bit_cast(u32x2v, d.h);
  dh[0] = mask_nz16x2(dh[0], m[0]); dh[1] = mask_nz16x2(dh[1], m[1]);
  d.h = __builtin_bit_cast(h16x4, dh);
  if constexpr (X3) {
    u32x2v dl = __builtin_bit_cast(u32x2v, d.l);
    dl[0] = mask_nz16x2(dl[0], m[0]); dl[1] = mask_nz16x2(dl[1], m[1]);
    d.l = __builtin_bit_cast(h16x4, dl);
  }
}
// two ds_read_b64_tr_b16: lane (n, g) receives img[r1 + j][col(n)] (j < 4), img[r1 + d2 + j - 4]
// (j >= 4), where lane (q, p) of each 16-lane group addresses row r1 + q at column c + 4p
DEV h16x8 tr_pair16(const h16* img, int stride, int r1, int d2, int colp, int lane) {
  const int q = (lane & 15) >> 2;
  const LDS_AS h16* im = lds_ptr(img);
  const LDS_AS h16* a1 = im + (r1 + q) * stride + colp;
  const LDS_AS h16* a2 = a1 + d2 * stride;
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
  const s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a2));
  const h16x4 b1 = __builtin_bit_cast(h16x4, v1), b2 = __builtin_bit_cast(h16x4, v2);
  h16x8 r;
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}
// stage operand over evaluations: lane (n, g) elem j = img[e0 + 8g + j][c0 + n]
DEV h16x8 tr16(const h16* img, int stride, int e0, int c0, int lane) {
  return tr_pair16(img, stride, e0 + 8 * (lane >> 4), 4, c0 + 4 * (lane & 3), lane);
}
DEV Fr tr16_fr(const h16* img, int stride, int lo, int e0, int c0, int lane) {
  Fr r;
  r.h = tr16(img, stride, e0, c0, lane);
  if constexpr (X3) r.l = tr16(img + lo, stride, e0, c0, lane);
  return r;
}
// store a packed C tile (rows 16mt + 4g + i of evaluation row `erow`) into an edge-major image
DEV void store4(h16* img, int stride, int lo, int erow, int mt, int g, const Pk4& v) {
  h16* p = img + erow * stride + 16 * mt + 4 * g;
  *reinterpret_cast<h16x4*>(p) = v.h;
  if constexpr (X3) *reinterpret_cast<h16x4*>(p + lo) = v.l;
}
// row-major slab tile write: rows 16mt + 4g + i, column 16nt + n
DEV void write_tile16(float* P, int ncols, int mt, int nt, const f32x4& c, int lane) {
  const int n = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) P[(16 * mt + 4 * g + i) * ncols + 16 * nt + n] = c[i];
}

// sum of v[k] over the 16 lanes of this lane's 16-lane row, returned in lane n for k = n (a
// butterfly reduce-scatter: each xor step halves the values a lane carries; fixed order)
DEV float reduce_scatter16(float (&v)[16], int n) {
  float a8[8], a4[4], a2[2];
  const bool b3 = (n >> 3) & 1, b2 = (n >> 2) & 1, b1 = (n >> 1) & 1, b0 = n & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float keep = b3 ? v[8 + k] : v[k], send = b3 ? v[k] : v[8 + k];
    a8[k] = keep + lane_xorf<8>(send);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float keep = b2 ? a8[4 + k] : a8[k], send = b2 ? a8[k] : a8[4 + k];
    a4[k] = keep + lane_xorf<4>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float keep = b1 ? a4[2 + k] : a4[k], send = b1 ? a4[k] : a4[2 + k];
    a2[k] = keep + lane_xorf<2>(send);
  }
  const float keep = b0 ? a2[1] : a2[0], send = b0 ? a2[0] : a2[1];
  return keep + lane_xorf<1>(send);
}

}  // namespace MB_PREC
}  // namespace mb
