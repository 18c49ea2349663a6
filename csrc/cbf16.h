// 16x16x32 CBF backward over the active evaluation list: the fp32-accurate (3-term split-bf16) x3
// backward of the CBF edge MLP at TWO waves per SIMD, and the same kernel in the 1-pass bf16 /
// fp16 builds (no lo planes: half the weight-image and stage LDS, one MFMA per product).
//
// Why a second kernel: the 32x32x16 x3 backward (cbf_bwd_kernel) keeps 32 evaluations per wave
// and needs 464 registers, so it runs one wave per SIMD; its phase clocks (scripts/stamps_cbf.py,
// profiles/r3_cbf16/) show every phase at ~3x its MFMA issue time -- LDS round trips, the
// dependent split/relu VALU chain and the edge-gather chain are exposed with no second wave to
// hide them. Here a wave owns 16 evaluations and every tile is a 16x16 v_mfma_f32_16x16x32_bf16
// tile (4 accumulator registers instead of 16), so the activations of a wave fit in 256
// registers: an 8-wave workgroup (128 evaluations per chunk) runs two waves per SIMD.
//
// v_mfma_f32_16x16x32_bf16, lane l: n = l & 15, g = l >> 4.
//   A (16x32): elem j = A[n][8g + j]   B (32x16): elem j = B[8g + j][n]   C: reg i = C[4g + i][n]
// Data path (standard orientation, rows = hidden units, columns = this wave's evaluations): the
// B operand of K-step s is the packed pair of C tiles 2s, 2s+1 (k(8g + j) = 32s + 16(j >> 2) +
// 4g + (j & 3), layout.kacc16); the weight images (layout.cbf_rm16) store every 32-column block
// in that order, so A = W is ONE 16-byte LDS read per plane and A = W^T two ds_read_b64_tr_b16.
// Weight gradients: the chunk's deltas / activations go through edge-major LDS stage images and
// are contracted over the evaluations with transposed reads (natural k on both sides); every
// wave owns a 2x2 block of 16x16 output tiles; bias gradients are the same A fragments times a
// ones operand; dw4 / db4 are exact fp32 per-lane sums (no stage).
// Loads: cbf_compact writes one 16-byte record per active evaluation {u, e | pass << 31, j, dh}
// so a chunk's inputs are one record load plus the two state records; records are requested two
// chunks ahead and the state records one chunk ahead (no dependent load chain in the loop).
// Reference op: /root/reference/cbf.py:40-43 (the Conv1d stack), its autograd backward through
// /root/reference/train.py:103.
#pragma once
#include "mfma16.h"

namespace mb {
namespace MB_PREC {

constexpr int S16_W2 = 80, S16_W3 = 144;                   // layout.CBF16_STRIDES
constexpr int RM16_W2 = 128 * S16_W2, RM16_W3 = 64 * S16_W3;
constexpr int RM16 = RM16_W2 + RM16_W3;                    // lo-plane offset of the images (x3)
constexpr int C16_PLANES = X3 ? 2 : 1;
constexpr int C16_NW = 8, C16_CH = 16 * C16_NW, C16_RT = 64;   // waves, evaluations per chunk, rows per turn
constexpr int S16_64 = 68, S16_128 = 148, S16_F = 24;      // stage image strides (scripts: bank model)
// stage A region: D3 [64 x S16_64] | H2 [64 x S16_128], lo plane at +PLA
constexpr int C16_PLA = C16_RT * (S16_64 + S16_128);
// stage BC region: D2 [64 x S16_128] | H1 [64 x S16_64] | D1 [64 x S16_64], lo plane at +PLB, then F
constexpr int C16_PLB = C16_RT * (S16_128 + 2 * S16_64);
constexpr int C16_REGION = C16_PLANES * C16_PLB + C16_RT * S16_F;   // elements (>= planes * C16_PLA)
constexpr size_t C16_LDS_W = (size_t)C16_PLANES * RM16 * 2;        // W2 | W3 images, hi [+ lo]
constexpr size_t C16_LDS_F = 2 * FRAG_SZ;                          // w1ft16 (2 fragments, hi [+ lo])
constexpr size_t C16_LDS = C16_LDS_W + C16_LDS_F + CBF_VEC * 4 + (size_t)C16_REGION * 2;
// x3: one 8-wave workgroup per CU (2 waves / SIMD); 1-pass: two (<= 80 KiB each, 4 waves / SIMD at
// <= 128 registers; the second __launch_bounds__ argument is HIP's minimum waves per SIMD).
constexpr int C16_WG_PER_CU = CBF16_WGPC;
static_assert(C16_REGION >= C16_PLANES * C16_PLA, "stage A fits the region");
static_assert(C16_LDS <= 160 * 1024 / C16_WG_PER_CU - 64, "LDS budget");

#define CBF16_DBG ((MB_DIAG & 2) != 0)    // per-record forward sums to a.dbg (scripts/check_cbf16.py)

DEV f32x4 bias4(const float* b, int row0, int g) {
  const float4 v = *reinterpret_cast<const float4*>(b + row0 + 4 * g);
  return f32x4{v.x, v.y, v.z, v.w};
}
// A = W (rows m0..m0+15 of a permuted row-major image), K-step s: one 16-byte read per plane
DEV Fr w16_fr(const h16* W, int stride, int m0, int s, int lane) {
  const int n = lane & 15, g = lane >> 4;
  const h16* p = W + (m0 + n) * stride + 32 * s + 8 * g;
  Fr r;
  r.h = *reinterpret_cast<const h16x8*>(p);
  if constexpr (X3) r.l = *reinterpret_cast<const h16x8*>(p + RM16);
  return r;
}
// A = W^T: rows = logical columns m0..m0+15 of the permuted image, K-step s over W's rows in
// accumulator order (rows 32s + 4g + j, 32s + 16 + 4g + j - 4)
DEV Fr w16T_fr(const h16* W, int stride, int m0, int s, int lane) {
  const int g = lane >> 4, p = lane & 3;
  const int colp = 32 * (m0 >> 5) + 4 * ((m0 >> 4) & 1) + 8 * p;
  Fr r;
  r.h = tr_pair16(W, stride, 32 * s + 4 * g, 16, colp, lane);
  if constexpr (X3) r.l = tr_pair16(W + RM16, stride, 32 * s + 4 * g, 16, colp, lane);
  return r;
}
// record of one active evaluation (cbf_compact): {u, e | pass << 31, neighbour j, dh bits}
template <int D>
struct Ev16 {
  int4 r;                      // record
  float4 si[D == 2 ? 1 : 2], sj[D == 2 ? 1 : 2];   // raw state records of i and j
};

// branch-free: r is always a real record (the index is clamped), so the loads need no guard and
// no merge -- a conditional load would make the compiler wait for it right at the merge
template <int D>
DEV void ev16_issue(const CbfBwdArgs& a, const int4& r, Ev16<D>& x) {
  x.r = r;
  const unsigned e = (unsigned)r.y & 0x7fffffffu, pass = (unsigned)r.y >> 31;
  const unsigned ik = e / (unsigned)a.K;
  const unsigned tb = ik / (unsigned)a.N;
  const unsigned i = ik - tb * (unsigned)a.N;
  const unsigned t = tb / (unsigned)a.B;
  const unsigned b = tb - t * (unsigned)a.B;
  const float4* Sb = a.S + ((unsigned)b * (unsigned)a.s_env + (t + pass) * (unsigned)a.s_step) * REC<D>;
  if constexpr (D == 2) {
    x.si[0] = Sb[i];
    x.sj[0] = Sb[(unsigned)r.z];
  } else {
    x.si[0] = Sb[2 * i]; x.si[1] = Sb[2 * i + 1];
    x.sj[0] = Sb[2 * (unsigned)r.z]; x.sj[1] = Sb[2 * (unsigned)r.z + 1];
  }
}

// ST: phase clocks (a.stamps, diagnostics) -- a separate instantiation, so the production kernel
// has no runtime stamp branches: a branch taken right after the forward's last MFMA left its
// VALU consumers without the MFMA result wait states on that path (the round-3 "miscompile",
// docs/ARCHITECTURE.md "MFMA result hazard across a branch")
template <int D, bool ST>
__global__ __launch_bounds__(C16_NW * 64, 2 * C16_WG_PER_CU) void cbf_bwd16_kernel(CbfBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* W2 = reinterpret_cast<h16*>(smem);
  h16* W3 = W2 + RM16_W2;
  h16* wft = W2 + C16_PLANES * RM16;                          // w1ft16: 2 fragments [hi | lo]
  float* vl = reinterpret_cast<float*>(smem + C16_LDS_W + C16_LDS_F);
  h16* stg = reinterpret_cast<h16*>(smem + C16_LDS_W + C16_LDS_F + CBF_VEC * 4);
  __shared__ float red4[C16_NW];
  block_copy16(W2, a.wrm16, (int)C16_LDS_W, false);
  block_copy16(wft, a.w16 + 4 * FRAG_ELEMS, (int)C16_LDS_F, false);
  block_copy16(vl, a.wvec, CBF_VEC * 4);
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
  const long EV = (long)*a.nact;
  const long nchunks = (EV + C16_CH - 1) / C16_CH;
  const float* b2 = vl;
  const float* b3 = vl + 128;
  const float* w4 = vl + 192;
  const int4* rec = a.rec;
  h16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (h16)1.f;

  // tile ownership: stage A dW3 (64 x 128): M-tiles 2(w&1)+{0,1}, N-tiles 2(w>>1)+{0,1}, db3 of
  // the M-tiles over K-step (w>>1) of the chunk; stage BC dW2 (128 x 64): M-tiles 2(w>>1)+{0,1},
  // N-tiles 2(w&1)+{0,1}, db2 over turn (w&1); dW1f (64 x 16): M-tile w&3, K-step w>>2 of a turn
  const int ma0 = 2 * (wave & 1), na0 = 2 * (wave >> 1);
  const int mb0 = 2 * (wave >> 1), nb0 = 2 * (wave & 1);
  // bias rows: stage A M-tile ma0 + ua over turn (w >> 2); stage B M-tile mb0 + ub over the chunk
  const int ua = (wave >> 1) & 1, ub = wave & 1;
  f32x4 accA[2][2], accB[2][2], biasA = zero4(), biasB = zero4(), accC = zero4();
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) accA[u][v] = accB[u][v] = zero4();
  // dw4 row 16(n>>2) + 4g + (n&3) of this lane: the chunk's 16 per-lane products are
  // reduce-scattered over the 16 evaluation lanes (lane n keeps index n), one register
  float dw4acc = 0.f, db4 = 0.f;

  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tck = 0;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[k] += t - tck;
      tck = t;
    }
  };

  // load pipeline: records two chunks ahead, state records one chunk ahead
  const long stride = gridDim.x;
  // (indices past the list are clamped to its last record: unconditional loads, no merges)
  auto rec_at = [&](long chunk) -> int4 {
    const long v = chunk * C16_CH + wave * 16 + n;
    return rec[v < EV ? v : EV - 1];
  };
  auto in_at = [&](long chunk) { return chunk * C16_CH + wave * 16 + n < EV; };
  const long c0 = CBF_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  if (c0 < nchunks) {   // else no chunk for this workgroup (EV may be 0): zero slab
  Ev16<D> nx;
  ev16_issue<D>(a, rec_at(c0), nx);
  int4 r2 = rec_at(c0 + stride);

  for (long chunk = c0; chunk < nchunks; chunk += stride) {
    if constexpr (ST) { tck = __builtin_amdgcn_s_memtime(); ph[7] += 1; }
    const Ev16<D> cur = nx;
    const bool in = in_at(chunk);
    ev16_issue<D>(a, r2, nx);                                 // state records of the next chunk
    r2 = rec_at(chunk + 2 * stride);                          // records two chunks ahead
    // ---- edge features of this lane's evaluation (all four g-lanes of column n hold it)
    float rp[D], rv[D];
    {
      float pi[D], vi[D], pj[D], vj[D];
      if constexpr (D == 2) {
        pi[0] = cur.si[0].x; pi[1] = cur.si[0].y; vi[0] = cur.si[0].z; vi[1] = cur.si[0].w;
        pj[0] = cur.sj[0].x; pj[1] = cur.sj[0].y; vj[0] = cur.sj[0].z; vj[1] = cur.sj[0].w;
      } else {
        pi[0] = cur.si[0].x; pi[1] = cur.si[0].y; pi[2] = cur.si[0].z;
        vi[0] = cur.si[1].x; vi[1] = cur.si[1].y; vi[2] = cur.si[1].z;
        pj[0] = cur.sj[0].x; pj[1] = cur.sj[0].y; pj[2] = cur.sj[0].z;
        vj[0] = cur.sj[1].x; vj[1] = cur.sj[1].y; vj[2] = cur.sj[1].z;
      }
#pragma unroll
      for (int q = 0; q < D; ++q) {
        rp[q] = in ? pi[q] - pj[q] : 0.f;
        rv[q] = in ? vi[q] - vj[q] : 0.f;
      }
    }
    const unsigned e_ = (unsigned)cur.r.y & 0x7fffffffu;
    const unsigned i_ = (e_ / (unsigned)a.K) % (unsigned)a.N;
    const bool self = in && ((unsigned)cur.r.z == i_);
    const float dist = sqrtf(sqsum<D>(rp) + a.dist_eps);
    const float dhv = in ? __int_as_float(cur.r.w) : 0.f;
    const h16x8 F = cbf_edge_frag<D>(rp, rv, self ? 1.f : 0.f, dist - a.dist_thr, in && g < 2, g & 1);
    const h16* W2c = W2 + opaque_zero();
    const h16* W3c = W3 + opaque_zero();
    // ---- forward recompute
    Pk4 H1[4], H2[8];
    f32x4 H3[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const f32x4 t = mma16_bx(frag_fr(a.w16, mt, lane), F, zero4());
      H1[mt] = to_pk4(relu4(t));
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 t = bias4(b2, 16 * mt, g);
#pragma unroll
      for (int s = 0; s < 2; ++s) t = mma16(w16_fr(W2c, S16_W2, 16 * mt, s, lane), pk4_fr(H1[2 * s], H1[2 * s + 1]), t);
      H2[mt] = to_pk4(relu4(t));
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 t = bias4(b3, 16 * mt, g);
#pragma unroll
      for (int s = 0; s < 4; ++s) t = mma16(w16_fr(W3c, S16_W3, 16 * mt, s, lane), pk4_fr(H2[2 * s], H2[2 * s + 1]), t);
      H3[mt] = relu4(t);
    }
#if CBF16_DBG
    if (a.dbg) {   // diagnostics: sum H1, sum H2, sum w4 . H3 per record
      float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s1 += (float)H1[mt].h[i] + (float)H1[mt].l[i];
          s3 += vl[192 + 16 * mt + 4 * g + i] * H3[mt][i];
        }
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) s2 += (float)H2[mt].h[i] + (float)H2[mt].l[i];
      s1 += lane_xorf<16>(s1); s1 += lane_xorf<32>(s1);
      s2 += lane_xorf<16>(s2); s2 += lane_xorf<32>(s2);
      s3 += lane_xorf<16>(s3); s3 += lane_xorf<32>(s3);
      const long v = chunk * C16_CH + wave * 16 + n;
      if (in && g == 0) { a.dbg[3 * v] = s1; a.dbg[3 * v + 1] = s2; a.dbg[3 * v + 2] = s3; }
    }
#endif
    // (Round 3 kept a __builtin_amdgcn_sched_barrier(0) here against a deterministic ~20 % of wrong
    // forwards. Round 4 found the cause -- a runtime stamp branch taken with the forward's last MFMA
    // result read 1 wait state later, 8 needed; docs/ARCHITECTURE.md "MFMA result hazard" -- made
    // the stamps a template instantiation, and dropped the barrier: the no-barrier build passes the
    // float64-oracle tests and runs as fast (11.13 vs 11.13 ms, profiles/r4_validate/).)
    stamp(0);
    // ---- head backward: dW4 / db4 exact fp32 per lane, dH3pre = w4 * dh . relu'(H3)
    if (g == 0) db4 += dhv;
    Pk4 D3[4];
    {
      float v[16];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 w = bias4(w4, 16 * mt, g);
        f32x4 d;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[4 * mt + i] = dhv * H3[mt][i];
          d[i] = H3[mt][i] > 0.f ? w[i] * dhv : 0.f;
        }
        D3[mt] = to_pk4(d);
      }
      dw4acc += reduce_scatter16(v, n);
    }
    // ---- stage A: dW3 += dH3pre . H2^T, db3 (two turns of 64 evaluation rows)
#pragma unroll
    for (int turn = 0; turn < 2; ++turn) {
      h16* imD = stg;
      h16* imH = stg + C16_RT * S16_64;
      if ((wave >> 2) == turn) {
        const int row = (wave & 3) * 16 + n;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store4(imD, S16_64, C16_PLA, row, mt, g, D3[mt]);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) store4(imH, S16_128, C16_PLA, row, mt, g, H2[mt]);
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const Fr B0 = tr16_fr(imH, S16_128, C16_PLA, 32 * ks, 16 * na0, lane);
        const Fr B1 = tr16_fr(imH, S16_128, C16_PLA, 32 * ks, 16 * (na0 + 1), lane);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const Fr A = tr16_fr(imD, S16_64, C16_PLA, 32 * ks, 16 * (ma0 + u), lane);
          accA[u][0] = mma16(A, B0, accA[u][0]);
          accA[u][1] = mma16(A, B1, accA[u][1]);
          if (ua == u && (wave >> 2) == turn) biasA = mma16_bx(A, ones, biasA);
        }
      }
      __syncthreads();
    }
    stamp(1);
    // ---- dH2pre = (W3^T dH3pre) . relu'(H2); dH1pre = (W2^T dH2pre) . relu'(H1)
    Pk4 D2[8], D1[4];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 t = zero4();
#pragma unroll
      for (int s = 0; s < 2; ++s) t = mma16(w16T_fr(W3c, S16_W3, 16 * mt, s, lane), pk4_fr(D3[2 * s], D3[2 * s + 1]), t);
      D2[mt] = to_pk4(t);
      mask_pk4(D2[mt], H2[mt]);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 t = zero4();
#pragma unroll
      for (int s = 0; s < 4; ++s) t = mma16(w16T_fr(W2c, S16_W2, 16 * mt, s, lane), pk4_fr(D2[2 * s], D2[2 * s + 1]), t);
      D1[mt] = to_pk4(t);
      mask_pk4(D1[mt], H1[mt]);
    }
    // ---- dF = W1^T dH1pre (rows = feature columns 4g + i) -> dL/d(s_i - s_j)
    {
      const h16* wtc = wft + opaque_zero();
      f32x4 t = zero4();
#pragma unroll
      for (int s = 0; s < 2; ++s) t = mma16(frag_fr(wtc, s, lane), pk4_fr(D1[2 * s], D1[2 * s + 1]), t);
      float g8[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) { g8[i] = t[i]; g8[4 + i] = lane_xorf<16>(t[i]); }
      if (a.dE && in && g == 0) {
        float dp[D], dv[D];
#pragma unroll
        for (int q = 0; q < D; ++q) { dp[q] = 0.f; dv[q] = 0.f; }
        if (!self) {
          const float ddist = g8[2 * D + 1] * (1.f / dist);
#pragma unroll
          for (int q = 0; q < D; ++q) { dp[q] = g8[q] + ddist * rp[q]; dv[q] = g8[D + q]; }
        }
        store_rec<D>(a.dE, (unsigned)cur.r.x, dp, dv);
      }
    }
    stamp(2);
    // ---- stage BC: dW2 += dH2pre . H1^T, db2; dW1f += dH1pre . F^T (two turns)
#pragma unroll
    for (int turn = 0; turn < 2; ++turn) {
      h16* imD2 = stg;
      h16* imH1 = imD2 + C16_RT * S16_128;
      h16* imD1 = imH1 + C16_RT * S16_64;
      h16* imF = stg + C16_PLANES * C16_PLB;
      if ((wave >> 2) == turn) {
        const int row = (wave & 3) * 16 + n;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) store4(imD2, S16_128, C16_PLB, row, mt, g, D2[mt]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          store4(imH1, S16_64, C16_PLB, row, mt, g, H1[mt]);
          store4(imD1, S16_64, C16_PLB, row, mt, g, D1[mt]);
        }
        if (g < 2) *reinterpret_cast<h16x8*>(imF + row * S16_F + 8 * g) = F;
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const Fr B0 = tr16_fr(imH1, S16_64, C16_PLB, 32 * ks, 16 * nb0, lane);
        const Fr B1 = tr16_fr(imH1, S16_64, C16_PLB, 32 * ks, 16 * (nb0 + 1), lane);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const Fr A = tr16_fr(imD2, S16_128, C16_PLB, 32 * ks, 16 * (mb0 + u), lane);
          accB[u][0] = mma16(A, B0, accB[u][0]);
          accB[u][1] = mma16(A, B1, accB[u][1]);
          if (ub == u) biasB = mma16_bx(A, ones, biasB);
        }
        if ((wave >> 2) == ks) {
          const Fr Ac = tr16_fr(imD1, S16_64, C16_PLB, 32 * ks, 16 * (wave & 3), lane);
          accC = mma16_bx(Ac, tr16(imF, S16_F, 32 * ks, 0, lane), accC);
        }
      }
      __syncthreads();
    }
    stamp(3);
  }
  }
  if (ST && lane == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) a.stamps[((long)blockIdx.x * C16_NW + wave) * 8 + k] = ph[k];

  // ---- per-workgroup slab (same layout as cbf_bwd_kernel: P_W3, P_B3, P_W2, P_B2, P_W1, P_W4, P_B4)
  float* P = a.partial + (long)blockIdx.x * CBF_PARTIAL;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      write_tile16(P + P_W3, 128, ma0 + u, na0 + v, accA[u][v], lane);
      write_tile16(P + P_W2, 64, mb0 + u, nb0 + v, accB[u][v], lane);
    }
  // fixed-order cross-wave sums through LDS (the stage region is free after the last barrier):
  // bias rows (column 0 of the ones products), dW1f halves, dw4 lane sums, db4
  float* red = reinterpret_cast<float*>(stg);            // [wave][192 bias | 64 dw4] + [4][256] dW1f
  float* w1r = red + C16_NW * 256;
  for (int q = threadIdx.x; q < C16_NW * 256; q += blockDim.x) red[q] = 0.f;
  __syncthreads();
  if (n == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      red[wave * 256 + 16 * (ma0 + ua) + 4 * g + i] = biasA[i];
      red[wave * 256 + 64 + 16 * (mb0 + ub) + 4 * g + i] = biasB[i];
    }
  }
  red[wave * 256 + 192 + 16 * (n >> 2) + 4 * g + (n & 3)] = dw4acc;
  if (wave >= 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) w1r[(wave - 4) * 256 + (4 * g + i) * 16 + n] = accC[i];
  }
  const float s4 = wave_sum(db4);
  if (lane == 0) red4[wave] = s4;
  __syncthreads();
  if (wave < 4) {
    // dW1f M-tile `wave` (rows 16 wave + 4g + i, slot columns 0..15 of the 32-column slab rows)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = accC[i] + w1r[wave * 256 + (4 * g + i) * 16 + n];
      P[P_W1 + (16 * wave + 4 * g + i) * 32 + n] = v;
      P[P_W1 + (16 * wave + 4 * g + i) * 32 + 16 + n] = 0.f;
    }
  }
  if (threadIdx.x < 256) {
    float t = 0.f;
    for (int w = 0; w < C16_NW; ++w) t += red[w * 256 + threadIdx.x];
    if (threadIdx.x < 64) P[P_B3 + threadIdx.x] = t;
    else if (threadIdx.x < 192) P[P_B2 + threadIdx.x - 64] = t;
    else P[P_W4 + threadIdx.x - 192] = t;
  }
  if (threadIdx.x == 256) {
    float t4 = 0.f;
    for (int w = 0; w < C16_NW; ++w) t4 += red4[w];
    P[P_B4] = t4;
  }
  if (threadIdx.x >= 288 && threadIdx.x < 298) P[P_LOSS + threadIdx.x - 288] = 0.f;
}

template <int D>
static void launch_cbf_bwd16(const CbfBwdArgs& a, int num_blocks, hipStream_t st) {
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)C16_LDS);
    hipLaunchKernelGGL(kern, dim3(num_blocks), dim3(C16_NW * 64), C16_LDS, st, a);
  };
  if (a.stamps) go(cbf_bwd16_kernel<D, true>);
  else go(cbf_bwd16_kernel<D, false>);
}

}  // namespace MB_PREC
}  // namespace mb
