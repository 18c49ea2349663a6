// 16x16x32 controller edge backward: the fp32-accurate x3 BPTT edge step at TWO waves per SIMD, and
// the same kernel in the 1-pass bf16 / fp16 builds (no lo planes).
//
// Same math as edge_bwd_body (ctrl.hip): per edge of the 1024-agent step, layer-1 recompute
// H1 = relu(W1 [s_i - s_j, eye, 1]), the max-pool backward (dP of each pooled feature routed to
// the edge of its argmax slot: dZ), dH1 = W2^T dZ . relu'(H1), dL/d(s_i - s_j) = W1^T dH1, and
// the weight gradients dW2 += dZ . H1^T, db2 += sum dZ (fp32 sums of the routed values),
// dW1f += dH1 . F^T. The 32x32x16 kernel holds 32 edges per wave in 322 registers (one wave per
// SIMD, ~3x its MFMA issue time); here a wave owns 16 agents (K = 12 tiles of 16 dense edge rows) and 16x16 tiles (csrc/mfma16.h), so an
// 8-wave workgroup (128 agents, 128 edges per tile round) runs two waves per SIMD and the shared
// dW2 stage contracts the whole round in one barrier pair (the dZ and H1 images of 128 rows fit
// next to the 44 KB of weight fragments). Reference op: /root/reference/controller.py:43-50
// (centralized Conv1d layers + masked max-pool), differentiated by train.py:103.
#pragma once
#include "mfma16.h"

namespace mb {
namespace MB_PREC {

constexpr int E16_NW = 8, E16_AG = 16, E16_CH = E16_NW * E16_AG;   // waves, agents per wave / chunk
constexpr int E16_SZ = 144, E16_SH = 68;                           // dZ / H1 image strides (bank model)
constexpr int E16_PL = E16_CH * (E16_SZ + E16_SH);                 // lo-plane offset (elements)
constexpr int E16_FRAGS = 22;                                      // ew1f16 4 | ew2tn16 16 | ew1ft16 2
constexpr size_t E16_LDS = (size_t)E16_FRAGS * FRAG_SZ + (size_t)(X3 ? 2 : 1) * E16_PL * 2;
constexpr int E16_WG_PER_CU = E16_WGPC;
static_assert(E16_LDS <= 160 * 1024 / E16_WG_PER_CU - 1024, "LDS budget");

template <int D>
struct E16Idx { int j, b, i, slot; bool ok; };

// ST: phase clocks (a.stamps, diagnostics) -- a separate instantiation, no runtime stamp branches
// in the production kernel (docs/ARCHITECTURE.md "MFMA result hazard across a branch")
template <int D, bool ST>
__global__ __launch_bounds__(E16_NW * 64, 2 * E16_WG_PER_CU) void ctrl_edge_bwd16_kernel(CtrlEdgeBwdArgs a) {
  constexpr int K = 12;                           // TOP_K (the host falls back to the 32x32 kernel)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* wf = reinterpret_cast<h16*>(smem);
  h16* imZ = reinterpret_cast<h16*>(smem + (size_t)E16_FRAGS * FRAG_SZ);    // dZ [128][E16_SZ]
  h16* imH = imZ + E16_CH * E16_SZ;                                        // H1 [128][E16_SH]
  block_copy16(wf, a.w16, E16_FRAGS * FRAG_SZ);
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
  const int r = lane & 31, h = lane >> 5;         // max-pool lanes: features 4r..4r+3, agent half h
  const int N = a.N, total = a.B * N;
  const long nchunks = (total + E16_CH - 1) / E16_CH;
  const int QP = a.qsplit > 1 ? a.qsplit : 1;
  const long nwork = nchunks * QP;
  const unsigned invK = (65536u + K - 1u) / K;
  const int row0 = wave * E16_AG;                 // this wave's rows in the round images
  const int mb0 = 2 * (wave >> 1), nb0 = 2 * (wave & 1);
  f32x4 accB[2][2], accC[4];
  // db2 = sum over edges of dZ = the routed dL/dpooled values: summed in fp32 as they are routed
  // (lane (r, h): features 4r..4r+3 of its agents; x3: hi + lo) -- no ones-operand MFMAs
  float db2r[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u) accB[u][0] = accB[u][1] = zero4();
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) accC[mt] = zero4();
  // phases (scripts/stamps_edge16.py): 0 load issue, 1 F, 2 layer 1, 3 dZ zero fill, 4 routing,
  // 5 dH1, 6 dF + dEc, 7 H1 stage store, 8 first barrier, 9 S1, 10 second barrier, 11 S2 stores,
  // 12 S2 contraction; slot 15 counts tiles
  unsigned long long ph[16] = {}, tck = 0;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[k] += t - tck;
      tck = t;
    }
  };

  for (long w = BPTT_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x; w < nwork; w += gridDim.x) {
    const long chunk = w / QP;
    const int part = (int)(w - chunk * QP);
    const int q0 = part * K / QP, q1 = (part + 1) * K / QP;
    const int g0 = (int)(chunk * E16_CH) + row0;
    const AgentBase ab = agent_base(g0, N);
    // edge e = 16q + n of this wave's 16 x K dense rows -> (agent, slot); loads pipelined: idx two
    // tiles ahead, states one tile ahead (as edge_bwd_body); every load unconditional (ctrl.hip
    // ctrl_st_load: a conditional load costs one memory latency per tile)
    auto idx_load = [&](int q, E16Idx<D>& o) {
      const int e = E16_AG * q + n;
      const int al = dense_agent(e, invK);
      o.ok = (q < q1) && (al < E16_AG) && (ab.g0 + al < total);
      int bb, ii;
      agent_bi(ab, al, N, bb, ii);
      o.b = o.ok ? bb : 0;
      o.i = o.ok ? ii : 0;
      o.slot = o.ok ? e - al * K : 0;
      o.j = a.idx[o.b * (int)a.i_env + o.i * K + o.slot];
    };
    auto st_load = [&](const E16Idx<D>& x, EdgeSt<D>& o) {
      EdgeIdx xi;
      xi.j = x.j; xi.b = x.b; xi.i = x.i; xi.ok = x.ok;
      ctrl_st_load<D>(a.S, a.s_env, xi, o);
    };
    // the argmax slots / dL/dpooled of the (<= 3) agents of a tile: pass p = agents af + 2p + h
    // (E16_AG: none; agents past `total` are dropped by the routing)
    auto pass_agent = [&](int q, int p) {
      const int af = dense_agent(E16_AG * q, invK);
      const int al = af + 2 * p + h;
      return (q < q1 && al < E16_AG && al * K < E16_AG * q + E16_AG) ? al : E16_AG;
    };
    auto pool_load = [&](int q, unsigned (&am)[2], h16x4 (&dp)[2], h16x4 (&dl)[2]) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int al = pass_agent(q, p);
        const bool v = al < E16_AG && ab.g0 + al < total;
        int bb, ii;
        agent_bi(ab, al, N, bb, ii);
        bb = v ? bb : 0;
        ii = v ? ii : 0;
        am[p] = *reinterpret_cast<const unsigned*>(a.argmax + bb * (int)a.am_env + ii * 128 + 4 * r);
        const h16* dpr = a.dP + bb * (int)a.dp_env + ii * PROW + 4 * r;
        dp[p] = *reinterpret_cast<const h16x4*>(dpr);
        if constexpr (X3) dl[p] = *reinterpret_cast<const h16x4*>(dpr + 128);
      }
    };
    E16Idx<D> xc, xn;
    EdgeSt<D> xs;
    {
      E16Idx<D> x0;
      idx_load(q0, x0);
      st_load(x0, xs);
      xc = x0;
      idx_load(q0 + 1, xn);
    }
    unsigned am_n[2];
    h16x4 dp_n[2], dl_n[2];
    pool_load(q0, am_n, dp_n, dl_n);
    for (int q = q0; q < q1; ++q) {
      if constexpr (ST) { tck = __builtin_amdgcn_s_memtime(); ph[15] += 1; }
      const EdgeSt<D> cur = xs;
      const E16Idx<D> ci = xc;
      unsigned am[2];
      h16x4 dp[2], dl[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) { am[p] = am_n[p]; dp[p] = dp_n[p]; dl[p] = dl_n[p]; }
      st_load(xn, xs);
      xc = xn;
      idx_load(q + 2, xn);
      pool_load(q + 1, am_n, dp_n, dl_n);
      stamp(0);
      const bool ok = cur.ok;
      const bool self = cur.j == cur.i;
      float rp[D], rv[D];
      edge_rel<D>(cur, rp, rv);
      const h16x8 F = ctrl_edge_frag<D>(rp, rv, self ? 1.f : 0.f, ok && g < 2, g & 1);
      stamp(1);
      // ---- layer-1 recompute
      Pk4 H1[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) H1[mt] = to_pk4(relu4(mma16_bx(frag_fr(wf, mt, lane), F, zero4())));
      stamp(2);
      // ---- max-pool backward: zero this wave's 16 dZ rows, route dP[f] of each tile agent to the
      //      row of (agent, argmax slot f) when that row is in the tile
      {
        const u32x4 z4 = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int rr = row0 + 4 * c + (lane >> 4);
          *reinterpret_cast<u32x4*>(imZ + rr * E16_SZ + 8 * (lane & 15)) = z4;
          if constexpr (X3) *reinterpret_cast<u32x4*>(imZ + E16_PL + rr * E16_SZ + 8 * (lane & 15)) = z4;
        }
        lds_wave_order();
        stamp(3);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int al = pass_agent(q, p);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const unsigned sl = (am[p] >> (8 * jj)) & 0xFFu;
            const int row = al * K + (int)sl - E16_AG * q;
            if (sl < 16u && (unsigned)row < (unsigned)E16_AG && ab.g0 + al < total) {
              const int o = (row0 + row) * E16_SZ + 4 * r + jj;
              imZ[o] = dp[p][jj];
              db2r[jj] += (float)dp[p][jj];
              if constexpr (X3) {
                imZ[E16_PL + o] = dl[p][jj];
                db2r[jj] += (float)dl[p][jj];
              }
            }
          }
        }
        lds_wave_order();
      }
      stamp(4);
      // ---- dH1 = W2^T dZ . relu'(H1): B = this edge's dZ row (natural k, one 16-byte read per plane)
      Pk4 D1[4];
      {
        f32x4 c[4] = {zero4(), zero4(), zero4(), zero4()};
        const h16* zr = imZ + (row0 + n) * E16_SZ + 8 * g;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          Fr bz;
          bz.h = *reinterpret_cast<const h16x8*>(zr + 32 * s);
          if constexpr (X3) bz.l = *reinterpret_cast<const h16x8*>(zr + E16_PL + 32 * s);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) c[mt] = mma16(frag_fr(wf, 4 + 4 * mt + s, lane), bz, c[mt]);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          D1[mt] = to_pk4(c[mt]);
          mask_pk4(D1[mt], H1[mt]);
        }
      }
      stamp(5);
      // ---- dF = W1^T dH1 (rows 4g + i: relative-state features) -> dL/d(s_i - s_j)
      {
        f32x4 t = zero4();
#pragma unroll
        for (int s = 0; s < 2; ++s) t = mma16(frag_fr(wf, 20 + s, lane), pk4_fr(D1[2 * s], D1[2 * s + 1]), t);
        float g8[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) { g8[i] = t[i]; g8[4 + i] = lane_xorf<16>(t[i]); }
        if (ok && g == 0 && a.dEc) {
          float gp[D], gv[D];
#pragma unroll
          for (int q2 = 0; q2 < D; ++q2) {
            gp[q2] = self ? 0.f : g8[q2];
            gv[q2] = self ? 0.f : g8[D + q2];
          }
          store_rec<D>(a.dEc, (unsigned)(ci.b * (int)a.de_env + ci.i * K + ci.slot), gp, gv);
        }
      }
      stamp(6);
      // ---- S1: dW2 (128 x 64) += dZ . H1^T, db2 over the round's 128 edges (one barrier pair)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) store4(imH, E16_SH, E16_PL, row0 + n, mt, g, H1[mt]);
      stamp(7);
      __syncthreads();
      stamp(8);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const Fr B0 = tr16_fr(imH, E16_SH, E16_PL, 32 * ks, 16 * nb0, lane);
        const Fr B1 = tr16_fr(imH, E16_SH, E16_PL, 32 * ks, 16 * (nb0 + 1), lane);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const Fr A = tr16_fr(imZ, E16_SZ, E16_PL, 32 * ks, 16 * (mb0 + u), lane);
          accB[u][0] = mma16(A, B0, accB[u][0]);
          accB[u][1] = mma16(A, B1, accB[u][1]);
        }
      }
      stamp(9);
      __syncthreads();
      stamp(10);
      // ---- S2 (wave-local, no barrier): dW1f (64 x 16) += dH1 . F^T over this wave's 16 edges;
      //      images in the wave's own dZ rows (free after S1): dH1 hi cols 0..63, lo 64..127, F
      //      128..143; K = 32 rows per MFMA: lanes g >= 2 (rows 16..31) re-read rows 0..15 and
      //      their F operand is zero
      {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store4(imZ, E16_SZ, 64, row0 + n, mt, g, D1[mt]);
        if (g < 2) *reinterpret_cast<h16x8*>(imZ + (row0 + n) * E16_SZ + 128 + 8 * g) = F;
        lds_wave_order();
        stamp(11);
        const int rb = row0 + 8 * (g & 1);
        h16x8 bf = tr_pair16(imZ, E16_SZ, rb, 4, 128 + 4 * (lane & 3), lane);
        if (g >= 2) bf = zero_h8();
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          Fr A;
          A.h = tr_pair16(imZ, E16_SZ, rb, 4, 16 * mt + 4 * (lane & 3), lane);
          if constexpr (X3) A.l = tr_pair16(imZ, E16_SZ, rb, 4, 64 + 16 * mt + 4 * (lane & 3), lane);
          accC[mt] = mma16_bx(A, bf, accC[mt]);
        }
        lds_wave_order();                      // reads done before the next tile's zero fill
      }
      stamp(12);
    }
  }
  if (ST && lane == 0)
#pragma unroll
    for (int k = 0; k < 16; ++k) a.stamps[((long)blockIdx.x * E16_NW + wave) * 16 + k] = ph[k];
  // ---- slab: dW2 tiles (one owner each), db2 rows and dW1f summed over the waves in fixed order
  float* P = a.partial + (long)blockIdx.x * CTRL_EDGE_PARTIAL;
  const bool acc = !a.init;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* d = P + EP_W2 + (16 * (mb0 + u) + 4 * g + i) * 64 + 16 * (nb0 + v) + n;
        *d = (acc ? *d : 0.f) + accB[u][v][i];
      }
  __syncthreads();                            // every wave is out of the loop: the region is free
  float* red = reinterpret_cast<float*>(imZ); // [wave][128] db2 rows | [wave][4 tiles][16][16] dW1f
  float* w1r = red + E16_NW * 128;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {             // the two agent halves h, then one row per feature
    const float v = db2r[jj] + lane_xorf<32>(db2r[jj]);
    if (h == 0) red[wave * 128 + 4 * r + jj] = v;
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) w1r[((wave * 4 + mt) * 16 + 4 * g + i) * 16 + n] = accC[mt][i];
  __syncthreads();
  if (threadIdx.x < 128) {
    float t = 0.f;
    for (int w2 = 0; w2 < E16_NW; ++w2) t += red[w2 * 128 + threadIdx.x];
    float* d = P + EP_B2 + threadIdx.x;
    *d = (acc ? *d : 0.f) + t;
  }
  for (int q = threadIdx.x; q < 64 * 32; q += blockDim.x) {     // dW1f rows o, slot columns k < 32
    const int o = q >> 5, k = q & 31;
    float t = 0.f;
    if (k < 16)
      for (int w2 = 0; w2 < E16_NW; ++w2) t += w1r[((w2 * 4 + (o >> 4)) * 16 + (o & 15)) * 16 + k];
    float* d = P + EP_W1 + q;
    *d = (acc ? *d : 0.f) + t;
  }
}

template <int D>
static void launch_ctrl_edge_bwd16(const CtrlEdgeBwdArgs& a, int num_blocks, hipStream_t st) {
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)E16_LDS);
    hipLaunchKernelGGL(kern, dim3(num_blocks), dim3(E16_NW * 64), E16_LDS, st, a);
  };
  if (a.stamps) go(ctrl_edge_bwd16_kernel<D, true>);
  else go(ctrl_edge_bwd16_kernel<D, false>);
}

}  // namespace MB_PREC
}  // namespace mb
