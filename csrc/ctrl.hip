// Controller kernels (reference controller.py:31-63 + the Euler step of train.py:70), gfx950.
//
// A wave owns 32 agents. Edge phase: 16 tiles of 32 edges = 2 agents x 16 neighbour slots
// (K <= 16 real, the rest masked). Per tile:
//   F   (B operand, built in registers): [dx dy dvx dvy eye 1] hi-h16 in lanes 0-31, the
//       h16 residuals (x - h16(x)) in lanes 32-63 -> layer 1 sees ~fp32 inputs for free
//   H1  = relu(W1f . F)               2 MFMA, standard orientation (rows = features)
//   Z^T = H1^T . W2^T + b2           16 MFMA, H1's accumulator used directly as the A
//                                      operand (rows = edges, lanes = features)
//   masked max-pool over each agent's 16 rows: in-lane max over 8 regs + one lane^32 swap
// Node phase (32 agents = one MFMA column tile): pooled features are re-laid through a
// per-wave LDS image (the only transpose), then Y1..Y4 chain on MFMA with the accumulator
// as the next B operand, bias folded into layer 1 / accumulator init, gains 2*sigmoid+0.2,
// PD law, Euler step, per-env goal-distance and action-loss sums. Weights live in LDS as
// pre-packed 1 KiB fragments (ops/layout.py); all intermediate activations stay in VGPRs.
#pragma clang fp contract(off)
#include <climits>
#include "common.h"
#include "args.h"
#include "state.h"
#include "ttc.h"
#include "combine.h"

namespace mb {
namespace MB_PREC {

constexpr int PSTR = 136;            // pooled-image row stride (h16): 128 + 8 pad, 272 B
constexpr int CTRL_FWD_FRAGS = 72;   // ew1f 2 + ew2 16 | nw1f 18 + nw2 16 + nw3 16 + nw4 4
constexpr int CTRL_VEC = 352;        // eb2 128 | nb2 128 | nb3 64 | nb4 32 (padded)


// edge layer-1 B fragment (layout.ctrl_edge_slot): hi [s_i - s_j (2D), eye, 1], lo [s_i - s_j]
template <int D>
DEV h16x8 ctrl_edge_frag(const float (&rp)[D], const float (&rv)[D], float eye, bool ok, int h) {
  h16x8 f;
  const h16 z = (h16)0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = z;
  if (!ok) return f;
  h16 hi[2 * D], lo[2 * D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    split_h16(rp[q], hi[q], lo[q]);
    split_h16(rv[q], hi[D + q], lo[D + q]);
  }
  if (h == 0) {
#pragma unroll
    for (int q = 0; q < 2 * D; ++q) f[q] = hi[q];
    f[2 * D] = (h16)eye;
    f[2 * D + 1] = (h16)1.f;
  } else {
#pragma unroll
    for (int q = 0; q < 2 * D; ++q) f[q] = lo[q];
  }
  return f;
}

// node layer-1 state fragment (layout.ctrl_node_slot): hi [p - g, v, 1], lo [p - g, v]
template <int D>
DEV h16x8 node_state_frag(const float (&e)[D], const float (&v)[D], bool ok, int h) {
  h16x8 f;
  const h16 z = (h16)0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = z;
  if (!ok) return f;
  h16 hi[2 * D], lo[2 * D];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    split_h16(e[q], hi[q], lo[q]);
    split_h16(v[q], hi[D + q], lo[D + q]);
  }
  if (h == 0) {
#pragma unroll
    for (int q = 0; q < 2 * D; ++q) f[q] = hi[q];
    f[2 * D] = (h16)1.f;
  } else {
#pragma unroll
    for (int q = 0; q < 2 * D; ++q) f[q] = lo[q];
  }
  return f;
}

// rows 0..2D-1 of an accumulator tile for lanes h == 0: rows 0..3 are regs 0..3 of this lane,
// rows 4..7 regs 0..3 of lane r + 32 (all lanes must call: lane swap)
DEV void acc_rows8(const f32x16& c, float (&o)[8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) { o[q] = c[q]; o[4 + q] = shfl_xor32(c[q]); }
}

// One edge tile in the transposed orientation: returns Z^T (4 column tiles) for 32 edges.
// ZB (optional): loop-invariant bias accumulators (4 x 16 registers, one bias per lane column),
// the C operand of each column tile's first MFMA -> no per-tile bias broadcast (64 VALU moves)
DEV void ctrl_edge_tile(const h16x8& F, const h16* wl, const float* eb2, int lane, f32x16 (&Z)[4],
                        const f32x16* ZB = nullptr) {
  const int r = lane & 31;
  f32x16 H1[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    H1[mt] = mma_bx(frag_fr(wl, mt, lane), F, zero16());
    relu_(H1[mt]);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    f32x16 z;
    if (ZB) {
      z = ZB[nt];
    } else {
      const float bv = eb2[32 * nt + r];
#pragma unroll
      for (int q = 0; q < 16; ++q) z[q] = bv;
    }
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      z = mma(acc_fr<kk & 1>(H1[kk >> 1]), frag_fr(wl, 2 + nt * 4 + kk, lane), z);
    });
    Z[nt] = z;
  }
}

// node MLP forward for 32 agents; returns Y4 (rows 0..3 = the 4 gain pre-activations)
struct NodeActs { f32x16 Y1[2], Y2[4], Y3[2], Y4; };

// Node activations kept from the rollout (CtrlArgs.acts) for the cooperative node backward: per
// agent, tiles 0..7 = Y1[2] | Y2[4] | Y3[2] (relu'd, packed hi [| lo] as the backward's to_pk) per
// lane half h of the 32x32 C layout, then Y4 (raw fp32, 16 per half) -- the C-layout lane (agent r,
// half h) stores and loads exactly its own registers
constexpr int NODE_ACT_PKB = X3 ? 64 : 32;
constexpr int NODE_ACT_BYTES = 16 * NODE_ACT_PKB + 128;
DEV h16x16 zero_h16x16() {
  h16x16 z;
#pragma unroll
  for (int j = 0; j < 16; ++j) z[j] = (h16)0.f;
  return z;
}
DEV void act_store_pk(unsigned char* base, int tile, int h, const f32x16& c) {
  const Pk p = to_pk(c);
  unsigned char* q = base + (tile * 2 + h) * NODE_ACT_PKB;
  *reinterpret_cast<h16x16*>(q) = p.h;
  if constexpr (X3) *reinterpret_cast<h16x16*>(q + 32) = p.l;
}
DEV Pk act_load_pk(const unsigned char* base, int tile, int h) {
  const unsigned char* q = base + (tile * 2 + h) * NODE_ACT_PKB;
  Pk p;
  p.h = *reinterpret_cast<const h16x16*>(q);
  if constexpr (X3) p.l = *reinterpret_cast<const h16x16*>(q + 32);
  return p;
}

// pool(kk): the pooled-feature B fragment of k-step kk (features 16kk + 8h + j of agent r)
template <typename PoolFr>
DEV void node_forward(PoolFr pool, const h16x8& sfrag, const h16* wn, const float* nb2,
                      const float* nb3, const float* nb4, int lane, NodeActs& o) {
  const int h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x16 c = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) c = mma(frag_fr(wn, mt * 9 + kk, lane), pool(kk), c);
    c = mma_bx(frag_fr(wn, mt * 9 + 8, lane), sfrag, c);
    relu_(c);
    o.Y1[mt] = c;
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    f32x16 c = bias_rows(nb2, 32 * mt, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mma(frag_fr(wn, 18 + mt * 4 + kk, lane), acc_fr<kk & 1>(o.Y1[kk >> 1]), c);
    });
    relu_(c);
    o.Y2[mt] = c;
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x16 c = bias_rows(nb3, 32 * mt, h);
    static_for<8>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mma(frag_fr(wn, 34 + mt * 8 + kk, lane), acc_fr<kk & 1>(o.Y2[kk >> 1]), c);
    });
    relu_(c);
    o.Y3[mt] = c;
  }
  {
    f32x16 c = bias_rows(nb4, 0, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mma(frag_fr(wn, 50 + kk, lane), acc_fr<kk & 1>(o.Y3[kk >> 1]), c);
    });
    o.Y4 = c;
  }
}

// Two-stage software pipeline for the per-edge gathers (idx -> s_j are dependent global
// loads): at tile q the kernel issues the idx load of tile q+2 and the state loads of tile
// q+1, then computes tile q, so every load has a full tile of MFMA work to land under.
struct EdgeIdx { int j, b, i; bool ok; };
template <int D> struct EdgeSt { float4 si[D == 2 ? 1 : 2], sj[D == 2 ? 1 : 2]; int j, i; bool ok; };   // ctrl_st_load

// (env, index) of the agents g0 + al, 0 <= al < 32, of a 32-agent group: one division per group;
// with N >= 32 the group wraps into the next env at most once (a per-tile 32-bit division by the
// runtime N is a dozen VALU instructions, two of them quarter rate)
constexpr int CTRL_GROUP_BASE = 1;
struct AgentBase { int g0, b0, i0; };
DEV AgentBase agent_base(int g0, int N) {
  AgentBase o;
  o.g0 = g0;
  o.b0 = g0 / N;
  o.i0 = g0 - o.b0 * N;
  return o;
}
DEV void agent_bi(const AgentBase& ab, int al, int N, int& b, int& i) {
  if (CTRL_GROUP_BASE && N >= 32) {
    i = ab.i0 + al;
    b = ab.b0;
    if (i >= N) { i -= N; ++b; }
  } else {
    const int g = ab.g0 + al;
    b = g / N;
    i = g - b * N;
  }
}

DEV void ctrl_idx_load(const int* idx, long i_env, int N, int K, const AgentBase& ab, int q, int r, int total,
                       EdgeIdx& o) {
  const int al = 2 * q + (r >> 4);
  const int slot = r & 15;
  const int gi = ab.g0 + al;
  o.ok = (q < 16) && (gi < total) && (slot < K);
  int bb, ii;
  agent_bi(ab, al, N, bb, ii);
  o.b = o.ok ? bb : 0;
  o.i = o.ok ? ii : 0;
  o.j = idx[o.b * (int)i_env + o.i * K + (o.ok ? slot : 0)];   // unconditional (see ctrl_st_load)
}

// dense edge rows (edge backward): a wave's 32 agents x K slots are 32K consecutive rows =
// K tiles; row e = 32q + r -> agent e / K, slot e % K (invK = ceil(2^16 / K): exact for e < 512)
DEV int dense_agent(int e, unsigned invK) { return (int)(((unsigned)e * invK) >> 16); }

DEV void ctrl_idx_load_dense(const int* idx, long i_env, int N, int K, unsigned invK, const AgentBase& ab, int q,
                             int r, int total, EdgeIdx& o, int nag = 32) {
  const int e = 32 * q + r;
  const int al = dense_agent(e, invK);
  const int slot = e - al * K;
  const int gi = ab.g0 + al;
  o.ok = (al < nag) && (gi < total);
  int bb, ii;
  agent_bi(ab, al, N, bb, ii);
  o.b = o.ok ? bb : 0;
  o.i = o.ok ? ii : 0;
  o.j = idx[o.b * (int)i_env + o.i * K + (o.ok ? slot : 0)];
}

// The endpoint records of an edge, loaded one tile ahead of their use. Every load is
// unconditional (a lane without an edge reads env 0's node 0 / slot 0: ctrl_idx_load*) and the
// relative state is formed only when the tile is processed (edge_rel): a load inside an `if`, or
// arithmetic on its value right after it, makes the compiler wait for the load there -- one full
// memory latency per tile (the 16x16x32 edge backward's phase clocks: 1.4 k cycles per tile).
template <int D>
DEV void ctrl_st_load(const float4* S, long s_env, const EdgeIdx& x, EdgeSt<D>& o) {
  o.ok = x.ok;
  o.j = x.j;
  o.i = x.i;
  const float4* Sb = S + (x.b * (int)s_env) * REC<D>;
  if constexpr (D == 2) {
    o.si[0] = Sb[x.i];
    o.sj[0] = Sb[x.j];
  } else {
    o.si[0] = Sb[2 * x.i]; o.si[1] = Sb[2 * x.i + 1];
    o.sj[0] = Sb[2 * x.j]; o.sj[1] = Sb[2 * x.j + 1];
  }
}
// s_i - s_j of a loaded edge (zero without an edge)
template <int D>
DEV void edge_rel(const EdgeSt<D>& c, float (&rp)[D], float (&rv)[D]) {
  float pi[D], vi[D], pj[D], vj[D];
  if constexpr (D == 2) {
    pi[0] = c.si[0].x; pi[1] = c.si[0].y; vi[0] = c.si[0].z; vi[1] = c.si[0].w;
    pj[0] = c.sj[0].x; pj[1] = c.sj[0].y; vj[0] = c.sj[0].z; vj[1] = c.sj[0].w;
  } else {
    pi[0] = c.si[0].x; pi[1] = c.si[0].y; pi[2] = c.si[0].z;
    vi[0] = c.si[1].x; vi[1] = c.si[1].y; vi[2] = c.si[1].z;
    pj[0] = c.sj[0].x; pj[1] = c.sj[0].y; pj[2] = c.sj[0].z;
    vj[0] = c.sj[1].x; vj[1] = c.sj[1].y; vj[2] = c.sj[1].z;
  }
#pragma unroll
  for (int q = 0; q < D; ++q) {
    rp[q] = c.ok ? pi[q] - pj[q] : 0.f;
    rv[q] = c.ok ? vi[q] - vj[q] : 0.f;
  }
}

// Node phase of the controller step for the 32-column group at g0 (lane column r = agent
// g0 + r, r < APW): node MLP (pooled fragments from `pool`), gains 2*sigmoid+0.2, PD law, Euler
// step, per-env goal-distance and action-loss sums.
// ACTS: the activations go to a.acts (a separate instantiation: the stores' registers would make
// the fused x3 step kernel spill where they are not wanted)
template <int D, bool ACTS, typename PoolFr>
DEV void node_phase(const CtrlArgs& a, int g0, int APW, int total, PoolFr pool, const h16* wn, const float* nb2,
                    const float* nb3, const float* nb4, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const int N = a.N;
  const int gi = g0 + r;
  const bool ok = r < APW && gi < total;
  int b = 0, i = 0;
  float sp[D], sv[D], gg[D];
#pragma unroll
  for (int q = 0; q < D; ++q) { sp[q] = 0.f; sv[q] = 0.f; gg[q] = 0.f; }
  if (ok) {
    b = gi / N; i = gi - b * N;
    load_rec<D>(a.S + (long)b * a.s_env * REC<D>, (unsigned)i, sp, sv);
#pragma unroll
    for (int q = 0; q < D; ++q) gg[q] = a.G[((long)b * N + i) * D + q];
  }
  float ex[D];
#pragma unroll
  for (int q = 0; q < D; ++q) ex[q] = sp[q] - gg[q];
  const h16x8 sf = node_state_frag<D>(ex, sv, ok, h);
  NodeActs na;
  node_forward(pool, sf, wn + opaque_zero(), nb2, nb3, nb4, lane, na);
  if (ACTS && ok) {            // kept for the cooperative node backward (NODE_ACT_BYTES layout)
    unsigned char* ab = a.acts + ((long)b * a.na_env + i) * NODE_ACT_BYTES;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      act_store_pk(ab, mt, h, na.Y1[mt]);
      act_store_pk(ab, 6 + mt, h, na.Y3[mt]);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) act_store_pk(ab, 2 + mt, h, na.Y2[mt]);
    *reinterpret_cast<f32x16*>(ab + 16 * NODE_ACT_PKB + 64 * h) = na.Y4;
  }
  float y4r[8];
  acc_rows8(na.Y4, y4r);                                     // gain pre-activations 0..2D-1
  float dsum = 0.f, asum = 0.f;
  if (ok && h == 0) {
    float av[D], snp[D], snv[D], ar[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const float kp = 2.f / (1.f + __expf(-y4r[2 * q])) + 0.2f;
      const float kv = 2.f / (1.f + __expf(-y4r[2 * q + 1])) + 0.2f;
      av[q] = -(kp * ex[q] + kv * sv[q]);
      if (a.noise) av[q] += a.noise[((long)b * a.n_env + i) * D + q];
    }
    if (a.noise_key) {
      // one coin per (env, step), Box-Muller normals per (agent, axis): the same draws for any
      // launch geometry, the native driver and the Python loop
      const int nbt = a.nb_total ? a.nb_total : a.B;     // per-env sub-arguments: global env b0 + b
      const uint64_t kb = mix64(*a.noise_key ^ (0x9E3779B97F4A7C15ull * (uint64_t)(a.noise_t * nbt + a.b0 + b + 1)));
      if (u01(kb) < a.noise_prob) {
#pragma unroll
        for (int q = 0; q < D; ++q) {
          const uint64_t ka = kb + 2ull * (uint64_t)(i * D + q) + 1ull;
          const float u1 = fmaxf(u01(mix64(ka)), 1e-12f), u2 = u01(mix64(ka + 0xD1B54A32D192ED03ull));
          av[q] += a.noise_scale * sqrtf(-2.f * __logf(u1)) * __cosf(6.28318530718f * u2);
        }
      }
    }
    if (a.A) {
#pragma unroll
      for (int q = 0; q < D; ++q) a.A[((long)b * a.a_env + i) * D + q] = av[q];
    }
#pragma unroll
    for (int q = 0; q < D; ++q) {
      snp[q] = sp[q] + sv[q] * a.dt;
      snv[q] = sv[q] + av[q] * a.dt;
      ar[q] = -(ex[q] + a.sqrt3 * sv[q]);
    }
    if (a.Snext) store_rec<D>(a.Snext + (long)b * a.sn_env * REC<D>, (unsigned)i, snp, snv);
    float dd[D];
#pragma unroll
    for (int q = 0; q < D; ++q) dd[q] = snp[q] - gg[q];
    dsum = sqrtf(sqsum<D>(dd));
    asum = fabsf(sqsum<D>(av) - sqsum<D>(ar));
  }
  // per-env sums in fixed point: every agent's term is rounded to an integer first, so the
  // integer wave sums and atomics give the same value for any grouping of agents over waves and
  // any arrival order (the early-stop input is launch-geometry independent)
  // (NaN / Inf / out of range -> FX_SAT: the float -> int conversion is undefined for them)
  auto fx = [](float v, double s) {
    const double x = (double)v * s;
    return (x >= 0.0 && x < FX_SAT) ? (unsigned long long)__double2ll_rn(x) : (unsigned long long)FX_SAT;
  };
  unsigned long long dq = 0, aq = 0;
  if (ok && h == 0) { dq = fx(dsum, FX_DIST); aq = fx(asum, FX_ACT); }
  const int last = min(g0 + APW - 1, total - 1);
  if (g0 / N == last / N) {      // the wave's agents share an env: one atomic per wave
    dq = wave_sum_u64(dq);
    aq = wave_sum_u64(aq);
    if (lane == 0) {
      const int be = g0 / N;
      if (a.dist_sum) atomicAdd(a.dist_sum + (long)be * a.d_env, dq);
      if (a.act_sum) atomicAdd(a.act_sum + (long)be * a.ac_env, aq);
    }
  } else if (ok && h == 0) {
    if (a.dist_sum) atomicAdd(a.dist_sum + (long)b * a.d_env, dq);
    if (a.act_sum) atomicAdd(a.act_sum + (long)b * a.ac_env, aq);
  }
}

// DENSE12 emission target of one lane for one tile: the row pointers of a group agent (pooled
// row [+ lo plane], argmax row; LDS pool row for the non-GPOOL path), computed once per tile
struct PoolDst { h16* prow; uint8_t* arow; bool ok; };

DEV PoolDst pool_dst(const CtrlArgs& a, const AgentBase& ab, int g0, int APW, int total, int al, h16* pool, bool gpool,
                     int r) {
  PoolDst d;
  d.ok = al < APW && g0 + al < total;
  d.prow = nullptr;
  d.arow = nullptr;
  if (d.ok) {
    int bb, ii;
    agent_bi(ab, al, a.N, bb, ii);
    d.prow = gpool ? a.pooled + (long)bb * a.p_env + (long)ii * PROW + r : pool + al * PSTR + r;
    if (a.argmax) d.arow = a.argmax + (long)bb * a.am_env + (long)ii * 128 + r;
  }
  return d;
}

template <bool IS_X3, bool GPOOL>
DEV void pool_store(const PoolDst& d, int nt, int pw_) {
  if constexpr ((MB_DIAG & 16) != 0) {           // diagnostics build: no pooled / argmax stores
    if (d.ok && pw_ == 0x7ffffff0) d.prow[32 * nt] = (h16)0.f;   // (keeps the pool computed)
    return;
  }
  if (!d.ok) return;
  const float pv = __int_as_float(pw_ & -16);
  const h16 ph = (h16)pv;
  d.prow[32 * nt] = ph;
  if constexpr (IS_X3 && GPOOL) d.prow[32 * nt + 128] = (h16)(pv - (float)ph);
  if (d.arow) d.arow[32 * nt] = (pw_ > 15) ? (uint8_t)(15 - (pw_ & 15)) : (uint8_t)0xFF;
}

// DENSE12 pool of edge tile q (see ctrl_fwd_groups): Z = relu-free pre-activations of the tile's
// 32 edges (rows) x 128 features (4 column tiles), mask32 = in-radius rows: the tile's context
// (emission targets, per-row slot codes), then one step per column tile. (Issuing each column
// tile's pool right after the next one's MFMA chain measured neutral in round 5: phase clocks
// 6.8 -> 6.4 k cycles per tile, headline within noise, profiles/r5_b11/.)
struct PoolCtx { PoolDst d1, d2; int crow[16]; int ph; };

template <bool GPOOL>
DEV PoolCtx pool_ctx12(const CtrlArgs& a, const AgentBase& ab, int g0, int APW, int total, int q, unsigned mask32,
                       h16* pool, int lane) {
  const int r = lane & 31, h = lane >> 5;
  PoolCtx c;
  c.ph = (2 * q) % 3;                          // tile phase (uniform)
  const int af = (8 * q) / 3;                  // first agent (group-relative) with rows in the tile
  const bool three = c.ph != 0;                // agents completed in this tile: 2 (ph 0) or 3
  // this lane's emissions: half 0 the tile's 1st and 3rd completed agent, half 1 the 2nd
  c.d1 = pool_dst(a, ab, g0, APW, total, af + h, pool, GPOOL, r);
  c.d2 = pool_dst(a, ab, g0, APW, total, (h == 0 && three) ? af + 2 : APW, pool, GPOOL, r);
  // slot code of every accumulator row: quad j = 2m + h holds slots 4 ((ph + j) mod 3) + i
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int sq = 4 * ((c.ph + 2 * m + h) % 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int reg = 4 * m + i;
      c.crow[reg] = ((mask32 >> acc_row(reg, h)) & 1u) ? (15 - (sq + i)) : INT_MIN;
    }
  }
  return c;
}

template <bool IS_X3, bool GPOOL>
DEV void pool_step12(const PoolCtx& c, int nt, const f32x16& Zn, int& carry, int lane) {
  const int h = lane >> 5;
  int g[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    int v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (__float_as_int(Zn[4 * m + i]) & -16) | c.crow[4 * m + i];
    g[m] = max(max(max(0, v[0]), max(v[1], v[2])), v[3]);
  }
  int Q[8];                                    // quad maxima of the whole tile, in row order
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int o = shfl_xor32i(g[m]);
    Q[2 * m] = h ? o : g[m];
    Q[2 * m + 1] = h ? g[m] : o;
  }
  // agents of the tile: ph 0: [0-2] [3-5] [6,7 -> carry]; ph 2: [carry, 0] [1-3] [4-6] [7 -> carry];
  // ph 1: [carry, 0, 1] [2-4] [5-7]
  int e0, e1, e2;
  if (c.ph == 0) {
    e0 = max(max(Q[0], Q[1]), Q[2]);
    e1 = max(max(Q[3], Q[4]), Q[5]);
    e2 = 0;
    carry = max(Q[6], Q[7]);
  } else if (c.ph == 2) {
    e0 = max(carry, Q[0]);
    e1 = max(max(Q[1], Q[2]), Q[3]);
    e2 = max(max(Q[4], Q[5]), Q[6]);
    carry = Q[7];
  } else {
    e0 = max(max(carry, Q[0]), Q[1]);
    e1 = max(max(Q[2], Q[3]), Q[4]);
    e2 = max(max(Q[5], Q[6]), Q[7]);
    carry = 0;
  }
  pool_store<IS_X3, GPOOL>(c.d1, nt, h ? e1 : e0);
  pool_store<IS_X3, GPOOL>(c.d2, nt, e2);
}

template <bool IS_X3, bool GPOOL>
DEV void pool_dense12(const CtrlArgs& a, const AgentBase& ab, int g0, int APW, int total, int q, unsigned mask32,
                      const f32x16 (&Z)[4], int (&carry)[4], h16* pool, int lane) {
  const PoolCtx c = pool_ctx12<GPOOL>(a, ab, g0, APW, total, q, mask32, pool, lane);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) pool_step12<IS_X3, GPOOL>(c, nt, Z[nt], carry[nt], lane);
}

// Controller step. bf16 / fp16: edge and node phase in one kernel, the pooled features cross
// from the edge lanes (features) to the node lanes (agents) through a per-wave LDS image.
// x3: the split weights do not fit one workgroup's LDS together, so this kernel runs the edge
// phase only and writes the pooled features ([hi | lo] rows, always stored) straight to global
// memory; ctrl_node_fwd_kernel reads them back as node-layer B fragments.
// Body of the controller step over the agent groups grp0, grp0 + gstride, ... of `a` (weights
// already in LDS: wl = ew1f|ew2, wn = nw1f..nw4, vl = CTRL_VEC floats, pools = one 32-row pool
// image per wave). SPLIT (always for x3): edge phase only, the pooled rows go to global memory
// and ctrl_node_groups runs the node phase.
constexpr int CTRL_HOIST_EB = 1;
constexpr int CTRL_FWD_DENSE = 1;
// DENSE12 (K = 12, agents per wave a multiple of 8): dense edge rows -- a group's APW agents x 12
// slots are APW * 12 / 32 tiles of 32 consecutive edges (no padding slots). Rows come in quads of
// 4 that never straddle an agent (12 = 3 quads); tile q covers quads j = 0..7 of agents
// floor((8q + j) / 3), a pattern with period 3 tiles (8 agents): phase ph = 2q mod 3. The pool
// takes the max per quad, exchanges quads across the lane halves, then per agent the max of its
// quads (an agent that straddles two tiles carries its partial max in a register). Pooled values
// and argmax slots are bit-identical to the 2-agent x 16-slot path (same per-edge MFMA values,
// same slot codes and tie rule).
// ST (diagnostics, x3 fused step): per-wave phase clocks to a.stamps[(block * 8 + wave) * 16 + k]:
// 0 weight staging (from t0, the kernel start), 1 group prologue loads, per edge tile 2 load issue,
// 3 edge features, 4 edge MLP, 5 pool + stores; 6 pooled-store wait, 7 node phase; 15 tile count
// (scripts/stamps_ctrl.py). A separate instantiation: no runtime stamp branches in production.
template <int D, bool SPLIT, bool GNODE = false, bool DENSE12 = false, bool ST = false, bool ACTS = false>
DEV void ctrl_fwd_groups(const CtrlArgs& a, const h16* wl, const h16* wn, const float* vl, h16* pools, int grp0,
                         int gstride, unsigned long long t0 = 0) {
  constexpr bool GPOOL = X3 || SPLIT;
  unsigned long long ph[16] = {}, tck = t0;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[k] += t - tck;
      tck = t;
    }
  };
  stamp(0);
  const float* eb2 = vl;
  const float* nb2 = vl + 128;
  const float* nb3 = vl + 256;
  const float* nb4 = vl + 320;

  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  h16* pool = pools + wave * 32 * PSTR;
  const int N = a.N, K = a.K;
  const int total = a.B * N;

  // agents per wave: 32, or 4..16 for small scenes (more waves share the edge phase; the node
  // phase's MFMA rows beyond APW carry ignored data)
  const int APW = (a.apw >= 2 && a.apw <= 32) ? a.apw : 32;
  // x3 fused step: 2 waves/SIMD whatever the register count (145 KB LDS per 8-wave workgroup),
  // so the 64 bias registers are free
  constexpr bool HOIST_EB = CTRL_HOIST_EB && X3 && GNODE;
  f32x16 zb[4];
  if constexpr (HOIST_EB) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float bv = eb2[32 * nt + r];
#pragma unroll
      for (int q = 0; q < 16; ++q) zb[nt][q] = bv;
    }
  }
  for (int grp = grp0; grp * APW < total; grp += gstride) {
    const int g0 = grp * APW;
    const AgentBase ab = agent_base(g0, N);
    // ---------------- edge phase: APW/2 tiles x (2 agents x 16 slots), or APW*12/32 dense tiles
    // (DENSE12); the gathers of tile q+1
    // (idx -> s_j, dependent global loads) are issued before tile q's MFMA chain
    constexpr unsigned INV12 = (65536u + 11u) / 12u;
    auto idx_load = [&](int q, EdgeIdx& o) {
      if constexpr (DENSE12) ctrl_idx_load_dense(a.idx, a.i_env, N, 12, INV12, ab, q, r, total, o, APW);
      else ctrl_idx_load(a.idx, a.i_env, N, K, ab, q, r, total, o);
    };
    const int NTL = DENSE12 ? APW * 12 / 32 : APW / 2;          // edge tiles of the group
    int carry[4] = {0, 0, 0, 0};                                // DENSE12: straddling agent's partial pool
    EdgeIdx xi1;
    EdgeSt<D> xs0;
    {
      EdgeIdx xi0;
      idx_load(0, xi0);
      ctrl_st_load<D>(a.S, a.s_env, xi0, xs0);
      idx_load(1, xi1);
    }
    stamp(1);
    for (int q = 0; q < NTL; ++q) {
      if constexpr (ST) ph[15] += 1;
      const EdgeSt<D> cur = xs0;
      ctrl_st_load<D>(a.S, a.s_env, xi1, xs0);                    // states of tile q+1
      idx_load(q + 2, xi1);                                        // idx of tile q+2
      stamp(2);
      const bool ok = cur.ok;
      const float eye = (cur.j == cur.i) ? 1.f : 0.f;
      float rp[D], rv[D];
      edge_rel<D>(cur, rp, rv);
      const bool m = ok && (sqrtf(sqsum<D>(rp)) < a.obs_r);   // strict, un-eps'd (controller.py:38-39)
      const h16x8 F = ctrl_edge_frag<D>(rp, rv, eye, ok, h);
      stamp(3);
      f32x16 Z[4];
      ctrl_edge_tile(F, wl + opaque_zero(), eb2, lane, Z, HOIST_EB ? zb : nullptr);
      const unsigned mask32 = (unsigned)(__ballot(m) & 0xffffffffull);
      stamp(4);
      if constexpr (DENSE12) {
        pool_dense12<X3, GPOOL>(a, ab, g0, APW, total, q, mask32, Z, carry, pool, lane);
        stamp(5);
        continue;
      }
      // Masked max-pool of relu(Z) over each agent's 16 rows with the first-occurrence argmax,
      // as ONE signed-int max per element: v = (bits(Z) & ~15) | c_row, c_row = 15 - slot for
      // in-radius rows and INT_MIN for masked ones. Non-negative floats order as ints, so the
      // max is the largest value (its low 4 mantissa bits replaced: < 16 ulp, below the h16
      // rounding of the pooled value), ties and near-ties (< 16 ulp) go to the lowest slot,
      // negative / masked rows never beat the initial 0 (relu), and the winning slot is read
      // back from the low bits. (replaces compare + 3 selects per element and the tie logic)
      int crow[16];
#pragma unroll
      for (int reg = 0; reg < 16; ++reg)
        crow[reg] = ((mask32 >> acc_row(reg, h)) & 1u) ? (15 - (acc_row(reg, h) & 15)) : INT_MIN;
      const int arow = 2 * q + h;   // h==0 writes agent 2q, h==1 agent 2q+1
      int bb = 0, ii = 0;
      const int ga = g0 + arow;
      const bool gout = (a.argmax || GPOOL) && ga < total;
      if (gout) agent_bi(ab, arow, N, bb, ii);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        int p0 = 0, p1 = 0;
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) {
          p0 = max(p0, (__float_as_int(Z[nt][reg]) & -16) | crow[reg]);
          p1 = max(p1, (__float_as_int(Z[nt][reg + 8]) & -16) | crow[reg + 8]);
        }
        p0 = max(p0, shfl_xor32i(p0));
        p1 = max(p1, shfl_xor32i(p1));
        const int pw_ = (h == 0) ? p0 : p1;
        const float pv = __int_as_float(pw_ & -16);
        if constexpr (GPOOL) {
          if (gout) {
            h16* prow = a.pooled + (long)bb * a.p_env + (long)ii * PROW + 32 * nt + r;
            const h16 ph = (h16)pv;
            prow[0] = ph;
            if constexpr (X3) prow[128] = (h16)(pv - (float)ph);
          }
        } else {
          pool[arow * PSTR + 32 * nt + r] = (h16)pv;
        }
        if (a.argmax && ga < total)
          a.argmax[(long)bb * a.am_env + (long)ii * 128 + 32 * nt + r] =
              (pw_ > 15) ? (uint8_t)(15 - (pw_ & 15)) : (uint8_t)0xFF;
      }
    }
    if constexpr (GPOOL && GNODE) {
      // x3 fused step: the group's node phase right here, over the pooled rows this wave just
      // wrote to global memory (the stores are complete after the wait; the rows were not read
      // before, so no stale L1 line can hide them)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(6);
      const int gi = min(g0 + min(r, APW - 1), total - 1);
      int bb, ii;
      agent_bi(ab, gi - g0, N, bb, ii);
      const h16* prow = a.pooled + (long)bb * a.p_env + (long)ii * PROW + 8 * h;
      node_phase<D, ACTS>(a, g0, APW, total, [&](int kk) { return row_fr(prow + 16 * kk, 128); }, wn, nb2, nb3, nb4, lane);
      stamp(7);
      continue;
    }
    if constexpr (GPOOL) continue;     // node phase: ctrl_node_groups
    lds_wave_sync();
    if (a.pooled) {   // 32 agents x 256 B, 16 B per lane
      for (int u = lane; u < 32 * 16; u += 64) {
        const int ag = u >> 4, ch = u & 15;
        const int ga = g0 + ag;
        if (ag < APW && ga < total) {
          const int bb = ga / N, ii = ga - bb * N;
          *reinterpret_cast<h16x8*>(a.pooled + (long)bb * a.p_env + (long)ii * 128 + ch * 8) =
              *reinterpret_cast<const h16x8*>(pool + ag * PSTR + ch * 8);
        }
      }
    }
    // ---------------- node phase: lane column r = agent g0 + r
    node_phase<D, ACTS>(a, g0, APW, total, [&](int kk) { return row_fr(pool + r * PSTR + 16 * kk + 8 * h, 0); },
                  wn, nb2, nb3, nb4, lane);
    // the pool image is rewritten by the next group: finish all reads first
    lds_wave_sync();
  }
  if constexpr (ST) {
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < 16; ++k) a.stamps[((long)blockIdx.x * (blockDim.x / WAVE) + wave) * 16 + k] = ph[k];
  }
}

// Early-stop publication: the host decides the early stop from the per-env goal-distance sums
// of the previous step. Instead of a queue marker after every controller step (the next
// dispatch waits for its completion signal: ~7 us per step) and a copy on a side stream, the
// kernel that completes the sums hands them to the host itself: every workgroup retires its
// fixed-point atomics (agent-scope fence), then counts itself done; the last one reads the B
// sums from L2, stores them to host-coherent memory, and releases the step's flag (system
// scope) with the rollout's generation number, which the host polls. All threads call it.
DEV void publish_step(const CtrlArgs& a) {
  if (!a.pub_ctr) return;
  // Per-workgroup path: no fence instructions (an agent- or system-scope fence in EVERY workgroup
  // writes back / invalidates the L2 -- measured +0.7 ms per iteration). Each wave waits until its
  // dist_sum atomics are acknowledged (performed at the device-coherent level) before the
  // workgroup counts itself done with a relaxed agent-scope add: the remaining hardware-order
  // assumption (gfx950: an acknowledged device-scope atomic is visible to every later agent-scope
  // access; MI355X_MICROARCH "Valid forms", row 1). The single last workgroup then acquires
  // (agent scope) before reading the sums and releases (system scope) before the host flag.
  __shared__ unsigned pub_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's dist_sum atomics acknowledged
  __syncthreads();
  if (threadIdx.x == 0) {
    pub_last = __hip_atomic_fetch_add(a.pub_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 ? 1u : 0u;
    if (pub_last) {
      // every workgroup has counted itself: re-arm the counter for the next rollout (no memset
      // launch per rollout; the kernel boundary orders it before the next use)
      __hip_atomic_store(a.pub_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!pub_last) return;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    const unsigned long long v = __hip_atomic_load(a.dist_sum + (long)b * a.d_env, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.pub_dist + b, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the host-coherent stores acknowledged
  __syncthreads();
  if (threadIdx.x == 0) {
    // release (system scope) by one lane of one workgroup, then the flag; the explicit wait keeps
    // the write-back ahead of the flag (MI355X_MICROARCH: compiler hazard after buffer_wbl2).
    // The host polls the flag with an acquire load (csrc/runtime.cpp wait_published).
    // (Without the release -- the host reads only pub_dist and the flag, both written to
    // fine-grained host memory by system-scope stores -- the headline ran the same: 10.686-10.712
    // vs 10.703-10.706 ms, profiles/r5_b1/; kept.)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.pub_flag, a.pub_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// FUSE (x3): all 72 fragments in LDS (145 KB) and the node phase of each group in the same
// wave right after its edge phase (pooled rows through global memory): one launch per step.
template <int WAVES, int D, bool FUSE, bool ST, bool ACTS>
DEV void ctrl_fwd_body(const CtrlArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned long long t0 = ST ? __builtin_amdgcn_s_memtime() : 0ull;
  constexpr int NFR = (X3 && !FUSE) ? 18 : CTRL_FWD_FRAGS;          // fragments staged in LDS
  h16* wl = reinterpret_cast<h16*>(smem);                            // ew1f, ew2 (18 frags)
  h16* wn = wl + 18 * FRAG_ELEMS;                                     // nw1f..nw4 (54 frags)
  float* vl = reinterpret_cast<float*>(smem + NFR * FRAG_SZ);
  h16* pools = reinterpret_cast<h16*>(smem + NFR * FRAG_SZ + CTRL_VEC * 4);
  block_copy16(wl, a.wpack + (size_t)a.f_edge * FRAG_ELEMS, 18 * FRAG_SZ, false);
  if constexpr (!X3 || FUSE) block_copy16(wn, a.wpack + (size_t)a.f_node * FRAG_ELEMS, 54 * FRAG_SZ, false);
  block_copy16(vl, a.wvec, CTRL_VEC * 4);
  __syncthreads();
  const int apw = (a.apw >= 2 && a.apw <= 32) ? a.apw : 32;
  // remap over the blocks that have a group (a small scene leaves most of the grid idle: the
  // remap must not gather the busy ones onto one XCD)
  const int ngrp = (a.B * a.N + apw - 1) / apw;
  const int nact = min((int)gridDim.x, (ngrp + WAVES - 1) / WAVES);
  const int lb = (ROLL_XCD && (int)blockIdx.x < nact) ? xcd_block((int)blockIdx.x, nact) : (int)blockIdx.x;
  if (CTRL_FWD_DENSE && a.K == 12 && apw % 8 == 0)
    ctrl_fwd_groups<D, false, FUSE, true, ST, ACTS>(a, wl, wn, vl, pools, lb * WAVES + wave_id(), gridDim.x * WAVES, t0);
  else
    ctrl_fwd_groups<D, false, FUSE, false, ST, ACTS>(a, wl, wn, vl, pools, lb * WAVES + wave_id(), gridDim.x * WAVES, t0);
  if constexpr (!X3 || FUSE) publish_step(a);   // the x3 split path publishes from its node kernel
}

template <int WAVES, int D, bool FUSE = false, bool ST = false>
__global__ __launch_bounds__(WAVES * 64) void ctrl_fwd_kernel(CtrlArgs a) {
  ctrl_fwd_body<WAVES, D, FUSE, ST, false>(a);
}

// the same step, also storing each agent's node activations for the backward (node_acts)
template <int WAVES, int D, bool FUSE = false>
__global__ __launch_bounds__(WAVES * 64) void ctrl_fwd_acts_kernel(CtrlArgs a) {
  ctrl_fwd_body<WAVES, D, FUSE, false, true>(a);
}

// Node phase of the controller step over the pooled rows in global memory, 32-agent groups
// grp0, grp0 + gstride, ... (x3 steps, and the persistent small-scene rollout)
template <int D, bool ACTS = false>
DEV void ctrl_node_groups(const CtrlArgs& a, const h16* wn, const float* vl, int grp0, int gstride) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int N = a.N;
  const int total = a.B * N;
  for (int grp = grp0; grp * 32 < total; grp += gstride) {
    const int g0 = grp * 32;
    const int gi = min(g0 + r, total - 1);
    const int b = gi / N, i = gi - b * N;
    const h16* prow = a.pooled + (long)b * a.p_env + (long)i * PROW + 8 * h;
    node_phase<D, ACTS>(a, g0, 32, total, [&](int kk) { return row_fr(prow + 16 * kk, 128); }, wn, vl + 128, vl + 256,
                  vl + 320, lane);
  }
}

// x3 node phase of the controller step over the pooled rows written by ctrl_fwd_kernel
template <int WAVES, int D, bool ACTS = false>
__global__ __launch_bounds__(WAVES * 64) void ctrl_node_fwd_kernel(CtrlArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* wn = reinterpret_cast<h16*>(smem);                             // nw1f..nw4 (54 frags)
  float* vl = reinterpret_cast<float*>(smem + 54 * FRAG_SZ);
  block_copy16(wn, a.wpack + (size_t)a.f_node * FRAG_ELEMS, 54 * FRAG_SZ, false);
  block_copy16(vl, a.wvec, CTRL_VEC * 4);
  __syncthreads();
  ctrl_node_groups<D, ACTS>(a, wn, vl, blockIdx.x * WAVES + wave_id(), gridDim.x * WAVES);
  publish_step(a);
}

constexpr int CTRL_WAVES = 8;

size_t ctrl_fwd_lds() {
  if constexpr (X3) return (size_t)18 * FRAG_SZ + CTRL_VEC * 4;
  return (size_t)CTRL_FWD_FRAGS * FRAG_BYTES + CTRL_VEC * 4 + (size_t)CTRL_WAVES * 32 * PSTR * 2;
}

}  // namespace MB_PREC
}  // namespace mb

extern "C" int MB_SYM(ctrl_fwd)(const mb::CtrlArgs* a, int num_cu, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (a->K > 16 || a->K < 1) return -1;
  if (X3 && !a->pooled) return -2;            // the x3 node phase reads the stored pooled rows
  const int apw = (a->apw >= 2 && a->apw <= 32 && !(a->apw & 1)) ? a->apw : 32;
  const int groups = (a->B * a->N + apw - 1) / apw;
  int blocks = (groups + CTRL_WAVES - 1) / CTRL_WAVES;
  const int maxb = num_cu > 0 ? num_cu * 2 : blocks;
  if (blocks > maxb) blocks = maxb;
  CtrlArgs b = *a;
  b.apw = apw;
  // x3: one fused launch (edge + node phase per group, 145 KB of weights: one workgroup per CU)
  if (X3) {
    const size_t ldf = (size_t)CTRL_FWD_FRAGS * FRAG_SZ + CTRL_VEC * 4;
    auto go = [&](auto kern) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldf);
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(CTRL_WAVES * 64), ldf, st, b);
    };
    // (4-wave workgroups for the slices' small grids -- one wave per SIMD on twice the CUs --
    // measured no faster: 8-env slice 2.825-2.833 vs 2.797-2.820 ms, profiles/r6b/)
    if (a->dim == 3) {
      if (a->stamps) go(ctrl_fwd_kernel<CTRL_WAVES, 3, true, true>);
      else if (a->acts) go(ctrl_fwd_acts_kernel<CTRL_WAVES, 3, true>);
      else go(ctrl_fwd_kernel<CTRL_WAVES, 3, true>);
    } else {
      if (a->stamps) go(ctrl_fwd_kernel<CTRL_WAVES, 2, true, true>);
      else if (a->acts) go(ctrl_fwd_acts_kernel<CTRL_WAVES, 2, true>);
      else go(ctrl_fwd_kernel<CTRL_WAVES, 2, true>);
    }
    return (int)hipGetLastError();
  }
  const size_t lds = ctrl_fwd_lds();
  auto go1 = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(CTRL_WAVES * 64), lds, st, b);
  };
  if (a->dim == 3) {
    if (a->acts) go1(ctrl_fwd_acts_kernel<CTRL_WAVES, 3>);
    else go1(ctrl_fwd_kernel<CTRL_WAVES, 3>);
  } else {
    if (a->acts) go1(ctrl_fwd_acts_kernel<CTRL_WAVES, 2>);
    else go1(ctrl_fwd_kernel<CTRL_WAVES, 2>);
  }
  if constexpr (X3) {
    const size_t ldn = (size_t)54 * FRAG_SZ + CTRL_VEC * 4;
    int nblocks = (a->B * a->N + 32 * CTRL_WAVES - 1) / (32 * CTRL_WAVES);     // 32-agent node groups
    if (nblocks > maxb) nblocks = maxb;
    if (a->dim == 3) {
      (void)hipFuncSetAttribute((const void*)ctrl_node_fwd_kernel<CTRL_WAVES, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldn);
      hipLaunchKernelGGL((ctrl_node_fwd_kernel<CTRL_WAVES, 3>), dim3(nblocks), dim3(CTRL_WAVES * 64), ldn, st, b);
    } else {
      (void)hipFuncSetAttribute((const void*)ctrl_node_fwd_kernel<CTRL_WAVES, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldn);
      hipLaunchKernelGGL((ctrl_node_fwd_kernel<CTRL_WAVES, 2>), dim3(nblocks), dim3(CTRL_WAVES * 64), ldn, st, b);
    }
  }
  return (int)hipGetLastError();
}

// =======================================================================================
// Controller backward for one timestep of the BPTT recursion (reference: autograd through
// controller.py:31-63 inside train.py:103). Two kernels, because the node MLP (4 layers,
// forward + transposed weights) and the edge MLP (recompute + backward) do not fit one
// workgroup's LDS together with the weight-gradient staging:
//   ctrl_node_bwd: pooled features (stored by the rollout) -> node MLP recompute -> gain law
//     backward (dA = dt*G_{t+1}[v] + action-loss grad) -> dY4..dY1 -> dL/dpooled (to
//     global, h16) + dL/ds_t of the ego terms; node weight grads (WG-shared, 4 stages).
//   ctrl_edge_bwd: edge MLP recompute, max-pool backward via the stored argmax slots,
//     dH1 = W2^T dZ, dF = W1^T dH1 -> per-edge dL/d(s_i - s_j); edge weight grads.
// Weight gradients accumulate into a fixed per-workgroup slab across all timesteps
// (slab += partial, deterministic) and are reduced once after the recursion.
// =======================================================================================
namespace mb {
namespace MB_PREC {

constexpr int NB_WAVES = 4;
constexpr int NB_CH = NB_WAVES * 32;                  // agents per chunk
constexpr int NS1 = 168, NS2 = 68, NS3 = 132, NS4 = 68;   // row-major image strides (NS2..4: 2*odd dwords, conflict-free ds_read_b64 row reads)
constexpr int NODE_RM_ELEMS = 64 * NS1 + 128 * NS2 + 64 * NS3 + 32 * NS4;
constexpr int NODE_RM_LO = NODE_RM_ELEMS;             // lo plane offset of the images (x3)
constexpr int NP_W1 = 0, NP_W2 = 10240, NP_B2 = 18432, NP_W3 = 18560, NP_B3 = 26752, NP_W4 = 26816, NP_B4 = 28864;
constexpr int CTRL_NODE_PARTIAL = 28896;
// weight-gradient stages: a region holds the rows of NB_TW waves (all of them in the 1-pass
// builds; one in x3, whose images carry a lo plane) -> NB_NT turns per stage
constexpr int NB_TW = X3 ? 1 : NB_WAVES;
constexpr int NB_NT = NB_WAVES / NB_TW;
constexpr int NB_RT = NB_TW * 32;                     // region rows
constexpr int NB_KST = NB_RT / 16;                    // agent steps per turn
// stage image row strides (h16 elements) for 32 / 64 / 128-wide images and the 160-wide
// pooled|state image of S1
constexpr int NBS64 = 72;
constexpr int NBS128 = 136;
constexpr int NBSP = 168;
// stages S4 and S3 share one set of turns (their four images fit one region)
constexpr int NBS_32 = 40, NBS_64 = NBS64, NBS_128 = NBS128, NBS_P = NBSP;
constexpr int nb_max(int a, int b) { return a > b ? a : b; }
constexpr int NB_PL = nb_max(nb_max(NBS_P + NBS_64, NBS_128 + NBS_64),
                             NBS_32 + 2 * NBS_64 + NBS_128) * NB_RT;   // elements per region plane
constexpr size_t NB_STAGE = (size_t)(X3 ? 2 : 1) * NB_PL * 2;

size_t ctrl_node_bwd_lds() { return (size_t)(X3 ? 2 : 1) * NODE_RM_ELEMS * 2 + CTRL_VEC * 4 + NB_STAGE; }

DEV float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

DEV void add_tile(float* dst, int ncols, int mt, int nt, const f32x16& c, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) dst[(32 * mt + acc_row(reg, h)) * ncols + 32 * nt + r] += c[reg];
}

// Split slab read-modify-write: the compiler may not move a slab load above an earlier slab
// store (same base pointer, runtime tile offsets), so back-to-back add_tile calls serialise one
// memory round trip per tile. Tails load every owned slab element first (load_tile), then add
// and store (store_tile_add): one round trip in total.
DEV void load_tile(f32x16& v, const float* src, int ncols, int mt, int nt, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) v[reg] = src[(32 * mt + acc_row(reg, h)) * ncols + 32 * nt + r];
}

DEV void store_tile_add(float* dst, int ncols, int mt, int nt, const f32x16& old, const f32x16& c, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) dst[(32 * mt + acc_row(reg, h)) * ncols + 32 * nt + r] = old[reg] + c[reg];
}

// Fused BPTT combine (replaces the node_combine launch between two reverse steps): G_{t+1} of
// agent i = dS_{t+1} + ego_{t+1} + sum_k dEc[i,k] - sum_in dEc[e] + the Euler adjoint of G_{t+2},
// the terms and addition order of combine.h combine_node. The agent's two lane halves (h) split
// its out- and in-edges, one lane swap adds the halves: fixed order, deterministic. All lanes
// call it (lane swaps); lanes without an agent get zeros. Both halves return G_{t+1}; half 0
// stores it (the next reverse step's Euler term).
// XO: lane distance between the two halves of an agent (32: lane halves h; 16: the g = 0 / 1
// lanes of the 16x16x32 node kernel)
constexpr int CMB_BT = 4;        // edge records per batch of the fused combine's gathers
template <int D, int XO = 32>
DEV void fused_combine(const CtrlNodeBwdArgs& a, bool ok, int b, int i, int h, float (&gp)[D], float (&gv)[D]) {
  constexpr int R = REC<D>;
  const int N = a.N, K = a.K;
  float4 g[R];
#pragma unroll
  for (int q = 0; q < R; ++q) g[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  float dp[D], dv[D], ep[D], ev[D], np_[D], nv[D];
#pragma unroll
  for (int q = 0; q < D; ++q) { dp[q] = dv[q] = ep[q] = ev[q] = np_[q] = nv[q] = 0.f; }
  if (ok) {
    load_rec<D>(a.cdS + (long)b * a.cds_env * R, (unsigned)i, dp, dv);
    load_rec<D>(a.cego + (long)b * N * R, (unsigned)i, ep, ev);
    if (a.cGn) load_rec<D>(a.cGn + (long)b * a.cgn_env * R, (unsigned)i, np_, nv);
    const float4* dE = a.cdEc + (long)b * N * K * R;
    // batches of CMB_BT records in flight (clamped indices, unconditional loads, predicated adds in
    // the original order): a loop of dependent load -> add iterations waits one memory latency per
    // edge (ptr -> edges -> record for the in-edges), ~12 latencies per agent
#pragma unroll 1
    for (int k0 = h; k0 < K; k0 += 2 * CMB_BT) {
      float4 v[CMB_BT][R];
#pragma unroll
      for (int u = 0; u < CMB_BT; ++u) {
        const int k = min(k0 + 2 * u, K - 1);
#pragma unroll
        for (int q = 0; q < R; ++q) v[u][q] = dE[((long)i * K + k) * R + q];
      }
#pragma unroll
      for (int u = 0; u < CMB_BT; ++u)
        if (k0 + 2 * u < K) acc_rec_v<R, 1>(g, v[u]);
    }
    const int* ptr = a.cptr + (long)b * a.cptr_env;
    const int* edges = a.cedges + (long)b * a.cedges_env;
    const int q0 = ptr[i], q1 = ptr[i + 1];
#pragma unroll 1
    for (int qb = q0 + h; qb < q1; qb += 2 * CMB_BT) {
      int e[CMB_BT];
#pragma unroll
      for (int u = 0; u < CMB_BT; ++u) e[u] = edges[min(qb + 2 * u, q1 - 1)];
      float4 v[CMB_BT][R];
#pragma unroll
      for (int u = 0; u < CMB_BT; ++u)
#pragma unroll
        for (int q = 0; q < R; ++q) v[u][q] = dE[(long)e[u] * R + q];
#pragma unroll
      for (int u = 0; u < CMB_BT; ++u)
        if (qb + 2 * u < q1) acc_rec_v<R, -1>(g, v[u]);
    }
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    g[q].x += lane_xorf<XO>(g[q].x); g[q].y += lane_xorf<XO>(g[q].y);
    g[q].z += lane_xorf<XO>(g[q].z); g[q].w += lane_xorf<XO>(g[q].w);
  }
  float eg_p[D], eg_v[D];
  if (D == 2) { eg_p[0] = g[0].x; eg_p[1] = g[0].y; eg_v[0] = g[0].z; eg_v[1] = g[0].w; }
  else { eg_p[0] = g[0].x; eg_p[1] = g[0].y; eg_p[2] = g[0].z; eg_v[0] = g[R - 1].x; eg_v[1] = g[R - 1].y; eg_v[2] = g[R - 1].z; }
#pragma unroll
  for (int q = 0; q < D; ++q) {
    gp[q] = dp[q] + ep[q];
    gv[q] = dv[q] + ev[q];
    gp[q] += eg_p[q];
    gv[q] += eg_v[q];
    if (a.cGn) {
      gp[q] += np_[q];
      gv[q] += nv[q] + a.dt * np_[q];
    }
  }
  if (ok && h == 0 && a.cGout) store_rec<D>(a.cGout + (long)b * a.cgo_env * R, (unsigned)i, gp, gv);
}

// Node backward over the chunks c0, c0 + cstride, ... of `a` (smem: the kernel's dynamic LDS;
// P: this workgroup's slab row)
template <int D>
DEV void node_bwd_body(const CtrlNodeBwdArgs& a, unsigned char* smem, long c0, long cstride, float* P) {
  constexpr int RM = (X3 ? 2 : 1) * NODE_RM_ELEMS;
  h16* wr = reinterpret_cast<h16*>(smem);
  float* vl = reinterpret_cast<float*>(smem + RM * 2);
  h16* stg = reinterpret_cast<h16*>(smem + RM * 2 + CTRL_VEC * 4);
  block_copy16(wr, a.wrm, RM * 2, false);
  block_copy16(vl, a.wvec, CTRL_VEC * 4);
  __syncthreads();
  const float* nb2 = vl + 128;
  const float* nb3 = vl + 256;
  const float* nb4 = vl + 320;
  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int N = a.N;
  const int total = a.B * N;
  const int CA = (a.chunk == 32 || a.chunk == 64) ? a.chunk : NB_CH;   // agents per chunk
  const long nchunks = (total + CA - 1) / CA;
  const int erow = wave * 32 + r;
  const int trow = NB_NT == 1 ? erow : (wave % NB_TW) * 32 + r;   // this wave's rows inside a turn's region
  const int myturn = wave / NB_TW;
  constexpr int LO = NODE_RM_LO;

  f32x16 acc1[3], acc2[2], acc3[2], acc4;
#pragma unroll
  for (int q = 0; q < 3; ++q) acc1[q] = zero16();
  acc2[0] = acc2[1] = acc3[0] = acc3[1] = acc4 = zero16();
  float bs2[2] = {0.f, 0.f}, bs3[2] = {0.f, 0.f}, bs4 = 0.f;
  const int n1 = (wave < 2) ? 3 : 2;
  const h16x8 zz = zero_h8();

  // NB_PREFETCH: the next chunk's pooled rows are requested right after this chunk's layer 1 (the
  // last use of its own): their latency overlaps the rest of the chunk instead of stalling the
  // next chunk's layer 1 (one wave per SIMD has nothing else to run meanwhile)
constexpr int NB_PREFETCH = 1;
  Fr Pn[8];
  auto pooled_rows = [&](long ch, Fr (&dst)[8]) {
    const int gq = (int)(ch * CA) + erow;
    if (ch < nchunks && erow < CA && gq < total) {
      const int bq = gq / N, iq = gq - bq * N;
      const h16* prow = a.pooled + (long)bq * a.p_env + (long)iq * PROW;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) dst[kk] = row_fr(prow + 16 * kk + 8 * h, 128);
    } else {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) dst[kk].h = dst[kk].l = zz;
    }
  };
  if (NB_PREFETCH) pooled_rows(c0, Pn);
  for (long chunk = c0; chunk < nchunks; chunk += cstride) {
    const int ga = (int)(chunk * CA) + erow;
    const bool ok = erow < CA && ga < total;
    // stage turns holding at least one valid agent (a partial last chunk -- all but the first
    // for small scenes -- skips the turns of its empty waves: zero rows contribute nothing)
    const int nturn = min(NB_NT, (int)((min((long)CA, total - chunk * CA) + NB_RT - 1) / NB_RT));
    int b = 0, i = 0;
    float sp[D], sv[D], gg[D], av[D], gnp[D], gnv[D];
#pragma unroll
    for (int q = 0; q < D; ++q) { sp[q] = sv[q] = gg[q] = av[q] = gnp[q] = gnv[q] = 0.f; }
    bool vld = false;
    Fr Pf[8];                 // dead after Y1; S1 re-reads the pooled rows
    if (ok) {
      b = ga / N; i = ga - b * N;
      load_rec<D>(a.S + (long)b * a.s_env * REC<D>, (unsigned)i, sp, sv);
#pragma unroll
      for (int q = 0; q < D; ++q) {
        gg[q] = a.G[((long)b * N + i) * D + q];
        av[q] = a.A[((long)b * a.a_env + i) * D + q];
      }
      if (a.Gn && !a.cdS) load_rec<D>(a.Gn + (long)b * a.gn_env * REC<D>, (unsigned)i, gnp, gnv);
      vld = a.valid ? (a.valid[(long)b * a.v_env] != 0) : true;
      if (!NB_PREFETCH) {
        const h16* prow = a.pooled + (long)b * a.p_env + (long)i * PROW;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) Pf[kk] = row_fr(prow + 16 * kk + 8 * h, 128);
      }
    } else if (!NB_PREFETCH) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) Pf[kk].h = Pf[kk].l = zz;
    }
    if (NB_PREFETCH) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) Pf[kk] = Pn[kk];
    }
    if (a.cdS) fused_combine<D>(a, ok, b, i, h, gnp, gnv);      // G_{t+1} (all lanes: lane swaps)
    float ex[D];
#pragma unroll
    for (int q = 0; q < D; ++q) ex[q] = sp[q] - gg[q];
    const h16x8 sfr = node_state_frag<D>(ex, sv, ok, h);
    const h16* W1 = wr + opaque_zero();
    const h16* W2 = W1 + 64 * NS1;
    const h16* W3 = W2 + 128 * NS2;
    const h16* W4 = W3 + 64 * NS3;
    // ---- forward recompute
    Pk Y1b[2], Y2b[4], Y3b[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) c = mma(wrm_nat_fr(W1 + opaque_zero(), NS1, 32 * mt, kk, lane, LO), Pf[kk], c);
      c = mma_bx(wrm_nat_fr(W1 + opaque_zero(), NS1, 32 * mt, 8, lane, LO), sfr, c);
      relu_(c);
      Y1b[mt] = to_pk(c);
    }
    if (NB_PREFETCH) pooled_rows(chunk + cstride, Pn);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x16 c = bias_rows(nb2, 32 * mt, h);
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        c = mma(wrm_acc_fr(W2 + opaque_zero(), NS2, 32 * mt, kk, lane, LO), pk_fr<kk & 1>(Y1b[kk >> 1]), c);
      });
      relu_(c);
      Y2b[mt] = to_pk(c);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 c = bias_rows(nb3, 32 * mt, h);
      static_for<8>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        c = mma(wrm_acc_fr(W3 + opaque_zero(), NS3, 32 * mt, kk, lane, LO), pk_fr<kk & 1>(Y2b[kk >> 1]), c);
      });
      relu_(c);
      Y3b[mt] = to_pk(c);
    }
    f32x16 y4 = bias_rows(nb4, 0, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      y4 = mma(wrm_acc_fr(W4 + opaque_zero(), NS4, 0, kk, lane, LO), pk_fr<kk & 1>(Y3b[kk >> 1]), y4);
    });
    // ---- gain law + action loss backward (lanes h == 0 own agent r; gain rows 0..2D-1 are
    //      regs 0..3 of lane r and (D = 3) regs 0,1 of lane r + 32)
    float y4r[8];
    acc_rows8(y4, y4r);
    float d4r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) d4r[q] = 0.f;
    float egp[D], egv[D];                         // dL/d(p - g), dL/dv of the ego terms
#pragma unroll
    for (int q = 0; q < D; ++q) { egp[q] = 0.f; egv[q] = 0.f; }
    if (ok && h == 0) {
      float da[D], ar[D];
#pragma unroll
      for (int q = 0; q < D; ++q) { da[q] = a.dt * gnv[q]; ar[q] = -(ex[q] + a.sqrt3 * sv[q]); }
      float act_coef = a.act_scale ? a.act_coef / fmaxf(*a.act_scale, 1.f) : a.act_coef;
      if (a.gscale) act_coef *= *a.gscale;        // fp16: device loss scale
      if (vld && act_coef != 0.f) {
        const float diff = sqsum<D>(av) - sqsum<D>(ar);
        const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
        const float c = act_coef * sg;
#pragma unroll
        for (int q = 0; q < D; ++q) {
          da[q] += c * 2.f * av[q];
          egp[q] += c * 2.f * ar[q];
          egv[q] += c * 2.f * a.sqrt3 * ar[q];
        }
      }
      // a_d = -(k_{2d} e_d + k_{2d+1} v_d), k = 2 sigmoid(y) + 0.2
#pragma unroll
      for (int q = 0; q < D; ++q) {
        const float s0 = sigm(y4r[2 * q]), s1 = sigm(y4r[2 * q + 1]);
        const float kp = 2.f * s0 + 0.2f, kv = 2.f * s1 + 0.2f;
        egp[q] += -kp * da[q];
        egv[q] += -kv * da[q];
        d4r[2 * q] = -da[q] * ex[q] * 2.f * s0 * (1.f - s0);
        d4r[2 * q + 1] = -da[q] * sv[q] * 2.f * s1 * (1.f - s1);
      }
    }
    // back to the accumulator layout: rows 0..3 -> regs 0..3 of h = 0, rows 4..7 -> of h = 1
    f32x16 d4 = zero16();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float hi4 = shfl_xor32(d4r[4 + q]);
      d4[q] = (h == 0) ? d4r[q] : hi4;
    }
    const Pk d4b = to_pk(d4);
    // Backward chain interleaved with the WG-shared weight-gradient stages so that each
    // activation dies right after its last use (register pressure). A stage runs in NB_NT
    // turns: the waves of a turn store their rows, every wave contracts them.
    // ---- dY3 = W4^T dY4 (K = 32) . relu'(Y3)
    Pk d3b[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 c = zero16();
      static_for<2>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        c = mma(wrmT_acc_fr(W4 + opaque_zero(), NS4, 32 * mt, kk, lane, LO), pk_fr<kk & 1>(d4b), c);
      });
      d3b[mt] = to_pk(c);
      mask_pk(d3b[mt], Y3b[mt]);
    }
#pragma unroll 1
    for (int turn = 0; turn < nturn; ++turn) {   // S4 + S3: dWn4pad += dY4 . Y3^T ; nb4 | dWn3 += dY3 . Y2^T ; nb3
      h16* im4A = stg;
      h16* im4B = im4A + NB_RT * NBS_32;
      h16* im3A = im4B + NB_RT * NBS_64;
      h16* im3B = im3A + NB_RT * NBS_64;
      if (NB_NT == 1 || myturn == turn) {
        store_pk(im4A, NBS_32, trow, 0, d4b, h, NB_PL);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          store_pk(im4B, NBS_64, trow, 32 * mt, Y3b[mt], h, NB_PL);
          store_pk(im3A, NBS_64, trow, 32 * mt, d3b[mt], h, NB_PL);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store_pk(im3B, NBS_128, trow, 32 * mt, Y2b[mt], h, NB_PL);
      }
      __syncthreads();
      if (wave < 2)
        bs4 += stage_mma_fr<NB_KST>(im4A, NBS_32, NB_PL, im4B, NBS_64, NB_PL, 0, wave, lane, acc4, 0, wave == 0 ? NB_KST : 0);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = wave + 4 * u;
        bs3[u] += stage_mma_fr<NB_KST>(im3A, NBS_64, NB_PL, im3B, NBS_128, NB_PL, t / 4, t % 4, lane, acc3[u], 0,
                                       t % 4 == 0 ? NB_KST : 0);
      }
      __syncthreads();
    }
    // ---- dY2 = W3^T dY3 . relu'(Y2)
    Pk d2b[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x16 c = zero16();
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        c = mma(wrmT_acc_fr(W3 + opaque_zero(), NS3, 32 * mt, kk, lane, LO), pk_fr<kk & 1>(d3b[kk >> 1]), c);
      });
      d2b[mt] = to_pk(c);
      mask_pk(d2b[mt], Y2b[mt]);
    }
    // ---- dY1 = W2^T dY2 . relu'(Y1)
    Pk d1b[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 c = zero16();
      static_for<8>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        c = mma(wrmT_acc_fr(W2 + opaque_zero(), NS2, 32 * mt, kk, lane, LO), pk_fr<kk & 1>(d2b[kk >> 1]), c);
      });
      d1b[mt] = to_pk(c);
      mask_pk(d1b[mt], Y1b[mt]);
    }
#pragma unroll 1
    for (int turn = 0; turn < nturn; ++turn) {   // S2: dWn2 (128x64) += dY2 . Y1^T ; nb2
      h16* imA = stg;
      h16* imB = stg + NB_RT * NBS_128;
      if (NB_NT == 1 || myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store_pk(imA, NBS_128, trow, 32 * mt, d2b[mt], h, NB_PL);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk(imB, NBS_64, trow, 32 * mt, Y1b[mt], h, NB_PL);
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = wave + 4 * u;
        bs2[u] += stage_mma_fr<NB_KST>(imA, NBS_128, NB_PL, imB, NBS_64, NB_PL, t / 2, t % 2, lane, acc2[u], 0,
                                       t % 2 == 0 ? NB_KST : 0);
      }
      __syncthreads();
    }
    // ---- dP = W1f^T dY1 : rows 0..127 pooled grads -> global; rows 128..131 state grads
#pragma unroll
    for (int mt = 0; mt < 5; ++mt) {
      f32x16 c = zero16();
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        c = mma(wrmT_acc_fr(W1 + opaque_zero(), NS1, 32 * mt, kk, lane, LO), pk_fr<kk & 1>(d1b[kk >> 1]), c);
      });
      if (mt < 4) {
        if (ok) {
          h16* drow = a.dP + (long)b * a.dp_env + (long)i * PROW + 32 * mt;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            h16x4 v, vl_;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = (h16)c[4 * g + e];
              if constexpr (X3) vl_[e] = (h16)(c[4 * g + e] - (float)v[e]);
            }
            *reinterpret_cast<h16x4*>(drow + 8 * g + 4 * h) = v;
            if constexpr (X3) *reinterpret_cast<h16x4*>(drow + 128 + 8 * g + 4 * h) = vl_;
          }
        }
      } else {
        float er[8];
        acc_rows8(c, er);                       // rows 128..128+2D-1: d/d[p - g, v]
        if (ok && h == 0 && a.ego) {
#pragma unroll
          for (int q = 0; q < D; ++q) { egp[q] += er[q]; egv[q] += er[D + q]; }
          store_rec<D>(a.ego + (long)b * N * REC<D>, (unsigned)i, egp, egv);
        }
      }
    }
#pragma unroll 1
    for (int turn = 0; turn < nturn; ++turn) {   // S1: dWn1f (64x160) += dY1 . P^T (P re-read: L2-hot)
      h16* imA = stg;
      h16* imB = stg + NB_RT * NBS_64;
      if (NB_NT == 1 || myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk(imA, NBS_64, trow, 32 * mt, d1b[mt], h, NB_PL);
        const h16* prow = a.pooled + (long)b * a.p_env + (long)i * PROW;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const h16x8 pv = ok ? *reinterpret_cast<const h16x8*>(prow + 16 * kk + 8 * h) : zz;
          *reinterpret_cast<h16x8*>(imB + trow * NBS_P + 16 * kk + 8 * h) = pv;
          if constexpr (X3) {
            const h16x8 pl = ok ? *reinterpret_cast<const h16x8*>(prow + 128 + 16 * kk + 8 * h) : zz;
            *reinterpret_cast<h16x8*>(imB + NB_PL + trow * NBS_P + 16 * kk + 8 * h) = pl;
          }
        }
        *reinterpret_cast<h16x8*>(imB + trow * NBS_P + 128 + 8 * h) = sfr;
        *reinterpret_cast<h16x8*>(imB + trow * NBS_P + 144 + 8 * h) = zz;
        if constexpr (X3) {      // the state fragment is exact: zero lo plane
          *reinterpret_cast<h16x8*>(imB + NB_PL + trow * NBS_P + 128 + 8 * h) = zz;
          *reinterpret_cast<h16x8*>(imB + NB_PL + trow * NBS_P + 144 + 8 * h) = zz;
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int t = wave + 4 * u;
        if (u < n1) stage_mma_fr<NB_KST>(imA, NBS_64, NB_PL, imB, NBS_P, NB_PL, t / 5, t % 5, lane, acc1[u]);
      }
      __syncthreads();
    }
  }
  // ---- slab += this workgroup's partial (fixed WG -> slab map: deterministic)
  // all slab loads first (see load_tile), then the adds and stores; the first BPTT step writes
  // the slab (no zero-fill pass, no loads)
  f32x16 o1[3], o2[2], o3[2], o4 = zero16();
  float ob2[2] = {0.f, 0.f}, ob3[2] = {0.f, 0.f}, ob4 = 0.f;
  o1[0] = o1[1] = o1[2] = o2[0] = o2[1] = o3[0] = o3[1] = zero16();
  if (!a.init) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int t = wave + 4 * u;
      if (u < n1) load_tile(o1[u], P + NP_W1, 160, t / 5, t % 5, lane);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 4 * u;
      load_tile(o2[u], P + NP_W2, 64, t / 2, t % 2, lane);
      load_tile(o3[u], P + NP_W3, 128, t / 4, t % 4, lane);
      ob2[u] = P[NP_B2 + 32 * (t / 2) + r];
      ob3[u] = P[NP_B3 + 32 * (t / 4) + r];
    }
    if (wave < 2) {
      load_tile(o4, P + NP_W4, 64, 0, wave, lane);
      ob4 = P[NP_B4 + r];
    }
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int t = wave + 4 * u;
    if (u < n1) store_tile_add(P + NP_W1, 160, t / 5, t % 5, o1[u], acc1[u], lane);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t2 = wave + 4 * u;
    store_tile_add(P + NP_W2, 64, t2 / 2, t2 % 2, o2[u], acc2[u], lane);
    const float s2 = bs2[u] + shfl_xor32(bs2[u]);
    if (t2 % 2 == 0 && h == 0) P[NP_B2 + 32 * (t2 / 2) + r] = ob2[u] + s2;
    const int t3 = wave + 4 * u;
    store_tile_add(P + NP_W3, 128, t3 / 4, t3 % 4, o3[u], acc3[u], lane);
    const float s3 = bs3[u] + shfl_xor32(bs3[u]);
    if (t3 % 4 == 0 && h == 0) P[NP_B3 + 32 * (t3 / 4) + r] = ob3[u] + s3;
  }
  if (wave < 2) {
    store_tile_add(P + NP_W4, 64, 0, wave, o4, acc4, lane);
    if (wave == 0) {
      const float s4 = bs4 + shfl_xor32(bs4);
      if (h == 0) P[NP_B4 + r] = ob4 + s4;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Cooperative node backward for 32-agent chunks (strong-scaling slices and small scenes, where
// a workgroup holds one 32-agent chunk): in node_bwd_body one wave would run the whole
// forward-recompute / backward MFMA chain of its 32 agents while three idle. Here the four waves
// split every layer's 32-row output tiles and meet in LDS between layers: a layer's tiles are
// stored agent-major into the stage region (natural feature order), read back by every wave as
// natural-k B fragments (the weights as natural-k A fragments, wrm_nat / wrmT_nat), and the same
// images are the operands of the weight-gradient contractions (one turn: 32 rows). Critical path
// per chunk: about a quarter of the MFMA chain plus ~10 workgroup barriers. Same slab layout and
// outputs (dP, ego, fused combine) as node_bwd_body; only the summation order of the weight
// gradients differs (per tile owner instead of per turn).
//   layer tiles -> waves: L1 {0,1} | L2 {0..3} | L3 {2,3} | L4 {0} (+ gain law, combine, ego) |
//   dY3 {1,2} | dY2 {0..3} | dY1 {0,1} | dP {0..3} + the state tile on wave 0
//   region columns (NC_SW per row, 32 rows, lo plane at NB_PL):
//     [Y1 0..63]  -> [Y2 0..127] -> + [Y3 128..191] + [d4 192..223] + [d3 224..287]  (S4, S3)
//     -> [d2 0..127 | Y1 128..191] (S2) -> [d1 0..63 | P, s 64..223] (S1)
constexpr int NC_SW = 296;                           // 148 dwords: row reads spread over the banks
static_assert(NC_SW * 32 <= NB_PL, "cooperative region must fit the stage plane");

template <int D>
DEV void node_bwd_coop(const CtrlNodeBwdArgs& a, unsigned char* smem, long c0, long cstride, float* P) {
  constexpr int RM = (X3 ? 2 : 1) * NODE_RM_ELEMS;
  constexpr int SW = NC_SW, PLN = NB_PL;
  h16* wr = reinterpret_cast<h16*>(smem);
  float* vl = reinterpret_cast<float*>(smem + RM * 2);
  h16* stg = reinterpret_cast<h16*>(smem + RM * 2 + CTRL_VEC * 4);
  block_copy16(wr, a.wrm, RM * 2);
  if (MB_STAMPS && a.stamps && (threadIdx.x & 63) == 0)
    a.stamps[((long)blockIdx.x * NB_WAVES + threadIdx.x / WAVE) * 16] = __builtin_amdgcn_s_memtime();
  block_copy16(vl, a.wvec, CTRL_VEC * 4);
  __syncthreads();
  const float* nb2 = vl + 128;
  const float* nb3 = vl + 256;
  const float* nb4 = vl + 320;
  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int N = a.N;
  const int total = a.B * N;
  const long nchunks = (total + 31) / 32;
  constexpr int LO = NODE_RM_LO;
  const h16x8 zz = zero_h8();
  // diagnostics: shader clock at the phase boundaries (a.stamps, normally null; a workgroup with
  // several chunks keeps its last chunk's clocks, slot 15 = that chunk's start)
  auto stamp = [&](int k) {
    if (MB_STAMPS && a.stamps) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) a.stamps[((long)blockIdx.x * NB_WAVES + wave) * 16 + k] = t;
    }
  };
  stamp(1);                                            // weights staged
  // owned weight-gradient tiles: S4 (dW4pad 1x2) wave < 2 nt = wave; S3 (2x4) t = wave + 4u;
  // S2 (4x2) t = wave + 4u; S1 (2x5) t = wave + 4u (u < 3, t < 10)
  f32x16 acc4 = zero16(), acc3[2], acc2[2], acc1[3];
  float bs4 = 0.f, bs3[2] = {0.f, 0.f}, bs2[2] = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u) { acc3[u] = zero16(); acc2[u] = zero16(); }
#pragma unroll
  for (int u = 0; u < 3; ++u) acc1[u] = zero16();
  const int n1 = (wave < 2) ? 3 : 2;
  // B fragment (natural k) of image columns c0 + 16kk.. for this lane's agent row
  auto img_fr = [&](int col0, int kk) { return row_fr(stg + r * SW + col0 + 16 * kk + 8 * h, PLN); };
  // the slab's old values (read-modify-write at the end), loaded by slab_loads()
  f32x16 o1[3], o2[2], o3[2], o4 = zero16();
  float ob2[2] = {0.f, 0.f}, ob3[2] = {0.f, 0.f}, ob4 = 0.f;
  o1[0] = o1[1] = o1[2] = o2[0] = o2[1] = o3[0] = o3[1] = zero16();
  bool loaded = false;
  auto slab_loads = [&]() {
    loaded = true;
    if (a.init) return;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int t = wave + 4 * u;
      if (u < n1) load_tile(o1[u], P + NP_W1, 160, t / 5, t % 5, lane);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 4 * u;
      load_tile(o2[u], P + NP_W2, 64, t / 2, t % 2, lane);
      load_tile(o3[u], P + NP_W3, 128, t / 4, t % 4, lane);
      ob2[u] = P[NP_B2 + 32 * (t / 2) + r];
      ob3[u] = P[NP_B3 + 32 * (t / 4) + r];
    }
    if (wave < 2) {
      load_tile(o4, P + NP_W4, 64, 0, wave, lane);
      ob4 = P[NP_B4 + r];
    }
  };

  for (long chunk = c0; chunk < nchunks; chunk += cstride) {
    stamp(15);
    const int ga = (int)(chunk * 32) + r;
    const bool ok = ga < total;
    int b = 0, i = 0;
    float sp[D], sv[D], gg[D], av[D], gnp[D], gnv[D];
#pragma unroll
    for (int q = 0; q < D; ++q) { sp[q] = sv[q] = gg[q] = av[q] = gnp[q] = gnv[q] = 0.f; }
    bool vld = false;
    if (ok) {
      b = ga / N; i = ga - b * N;
      load_rec<D>(a.S + (long)b * a.s_env * REC<D>, (unsigned)i, sp, sv);
#pragma unroll
      for (int q = 0; q < D; ++q) gg[q] = a.G[((long)b * N + i) * D + q];
      if (wave == 0) {
#pragma unroll
        for (int q = 0; q < D; ++q) av[q] = a.A[((long)b * a.a_env + i) * D + q];
        if (a.Gn && !a.cdS) load_rec<D>(a.Gn + (long)b * a.gn_env * REC<D>, (unsigned)i, gnp, gnv);
        vld = a.valid ? (a.valid[(long)b * a.v_env] != 0) : true;
      }
    }
    if (wave == 0 && a.cdS) fused_combine<D>(a, ok, b, i, h, gnp, gnv);    // G_{t+1} (wave 0 only)
    float ex[D];
#pragma unroll
    for (int q = 0; q < D; ++q) ex[q] = sp[q] - gg[q];
    stamp(2);
    const h16x8 sfr = node_state_frag<D>(ex, sv, ok, h);
    const h16* prow = a.pooled + (long)b * a.p_env + (long)i * PROW;
    const h16* W1 = wr + opaque_zero();
    const h16* W2 = W1 + 64 * NS1;
    const h16* W3 = W2 + 128 * NS2;
    const h16* W4 = W3 + 64 * NS3;
    Pk Y1b, Y2b, Y3b;
    // the rollout's activations of this step (a.acts): Y1 / Y2 / Y3 tiles and y4 loaded instead of
    // the L1..L4 recompute; the stage images end up as after L3 (Y2 cols 0..127, Y3 128..191)
    const unsigned char* abase = a.acts ? a.acts + ((long)b * a.na_env + i) * NODE_ACT_BYTES : nullptr;
    if (a.acts) {
      const Pk zp = {zero_h16x16(), zero_h16x16()};
      if (wave < 2) Y1b = ok ? act_load_pk(abase, wave, h) : zp;
      Y2b = ok ? act_load_pk(abase, 2 + wave, h) : zp;
      if (wave >= 2) Y3b = ok ? act_load_pk(abase, 6 + wave - 2, h) : zp;
      store_pk(stg, SW, r, 32 * wave, Y2b, h, PLN);
      if (wave >= 2) store_pk(stg, SW, r, 128 + 32 * (wave - 2), Y3b, h, PLN);
      __syncthreads();
      stamp(3);
      stamp(4);
    } else {
    // ---- L1 (waves 0, 1): Y1 tile `wave` = relu(W1f [P; s])
    if (wave < 2) {
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        Fr pf;
        if (ok) pf = row_fr(prow + 16 * kk + 8 * h, 128);
        else pf.h = pf.l = zz;
        c = mma(wrm_nat_fr(W1, NS1, 32 * wave, kk, lane, LO), pf, c);
      }
      c = mma_bx(wrm_nat_fr(W1, NS1, 32 * wave, 8, lane, LO), sfr, c);
      relu_(c);
      Y1b = to_pk(c);
      store_pk(stg, SW, r, 32 * wave, Y1b, h, PLN);
    }
    __syncthreads();
    stamp(3);
    // ---- L2 (all waves): Y2 tile `wave`
    {
      f32x16 c = bias_rows(nb2, 32 * wave, h);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) c = mma(wrm_nat_fr(W2, NS2, 32 * wave, kk, lane, LO), img_fr(0, kk), c);
      relu_(c);
      Y2b = to_pk(c);
    }
    __syncthreads();                                   // Y1 image read by every wave
    store_pk(stg, SW, r, 32 * wave, Y2b, h, PLN);
    __syncthreads();
    stamp(4);
    // ---- L3 (waves 2, 3): Y3 tile wave - 2
    if (wave >= 2) {
      const int mt = wave - 2;
      f32x16 c = bias_rows(nb3, 32 * mt, h);
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) c = mma(wrm_nat_fr(W3, NS3, 32 * mt, kk, lane, LO), img_fr(0, kk), c);
      relu_(c);
      Y3b = to_pk(c);
      store_pk(stg, SW, r, 128 + 32 * mt, Y3b, h, PLN);
    }
    __syncthreads();
    }
    stamp(5);
    // ---- L4 + gain law + action-loss backward (wave 0) -> d4, ego terms
    float egp[D], egv[D];
#pragma unroll
    for (int q = 0; q < D; ++q) { egp[q] = 0.f; egv[q] = 0.f; }
    if (wave == 0) {
      f32x16 y4;
      if (a.acts) {
        y4 = ok ? *reinterpret_cast<const f32x16*>(abase + 16 * NODE_ACT_PKB + 64 * h) : zero16();
      } else {
        y4 = bias_rows(nb4, 0, h);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) y4 = mma(wrm_nat_fr(W4, NS4, 0, kk, lane, LO), img_fr(128, kk), y4);
      }
      float y4r[8];
      acc_rows8(y4, y4r);
      float d4r[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) d4r[q] = 0.f;
      if (ok && h == 0) {
        float da[D], ar[D];
#pragma unroll
        for (int q = 0; q < D; ++q) { da[q] = a.dt * gnv[q]; ar[q] = -(ex[q] + a.sqrt3 * sv[q]); }
        float act_coef = a.act_scale ? a.act_coef / fmaxf(*a.act_scale, 1.f) : a.act_coef;
        if (a.gscale) act_coef *= *a.gscale;
        if (vld && act_coef != 0.f) {
          const float diff = sqsum<D>(av) - sqsum<D>(ar);
          const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
          const float cf = act_coef * sg;
#pragma unroll
          for (int q = 0; q < D; ++q) {
            da[q] += cf * 2.f * av[q];
            egp[q] += cf * 2.f * ar[q];
            egv[q] += cf * 2.f * a.sqrt3 * ar[q];
          }
        }
#pragma unroll
        for (int q = 0; q < D; ++q) {
          const float s0 = sigm(y4r[2 * q]), s1 = sigm(y4r[2 * q + 1]);
          const float kp = 2.f * s0 + 0.2f, kv = 2.f * s1 + 0.2f;
          egp[q] += -kp * da[q];
          egv[q] += -kv * da[q];
          d4r[2 * q] = -da[q] * ex[q] * 2.f * s0 * (1.f - s0);
          d4r[2 * q + 1] = -da[q] * sv[q] * 2.f * s1 * (1.f - s1);
        }
      }
      f32x16 d4 = zero16();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float hi4 = shfl_xor32(d4r[4 + q]);
        d4[q] = (h == 0) ? d4r[q] : hi4;
      }
      store_pk(stg, SW, r, 192, to_pk(d4), h, PLN);
    }
    __syncthreads();
    stamp(6);
    // ---- dY3 (waves 1, 2): tile wave - 1 = (W4^T d4) . relu'(Y3)
    if (wave == 1 || wave == 2) {
      const int mt = wave - 1;
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) c = mma(wrmT_nat_fr(W4, NS4, 32 * mt, kk, lane, LO), img_fr(192, kk), c);
      Pk d3b = to_pk(c);
      Pk y3;
      y3.h = load_tile_h(stg, SW, r, 128 + 32 * mt, h);
      mask_pk(d3b, y3);
      store_pk(stg, SW, r, 224 + 32 * mt, d3b, h, PLN);
    }
    __syncthreads();
    stamp(7);
    // ---- S4: dW4pad (32x64) += d4 . Y3^T ; nb4  (waves 0, 1)   S3: dW3 (64x128) += d3 . Y2^T ; nb3
    if (wave < 2)
      bs4 += stage_mma_fr<2>(stg + 192, SW, PLN, stg + 128, SW, PLN, 0, wave, lane, acc4, 0, wave == 0 ? 2 : 0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 4 * u;
      bs3[u] += stage_mma_fr<2>(stg + 224, SW, PLN, stg, SW, PLN, t / 4, t % 4, lane, acc3[u], 0, t % 4 == 0 ? 2 : 0);
    }
    // ---- dY2 (all waves): tile `wave` = (W3^T d3) . relu'(Y2)
    Pk d2b;
    {
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) c = mma(wrmT_nat_fr(W3, NS3, 32 * wave, kk, lane, LO), img_fr(224, kk), c);
      d2b = to_pk(c);
      mask_pk(d2b, Y2b);
    }
    __syncthreads();                                   // S4 / S3 images and d3 read by every wave
    store_pk(stg, SW, r, 32 * wave, d2b, h, PLN);
    if (wave < 2) store_pk(stg, SW, r, 128 + 32 * wave, Y1b, h, PLN);
    __syncthreads();
    stamp(8);
    // ---- S2: dW2 (128x64) += d2 . Y1^T ; nb2
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 4 * u;
      bs2[u] += stage_mma_fr<2>(stg, SW, PLN, stg + 128, SW, PLN, t / 2, t % 2, lane, acc2[u], 0, t % 2 == 0 ? 2 : 0);
    }
    // ---- dY1 (waves 0, 1): tile `wave` = (W2^T d2) . relu'(Y1)
    Pk d1b;
    if (wave < 2) {
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) c = mma(wrmT_nat_fr(W2, NS2, 32 * wave, kk, lane, LO), img_fr(0, kk), c);
      d1b = to_pk(c);
      mask_pk(d1b, Y1b);
    }
    __syncthreads();                                   // S2 images and d2 read by every wave
    stamp(9);
    // (requesting the slab's old values here, in the workgroup's last chunk, to hide their latency
    // behind S1 and the dP tiles: 8-env slice 3.40 vs 2.80 ms -- the 128 held registers spill; r6c)
    // ---- S1 images: d1 (cols 0..63), [P | s | 0] (cols 64..223: pooled 128, state fragment 16, zeros 16)
    if (wave < 2) store_pk(stg, SW, r, 32 * wave, d1b, h, PLN);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kk = 2 * wave + u;
      const h16x8 pv = ok ? *reinterpret_cast<const h16x8*>(prow + 16 * kk + 8 * h) : zz;
      *reinterpret_cast<h16x8*>(stg + r * SW + 64 + 16 * kk + 8 * h) = pv;
      if constexpr (X3) {
        const h16x8 pl = ok ? *reinterpret_cast<const h16x8*>(prow + 128 + 16 * kk + 8 * h) : zz;
        *reinterpret_cast<h16x8*>(stg + PLN + r * SW + 64 + 16 * kk + 8 * h) = pl;
      }
    }
    if (wave == 3) {
      *reinterpret_cast<h16x8*>(stg + r * SW + 64 + 128 + 8 * h) = sfr;
      *reinterpret_cast<h16x8*>(stg + r * SW + 64 + 144 + 8 * h) = zz;
      if constexpr (X3) {      // the state fragment is exact: zero lo plane
        *reinterpret_cast<h16x8*>(stg + PLN + r * SW + 64 + 128 + 8 * h) = zz;
        *reinterpret_cast<h16x8*>(stg + PLN + r * SW + 64 + 144 + 8 * h) = zz;
      }
    }
    __syncthreads();
    stamp(10);
    // ---- S1: dW1f (64x160) += d1 . [P | s]^T
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int t = wave + 4 * u;
      if (u < n1) stage_mma_fr<2>(stg, SW, PLN, stg + 64, SW, PLN, t / 5, t % 5, lane, acc1[u]);
    }
    stamp(11);
    // ---- dP = W1f^T d1: tiles 0..3 (one per wave) -> dL/dpooled rows; tile 4 (wave 0) -> ego
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int mt = u == 0 ? wave : 4;
      if (u == 1 && wave != 0) break;
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) c = mma(wrmT_nat_fr(W1, NS1, 32 * mt, kk, lane, LO), img_fr(0, kk), c);
      if (mt < 4) {
        if (ok) {
          h16* drow = a.dP + (long)b * a.dp_env + (long)i * PROW + 32 * mt;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            h16x4 v, vl_;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = (h16)c[4 * g + e];
              if constexpr (X3) vl_[e] = (h16)(c[4 * g + e] - (float)v[e]);
            }
            *reinterpret_cast<h16x4*>(drow + 8 * g + 4 * h) = v;
            if constexpr (X3) *reinterpret_cast<h16x4*>(drow + 128 + 8 * g + 4 * h) = vl_;
          }
        }
      } else {
        float er[8];
        acc_rows8(c, er);                       // rows 128..128+2D-1: d/d[p - g, v]
        if (ok && h == 0 && a.ego) {
#pragma unroll
          for (int q = 0; q < D; ++q) { egp[q] += er[q]; egv[q] += er[D + q]; }
          store_rec<D>(a.ego + (long)b * N * REC<D>, (unsigned)i, egp, egv);
        }
      }
    }
    __syncthreads();                                   // region reused by the next chunk
    stamp(12);
  }
  stamp(13);
  // ---- slab += this workgroup's partial (fixed tile owners: deterministic); loads first
  if (!loaded) slab_loads();
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int t = wave + 4 * u;
    if (u < n1) store_tile_add(P + NP_W1, 160, t / 5, t % 5, o1[u], acc1[u], lane);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = wave + 4 * u;
    store_tile_add(P + NP_W2, 64, t / 2, t % 2, o2[u], acc2[u], lane);
    const float s2 = bs2[u] + shfl_xor32(bs2[u]);
    if (t % 2 == 0 && h == 0) P[NP_B2 + 32 * (t / 2) + r] = ob2[u] + s2;
    store_tile_add(P + NP_W3, 128, t / 4, t % 4, o3[u], acc3[u], lane);
    const float s3 = bs3[u] + shfl_xor32(bs3[u]);
    if (t % 4 == 0 && h == 0) P[NP_B3 + 32 * (t / 4) + r] = ob3[u] + s3;
  }
  if (wave < 2) {
    store_tile_add(P + NP_W4, 64, 0, wave, o4, acc4, lane);
    if (wave == 0) {
      const float s4 = bs4 + shfl_xor32(bs4);
      if (h == 0) P[NP_B4 + r] = ob4 + s4;
    }
  }
  if (MB_STAMPS && a.stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(14);                                           // slab stores complete
}

template <int D>
__global__ __launch_bounds__(NB_WAVES * 64, 1) void ctrl_node_bwd_kernel(CtrlNodeBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  node_bwd_body<D>(a, smem, blockIdx.x, gridDim.x, a.partial + (long)blockIdx.x * CTRL_NODE_PARTIAL);
}

// separate kernel: one shared body would size both paths' registers for the larger (spills)
template <int D>
__global__ __launch_bounds__(NB_WAVES * 64, 1) void ctrl_node_bwd_coop_kernel(CtrlNodeBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  node_bwd_coop<D>(a, smem, blockIdx.x, gridDim.x, a.partial + (long)blockIdx.x * CTRL_NODE_PARTIAL);
}

// ---------------------------------------------------------------------------------------
// EB_WAVES waves share a chunk of 32*EB_WAVES agents; each stage contracts the 32*EB_WAVES edges
// of one tile round (8 waves: 256 edges per barrier pair, one dW2 tile per wave; 4 waves: 128
// edges, two tiles per wave, two workgroups per CU)
constexpr int CTRL_EB_WAVES = 4;
constexpr int EB_WAVES = CTRL_EB_WAVES;
constexpr int EB_CH = EB_WAVES * 32;     // agents per chunk (each round: EB_CH edges)
constexpr int EB_TA = 8 / EB_WAVES;      // owned dW2 tiles per wave
// dense edge rows: K tiles per 32-agent wave (12 at K = 12) instead of 16 tiles of 2 agents x 16
// slots (a quarter of them padding rows at K = 12)
constexpr int CTRL_EB_DENSE = 1;
constexpr bool EB_DENSE = CTRL_EB_DENSE;
constexpr int EP_W2 = 0, EP_B2 = 8192, EP_W1 = 8320;
constexpr int CTRL_EDGE_PARTIAL = 10368;
constexpr int EB_PL = (128 + 64) * EB_CH;             // elements per stage plane (x3: lo plane at +EB_PL)
constexpr size_t EB_STAGE = (size_t)(X3 ? 2 : 1) * EB_PL * 2;

size_t ctrl_edge_bwd_lds() { return (size_t)22 * FRAG_SZ + EB_STAGE; }

// Edge backward over the work items w0, w0 + wstride, ... of `a` (smem: the kernel's dynamic
// LDS; P: this workgroup's slab row)
// KC: compile-time neighbour count (12 = TOP_K: the slot / agent / row index arithmetic of the
// dense rows folds to constants), 0 = runtime a.K
// SPLIT (the persistent small-scene BPTT): a work item is ONE 32-agent group whose K edge tiles
// are spread over the waves (wave w: tiles w, w + EB_WAVES, ...; a round's shared dW2 stage
// contracts the EB_WAVES tiles of the round) instead of one 32-agent group per wave -- a
// 32-agent env keeps all four waves busy. Waves without a tile in the last round (K not a
// multiple of EB_WAVES) contribute zero rows.
template <int D, int KC = 0, bool SPLIT = false>
DEV void edge_bwd_body(const CtrlEdgeBwdArgs& a, unsigned char* smem, long w0, long wstride, float* P) {
  h16* wf = reinterpret_cast<h16*>(smem);                 // ew1f (2) | ew2tn (16) | ew1ft (4)
  h16* stg = reinterpret_cast<h16*>(smem + 22 * FRAG_SZ);
  block_copy16(wf, a.wpack + (size_t)a.f_ew1f * FRAG_ELEMS, 2 * FRAG_SZ, false);
  block_copy16(wf + 2 * FRAG_ELEMS, a.wpack + (size_t)a.f_ew2tn * FRAG_ELEMS, 20 * FRAG_SZ);
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int N = a.N, K = KC ? KC : a.K;
  const int total = a.B * N;
  const long nchunks = SPLIT ? (total + 31) / 32 : (total + EB_CH - 1) / EB_CH;
  const int erow = wave * 32 + r;
  f32x16 accW2[EB_TA], accW1[2];
  accW1[0] = accW1[1] = zero16();
  float bs[EB_TA];
#pragma unroll
  for (int u = 0; u < EB_TA; ++u) { accW2[u] = zero16(); bs[u] = 0.f; }
  const h16 z = (h16)0.f;

  // work item = (chunk, tile range): small scenes split a chunk's NT tile rounds over
  // qsplit workgroups (tiles are independent; every workgroup owns its dW slab), large ones
  // use qsplit = 1
  const int QP = (!SPLIT && a.qsplit > 1) ? a.qsplit : 1;
  const long nwork = nchunks * QP;
  const int NT = EB_DENSE ? K : 16;                         // tiles per 32-agent wave
  const unsigned invK = (65536u + (unsigned)K - 1u) / (unsigned)K;
  auto idx_load = [&](const AgentBase& ab_, int q, EdgeIdx& o) {
    if constexpr (EB_DENSE) ctrl_idx_load_dense(a.idx, a.i_env, N, K, invK, ab_, q, r, total, o);
    else ctrl_idx_load(a.idx, a.i_env, N, K, ab_, q, r, total, o);
  };
  for (long w = w0; w < nwork; w += wstride) {
    const long chunk = w / QP;
    const int part = (int)(w - chunk * QP);
    // tiles of this wave: q0, q0 + QS, ... (< q1); every wave runs NR rounds (stage barriers)
    const int QS = SPLIT ? EB_WAVES : 1;
    const int q0 = SPLIT ? wave : part * NT / QP, q1 = SPLIT ? NT : (part + 1) * NT / QP;
    const int NR = SPLIT ? (NT + EB_WAVES - 1) / EB_WAVES : q1 - q0;
    EdgeIdx xi1;
    EdgeSt<D> xs0;
    const int g0 = SPLIT ? (int)(chunk * 32) : (int)(chunk * EB_CH) + wave * 32;
    const AgentBase ab = agent_base(g0, N);
    {
      EdgeIdx xi0;
      idx_load(ab, q0, xi0);
      ctrl_st_load<D>(a.S, a.s_env, xi0, xs0);
      idx_load(ab, q0 + QS, xi1);
    }
    // argmax slots / dL/dpooled of a tile's agents (lane (r, h): features 4r..4r+3 of one
    // agent per pass), loaded one tile ahead like the edge gathers. 16-slot rows: tile q = agents
    // 2q + h, one pass; dense rows: tile q holds agents af(q) .. (32q + 31) / K, pass p = agents
    // af + 2p + h (lane half h), two passes prefetched (all of a tile's agents for K >= 11)
    auto pool_load_ag = [&](int al, unsigned& am4, h16x4& dp4, h16x4& dl4) {
      const int ag = g0 + al;
      am4 = 0xFFFFFFFFu;
      if (al < 32 && ag < total) {
        int bb, ii;
        agent_bi(ab, al, N, bb, ii);
        am4 = *reinterpret_cast<const unsigned*>(a.argmax + bb * (int)a.am_env + ii * 128 + 4 * r);
        const h16* dpr = a.dP + bb * (int)a.dp_env + ii * PROW + 4 * r;
        dp4 = *reinterpret_cast<const h16x4*>(dpr);
        if constexpr (X3) dl4 = *reinterpret_cast<const h16x4*>(dpr + 128);
      }
    };
    constexpr int NPF = EB_DENSE ? 2 : 1;                 // prefetched agent passes per tile
    auto pass_agent = [&](int q, int p) {
      if constexpr (EB_DENSE) {
        const int af = dense_agent(32 * q, invK);
        const int al = af + 2 * p + h;
        return (q < NT && al * K < 32 * q + 32) ? al : 32;      // 32: no agent
      } else {
        return q < NT ? 2 * q + h : 32;
      }
    };
    auto pool_load = [&](int q, unsigned (&am4)[NPF], h16x4 (&dp4)[NPF], h16x4 (&dl4)[NPF]) {
#pragma unroll
      for (int p = 0; p < NPF; ++p) pool_load_ag(pass_agent(q, p), am4[p], dp4[p], dl4[p]);
    };
    unsigned am_n[NPF];
    h16x4 dp_n[NPF], dl_n[NPF];
    pool_load(q0, am_n, dp_n, dl_n);
    for (int rd = 0; rd < NR; ++rd) {
      const int q = q0 + rd * QS;               // SPLIT: q >= NT in a wave's empty last round
      const EdgeSt<D> cur = xs0;
      unsigned am4[NPF];
      h16x4 dp4[NPF], dl4[NPF];
#pragma unroll
      for (int p = 0; p < NPF; ++p) { am4[p] = am_n[p]; dp4[p] = dp_n[p]; dl4[p] = dl_n[p]; }
      ctrl_st_load<D>(a.S, a.s_env, xi1, xs0);
      idx_load(ab, q + 2 * QS, xi1);
      pool_load(q + QS, am_n, dp_n, dl_n);
      int slot, al;
      if constexpr (EB_DENSE) {
        const int e = 32 * q + r;
        al = dense_agent(e, invK);
        slot = e - al * K;
      } else {
        slot = r & 15;
        al = 2 * q + (r >> 4);
      }
      const bool ok = cur.ok;
      int b = 0, ib_;
      if (ok) agent_bi(ab, al, N, b, ib_);
      const int i = cur.i, j = cur.j;
      const float eye = (j == i) ? 1.f : 0.f;
      float rp[D], rv[D];
      edge_rel<D>(cur, rp, rv);
      const h16x8 F = ctrl_edge_frag<D>(rp, rv, eye, ok, h);
      const h16* wt = wf + opaque_zero();
      Pk H1b[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f32x16 c = mma_bx(frag_fr(wt, mt, lane), F, zero16());
        relu_(c);
        H1b[mt] = to_pk(c);
      }
      // max-pool backward as an LDS scatter into the S1 image (rows = this wave's 32 edges of the
      // tile): zero the rows, then lane (r, h) routes dP[f] of its pass agent, f = 4r..4r+3, to
      // the row of (agent, argmax slot) when that row lies in the tile. One coalesced argmax/dP
      // load per lane and pass instead of redundant row loads + compare/selects per edge lane.
      h16* imS = stg;                                           // S1 dZ image (128 wide, swizzled)
      {
        const u32x4 zero4 = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8) {   // whole rows are zeroed (unit permutation irrelevant); 8
          // consecutive lanes fill 128 contiguous bytes: conflict-free 16-byte stores
          *reinterpret_cast<u32x4*>(imS + wave * 32 * 128 + (c8 * 64 + lane) * 8) = zero4;
          if constexpr (X3) *reinterpret_cast<u32x4*>(imS + EB_PL + wave * 32 * 128 + (c8 * 64 + lane) * 8) = zero4;
        }
        // (am4 = all 0xFF: agent out of range)
        auto scatter = [&](int al, unsigned am, const h16x4& dp, const h16x4& dl) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const unsigned sl = (am >> (8 * jj)) & 0xFFu;
            if (sl < 16u) {
              const int row = EB_DENSE ? al * K + (int)sl - 32 * q : 16 * h + (int)sl;
              if (!EB_DENSE || (unsigned)row < 32u) {
                const int o = swz_off<128>(wave * 32 + row, 4 * r + jj);
                imS[o] = dp[jj];
                if constexpr (X3) imS[EB_PL + o] = dl[jj];
              }
            }
          }
        };
#pragma unroll
        for (int p = 0; p < NPF; ++p) scatter(pass_agent(q, p), am4[p], dp4[p], dl4[p]);
        if constexpr (EB_DENSE) {      // K <= 10: a tile spans more than 4 agents (not prefetched)
          for (int p = NPF; p < 16; ++p) {
            const int a0 = dense_agent(32 * q, invK) + 2 * p;      // the pass's first agent (uniform)
            if (a0 > 31 || a0 * K >= 32 * q + 32) break;
            const int al = pass_agent(q, p);
            unsigned am;
            h16x4 dp, dl;
            pool_load_ag(al, am, dp, dl);
            scatter(al, am, dp, dl);
          }
        }
        lds_wave_sync();
      }
      // dH1 = W2^T dZ (natural k) . relu'(H1)
      Pk d1b[2];
      if constexpr (X3) {      // k-outer: one split dZ fragment (8 VGPRs) live at a time
        f32x16 c[2] = {zero16(), zero16()};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const Fr dzk = row_fr(imS + swz_off<128>(erow, 16 * kk + 8 * h), EB_PL);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) c[mt] = mma(frag_fr(wt, 2 + mt * 8 + kk, lane), dzk, c[mt]);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          d1b[mt] = to_pk(c[mt]);
          mask_pk(d1b[mt], H1b[mt]);
        }
      } else {
        Fr dz[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) dz[kk] = row_fr(imS + swz_off<128>(erow, 16 * kk + 8 * h), EB_PL);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          f32x16 c = zero16();
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) c = mma(frag_fr(wt, 2 + mt * 8 + kk, lane), dz[kk], c);
          d1b[mt] = to_pk(c);
          mask_pk(d1b[mt], H1b[mt]);
        }
      }
      // dF = W1^T dH1 -> rows dx dy dvx dvy (lanes h == 0, regs 0..3)
      {
        f32x16 c = zero16();
        static_for<4>([&](auto kk_) {
          constexpr int kk = decltype(kk_)::value;
          c = mma(frag_fr(wt, 18 + kk, lane), pk_fr<kk & 1>(d1b[kk >> 1]), c);
        });
        float gr[8];
        acc_rows8(c, gr);                       // rows 0..2D-1 = dL/d(s_i - s_j)
        if (ok && h == 0 && a.dEc) {
          float gp[D], gv[D];
#pragma unroll
          for (int q2 = 0; q2 < D; ++q2) {
            gp[q2] = (j != i) ? gr[q2] : 0.f;
            gv[q2] = (j != i) ? gr[D + q2] : 0.f;
          }
          store_rec<D>(a.dEc, (unsigned)(b * (int)a.de_env + i * K + slot), gp, gv);
        }
      }
      // S1: dW2 (128x64) += dZ . H1^T ; eb2 (dZ is already in the image; bias-sum steps split
      //     between the two waves that read each row block)
      {
        h16* imA = stg;
        h16* imB = stg + EB_CH * 128;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk_sw<64>(imB, erow, 32 * mt, H1b[mt], h, EB_PL);
        __syncthreads();
        constexpr int KS = EB_CH / 16;
#pragma unroll
        for (int u = 0; u < EB_TA; ++u) {
          const int t = wave + EB_WAVES * u;
          bs[u] += stage_mma_sw_fr<KS, 128, 64>(imA, EB_PL, imB, EB_PL, t / 2, t % 2, lane, accW2[u],
                                                (KS / 2) * (wave & 1), (KS / 2) * (wave & 1) + KS / 2);
        }
        __syncthreads();
      }
      // S2: dW1f (64x32) += dH1 . F^T over this wave's own 32 edges -- wave-local, no barrier:
      //     the images live in the wave's own 32 rows of the dZ image (free after S1's closing
      //     barrier, rewritten by this wave's next scatter only), each wave accumulates both dW1
      //     tiles; the per-wave partials are summed in fixed order at the end
      {
        h16* imA = stg + wave * 32 * 128;          // dH1, 32 rows x 64 (swizzled)
        h16* imB = imA + 32 * 64;                  // [F | 0], 32 rows x 32 (swizzled)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk_sw<64>(imA, r, 32 * mt, d1b[mt], h, EB_PL);
        h16x8 zz;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) zz[jj] = z;
        *reinterpret_cast<h16x8*>(imB + swz_off<32>(r, 8 * h)) = F;
        *reinterpret_cast<h16x8*>(imB + swz_off<32>(r, 16 + 8 * h)) = zz;
        lds_wave_sync();
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) stage_mma_sw_fr<2, 64, 32, true>(imA, EB_PL, imB, 0, mt, 0, lane, accW1[mt]);
        lds_wave_sync();                           // reads done before the next scatter
      }
    }
  }
  __shared__ float ebred[EB_WAVES][EB_TA][32];
  // every slab load of the tail first (see load_tile): dW2 tiles, this thread's dW1 elements,
  // the eb2 element
  constexpr int NQ1 = 2 * 32 * 32 / (EB_WAVES * 64);
  f32x16 o2[EB_TA];
  float o1[NQ1];
  float ob2 = 0.f;
#pragma unroll
  for (int u = 0; u < EB_TA; ++u) o2[u] = zero16();
#pragma unroll
  for (int j = 0; j < NQ1; ++j) o1[j] = 0.f;
  if (!a.init) {      // the first BPTT step writes the slab (no zero-fill pass, no loads)
#pragma unroll
    for (int u = 0; u < EB_TA; ++u) {
      const int t = wave + EB_WAVES * u;
      load_tile(o2[u], P + EP_W2, 64, t / 2, t % 2, lane);
    }
#pragma unroll
    for (int j = 0; j < NQ1; ++j) o1[j] = P[EP_W1 + threadIdx.x + j * EB_WAVES * 64];
    if (threadIdx.x < 128) ob2 = P[EP_B2 + threadIdx.x];
  }
#pragma unroll
  for (int u = 0; u < EB_TA; ++u) {
    const int t = wave + EB_WAVES * u;
    store_tile_add(P + EP_W2, 64, t / 2, t % 2, o2[u], accW2[u], lane);
    const float s = bs[u] + shfl_xor32(bs[u]);
    if (h == 0) ebred[wave][u][r] = s;
  }
  // dW1: per-wave partials -> LDS (the stage region is free: every wave has left the loop) ->
  // fixed-order sum over the waves
  __syncthreads();
  float* w1red = reinterpret_cast<float*>(stg);    // [EB_WAVES][2][32 rows][32 cols]
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg)
      w1red[((wave * 2 + mt) * 32 + acc_row(reg, h)) * 32 + r] = accW1[mt][reg];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NQ1; ++j) {
    const int q = threadIdx.x + j * EB_WAVES * 64;
    float t = 0.f;
    for (int w = 0; w < EB_WAVES; ++w) t += w1red[w * 2048 + q];
    P[EP_W1 + q] = o1[j] + t;                     // rows 32mt + row, 32 cols: the slab layout
  }
  __syncthreads();
  // eb2 row block mt was summed half by the owner of tile 2mt and half by the owner of tile
  // 2mt+1 (waves w, w^1): add in fixed order
  if (threadIdx.x < 128) {
    const int mt = threadIdx.x >> 5, rr = threadIdx.x & 31;    // row block 0..3
    const int t0 = 2 * mt, t1 = 2 * mt + 1;
    P[EP_B2 + 32 * mt + rr] = ob2 + (ebred[t0 % EB_WAVES][t0 / EB_WAVES][rr] + ebred[t1 % EB_WAVES][t1 / EB_WAVES][rr]);
  }
}

template <int D, int KC = 0>
__global__ __launch_bounds__(EB_WAVES * 64, (EB_WAVES == 4 && !X3) ? 2 : 1) void ctrl_edge_bwd_kernel(CtrlEdgeBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  edge_bwd_body<D, KC>(a, smem, blockIdx.x, gridDim.x, a.partial + (long)blockIdx.x * CTRL_EDGE_PARTIAL);
}

static_assert(EB_WAVES == NB_WAVES, "the fused BPTT step runs both phases with one block shape");
template <int D, int KC>
__global__ __launch_bounds__(NB_WAVES * 64, 1) void ctrl_bwd_step_kernel(CtrlNodeBwdArgs na, CtrlEdgeBwdArgs ea) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  node_bwd_coop<D>(na, smem, blockIdx.x, gridDim.x, na.partial + (long)blockIdx.x * CTRL_NODE_PARTIAL);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's dP / ego stores complete
  __syncthreads();                                      // (and the node phase's LDS reads done)
  edge_bwd_body<D, KC, true>(ea, smem, blockIdx.x, gridDim.x, ea.partial + (long)blockIdx.x * CTRL_EDGE_PARTIAL);
}

// =======================================================================================
// Persistent small-scene rollout (envs of <= SMALL_MAXN graph nodes; reference train.py:58-81).
// The per-step kernels of a 32-agent env are single-workgroup launches whose latency, not work,
// sets the step time (~60 us per step as scan + controller launches). Here ONE launch runs the
// whole rollout: one workgroup per env loops over the steps,
//   small_scan: brute-force kNN by rank selection, TTC danger bits and counts, all-pairs safety;
//   controller edge phase over all waves (groups of apw agents), node phase (32-agent groups),
//   Euler step, per-env goal-distance sums -> the env's early-stop state.
// Early stop without a grid barrier: an env that becomes done publishes its step (max into
// ctl[1], then ctl[0] += 1). A workgroup keeps simulating its env (done envs are masked later,
// as on the launch-per-step path) until every env has published and it has scanned s_T,
// T = max published step + 1, or until it has scanned s_Tmax. No workgroup ever waits for
// another, so the launch terminates for any residency / order; steps a fast workgroup computes
// beyond T are never read. Outputs are those of the per-step path, bit for bit.
// =======================================================================================
constexpr int SR_WAVES = 8;
constexpr int SMALL_MAXN = 64;
// kNN candidates per work item (JG of small_scan): 8 amortise each key over more compares, 2
// spread a 32-agent env's 32 x 32 pairs over all 512 threads (8 leaves 3 of 4 waves idle: the
// rank loop was half of the config-#2 step, profiles/r6_runs/r6y/); the rollout takes 2 when the
// env's work items fit one pass of the workgroup, else 8
constexpr int SR_JG = 8, SR_JG_SMALL = 2;

struct SmallScanLds {
  float4 tp[SMALL_MAXN], tv[SMALL_MAXN];       // positions / velocities of s_t (z = 0 in 2-D)
  int nbr[SMALL_MAXN * 16];                    // the env's kNN slots
  int unsafe[SMALL_MAXN];
  float red[2][SR_WAVES];
  int dec;
};

template <int D>
DEV void rel_d2(const float4& a, const float4& c, float (&dp)[D]) {
  dp[0] = a.x - c.x;
  dp[1] = a.y - c.y;
  if constexpr (D == 3) dp[2] = a.z - c.z;
}

// kNN / danger / counts / safety of one env's s_t (Sb: the env's records) by the whole workgroup.
// Same keys, arithmetic and tie order as scan_kernel: (d2 bits, node id) ranks, so the lists are
// those of the all-pairs oracle; the safety test runs on every pair (no culling pre-test).
template <int D, int JG>
DEV void small_scan(const RolloutSmallArgs& ra, const float4* Sb, int N, int Nn, int K, bool knn, bool dng,
                    int* idx_out, uint8_t* dang_out, float* cnt_out, float* safe_out, SmallScanLds& L) {
  const int tid = threadIdx.x, wave = tid / WAVE, lane = tid & 63;
  constexpr int NTH = SR_WAVES * WAVE;
  for (int q = tid; q < Nn; q += NTH) {
    float p[D], v[D];
    load_rec<D>(Sb, (unsigned)q, p, v);
    L.tp[q] = make_float4(p[0], p[1], D == 3 ? p[D - 1] : 0.f, 0.f);
    L.tv[q] = make_float4(v[0], v[1], D == 3 ? v[D - 1] : 0.f, 0.f);
    L.unsafe[q] = 0;
  }
  __syncthreads();
  if (knn) {
    // slot of candidate j in agent i's list = #{j' : key(i, j') < key(i, j)}; keys are unique
    const int ng = (Nn + JG - 1) / JG;
    for (int w = tid; w < N * ng; w += NTH) {
      const int i = w / ng, j0 = (w - i * ng) * JG;
      const float4 me = L.tp[i];
      uint64_t key[JG];
      int rank[JG];
#pragma unroll
      for (int u = 0; u < JG; ++u) {
        float dp[D];
        rel_d2<D>(me, L.tp[min(j0 + u, Nn - 1)], dp);
        key[u] = j0 + u < Nn ? knn_key(sqsum<D>(dp), (unsigned)(j0 + u)) : ~0ull;
        rank[u] = 0;
      }
      for (int jp = 0; jp < Nn; ++jp) {
        float dp[D];
        rel_d2<D>(me, L.tp[jp], dp);
        const uint64_t kp = knn_key(sqsum<D>(dp), (unsigned)jp);
#pragma unroll
        for (int u = 0; u < JG; ++u) rank[u] += kp < key[u] ? 1 : 0;
      }
#pragma unroll
      for (int u = 0; u < JG; ++u)
        if (j0 + u < Nn && rank[u] < K) {
          L.nbr[i * K + rank[u]] = j0 + u;
          idx_out[i * K + rank[u]] = j0 + u;
        }
    }
    __syncthreads();
  }
  float nd = 0.f, ns = 0.f;
  if (dng) {
    for (int w = tid; w < N * K; w += NTH) {
      const int i = w / K, j = L.nbr[w];
      const float eye = (j == i) ? 1.f : 0.f;
      const float pi[3] = {L.tp[i].x, L.tp[i].y, L.tp[i].z}, pj[3] = {L.tp[j].x, L.tp[j].y, L.tp[j].z};
      const float vi[3] = {L.tv[i].x, L.tv[i].y, L.tv[i].z}, vj[3] = {L.tv[j].x, L.tv[j].y, L.tv[j].z};
      float dp[D], dv[D];
#pragma unroll
      for (int d = 0; d < D; ++d) { dp[d] = (pi[d] - pj[d]) + eye; dv[d] = vi[d] - vj[d]; }
      const bool dg = ttc_danger<D>(dp, dv, ra.r2_train, ra.ttc_train);
      dang_out[w] = dg ? 1 : 0;
      nd += dg ? 1.f : 0.f;
    }
  }
  if (safe_out) {
    for (int w = tid; w < N * Nn; w += NTH) {
      const int i = w / Nn, j = w - i * Nn;
      if (j == i || L.unsafe[i]) continue;     // (a racy skip: the flag only ever goes 0 -> 1)
      float dp[D], dv[D];
      rel_d2<D>(L.tp[i], L.tp[j], dp);
      rel_d2<D>(L.tv[i], L.tv[j], dv);
      if (ttc_danger<D>(dp, dv, ra.r2_check, ra.ttc_check)) atomicOr(&L.unsafe[i], 1);
    }
    __syncthreads();
    for (int q = tid; q < N; q += NTH) ns += L.unsafe[q] ? 0.f : 1.f;
  }
  nd = wave_sum(nd);
  ns = wave_sum(ns);
  if (lane == 0) { L.red[0][wave] = nd; L.red[1][wave] = ns; }
  __syncthreads();
  if (tid == 0) {
    float s0 = 0.f, s1 = 0.f;
    for (int q = 0; q < SR_WAVES; ++q) { s0 += L.red[0][q]; s1 += L.red[1][q]; }
    if (dng) { cnt_out[0] = s0; cnt_out[1] = (float)(N * K) - s0; }
    if (safe_out) safe_out[0] = s1;
  }
}

template <int D, bool ACTS>
__global__ __launch_bounds__(SR_WAVES * 64) void rollout_small_kernel(RolloutSmallArgs ra) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ SmallScanLds L;
  h16* wl = reinterpret_cast<h16*>(smem);                            // ew1f, ew2 (18 frags)
  h16* wn = wl + 18 * FRAG_ELEMS;                                     // nw1f..nw4 (54 frags)
  float* vl = reinterpret_cast<float*>(smem + (size_t)CTRL_FWD_FRAGS * FRAG_SZ);
  const CtrlArgs& c = ra.c;
  block_copy16(wl, c.wpack + (size_t)c.f_edge * FRAG_ELEMS, 18 * FRAG_SZ, false);
  block_copy16(wn, c.wpack + (size_t)c.f_node * FRAG_ELEMS, 54 * FRAG_SZ, false);
  block_copy16(vl, c.wvec, CTRL_VEC * 4);
  const int b = blockIdx.x, B = c.B, N = c.N, K = c.K, Nn = ra.Nn, Tmax = ra.Tmax;
  const long nk = (long)N * K;
  if (ra.s0) {
    // this env's scenario straight from the sampler's buffers (no copy launches before the
    // rollout): S[0] agent records and goals, read back below by this workgroup only
    float4* S0 = const_cast<float4*>(c.S) + (long)b * Nn * REC<D>;
    for (int q = threadIdx.x; q < N; q += blockDim.x) {
      const float* x = ra.s0 + ((long)b * N + q) * 2 * D;
      if constexpr (D == 2) {
        S0[q] = make_float4(x[0], x[1], x[2], x[3]);
      } else {
        S0[2 * q] = make_float4(x[0], x[1], x[2], 0.f);
        S0[2 * q + 1] = make_float4(x[3], x[4], x[5], 0.f);
      }
    }
    float* Gb = const_cast<float*>(c.G) + (long)b * N * D;
    for (int q = threadIdx.x; q < N * D; q += blockDim.x) Gb[q] = ra.g0[(long)b * N * D + q];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int wave = wave_id();
  int T = -1;                  // horizon, once every env has published its first done step
  bool done = false;           // (thread 0) this env has published
  // diagnostics builds (MB_STAMPS, c.stamps set): per-wave cycles of each phase summed over the
  // steps -- 0 scan, 1 edge phase, 2 barrier, 3 node phase, 4 step tail; 15 steps
  unsigned long long ph[16] = {}, tck = 0;
  auto stamp = [&](int k) {
    if constexpr (MB_STAMPS) {
      const unsigned long long tn = __builtin_amdgcn_s_memtime();
      ph[k] += tn - tck;
      tck = tn;
    }
  };
  for (int t = 0; t <= Tmax; ++t) {
    if constexpr (MB_STAMPS) { tck = __builtin_amdgcn_s_memtime(); ph[15] += 1; }
    // one relaxed poll of the done count per step; once it reads B, ONE agent-scope acquire
    // (pairs with the publishers' release adds below) before ctl[1] is read
    if (threadIdx.x == 0) {
      if (T < 0 && __hip_atomic_load(ra.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == B) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        T = min(Tmax, __hip_atomic_load(ra.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1);
      }
      L.dec = T;
    }
    __syncthreads();
    T = L.dec;
    if (T >= 0 && t > T) break;
    const bool tail = t == Tmax || t == T;       // s_T: scan only
    const long tb = (long)t * B + b;
    const float4* St = c.S + tb * Nn * REC<D>;
    if (N * ((Nn + SR_JG_SMALL - 1) / SR_JG_SMALL) <= SR_WAVES * WAVE)
      small_scan<D, SR_JG_SMALL>(ra, St, N, Nn, K, t < Tmax || ra.knn_tail, t < Tmax, ra.idx + tb * nk,
                                 ra.dang + tb * nk, ra.cnt + tb * 2, ra.safe ? ra.safe + tb : nullptr, L);
    else
      small_scan<D, SR_JG>(ra, St, N, Nn, K, t < Tmax || ra.knn_tail, t < Tmax, ra.idx + tb * nk, ra.dang + tb * nk,
                           ra.cnt + tb * 2, ra.safe ? ra.safe + tb : nullptr, L);
    stamp(0);
    if (tail) break;
    // env b's view of step t: the per-step controller bodies over this env's agents only
    CtrlArgs e = c;
    e.S = St; e.s_env = Nn;
    e.G = c.G + (long)b * N * D;
    e.idx = ra.idx + tb * nk; e.i_env = nk;
    e.B = 1; e.b0 = b; e.nb_total = B;
    e.A = c.A ? c.A + tb * N * D : nullptr; e.a_env = N;
    e.Snext = const_cast<float4*>(c.S) + (tb + B) * Nn * REC<D>; e.sn_env = Nn;
    e.dist_sum = c.dist_sum + tb; e.d_env = 1;
    e.act_sum = c.act_sum ? c.act_sum + tb : nullptr; e.ac_env = 1;
    e.pooled = c.pooled + tb * N * PROW; e.p_env = (long)N * PROW;
    e.argmax = c.argmax + tb * N * 128; e.am_env = (long)N * 128;
    e.acts = c.acts ? c.acts + tb * N * NODE_ACT_BYTES : nullptr; e.na_env = N;
    e.noise_t = t;
    ctrl_fwd_groups<D, true>(e, wl, wn, vl, nullptr, wave, SR_WAVES);
    stamp(1);
    __syncthreads();                                // the env's pooled rows -> node phase
    stamp(2);
    ctrl_node_groups<D, ACTS>(e, wn, vl, wave, SR_WAVES);
    stamp(3);
    // s_{t+1} (read by this workgroup only) and the env's sum atomics (device scope) complete
    // before the barrier; the workgroup-scope barrier is enough for both
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && !done) {
      const unsigned long long d = __hip_atomic_load(e.dist_sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((float)((double)d / FX_DIST) / (float)N < ra.done_thr) {   // the host check's arithmetic
        done = true;
        __hip_atomic_fetch_max(ra.ctl + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // release (agent scope, once per env and rollout): the max is ordered before the count
        __hip_atomic_fetch_add(ra.ctl, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    stamp(4);
  }
  if constexpr (MB_STAMPS) {
    if (c.stamps && (threadIdx.x & 63) == 0)
      for (int k = 0; k < 16; ++k) c.stamps[((long)b * SR_WAVES + wave) * 16 + k] = ph[k];
  }
  // The last workgroup to finish hands the horizon to the host (host-coherent memory, polled by
  // csrc/runtime.cpp run_small) and re-arms the control words for the next launch: no memset,
  // read-back copy or stream synchronisation around the launch.
  if (ra.res && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(ra.ctl + 2, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == B - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const int nd = __hip_atomic_load(ra.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int mx = __hip_atomic_load(ra.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int q = 0; q < 3; ++q) __hip_atomic_store(ra.ctl + q, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ra.res, nd == B ? min(Tmax, mx + 1) : Tmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ra.res + 1, ra.res_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

size_t rollout_small_lds() { return (size_t)CTRL_FWD_FRAGS * FRAG_SZ + CTRL_VEC * 4; }


}  // namespace MB_PREC
}  // namespace mb

#include "ctrl16.h"
#include "node16.h"

extern "C" int MB_SYM(node_act_bytes)() { return mb::MB_PREC::NODE_ACT_BYTES; }

// kernel 0: CBF backward (cbf16.h), 1: edge backward (ctrl16.h), 2: node backward (node16.h)
extern "C" int MB_SYM(k16_wg_per_cu)(int kernel) {
  return kernel == 0 ? CBF16_WGPC : kernel == 1 ? mb::MB_PREC::E16_WG_PER_CU : 1;
}

extern "C" int MB_SYM(ctrl_node_bwd)(const mb::CtrlNodeBwdArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (a->wrm16) {   // 16x16x32 kernel (csrc/node16.h; 128-agent chunks)
    if (a->dim == 3) launch_ctrl_node_bwd16<3>(*a, num_blocks, st);
    else launch_ctrl_node_bwd16<2>(*a, num_blocks, st);
    return (int)hipGetLastError();
  }
  const size_t lds = ctrl_node_bwd_lds();
  CtrlNodeBwdArgs b = *a;
  b.coop = node_bwd_coop_enabled() && a->chunk == 32;     // 32-agent chunks: the four waves cooperate
  const void* fn = a->dim == 3 ? (b.coop ? (const void*)ctrl_node_bwd_coop_kernel<3> : (const void*)ctrl_node_bwd_kernel<3>)
                               : (b.coop ? (const void*)ctrl_node_bwd_coop_kernel<2> : (const void*)ctrl_node_bwd_kernel<2>);
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  void* kargs[] = {&b};
  const hipError_t rc = hipLaunchKernel(fn, dim3(num_blocks), dim3(NB_WAVES * 64), kargs, lds, st);
  if (rc != hipSuccess) return (int)rc;
  return (int)hipGetLastError();
}



extern "C" int MB_SYM(ctrl_edge_bwd)(const mb::CtrlEdgeBwdArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (a->K > 16 || a->K < 1) return -1;
  if (a->w16) {   // 16x16x32 kernel (csrc/ctrl16.h; K = 12)
    if (a->K != 12) return -7;
    if (a->dim == 3) launch_ctrl_edge_bwd16<3>(*a, num_blocks, st);
    else launch_ctrl_edge_bwd16<2>(*a, num_blocks, st);
    return (int)hipGetLastError();
  }
  const size_t lds = ctrl_edge_bwd_lds();
  // K = 12 (TOP_K): constant-K instantiation (A/B vs runtime K: 136.7 vs 137.1-139.6 us, PERF.md)
  constexpr bool k12_off = false;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(num_blocks), dim3(EB_WAVES * 64), lds, st, *a);
  };
  const bool k12 = a->K == 12 && !k12_off;
  if (a->dim == 3) {
    if (k12) go(ctrl_edge_bwd_kernel<3, 12>);
    else go(ctrl_edge_bwd_kernel<3>);
  } else {
    if (k12) go(ctrl_edge_bwd_kernel<2, 12>);
    else go(ctrl_edge_bwd_kernel<2>);
  }
  return (int)hipGetLastError();
}

// One BPTT step in one launch for the cooperative regime (32-agent chunks: strong-scaling slices):
// the node backward of a workgroup's chunks, then the edge backward of the SAME agents (SPLIT: a
// chunk's K edge tiles over the four waves). The edge phase needs only its own agents' dL/dpooled
// rows, written by this workgroup's node phase (stores drained + barrier, same CU), so no grid-wide
// synchronisation; the next step's node phase (fused combine: other agents' in-edges) is the next
// launch. Saves one launch and its drain per reverse step. Slab rows: one node and one edge row
// per workgroup.
extern "C" int MB_SYM(ctrl_bwd_step)(const mb::CtrlNodeBwdArgs* na, const mb::CtrlEdgeBwdArgs* ea, int num_blocks,
                                     hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (ea->K > 16 || ea->K < 1 || na->chunk != 32 || na->dim != ea->dim || na->B != ea->B || na->N != ea->N) return -1;
  const size_t lds = ctrl_node_bwd_lds() > ctrl_edge_bwd_lds() ? ctrl_node_bwd_lds() : ctrl_edge_bwd_lds();
  CtrlNodeBwdArgs n = *na;
  n.coop = 1;
  CtrlEdgeBwdArgs e = *ea;
  e.qsplit = 1;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(num_blocks), dim3(NB_WAVES * 64), lds, st, n, e);
  };
  const bool k12 = ea->K == 12;
  if (ea->dim == 3) {
    if (k12) go(ctrl_bwd_step_kernel<3, 12>);
    else go(ctrl_bwd_step_kernel<3, 0>);
  } else {
    if (k12) go(ctrl_bwd_step_kernel<2, 12>);
    else go(ctrl_bwd_step_kernel<2, 0>);
  }
  return (int)hipGetLastError();
}

extern "C" int MB_SYM(rollout_small)(const mb::RolloutSmallArgs* a, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  const CtrlArgs& c = a->c;
  if (c.K > 16 || c.K < 1 || c.N < 1 || a->Nn < c.N || a->Nn > SMALL_MAXN || c.K > a->Nn || a->Tmax < 1) return -1;
  if (!a->ctl || !a->idx || !a->dang || !a->cnt || !c.pooled || !c.argmax || !c.dist_sum || !c.S) return -2;
  if (c.apw < 2 || c.apw > 32 || (c.apw & 1)) return -3;
  const size_t lds = rollout_small_lds();
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(c.B), dim3(SR_WAVES * 64), lds, st, *a);
  };
  if (c.dim == 3) {
    if (c.acts) go(rollout_small_kernel<3, true>);
    else go(rollout_small_kernel<3, false>);
  } else {
    if (c.acts) go(rollout_small_kernel<2, true>);
    else go(rollout_small_kernel<2, false>);
  }
  return (int)hipGetLastError();
}

