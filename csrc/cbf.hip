// CBF kernels (reference cbf.py:21-45, losses core.py:89-171), gfx950.
//
// Per-edge barrier h(x_i, x_j): features [dx dy dvx dvy eye |dp|_eps - r] (+ constant 1 for
// the folded bias) -> 64 -> 128 -> 64 -> 1, radius-masked. A wave evaluates 32 edges per
// tile; every layer is a v_mfma_f32_32x32x16_bf16 chain whose accumulator is the next
// layer's B operand (no LDS traffic for activations), weights are pre-packed 1 KiB
// fragments in LDS, the 64->1 head is an in-lane dot + one lane^32 swap.
//
// cbf_fwd_kernel: over all (b, t, i, k) edges of a trajectory it evaluates h on s_t and
// h' on s_{t+1} (same neighbour slots, reuse_nbr_idx), applies the per-edge TTC danger bit
// and env-step validity, and emits
//   * per-workgroup partial sums of the 8 barrier/derivative loss terms + 2 counts
//     (no masked_select, no dynamic shapes, no host sync),
//   * the upstream gradients dL/dh, dL/dh' per edge (mask folded in), given the global
//     pooled counts -- consumed by cbf_bwd_kernel.
#pragma clang fp contract(off)
#include "common.h"
#include "args.h"
#include "state.h"

// waves per 32x32x16 CBF-backward workgroup: x3 4 (one per SIMD: the split activations double
// the register footprint), 1-pass 8 (two per SIMD)
constexpr int CBF_NW = MB_X3 ? 4 : 8;

namespace mb {
namespace MB_PREC {

constexpr int CBF_FWD_FRAGS = 34;  // w1f 2 + w2 16 + w3 16
constexpr int CBF_VEC = 260;       // b2 128 | b3 64 | w4 64 | b4 1 (+3 pad)



// Layer-1 B fragment of one edge (K slots: see layout.cbf_w1_slot): fp32 features split into
// h16 hi (lanes h = 0) and residual lo (lanes h = 1) parts.
template <int D>
DEV h16x8 cbf_edge_frag(const float (&rp)[D], const float (&rv)[D], float eye, float dfeat, bool ok, int h) {
  h16x8 f;
  const h16 z = (h16)0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = z;
  if (!ok) return f;
  h16 hi[2 * D + 1], lo[2 * D + 1];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    split_h16(rp[q], hi[q], lo[q]);
    split_h16(rv[q], hi[D + q], lo[D + q]);
  }
  split_h16(dfeat, hi[2 * D], lo[2 * D]);
  if constexpr (D == 2) {
    if (h == 0) {
      f[0] = hi[0]; f[1] = hi[1]; f[2] = hi[2]; f[3] = hi[3]; f[4] = (h16)eye; f[5] = hi[4]; f[6] = (h16)1.f;
    } else {
      f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3]; f[5] = lo[4];
    }
  } else {
    if (h == 0) {
#pragma unroll
      for (int q = 0; q < 7; ++q) f[q] = hi[q];
      f[7] = (h16)1.f;
    } else {
#pragma unroll
      for (int q = 0; q < 7; ++q) f[q] = lo[q];
      f[7] = (h16)eye;
    }
  }
  return f;
}

struct CbfActs { f32x16 H1[2], H2[4], H3[2]; };

// full forward for one 32-edge tile; returns the pre-mask head output for this lane's edge
DEV float cbf_mlp(const h16x8& F, const h16* wl, const float* vl, int lane, CbfActs& o) {
  const int h = lane >> 5;
  const float* b2 = vl;
  const float* b3 = vl + 128;
  const float* w4 = vl + 192;
  const float b4 = vl[256];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    o.H1[mt] = mma_bx(frag_fr(wl, mt, lane), F, zero16());
    relu_(o.H1[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    f32x16 c = bias_rows(b2, 32 * mt, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mma(frag_fr(wl, 2 + mt * 4 + kk, lane), acc_fr<kk & 1>(o.H1[kk >> 1]), c);
    });
    relu_(c);
    o.H2[mt] = c;
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x16 c = bias_rows(b3, 32 * mt, h);
    static_for<8>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mma(frag_fr(wl, 18 + mt * 8 + kk, lane), acc_fr<kk & 1>(o.H2[kk >> 1]), c);
    });
    o.H3[mt] = c;   // pre-activation kept (relu' needed in backward)
  }
  float s = 0.f;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg)
      s += w4[32 * mt + acc_row(reg, h)] * fmaxf(o.H3[mt][reg], 0.f);
  s += shfl_xor32(s);
  return s + b4;
}

template <int D>
struct EdgeCtx {
  bool ok;
  int b, t, i, j;
  float rp[D], rv[D];     // s_i - s_j: positions, velocities
  float eye, d, dfeat;
  bool mask;
};

// 32-bit index math throughout (host asserts passes*E < 2^31): 64-bit divisions/multiplies
// here cost dozens of VGPRs and instructions per edge. Strides are in node records.
template <int D>
DEV void cbf_edge(const float4* S, long s_env, long s_step, const int* idx, int B, int N, int K,
                  long e_, long E_, int tstep_off, float obs_r, float dist_thr, float dist_eps, EdgeCtx<D>& c) {
  const unsigned e = (unsigned)e_;
  c.ok = e_ < E_;
#pragma unroll
  for (int q = 0; q < D; ++q) { c.rp[q] = 0.f; c.rv[q] = 0.f; }
  c.eye = 0.f; c.d = 0.f; c.dfeat = 0.f; c.mask = false;
  c.b = c.t = c.i = c.j = 0;
  if (!c.ok) return;
  // time-major edge order: e = ((t*B + b)*N + i)*K + k
  const unsigned ik = e / (unsigned)K;
  const unsigned tb = ik / (unsigned)N;
  c.i = (int)(ik - tb * (unsigned)N);
  c.t = (int)(tb / (unsigned)B);
  c.b = (int)(tb - (unsigned)c.t * (unsigned)B);
  c.j = idx[e];
  const float4* Sb = S + ((unsigned)c.b * (unsigned)s_env + (unsigned)(c.t + tstep_off) * (unsigned)s_step) * REC<D>;
  float pi[D], vi[D], pj[D], vj[D];
  load_rec<D>(Sb, (unsigned)c.i, pi, vi);
  load_rec<D>(Sb, (unsigned)c.j, pj, vj);
#pragma unroll
  for (int q = 0; q < D; ++q) { c.rp[q] = pi[q] - pj[q]; c.rv[q] = vi[q] - vj[q]; }
  c.eye = (c.j == c.i) ? 1.f : 0.f;
  c.d = sqrtf(sqsum<D>(c.rp) + dist_eps);
  c.dfeat = c.d - dist_thr;
  c.mask = c.d <= obs_r;
}

template <int WAVES, int D>
__global__ __launch_bounds__(WAVES * 64) void cbf_fwd_kernel(CbfFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* wl = reinterpret_cast<h16*>(smem);
  float* vl = reinterpret_cast<float*>(smem + CBF_FWD_FRAGS * FRAG_SZ);
  __shared__ float red[10][WAVES];
  block_copy16(wl, a.wpack + (size_t)a.f_fwd * FRAG_ELEMS, CBF_FWD_FRAGS * FRAG_SZ, false);
  block_copy16(vl, a.wvec, CBF_VEC * 4);
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const long E = (long)a.B * a.T * a.N * a.K;
  const long ntiles = (E + 31) / 32;
  float nd = 0.f, ns = 0.f, lsc = a.lc.scale;
  if (a.dh_out) { nd = 1e-5f + a.counts[0]; ns = 1e-5f + a.counts[1]; lsc = lc_scale(a.lc); }
  float acc[10];
#pragma unroll
  for (int q = 0; q < 10; ++q) acc[q] = 0.f;
  CbfActs act;
  for (long tile = (long)blockIdx.x * WAVES + wave; tile < ntiles; tile += (long)gridDim.x * WAVES) {
    const long e = tile * 32 + r;
    EdgeCtx<D> c0;
    float hv = 0.f, hnv = 0.f;
    bool mask1 = false;
#pragma unroll 1
    for (int pass = 0; pass < 1 + a.two; ++pass) {
      const h16* wt = wl + opaque_zero();
      const float* vt = vl + opaque_zero();
      EdgeCtx<D> c;
      cbf_edge<D>(a.S, a.s_env, a.s_step, a.idx, a.B, a.N, a.K, e, E, pass, a.obs_r, a.dist_thr, a.dist_eps, c);
      const float hp = cbf_mlp(cbf_edge_frag<D>(c.rp, c.rv, c.eye, c.dfeat, c.ok, h), wt, vt, lane, act);
      if (pass == 0) { c0 = c; hv = c.mask ? hp : 0.f; }
      else { hnv = c.mask ? hp : 0.f; mask1 = c.mask; }
    }
    if (!c0.ok || h != 0) continue;
    if (a.h_out) a.h_out[e] = hv;
    if (a.hn_out) a.hn_out[e] = hnv;
    const bool vld = a.valid ? (a.valid[(long)c0.t * a.B + c0.b] != 0) : true;
    const bool dg = a.dang ? (a.dang[e] != 0) : false;
    float gh = 0.f, ghn = 0.f;
    if (vld && a.two) {
      const float deriv = hnv - hv + a.lc.dt_alpha * hv;
      if (dg) {
        acc[0] += 1.f;
        acc[2] += fmaxf(hv + a.lc.eps_dang, 0.f);
        acc[4] += (hv <= 0.f) ? 1.f : 0.f;
        acc[6] += fmaxf(-deriv + a.lc.eps_dang, 0.f);
        acc[8] += (deriv >= 0.f) ? 1.f : 0.f;
        if (a.dh_out) {
          const float c = lsc / nd;
          const float ind_b = (hv + a.lc.eps_dang > 0.f) ? 1.f : 0.f;
          const float ind_d = (-deriv + a.lc.eps_dang > 0.f) ? 1.f : 0.f;
          gh = c * (a.lc.w_dang * ind_b + a.lc.w_dang_d * ind_d * (1.f - a.lc.dt_alpha));
          ghn = -c * a.lc.w_dang_d * ind_d;
        }
      } else {
        acc[1] += 1.f;
        acc[3] += fmaxf(-hv, 0.f);
        acc[5] += (hv > 0.f) ? 1.f : 0.f;
        acc[7] += fmaxf(-deriv, 0.f);
        acc[9] += (deriv > 0.f) ? 1.f : 0.f;
        if (a.dh_out) {
          const float c = lsc / ns;
          const float ind_b = (-hv > 0.f) ? 1.f : 0.f;
          const float ind_d = (-deriv > 0.f) ? 1.f : 0.f;
          gh = c * (-a.lc.w_safe * ind_b + a.lc.w_safe_d * ind_d * (1.f - a.lc.dt_alpha));
          ghn = -c * a.lc.w_safe_d * ind_d;
        }
      }
    }
    if (a.dh_out) {
      a.dh_out[e] = c0.mask ? gh : 0.f;
      a.dh_out[E + e] = mask1 ? ghn : 0.f;
    }
  }
  if (!a.partial) return;
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    const float v = wave_sum(acc[q]);
    if (lane == 0) red[q][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 10) {
    float s = 0.f;
    for (int w = 0; w < WAVES; ++w) s += red[threadIdx.x][w];
    a.partial[(long)blockIdx.x * 10 + threadIdx.x] = s;
  }
}

constexpr int CBF_FWD_WAVES = 4;

}  // namespace MB_PREC
}  // namespace mb

extern "C" int MB_SYM(cbf_fwd)(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (a->K > 16 || a->K < 1) return -1;
  const size_t lds = (size_t)CBF_FWD_FRAGS * FRAG_SZ + CBF_VEC * 4;
  if (a->dim == 3) {
    (void)hipFuncSetAttribute((const void*)cbf_fwd_kernel<CBF_FWD_WAVES, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((cbf_fwd_kernel<CBF_FWD_WAVES, 3>), dim3(num_blocks), dim3(CBF_FWD_WAVES * 64), lds, st, *a);
  } else {
    (void)hipFuncSetAttribute((const void*)cbf_fwd_kernel<CBF_FWD_WAVES, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((cbf_fwd_kernel<CBF_FWD_WAVES, 2>), dim3(num_blocks), dim3(CBF_FWD_WAVES * 64), lds, st, *a);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// cbf_bwd_kernel<FUSED>: hand-written backward of the CBF edge MLP.
// Workgroup = 4 waves sharing a chunk of 128 evaluations (32 per wave):
//   data path (per wave, registers only): recompute H1,H2,H3 -> dH3 = w4*dh*relu'
//     -> dH2 = W3^T dH3 .relu' (16 MFMA) -> dH1 = W2^T dH2 .relu' (16) -> dF = W1^T dH1 (4)
//     -> dL/d(s_i - s_j) incl. the |dp|_eps feature; written per evaluation (self edges 0)
//   weight gradients (workgroup-shared): activations / deltas of the chunk are staged as
//     edge-major h16 LDS images; each wave owns a fixed subset of the 32x32 output tiles of
//     dW3 (64x128), dW2 (128x64), dW1f (64x32) and contracts over the chunk's 128 edges with
//     ds_read_b64_tr_b16 fragments -> MFMA; bias grads are row sums of the A fragments, split
//     over the waves that read the same row block; the 64->1 head (w4, b4) accumulates per
//     lane. Fixed ownership -> deterministic per-WG slabs, reduced by a separate pass.
// FUSED (training): the chunk is 64 edges x {h(s_t) (waves 0,1), h'(s_{t+1}) (waves 2,3)}. The
//   forward recompute includes the 64->1 head; h and h' of each edge meet in LDS, every wave
//   forms its upstream dL/dh locally (barrier + derivative hinge losses with the danger bit,
//   step validity and the global pooled counts) and the loss partial sums go to the slab. This
//   replaces the separate forward/loss kernel and the dh round trip through HBM.
// ---------------------------------------------------------------------------------------
namespace mb {
namespace MB_PREC {

// LDS row strides (h16 elements), chosen with a bank model of the access patterns
// (ds_read_b64 / ds_read_b64_tr_b16: 64 banks per 32-lane half; ds_write_b64: 32 banks per
// 16-lane group): 68 = 34 dwords and 148 = 74 dwords keep 32-row weight reads, 4-row transposed
// reads and 16-row tile stores conflict-free or 2-way at most (72 / 136 were 2-4 way).
constexpr int SA128 = 148, SA64 = 68, SA32 = 40;
constexpr int WS2 = 68, WS3 = 148;                  // row-major W2 [128][WS2], W3 [64][WS3] images
constexpr int RM_W2 = 128 * WS2, RM_W3 = 64 * WS3;  // row-major image sizes (elements)
constexpr int RM_LO = RM_W2 + RM_W3;                // lo plane offset of the images (x3)
constexpr int RMP = (X3 ? 2 : 1) * RM_LO;           // elements of the W2|W3 (+ lo) images
// per-WG partial slab layout (floats)
constexpr int P_W3 = 0, P_B3 = 8192, P_W2 = 8256, P_B2 = 16448, P_W1 = 16576, P_W4 = 18624, P_B4 = 18688;
constexpr int P_LOSS = 18692;                 // 10 loss partial sums (fused mode)
constexpr int CBF_PARTIAL = 18704;
constexpr size_t CBF_BWD_W_BYTES = (size_t)RMP * 2 + 6 * FRAG_SZ;

// Stage regions. NW = 4 waves (one per SIMD): two regions used alternately (stage k of the
// running sequence A,B,C,A,B,C,... writes region k&1): a region is rewritten only after every
// wave has passed the NEXT stage's barrier, i.e. finished reading it -> one barrier per stage.
// NW = 8 waves (two per SIMD, chunk of 256): one region (LDS), two barriers per stage.
// Stage A/B: (128 + 64)-wide images; stage C+D: dH1 | [F, dh, 0] | relu(H3) = 64+32+64 wide.
// x3: the images carry a lo plane, so a region holds the rows of TW = 2 waves: every stage runs
// in NT = NW / TW turns (the waves of a turn store, everybody contracts their rows), one region,
// two barriers per turn.
template <int NW> struct CbfCfg {
  static constexpr int CH = NW * 32;                          // evaluations per chunk
  static constexpr int KS = CH / 16;                          // edge steps per stage contraction
  static constexpr int TW = X3 ? 2 : NW;                      // waves whose rows a region holds
  static constexpr int NT = NW / TW;                          // turns per stage
  static constexpr int RT = TW * 32;                          // region rows
  static constexpr int KST = RT / 16;                         // edge steps per turn
  static constexpr int NREG = (NW == 4 && NT == 1) ? 2 : 1;
  static constexpr int PLANE = (SA64 + SA128) * RT;           // elements per region plane
  static constexpr int REGION = (X3 ? 2 : 1) * PLANE;         // elements per region
  static constexpr size_t LDS = CBF_BWD_W_BYTES + CBF_VEC * 4 + (size_t)NREG * REGION * 2;
};

template <int D>
struct CbfIn {
  EdgeCtx<D> c;
  float dh;       // upstream gradient (non-fused)
  bool in;
  bool dg, vld;   // fused: danger bit, env-step validity
  unsigned ev;    // evaluation index (pass*E + e)
};

template <bool FUSED, int NW, int D>
DEV void cbf_load(const CbfBwdArgs& a, long chunk, int wave, int r, long E, long EV, CbfIn<D>& x) {
  constexpr int CH = CbfCfg<NW>::CH;
  int pass;
  unsigned e;
  if constexpr (FUSED) {
    pass = wave / (NW / 2);
    e = (unsigned)chunk * (CH / 2) + (wave % (NW / 2)) * 32 + r;
    x.in = e < (unsigned)E;
    x.ev = (unsigned)pass * (unsigned)E + e;
  } else {
    const unsigned v = (unsigned)chunk * CH + wave * 32 + r;
    x.in = v < (unsigned)EV;
    const unsigned ev = (a.act && x.in) ? (unsigned)a.act[v] : v;   // active list: v -> evaluation
    pass = (x.in && ev >= (unsigned)E) ? 1 : 0;
    if (a.src) e = pass ? (unsigned)a.src[ev] : ev;   // deduplicated list: extras name their slot
    else e = ev - (unsigned)pass * (unsigned)E;
    x.ev = ev;
  }
  const int* idxp = (pass == 1 && a.idx1) ? a.idx1 : a.idx;
  cbf_edge<D>(a.S, a.s_env, a.s_step, idxp, a.B, a.N, a.K, e, x.in ? E : 0, pass, a.obs_r, a.dist_thr, a.dist_eps, x.c);
  if constexpr (FUSED) {
    x.dh = 0.f;
    x.dg = x.in && a.dang[e] != 0;
    x.vld = x.in && (a.valid ? (a.valid[(unsigned)x.c.t * (unsigned)a.B + (unsigned)x.c.b] != 0) : true);
  } else {
    x.dh = x.in ? a.dh[x.ev] : 0.f;
    x.dg = false;
    x.vld = false;
  }
}

// ---------------------------------------------------------------------------------------
// cbf_bwd_kernel<FUSED, NW>: hand-written backward of the CBF edge MLP.
// Workgroup = NW waves sharing a chunk of 32*NW evaluations (32 per wave):
//   data path (per wave, registers only): recompute H1,H2,H3 -> dH3 = w4*dh*relu'
//     -> dH2 = W3^T dH3 .relu' (16 MFMA) -> dH1 = W2^T dH2 .relu' (16) -> dF = W1^T dH1 (4)
//     -> dL/d(s_i - s_j) incl. the |dp|_eps feature; written per evaluation (self edges 0)
//   weight gradients (workgroup-shared): activations / deltas of the chunk are staged as
//     edge-major h16 LDS images; each wave owns a fixed subset of the 8 + 8 + 2 + 2 32x32
//     output tiles of dW3 (64x128), dW2 (128x64), dW1f (64x32), dW4pad (32x64) and contracts
//     over the chunk's edges with ds_read_b64_tr_b16 fragments -> MFMA; bias grads are row
//     sums of the A fragments, split over the waves that read the same row block; fixed
//     ownership -> deterministic per-WG slabs, reduced by a separate pass (no float atomics).
// FUSED (training): the chunk is CH/2 edges x {h(s_t) (waves < NW/2), h'(s_{t+1}) (the rest)}.
//   The forward recompute includes the 64->1 head; h and h' of each edge meet in LDS, every
//   wave forms its upstream dL/dh locally (barrier + derivative hinge losses with the danger
//   bit, step validity and the global pooled counts) and the loss partial sums go to the slab.
// ---------------------------------------------------------------------------------------

// h over a deduplicated evaluation list (dedup.hip): evaluation u < E is main slot u on s_t,
// u >= E the extra evaluation of slot src[u] on s_{t+1} (neighbour idx1[src[u]]). Writes the
// masked h and the radius mask per evaluation; the losses / upstream gradients are formed by
// cbf_dh_kernel from these values and the backward runs as cbf_bwd_kernel<false> on the same
// list. The forward is the backward kernel's recompute chain (row-major W2/W3 images shared
// with it, packed relu, fp32 head), without the weight-gradient stages: ~40 KB of LDS, so
// four 8-wave workgroups share a CU; the edge gathers of the next tile are issued before the
// MFMA chain of the current one.
// x3: without the next-tile prefetch the kernel fits 122 VGPRs -> two 8-wave workgroups
// (4 waves/SIMD, LDS 2 x 70 KB) per CU instead of one: 1.31 -> 1.22 ms per iteration's h
// (profiles/r2_hfwd/); the 16-bit builds keep the prefetch (40 KB LDS, more resident waves)
constexpr int CBF_HFWD_MINW = MB_X3 ? 4 : 1;
template <int NW, int D>
__global__ __launch_bounds__(NW * 64, CBF_HFWD_MINW) void cbf_hfwd_kernel(CbfFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* W2 = reinterpret_cast<h16*>(smem);
  h16* W3 = W2 + RM_W2;
  h16* wf = W2 + RMP;                         // w1f (2 frags)
  float* vl = reinterpret_cast<float*>(smem + (size_t)RMP * 2 + 2 * FRAG_SZ);
  block_copy16(W2, a.wrm, RMP * 2, false);
  block_copy16(wf, a.wpack + (size_t)a.f_fwd * FRAG_ELEMS, 2 * FRAG_SZ, false);
  block_copy16(vl, a.wvec, CBF_VEC * 4);
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const unsigned E = (unsigned)a.B * a.T * a.N * a.K;
  const unsigned U = a.u_end ? a.u_end : (unsigned)*a.nev;
  const unsigned U0 = a.u_begin;
  const unsigned ntiles = U > U0 ? (U - U0 + 31) / 32 : 0;
  const unsigned stride = gridDim.x * NW;
  auto load = [&](unsigned tile, EdgeCtx<D>& c) {
    const unsigned u = U0 + tile * 32 + r;
    const bool in = u < U;
    const int pass = (in && u >= E) ? 1 : 0;
    const unsigned e = pass ? (unsigned)a.src[u] : u;
    cbf_edge<D>(a.S, a.s_env, a.s_step, pass ? a.idx1 : a.idx, a.B, a.N, a.K, e, in ? E : 0, pass, a.obs_r,
                a.dist_thr, a.dist_eps, c);
  };
// 1-pass builds: the three-stage gather pipeline below (bf16 headline 6.86-6.88 vs 6.89-6.91 ms,
// profiles/r4_loads/); x3: no prefetch at all -- the pipeline's registers spill at the 128 of four
// waves per SIMD (10.91-10.94 vs 10.93 ms, 3 waves per SIMD 10.96-10.98 ms; the one-tile-ahead
// prefetch variant is in the git history, round 5)
#if !MB_X3
  // Gather pipeline over a wave's tiles k, k + stride, ...: the chain src[u] (extras) -> idx[e] ->
  // S[i], S[j] is three dependent loads, so each runs one tile apart -- src three tiles ahead, idx
  // two ahead, the two node records one ahead -- every load unconditional (clamped indices) and
  // consumed an iteration after its issue: no memory latency inside the MFMA loop.
  struct P0 { unsigned srcv; };
  struct P1 { int j; unsigned e; int pass; bool in; };
  struct P2 { float4 si[REC<D>], sj[REC<D>]; int i, j; bool in; };
  auto tile_u = [&](unsigned tl) { return U0 + tl * 32 + r; };
  auto s0 = [&](unsigned tl, P0& o) {
    const unsigned u = tile_u(tl);
    const bool pass = u < U && u >= E;
    o.srcv = (unsigned)a.src[pass ? u : 0u];
  };
  auto s1 = [&](unsigned tl, const P0& x, P1& o) {
    const unsigned u = tile_u(tl);
    o.in = u < U;
    o.pass = (o.in && u >= E) ? 1 : 0;
    o.e = o.in ? (o.pass ? x.srcv : u) : 0u;
    o.j = (o.pass ? a.idx1 : a.idx)[o.e];
  };
  auto s2 = [&](const P1& x, P2& o) {
    const unsigned ik = x.e / (unsigned)a.K;
    const unsigned tb = ik / (unsigned)a.N;
    const unsigned i = ik - tb * (unsigned)a.N;
    const unsigned t = tb / (unsigned)a.B;
    const unsigned b = tb - t * (unsigned)a.B;
    const float4* Sb = a.S + ((unsigned)b * (unsigned)a.s_env + (t + (unsigned)x.pass) * (unsigned)a.s_step) * REC<D>;
#pragma unroll
    for (int k = 0; k < REC<D>; ++k) { o.si[k] = Sb[REC<D> * i + k]; o.sj[k] = Sb[REC<D> * (unsigned)x.j + k]; }
    o.i = (int)i;
    o.j = x.j;
    o.in = x.in;
  };
  const unsigned t0 = (CBF_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x) * NW + wave;
  P0 p0{};
  P1 p1{};
  P2 p2{};
  {
    // prologue: tiles t0 (-> P2), t0 + stride (-> P1), t0 + 2 stride (-> P0); tiles past the end
    // load clamped records (never used)
    P0 q0;
    s0(t0, q0);
    P1 q1;
    s1(t0, q0, q1);
    s2(q1, p2);
    s0(t0 + stride, q0);
    s1(t0 + stride, q0, p1);
    s0(t0 + 2 * stride, p0);
  }
  for (unsigned tile = t0; tile < ntiles; tile += stride) {
    const P2 cur = p2;
    s2(p1, p2);                                   // node j of tile + stride
    s1(tile + 2 * stride, p0, p1);                // idx + node i of tile + 2 stride
    s0(tile + 3 * stride, p0);                    // src of tile + 3 stride
    EdgeCtx<D> c;
    {
      float pi[D], vi[D], pj[D], vj[D];
      load_rec_regs<D>(cur.si, pi, vi);
      load_rec_regs<D>(cur.sj, pj, vj);
      c.ok = cur.in;
#pragma unroll
      for (int q = 0; q < D; ++q) {
        c.rp[q] = cur.in ? pi[q] - pj[q] : 0.f;
        c.rv[q] = cur.in ? vi[q] - vj[q] : 0.f;
      }
      c.eye = (cur.in && cur.j == cur.i) ? 1.f : 0.f;
      c.d = sqrtf(sqsum<D>(c.rp) + a.dist_eps);
      c.dfeat = cur.in ? c.d - a.dist_thr : 0.f;
      c.mask = cur.in && c.d <= a.obs_r;
    }
#else
  unsigned tile = (CBF_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x) * NW + wave;
  for (; tile < ntiles; tile += stride) {
    EdgeCtx<D> c;
    load(tile, c);
#endif
    const h16x8 F = cbf_edge_frag<D>(c.rp, c.rv, c.eye, c.dfeat, c.ok, h);
    const h16* wt = wf + opaque_zero();
    const h16* W2c = W2 + opaque_zero();
    const h16* W3c = W3 + opaque_zero();
    const float* vlc = vl + opaque_zero();
    const float* b2 = vlc;
    const float* b3 = vlc + 128;
    const float* w4 = vlc + 192;
    Pk H1b[2], H2b[4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) H1b[mt] = to_pk_relu(mma_bx(frag_fr(wt, mt, lane), F, zero16()));
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x16 t2 = bias_rows4(b2, 32 * mt, h);
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t2 = mma(wrm_acc_fr(W2c, WS2, 32 * mt, kk, lane, RM_LO), pk_fr<kk & 1>(H1b[kk >> 1]), t2);
      });
      H2b[mt] = to_pk_relu(t2);
    }
    f32x2 hs2 = {0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 t3 = bias_rows4(b3, 32 * mt, h);
      static_for<8>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t3 = mma(wrm_acc_fr(W3c, WS3, 32 * mt, kk, lane, RM_LO), pk_fr<kk & 1>(H2b[kk >> 1]), t3);
      });
      relu_(t3);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 w = *reinterpret_cast<const float4*>(w4 + 32 * mt + 8 * g + 4 * h);
        hs2 = __builtin_elementwise_fma(f32x2{w.x, w.y}, f32x2{t3[4 * g], t3[4 * g + 1]}, hs2);
        hs2 = __builtin_elementwise_fma(f32x2{w.z, w.w}, f32x2{t3[4 * g + 2], t3[4 * g + 3]}, hs2);
      }
    }
    float hs = hs2.x + hs2.y;
    hs += shfl_xor32(hs);
    const unsigned u = U0 + tile * 32 + r;
    if (u < U && h == 0) {
      a.h_out[u] = c.mask ? hs + vlc[256] : 0.f;
      a.mask_out[u] = c.mask ? 1 : 0;
    }
  }
}

constexpr int HFWD_WAVES = 8;
constexpr size_t HFWD_LDS = (size_t)RMP * 2 + 2 * FRAG_SZ + CBF_VEC * 4;

template <bool FUSED, int NW, int D>
__global__ __launch_bounds__(NW * 64, 1) void cbf_bwd_kernel(CbfBwdArgs a) {
  using Cfg = CbfCfg<NW>;
  constexpr int CH = Cfg::CH, KS = Cfg::KS, KST = Cfg::KST, RT = Cfg::RT, TW = Cfg::TW, NT = Cfg::NT;
  constexpr int PL = Cfg::PLANE;               // lo plane offset inside a region (x3)
  constexpr int TA = 8 / NW;                   // owned dW3 tiles (and dW2 tiles) per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* W2 = reinterpret_cast<h16*>(smem);
  h16* W3 = W2 + RM_W2;
  h16* wf = W2 + RMP;                         // w1f (2 frags) | w1ft (4 frags)
  float* vl = reinterpret_cast<float*>(smem + CBF_BWD_W_BYTES);
  h16* stg = reinterpret_cast<h16*>(smem + CBF_BWD_W_BYTES + CBF_VEC * 4);
  __shared__ float hx[CH];                     // fused: h / h' exchange
  __shared__ float lacc[8][FUSED ? CH / 2 : 1];  // fused: per-lane loss partial sums (pass-0 lanes)
  __shared__ float lred[NW][10];
  __shared__ float red4[NW];
  block_copy16(W2, a.wrm, RMP * 2, false);
  block_copy16(wf, a.wpack + (size_t)a.f_bwd * FRAG_ELEMS, 2 * FRAG_SZ, false);
  block_copy16(wf + 2 * FRAG_ELEMS, a.wpack + (size_t)(a.f_bwd + 66) * FRAG_ELEMS, 4 * FRAG_SZ, false);
  block_copy16(vl, a.wvec, CBF_VEC * 4);
  if constexpr (FUSED)
    for (int q = threadIdx.x; q < 8 * CH / 2; q += blockDim.x) (&lacc[0][0])[q] = 0.f;
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const long E = (long)a.B * a.T * a.N * a.K;
  const long EV = (!FUSED && a.nact) ? (long)*a.nact : (!FUSED && a.nev) ? (long)*a.nev : E * a.passes;
  const long nchunks = FUSED ? (E + CH / 2 - 1) / (CH / 2) : (EV + CH - 1) / CH;
  const int erow = wave * 32 + r;
  const int trow = NT == 1 ? erow : (wave % TW) * 32 + r;   // this wave's rows inside a turn's region
  const int myturn = wave / TW;
  const int pass_w = wave / (NW / 2);          // fused: this wave's pass
  float nd = 1.f, ns = 1.f, lsc = a.lc.scale;
  if constexpr (FUSED) { nd = 1e-5f + a.counts[0]; ns = 1e-5f + a.counts[1]; lsc = lc_scale(a.lc); }
  f32x16 accA[TA], accB[TA], accC = zero16();
  float bA[TA], bB[TA], db4 = 0.f;
#pragma unroll
  for (int u = 0; u < TA; ++u) { accA[u] = accB[u] = zero16(); bA[u] = bB[u] = 0.f; }
  // bias-sum edge steps of the whole chunk: 4 waves read each dW3 row block, 2 waves each dW2
  // row block (split per turn by turn_range)
  const int bsA = (KS / 4) * (wave % 4), bsB = (KS / 2) * (wave % 2);
  int par = 0;                                 // stage region parity (NREG == 2)

  // diagnostics (a.stamps, normally null): shader-clock cycles per phase summed over the chunks
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tck = 0;
  auto stamp = [&](int k) {
    if (MB_STAMPS && a.stamps) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[k] += t - tck;
      tck = t;
    }
  };
  CbfIn<D> nx;
  if ((long)blockIdx.x < nchunks) cbf_load<FUSED, NW, D>(a, blockIdx.x, wave, r, E, EV, nx);
  for (long chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    if (MB_STAMPS && a.stamps) { tck = __builtin_amdgcn_s_memtime(); ph[7] += 1; }
    const CbfIn<D> cur = nx;
    if (chunk + gridDim.x < nchunks) cbf_load<FUSED, NW, D>(a, chunk + gridDim.x, wave, r, E, EV, nx);   // prefetch
    const EdgeCtx<D>& c = cur.c;
    const h16x8 F = cbf_edge_frag<D>(c.rp, c.rv, c.eye, c.dfeat, c.ok, h);
    // one opaque base per LDS image per chunk: the per-lane address math is computed once and
    // shared by all fragment reads (immediate offsets), while the loads themselves cannot be
    // hoisted out of the chunk loop (~100 weight VGPRs otherwise)
    const h16* wt = wf + opaque_zero();
    const h16* W2c = W2 + opaque_zero();
    const h16* W3c = W3 + opaque_zero();
    const float* vlc = vl + opaque_zero();
    const float* b2 = vlc;
    const float* b3 = vlc + 128;
    const float* w4 = vlc + 192;
    // ---- forward recompute
    Pk H1b[2], H2b[4];
    f32x16 H3p[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const f32x16 t1 = mma_bx(frag_fr(wt, mt, lane), F, zero16());
      H1b[mt] = to_pk_relu(t1);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x16 t2 = bias_rows4(b2, 32 * mt, h);
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t2 = mma(wrm_acc_fr(W2c, WS2, 32 * mt, kk, lane, RM_LO), pk_fr<kk & 1>(H1b[kk >> 1]), t2);
      });
      H2b[mt] = to_pk_relu(t2);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 t3 = bias_rows4(b3, 32 * mt, h);
      static_for<8>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t3 = mma(wrm_acc_fr(W3c, WS3, 32 * mt, kk, lane, RM_LO), pk_fr<kk & 1>(H2b[kk >> 1]), t3);
      });
      relu_(t3);                                   // relu(H3) in fp32 (the head is fp32)
      H3p[mt] = t3;
    }
    stamp(0);                                      // loads + forward recompute
    float dhv = cur.dh;
    if constexpr (FUSED) {
      // ---- head, h/h' exchange, local loss + upstream gradient
      f32x2 hs2 = {0.f, 0.f};                      // packed fp32 FMAs (v_pk_fma_f32)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 w = *reinterpret_cast<const float4*>(w4 + 32 * mt + 8 * g + 4 * h);
          hs2 = __builtin_elementwise_fma(f32x2{w.x, w.y}, f32x2{H3p[mt][4 * g], H3p[mt][4 * g + 1]}, hs2);
          hs2 = __builtin_elementwise_fma(f32x2{w.z, w.w}, f32x2{H3p[mt][4 * g + 2], H3p[mt][4 * g + 3]}, hs2);
        }
      float hs = hs2.x + hs2.y;
      hs += shfl_xor32(hs);
      const float hm = (cur.in && c.mask) ? hs + vlc[256] : 0.f;
      if (h == 0) hx[erow] = hm;
      __syncthreads();
      const float other = hx[(wave ^ (NW / 2)) * 32 + r];
      const float hv = pass_w == 0 ? hm : other;
      const float hnv = pass_w == 0 ? other : hm;
      float gh = 0.f, ghn = 0.f;
      if (cur.vld) {
        const float deriv = hnv - hv + a.lc.dt_alpha * hv;
        const bool acc_here = (pass_w == 0) && (h == 0);
        if (cur.dg) {
          const float cc = lsc / nd;
          const float ind_b = (hv + a.lc.eps_dang > 0.f) ? 1.f : 0.f;
          const float ind_d = (-deriv + a.lc.eps_dang > 0.f) ? 1.f : 0.f;
          gh = cc * (a.lc.w_dang * ind_b + a.lc.w_dang_d * ind_d * (1.f - a.lc.dt_alpha));
          ghn = -cc * a.lc.w_dang_d * ind_d;
          if (acc_here) {   // loss sums live in LDS (registers are the limit at 2 waves/SIMD)
            lacc[0][erow] += fmaxf(hv + a.lc.eps_dang, 0.f);
            lacc[2][erow] += (hv <= 0.f) ? 1.f : 0.f;
            lacc[4][erow] += fmaxf(-deriv + a.lc.eps_dang, 0.f);
            lacc[6][erow] += (deriv >= 0.f) ? 1.f : 0.f;
          }
        } else {
          const float cc = lsc / ns;
          const float ind_b = (-hv > 0.f) ? 1.f : 0.f;
          const float ind_d = (-deriv > 0.f) ? 1.f : 0.f;
          gh = cc * (-a.lc.w_safe * ind_b + a.lc.w_safe_d * ind_d * (1.f - a.lc.dt_alpha));
          ghn = -cc * a.lc.w_safe_d * ind_d;
          if (acc_here) {
            lacc[1][erow] += fmaxf(-hv, 0.f);
            lacc[3][erow] += (hv > 0.f) ? 1.f : 0.f;
            lacc[5][erow] += fmaxf(-deriv, 0.f);
            lacc[7][erow] += (deriv > 0.f) ? 1.f : 0.f;
          }
        }
      }
      dhv = (cur.in && c.mask) ? (pass_w == 0 ? gh : ghn) : 0.f;
    }
    if (h == 0) db4 += dhv;
    // ---- head backward
    // dH3pre = w4 * dh . relu'(H3): packed products, then the 16-bit relu' mask of relu(H3)
    Pk d3b[2], H3b[2];
    const f32x2 dh2 = {dhv, dhv};
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 d3;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 w = *reinterpret_cast<const float4*>(w4 + 32 * mt + 8 * g + 4 * h);
        const f32x2 lo = f32x2{w.x, w.y} * dh2, hi = f32x2{w.z, w.w} * dh2;
        d3[4 * g] = lo.x; d3[4 * g + 1] = lo.y; d3[4 * g + 2] = hi.x; d3[4 * g + 3] = hi.y;
      }
      H3b[mt] = to_pk(H3p[mt]);
      d3b[mt] = to_pk(d3);
      mask_pk(d3b[mt], H3b[mt]);
    }
    // ---- stage A: dW3 (64x128) += dH3pre . H2^T ; db3   (tiles t = wave + NW u -> (t/4, t%4))
#pragma unroll
    for (int turn = 0; turn < NT; ++turn) {
      h16* imA = stg + par * Cfg::REGION;
      h16* imB = imA + RT * SA64;
      if (NT == 1 || myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk(imA, SA64, trow, 32 * mt, d3b[mt], h, PL);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store_pk(imB, SA128, trow, 32 * mt, H2b[mt], h, PL);
      }
      __syncthreads();
      int blo, bhi;
      if constexpr (NT == 1) { blo = bsA; bhi = bsA + KS / 4; }
      else turn_range(bsA, bsA + KS / 4, turn, KST, blo, bhi);
#pragma unroll
      for (int u = 0; u < TA; ++u) {
        const int t = wave + NW * u;
        bA[u] += stage_mma_fr<KST>(imA, SA64, PL, imB, SA128, PL, t / 4, t % 4, lane, accA[u], blo, bhi);
      }
      if constexpr (Cfg::NREG == 2) par ^= 1; else __syncthreads();
    }
    stamp(1);                                      // head backward + stage A
    // ---- dH2pre = (W3^T dH3pre) . relu'(H2)
    Pk d2b[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x16 t = zero16();
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t = mma(wrmT_acc_fr(W3c, WS3, 32 * mt, kk, lane, RM_LO), pk_fr<kk & 1>(d3b[kk >> 1]), t);
      });
      d2b[mt] = to_pk(t);
      mask_pk(d2b[mt], H2b[mt]);
    }
    stamp(2);                                      // dH2
    // ---- stage B: dW2 (128x64) += dH2pre . H1^T ; db2   (tiles t = wave + NW u -> (t/2, t%2))
#pragma unroll
    for (int turn = 0; turn < NT; ++turn) {
      h16* imA = stg + par * Cfg::REGION;
      h16* imB = imA + RT * SA128;
      if (NT == 1 || myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store_pk(imA, SA128, trow, 32 * mt, d2b[mt], h, PL);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk(imB, SA64, trow, 32 * mt, H1b[mt], h, PL);
      }
      __syncthreads();
      int blo, bhi;
      if constexpr (NT == 1) { blo = bsB; bhi = bsB + KS / 2; }
      else turn_range(bsB, bsB + KS / 2, turn, KST, blo, bhi);
#pragma unroll
      for (int u = 0; u < TA; ++u) {
        const int t = wave + NW * u;
        bB[u] += stage_mma_fr<KST>(imA, SA128, PL, imB, SA64, PL, t / 2, t % 2, lane, accB[u], blo, bhi);
      }
      if constexpr (Cfg::NREG == 2) par ^= 1; else __syncthreads();
    }
    stamp(3);                                      // stage B
    // ---- dH1pre = (W2^T dH2pre) . relu'(H1)
    Pk d1b[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 t = zero16();
      static_for<8>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t = mma(wrmT_acc_fr(W2c, WS2, 32 * mt, kk, lane, RM_LO), pk_fr<kk & 1>(d2b[kk >> 1]), t);
      });
      d1b[mt] = to_pk(t);
      mask_pk(d1b[mt], H1b[mt]);
    }
    // ---- dF = W1^T dH1pre (rows: dx dy dvx dvy eye dist) -> dL/d(s_i - s_j)
    {
      f32x16 t = zero16();
      static_for<4>([&](auto kk_) {
        constexpr int kk = decltype(kk_)::value;
        t = mma(frag_fr(wt, 2 + kk, lane), pk_fr<kk & 1>(d1b[kk >> 1]), t);
      });
      // rows = feature columns: s_i - s_j (0..2D-1), eye (2D), dist (2D+1); lane h = 0 holds rows
      // 0..3 in regs 0..3, lane h = 1 rows 4..7
      float g4[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) { g4[q] = t[q]; g4[4 + q] = shfl_xor32(t[q]); }
      if (a.dE && cur.in && h == 0) {
        float dp[D], dv[D];
#pragma unroll
        for (int q = 0; q < D; ++q) { dp[q] = 0.f; dv[q] = 0.f; }
        if (c.ok && c.j != c.i) {
          const float ddist = g4[2 * D + 1] * (1.f / c.d);
#pragma unroll
          for (int q = 0; q < D; ++q) { dp[q] = g4[q] + ddist * c.rp[q]; dv[q] = g4[D + q]; }
        }
        store_rec<D>(a.dE, cur.ev, dp, dv);
      }
    }
    stamp(4);                                      // dH1, dF, dE store
    // ---- stage C+D: dW1f (64x32) += dH1pre . [F|dh|0]^T (waves 0,1; cols >= 16 unused);
    //      dW4pad (32x64) += [dh;0..] . relu(H3)^T, A = image cols 16..47 -> row 0 = dw4 (waves 2,3;
    //      rows >= 1 read padding / the next row and are discarded: MFMA rows are independent).
    //      x3: F is exact in h16 (its lo plane is zero); dh's residual goes to the lo plane.
#pragma unroll
    for (int turn = 0; turn < NT; ++turn) {
      h16* imC = stg + par * Cfg::REGION;
      h16* imF = imC + RT * SA64;
      h16* imH = imF + RT * SA32;
      if (NT == 1 || myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk(imC, SA64, trow, 32 * mt, d1b[mt], h, PL);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) store_pk(imH, SA64, trow, 32 * mt, H3b[mt], h, PL);
        h16x8 dv = zero_h8();
        const h16 dvh = (h16)dhv;
        if (h == 0) dv[0] = dvh;
        *reinterpret_cast<h16x8*>(imF + trow * SA32 + 8 * h) = F;
        *reinterpret_cast<h16x8*>(imF + trow * SA32 + 16 + 8 * h) = dv;
        if constexpr (X3) {
          h16x8 dvl = zero_h8();
          if (h == 0) dvl[0] = (h16)(dhv - (float)dvh);
          *reinterpret_cast<h16x8*>(imF + PL + trow * SA32 + 8 * h) = zero_h8();
          *reinterpret_cast<h16x8*>(imF + PL + trow * SA32 + 16 + 8 * h) = dvl;
        }
      }
      __syncthreads();
      if (wave < 2) stage_mma_fr<KST>(imC, SA64, PL, imF, SA32, PL, wave, 0, lane, accC);
      else if (wave < 4) stage_mma_fr<KST>(imF + 16, SA32, PL, imH, SA64, PL, 0, wave - 2, lane, accC);
      if constexpr (Cfg::NREG == 2) par ^= 1; else __syncthreads();
    }
    stamp(5);                                      // stage C+D
  }
  if (MB_STAMPS && a.stamps && lane == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) a.stamps[((long)blockIdx.x * NW + wave) * 8 + k] = ph[k];
  __syncthreads();   // all stage reads done: the stage region is reused below
  float* bred = reinterpret_cast<float*>(stg);        // [NW][192] bias partials: b3 (64) | b2 (128)
  for (int q = threadIdx.x; q < NW * 192; q += blockDim.x) bred[q] = 0.f;
  __syncthreads();

  // ---- per-workgroup slab
  float* P = a.partial + (long)blockIdx.x * CBF_PARTIAL;
#pragma unroll
  for (int u = 0; u < TA; ++u) {
    const int t = wave + NW * u;
    write_tile(P + P_W3, 128, t / 4, t % 4, accA[u], lane);
    write_tile(P + P_W2, 64, t / 2, t % 2, accB[u], lane);
    const float s3 = bA[u] + shfl_xor32(bA[u]);
    const float s2 = bB[u] + shfl_xor32(bB[u]);
    if (h == 0) {
      bred[wave * 192 + 32 * (t / 4) + r] = s3;
      bred[wave * 192 + 64 + 32 * (t / 2) + r] = s2;
    }
  }
  if (wave < 2) {
    write_tile(P + P_W1, 32, wave, 0, accC, lane);
  } else if (wave < 4) {
    if (h == 0) P[P_W4 + 32 * (wave - 2) + r] = accC[0];   // dW4pad row 0 = dw4
  }
  // db4 (exact fp32) and loss sums: per-wave partials, fixed-order sums through LDS
  const float s4 = wave_sum(db4);
  if (lane == 0) red4[wave] = s4;
  if constexpr (FUSED) {
    if (wave < NW / 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = wave_sum(h == 0 ? lacc[q][erow] : 0.f);
        if (lane == 0) lred[wave][2 + q] = v;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 192) {
    float t = 0.f;
    for (int w = 0; w < NW; ++w) t += bred[w * 192 + threadIdx.x];
    if (threadIdx.x < 64) P[P_B3 + threadIdx.x] = t;
    else P[P_B2 + threadIdx.x - 64] = t;
  }
  if (threadIdx.x == 0) {
    float t4 = 0.f;
    for (int w = 0; w < NW; ++w) t4 += red4[w];
    P[P_B4] = t4;
  }
  if (threadIdx.x >= 192 && threadIdx.x < 202) {
    const int q = threadIdx.x - 192;
    float t = 0.f;
    if constexpr (FUSED) {
      if (q >= 2)
        for (int w = 0; w < NW / 2; ++w) t += lred[w][q];
      else if (blockIdx.x == 0)
        t = a.counts[q];     // global pooled counts (slot layout kept for the two-kernel path)
    }
    P[P_LOSS + q] = t;
  }
}

template <bool FUSED, int NW, int D>
static void launch_cbf_bwd(const CbfBwdArgs& a, int num_blocks, hipStream_t st) {
  const size_t lds = CbfCfg<NW>::LDS;
  (void)hipFuncSetAttribute((const void*)cbf_bwd_kernel<FUSED, NW, D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((cbf_bwd_kernel<FUSED, NW, D>), dim3(num_blocks), dim3(NW * 64), lds, st, a);
}

}  // namespace MB_PREC
}  // namespace mb

#include "cbf16.h"
// (A barrier-free variant with per-wave, register-resident weight gradients -- 4 waves, one per
// SIMD -- passed the oracle tests and lost 12.3 vs 10.2 ms: docs/PERF.md round 6, git history.)

extern "C" int MB_SYM(cbf_bwd)(const mb::CbfBwdArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (a->K > 16 || a->K < 1 || a->passes < 1 || a->passes > 2) return -1;
  if (a->rec) {   // 16x16x32 backward over cbf_compact's records (csrc/cbf16.h)
    if (a->fused || !a->nact || !a->wrm16 || !a->w16) return -5;
    if (a->dim == 3) launch_cbf_bwd16<3>(*a, num_blocks, st);
    else launch_cbf_bwd16<2>(*a, num_blocks, st);
    return (int)hipGetLastError();
  }
  if (a->fused && (a->passes != 2 || !a->dang || !a->counts)) return -2;
  if (a->src && (a->fused || !a->nev || a->passes != 2)) return -3;
  if (a->act && (!a->src || !a->nact)) return -4;
  if (a->dim == 3) {
    if (a->fused) launch_cbf_bwd<true, CBF_NW, 3>(*a, num_blocks, st);
    else launch_cbf_bwd<false, CBF_NW, 3>(*a, num_blocks, st);
  } else {
    if (a->fused) launch_cbf_bwd<true, CBF_NW, 2>(*a, num_blocks, st);
    else launch_cbf_bwd<false, CBF_NW, 2>(*a, num_blocks, st);
  }
  return (int)hipGetLastError();
}

extern "C" int MB_SYM(cbf_hfwd)(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  using namespace mb::MB_PREC;
  if (a->K > 16 || a->K < 1) return -1;
  if (!a->src || !a->nev || !a->idx1 || !a->h_out || !a->mask_out || !a->wrm) return -2;
  if (a->dim == 3) {
    (void)hipFuncSetAttribute((const void*)cbf_hfwd_kernel<HFWD_WAVES, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)HFWD_LDS);
    hipLaunchKernelGGL((cbf_hfwd_kernel<HFWD_WAVES, 3>), dim3(num_blocks), dim3(HFWD_WAVES * 64), HFWD_LDS, st, *a);
  } else {
    (void)hipFuncSetAttribute((const void*)cbf_hfwd_kernel<HFWD_WAVES, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)HFWD_LDS);
    hipLaunchKernelGGL((cbf_hfwd_kernel<HFWD_WAVES, 2>), dim3(num_blocks), dim3(HFWD_WAVES * 64), HFWD_LDS, st, *a);
  }
  return (int)hipGetLastError();
}
