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

namespace mb {

constexpr int CBF_FWD_FRAGS = 34;  // w1f 2 + w2 16 + w3 16
constexpr int CBF_VEC = 260;       // b2 128 | b3 64 | w4 64 | b4 1 (+3 pad)



DEV bf16x8 cbf_edge_frag(float4 rel, float eye, float dfeat, bool ok, int h) {
  bf16x8 f;
  const bf16 z = (bf16)0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = z;
  if (!ok) return f;
  bf16 hx, lx, hy, ly, hvx, lvx, hvy, lvy, hd, ld;
  split_bf16(rel.x, hx, lx);
  split_bf16(rel.y, hy, ly);
  split_bf16(rel.z, hvx, lvx);
  split_bf16(rel.w, hvy, lvy);
  split_bf16(dfeat, hd, ld);
  if (h == 0) {
    f[0] = hx; f[1] = hy; f[2] = hvx; f[3] = hvy; f[4] = (bf16)eye; f[5] = hd; f[6] = (bf16)1.f;
  } else {
    f[0] = lx; f[1] = ly; f[2] = lvx; f[3] = lvy; f[5] = ld;
  }
  return f;
}

struct CbfActs { f32x16 H1[2], H2[4], H3[2]; };

// full forward for one 32-edge tile; returns the pre-mask head output for this lane's edge
DEV float cbf_mlp(const bf16x8& F, const bf16* wl, const float* vl, int lane, CbfActs& o) {
  const int h = lane >> 5;
  const float* b2 = vl;
  const float* b3 = vl + 128;
  const float* w4 = vl + 192;
  const float b4 = vl[256];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    o.H1[mt] = mfma(frag_ld(wl, mt, lane), F, zero16());
    relu_(o.H1[mt]);
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    f32x16 c = bias_rows(b2, 32 * mt, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mfma(frag_ld(wl, 2 + mt * 4 + kk, lane), acc_frag<kk & 1>(o.H1[kk >> 1]), c);
    });
    relu_(c);
    o.H2[mt] = c;
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x16 c = bias_rows(b3, 32 * mt, h);
    static_for<8>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mfma(frag_ld(wl, 18 + mt * 8 + kk, lane), acc_frag<kk & 1>(o.H2[kk >> 1]), c);
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

struct EdgeCtx {
  bool ok;
  int b, t, i, j;
  float4 rel;
  float eye, d, dfeat;
  bool mask;
};

DEV void cbf_edge(const float4* S, long s_env, long s_step, const int* idx, int T, int N, int K,
                  long e, long E, int tstep_off, float obs_r, float dist_thr, float dist_eps, EdgeCtx& c) {
  c.ok = e < E;
  c.rel = make_float4(0.f, 0.f, 0.f, 0.f);
  c.eye = 0.f; c.d = 0.f; c.dfeat = 0.f; c.mask = false;
  c.b = c.t = c.i = c.j = 0;
  if (!c.ok) return;
  const long NK = (long)N * K;
  const long bt = e / NK;
  const long rem = e - bt * NK;
  c.i = (int)(rem / K);
  c.b = (int)(bt / T);
  c.t = (int)(bt - (long)c.b * T);
  c.j = idx[e];
  const float4* Sb = S + (long)c.b * s_env + (long)(c.t + tstep_off) * s_step;
  const float4 si = Sb[c.i];
  const float4 sj = Sb[c.j];
  c.rel = make_float4(si.x - sj.x, si.y - sj.y, si.z - sj.z, si.w - sj.w);
  c.eye = (c.j == c.i) ? 1.f : 0.f;
  c.d = sqrtf(c.rel.x * c.rel.x + c.rel.y * c.rel.y + dist_eps);
  c.dfeat = c.d - dist_thr;
  c.mask = c.d <= obs_r;
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void cbf_fwd_kernel(CbfFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* wl = reinterpret_cast<bf16*>(smem);
  float* vl = reinterpret_cast<float*>(smem + CBF_FWD_FRAGS * FRAG_BYTES);
  __shared__ float red[10][WAVES];
  block_copy16(wl, a.wpack + (size_t)a.f_fwd * 512, CBF_FWD_FRAGS * FRAG_BYTES);
  block_copy16(vl, a.wvec, CBF_VEC * 4);
  __syncthreads();
  const int wave = threadIdx.x / WAVE, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const long E = (long)a.B * a.T * a.N * a.K;
  const long ntiles = (E + 31) / 32;
  float nd = 0.f, ns = 0.f;
  if (a.dh_out) { nd = 1e-5f + a.counts[0]; ns = 1e-5f + a.counts[1]; }
  float acc[10];
#pragma unroll
  for (int q = 0; q < 10; ++q) acc[q] = 0.f;
  CbfActs act;
  for (long tile = (long)blockIdx.x * WAVES + wave; tile < ntiles; tile += (long)gridDim.x * WAVES) {
    const long e = tile * 32 + r;
    EdgeCtx c0;
    float hv = 0.f, hnv = 0.f;
    bool mask1 = false;
#pragma unroll 1
    for (int pass = 0; pass < 1 + a.two; ++pass) {
      const bf16* wt = wl + opaque_zero();
      const float* vt = vl + opaque_zero();
      EdgeCtx c;
      cbf_edge(a.S, a.s_env, a.s_step, a.idx, a.T, a.N, a.K, e, E, pass, a.obs_r, a.dist_thr, a.dist_eps, c);
      const float hp = cbf_mlp(cbf_edge_frag(c.rel, c.eye, c.dfeat, c.ok, h), wt, vt, lane, act);
      if (pass == 0) { c0 = c; hv = c.mask ? hp : 0.f; }
      else { hnv = c.mask ? hp : 0.f; mask1 = c.mask; }
    }
    if (!c0.ok || h != 0) continue;
    if (a.h_out) a.h_out[e] = hv;
    if (a.hn_out) a.hn_out[e] = hnv;
    const bool vld = a.valid ? (a.valid[(long)c0.b * a.T + c0.t] != 0) : true;
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
          const float c = a.lc.scale / nd;
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
          const float c = a.lc.scale / ns;
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

}  // namespace mb

extern "C" int mb_cbf_fwd(const mb::CbfFwdArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  if (a->K > 16 || a->K < 1) return -1;
  const size_t lds = (size_t)CBF_FWD_FRAGS * FRAG_BYTES + CBF_VEC * 4;
  (void)hipFuncSetAttribute((const void*)cbf_fwd_kernel<CBF_FWD_WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(cbf_fwd_kernel<CBF_FWD_WAVES>, dim3(num_blocks), dim3(CBF_FWD_WAVES * 64), lds, st, *a);
  return (int)hipGetLastError();
}
