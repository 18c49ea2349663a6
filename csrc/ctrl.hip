// Controller kernels (reference controller.py:31-63 + the Euler step of train.py:70), gfx950.
//
// A wave owns 32 agents. Edge phase: 16 tiles of 32 edges = 2 agents x 16 neighbour slots
// (K <= 16 real, the rest masked). Per tile:
//   F   (B operand, built in registers): [dx dy dvx dvy eye 1] hi-bf16 in lanes 0-31, the
//       bf16 residuals (x - bf16(x)) in lanes 32-63 -> layer 1 sees ~fp32 inputs for free
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
#include "common.h"
#include "args.h"

namespace mb {

constexpr int PSTR = 136;            // pooled-image row stride (bf16): 128 + 8 pad, 272 B
constexpr int CTRL_FWD_FRAGS = 72;   // ew1f 2 + ew2 16 | nw1f 18 + nw2 16 + nw3 16 + nw4 4
constexpr int CTRL_VEC = 352;        // eb2 128 | nb2 128 | nb3 64 | nb4 32 (padded)


DEV bf16x8 ctrl_edge_frag(float4 rel, float eye, bool ok, int h) {
  bf16x8 f;
  bf16 hx, lx, hy, ly, hvx, lvx, hvy, lvy;
  split_bf16(rel.x, hx, lx);
  split_bf16(rel.y, hy, ly);
  split_bf16(rel.z, hvx, lvx);
  split_bf16(rel.w, hvy, lvy);
  const bf16 z = (bf16)0.f;
  if (!ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = z;
    return f;
  }
  if (h == 0) {
    f[0] = hx; f[1] = hy; f[2] = hvx; f[3] = hvy; f[4] = (bf16)eye; f[5] = (bf16)1.f; f[6] = z; f[7] = z;
  } else {
    f[0] = lx; f[1] = ly; f[2] = lvx; f[3] = lvy; f[4] = z; f[5] = z; f[6] = z; f[7] = z;
  }
  return f;
}

DEV bf16x8 node_state_frag(float ex, float ey, float vx, float vy, bool ok, int h) {
  bf16x8 f;
  bf16 a0, a1, b0, b1, c0, c1, d0, d1;
  split_bf16(ex, a0, a1);
  split_bf16(ey, b0, b1);
  split_bf16(vx, c0, c1);
  split_bf16(vy, d0, d1);
  const bf16 z = (bf16)0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = z;
  if (!ok) return f;
  if (h == 0) { f[0] = a0; f[1] = b0; f[2] = c0; f[3] = d0; f[4] = (bf16)1.f; }
  else        { f[0] = a1; f[1] = b1; f[2] = c1; f[3] = d1; }
  return f;
}

// One edge tile in the transposed orientation: returns Z^T (4 column tiles) for 32 edges.
DEV void ctrl_edge_tile(const bf16x8& F, const bf16* wl, const float* eb2, int lane, f32x16 (&Z)[4]) {
  const int r = lane & 31;
  f32x16 H1[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    H1[mt] = mfma(frag_ld(wl, mt, lane), F, zero16());
    relu_(H1[mt]);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const float bv = eb2[32 * nt + r];
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = bv;
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      z = mfma(acc_frag<kk & 1>(H1[kk >> 1]), frag_ld(wl, 2 + nt * 4 + kk, lane), z);
    });
    Z[nt] = z;
  }
}

// node MLP forward for 32 agents; returns Y4 (rows 0..3 = the 4 gain pre-activations)
struct NodeActs { f32x16 Y1[2], Y2[4], Y3[2], Y4; };

DEV void node_forward(const bf16* pool, const bf16x8& sfrag, const bf16* wn, const float* nb2,
                      const float* nb3, const float* nb4, int lane, NodeActs& o) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x16 c = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const bf16x8 p = *reinterpret_cast<const bf16x8*>(pool + r * PSTR + 16 * kk + 8 * h);
      c = mfma(frag_ld(wn, mt * 9 + kk, lane), p, c);
    }
    c = mfma(frag_ld(wn, mt * 9 + 8, lane), sfrag, c);
    relu_(c);
    o.Y1[mt] = c;
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    f32x16 c = bias_rows(nb2, 32 * mt, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mfma(frag_ld(wn, 18 + mt * 4 + kk, lane), acc_frag<kk & 1>(o.Y1[kk >> 1]), c);
    });
    relu_(c);
    o.Y2[mt] = c;
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    f32x16 c = bias_rows(nb3, 32 * mt, h);
    static_for<8>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mfma(frag_ld(wn, 34 + mt * 8 + kk, lane), acc_frag<kk & 1>(o.Y2[kk >> 1]), c);
    });
    relu_(c);
    o.Y3[mt] = c;
  }
  {
    f32x16 c = bias_rows(nb4, 0, h);
    static_for<4>([&](auto kk_) {
      constexpr int kk = decltype(kk_)::value;
      c = mfma(frag_ld(wn, 50 + kk, lane), acc_frag<kk & 1>(o.Y3[kk >> 1]), c);
    });
    o.Y4 = c;
  }
}

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void ctrl_fwd_kernel(CtrlArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* wl = reinterpret_cast<bf16*>(smem);                            // ew1f, ew2 (18 frags)
  bf16* wn = wl + 18 * 512;                                            // nw1f..nw4 (54 frags)
  float* vl = reinterpret_cast<float*>(smem + CTRL_FWD_FRAGS * FRAG_BYTES);
  bf16* pools = reinterpret_cast<bf16*>(smem + CTRL_FWD_FRAGS * FRAG_BYTES + CTRL_VEC * 4);
  block_copy16(wl, a.wpack + (size_t)a.f_edge * 512, 18 * FRAG_BYTES);
  block_copy16(wn, a.wpack + (size_t)a.f_node * 512, 54 * FRAG_BYTES);
  block_copy16(vl, a.wvec, CTRL_VEC * 4);
  __syncthreads();
  const float* eb2 = vl;
  const float* nb2 = vl + 128;
  const float* nb3 = vl + 256;
  const float* nb4 = vl + 320;

  const int wave = threadIdx.x / WAVE, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  bf16* pool = pools + wave * 32 * PSTR;
  const int N = a.N, K = a.K;
  const int total = a.B * N;

  for (int grp = blockIdx.x * WAVES + wave; grp * 32 < total; grp += gridDim.x * WAVES) {
    const int g0 = grp * 32;
    // ---------------- edge phase: 16 tiles x (2 agents x 16 slots)
    for (int q = 0; q < 16; ++q) {
      const int al = 2 * q + (r >> 4);
      const int slot = r & 15;
      const int gi = g0 + al;
      const bool ok = (gi < total) && (slot < K);
      float4 rel = make_float4(0.f, 0.f, 0.f, 0.f);
      float eye = 0.f;
      bool m = false;
      if (ok) {
        const int b = gi / N, i = gi - b * N;
        const int j = a.idx[(long)b * a.i_env + (long)i * K + slot];
        const float4 si = a.S[(long)b * a.s_env + i];
        const float4 sj = a.S[(long)b * a.s_env + j];
        rel = make_float4(si.x - sj.x, si.y - sj.y, si.z - sj.z, si.w - sj.w);
        eye = (j == i) ? 1.f : 0.f;
        // strict < on the un-eps'd norm (controller.py:38-39)
        m = sqrtf(rel.x * rel.x + rel.y * rel.y) < a.obs_r;
      }
      const bf16x8 F = ctrl_edge_frag(rel, eye, ok, h);
      f32x16 Z[4];
      ctrl_edge_tile(F, wl + opaque_zero(), eb2, lane, Z);
      const unsigned mask32 = (unsigned)(__ballot(m) & 0xffffffffull);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        float p0 = 0.f, p1 = 0.f;
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) {
          const int e = acc_row(reg, h);
          const float v = ((mask32 >> e) & 1u) ? fmaxf(Z[nt][reg], 0.f) : 0.f;
          p0 = fmaxf(p0, v);
        }
#pragma unroll
        for (int reg = 8; reg < 16; ++reg) {
          const int e = acc_row(reg, h);
          const float v = ((mask32 >> e) & 1u) ? fmaxf(Z[nt][reg], 0.f) : 0.f;
          p1 = fmaxf(p1, v);
        }
        p0 = fmaxf(p0, shfl_xor32(p0));
        p1 = fmaxf(p1, shfl_xor32(p1));
        const int arow = 2 * q + h;   // h==0 writes agent 2q, h==1 agent 2q+1
        pool[arow * PSTR + 32 * nt + r] = (bf16)(h == 0 ? p0 : p1);
      }
    }
    lds_wave_sync();
    // ---------------- node phase: lane column r = agent g0 + r
    const int gi = g0 + r;
    const bool ok = gi < total;
    int b = 0, i = 0;
    float4 si = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 gg = make_float2(0.f, 0.f);
    if (ok) {
      b = gi / N; i = gi - b * N;
      si = a.S[(long)b * a.s_env + i];
      gg = a.G[(long)b * N + i];
    }
    const float ex = si.x - gg.x, ey = si.y - gg.y;
    const bf16x8 sf = node_state_frag(ex, ey, si.z, si.w, ok, h);
    NodeActs na;
    node_forward(pool, sf, wn + opaque_zero(), nb2, nb3, nb4, lane, na);
    float dsum = 0.f, asum = 0.f;
    if (ok && h == 0) {
      const float k0 = 2.f / (1.f + __expf(-na.Y4[0])) + 0.2f;
      const float k1 = 2.f / (1.f + __expf(-na.Y4[1])) + 0.2f;
      const float k2 = 2.f / (1.f + __expf(-na.Y4[2])) + 0.2f;
      const float k3 = 2.f / (1.f + __expf(-na.Y4[3])) + 0.2f;
      float ax = -(k0 * ex + k1 * si.z);
      float ay = -(k2 * ey + k3 * si.w);
      if (a.noise) {
        const float2 nz = a.noise[(long)b * a.n_env + i];
        ax += nz.x;
        ay += nz.y;
      }
      if (a.A) a.A[(long)b * a.a_env + i] = make_float2(ax, ay);
      const float4 sn = make_float4(si.x + si.z * a.dt, si.y + si.w * a.dt, si.z + ax * a.dt, si.w + ay * a.dt);
      if (a.Snext) a.Snext[(long)b * a.sn_env + i] = sn;
      const float dx = sn.x - gg.x, dy = sn.y - gg.y;
      dsum = sqrtf(dx * dx + dy * dy);
      const float rx = -(ex + a.sqrt3 * si.z), ry = -(ey + a.sqrt3 * si.w);
      asum = fabsf((ax * ax + ay * ay) - (rx * rx + ry * ry));
    }
    // per-env sums: one atomic per wave when its 32 agents share an env
    const int last = min(g0 + 31, total - 1);
    if (g0 / N == last / N) {
      dsum = wave_sum(dsum);
      asum = wave_sum(asum);
      if (lane == 0) {
        const int be = g0 / N;
        if (a.dist_sum) atomicAdd(a.dist_sum + (long)be * a.d_env, dsum);
        if (a.act_sum) atomicAdd(a.act_sum + (long)be * a.ac_env, asum);
      }
    } else if (ok && h == 0) {
      if (a.dist_sum) atomicAdd(a.dist_sum + (long)b * a.d_env, dsum);
      if (a.act_sum) atomicAdd(a.act_sum + (long)b * a.ac_env, asum);
    }
    // the pool image is rewritten by the next group: finish all reads first
    lds_wave_sync();
  }
}

constexpr int CTRL_WAVES = 8;

size_t ctrl_fwd_lds() {
  return (size_t)CTRL_FWD_FRAGS * FRAG_BYTES + CTRL_VEC * 4 + (size_t)CTRL_WAVES * 32 * PSTR * 2;
}

}  // namespace mb

extern "C" int mb_ctrl_fwd(const mb::CtrlArgs* a, int num_cu, hipStream_t st) {
  using namespace mb;
  if (a->K > 16 || a->K < 1) return -1;
  const int groups = (a->B * a->N + 31) / 32;
  int blocks = (groups + CTRL_WAVES - 1) / CTRL_WAVES;
  const int maxb = num_cu > 0 ? num_cu * 2 : blocks;
  if (blocks > maxb) blocks = maxb;
  const size_t lds = ctrl_fwd_lds();
  (void)hipFuncSetAttribute((const void*)ctrl_fwd_kernel<CTRL_WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(ctrl_fwd_kernel<CTRL_WAVES>, dim3(blocks), dim3(CTRL_WAVES * 64), lds, st, *a);
  return (int)hipGetLastError();
}
