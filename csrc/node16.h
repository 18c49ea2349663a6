// 16x16x32 controller NODE backward: the fp32-accurate x3 BPTT node step at TWO waves per SIMD, and
// the same kernel in the 1-pass bf16 / fp16 builds (hi planes only, one MFMA per product).
//
// Same math as node_bwd_body (ctrl.hip) -- per agent of the step: node MLP recompute
// Y1 = relu(W1 [P; s]), Y2 = relu(W2 Y1 + b2), Y3 = relu(W3 Y2 + b3), y4 = W4 Y3 + b4; gain law
// + action-loss backward (dA = dt G_{t+1}[v] + action-loss grad) -> d4 and the ego terms;
// dY3 = W4^T d4 . relu'(Y3), dY2 = W3^T dY3 . relu'(Y2), dY1 = W2^T dY2 . relu'(Y1),
// [dL/dpooled; d/ds] = W1^T dY1; weight gradients dW4 / dW3 / dW2 / dW1f (+ biases) summed over the
// agents. node_bwd_body keeps 32 agents per wave in 32x32 tiles (444 registers: one wave per SIMD,
// ~19 % of its issue bound, its stage turns behind barriers with nothing to hide them). Here a wave
// owns 16 agents (columns n = lane & 15) and every tile is a v_mfma_f32_16x16x32_bf16 tile
// (csrc/mfma16.h), so the data path fits 256 registers and an 8-wave workgroup (128 agents per
// chunk) runs two waves per SIMD.
//
// Weights: column-permuted row-major images (layout.node_rm16), hi plane then lo plane, in LDS
// (125 KB): A = W is one 16-byte read per plane, A = W^T two ds_read_b64_tr_b16 per plane (the
// cbf16.h scheme); W1's columns stay in natural order (its forward B operand is the pooled row as
// stored by the rollout, natural k).
// Weight gradients: three stages (dW3 + dW4 | dW2 | dW1f), each in four turns of 32 agent rows
// (the rows of two waves) through one 34 KB region: the owners store their rows, every wave
// contracts one 32-agent K-step into the tiles it owns (fixed owners: deterministic).
// Reference op: /root/reference/controller.py:23-29,47-61 (the decentralised node MLP and the
// gain-scheduled PD law), differentiated through the rollout by /root/reference/train.py:103.
#pragma once
#include "mfma16.h"

namespace mb {
namespace MB_PREC {

// dL/dpooled stores: lanes g / g^1 swap one tile's values (permlane16) so every lane stores 16 B
// hi + 16 B lo of 8 consecutive features, instead of 8 B of 4 from each tile (default since round 5:
// dP phase 11.9 -> 5.5 k cycles per chunk, headline 10.649-10.658 -> 10.602-10.636 ms fp32, 6.732-6.742
// -> 6.705-6.724 bf16, interleaved, profiles/r5_b7/; 0 = the 8-byte stores)
constexpr bool N16_DP_PAIRED = true;
constexpr bool N16_DIAG_NOSTORE = (MB_DIAG & 4) != 0;   // diagnostics build only: skip the dL/dpooled stores
constexpr int N16_NW = 8, N16_CH = 16 * N16_NW;           // waves, agents per chunk
constexpr int N16_S1 = 176, N16_S2 = 80, N16_S3 = 144, N16_S4 = 80;   // layout.NODE16_STRIDES (bank model)
constexpr int N16_O2 = 64 * N16_S1, N16_O3 = N16_O2 + 128 * N16_S2, N16_O4 = N16_O3 + 64 * N16_S3;
constexpr int N16_RM = N16_O4 + 16 * N16_S4;              // elements per plane (lo plane at +N16_RM)
constexpr int N16_VEC = 224;                              // nb2 128 | nb3 64 | nb4 32 (ctrl_v[128:352])
constexpr int N16_RT = 32, N16_SW = 272;                  // stage: rows per turn, row stride (elements)
constexpr int N16_PL = N16_RT * N16_SW;                   // lo-plane offset of the stage region
// stage columns. 1: [dY3 0..63 | d4 64..79 | Y3 80..143 | Y2 144..271]  2: [dY2 0..127 | Y1 128..191]
//                 3: [dY1 0..63 | P 64..191 | s 192..207 | 0 208..223]
constexpr int N16_C_D4 = 64, N16_C_Y3 = 80, N16_C_Y2 = 144, N16_C_Y1 = 128, N16_C_P = 64, N16_C_S = 192;
constexpr int N16_PLANES = X3 ? 2 : 1;
constexpr size_t N16_LDS_W = (size_t)N16_PLANES * N16_RM * 2;   // weight images, hi [+ lo]
constexpr size_t N16_LDS = N16_LDS_W + N16_VEC * 4 + (size_t)N16_PLANES * N16_PL * 2;
// tile-major slab (floats): 32 dW2 tiles | 32 dW3 tiles | 8 x 5 dW1f tile slots | 4 dW4 tiles | b2 | b3 | b4
constexpr int N16_SL_W2 = 0, N16_SL_W3 = 32 * 256, N16_SL_W1 = 64 * 256, N16_SL_W4 = 104 * 256;
constexpr int N16_SL_B2 = 108 * 256, N16_SL_B3 = N16_SL_B2 + 128, N16_SL_B4 = N16_SL_B3 + 64;
static_assert(N16_SL_B4 + 16 <= CTRL_NODE_PARTIAL, "slab row");
static_assert(N16_LDS <= 160 * 1024, "LDS budget");
static_assert(N16_C_S + 32 <= N16_SW && N16_C_Y2 + 128 <= N16_SW, "stage columns");

// A = W rows m0..m0+15, K-step s: one 16-byte read per plane (columns as stored)
DEV Fr n16_w(const h16* W, int stride, int m0, int s, int lane) {
  const h16* p = W + (m0 + (lane & 15)) * stride + 32 * s + 8 * (lane >> 4);
  Fr r;
  r.h = *reinterpret_cast<const h16x8*>(p);
  if constexpr (X3) r.l = *reinterpret_cast<const h16x8*>(p + N16_RM);
  return r;
}
// A = W^T of a column-permuted image (W2 / W3 / W4): rows = logical columns m0.., K-step s over
// W's rows in accumulator order (the B operand is a packed C-tile pair)
DEV Fr n16_wT_perm(const h16* W, int stride, int m0, int s, int lane) {
  const int g = lane >> 4, p = lane & 3;
  const int colp = 32 * (m0 >> 5) + 4 * ((m0 >> 4) & 1) + 8 * p;
  Fr r;
  r.h = tr_pair16(W, stride, 32 * s + 4 * g, 16, colp, lane);
  if constexpr (X3) r.l = tr_pair16(W + N16_RM, stride, 32 * s + 4 * g, 16, colp, lane);
  return r;
}
// A = W4^T (16 real rows: K-step elements j >= 4 would be rows 16..31, past the image): one
// ds_read_b64_tr_b16 per plane, elements 4..7 zero
DEV Fr n16_w4T(const h16* W, int m0, int lane) {
  const int g = lane >> 4, p = lane & 3, q = (lane & 15) >> 2;
  const int colp = 32 * (m0 >> 5) + 4 * ((m0 >> 4) & 1) + 8 * p;
  Fr r;
#pragma unroll
  for (int pl = 0; pl < N16_PLANES; ++pl) {
    const LDS_AS h16* a1 = lds_ptr(W + pl * N16_RM) + (4 * g + q) * N16_S4 + colp;
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
    const h16x4 b4 = __builtin_bit_cast(h16x4, v);
    h16x8 f;
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[j] = b4[j]; f[4 + j] = (h16)0.f; }
    if (pl == 0) r.h = f; else r.l = f;
  }
  return r;
}
DEV f32x4 bias4n(const float* b, int row0, int g) {
  const float4 v = *reinterpret_cast<const float4*>(b + row0 + 4 * g);
  return f32x4{v.x, v.y, v.z, v.w};
}
// A = W1^T (natural columns): rows = W1 columns m0.., K-step s over W1's rows in accumulator order
DEV Fr n16_w1T(const h16* W, int m0, int s, int lane) {
  const int g = lane >> 4, p = lane & 3;
  Fr r;
  r.h = tr_pair16(W, N16_S1, 32 * s + 4 * g, 16, m0 + 4 * p, lane);
  if constexpr (X3) r.l = tr_pair16(W + N16_RM, N16_S1, 32 * s + 4 * g, 16, m0 + 4 * p, lane);
  return r;
}

// ST: phase clocks (diagnostics) in a separate instantiation (no runtime stamp branches in the
// production kernel: see cbf16.h)
template <int D, bool ST>
__global__ __launch_bounds__(N16_NW * 64) void ctrl_node_bwd16_kernel(CtrlNodeBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* W1 = reinterpret_cast<h16*>(smem);
  float* vl = reinterpret_cast<float*>(smem + N16_LDS_W);
  h16* stg = reinterpret_cast<h16*>(smem + N16_LDS_W + N16_VEC * 4);
  // diagnostics: shader clock at the phase boundaries (a.stamps, normally null; [workgroup][wave][16],
  // a workgroup with several chunks keeps its last chunk's clocks; scripts/stamps_node.py --node16)
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if ((threadIdx.x & 63) == 0) a.stamps[((long)blockIdx.x * N16_NW + threadIdx.x / WAVE) * 16 + k] = t;
    }
  };
  stamp(0);
  block_copy16(W1, a.wrm16, (int)N16_LDS_W, false);
  block_copy16(vl, a.wvec + 128, N16_VEC * 4);
  __syncthreads();
  stamp(1);
  const float* nb2 = vl;
  const float* nb3 = vl + 128;
  const float* nb4 = vl + 192;
  const int wave = wave_id(), lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
  const int N = a.N;
  const int total = a.B * N;
  const long nchunks = (total + N16_CH - 1) / N16_CH;
  h16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (h16)1.f;

  // owned weight-gradient tiles (16x16; rows = output units, columns = input units):
  //   dW2 (128 x 64): M-tile `wave`, N-tiles 0..3, db2 rows of M-tile `wave`
  //   dW3 (64 x 128): M-tile wave & 3, N-tiles 4 (wave >> 2) .. +3; db3 (waves 0..3)
  //   dW4 (16 x 64): waves 0..3, N-tile `wave`; db4 (wave 0)
  //   dW1f (64 x 160): M-tile wave & 3, N-tiles (wave >> 2) + 2v (v < 5, < 9: column tile 9 is
  //   padding, never read by the gradient map)
  const int m3 = wave & 3, n3 = 4 * (wave >> 2);
  const int m1 = wave & 3, n1 = wave >> 2;
  const int nv1 = n1 == 0 ? 5 : 4;
  f32x4 acc2[4], acc3[4], acc1[5], acc4 = zero4(), bias2 = zero4(), bias3 = zero4(), bias4_ = zero4();
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = acc3[u] = zero4();
#pragma unroll
  for (int u = 0; u < 5; ++u) acc1[u] = zero4();

  const int trow = (wave & 1) * 16 + n;        // this wave's rows inside its turn
  const int myturn = wave >> 1;

  for (long chunk = BPTT_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    stamp(15);
    const int ga = (int)(chunk * N16_CH) + wave * 16 + n;
    const bool ok = ga < total;
    // stage turns holding at least one valid agent (a partial chunk skips its empty turns)
    const int nturn = min(4, (int)((min((long)N16_CH, total - chunk * N16_CH) + N16_RT - 1) / N16_RT));
    // every load unconditional (a lane past the end reads agent 0) and issued before any use: a
    // load inside `if (ok)` waits at the branch merge, serialising this block, the pooled rows
    // and the combine's gathers (ctrl.hip ctrl_st_load)
    const int gac = ok ? ga : 0;
    const int b = gac / N, i = gac - b * N;
    float sp[D], sv[D], gg[D], av[D], gnp[D], gnv[D];
    load_rec<D>(a.S + (long)b * a.s_env * REC<D>, (unsigned)i, sp, sv);
#pragma unroll
    for (int q = 0; q < D; ++q) {
      gg[q] = a.G[((long)b * N + i) * D + q];
      av[q] = a.A[((long)b * a.a_env + i) * D + q];
      gnp[q] = gnv[q] = 0.f;
    }
    if (a.Gn && !a.cdS) load_rec<D>(a.Gn + (long)b * a.gn_env * REC<D>, (unsigned)i, gnp, gnv);
    const bool vld = ok && (a.valid ? (a.valid[(long)b * a.v_env] != 0) : true);
    const h16* prow = a.pooled + (long)b * a.p_env + (long)i * PROW;
    Fr Pf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) Pf[s] = row_fr(prow + 32 * s + 8 * g, 128);
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (!ok) Pf[s].h = Pf[s].l = zero_h8();
#pragma unroll
    for (int q = 0; q < D; ++q) {
      sp[q] = ok ? sp[q] : 0.f; sv[q] = ok ? sv[q] : 0.f;
      gg[q] = ok ? gg[q] : 0.f; av[q] = ok ? av[q] : 0.f;
      gnp[q] = ok ? gnp[q] : 0.f; gnv[q] = ok ? gnv[q] : 0.f;
    }
    // G_{t+1} (fused BPTT combine): lanes g = 0 / 1 split the agent's out- and in-edges exactly
    // as the 2-lane combine of the other node kernels (same terms, same order: bit-identical);
    // lanes g >= 2 join the lane exchange with zeros
    if (a.cdS) fused_combine<D, 16>(a, ok && g < 2, b, i, g & 1, gnp, gnv);
    stamp(2);
    float ex[D];
#pragma unroll
    for (int q = 0; q < D; ++q) ex[q] = sp[q] - gg[q];
    const h16x8 sfr = g < 2 ? node_state_frag<D>(ex, sv, ok, g) : zero_h8();
    // opaque bases: every weight fragment is re-read from LDS per chunk (loop-invariant loads
    // hoisted out of the chunk loop would pin registers and spill)
    const h16* W1c = W1 + opaque_zero();
    const h16* W2 = W1c + N16_O2;
    const h16* W3 = W1c + N16_O3;
    const h16* W4 = W1c + N16_O4;
    // ---- forward recompute
    Pk4 Y1[4], Y2[8], Y3[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 c = zero4();
#pragma unroll
      for (int s = 0; s < 4; ++s) c = mma16(n16_w(W1c, N16_S1, 16 * mt, s, lane), Pf[s], c);
      c = mma16_bx(n16_w(W1c, N16_S1, 16 * mt, 4, lane), sfr, c);
      Y1[mt] = to_pk4(relu4(c));
    }
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 c = bias4n(nb2, 16 * mt, g);
#pragma unroll
      for (int s = 0; s < 2; ++s) c = mma16(n16_w(W2, N16_S2, 16 * mt, s, lane), pk4_fr(Y1[2 * s], Y1[2 * s + 1]), c);
      Y2[mt] = to_pk4(relu4(c));
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 c = bias4n(nb3, 16 * mt, g);
#pragma unroll
      for (int s = 0; s < 4; ++s) c = mma16(n16_w(W3, N16_S3, 16 * mt, s, lane), pk4_fr(Y2[2 * s], Y2[2 * s + 1]), c);
      Y3[mt] = to_pk4(relu4(c));
    }
    f32x4 y4 = bias4n(nb4, 0, g);
#pragma unroll
    for (int s = 0; s < 2; ++s) y4 = mma16(n16_w(W4, N16_S4, 0, s, lane), pk4_fr(Y3[2 * s], Y3[2 * s + 1]), y4);
    stamp(3);
    // ---- gain law + action-loss backward on the g = 0 lane of each agent (rows 0..3 of y4 are its
    //      regs, rows 4..7 the regs of lane g = 1)
    float y4r[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) { y4r[q] = y4[q]; y4r[4 + q] = lane_xorf<16>(y4[q]); }
    float d4r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) d4r[q] = 0.f;
    float egp[D], egv[D];                         // dL/d(p - g), dL/dv of the ego terms
#pragma unroll
    for (int q = 0; q < D; ++q) { egp[q] = 0.f; egv[q] = 0.f; }
    if (ok && g == 0) {
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
    // back to the C layout: lane (n, g) reg q = d4 row 4g + q (rows >= 2D are zero)
    f32x4 d4c = zero4();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float hi4 = lane_xorf<16>(d4r[4 + q]);
      d4c[q] = g == 0 ? d4r[q] : (g == 1 ? hi4 : 0.f);
    }
    const Pk4 d4 = to_pk4(d4c);
    Pk4 zp;
    zp.h = zp.l = h16x4{(h16)0.f, (h16)0.f, (h16)0.f, (h16)0.f};
    // ---- dY3 = W4^T d4 . relu'(Y3) (K = 16 real rows: the pair's second tile is zero)
    Pk4 dY3[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const f32x4 c = mma16(n16_w4T(W4, 16 * mt, lane), pk4_fr(d4, zp), zero4());
      dY3[mt] = to_pk4(c);
      mask_pk4(dY3[mt], Y3[mt]);
    }
    stamp(4);
    // ---- stage 1: dW3 += dY3 . Y2^T, db3; dW4 += d4 . Y3^T, db4
#pragma unroll 1
    for (int turn = 0; turn < nturn; ++turn) {
      if (myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          store4(stg, N16_SW, N16_PL, trow, mt, g, dY3[mt]);
          store4(stg + N16_C_Y3, N16_SW, N16_PL, trow, mt, g, Y3[mt]);
        }
        store4(stg + N16_C_D4, N16_SW, N16_PL, trow, 0, g, d4);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) store4(stg + N16_C_Y2, N16_SW, N16_PL, trow, mt, g, Y2[mt]);
      }
      __syncthreads();
      {
        const Fr A = tr16_fr(stg, N16_SW, N16_PL, 0, 16 * m3, lane);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc3[u] = mma16(A, tr16_fr(stg + N16_C_Y2, N16_SW, N16_PL, 0, 16 * (n3 + u), lane), acc3[u]);
        if (wave < 4) {
          bias3 = mma16_bx(A, ones, bias3);
          const Fr A4 = tr16_fr(stg + N16_C_D4, N16_SW, N16_PL, 0, 0, lane);
          acc4 = mma16(A4, tr16_fr(stg + N16_C_Y3, N16_SW, N16_PL, 0, 16 * wave, lane), acc4);
          if (wave == 0) bias4_ = mma16_bx(A4, ones, bias4_);
        }
      }
      __syncthreads();
    }
    stamp(5);
    // ---- dY2 = W3^T dY3 . relu'(Y2); dY1 = W2^T dY2 . relu'(Y1)
    Pk4 dY2[8], dY1[4];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 c = zero4();
#pragma unroll
      for (int s = 0; s < 2; ++s) c = mma16(n16_wT_perm(W3, N16_S3, 16 * mt, s, lane), pk4_fr(dY3[2 * s], dY3[2 * s + 1]), c);
      dY2[mt] = to_pk4(c);
      mask_pk4(dY2[mt], Y2[mt]);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 c = zero4();
#pragma unroll
      for (int s = 0; s < 4; ++s) c = mma16(n16_wT_perm(W2, N16_S2, 16 * mt, s, lane), pk4_fr(dY2[2 * s], dY2[2 * s + 1]), c);
      dY1[mt] = to_pk4(c);
      mask_pk4(dY1[mt], Y1[mt]);
    }
    stamp(6);
    // the pooled rows for stage 3, requested now: their latency hides behind stage 2 (issued after
    // every store of this chunk so far, they wait for nothing else)
    h16x8 Ph[4], Pl[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      Ph[s] = ok ? *reinterpret_cast<const h16x8*>(prow + 32 * s + 8 * g) : zero_h8();
      if constexpr (X3) Pl[s] = ok ? *reinterpret_cast<const h16x8*>(prow + 128 + 32 * s + 8 * g) : zero_h8();
    }
    // ---- stage 2: dW2 += dY2 . Y1^T, db2
#pragma unroll 1
    for (int turn = 0; turn < nturn; ++turn) {
      if (myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) store4(stg, N16_SW, N16_PL, trow, mt, g, dY2[mt]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store4(stg + N16_C_Y1, N16_SW, N16_PL, trow, mt, g, Y1[mt]);
      }
      __syncthreads();
      {
        const Fr A = tr16_fr(stg, N16_SW, N16_PL, 0, 16 * wave, lane);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc2[u] = mma16(A, tr16_fr(stg + N16_C_Y1, N16_SW, N16_PL, 0, 16 * u, lane), acc2[u]);
        bias2 = mma16_bx(A, ones, bias2);
      }
      __syncthreads();
    }
    stamp(7);
    // ---- stage 3: dW1f += dY1 . [P | s]^T (P: the rows requested before stage 2)
#pragma unroll 1
    for (int turn = 0; turn < nturn; ++turn) {
      if (myturn == turn) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) store4(stg, N16_SW, N16_PL, trow, mt, g, dY1[mt]);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          *reinterpret_cast<h16x8*>(stg + trow * N16_SW + N16_C_P + 32 * s + 8 * g) = Ph[s];
          if constexpr (X3) *reinterpret_cast<h16x8*>(stg + N16_PL + trow * N16_SW + N16_C_P + 32 * s + 8 * g) = Pl[s];
        }
        if (g < 2) {      // the state fragment is exact: zero lo plane
          *reinterpret_cast<h16x8*>(stg + trow * N16_SW + N16_C_S + 8 * g) = sfr;
          if constexpr (X3) *reinterpret_cast<h16x8*>(stg + N16_PL + trow * N16_SW + N16_C_S + 8 * g) = zero_h8();
        }
      }
      __syncthreads();
      {
        const Fr A = tr16_fr(stg, N16_SW, N16_PL, 0, 16 * m1, lane);
#pragma unroll
        for (int v = 0; v < 5; ++v) {
          if (v < nv1) {
            const int nt = n1 + 2 * v;
            acc1[v] = mma16(A, tr16_fr(stg + N16_C_P, N16_SW, N16_PL, 0, 16 * nt, lane), acc1[v]);
          }
        }
      }
      __syncthreads();
    }
    stamp(8);
    // ---- [dL/dpooled; d/ds] = W1^T dY1: tiles 0..7 -> dP rows (hi | lo), tile 8 -> ego terms
    f32x4 dpair = zero4();
    // tiles in pairs: two independent MFMA chains per step, the next pair's W1^T reads issued
    // while the current pair's chains run (one tile at a time left the LDS latency and the
    // dependent 6-MFMA chain exposed nine times: 13.7 k cycles per chunk, profiles/r4_validate/)
#pragma unroll
    for (int mt = 0; mt < 9; ++mt) {
      f32x4 c = zero4();
      if (mt % 2 == 0 && mt + 1 < 9) {
        f32x4 c1 = zero4();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const Fr B = pk4_fr(dY1[2 * s], dY1[2 * s + 1]);
          c = mma16(n16_w1T(W1c, 16 * mt, s, lane), B, c);
          c1 = mma16(n16_w1T(W1c, 16 * (mt + 1), s, lane), B, c1);
        }
        dpair = c1;
      } else if (mt % 2 == 1) {
        c = dpair;
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) c = mma16(n16_w1T(W1c, 16 * mt, s, lane), pk4_fr(dY1[2 * s], dY1[2 * s + 1]), c);
      }
      if (mt < 8) {
        if constexpr (N16_DP_PAIRED) {
          // tile pair (mt, mt + 1): lanes g and g ^ 1 swap one tile's 4 features, so every lane holds
          // 8 consecutive ones -- g even: 16 mt + 4g .. +7, g odd: 16 (mt + 1) + 4 (g - 1) .. +7 --
          // and stores 16 B per plane (a row gets 64 contiguous bytes per store, not 32)
          if (mt % 2 == 0) {
            const Pk4 va = to_pk4(c), vb = to_pk4(dpair);
            const bool odd = (g & 1) != 0;
            const Pk4 sd = odd ? va : vb;
            Pk4 rv;
            {
              const u32x2v sh = __builtin_bit_cast(u32x2v, sd.h);
              rv.h = __builtin_bit_cast(h16x4, u32x2v{lane_xor<16>(sh[0]), lane_xor<16>(sh[1])});
              if constexpr (X3) {
                const u32x2v sl = __builtin_bit_cast(u32x2v, sd.l);
                rv.l = __builtin_bit_cast(h16x4, u32x2v{lane_xor<16>(sl[0]), lane_xor<16>(sl[1])});
              }
            }
            const Pk4& lo4 = odd ? rv : va;          // features +0..3 of the 8
            const Pk4& hi4 = odd ? vb : rv;          // features +4..7
            if (ok && !N16_DIAG_NOSTORE) {
              h16* drow = a.dP + (long)b * a.dp_env + (long)i * PROW + (odd ? 16 * (mt + 1) + 4 * (g - 1) : 16 * mt + 4 * g);
              h16x8 oh;
#pragma unroll
              for (int q = 0; q < 4; ++q) { oh[q] = lo4.h[q]; oh[4 + q] = hi4.h[q]; }
              *reinterpret_cast<h16x8*>(drow) = oh;
              if constexpr (X3) {
                h16x8 ol;
#pragma unroll
                for (int q = 0; q < 4; ++q) { ol[q] = lo4.l[q]; ol[4 + q] = hi4.l[q]; }
                *reinterpret_cast<h16x8*>(drow + 128) = ol;
              }
            }
          }
        } else if (ok && !N16_DIAG_NOSTORE) {
          h16* drow = a.dP + (long)b * a.dp_env + (long)i * PROW + 16 * mt + 4 * g;
          const Pk4 v = to_pk4(c);
          *reinterpret_cast<h16x4*>(drow) = v.h;
          if constexpr (X3) *reinterpret_cast<h16x4*>(drow + 128) = v.l;
        }
        if (mt == 3) stamp(10);                // diagnostics: dP tiles 0..3 done
        if (mt == 7) stamp(11);                // tiles 4..7 done
      } else {
        // rows 128 + 4g + q: the state slots [p - g, v] (hi: slots 0..2D-1; lane g = 0 holds rows
        // 0..3, lane g = 1 rows 4..7)
        float er[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) { er[q] = c[q]; er[4 + q] = lane_xorf<16>(c[q]); }
        if (ok && g == 0 && a.ego) {
#pragma unroll
          for (int q = 0; q < D; ++q) { egp[q] += er[q]; egv[q] += er[D + q]; }
          store_rec<D>(a.ego + (long)b * N * REC<D>, (unsigned)i, egp, egv);
        }
      }
    }
    stamp(9);
  }
  stamp(13);
  // ---- slab: TILE-MAJOR (layout.ctrl_node16_grad_map): every owned 16x16 tile is 64 lanes x 4
  //      floats, one 16-byte load + store per lane (the row-major layout of the other node kernels
  //      costs 4 scattered 64-byte segments per wave instruction: 22 k cycles of a 170 k call).
  //      Owned elements are read first, then added and stored; the first BPTT step writes.
  //      [dW2: wave x 4 tiles | dW3: wave x 4 | dW1f: wave x 5 slots | dW4: waves 0..3 | biases]
  float4* P4 = reinterpret_cast<float4*>(a.partial + (long)blockIdx.x * CTRL_NODE_PARTIAL);
  float* P = a.partial + (long)blockIdx.x * CTRL_NODE_PARTIAL;
  const bool accum = !a.init;
  const int t2 = N16_SL_W2 / 256 + wave * 4, t3 = N16_SL_W3 / 256 + wave * 4, t1 = N16_SL_W1 / 256 + wave * 5;
  float4 o2[4], o3[4], o1[5], o4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    o2[u] = accum ? P4[(t2 + u) * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    o3[u] = accum ? P4[(t3 + u) * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int v = 0; v < 5; ++v) o1[v] = (accum && v < nv1) ? P4[(t1 + v) * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  if (accum && wave < 4) o4 = P4[(N16_SL_W4 / 256 + wave) * 64 + lane];
  float ob[3] = {0.f, 0.f, 0.f};          // bias rows (n == 0 lanes): b2 | b3 | b4, 4 per lane
  auto add4 = [](const float4& o, const f32x4& c) { return make_float4(o.x + c[0], o.y + c[1], o.z + c[2], o.w + c[3]); };
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    P4[(t2 + u) * 64 + lane] = add4(o2[u], acc2[u]);
    P4[(t3 + u) * 64 + lane] = add4(o3[u], acc3[u]);
  }
#pragma unroll
  for (int v = 0; v < 5; ++v)
    if (v < nv1) P4[(t1 + v) * 64 + lane] = add4(o1[v], acc1[v]);
  if (wave < 4) P4[(N16_SL_W4 / 256 + wave) * 64 + lane] = add4(o4, acc4);
  (void)ob;
  if (n == 0) {     // bias rows: column 0 of the ones products (every column holds the row sum)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r2 = 16 * wave + 4 * g + q;
      P[N16_SL_B2 + r2] = (accum ? P[N16_SL_B2 + r2] : 0.f) + bias2[q];
      if (wave < 4) {
        const int r3 = 16 * m3 + 4 * g + q;
        P[N16_SL_B3 + r3] = (accum ? P[N16_SL_B3 + r3] : 0.f) + bias3[q];
      }
      if (wave == 0) {
        const int r4 = 4 * g + q;
        P[N16_SL_B4 + r4] = (accum ? P[N16_SL_B4 + r4] : 0.f) + bias4_[q];
      }
    }
  }
  if constexpr (ST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(14);                                           // slab stores complete
}

template <int D>
static void launch_ctrl_node_bwd16(const CtrlNodeBwdArgs& a, int num_blocks, hipStream_t st) {
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)N16_LDS);
    hipLaunchKernelGGL(kern, dim3(num_blocks), dim3(N16_NW * 64), N16_LDS, st, a);
  };
  if (a.stamps) go(ctrl_node_bwd16_kernel<D, true>);
  else go(ctrl_node_bwd16_kernel<D, false>);
}

}  // namespace MB_PREC
}  // namespace mb
