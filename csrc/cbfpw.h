// CBF backward over the active evaluation list with PER-WAVE weight gradients: every wave owns 16
// evaluations per step AND the whole dW3 | dW2 | dW1f in its accumulators (277 registers), so the
// chunk loop has no barrier and no cross-wave stage at all.
//
// Why: cbf_bwd16 (csrc/cbf16.h) splits the weight-gradient output tiles over its 8 waves, so every
// chunk's deltas / activations go through shared LDS stage images with four barrier pairs per
// 128-evaluation chunk, and its phase clocks (scripts/stamps_cbf.py, round 6: 6.4 k forward, 5.7 k
// stage A, 6.0 k dH, 5.5 k stage BC cycles per chunk) show the two stage phases at 29 % / 38 % MFMA
// busy -- the waves of a SIMD sit in the same barrier-locked phase. Here the transposes are
// wave-private: a wave stores its own C tiles (evaluation-major) into its own LDS image and reads
// them straight back with ds_read_b64_tr_b16 as the operands of a contraction over its 16
// evaluations -- v_mfma_f32_32x32x16_bf16 (K = 16, the full-rate bf16 shape), so no K padding.
// LDS ops of one wave complete in order: no barrier between a wave's image stores and its reads,
// nor between the reads and the next image's stores over the same bytes. One wave per SIMD (512
// registers: dW3 128 + dW2 128 + dW1f 16 accumulators + the 16x16x32 data path of cbf_bwd16); the
// independent dW MFMAs fill the latency of the dependent data-path chain.
// Bias gradients db3 / db2 and dw4 are exact fp32 lane sums (reduce-scatter over the 16 evaluation
// lanes), dW1f a v_mfma_f32_16x16x16 contraction against the exact layer-1 input fragment.
// Image layout (per wave, per plane): 16 evaluation rows, row stride S with S / 2 = 16 (mod 32)
// dwords and the 4-column block XOR-swizzled by (row >> 1) & 7 -- ds_write_b64 of a C tile (16
// rows, one block) and ds_read_b64_tr_b16 of an operand (4 rows, 8 blocks) both conflict-free.
// Reference op: /root/reference/cbf.py:40-43 (the Conv1d stack), its autograd backward through
// /root/reference/train.py:103. Same slab layout and inputs as cbf_bwd16.
#pragma once

namespace mb {
namespace MB_PREC {

constexpr int PW_NW = 4;                                   // waves per workgroup (one per SIMD)
constexpr int PW_SA = 224, PW_SB = 288, PW_SF = 16;        // image strides (elements)
constexpr int PW_PLA = 16 * PW_SA;                         // image A: D3 | H2, lo plane at +PLA
constexpr int PW_PLB = 16 * PW_SB;                         // image B: D2 | H1 | D1, lo at +PLB
constexpr int PW_REG = C16_PLANES * PW_PLB + 16 * PW_SF;  // per-wave region (elements), F last
constexpr size_t PW_OFF = C16_LDS_W + C16_LDS_F + CBF_VEC * 4;
constexpr size_t PW_LDS = PW_OFF + (size_t)PW_NW * PW_REG * 2;
static_assert(PW_REG >= C16_PLANES * PW_PLA, "image A fits the region");
static_assert(PW_LDS <= 160 * 1024 - 256, "LDS budget");
// the allocation also holds the final cross-wave sums (4 x 64 x 128 fp32; one workgroup per CU
// either way: 512 registers per wave)
constexpr size_t PW_LDS_ALLOC = PW_LDS > (size_t)PW_NW * 8192 * 4 ? PW_LDS : (size_t)PW_NW * 8192 * 4;

DEV int pw_swz(int row) { return ((row >> 1) & 7) << 2; }

// LDS accesses of this kernel take a 32-bit byte address whose sign bit the compiler can see is
// clear (base & 0x3ffff + small lane terms): only then does it fold the constant part of an address
// into the ds instruction's 16-bit offset -- without that every distinct weight / image address
// was its own loop-invariant VGPR, 90 of them spilled to scratch.
DEV unsigned pw_lds(const void* p) { return (unsigned)(size_t)p & 0x3ffffu; }
template <class T>
DEV T pw_ld(unsigned addr) { return *(const LDS_AS T*)(uintptr_t)addr; }
template <class T>
DEV void pw_st(unsigned addr, const T& v) { *(LDS_AS T*)(uintptr_t)addr = v; }
DEV h16x4 pw_rd(unsigned addr) {
  return __builtin_bit_cast(h16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)addr));
}

// Loop-invariant lane byte offsets into a wave's images: every access below is one of these plus
// a compile-time constant (the 32-column group and the plane) -- a 32-column-aligned group keeps
// the swizzle inside it.
struct PwOff {
  unsigned stA[2], stB[2];   // C-tile store of row n, inner column 16o + 4g
  unsigned trA[2], trB[2];   // 32x32x16 operand rows 8h + q (+4), inner column 16gg + 4p
  unsigned k16B[2], k16F;    // 16x16x16 operand rows 4g + q, inner column 16o + 4p (D1) / 4p (F)
  unsigned stF;              // F store: row n, column 8g
};
DEV PwOff pw_offsets(int lane) {
  const int n = lane & 15, g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, gg = (lane >> 4) & 1, h = lane >> 5;
  PwOff o;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    o.stA[k] = 2u * (n * PW_SA + ((16 * k + 4 * g) ^ pw_swz(n)));
    o.stB[k] = 2u * (n * PW_SB + ((16 * k + 4 * g) ^ pw_swz(n)));
    const int r = 8 * h + q + 4 * k;
    o.trA[k] = 2u * (r * PW_SA + ((16 * gg + 4 * p) ^ pw_swz(r)));
    o.trB[k] = 2u * (r * PW_SB + ((16 * gg + 4 * p) ^ pw_swz(r)));
    const int r4 = 4 * g + q;
    o.k16B[k] = 2u * (r4 * PW_SB + ((16 * k + 4 * p) ^ pw_swz(r4)));
  }
  o.k16F = 2u * ((4 * g + q) * PW_SF + 4 * p);
  o.stF = 2u * (n * PW_SF + 8 * (g & 1));
  return o;
}
// C tile mt of a delta / activation -> image columns c0 + 16mt + 4g (c0 % 32 == 0) of row n
DEV void pw_store4(unsigned img, unsigned lo, const unsigned (&st)[2], int c0, int mt, const Pk4& v) {
  const unsigned p = img + 2u * (c0 + 32 * (mt >> 1)) + st[mt & 1];
  pw_st<h16x4>(p, v.h);
  if constexpr (X3) pw_st<h16x4>(p + 2u * lo, v.l);
}
// 32x32x16 operand over the 16 evaluations: lane (r, h) elem j = img[8h + j][m0 + r] (m0 % 32 == 0)
DEV h16x8 pw_tr32(unsigned img, const unsigned (&tr)[2], int m0) {
  const h16x4 b1 = pw_rd(img + 2u * m0 + tr[0]), b2 = pw_rd(img + 2u * m0 + tr[1]);
  h16x8 r;
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}
DEV Fr pw_tr32_fr(unsigned img, unsigned lo, const unsigned (&tr)[2], int m0) {
  Fr f;
  f.h = pw_tr32(img, tr, m0);
  if constexpr (X3) f.l = pw_tr32(img + 2u * lo, tr, m0);
  return f;
}
// weight operands from the permuted images (w16_fr / w16T_fr of cbf16.h on 32-bit addresses):
// A = W rows m0.. K-step s; A = W^T columns m0.. K-step s
// a loop-invariant base made opaque per iteration (weights are re-read, not pinned in registers),
// masked so that its sign bit is visibly clear (offset folding)
DEV unsigned pw_fresh(unsigned x) {
  asm volatile("" : "+v"(x));
  return x & 0x3ffffu;
}
// lb = image base + 2 (n stride + 8g)
DEV Fr pw_w_fr(unsigned lb, int stride, int m0, int s) {
  const unsigned p = lb + 2u * (m0 * stride + 32 * s);
  Fr r;
  r.h = pw_ld<h16x8>(p);
  if constexpr (X3) r.l = pw_ld<h16x8>(p + 2u * RM16);
  return r;
}
// lb = image base + 2 ((4g + q) stride + 8p)
DEV h16x8 pw_wT(unsigned lb, int stride, int m0, int s) {
  const int colp = 32 * (m0 >> 5) + 4 * ((m0 >> 4) & 1);
  const unsigned a1 = lb + 2u * (32 * s * stride + colp);
  const h16x4 b1 = pw_rd(a1), b2 = pw_rd(a1 + 2u * 16 * stride);
  h16x8 r;
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}
DEV Fr pw_wT_fr(unsigned lb, int stride, int m0, int s) {
  Fr r;
  r.h = pw_wT(lb, stride, m0, s);
  if constexpr (X3) r.l = pw_wT(lb + 2u * RM16, stride, m0, s);
  return r;
}
// lb = vector base + 16g
DEV f32x4 pw_bias4(unsigned lb, int row0) {
  return pw_ld<f32x4>(lb + 4u * row0);
}
// lb = fragment base + 16 lane
DEV Fr pw_frag_fr(unsigned lb, int f) {
  const unsigned p = lb + 2u * (f * FRAG_ELEMS);
  Fr r;
  r.h = pw_ld<h16x8>(p);
  if constexpr (X3) r.l = pw_ld<h16x8>(p + 2u * 512);
  return r;
}
DEV f32x4 mfma16k16(const h16x4& a, const h16x4& b, const f32x4& c) {
#if MB_FP16
  return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c, 0, 0, 0);
#endif
}

template <int D, bool ST>
__global__ __launch_bounds__(PW_NW * 64, 1) void cbf_bwd_pw_kernel(CbfBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  h16* W2 = reinterpret_cast<h16*>(smem);
  h16* wft = W2 + C16_PLANES * RM16;
  float* vl = reinterpret_cast<float*>(smem + C16_LDS_W + C16_LDS_F);
  block_copy16(W2, a.wrm16, (int)C16_LDS_W, false);
  block_copy16(wft, a.w16 + 4 * FRAG_ELEMS, (int)C16_LDS_F, false);
  block_copy16(vl, a.wvec, CBF_VEC * 4);
  __syncthreads();
  const int wave = wave_id(), lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
  const unsigned L0 = pw_lds(smem);
  const unsigned imA = L0 + (unsigned)PW_OFF + 2u * PW_REG * (unsigned)(wave & 3);   // D3 | H2
  const unsigned imB = imA;                                    // D2 | H1 | D1 (over image A)
  const unsigned imF = imA + 2u * C16_PLANES * PW_PLB;         // F, 16 x 16
  const PwOff po = pw_offsets(lane);
  const long EV = (long)*a.nact;
  const long ngrp = (EV + 15) / 16;
  const int4* rec = a.rec;

  f32x16 aW3[2][4], aW2[4][2];
  f32x4 aW1[4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) aW3[u][v] = zero16();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    aW2[u][0] = aW2[u][1] = zero16();
    aW1[u] = zero4();
  }
  // per-lane exact sums, row 16(n >> 2) + 4g + (n & 3) of their vector (reduce-scatter layout)
  float db3 = 0.f, db2a = 0.f, db2b = 0.f, dw4acc = 0.f, db4 = 0.f;

  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tck = 0;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ph[k] += t - tck;
      tck = t;
    }
  };

  const long stride = (long)gridDim.x * PW_NW;
  auto rec_at = [&](long grp) -> int4 {
    const long v = grp * 16 + n;
    return rec[v < EV ? v : EV - 1];
  };
  const long blk = CBF_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const long g0 = blk * PW_NW + wave;
  if (g0 < ngrp) {
  Ev16<D> nx;
  ev16_issue<D>(a, rec_at(g0), nx);
  int4 r2 = rec_at(g0 + stride);

  for (long grp = g0; grp < ngrp; grp += stride) {
    if constexpr (ST) { tck = __builtin_amdgcn_s_memtime(); ph[7] += 1; }
    const Ev16<D> cur = nx;
    const bool in = grp * 16 + n < EV;
    ev16_issue<D>(a, r2, nx);
    r2 = rec_at(grp + 2 * stride);
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
    // weights re-read per step (opaque zero: no loop-invariant operand pinned in registers)
    const int q4 = (lane & 15) >> 2, p4 = lane & 3;
    const unsigned W2c = pw_fresh(L0 + 2u * (n * S16_W2 + 8 * g));
    const unsigned W3c = pw_fresh(L0 + 2u * (RM16_W2 + n * S16_W3 + 8 * g));
    const unsigned W2t = pw_fresh(L0 + 2u * ((4 * g + q4) * S16_W2 + 8 * p4));
    const unsigned W3t = pw_fresh(L0 + 2u * (RM16_W2 + (4 * g + q4) * S16_W3 + 8 * p4));
    const unsigned wtc = pw_fresh(L0 + 2u * C16_PLANES * RM16 + 16u * lane);
    const unsigned b2 = pw_fresh(L0 + (unsigned)(C16_LDS_W + C16_LDS_F) + 16u * g), b3 = b2 + 4u * 128, w4 = b2 + 4u * 192;
    const h16* w1c = a.w16 + opaque_zero();
    // ---- forward recompute (16x16x32, columns = this wave's 16 evaluations)
    Pk4 H1[4], H2[8];
    f32x4 H3[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) H1[mt] = to_pk4(relu4(mma16_bx(frag_fr(w1c, mt, lane), F, zero4())));
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 t = pw_bias4(b2, 16 * mt);
#pragma unroll
      for (int s = 0; s < 2; ++s) t = mma16(pw_w_fr(W2c, S16_W2, 16 * mt, s), pk4_fr(H1[2 * s], H1[2 * s + 1]), t);
      H2[mt] = to_pk4(relu4(t));
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 t = pw_bias4(b3, 16 * mt);
#pragma unroll
      for (int s = 0; s < 4; ++s) t = mma16(pw_w_fr(W3c, S16_W3, 16 * mt, s), pk4_fr(H2[2 * s], H2[2 * s + 1]), t);
      H3[mt] = relu4(t);
    }
    stamp(0);
    // ---- head: dW4 / db4 / db3 exact fp32, dH3pre = w4 * dh . relu'(H3) -> image A with H2
    if (g == 0) db4 += dhv;
    Pk4 D3[4];
    {
      float v[16], d3[16];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 w = pw_bias4(w4, 16 * mt);
        f32x4 d;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[4 * mt + i] = dhv * H3[mt][i];
          d[i] = H3[mt][i] > 0.f ? w[i] * dhv : 0.f;
          d3[4 * mt + i] = d[i];
        }
        D3[mt] = to_pk4(d);
      }
      dw4acc += reduce_scatter16(v, n);
      db3 += reduce_scatter16(d3, n);
    }
    // relu'(H2) as 32 bits, so H2 dies at its image store
    unsigned m2 = 0;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const u32x2v m = __builtin_bit_cast(u32x2v, H2[mt].h);
#pragma unroll
      for (int i = 0; i < 4; ++i) m2 |= (((m[i >> 1] >> (16 * (i & 1))) & 0xffffu) ? 1u : 0u) << (4 * mt + i);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) pw_store4(imA, PW_PLA, po.stA, 0, mt, D3[mt]);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) pw_store4(imA, PW_PLA, po.stA, 64, mt, H2[mt]);
    // ---- dW3 (64 x 128) += D3 . H2^T over the 16 evaluations
    {
      Fr Bh[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) Bh[nt] = pw_tr32_fr(imA, PW_PLA, po.trA, 64 + 32 * nt);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const Fr A = pw_tr32_fr(imA, PW_PLA, po.trA, 32 * mt);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) aW3[mt][nt] = mma(A, Bh[nt], aW3[mt][nt]);
      }
    }
    stamp(1);
    // ---- dH2pre = (W3^T dH3pre) . relu'(H2); dH1pre = (W2^T dH2pre) . relu'(H1)
    Pk4 D2[8], D1[4];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 t = zero4();
#pragma unroll
      for (int s = 0; s < 2; ++s) t = mma16(pw_wT_fr(W3t, S16_W3, 16 * mt, s), pk4_fr(D3[2 * s], D3[2 * s + 1]), t);
#pragma unroll
      for (int i = 0; i < 4; ++i) t[i] = ((m2 >> (4 * mt + i)) & 1u) ? t[i] : 0.f;
      D2[mt] = to_pk4(t);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 t = zero4();
#pragma unroll
      for (int s = 0; s < 4; ++s) t = mma16(pw_wT_fr(W2t, S16_W2, 16 * mt, s), pk4_fr(D2[2 * s], D2[2 * s + 1]), t);
      D1[mt] = to_pk4(t);
      mask_pk4(D1[mt], H1[mt]);
    }
    // ---- dF = W1^T dH1pre -> dL/d(s_i - s_j)
    {
      f32x4 t = zero4();
#pragma unroll
      for (int s = 0; s < 2; ++s) t = mma16(pw_frag_fr(wtc, s), pk4_fr(D1[2 * s], D1[2 * s + 1]), t);
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
    // ---- image B (over image A: this wave's reads of A were issued first and LDS ops of a wave
    // complete in order): D2 | H1 | D1, and F (lanes g < 2 hold the 16 input slots)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) pw_store4(imB, PW_PLB, po.stB, 0, mt, D2[mt]);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      pw_store4(imB, PW_PLB, po.stB, 128, mt, H1[mt]);
      pw_store4(imB, PW_PLB, po.stB, 192, mt, D1[mt]);
    }
    if (g < 2) pw_st<h16x8>(imF + po.stF, F);
    // db2: lane sums of the packed deltas (hi + lo: the x3 operand's value)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      float v[16];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[4 * mt + i] = (float)D2[4 * half + mt].h[i];
          if constexpr (X3) v[4 * mt + i] += (float)D2[4 * half + mt].l[i];
        }
      (half ? db2b : db2a) += reduce_scatter16(v, n);
    }
    // ---- dW2 (128 x 64) += D2 . H1^T; dW1f (64 x 16) += D1 . F^T
    {
      Fr Bh[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) Bh[nt] = pw_tr32_fr(imB, PW_PLB, po.trB, 128 + 32 * nt);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const Fr A = pw_tr32_fr(imB, PW_PLB, po.trB, 32 * mt);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) aW2[mt][nt] = mma(A, Bh[nt], aW2[mt][nt]);
      }
      const h16x4 Fk = pw_rd(imF + po.k16F);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const unsigned d1 = imB + 2u * (192 + 32 * (mt >> 1)) + po.k16B[mt & 1];
        if constexpr (X3) aW1[mt] = mfma16k16(pw_rd(d1 + 2u * PW_PLB), Fk, aW1[mt]);
        aW1[mt] = mfma16k16(pw_rd(d1), Fk, aW1[mt]);
      }
    }
    stamp(3);
  }
  }
  if (ST && lane == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) a.stamps[((long)blockIdx.x * 8 + wave) * 8 + k] = ph[k];

  // ---- per-workgroup slab (cbf_bwd16's layout): fixed-order sums of the 4 waves through LDS
  float* P = a.partial + (long)blockIdx.x * CBF_PARTIAL;
  float* red = reinterpret_cast<float*>(smem);
  const int r = lane & 31, hh = lane >> 5;
  __syncthreads();                                   // every wave is done with weights and images
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[wave * 8192 + (32 * mt + acc_row(i, hh)) * 128 + 32 * nt + r] = aW3[mt][nt][i];
  __syncthreads();
  for (int e = threadIdx.x; e < 8192; e += PW_NW * 64)
    P[P_W3 + e] = ((red[e] + red[8192 + e]) + red[16384 + e]) + red[24576 + e];
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[wave * 8192 + (32 * mt + acc_row(i, hh)) * 64 + 32 * nt + r] = aW2[mt][nt][i];
  __syncthreads();
  for (int e = threadIdx.x; e < 8192; e += PW_NW * 64)
    P[P_W2 + e] = ((red[e] + red[8192 + e]) + red[16384 + e]) + red[24576 + e];
  __syncthreads();
  // [wave][1024 dW1f | 64 db3 | 128 db2 | 64 dw4 | db4]
  constexpr int RW = 1024 + 64 + 128 + 64 + 4;
  float* rw = red + wave * RW;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) rw[(16 * mt + 4 * g + i) * 16 + n] = aW1[mt][i];
  const int vrow = 16 * (n >> 2) + 4 * g + (n & 3);
  rw[1024 + vrow] = db3;
  rw[1088 + vrow] = db2a;
  rw[1088 + 64 + vrow] = db2b;
  rw[1216 + vrow] = dw4acc;
  const float s4 = wave_sum(db4);
  if (lane == 0) rw[1280] = s4;
  __syncthreads();
  for (int e = threadIdx.x; e < 1281; e += PW_NW * 64) {
    const float t = ((red[e] + red[RW + e]) + red[2 * RW + e]) + red[3 * RW + e];
    if (e < 1024) {
      P[P_W1 + (e >> 4) * 32 + (e & 15)] = t;
      P[P_W1 + (e >> 4) * 32 + 16 + (e & 15)] = 0.f;
    } else if (e < 1088) {
      P[P_B3 + e - 1024] = t;
    } else if (e < 1216) {
      P[P_B2 + e - 1088] = t;
    } else if (e < 1280) {
      P[P_W4 + e - 1216] = t;
    } else {
      P[P_B4] = t;
    }
  }
  if (threadIdx.x < 10) P[P_LOSS + threadIdx.x] = 0.f;
}

template <int D>
static void launch_cbf_bwd_pw(const CbfBwdArgs& a, int num_blocks, hipStream_t st) {
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)PW_LDS_ALLOC);
    hipLaunchKernelGGL(kern, dim3(num_blocks), dim3(PW_NW * 64), PW_LDS_ALLOC, st, a);
  };
  if (a.stamps) go(cbf_bwd_pw_kernel<D, true>);
  else go(cbf_bwd_pw_kernel<D, false>);
}

}  // namespace MB_PREC
}  // namespace mb
