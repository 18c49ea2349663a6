// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels of macbf_gnn_amd.
//
// MFMA: v_mfma_f32_32x32x16_bf16, wave64. Lane l: r = l & 31, h = l >> 5.
//   A frag: elem j = A[r][k(h,j)]      B frag: elem j = B[k(h,j)][r]
//   C/D   : reg   = D[(reg&3) + 8*(reg>>2) + 4*h][r]
// k(h,j) = 8h+j for data-built operands, kacc(s,h,j) = 16s+8(j>>2)+4h+(j&3) for operands
// converted from accumulator regs 8s..8s+7 (see macbf_gnn_amd/ops/layout.py, which packs the
// weight fragments in exactly these orders: 64 lanes x 16 B per fragment).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "prec.h"
typedef h16 h16x8 __attribute__((ext_vector_type(8)));
typedef h16 h16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__
#define LDS_AS __attribute__((address_space(3)))

namespace mb {

constexpr int WAVE = 64;
constexpr int FRAG_BYTES = 1024;      // one packed weight fragment (64 lanes x 16 B)

template <int N, typename F>
DEV void static_for(F&& f) {
  if constexpr (N > 0) {
    static_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}

DEV f32x16 mfma(const h16x8& a, const h16x8& b, const f32x16& c) {
#if MB_FP16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}

DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

DEV int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// accumulator regs 8S..8S+7 -> h16 operand fragment
template <int S>
DEV h16x8 acc_frag(const f32x16& c) {
  h16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (h16)c[8 * S + j];
  return r;
}

// relu on fp32 bit patterns: max as signed int32 (negative floats are negative ints) -- one
// v_max_i32 per element, where fmaxf costs a canonicalising v_max plus the max in IEEE mode.
// -0 and negative values map to +0; +NaN passes through.
DEV float relu_f(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

DEV void relu_(f32x16& c) {
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = relu_f(c[i]);
}

// accumulator init with a per-row bias b[row0 + acc_row(reg,h)] (standard orientation)
DEV f32x16 bias_rows(const float* b, int row0, int h) {
  f32x16 c;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) c[reg] = b[row0 + acc_row(reg, h)];
  return c;
}

// 16-byte fragment load (LDS or global): fragment f, lane l
DEV h16x8 frag_ld(const h16* base, int f, int lane) {
  return *reinterpret_cast<const h16x8*>(base + ((size_t)f * WAVE + lane) * 8);
}

// LDS view of a generic pointer into LDS (its low 32 bits are the LDS offset): index math on
// the result stays 32-bit instead of 64-bit generic-pointer arithmetic.
DEV const LDS_AS h16* lds_ptr(const h16* p) {
  return (const LDS_AS h16*)(uintptr_t)(unsigned)(size_t)p;
}

// An opaque scalar zero: adding it to an LDS base inside a loop stops the compiler from
// hoisting every loop-invariant weight-fragment load out of the loop (which would pin
// 100+ VGPRs and spill); the weights stay in LDS and are re-read per tile.
DEV int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}

// Phase clocks (a.stamps) of the 32x32x16 backward kernels: compiled only into diagnostics builds
// (scripts/build_variant.sh stamps cbf,ctrl "-DMB_STAMPS=1"). A runtime `if (a.stamps)` block right
// after an MFMA chain is a branch whose taken path reaches the MFMA's VALU consumers with too few
// wait states (scripts/check_mfma_exec.py; the round-3 "miscompile" of the 16x16x32 CBF kernel, whose
// stamps are now a template instantiation)
// Diagnostics builds: ONE switch, MB_DIAG (a bit mask; scripts/build_variant.sh NAME KERNELS
// "-DMB_DIAG=<bits>"), never set in production: 1 phase clocks of the 32x32x16 backward kernels
// (MB_STAMPS), 2 per-record forward sums of the 16x16x32 CBF backward (scripts/check_cbf16.py), 4 the
// 16x16x32 node backward without its dL/dpooled stores (phase clocks), 8 the kNN scan's cell search
// box shrunk to 0.7x (negative check: the oracle tests must fail, tests/test_gpu_scan_plans.py), 16
// the controller step without its pooled / argmax stores (phase clocks).
#ifndef MB_DIAG
#define MB_DIAG 0
#endif
#define MB_STAMPS ((MB_DIAG & 1) != 0)

// The wave's index in its workgroup as a wave-uniform (SGPR) value. Every branch on it is then a
// scalar branch (s_cbranch_scc) rather than an EXEC-masked region. This matters for MFMAs: the
// compiler drops the s_cbranch_execz skip of a short EXEC-masked block and lets it run with EXEC
// = 0 -- harmless for VALU, but a v_mfma there still updates its accumulator, and with operand
// registers the masked block was meant to set (measured: the 1-pass 16x16x32 edge backward's
// `if (ub == u) biasB = mfma(A, ones)` with threadIdx.x / 64 put the bias MFMA of the other wave
// parity in a masked block without the skip; every wave then added A x {ones, stale registers}
// and db2 came out 90 % wrong, docs/ARCHITECTURE.md "MFMA and EXEC"). Rule in these kernels: no
// MFMA under a lane-divergent condition, wave-dependent conditions on wave_id().
DEV int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE)); }

// XCD-aware block order: the dispatcher hands consecutive workgroups to the 8 XCDs in turn (each
// with its own L2), so a kernel whose neighbouring blocks gather from the same data (one graph's
// edge records) re-fetches it in every XCD. xcd_block maps the blocks sharing an XCD (bid % 8,
// a label, not the XCD id) to one contiguous range of logical blocks -- bijective for any count
// (cdna_hip_programming.md T1). A pure speed choice: any mapping is correct.
constexpr int NXCD = 8;
DEV int xcd_block(int bid, int nwg) {
  const int q = nwg / NXCD, r = nwg % NXCD, x = bid % NXCD;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / NXCD;
}
// BPTT_XCD: the 128-agent chunks of one env (graph) on one XCD in the BPTT chain's edge and node
// backward kernels, so a graph's records stay in one L2 from kernel to kernel (fp32 headline
// 10.85 -> 10.69 ms, bf16 6.85 -> 6.74, profiles/r4_xcd/). ROLL_XCD: the same for the rollout's
// forward step and kNN scan (blocks of one env on one XCD: 10.68-10.69 -> 10.67-10.68 ms, bf16
// 6.73 -> 6.72). node_reduce (graph.hip NODE_RED_XCD): neutral, kept for the same locality.
constexpr bool BPTT_XCD = true;
constexpr bool ROLL_XCD = true;
// CBF_XCD: the CBF h forward / backward over the evaluation list, x3 builds (10.77 -> 10.74 ms;
// bf16 6.74 vs 6.75: off there)
constexpr bool CBF_XCD = MB_X3 != 0;

// lane l <- lane l^32 with v_permlane32_swap (CDNA4, VALU) instead of ds_bpermute (LDS path)
DEV unsigned xor32u(unsigned u) {
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
DEV float shfl_xor32(float v) { return __uint_as_float(xor32u(__float_as_uint(v))); }
DEV int shfl_xor32i(int v) { return (int)xor32u((unsigned)v); }

// hi/lo h16 split of an fp32 value: x ~= hi + lo with ~16 significant bits
DEV void split_h16(float x, h16& hi, h16& lo) {
  hi = (h16)x;
  lo = (h16)(x - (float)hi);
}

// wave-local LDS visibility: all prior LDS writes of this wave done before later LDS reads
DEV void lds_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Order LDS accesses of ONE wave (a store, then another lane's read of it): the LDS processes a
// wave's DS instructions in issue order (lgkmcnt counts them back in order), so program order is
// enough -- a compiler-only fence keeps the compiler from moving the accesses across, without the
// lgkmcnt(0) drain of lds_wave_sync (same speed in the 16x16x32 edge backward, profiles/r4_loads/
// notes; the float64-oracle tests pass with either)
DEV void lds_wave_order() { asm volatile("" ::: "memory"); }

// cooperative copy of `bytes` (multiple of 16) from global to LDS by the whole block
// (8 independent 16-byte loads in flight per thread before the stores: the weight staging at
// kernel start is latency-bound, which dominates small launches -- a 120 KB x3 image is 30
// loads per thread of a 256-thread block)
// LDS-DMA (the VGPR copy it replaced is in the git history, round 5) -- every wave issues all of its 16-byte
// global_load_lds_dwordx4 copies back to back (no VGPR staging, one latency round trip for the
// whole image instead of one per 8 loads), then waits for them before the caller's barrier.
// The destination of one wave instruction is its wave-uniform base + lane x 16: a lane-linear
// image, which a plain copy is. Callers pass LDS destinations and global sources.
// A kernel's back-to-back weight copies wait once, after the last (pass wait = false to all but
// the last; round 5: controller-step staging 6.0 -> 4.7 k cycles, headline fp32 10.609-10.643 -> 10.557-10.587
// ms interleaved, bf16 neutral, profiles/r5_b18/)
// wait = false (LDS-DMA path): issue only -- consecutive copies then share one latency round trip;
// the LAST copy before the caller's barrier must wait (vmcnt(0) covers every copy issued before)
DEV void block_copy16(void* dst, const void* src, int bytes, bool wait = true) {
  const u32x4* s = reinterpret_cast<const u32x4*>(src);
  u32x4* d = reinterpret_cast<u32x4*>(dst);
  const int n = bytes / 16, bd = blockDim.x;
  int i = threadIdx.x;
  const int lane = threadIdx.x & 63;
  for (; i - lane < n; i += bd) {       // wave-uniform trip count (the wave's first index)
    if (i < n)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(s + i),
          (__attribute__((address_space(3))) void*)(d + (i - lane)), 16, 0, 0);
  }
  if (wait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- lane exchanges without the LDS crossbar. __shfl_xor is a ds_bpermute_b32: an LDS-unit
// round trip (~50+ cycles of latency plus the lgkmcnt wait) per step, six of them per wave
// reduction -- in a latency-bound loop (the kNN scan's per-chunk threshold update) that was most of
// the wave's time. lane_xor<O> returns the value of lane (lane ^ O) exactly, on the VALU:
//   O = 1, 2   DPP quad_perm          O = 4   DPP row_shl:4 / row_shr:4 + select
//   O = 8      DPP row_ror:8 (a rotation by 8 inside a 16-lane row is the xor)
//   O = 16     v_permlane16_swap      O = 32  v_permlane32_swap (CDNA4)
// Same partners as the xor butterfly, so every reduction below adds / compares in the same order
// as before (bit-identical results).
template <int O>
DEV unsigned lane_xor(unsigned v) {
  static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "xor distance");
  if constexpr (O == 32) {
    return xor32u(v);
  } else if constexpr (O == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? r[0] : r[1];
  } else if constexpr (O == 8) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);        // row_ror:8
  } else if constexpr (O == 4) {
    const int up = __builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, false);          // row_shl:4: lane + 4
    const int dn = __builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);          // row_shr:4: lane - 4
    return (unsigned)((threadIdx.x & 4) ? dn : up);
  } else if constexpr (O == 2) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);         // quad_perm [2,3,0,1]
  } else {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);         // quad_perm [1,0,3,2]
  }
}
template <int O>
DEV float lane_xorf(float v) { return __uint_as_float(lane_xor<O>(__float_as_uint(v))); }
// runtime distance (folds to one branch when o is a constant after unrolling)
DEV unsigned lane_xor_rt(unsigned v, int o) {
  switch (o) {
    case 1: return lane_xor<1>(v);
    case 2: return lane_xor<2>(v);
    case 4: return lane_xor<4>(v);
    case 8: return lane_xor<8>(v);
    case 16: return lane_xor<16>(v);
    default: return lane_xor<32>(v);
  }
}

DEV float wave_sum(float v) {
  v += lane_xorf<32>(v);
  v += lane_xorf<16>(v);
  v += lane_xorf<8>(v);
  v += lane_xorf<4>(v);
  v += lane_xorf<2>(v);
  v += lane_xorf<1>(v);
  return v;
}

// integer wave sum (exact, so independent of how the addends are grouped over waves)
DEV unsigned long long wave_sum_u64(unsigned long long v) {
  auto step = [](unsigned long long x, auto o_) {
    constexpr int O = decltype(o_)::value;
    const unsigned lo = lane_xor<O>((unsigned)x), hi = lane_xor<O>((unsigned)(x >> 32));
    return x + (((unsigned long long)hi << 32) | lo);
  };
  v = step(v, std::integral_constant<int, 32>{});
  v = step(v, std::integral_constant<int, 16>{});
  v = step(v, std::integral_constant<int, 8>{});
  v = step(v, std::integral_constant<int, 4>{});
  v = step(v, std::integral_constant<int, 2>{});
  v = step(v, std::integral_constant<int, 1>{});
  return v;
}

DEV float wave_max(float v) {
  v = fmaxf(v, lane_xorf<32>(v));
  v = fmaxf(v, lane_xorf<16>(v));
  v = fmaxf(v, lane_xorf<8>(v));
  v = fmaxf(v, lane_xorf<4>(v));
  v = fmaxf(v, lane_xorf<2>(v));
  v = fmaxf(v, lane_xorf<1>(v));
  return v;
}

// counter-based RNG (splitmix64 finaliser) -> uniform [0,1)
DEV uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
DEV float u01(uint64_t key) { return (float)(mix64(key) >> 40) * (1.0f / 16777216.0f); }

}  // namespace mb

namespace mb {

typedef h16 h16x16 __attribute__((ext_vector_type(16)));

// f32x16 accumulator -> packed h16 copy (8 VGPRs), element q = reg q
DEV h16x16 to_h16x16(const f32x16& c) {
  h16x16 r;
#pragma unroll
  for (int q = 0; q < 16; ++q) r[q] = (h16)c[q];
  return r;
}

// relu on packed 16-bit floats (bf16 / fp16): signed 16-bit max with 0, two elements per op.
// Rounding commutes with relu, so to_h16x16_relu(c) == to_h16x16(relu(c)) bit for bit.
DEV unsigned relu_pk16(unsigned x) {
  unsigned r;
  asm volatile("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}

typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));

DEV h16x16 to_h16x16_relu(const f32x16& c) {
  u32x8 v = __builtin_bit_cast(u32x8, to_h16x16(c));
#pragma unroll
  for (int p = 0; p < 8; ++p) v[p] = relu_pk16(v[p]);
  return __builtin_bit_cast(h16x16, v);
}

// sum of the 8 16-bit elements of a fragment into an fp32 accumulator: 4 v_dot2 with (1, 1)
typedef h16 h16x2 __attribute__((ext_vector_type(2)));
DEV float dot_sum8(const h16x8& a, float s) {
  const h16x2 one = {(h16)1.f, (h16)1.f};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    // element pairs by shuffle, not bit_cast: hipcc 7.2 folds a u32x4 bit_cast of the fragment
    // into four reads of its first dword
    const h16x2 x = {a[2 * p], a[2 * p + 1]};
#if MB_FP16
    s = __builtin_amdgcn_fdot2(x, one, s, false);
#else
    s = __builtin_amdgcn_fdot2_f32_bf16(x, one, s, false);
#endif
  }
  return s;
}

template <int S>
DEV h16x8 bacc_frag(const h16x16& c) {
  h16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = c[8 * S + j];
  return r;
}

// store one standard-orientation tile (lane = edge row `erow` of the image, regs = features
// col0 + acc_row(reg,h)) into an edge-major h16 LDS image: 4 x 8-byte writes per lane
DEV void store_tile(h16* img, int stride, int erow, int col0, const h16x16& v, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    h16x4 q;
    q[0] = v[4 * g]; q[1] = v[4 * g + 1]; q[2] = v[4 * g + 2]; q[3] = v[4 * g + 3];
    *reinterpret_cast<h16x4*>(img + erow * stride + col0 + 8 * g + 4 * h) = q;
  }
}

// Transposed operand fragment from an edge-major LDS image img[e][m] (row stride `stride`
// elements, 8-byte aligned): lane (r, h) receives img[e0 + 8h + j][m0 + r], j = 0..7, via two
// ds_read_b64_tr_b16. Used as A (rows = m, k = e) or B (k = e, cols = m) of a contraction over
// edges (the weight-gradient GEMMs). Requires EXEC = all 64 lanes.
DEV h16x8 tr_frag(const h16* img, int stride, int e0, int m0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3, gg = (lane >> 4) & 1, h = lane >> 5;
  const LDS_AS h16* im = lds_ptr(img);                // 32-bit LDS address arithmetic
  const LDS_AS h16* a1 = im + (e0 + 8 * h + q) * stride + m0 + 16 * gg + 4 * p;
  const LDS_AS h16* a2 = a1 + 4 * stride;
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
  const s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a2));
  const h16x4 b1 = __builtin_bit_cast(h16x4, v1);
  const h16x4 b2 = __builtin_bit_cast(h16x4, v2);
  h16x8 r;
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}

// acc += A_img[rows 32mt.., k = e] . B_img[k = e, cols 32nt..] over ES x 16 edges;
// returns the row sums of A over the edge steps [bs_lo, bs_hi) (bias gradient partial; per
// lane: row 32mt + r over half h; 4 v_dot2 per step). Callers split the steps between the
// waves that read the same row block. The fragments of step ks+2 are requested before the
// MFMA of step ks, so the ds_read_b64_tr latency hides behind two MFMAs.
template <int ES>
DEV float stage_mma(const h16* imgA, int sA, const h16* imgB, int sB, int mt, int nt, int lane, f32x16& acc,
                    int bs_lo = 0, int bs_hi = 0) {
  static_assert(ES % 2 == 0, "even edge-step count");
  bs_lo = __builtin_amdgcn_readfirstlane(bs_lo);   // wave-uniform: scalar branches below
  bs_hi = __builtin_amdgcn_readfirstlane(bs_hi);
  float s = 0.f;
  h16x8 a0 = tr_frag(imgA, sA, 0, 32 * mt, lane), b0 = tr_frag(imgB, sB, 0, 32 * nt, lane);
  h16x8 a1 = tr_frag(imgA, sA, 16, 32 * mt, lane), b1 = tr_frag(imgB, sB, 16, 32 * nt, lane);
#pragma nounroll
  for (int ks = 0; ks < ES; ks += 2) {
    acc = mfma(a0, b0, acc);
    if (ks >= bs_lo && ks < bs_hi) s = dot_sum8(a0, s);
    const int k2 = ks + 2 < ES ? ks + 2 : ks;       // last pair: harmless re-read, no branch
    a0 = tr_frag(imgA, sA, 16 * k2, 32 * mt, lane);
    b0 = tr_frag(imgB, sB, 16 * k2, 32 * nt, lane);
    acc = mfma(a1, b1, acc);
    if (ks + 1 >= bs_lo && ks + 1 < bs_hi) s = dot_sum8(a1, s);
    a1 = tr_frag(imgA, sA, 16 * (k2 + 1), 32 * mt, lane);
    b1 = tr_frag(imgB, sB, 16 * (k2 + 1), 32 * nt, lane);
  }
  return s;
}

// accumulator init with bias rows, 4 x 16-byte loads (rows acc_row(4g..4g+3, h) are contiguous)
DEV f32x16 bias_rows4(const float* b, int row0, int h) {
  f32x16 c;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 v = *reinterpret_cast<const float4*>(b + row0 + 8 * g + 4 * h);
    c[4 * g] = v.x; c[4 * g + 1] = v.y; c[4 * g + 2] = v.z; c[4 * g + 3] = v.w;
  }
  return c;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// d *= relu'(pre) given the h16 post-activation H = relu(pre) (>= +0): per 16-bit element,
// m = min(H, 1) (1 where H != 0, else 0) and d * m as a 16-bit integer product (d or 0):
// two packed ops per element pair. (inline asm: an ext_vector u16x2 formulation was
// miscompiled by hipcc 7.2 into a mask taken from only one register of H)
DEV unsigned mask_nz16x2(unsigned d, unsigned x) {
  unsigned m;
  const unsigned ones = 0x00010001u;   // both halves (an inline constant would only fill the low half)
  asm volatile("v_pk_min_u16 %0, %1, %3\n\tv_pk_mul_lo_u16 %0, %2, %0" : "=&v"(m) : "v"(x), "v"(d), "v"(ones));
  return m;
}

DEV void mask_by_nonzero(h16x16& d, const h16x16& H) {
  u32x8 dv = __builtin_bit_cast(u32x8, d);
  const u32x8 hv = __builtin_bit_cast(u32x8, H);
#pragma unroll
  for (int p = 0; p < 8; ++p) dv[p] = mask_nz16x2(dv[p], hv[p]);
  d = __builtin_bit_cast(h16x16, dv);
}

// write an owned dW tile (rows 32mt.., cols 32nt..) of a row-major (ncols) fp32 slab
DEV void write_tile(float* dst, int ncols, int mt, int nt, const f32x16& c, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) dst[(32 * mt + acc_row(reg, h)) * ncols + 32 * nt + r] = c[reg];
}

DEV float sum32(float v) {   // sum over the 32 lanes of this lane's half
  v += lane_xorf<16>(v);
  v += lane_xorf<8>(v);
  v += lane_xorf<4>(v);
  v += lane_xorf<2>(v);
  v += lane_xorf<1>(v);
  return v;
}

// ---- XOR-swizzled edge-major LDS images (no row padding). Logical element (row, col) of an
// image W elements wide lives at row*W + (((col>>3) ^ swz<W>(row)) << 3) + (col & 7): 16-byte
// units are permuted per row, so 16-byte / 8-byte pieces stay contiguous. The permutations make
//   * ds_read_b64_tr_b16 fragments (rows e0..e0+3, e0 % 4 == 0, a 32-column block) hit 4
//     disjoint 16-bank ranges (padding strides could only make them 2-way at best),
//   * 16-byte row reads of 16 different rows (W = 128) conflict-free,
//   * 8-byte tile stores (16 rows, one column piece) at most 2-way (W = 32: conflict-free).
template <int W> DEV int swz(int row);
template <> DEV int swz<128>(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
template <> DEV int swz<64>(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
template <> DEV int swz<32>(int row) { return (row >> 1) & 3; }

template <int W>
DEV int swz_off(int row, int col) { return row * W + ((((col >> 3) ^ swz<W>(row))) << 3) + (col & 7); }

// store_tile into a swizzled image (4 x 8-byte writes per lane; col0 % 32 == 0)
template <int W>
DEV void store_tile_sw(h16* img, int erow, int col0, const h16x16& v, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    h16x4 q;
    q[0] = v[4 * g]; q[1] = v[4 * g + 1]; q[2] = v[4 * g + 2]; q[3] = v[4 * g + 3];
    *reinterpret_cast<h16x4*>(img + swz_off<W>(erow, col0 + 8 * g + 4 * h)) = q;
  }
}

// Per-lane offsets of the two ds_read_b64_tr_b16 of a fragment at edge rows e0 + 8h + q (+4),
// column block m0: e0 % 16 == 0 keeps the row's swizzle independent of e0, so a contraction
// adds only the uniform e0 * W to these (immediate offsets in the loop).
struct TrOff { int o1, o2; };

template <int W>
DEV TrOff tr_off_sw(int m0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3, gg = (lane >> 4) & 1, h = lane >> 5;
  const int col = m0 + 16 * gg + 4 * p;
  return {swz_off<W>(8 * h + q, col), swz_off<W>(8 * h + q + 4, col)};
}

// tr_frag on a swizzled image: lane (r, h) receives img[e0 + 8h + j][m0 + r], j = 0..7
template <int W>
DEV h16x8 tr_frag_sw(const h16* img, int e0, const TrOff& o) {
  const LDS_AS h16* im = lds_ptr(img) + e0 * W;
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(im + o.o1));
  const s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(im + o.o2));
  const h16x4 b1 = __builtin_bit_cast(h16x4, v1);
  const h16x4 b2 = __builtin_bit_cast(h16x4, v2);
  h16x8 r;
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}

// stage_mma on swizzled images (A: WA wide, B: WB wide); same contract as stage_mma
template <int ES, int WA, int WB>
DEV float stage_mma_sw(const h16* imgA, const h16* imgB, int mt, int nt, int lane, f32x16& acc,
                       int bs_lo = 0, int bs_hi = 0) {
  static_assert(ES % 2 == 0, "even edge-step count");
  bs_lo = __builtin_amdgcn_readfirstlane(bs_lo);
  bs_hi = __builtin_amdgcn_readfirstlane(bs_hi);
  const TrOff oa = tr_off_sw<WA>(32 * mt, lane), ob = tr_off_sw<WB>(32 * nt, lane);
  float s = 0.f;
  h16x8 a0 = tr_frag_sw<WA>(imgA, 0, oa), b0 = tr_frag_sw<WB>(imgB, 0, ob);
  h16x8 a1 = tr_frag_sw<WA>(imgA, 16, oa), b1 = tr_frag_sw<WB>(imgB, 16, ob);
#pragma nounroll
  for (int ks = 0; ks < ES; ks += 2) {
    acc = mfma(a0, b0, acc);
    if (ks >= bs_lo && ks < bs_hi) s = dot_sum8(a0, s);
    const int k2 = ks + 2 < ES ? ks + 2 : ks;
    a0 = tr_frag_sw<WA>(imgA, 16 * k2, oa);
    b0 = tr_frag_sw<WB>(imgB, 16 * k2, ob);
    acc = mfma(a1, b1, acc);
    if (ks + 1 >= bs_lo && ks + 1 < bs_hi) s = dot_sum8(a1, s);
    a1 = tr_frag_sw<WA>(imgA, 16 * (k2 + 1), oa);
    b1 = tr_frag_sw<WB>(imgB, 16 * (k2 + 1), ob);
  }
  return s;
}

}  // namespace mb

namespace mb {

// ---- MFMA operand readers for row-major h16 weight images W[rows][stride] in LDS.
// One copy of a weight matrix serves the forward (W) and the backward (W^T) chains.

// A = W, natural k:  elem j = W[m0 + r][16kk + 8h + j]        (one 16-byte read)
DEV h16x8 wrm_nat(const h16* W, int stride, int m0, int kk, int lane) {
  const int r = lane & 31, h = lane >> 5;
  return *reinterpret_cast<const h16x8*>(W + (m0 + r) * stride + 16 * kk + 8 * h);
}

// A = W, accumulator k: elem j = W[m0 + r][32t + 16s + 8(j>>2) + 4h + (j&3)], kk = 2t + s
DEV h16x8 wrm_acc(const h16* W, int stride, int m0, int kk, int lane) {
  const int r = lane & 31, h = lane >> 5;
  const h16* p = W + (m0 + r) * stride + 16 * kk + 4 * h;
  const h16x4 lo = *reinterpret_cast<const h16x4*>(p);
  const h16x4 hi = *reinterpret_cast<const h16x4*>(p + 8);
  h16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// two ds_read_b64_tr_b16: lane (r = 16gg + i, h) receives img[rb1 + j][c0 + r] (j<4) and
// img[rb2 + j-4][c0 + r] (j>=4); rb1/rb2 may depend on h only (uniform per 16-lane group)
DEV h16x8 tr_pair(const h16* img, int stride, int rb1, int rb2, int c0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3, gg = (lane >> 4) & 1;
  const LDS_AS h16* im = lds_ptr(img);                // 32-bit LDS address arithmetic
  const LDS_AS h16* a1 = im + (rb1 + q) * stride + c0 + 16 * gg + 4 * p;
  const LDS_AS h16* a2 = im + (rb2 + q) * stride + c0 + 16 * gg + 4 * p;
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
  const s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a2));
  const h16x4 b1 = __builtin_bit_cast(h16x4, v1);
  const h16x4 b2 = __builtin_bit_cast(h16x4, v2);
  h16x8 r;
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}

// A = W^T, accumulator k: elem j = W[32t + 16s + 8(j>>2) + 4h + (j&3)][m0 + r]
DEV h16x8 wrmT_acc(const h16* W, int stride, int m0, int kk, int lane) {
  const int h = lane >> 5;
  const int rb = 16 * kk + 4 * h;
  return tr_pair(W, stride, rb, rb + 8, m0, lane);
}

// A = W^T, natural k: elem j = W[16kk + 8h + j][m0 + r]
DEV h16x8 wrmT_nat(const h16* W, int stride, int m0, int kk, int lane) {
  const int h = lane >> 5;
  const int rb = 16 * kk + 8 * h;
  return tr_pair(W, stride, rb, rb + 4, m0, lane);
}

}  // namespace mb

// =======================================================================================
// Operand-precision layer (csrc/prec.h). Kernels are written once against these types:
//   Fr  an MFMA operand fragment (8 x h16 per lane) with its residual plane `l` (x3 only),
//   Pk  a packed 32x32 activation tile (16 x h16 per lane, see to_h16x16) with its residual,
//   mma a product: one MFMA (bf16 / fp16) or hi*hi + hi*lo + lo*hi (x3, small terms first).
// In the 1-pass builds the `l` members are never written or read (the compiler drops them).
// Weight fragments are FRAG_ELEMS apart in the packed buffers: x3 stores each 1 KiB hi fragment
// followed by its 1 KiB lo fragment. Row-major images and LDS stage images keep their lo plane
// at a fixed element offset (`lo` arguments) from the hi plane.
// =======================================================================================
namespace mb {

constexpr bool X3 = MB_X3 != 0;
constexpr int FRAG_ELEMS = X3 ? 1024 : 512;     // h16 elements per packed fragment (hi [+ lo])
constexpr int FRAG_SZ = FRAG_ELEMS * 2;          // bytes
constexpr int PROW = X3 ? 256 : 128;             // h16 per pooled / dL/dpooled row: [hi 128 | lo 128]

struct Fr { h16x8 h, l; };
struct Pk { h16x16 h, l; };

DEV f32x16 mma(const Fr& a, const Fr& b, f32x16 c) {
  if constexpr (X3) {
    c = mfma(a.l, b.h, c);
    c = mfma(a.h, b.l, c);
  }
  return mfma(a.h, b.h, c);
}

// b exact in h16 (the layer-1 input fragments carry their own hi/lo split along k)
DEV f32x16 mma_bx(const Fr& a, const h16x8& b, f32x16 c) {
  if constexpr (X3) c = mfma(a.l, b, c);
  return mfma(a.h, b, c);
}

DEV h16x8 zero_h8() {
  h16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (h16)0.f;
  return z;
}

// accumulator regs 8S..8S+7 -> operand fragment (acc_frag + residual)
template <int S>
DEV Fr acc_fr(const f32x16& c) {
  Fr f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = c[8 * S + j];
    f.h[j] = (h16)x;
    if constexpr (X3) f.l[j] = (h16)(x - (float)f.h[j]);
  }
  return f;
}

DEV Pk to_pk(const f32x16& c) {
  Pk p;
  p.h = to_h16x16(c);
  if constexpr (X3) {
#pragma unroll
    for (int q = 0; q < 16; ++q) p.l[q] = (h16)(c[q] - (float)p.h[q]);
  }
  return p;
}

// relu(c) packed; x3: relu in fp32, then split (both planes are +0 where c <= 0)
DEV Pk to_pk_relu(const f32x16& c) {
  if constexpr (X3) {
    f32x16 r = c;
    relu_(r);
    return to_pk(r);
  } else {
    Pk p;
    p.h = to_h16x16_relu(c);
    return p;
  }
}

template <int S>
DEV Fr pk_fr(const Pk& p) {
  Fr f;
  f.h = bacc_frag<S>(p.h);
  if constexpr (X3) f.l = bacc_frag<S>(p.l);
  return f;
}

// d *= relu'(pre), H = relu(pre) packed (>= +0): both planes of d masked by H's hi plane
DEV void mask_pk(Pk& d, const Pk& H) {
  mask_by_nonzero(d.h, H.h);
  if constexpr (X3) mask_by_nonzero(d.l, H.h);
}

// ---- weight operands
DEV Fr frag_fr(const h16* base, int f, int lane) {
  const h16* p = base + ((size_t)f * FRAG_ELEMS + lane * 8);
  Fr r;
  r.h = *reinterpret_cast<const h16x8*>(p);
  if constexpr (X3) r.l = *reinterpret_cast<const h16x8*>(p + 512);
  return r;
}

DEV Fr wrm_nat_fr(const h16* W, int stride, int m0, int kk, int lane, int lo) {
  Fr r;
  r.h = wrm_nat(W, stride, m0, kk, lane);
  if constexpr (X3) r.l = wrm_nat(W + lo, stride, m0, kk, lane);
  return r;
}

DEV Fr wrm_acc_fr(const h16* W, int stride, int m0, int kk, int lane, int lo) {
  Fr r;
  r.h = wrm_acc(W, stride, m0, kk, lane);
  if constexpr (X3) r.l = wrm_acc(W + lo, stride, m0, kk, lane);
  return r;
}

DEV Fr wrmT_nat_fr(const h16* W, int stride, int m0, int kk, int lane, int lo) {
  Fr r;
  r.h = wrmT_nat(W, stride, m0, kk, lane);
  if constexpr (X3) r.l = wrmT_nat(W + lo, stride, m0, kk, lane);
  return r;
}

// hi plane of a standard-orientation tile stored by store_tile (row = this lane's agent/edge,
// regs = features col0 + acc_row(reg, h)): the inverse of store_tile, 4 x 8-byte reads
DEV h16x16 load_tile_h(const h16* img, int stride, int erow, int col0, int h) {
  h16x16 v;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const h16x4 q = *reinterpret_cast<const h16x4*>(img + erow * stride + col0 + 8 * g + 4 * h);
    v[4 * g] = q[0]; v[4 * g + 1] = q[1]; v[4 * g + 2] = q[2]; v[4 * g + 3] = q[3];
  }
  return v;
}

DEV Fr wrmT_acc_fr(const h16* W, int stride, int m0, int kk, int lane, int lo) {
  Fr r;
  r.h = wrmT_acc(W, stride, m0, kk, lane);
  if constexpr (X3) r.l = wrmT_acc(W + lo, stride, m0, kk, lane);
  return r;
}

// 16-byte row read of a [row][stride] h16 image / global row, with its lo plane at +lo
DEV Fr row_fr(const h16* p, int lo) {
  Fr r;
  r.h = *reinterpret_cast<const h16x8*>(p);
  if constexpr (X3) r.l = *reinterpret_cast<const h16x8*>(p + lo);
  return r;
}

// ---- LDS stage images (edge-major, hi plane + lo plane at +lo)
DEV void store_pk(h16* img, int stride, int erow, int col0, const Pk& v, int h, int lo) {
  store_tile(img, stride, erow, col0, v.h, h);
  if constexpr (X3) store_tile(img + lo, stride, erow, col0, v.l, h);
}

template <int W>
DEV void store_pk_sw(h16* img, int erow, int col0, const Pk& v, int h, int lo) {
  store_tile_sw<W>(img, erow, col0, v.h, h);
  if constexpr (X3) store_tile_sw<W>(img + lo, erow, col0, v.l, h);
}

// stage_mma with split operands: A = imgA (+loA), B = imgB (+loB); BX: B exact (no lo plane).
// Bias row sums of A cover both planes. x3: fully unrolled (ES <= 8 here) so every fragment read
// has an immediate LDS offset, double-buffered fragments (no register copies), the fragments of
// step ks+2 requested right after the three MFMAs of step ks have read their operands.
template <int ES, bool BX = false>
DEV float stage_mma_fr(const h16* imgA, int sA, int loA, const h16* imgB, int sB, int loB, int mt, int nt, int lane,
                       f32x16& acc, int bs_lo = 0, int bs_hi = 0) {
  if constexpr (!X3) {
    return stage_mma<ES>(imgA, sA, imgB, sB, mt, nt, lane, acc, bs_lo, bs_hi);
  } else {
    static_assert(ES % 2 == 0 && ES <= 16, "even edge-step count");
    bs_lo = __builtin_amdgcn_readfirstlane(bs_lo);
    bs_hi = __builtin_amdgcn_readfirstlane(bs_hi);
    float s = 0.f;
    Fr a[2], b[2];
    auto ld = [&](int ks, Fr& x, Fr& y) {
      x.h = tr_frag(imgA, sA, 16 * ks, 32 * mt, lane);
      x.l = tr_frag(imgA + loA, sA, 16 * ks, 32 * mt, lane);
      y.h = tr_frag(imgB, sB, 16 * ks, 32 * nt, lane);
      if constexpr (!BX) y.l = tr_frag(imgB + loB, sB, 16 * ks, 32 * nt, lane);
    };
    ld(0, a[0], b[0]);
    ld(1, a[1], b[1]);
    static_for<ES>([&](auto ks_) {
      constexpr int ks = decltype(ks_)::value, sl = ks & 1;
      if constexpr (BX) acc = mma_bx(a[sl], b[sl].h, acc);
      else acc = mma(a[sl], b[sl], acc);
      if (ks >= bs_lo && ks < bs_hi) {
        s = dot_sum8(a[sl].l, s);
        s = dot_sum8(a[sl].h, s);
      }
      if constexpr (ks + 2 < ES) ld(ks + 2, a[sl], b[sl]);
    });
    return s;
  }
}

template <int ES, int WA, int WB, bool BX = false>
DEV float stage_mma_sw_fr(const h16* imgA, int loA, const h16* imgB, int loB, int mt, int nt, int lane, f32x16& acc,
                          int bs_lo = 0, int bs_hi = 0) {
  if constexpr (!X3) {
    return stage_mma_sw<ES, WA, WB>(imgA, imgB, mt, nt, lane, acc, bs_lo, bs_hi);
  } else {
    static_assert(ES % 2 == 0 && ES <= 16, "even edge-step count");
    bs_lo = __builtin_amdgcn_readfirstlane(bs_lo);
    bs_hi = __builtin_amdgcn_readfirstlane(bs_hi);
    const TrOff oa = tr_off_sw<WA>(32 * mt, lane), ob = tr_off_sw<WB>(32 * nt, lane);
    float s = 0.f;
    Fr a[2], b[2];
    auto ld = [&](int ks, Fr& x, Fr& y) {
      x.h = tr_frag_sw<WA>(imgA, 16 * ks, oa);
      x.l = tr_frag_sw<WA>(imgA + loA, 16 * ks, oa);
      y.h = tr_frag_sw<WB>(imgB, 16 * ks, ob);
      if constexpr (!BX) y.l = tr_frag_sw<WB>(imgB + loB, 16 * ks, ob);
    };
    ld(0, a[0], b[0]);
    ld(1, a[1], b[1]);
    static_for<ES>([&](auto ks_) {
      constexpr int ks = decltype(ks_)::value, sl = ks & 1;
      if constexpr (BX) acc = mma_bx(a[sl], b[sl].h, acc);
      else acc = mma(a[sl], b[sl], acc);
      if (ks >= bs_lo && ks < bs_hi) {
        s = dot_sum8(a[sl].l, s);
        s = dot_sum8(a[sl].h, s);
      }
      if constexpr (ks + 2 < ES) ld(ks + 2, a[sl], b[sl]);
    });
    return s;
  }
}

// per-turn share [lo, hi) of the bias-sum edge steps: a wave owns steps [w0, w1) of the whole
// chunk (nturns x ks_turn steps); turn `turn` contracts steps [turn*ks_turn, (turn+1)*ks_turn)
DEV void turn_range(int w0, int w1, int turn, int ks_turn, int& lo, int& hi) {
  const int t0 = turn * ks_turn;
  lo = max(w0, t0) - t0;
  hi = min(w1, t0 + ks_turn) - t0;
  if (hi < lo) hi = lo;
}

}  // namespace mb
