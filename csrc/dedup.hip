// Deduplicated CBF evaluations (gfx950).
//
// The training loss needs, for every kNN slot (t,b,i,k) of the rollout (reference
// core.py:89-171), h on s_t and h' on s_{t+1} of the same neighbour pair (i, j). Because the
// barrier is a function of the pair's relative state only (cbf.py:21-45), h' of slot
// (t,b,i,k) IS h of the slot (t+1,b,i,k') that holds the same neighbour j at the next step --
// and between consecutive steps almost every neighbour set is unchanged (measured: 2.4 % of
// the slots change at 1024 agents). So the trainer evaluates
//   * every main slot once (u = e < E, on s_t), and
//   * one "extra" evaluation (u >= E, on s_{t+1}) per slot whose neighbour is not in the next
//     step's list (all slots of the last step),
// i.e. ~1.08 E evaluations instead of 2 E. The upstream gradient of an evaluation is then the
// sum of its h-role (barrier + derivative terms of its own slot) and its h'-role (derivative
// term of the source slot of the previous step); the backward is linear in it, so one backward
// pass per evaluation gives both roles (BPTT mode: both roles' state gradients land on s_t).
//
// cbf_match_kernel: phase 0 counts the extras of every (t,b,i) row; after an exclusive scan of
//   the counts (rows are in (t,b,i) order, so the extras list is ordered by (t,b,i,k) and the
//   offsets are exact integers: deterministic) phase 1 writes
//     map1[e] = evaluation index of the h' partner of main slot e,
//     src[u]  = the main slot whose h' evaluation u is (or -1).
// cbf_dh_kernel: per evaluation, the upstream gradient from the stored (masked) h values and
//   the 8 loss partial sums (deterministic per-block partials, fixed-order reduction after).
#pragma clang fp contract(off)
#include "common.h"
#include "args.h"

namespace mb {

constexpr int MATCH_BLOCK = 256;
constexpr int DH_BLOCK = 256;
constexpr int DH_PARTIAL = 12;
constexpr int DH_UNROLL = 4;   // loss partials per block: [0, 0, 8 sums, 0, 0] (rows padded to 4)

// Block-wide exclusive scan of one int per thread (NT threads, wave64): returns the exclusive
// prefix of this thread, *total = the block sum. Two barriers.
template <int NT>
DEV int block_excl_scan(int v, int* total) {
  __shared__ int wsum[NT / WAVE];
  const int lane = threadIdx.x % WAVE, wave = threadIdx.x / WAVE;
  int x = v;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == WAVE - 1) wsum[wave] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / WAVE; ++w) {
    pre += (w < wave) ? wsum[w] : 0;
    tot += wsum[w];
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// Sum of p[0..n) by the whole block (integer sums: exact in any order). Every block of a grid
// sums the counts of all blocks before it, so the loads are issued 8 per thread at a time (one
// dependent round trip per 8 x NT counts; the 4,608 match blocks at the headline took ~20 us
// with one load per round trip).
template <int NT>
DEV int block_sum_prefix(const int* p, int n) {
  int s = 0;
  for (int q0 = threadIdx.x; q0 < n; q0 += 8 * NT) {
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = q0 + u * NT < n ? p[q0 + u * NT] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  int tot;
  (void)block_excl_scan<NT>(s, &tot);
  return tot;
}

// One thread per (t,b,i) row, MATCH_BLOCK consecutive rows per block. Phase 0 stages the block's
// slot rows of step t and step t+1 (each one contiguous segment) in LDS with coalesced loads,
// matches in registers and writes everything that does not need the global extras offsets:
// map1 of the matched slots (final), a placeholder -1 - x for the row's x-th unmatched slot, the
// next step's src (final), the per-row extras counts and the block sums. Phase 1 turns the
// placeholders of the rows that have extras (a quarter of the rows at the headline) into
// E + offset and writes their src entries -- it reads one count per row instead of re-staging and
// re-matching both steps' slot rows (round 6; the two phases were 2 x 75 us at the headline).
__global__ __launch_bounds__(MATCH_BLOCK) void cbf_match_kernel(CbfMatchArgs a) {
  __shared__ int s0[MATCH_BLOCK * 16], s1[MATCH_BLOCK * 16];
  const long BN = (long)a.B * a.N;
  const long rows = (long)a.T * BN;
  const int K = a.K;
  const long NKB = BN * K;                 // slots per step
  const long E = (long)a.T * NKB;
  const long row0 = (long)blockIdx.x * MATCH_BLOCK;
  const int nr = (int)min((long)MATCH_BLOCK, rows - row0);
  const long e00 = row0 * K;
  const int ns = nr * K;
  const int lr = threadIdx.x;
  const long row = row0 + lr;
  const bool live = lr < nr;
  if (a.phase == 1) {
    // extras offset of this row: exclusive scan over the rows (in-kernel when off is null: block
    // prefix from the phase-0 block sums + the block-local scan; exact integers, deterministic)
    const int cnt = live ? a.cnt[row] : 0;
    long roff = 0;
    if (a.off) {
      roff = live ? a.off[row] : 0;
    } else {
      const int pre = block_sum_prefix<MATCH_BLOCK>(a.bsum, blockIdx.x);
      int tot;
      const int ex = block_excl_scan<MATCH_BLOCK>(cnt, &tot);
      roff = (long)pre + ex;
      if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0 && a.nev) *a.nev = (int)(E + pre + tot);
    }
    if (live && cnt > 0) {
      const long e0 = row * K, off = E + roff;
      int mv[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) mv[k] = k < K ? a.map1[e0 + k] : 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k < K && mv[k] < 0) {
          const long u = off - 1 - mv[k];          // placeholder -1 - x -> extra x of the row
          a.map1[e0 + k] = (int)u;
          a.src[u] = (int)(e0 + k);
        }
      }
    }
    return;
  }
  // next-step rows exist for rows < (T-1)*BN
  const int nn = (int)max(0L, min((long)nr, (long)(a.T - 1) * BN - row0));
  for (int q = threadIdx.x; q < ns; q += MATCH_BLOCK) s0[q] = a.idx[e00 + q];
  for (int q = threadIdx.x; q < nn * K; q += MATCH_BLOCK) s1[q] = a.idx[e00 + NKB + q];
  __syncthreads();
  const bool has_next = lr < nn;
  int m[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = -1;
  int nmatch = 0;
  if (live && has_next) {
    if (a.mode == 1) {
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = (k < K) ? k : -1;
      nmatch = K;
    } else {
      int j1[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) j1[q] = (q < K) ? s1[lr * K + q] : -2;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k < K) {
          const int j0 = s0[lr * K + k];
          int mk = -1;
#pragma unroll
          for (int q = 0; q < 16; ++q) mk = (j1[q] == j0) ? q : mk;
          m[k] = mk;
          nmatch += (mk >= 0) ? 1 : 0;
        }
      }
    }
  }
  const int cnt = live ? K - nmatch : 0;
  if (live && a.cnt) a.cnt[row] = cnt;
  int tot;
  (void)block_excl_scan<MATCH_BLOCK>(cnt, &tot);   // (its barriers also end the reads of s0 / s1)
  if (threadIdx.x == 0 && a.bsum) a.bsum[blockIdx.x] = tot;
  if (!a.map1) return;                             // counts only
  const long e0 = row * K;
  if (live) {
    int x = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k >= K) continue;
      if (m[k] >= 0) {
        s0[lr * K + k] = (int)(e0 + NKB + m[k]);
      } else {
        s0[lr * K + k] = -1 - x;                   // phase 1: E + the row's offset + x
        ++x;
      }
    }
    if (has_next) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q >= K) continue;
        int sv = -1;
#pragma unroll
        for (int k = 0; k < 16; ++k) sv = (m[k] == q) ? (int)(e0 + k) : sv;
        s1[lr * K + q] = sv;
      }
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < ns; q += MATCH_BLOCK) a.map1[e00 + q] = s0[q];
  for (int q = threadIdx.x; q < nn * K; q += MATCH_BLOCK) a.src[e00 + NKB + q] = s1[q];
  // first step: its main slots have no source
  const long first = min((long)ns, max(0L, NKB - e00));
  for (long q = threadIdx.x; q < first; q += MATCH_BLOCK) a.src[e00 + q] = -1;
}

// evaluations per dh / compact block: a multiple of DH_BLOCK, the same in both kernels
DEV unsigned dh_span(unsigned U, unsigned nblocks) {
  const unsigned per = (U + nblocks - 1) / nblocks;
  return (per + DH_BLOCK - 1) / DH_BLOCK * DH_BLOCK;
}

__global__ __launch_bounds__(DH_BLOCK) void cbf_dh_kernel(CbfDhArgs a) {
  const unsigned NK = (unsigned)a.N * a.K, BNK = (unsigned)a.B * NK;
  const unsigned E = (unsigned)a.T * BNK;
  const unsigned U = (unsigned)*a.nev;
  const float nd = 1e-5f + a.counts[0], ns = 1e-5f + a.counts[1];
  const float lsc = lc_scale(a.lc);
  const LossConsts lc = a.lc;
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  // contiguous per-block ranges (the active-list compaction keeps this order)
  const unsigned span = dh_span(U, gridDim.x);
  const unsigned u_hi = min(U, (blockIdx.x + 1) * span);
  int nact = 0;
  // DH_UNROLL evaluations per thread per round: every round issues the independent loads of all
  // of them first, then the dependent ones (partner h, source slot), then computes -- the same
  // per-thread order of u as a plain loop (u, u + DH_BLOCK, ...), so the partial sums are unchanged
  constexpr int UR = DH_UNROLL;
  for (unsigned u0 = blockIdx.x * span + threadIdx.x; u0 < u_hi; u0 += UR * DH_BLOCK) {
    bool in[UR], mv[UR], sv[UR];
    float hv0[UR], hn0[UR], hv1[UR], hn1[UR];
    unsigned m1[UR];
    int src[UR];
    uint8_t dg0[UR], dg1[UR], hm[UR];
#pragma unroll
    for (int j = 0; j < UR; ++j) {
      const unsigned u = u0 + j * DH_BLOCK;
      in[j] = u < u_hi;
      mv[j] = sv[j] = false;
      src[j] = -1;
      if (in[j]) {
        hm[j] = a.hmask[u];
        src[j] = a.src[u];
        hn1[j] = a.h[u];
        if (u < E) {
          const unsigned t = u / BNK, b = (u - t * BNK) / NK;
          mv[j] = !a.valid || a.valid[t * a.B + b];
          m1[j] = (unsigned)a.map1[u];
          dg0[j] = a.dang[u];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < UR; ++j) {
      const unsigned u = u0 + j * DH_BLOCK;
      if (mv[j]) {
        hv0[j] = hn1[j];            // h of main slot u
        hn0[j] = a.h[m1[j]];
      }
      if (in[j] && src[j] >= 0) {
        const unsigned su = (unsigned)src[j];
        const unsigned t = su / BNK, b = (su - t * BNK) / NK;
        sv[j] = !a.valid || a.valid[t * a.B + b];
        hv1[j] = a.h[su];
        dg1[j] = a.dang[su];
      }
      (void)u;
    }
#pragma unroll
    for (int j = 0; j < UR; ++j) {
      if (!in[j]) continue;
      const unsigned u = u0 + j * DH_BLOCK;
      float g = 0.f;
      if (mv[j]) {                                   // h-role of main slot u
        const float hv = hv0[j], hnv = hn0[j];
        const float deriv = hnv - hv + lc.dt_alpha * hv;
        if (dg0[j]) {
          const float cc = lsc / nd;
          const float ind_b = (hv + lc.eps_dang > 0.f) ? 1.f : 0.f;
          const float ind_d = (-deriv + lc.eps_dang > 0.f) ? 1.f : 0.f;
          g += cc * (lc.w_dang * ind_b + lc.w_dang_d * ind_d * (1.f - lc.dt_alpha));
          acc[0] += fmaxf(hv + lc.eps_dang, 0.f);
          acc[2] += (hv <= 0.f) ? 1.f : 0.f;
          acc[4] += fmaxf(-deriv + lc.eps_dang, 0.f);
          acc[6] += (deriv >= 0.f) ? 1.f : 0.f;
        } else {
          const float cc = lsc / ns;
          const float ind_b = (-hv > 0.f) ? 1.f : 0.f;
          const float ind_d = (-deriv > 0.f) ? 1.f : 0.f;
          g += cc * (-lc.w_safe * ind_b + lc.w_safe_d * ind_d * (1.f - lc.dt_alpha));
          acc[1] += fmaxf(-hv, 0.f);
          acc[3] += (hv > 0.f) ? 1.f : 0.f;
          acc[5] += fmaxf(-deriv, 0.f);
          acc[7] += (deriv > 0.f) ? 1.f : 0.f;
        }
      }
      if (sv[j]) {                                   // h'-role: derivative term of source slot s
        const float hv = hv1[j], hnv = hn1[j];
        const float deriv = hnv - hv + lc.dt_alpha * hv;
        if (dg1[j]) {
          const float ind_d = (-deriv + lc.eps_dang > 0.f) ? 1.f : 0.f;
          g += -(lsc / nd) * lc.w_dang_d * ind_d;
        } else {
          const float ind_d = (-deriv > 0.f) ? 1.f : 0.f;
          g += -(lsc / ns) * lc.w_safe_d * ind_d;
        }
      }
      const float d = hm[j] ? g : 0.f;
      a.dh[u] = d;
      nact += (d != 0.f) ? 1 : 0;
    }
  }
  __shared__ float red[8][DH_BLOCK / WAVE];
  __shared__ int cred[DH_BLOCK / WAVE];
  const int wave = threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float v = wave_sum(acc[q]);
    if (lane == 0) red[q][wave] = v;
  }
  nact = (int)wave_sum_u64((unsigned long long)(unsigned)nact);
  if (lane == 0) cred[wave] = nact;
  __syncthreads();
  if (a.blk_active && threadIdx.x == 0) {
    int c = 0;
    for (int w = 0; w < DH_BLOCK / WAVE; ++w) c += cred[w];
    a.blk_active[blockIdx.x] = c;
  }
  if (threadIdx.x < DH_PARTIAL) {
    float s = 0.f;
    if (threadIdx.x >= 2 && threadIdx.x < 10)
      for (int w = 0; w < DH_BLOCK / WAVE; ++w) s += red[threadIdx.x - 2][w];
    a.partial[(long)blockIdx.x * DH_PARTIAL + threadIdx.x] = s;
  }
}

// Active-evaluation list: the evaluations with a nonzero upstream gradient, in index order
// (every other evaluation contributes exactly zero to the weight and state gradients, so the
// backward skips it). Same block ranges as cbf_dh_kernel; blk_off = exclusive scan of its
// per-block counts.
// blk_off null: the block's offset is summed in-kernel from blk_active (cbf_dh's per-block
// counts) and the last block writes the total to *nact.
// rec (optional, the 16x16x32 x3 backward's input): instead of act, one 16-byte record per
// active evaluation {u, e | pass << 31, neighbour j, dh bits} -- the backward then needs no
// dependent index chain (act -> src -> idx -> states) inside its loop.
__global__ __launch_bounds__(DH_BLOCK) void cbf_compact_kernel(const float* dh, const int* nev, const int* blk_off,
                                                             int* act, const int* blk_active, int* nact,
                                                             const int* src, const int* idx, const int* idx1,
                                                             unsigned E, int4* rec) {
  const unsigned U = (unsigned)*nev;
  const unsigned span = dh_span(U, gridDim.x);
  const unsigned u_lo = blockIdx.x * span, u_hi = min(U, u_lo + span);
  const int wave = threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
  int base;
  if (blk_off) {
    base = blk_off[blockIdx.x];
  } else {
    base = block_sum_prefix<DH_BLOCK>(blk_active, blockIdx.x);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0 && nact) *nact = base + blk_active[blockIdx.x];
  }
  // CP_U rows of DH_BLOCK evaluations per round: their dh loads, then (for the active ones) the
  // source and neighbour-index loads, are in flight together, and one barrier pair serves the
  // round -- the same output order (u ascending) as one row per round (round 6: a row per round
  // was one dependent chain of three loads and two barriers per 256 evaluations, ~75 us at the
  // headline)
  constexpr int CP_U = 4;
  __shared__ int wcu[CP_U][DH_BLOCK / WAVE];
  for (unsigned u0 = u_lo; u0 < u_hi; u0 += CP_U * DH_BLOCK) {
    float dv[CP_U];
    bool f[CP_U];
    int below[CP_U];
#pragma unroll
    for (int r = 0; r < CP_U; ++r) {
      const unsigned u = u0 + r * DH_BLOCK + threadIdx.x;
      dv[r] = u < u_hi ? dh[u] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < CP_U; ++r) {
      f[r] = dv[r] != 0.f;
      const unsigned long long bal = __ballot(f[r]);
      below[r] = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) wcu[r][wave] = __popcll(bal);
    }
    // the records' source / neighbour indices, requested before the barrier
    unsigned ev[CP_U];
    int jn[CP_U];
    if (rec) {
      unsigned e0[CP_U];
#pragma unroll
      for (int r = 0; r < CP_U; ++r) {
        const unsigned u = u0 + r * DH_BLOCK + threadIdx.x;
        const unsigned pass = u >= E ? 1u : 0u;
        e0[r] = (f[r] && pass) ? (unsigned)src[u] : (f[r] ? u : 0u);
      }
#pragma unroll
      for (int r = 0; r < CP_U; ++r) {
        const unsigned u = u0 + r * DH_BLOCK + threadIdx.x;
        const unsigned pass = u >= E ? 1u : 0u;
        ev[r] = e0[r] | (pass << 31);
        jn[r] = f[r] ? ((pass && idx1) ? idx1 : idx)[e0[r]] : 0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < CP_U; ++r) {
      int wo = 0, tot = 0;
      for (int w = 0; w < DH_BLOCK / WAVE; ++w) {
        const int c = wcu[r][w];
        wo += (w < wave) ? c : 0;
        tot += c;
      }
      if (f[r]) {
        const unsigned u = u0 + r * DH_BLOCK + threadIdx.x;
        if (rec) rec[base + wo + below[r]] = int4{(int)u, (int)ev[r], jn[r], __float_as_int(dv[r])};
        else act[base + wo + below[r]] = (int)u;
      }
      base += tot;
    }
    __syncthreads();
  }
}

}  // namespace mb

extern "C" int mb_cbf_compact(const float* dh, const int* nev, const int* blk_off, int* act, int num_blocks,
                              const int* blk_active, int* nact, const int* src, const int* idx, const int* idx1,
                              unsigned E, void* rec, hipStream_t st) {
  using namespace mb;
  if (!blk_off && !blk_active) return -1;
  if (rec && (!src || !idx)) return -2;
  if (!rec && !act) return -3;
  hipLaunchKernelGGL(cbf_compact_kernel, dim3(num_blocks), dim3(DH_BLOCK), 0, st, dh, nev, blk_off, act, blk_active,
                     nact, src, idx, idx1, E, (int4*)rec);
  return (int)hipGetLastError();
}

extern "C" int mb_cbf_match(const mb::CbfMatchArgs* a, hipStream_t st) {
  using namespace mb;
  if (a->K < 1 || a->K > 16 || a->T < 1) return -1;
  const long rows = (long)a->T * a->B * a->N;
  hipLaunchKernelGGL(cbf_match_kernel, dim3((unsigned)((rows + MATCH_BLOCK - 1) / MATCH_BLOCK)), dim3(MATCH_BLOCK),
                     0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_cbf_dh(const mb::CbfDhArgs* a, int num_blocks, hipStream_t st) {
  using namespace mb;
  hipLaunchKernelGGL(cbf_dh_kernel, dim3(num_blocks), dim3(DH_BLOCK), 0, st, *a);
  return (int)hipGetLastError();
}
