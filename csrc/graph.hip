// Edge -> node gradient reduction without float atomics (deterministic), gfx950.
//
// A kNN graph is not symmetric, so dL/d(s_i - s_j) of edge (i -> slot k -> j) must be added
// to s_i and subtracted from s_j. Instead of per-edge atomics (64 lanes hitting 64 random
// rows = the slowest atomic shape on CDNA4), each timestep graph gets a reverse CSR (incoming
// edges per target, sorted by edge id), and one thread per agent gathers
//   G_i = sum_k dE[i,k] - sum_{e in in(i)} dE[e]
// in a fixed order. rev_csr_kernel builds the CSR for all B*T graphs in one launch
// (one workgroup per graph, LDS counting sort).
#include "common.h"
#include "args.h"
#include "state.h"
#include "combine.h"

namespace mb {

constexpr int CSR_BLOCK = 256;

// LDS_SORT (N*K <= 65536): the buckets are scattered into a 16-bit LDS buffer, insertion-sorted
// there and written out coalesced; otherwise they are scattered / sorted in global memory.
template <bool LDS_SORT>
__global__ __launch_bounds__(CSR_BLOCK) void rev_csr_kernel(CsrArgs a) {
  extern __shared__ __attribute__((aligned(16))) int sm[];
  const int Nt = a.Nn > 0 ? a.Nn : a.N;   // target nodes (agents + obstacle points)
  int* cnt = sm;                 // Nt + 1
  int* fill = sm + Nt + 1;       // Nt
  unsigned short* buf = reinterpret_cast<unsigned short*>(fill + Nt);   // LDS_SORT: N*K edge ids
  __shared__ int wsum[CSR_BLOCK];
  const long g = blockIdx.x;
  const int N = a.N, K = a.K, NK = N * K;
  const int* idx = a.idx + g * NK;
  for (int q = threadIdx.x; q <= Nt; q += CSR_BLOCK) cnt[q] = 0;
  for (int q = threadIdx.x; q < Nt; q += CSR_BLOCK) fill[q] = 0;
  __syncthreads();
  for (int e = threadIdx.x; e < NK; e += CSR_BLOCK) {
    const int j = idx[e];
    if (j != e / K) atomicAdd(&cnt[j + 1], 1);
  }
  __syncthreads();
  // exclusive scan of cnt[1..Nt] into cnt[0..Nt] (two-level: per-thread segment, then totals)
  const int seg = (Nt + CSR_BLOCK - 1) / CSR_BLOCK;
  const int lo = threadIdx.x * seg + 1, hi = min(lo + seg, Nt + 1);
  int run = 0;
  for (int q = lo; q < hi; ++q) { run += cnt[q]; cnt[q] = run; }
  wsum[threadIdx.x] = run;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < CSR_BLOCK; ++w) { const int v = wsum[w]; wsum[w] = acc; acc += v; }
  }
  __syncthreads();
  const int off = wsum[threadIdx.x];
  for (int q = lo; q < hi; ++q) cnt[q] += off;
  __syncthreads();
  int* ptr = a.ptr + g * (Nt + 1);
  for (int q = threadIdx.x; q <= Nt; q += CSR_BLOCK) ptr[q] = cnt[q];
  int* out = a.edges + g * NK;
  for (int e = threadIdx.x; e < NK; e += CSR_BLOCK) {
    const int j = idx[e];
    if (j != e / K) {
      const int p = atomicAdd(&fill[j], 1);
      if constexpr (LDS_SORT) buf[cnt[j] + p] = (unsigned short)e;
      else out[cnt[j] + p] = e;
    }
  }
  if constexpr (!LDS_SORT) __threadfence();     // global fill writes visible to the block
  __syncthreads();
  // deterministic order inside each bucket: insertion sort by edge id
  for (int j = threadIdx.x; j < Nt; j += CSR_BLOCK) {
    const int b0 = cnt[j], b1 = cnt[j + 1];
    for (int x = b0 + 1; x < b1; ++x) {
      if constexpr (LDS_SORT) {
        const unsigned short v = buf[x];
        int y = x - 1;
        while (y >= b0 && buf[y] > v) { buf[y + 1] = buf[y]; --y; }
        buf[y + 1] = v;
      } else {
        const int v = out[x];
        int y = x - 1;
        while (y >= b0 && out[y] > v) { out[y + 1] = out[y]; --y; }
        out[y + 1] = v;
      }
    }
  }
  if constexpr (LDS_SORT) {
    __syncthreads();
    const int tot = cnt[Nt];
    for (int q = threadIdx.x; q < tot; q += CSR_BLOCK) out[q] = buf[q];
  }
}

// Register-held path (the default where its LDS fits: the headline's 1024 x 12 graphs): the same
// CSR as rev_csr_kernel<true> with its two latency chains removed -- every thread requests all of
// its (<= CSR_JM) targets at once and keeps them in registers for the count and scatter passes
// (instead of one dependent global load per loop trip, twice), and the bucket offsets come from a
// wave-shuffle scan instead of one thread's serial pass over the 256 segment totals. 153 -> 134 us
// per headline iteration (profiles/r6_runs/r6r/). (Placing each edge by counting the smaller ids
// in its bucket, instead of the insertion sort, measured 240 us: divergent bucket loops, r6q.)
constexpr int CSR_RB = 512;
constexpr int CSR_JM = 32;           // edges per thread held in registers: N*K <= CSR_JM * CSR_RB
__global__ __launch_bounds__(CSR_RB) void rev_csr_reg_kernel(CsrArgs a) {
  extern __shared__ __attribute__((aligned(16))) int sm[];
  __shared__ int wsum[CSR_RB / WAVE];
  const int Nt = a.Nn > 0 ? a.Nn : a.N;
  const int N = a.N, K = a.K, NK = N * K;
  int* cnt = sm;                                                   // Nt + 1
  int* fill = sm + Nt + 1;                                         // Nt
  unsigned short* buf = reinterpret_cast<unsigned short*>(fill + Nt);   // NK, bucketed
  const long g = blockIdx.x;
  const int* idx = a.idx + g * NK;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid / WAVE;
  // source agent e / K = umulhi(e, ceil(2^32 / K)): exact for e < 2^16, 2 <= K <= 16
  const unsigned invK = K == 1 ? 0u : (unsigned)((0x100000000ull + (unsigned)K - 1u) / (unsigned)K);
  auto src = [&](int e) { return K == 1 ? e : (int)__umulhi((unsigned)e, invK); };
  // this thread's edges e = tid + u CSR_RB: every target requested at once (one memory latency,
  // not one per loop trip), kept in registers for the three passes; -1 = none / self edge
  int jv[CSR_JM];
#pragma unroll
  for (int u = 0; u < CSR_JM; ++u) {
    const int e = tid + u * CSR_RB;
    jv[u] = e < NK ? idx[e] : -1;
  }
  for (int q = tid; q <= Nt; q += CSR_RB) cnt[q] = 0;
  for (int q = tid; q < Nt; q += CSR_RB) fill[q] = 0;
#pragma unroll
  for (int u = 0; u < CSR_JM; ++u) {
    const int e = tid + u * CSR_RB;
    if (jv[u] == src(e)) jv[u] = -1;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < CSR_JM; ++u)
    if (jv[u] >= 0) atomicAdd(&cnt[jv[u] + 1], 1);
  __syncthreads();
  // exclusive scan of cnt[1..Nt] into cnt[0..Nt]: per-thread segment, wave shuffle scan of the
  // segment totals, then the waves' totals
  const int seg = (Nt + CSR_RB - 1) / CSR_RB;
  const int lo = tid * seg + 1, hi = min(lo + seg, Nt + 1);
  int run = 0;
  for (int q = lo; q < hi; ++q) { run += cnt[q]; cnt[q] = run; }
  int inc = run;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    const int v = __shfl_up(inc, o, WAVE);
    if (lane >= o) inc += v;
  }
  if (lane == WAVE - 1) wsum[wave] = inc;
  __syncthreads();
  int off = inc - run;
  for (int w = 0; w < wave; ++w) off += wsum[w];
  for (int q = lo; q < hi; ++q) cnt[q] += off;
  __syncthreads();
  int* ptr = a.ptr + g * (Nt + 1);
  for (int q = tid; q <= Nt; q += CSR_RB) ptr[q] = cnt[q];
#pragma unroll
  for (int u = 0; u < CSR_JM; ++u)
    if (jv[u] >= 0) buf[cnt[jv[u]] + atomicAdd(&fill[jv[u]], 1)] = (unsigned short)(tid + u * CSR_RB);
  __syncthreads();
  // deterministic order inside each bucket: insertion sort by edge id (one thread per bucket)
  for (int j = tid; j < Nt; j += CSR_RB) {
    const int b0 = cnt[j], b1 = cnt[j + 1];
    for (int x = b0 + 1; x < b1; ++x) {
      const unsigned short v = buf[x];
      int y = x - 1;
      while (y >= b0 && buf[y] > v) { buf[y + 1] = buf[y]; --y; }
      buf[y + 1] = v;
    }
  }
  __syncthreads();
  int* out = a.edges + g * NK;
  const int tot = cnt[Nt];
  for (int q = tid; q < tot; q += CSR_RB) out[q] = buf[q];
}

// Global path (envs whose 2 Nn + 1 counters exceed LDS, > ~19 K nodes): counters in global
// memory -- the counts in the ptr output itself, scanned in LDS tiles of CSR_TILE entries with a
// running carry, the bucket fill counters in a.ws; the buckets are scattered and insertion-sorted
// in global memory. Values another thread wrote are read with agent-scope atomic loads after a
// fence + barrier (they come from L2: this CU's L1 may hold a stale line of them).
constexpr int CSR_TILE = 4096;
DEV int ld_l2(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__global__ __launch_bounds__(CSR_BLOCK) void rev_csr_glb_kernel(CsrArgs a) {
  __shared__ int tile[CSR_TILE];
  __shared__ int wsum[CSR_BLOCK];
  const int Nt = a.Nn > 0 ? a.Nn : a.N;
  const long g = blockIdx.x;
  const int N = a.N, K = a.K, NK = N * K;
  const int* idx = a.idx + g * NK;
  int* cnt = a.ptr + g * (Nt + 1);
  int* fill = a.ws + g * Nt;
  int* out = a.edges + g * NK;
  for (int q = threadIdx.x; q <= Nt; q += CSR_BLOCK) cnt[q] = 0;
  for (int q = threadIdx.x; q < Nt; q += CSR_BLOCK) fill[q] = 0;
  __threadfence();
  __syncthreads();
  for (int e = threadIdx.x; e < NK; e += CSR_BLOCK) {
    const int j = idx[e];
    if (j != e / K) atomicAdd(&cnt[j + 1], 1);
  }
  __threadfence();
  __syncthreads();
  // exclusive scan of cnt[1..Nt] (cnt[0] stays 0), tile by tile with a running carry
  __shared__ int total;
  int carry = 0;
  constexpr int PER = CSR_TILE / CSR_BLOCK;
  for (int base = 1; base <= Nt; base += CSR_TILE) {
    const int n = min(CSR_TILE, Nt + 1 - base);
    for (int q = threadIdx.x; q < n; q += CSR_BLOCK) tile[q] = ld_l2(&cnt[base + q]);
    __syncthreads();
    int run = 0;
    const int lo = threadIdx.x * PER, hi = min(lo + PER, n);
    for (int q = lo; q < hi; ++q) { run += tile[q]; tile[q] = run; }
    wsum[threadIdx.x] = run;
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = carry;
      for (int w = 0; w < CSR_BLOCK; ++w) { const int v = wsum[w]; wsum[w] = acc; acc += v; }
      total = acc;
    }
    __syncthreads();
    const int off = wsum[threadIdx.x];
    for (int q = lo; q < hi; ++q) cnt[base + q] = tile[q] + off;
    carry = total;
    __syncthreads();                               // tile / wsum are reused by the next tile
  }
  __threadfence();
  __syncthreads();
  for (int e = threadIdx.x; e < NK; e += CSR_BLOCK) {
    const int j = idx[e];
    if (j != e / K) {
      const int p = atomicAdd(&fill[j], 1);
      out[ld_l2(&cnt[j]) + p] = e;
    }
  }
  __threadfence();
  __syncthreads();
  for (int j = threadIdx.x; j < Nt; j += CSR_BLOCK) {
    const int b0 = ld_l2(&cnt[j]), b1 = ld_l2(&cnt[j + 1]);
    if (b1 - b0 < 2) continue;
    // the bucket's entries were written by other threads: read them from L2 once, then sort in
    // place with this thread's own stores
    for (int x = b0 + 1; x < b1; ++x) {
      const int v = ld_l2(&out[x]);
      int y = x - 1;
      int w;
      while (y >= b0 && (w = ld_l2(&out[y])) > v) { out[y + 1] = w; __threadfence(); --y; }
      out[y + 1] = v;
      __threadfence();
    }
  }
}

constexpr bool NODE_RED_XCD = true;
// out[t', b, i] (+)= sum over passes p of [ sum_k dE_p[t'-p, b, i, k] - sum_{e in in(i)} dE_p[e] ]
// for the N agents (obstacle nodes receive no gradient). Records of REC<D> float4.
// NRL lanes per node (round 6; was 16): a node's K out-slots and its in-edges form one slot list,
// dealt to the lanes NRL apart and consumed NRB slots per lane at a time -- every load of a batch
// (in-edge index -> dedup map -> gate -> record) is requested for all NRB slots before the next
// stage needs it, so a lane keeps up to NRB records in flight instead of one dependent chain per
// slot, and the grid has a quarter of the threads (the 16-lane version ran ~38 rounds of full
// occupancy at the headline, 297 us, each paying the chain's 4-5 memory latencies). Fixed slot
// order per lane and a fixed xor butterfly: deterministic.
constexpr int NRL = 4, NRB = 4;
template <int D>
__global__ __launch_bounds__(256) void node_reduce_kernel(NodeRedArgs a) {
  const int t_hi = a.t_hi ? a.t_hi : a.T + 1;
  // one graph's nodes on one XCD: the in-edge gathers read the records the graph's out-edge reads
  // just brought into that XCD's L2
  const int lb = NODE_RED_XCD ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const long node = (long)a.t_lo * a.B * a.N + ((long)lb * blockDim.x + threadIdx.x) / NRL;
  const int l = threadIdx.x % NRL;
  const long total = (long)a.B * t_hi * a.N;
  if (node >= total) return;             // whole lane groups
  // time-major: out[(t'*B + b)*N + i], graphs g = t*B + b
  const int i = (int)(node % a.N);
  const long tb = node / a.N;
  const int tp = (int)(tb / a.B);
  const int b = (int)(tb - (long)tp * a.B);
  const int N = a.N, K = a.K;
  const int Nt = a.Nn > 0 ? a.Nn : N;
  const long E = (long)a.B * a.T * N * K;
  const int NK = N * K;
  constexpr int R = REC<D>;
  float4 g[R];
#pragma unroll
  for (int q = 0; q < R; ++q) g[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int pass = 0; pass < a.passes; ++pass) {
    if (a.pass_mask && !((a.pass_mask >> pass) & 1)) continue;
    const int t = tp - pass;
    if (t < 0 || t >= a.T) continue;
    const long ge = (long)t * a.B + b;                          // edge block of step t
    const long gi = ge + (pass == 1 ? (long)a.shift1 * a.B : 0);  // graph (CSR) the edges live in
    const int* ptr = a.ptr + gi * (Nt + 1);
    const int* edges = a.edges + gi * (long)NK;
    const int q0 = ptr[i], q1 = ptr[i + 1];
    // deduplicated evaluations: only the extras (map1 >= E) carry a pass-1 gradient; the matched
    // slots' h' gradient is part of the next step's main evaluation (pass 0)
    const bool dd = pass == 1 && a.map1;
    const int* mp = dd ? a.map1 + ge * NK : nullptr;
    const long eb = pass * E + ge * NK;                          // (non-dedup) record base of this block
    const int nsl = K + (q1 - q0);                              // out-slots, then in-edges
    for (int s0 = 0; s0 < nsl; s0 += NRL * NRB) {
      int loc[NRB];
      bool on[NRB], outs[NRB];
#pragma unroll
      for (int u = 0; u < NRB; ++u) {              // slot -> local edge index (in-edges: a load)
        const int sl = s0 + l + u * NRL;
        outs[u] = sl < K;
        on[u] = sl < nsl;
        const int q = min(q0 + max(sl - K, 0), NK - 1);
        const int e = edges[q];                    // clamped, unconditional
        loc[u] = outs[u] ? i * K + sl : e;
      }
      long x[NRB];
#pragma unroll
      for (int u = 0; u < NRB; ++u) {              // local edge -> evaluation index (dedup: a load)
        if (dd) {
          const int m = mp[min(max(loc[u], 0), NK - 1)];
          on[u] = on[u] && m >= E;
          x[u] = on[u] ? (long)m : 0;
        } else {
          x[u] = eb + loc[u];
        }
      }
      float gv[NRB];
#pragma unroll
      for (int u = 0; u < NRB; ++u) gv[u] = a.gate ? a.gate[on[u] ? x[u] : 0] : 1.f;
      float4 v[NRB][R];
#pragma unroll
      for (int u = 0; u < NRB; ++u) {
        // a zero gate: the record was never written (the active-list backward skips it)
        const bool rd = on[u] && gv[u] != 0.f;
#pragma unroll
        for (int q = 0; q < R; ++q) v[u][q] = rd ? a.dE[x[u] * R + q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < NRB; ++u) {
        if (outs[u]) acc_rec_v<R, 1>(g, v[u]);
        else acc_rec_v<R, -1>(g, v[u]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    g[q].x += lane_xorf<2>(g[q].x); g[q].y += lane_xorf<2>(g[q].y);
    g[q].z += lane_xorf<2>(g[q].z); g[q].w += lane_xorf<2>(g[q].w);
    g[q].x += lane_xorf<1>(g[q].x); g[q].y += lane_xorf<1>(g[q].y);
    g[q].z += lane_xorf<1>(g[q].z); g[q].w += lane_xorf<1>(g[q].w);
  }
  if (l != 0) return;
  float4* o = a.out + (((long)tp * a.B + b) * N + i) * R;
  if (a.accumulate) acc_rec<R, 1>(g, o);
#pragma unroll
  for (int q = 0; q < R; ++q) o[q] = g[q];
}

template <int D>
__global__ __launch_bounds__(256) void node_combine_kernel(CombineArgs a) {
  const long node = ((long)blockIdx.x * blockDim.x + threadIdx.x) / RG;
  if (node >= (long)a.B * a.N) return;   // whole 16-lane groups
  combine_node<D>(a, node, threadIdx.x % RG);
}

}  // namespace mb

extern "C" int mb_rev_csr(const mb::CsrArgs* a, hipStream_t st) {
  using namespace mb;
  const int Nt = a->Nn > 0 ? a->Nn : a->N;
  const long NK = (long)a->N * a->K;
  const size_t base = (size_t)(2 * Nt + 1) * 4;
  const size_t lds_sorted = base + (size_t)NK * 2;
  const size_t lds_reg = base + (size_t)NK * 2;
  // (small graphs keep the 256-thread kernel: 32 x 12 edges, config #2, 18 vs 28 us per launch)
  if (NK >= 4096 && NK <= CSR_JM * CSR_RB && lds_reg <= 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)rev_csr_reg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_reg);
    hipLaunchKernelGGL(rev_csr_reg_kernel, dim3(a->G), dim3(CSR_RB), lds_reg, st, *a);
  } else if (NK <= 65536 && lds_sorted <= 150 * 1024) {
    (void)hipFuncSetAttribute((const void*)rev_csr_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sorted);
    hipLaunchKernelGGL(rev_csr_kernel<true>, dim3(a->G), dim3(CSR_BLOCK), lds_sorted, st, *a);
  } else if (base <= 150 * 1024) {
    (void)hipFuncSetAttribute((const void*)rev_csr_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)base);
    hipLaunchKernelGGL(rev_csr_kernel<false>, dim3(a->G), dim3(CSR_BLOCK), base, st, *a);
  } else {
    if (!a->ws) return -2;                       // global path: the caller provides (G, Nn) ints
    hipLaunchKernelGGL(rev_csr_glb_kernel, dim3(a->G), dim3(CSR_BLOCK), 0, st, *a);
  }
  return (int)hipGetLastError();
}

extern "C" int mb_node_reduce(const mb::NodeRedArgs* a, hipStream_t st) {
  using namespace mb;
  const int t_hi = a->t_hi ? a->t_hi : a->T + 1;
  if (a->t_lo < 0 || t_hi > a->T + 1 || a->t_lo >= t_hi) return -1;
  const long total = (long)a->B * (t_hi - a->t_lo) * a->N * NRL;
  if (a->dim == 3) hipLaunchKernelGGL(node_reduce_kernel<3>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(node_reduce_kernel<2>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_node_combine(const mb::CombineArgs* a, hipStream_t st) {
  using namespace mb;
  const long total = (long)a->B * a->N * RG;
  if (a->dim == 3) hipLaunchKernelGGL(node_combine_kernel<3>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(node_combine_kernel<2>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}
