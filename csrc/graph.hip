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

namespace mb {

constexpr int CSR_BLOCK = 256;

__global__ __launch_bounds__(CSR_BLOCK) void rev_csr_kernel(CsrArgs a) {
  extern __shared__ __attribute__((aligned(16))) int sm[];
  const int Nt = a.Nn > 0 ? a.Nn : a.N;   // target nodes (agents + obstacle points)
  int* cnt = sm;                 // Nt + 1
  int* fill = sm + Nt + 1;       // Nt
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
      out[cnt[j] + p] = e;
    }
  }
  __threadfence();     // fill writes visible before other threads of the block sort them
  __syncthreads();
  // deterministic order inside each bucket: insertion sort by edge id
  for (int j = threadIdx.x; j < Nt; j += CSR_BLOCK) {
    const int b0 = cnt[j], b1 = cnt[j + 1];
    for (int x = b0 + 1; x < b1; ++x) {
      const int v = out[x];
      int y = x - 1;
      while (y >= b0 && out[y] > v) { out[y + 1] = out[y]; --y; }
      out[y + 1] = v;
    }
  }
}

// dS[b, t', i] (+)= reduce of pass-0 edges of graph (b,t') and pass-1 edges of graph (b,t'-1),
// for the N agents (obstacle nodes receive no gradient). Records of REC<D> float4.
template <int D>
__global__ __launch_bounds__(256) void node_reduce_kernel(NodeRedArgs a) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)a.B * (a.T + 1) * a.N;
  if (tid >= total) return;
  // time-major: out[(t'*B + b)*N + i], graphs g = t*B + b
  const int i = (int)(tid % a.N);
  const long tb = tid / a.N;
  const int tp = (int)(tb / a.B);
  const int b = (int)(tb - (long)tp * a.B);
  const int N = a.N, K = a.K;
  const int Nt = a.Nn > 0 ? a.Nn : N;
  const long E = (long)a.B * a.T * N * K;
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
    const float4* dE = a.dE + ((long)pass * E + ge * N * K) * R;
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const float4 v = dE[((long)i * K + k) * R + q];
        g[q].x += v.x; g[q].y += v.y; g[q].z += v.z; g[q].w += v.w;
      }
    }
    const int* ptr = a.ptr + gi * (Nt + 1);
    const int* edges = a.edges + gi * (long)N * K;
    const int q0 = ptr[i], q1 = ptr[i + 1];
    // incoming edges in batches of 4: the 4 edge ids, then the 4 independent record loads
    // (fixed order: the sum is the same as the one-by-one loop)
    int q2 = q0;
    for (; q2 + 4 <= q1; q2 += 4) {
      int e4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) e4[u] = edges[q2 + u];
      float4 v4[4][R];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < R; ++q) v4[u][q] = dE[(long)e4[u] * R + q];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < R; ++q) {
          g[q].x -= v4[u][q].x; g[q].y -= v4[u][q].y; g[q].z -= v4[u][q].z; g[q].w -= v4[u][q].w;
        }
    }
    for (; q2 < q1; ++q2) {
      const int e = edges[q2];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const float4 v = dE[(long)e * R + q];
        g[q].x -= v.x; g[q].y -= v.y; g[q].z -= v.z; g[q].w -= v.w;
      }
    }
  }
  float4* o = a.out + (((long)tp * a.B + b) * N + i) * R;
#pragma unroll
  for (int q = 0; q < R; ++q) {
    float4 v = g[q];
    if (a.accumulate) {
      const float4 p = o[q];
      v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
    }
    o[q] = v;
  }
}

// One reverse-time step of the BPTT recursion (train.py:58-103 through autograd in the
// reference; hand-derived here):
//   G_t = dS_direct[t] + ego_t + sum_k dEc[i,k] - sum_in dEc[e]
//         + Euler adjoint of s_{t+1} = s_t + dt [v_t, a_t]  (if bptt)
template <int D>
__global__ __launch_bounds__(256) void node_combine_kernel(CombineArgs a) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (long)a.B * a.N) return;
  const int b = (int)(tid / a.N), i = (int)(tid % a.N);
  const int N = a.N, K = a.K;
  float gp[D], gv[D], p[D], v[D];
  load_rec<D>(a.dS + (long)b * a.ds_env * REC<D>, (unsigned)i, gp, gv);
  if (a.ego) {
    load_rec<D>(a.ego + (long)b * N * REC<D>, (unsigned)i, p, v);
#pragma unroll
    for (int q = 0; q < D; ++q) { gp[q] += p[q]; gv[q] += v[q]; }
  }
  if (a.dEc) {
    const float4* dE = a.dEc + (long)b * N * K * REC<D>;
    for (int k = 0; k < K; ++k) {
      load_rec<D>(dE, (unsigned)(i * K + k), p, v);
#pragma unroll
      for (int q = 0; q < D; ++q) { gp[q] += p[q]; gv[q] += v[q]; }
    }
    const int* ptr = a.ptr + (long)b * a.ptr_env;
    const int* edges = a.edges + (long)b * a.edges_env;
    const int q0 = ptr[i], q1 = ptr[i + 1];
    int q2 = q0;
    for (; q2 + 4 <= q1; q2 += 4) {     // 4 ids, then 4 independent record loads (same sum order)
      int e4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) e4[u] = edges[q2 + u];
      float p4[4][D], v4[4][D];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_rec<D>(dE, (unsigned)e4[u], p4[u], v4[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < D; ++q) { gp[q] -= p4[u][q]; gv[q] -= v4[u][q]; }
    }
    for (; q2 < q1; ++q2) {
      load_rec<D>(dE, (unsigned)edges[q2], p, v);
#pragma unroll
      for (int q = 0; q < D; ++q) { gp[q] -= p[q]; gv[q] -= v[q]; }
    }
  }
  if (a.Gn) {
    // Euler adjoint of s_{t+1} = s_t + dt [v_t, a_t]: dp += G_p, dv += G_v + dt G_p
    load_rec<D>(a.Gn + (long)b * a.gn_env * REC<D>, (unsigned)i, p, v);
#pragma unroll
    for (int q = 0; q < D; ++q) { gp[q] += p[q]; gv[q] += v[q] + a.dt * p[q]; }
  }
  store_rec<D>(a.Gout + (long)b * a.go_env * REC<D>, (unsigned)i, gp, gv);
}

}  // namespace mb

extern "C" int mb_rev_csr(const mb::CsrArgs* a, hipStream_t st) {
  using namespace mb;
  const int Nt = a->Nn > 0 ? a->Nn : a->N;
  const size_t lds = (size_t)(2 * Nt + 1) * 4;
  if (lds > 150 * 1024) return -1;
  (void)hipFuncSetAttribute((const void*)rev_csr_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(rev_csr_kernel, dim3(a->G), dim3(CSR_BLOCK), lds, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_node_reduce(const mb::NodeRedArgs* a, hipStream_t st) {
  using namespace mb;
  const long total = (long)a->B * (a->T + 1) * a->N;
  if (a->dim == 3) hipLaunchKernelGGL(node_reduce_kernel<3>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(node_reduce_kernel<2>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_node_combine(const mb::CombineArgs* a, hipStream_t st) {
  using namespace mb;
  const long total = (long)a->B * a->N;
  if (a->dim == 3) hipLaunchKernelGGL(node_combine_kernel<3>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(node_combine_kernel<2>, dim3((total + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}
