// K1: per-step all-pairs scan of one timestep graph (B envs x N agents), gfx950.
//
// One pass over all candidate agents j of the env (positions+velocities staged in LDS in
// 1024-agent tiles, read as wave-wide broadcasts) produces, per agent i:
//   * the top-K nearest neighbours (self at slot 0, ties -> lower index), kept sorted in
//     registers with a statically unrolled insertion (reference core.py:234-250, which
//     builds a dense (N,N,C) tensor and topk's it 3x per step -- never materialised here);
//   * the training TTC danger bit of each kept edge (core.py:187-209: r=DIST_MIN_THRES,
//     ttc=TIME_TO_COLLISION) and per-env dangerous/safe edge counts (loss normalisers);
//   * the all-pairs safety flag (core.py:212-231 / train.py:74-75: r=DIST_MIN_CHECK,
//     ttc=TIME_TO_COLLISION_CHECK) -> per-env count of safe agents.
// fp contraction is OFF in this file so distances / TTC decisions are bit-identical to the
// PyTorch oracle (separately rounded products, same association order).
#pragma clang fp contract(off)
#include "common.h"
#include "args.h"

namespace mb {


DEV bool ttc_danger(float x, float y, float vx, float vy, float r2, float ttc) {
  float alpha = vx * vx + vy * vy;
  float beta = 2.0f * (x * vx + y * vy);
  float gamma = x * x + y * y - r2;
  float disc = beta * beta - (4.0f * alpha) * gamma;
  bool dist_d = gamma < 0.f;
  bool two_pos = (disc > 0.f) && (gamma > 0.f) && (beta < 0.f);
  float t2 = (2.0f * alpha) * ttc;
  float bt = beta + t2;
  bool lt = ((-beta) - t2 < 0.f) || (bt * bt < disc);
  return dist_d || (two_pos && lt);
}

// ---------------------------------------------------------------------------------------
// Spatial ordering. The top-K insertion is wave-divergent: a wave pays for the 12-step
// insertion whenever ANY of its 64 lanes inserts. With agents in random order every
// candidate is an insertion for some lane. cell_sort_kernel orders each env's agents along a
// Morton curve (32x32 grid over the scenario square), so a wave's 64 agents are spatial
// neighbours; scan_kernel then visits candidates outward from the wave's own position on
// the curve, the lists converge within the first ~100 candidates and later candidates
// almost never insert. Results do not depend on the order: (d2, index) is compared
// lexicographically, so idx/dang/counts/safety are exactly those of the plain all-pairs scan.
// ---------------------------------------------------------------------------------------
constexpr int SORT_BLOCK = 1024;
constexpr int MORTON_BINS = 1024;

DEV unsigned spread5(unsigned v) {   // 5 bits -> every other bit
  v &= 31u;
  v = (v | (v << 8)) & 0x00FF00FFu;
  v = (v | (v << 4)) & 0x0F0F0F0Fu;
  v = (v | (v << 2)) & 0x33333333u;
  v = (v | (v << 1)) & 0x55555555u;
  return v;
}

__global__ __launch_bounds__(SORT_BLOCK) void cell_sort_kernel(CellSortArgs a) {
  __shared__ int hist[MORTON_BINS];
  __shared__ int wsum[SORT_BLOCK / WAVE];
  const int b = blockIdx.x;
  const float4* Sb = a.S + (long)b * a.s_env;
  for (int q = threadIdx.x; q < MORTON_BINS; q += SORT_BLOCK) hist[q] = 0;
  __syncthreads();
  const float inv = 32.f / a.L;
  for (int i = threadIdx.x; i < a.N; i += SORT_BLOCK) {
    const float4 s = Sb[i];
    const int cx = min(31, max(0, (int)(s.x * inv)));
    const int cy = min(31, max(0, (int)(s.y * inv)));
    atomicAdd(&hist[spread5(cx) | (spread5(cy) << 1)], 1);
  }
  __syncthreads();
  // exclusive scan of 1024 bins with 1024 threads: wave scan + wave totals
  const int lane = threadIdx.x & 63, w = threadIdx.x / WAVE;
  int v = hist[threadIdx.x];
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int q = 0; q < SORT_BLOCK / WAVE; ++q) { const int t = wsum[q]; wsum[q] = acc; acc += t; }
  }
  __syncthreads();
  hist[threadIdx.x] = x - v + wsum[w];
  __syncthreads();
  int* perm = a.perm + (long)b * a.N;
  for (int i = threadIdx.x; i < a.N; i += SORT_BLOCK) {
    const float4 s = Sb[i];
    const int cx = min(31, max(0, (int)(s.x * inv)));
    const int cy = min(31, max(0, (int)(s.y * inv)));
    const int p = atomicAdd(&hist[spread5(cx) | (spread5(cy) << 1)], 1);
    perm[p] = i;
  }
}

constexpr int SCAN_BLOCK = 256;      // 4 waves x 64 agents (consecutive on the Morton curve)
constexpr int SCAN_MAXN = 4096;      // whole env staged in LDS (24 B per agent)

template <int K>
DEV void topk_insert(float (&bd)[K], int (&bi)[K], float d2, int j) {
  // caller guarantees (d2, j) < (bd[K-1], bi[K-1]) lexicographically
#pragma unroll
  for (int q = K - 1; q >= 1; --q) {
    const bool sh = (d2 < bd[q - 1]) || (d2 == bd[q - 1] && j < bi[q - 1]);
    const bool here = !sh && ((d2 < bd[q]) || (d2 == bd[q] && j < bi[q]));
    const float nd = sh ? bd[q - 1] : (here ? d2 : bd[q]);
    const int ni = sh ? bi[q - 1] : (here ? j : bi[q]);
    bd[q] = nd;
    bi[q] = ni;
  }
  if ((d2 < bd[0]) || (d2 == bd[0] && j < bi[0])) { bd[0] = d2; bi[0] = j; }
}

template <int K>
__global__ __launch_bounds__(SCAN_BLOCK) void scan_kernel(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float4* tp = reinterpret_cast<float4*>(smem);               // sorted: x, y, |v|, agent id (bits)
  float2* tv = reinterpret_cast<float2*>(tp + a.N);           // sorted: vx, vy
  __shared__ float red[3][SCAN_BLOCK / WAVE];
  const int b = blockIdx.y;
  const int N = a.N;
  const float4* Sb = a.S + (long)b * a.s_env;
  const int* perm = a.perm + (long)b * N;
  for (int q = threadIdx.x; q < N; q += SCAN_BLOCK) {
    const int id = perm[q];
    const float4 s = Sb[id];
    tp[q] = make_float4(s.x, s.y, sqrtf(s.z * s.z + s.w * s.w), __int_as_float(id));
    tv[q] = make_float2(s.z, s.w);
  }
  __syncthreads();
  const int wave = threadIdx.x / WAVE, lane = threadIdx.x & 63;
  const int pos = blockIdx.x * SCAN_BLOCK + threadIdx.x;      // my position on the curve
  const bool act = pos < N;
  float4 me = make_float4(0.f, 0.f, 0.f, 0.f);
  float2 mv = make_float2(0.f, 0.f);
  int i = 0;
  if (act) {
    me = tp[pos];
    mv = tv[pos];
    i = __float_as_int(me.w);
  }
  const float rc = sqrtf(a.r2_check);
  // geometric pre-test for the safety check: dangerous => |p| < r + ttc*|v_i - v_j| <= r + ttc*(|v_i|+|v_j|)
  const float base_i = rc + a.ttc_check * me.z;
  float bd[K];
  int bi[K];
#pragma unroll
  for (int q = 0; q < K; ++q) { bd[q] = INFINITY; bi[q] = 0x7fffffff; }
  bool danger = false;
  // outward walk along the curve from the centre of this wave's 64 positions
  int c0 = blockIdx.x * SCAN_BLOCK + wave * WAVE + 32;
  if (c0 >= N) c0 = N - 1;
  if (act) {
    for (int d = 0; d < N; ++d) {
      const int off = (d + 1) >> 1;
      int p = (d & 1) ? c0 + off : c0 - off;
      if (p >= N) p -= N;
      if (p < 0) p += N;
      const float4 c = tp[p];
      const int j = __float_as_int(c.w);
      const float dx = me.x - c.x;
      const float dy = me.y - c.y;
      const float d2 = dx * dx + dy * dy;
      if (a.do_knn && ((d2 < bd[K - 1]) || (d2 == bd[K - 1] && j < bi[K - 1]))) topk_insert<K>(bd, bi, d2, j);
      if (a.do_safety && !danger) {
        const float lim = 1.01f * (base_i + a.ttc_check * c.z) + 1e-4f;
        if (d2 < lim * lim && j != i) {
          const float2 v = tv[p];
          danger = ttc_danger(dx, dy, mv.x - v.x, mv.y - v.y, a.r2_check, a.ttc_check);
        }
      }
    }
  }
  float ndang = 0.f, nsafe_e = 0.f, safe_ag = 0.f;
  if (act && a.do_knn) {
    int* out = a.idx + (long)b * a.i_env + (long)i * K;
    uint8_t* dout = a.dang ? a.dang + (long)b * a.i_env + (long)i * K : nullptr;
    const float4 si = Sb[i];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const int j = bi[q];
      out[q] = j;
      const float4 sj = Sb[j];
      const float eye = (j == i) ? 1.f : 0.f;
      const bool dg = ttc_danger((si.x - sj.x) + eye, (si.y - sj.y) + eye, si.z - sj.z, si.w - sj.w,
                                 a.r2_train, a.ttc_train);
      if (dout) dout[q] = dg ? 1 : 0;
      ndang += dg ? 1.f : 0.f;
    }
    nsafe_e = (float)K - ndang;
  }
  if (act && a.do_safety) safe_ag = danger ? 0.f : 1.f;
  ndang = wave_sum(ndang);
  nsafe_e = wave_sum(nsafe_e);
  safe_ag = wave_sum(safe_ag);
  if (lane == 0) { red[0][wave] = ndang; red[1][wave] = nsafe_e; red[2][wave] = safe_ag; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int q = 0; q < SCAN_BLOCK / WAVE; ++q) { s0 += red[0][q]; s1 += red[1][q]; s2 += red[2][q]; }
    if (a.do_knn && a.cnt) {
      atomicAdd(a.cnt + (long)b * a.c_env + 0, s0);
      atomicAdd(a.cnt + (long)b * a.c_env + 1, s1);
    }
    if (a.do_safety && a.safe) atomicAdd(a.safe + (long)b * a.sf_env, s2);
  }
}

template <int K>
static void launch_k(const ScanArgs& a, hipStream_t st) {
  dim3 grid((a.N + SCAN_BLOCK - 1) / SCAN_BLOCK, a.B);
  const size_t lds = (size_t)a.N * 24;
  (void)hipFuncSetAttribute((const void*)scan_kernel<K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(scan_kernel<K>, grid, dim3(SCAN_BLOCK), lds, st, a);
}

}  // namespace mb

extern "C" int mb_cell_sort(const mb::CellSortArgs* a, hipStream_t st) {
  using namespace mb;
  hipLaunchKernelGGL(cell_sort_kernel, dim3(a->B), dim3(SORT_BLOCK), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" int mb_scan(const mb::ScanArgs* a, hipStream_t st) {
  using namespace mb;
  if (a->N > SCAN_MAXN || !a->perm) return -3;
  switch (a->do_knn ? a->K : 1) {
#define CASE(k) case k: launch_k<k>(*a, st); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default: return -1;
  }
  return (int)hipGetLastError();
}
