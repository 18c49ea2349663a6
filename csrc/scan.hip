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

constexpr int SCAN_TILE = 1024;
constexpr int SCAN_BLOCK = 256;

template <int K>
__global__ __launch_bounds__(SCAN_BLOCK) void scan_kernel(ScanArgs a) {
  __shared__ float4 tile[SCAN_TILE];
  __shared__ float red[3][SCAN_BLOCK / WAVE];
  const int b = blockIdx.y;
  const int i = blockIdx.x * SCAN_BLOCK + threadIdx.x;
  const bool act = i < a.N;
  const float4* Sb = a.S + (long)b * a.s_env;
  const float4 si = act ? Sb[i] : make_float4(0.f, 0.f, 0.f, 0.f);

  float bd[K];
  int bi[K];
#pragma unroll
  for (int q = 0; q < K; ++q) { bd[q] = INFINITY; bi[q] = 0; }
  bool danger = false;

  for (int base = 0; base < a.N; base += SCAN_TILE) {
    const int n = min(SCAN_TILE, a.N - base);
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += SCAN_BLOCK) tile[q] = Sb[base + q];
    __syncthreads();
    if (!act) continue;
    for (int jj = 0; jj < n; ++jj) {
      const float4 sj = tile[jj];
      const float dx = si.x - sj.x;
      const float dy = si.y - sj.y;
      if (a.do_knn) {
        const float d2 = dx * dx + dy * dy;
        if (d2 < bd[K - 1]) {
          const int j = base + jj;
#pragma unroll
          for (int q = K - 1; q >= 1; --q) {
            const bool sh = d2 < bd[q - 1];
            const bool here = !sh && (d2 < bd[q]);
            const float nd = sh ? bd[q - 1] : (here ? d2 : bd[q]);
            const int ni = sh ? bi[q - 1] : (here ? j : bi[q]);
            bd[q] = nd;
            bi[q] = ni;
          }
          if (d2 < bd[0]) { bd[0] = d2; bi[0] = j; }
        }
      }
      if (a.do_safety && !danger && (base + jj) != i) {
        danger = ttc_danger(dx, dy, si.z - sj.z, si.w - sj.w, a.r2_check, a.ttc_check);
      }
    }
  }

  float ndang = 0.f, nsafe_e = 0.f, safe_ag = 0.f;
  if (act && a.do_knn) {
    int* out = a.idx + (long)b * a.i_env + (long)i * K;
    uint8_t* dout = a.dang ? a.dang + (long)b * a.i_env + (long)i * K : nullptr;
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const int j = bi[q];
      out[q] = j;
      const float4 sj = Sb[j];
      const float eye = (j == i) ? 1.f : 0.f;
      const bool d = ttc_danger((si.x - sj.x) + eye, (si.y - sj.y) + eye, si.z - sj.z, si.w - sj.w,
                                a.r2_train, a.ttc_train);
      if (dout) dout[q] = d ? 1 : 0;
      ndang += d ? 1.f : 0.f;
    }
    nsafe_e = (float)K - ndang;
  }
  if (act && a.do_safety) safe_ag = danger ? 0.f : 1.f;

  ndang = wave_sum(ndang);
  nsafe_e = wave_sum(nsafe_e);
  safe_ag = wave_sum(safe_ag);
  const int w = threadIdx.x / WAVE;
  if ((threadIdx.x & 63) == 0) { red[0][w] = ndang; red[1][w] = nsafe_e; red[2][w] = safe_ag; }
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
  hipLaunchKernelGGL(scan_kernel<K>, grid, dim3(SCAN_BLOCK), 0, st, a);
}

}  // namespace mb

extern "C" int mb_scan(const mb::ScanArgs* a, hipStream_t st) {
  using namespace mb;
  switch (a->do_knn ? a->K : 1) {
#define CASE(k) case k: launch_k<k>(*a, st); break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default: return -1;
  }
  return (int)hipGetLastError();
}
