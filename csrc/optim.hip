// Optimizer-side kernels, gfx950: deterministic reduction of per-workgroup weight-gradient
// slabs, and the fused flat Adam (torch.optim.Adam semantics, L2 weight decay) over one
// contiguous parameter range -- the two reference optimizers (train.py:36-37) are two ranges
// of the single flat fp32 master buffer.
#include "common.h"
#include "args.h"

namespace mb {

// out[c] (+)= sum_r partial[r * cols + c] in a fixed order (bitwise reproducible).
// Block = 16 float4-column groups x 16 row slices: slice y sums rows y, y+16, ... in order, then
// the 16 slice sums are added in slice order through LDS. ~300 workgroups for the CBF slab
// instead of 19 with one serial thread per column.
constexpr int RR_COLS = 16, RR_SLICES = 16;
__global__ __launch_bounds__(RR_COLS * RR_SLICES) void reduce_rows_kernel(const float* partial, int rows, int cols,
                                                                          float* out, int accumulate) {
  __shared__ float4 red[RR_SLICES][RR_COLS];
  const int cx = threadIdx.x % RR_COLS, sy = threadIdx.x / RR_COLS;
  const int c4 = blockIdx.x * RR_COLS + cx;
  const bool ok = c4 * 4 < cols;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
#pragma unroll 4
    for (int r = sy; r < rows; r += RR_SLICES) {
      const float4 v = *reinterpret_cast<const float4*>(partial + (long)r * cols + c4 * 4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[sy][cx] = s;
  __syncthreads();
  if (sy == 0 && ok) {
    float4 t = red[0][cx];
    for (int y = 1; y < RR_SLICES; ++y) {
      const float4 v = red[y][cx];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out + c4 * 4);
    if (accumulate) {
      const float4 p = *o;
      t.x += p.x; t.y += p.y; t.z += p.z; t.w += p.w;
    }
    *o = t;
  }
}

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const int i = a.lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.hi) return;
  float g = a.grad[i];
  float p = a.param[i];
  if (a.wd != 0.f) g = g + a.wd * p;
  float m = a.m[i], v = a.v[i];
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  a.m[i] = m;
  a.v[i] = v;
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  a.param[i] = p - a.step_size * (m / denom);
}

}  // namespace mb

extern "C" int mb_reduce_rows(const float* partial, int rows, int cols, float* out, int accumulate, hipStream_t st) {
  if (cols % 4) return -1;
  const int groups = cols / 4;
  hipLaunchKernelGGL(mb::reduce_rows_kernel, dim3((groups + mb::RR_COLS - 1) / mb::RR_COLS),
                     dim3(mb::RR_COLS * mb::RR_SLICES), 0, st, partial, rows, cols, out, accumulate);
  return (int)hipGetLastError();
}

extern "C" int mb_adam(const mb::AdamArgs* a, hipStream_t st) {
  const int n = a->hi - a->lo;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mb::adam_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}
