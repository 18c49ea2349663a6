// Optimizer-side kernels, gfx950: deterministic reduction of per-workgroup weight-gradient
// slabs, and the fused flat Adam (torch.optim.Adam semantics, L2 weight decay) over one
// contiguous parameter range -- the two reference optimizers (train.py:36-37) are two ranges
// of the single flat fp32 master buffer.
#include "common.h"
#include "args.h"

namespace mb {

// out[c] (+)= sum_r partial[r * cols + c], fixed row order (bitwise reproducible)
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* partial, int rows, int cols, float* out,
                                                          int accumulate) {
  const int c4 = blockIdx.x * blockDim.x + threadIdx.x;   // one float4 column group per thread
  if (c4 * 4 >= cols) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < rows; ++r) {
    const float4 v = *reinterpret_cast<const float4*>(partial + (long)r * cols + c4 * 4);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float4* o = reinterpret_cast<float4*>(out + c4 * 4);
  if (accumulate) {
    const float4 p = *o;
    s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
  }
  *o = s;
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
  hipLaunchKernelGGL(mb::reduce_rows_kernel, dim3((groups + 255) / 256), dim3(256), 0, st, partial, rows, cols, out,
                     accumulate);
  return (int)hipGetLastError();
}

extern "C" int mb_adam(const mb::AdamArgs* a, hipStream_t st) {
  const int n = a->hi - a->lo;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mb::adam_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}
