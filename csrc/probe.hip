// Layout probes: check on the device the MFMA operand/accumulator maps and the
// ds_read_b64_tr_b16 transposed-read semantics that the fused kernels are built on.
#include "common.h"

namespace mb {

// D = A(32x16) * B(16x32) with natural fragments loaded from global: a/b (64 lanes x 8 bf16),
// d (64 lanes x 16 f32) raw accumulator registers.
__global__ void probe_mfma_kernel(const bf16* a, const bf16* b, float* d) {
  const int l = threadIdx.x;
  const bf16x8 af = *reinterpret_cast<const bf16x8*>(a + l * 8);
  const bf16x8 bf = *reinterpret_cast<const bf16x8*>(b + l * 8);
  const f32x16 c = mfma(af, bf, zero16());
#pragma unroll
  for (int q = 0; q < 16; ++q) d[l * 16 + q] = c[q];
}

// Transposed A-fragment read from an edge-major LDS image img[e][m] (row stride `stride`
// elements): lane (r, h) gets img[e0 + 8h + j][m0 + r], j = 0..7.
DEV bf16x8 tr_frag(const bf16* img, int stride, int e0, int m0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3, gg = (lane >> 4) & 1, h = lane >> 5;
  const bf16* a1 = img + (e0 + 8 * h + q) * stride + m0 + 16 * gg + 4 * p;
  const bf16* a2 = a1 + 4 * stride;
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
  const s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a2));
  bf16x8 r;
  const bf16x4 b1 = __builtin_bit_cast(bf16x4, v1);
  const bf16x4 b2 = __builtin_bit_cast(bf16x4, v2);
  r[0] = b1[0]; r[1] = b1[1]; r[2] = b1[2]; r[3] = b1[3];
  r[4] = b2[0]; r[5] = b2[1]; r[6] = b2[2]; r[7] = b2[3];
  return r;
}

__global__ void probe_tr_kernel(const bf16* img_g, int rows, int stride, int e0, int m0, bf16* out) {
  __shared__ __attribute__((aligned(16))) bf16 img[64 * 136];
  for (int i = threadIdx.x; i < rows * stride; i += blockDim.x) img[i] = img_g[i];
  __syncthreads();
  const bf16x8 f = tr_frag(img, stride, e0, m0, threadIdx.x);
  *reinterpret_cast<bf16x8*>(out + threadIdx.x * 8) = f;
}

}  // namespace mb

extern "C" int mb_probe_mfma(const void* a, const void* b, float* d, hipStream_t st) {
  hipLaunchKernelGGL(mb::probe_mfma_kernel, dim3(1), dim3(64), 0, st, (const bf16*)a, (const bf16*)b, d);
  return (int)hipGetLastError();
}

extern "C" int mb_probe_tr(const void* img, int rows, int stride, int e0, int m0, void* out, hipStream_t st) {
  if (rows * stride > 64 * 136) return -1;
  hipLaunchKernelGGL(mb::probe_tr_kernel, dim3(1), dim3(64), 0, st, (const bf16*)img, rows, stride, e0, m0, (bf16*)out);
  return (int)hipGetLastError();
}
