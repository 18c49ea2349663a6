// Layout probes: check on the device the MFMA operand/accumulator maps and the
// ds_read_b64_tr_b16 transposed-read semantics that the fused kernels are built on.
#include "common.h"

namespace mb {

// D = A(32x16) * B(16x32) with natural fragments loaded from global: a/b (64 lanes x 8 h16),
// d (64 lanes x 16 f32) raw accumulator registers.
__global__ void probe_mfma_kernel(const h16* a, const h16* b, float* d) {
  const int l = threadIdx.x;
  const h16x8 af = *reinterpret_cast<const h16x8*>(a + l * 8);
  const h16x8 bf = *reinterpret_cast<const h16x8*>(b + l * 8);
  const f32x16 c = mfma(af, bf, zero16());
#pragma unroll
  for (int q = 0; q < 16; ++q) d[l * 16 + q] = c[q];
}

// D = A(16x32) * B(32x16), v_mfma_f32_16x16x32 with natural fragments: a/b (64 x 8 h16), d (64 x 4)
__global__ void probe_mfma16_kernel(const h16* a, const h16* b, float* d) {
  const int l = threadIdx.x;
  const h16x8 af = *reinterpret_cast<const h16x8*>(a + l * 8);
  const h16x8 bf = *reinterpret_cast<const h16x8*>(b + l * 8);
#if MB_FP16
  const f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#else
  const f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#endif
#pragma unroll
  for (int q = 0; q < 4; ++q) d[l * 4 + q] = c[q];
}

__global__ void probe_tr_kernel(const h16* img_g, int rows, int stride, int e0, int m0, h16* out) {
  __shared__ __attribute__((aligned(16))) h16 img[64 * 136];
  for (int i = threadIdx.x; i < rows * stride; i += blockDim.x) img[i] = img_g[i];
  __syncthreads();
  const h16x8 f = tr_frag(img, stride, e0, m0, threadIdx.x);
  *reinterpret_cast<h16x8*>(out + threadIdx.x * 8) = f;
}

__global__ void probe_lane_xor_kernel(const unsigned* in, unsigned* out) {
  const int lane = threadIdx.x;
  const unsigned v = in[lane];
  out[0 * 64 + lane] = lane_xor<1>(v);
  out[1 * 64 + lane] = lane_xor<2>(v);
  out[2 * 64 + lane] = lane_xor<4>(v);
  out[3 * 64 + lane] = lane_xor<8>(v);
  out[4 * 64 + lane] = lane_xor<16>(v);
  out[5 * 64 + lane] = lane_xor<32>(v);
  const float f = __uint_as_float(v);
  out[6 * 64 + lane] = __float_as_uint(wave_sum(f));
  out[7 * 64 + lane] = __float_as_uint(wave_max(f));
  out[8 * 64 + lane] = __float_as_uint(sum32(f));
}

// MFMA under a wave-parity condition (the round-4 1-pass bias bug, csrc/common.h wave_id()): 8 waves;
// per wave acc = sum_{it,u} X X^T and bias = sum_it X_{it, wave & 1} x ones, X the 16x32 fragment
// a[it][u] (64 lanes x 8). UNIFORM: the condition on wave_id() (scalar branch); else on the wave
// index in a VGPR (an EXEC-masked block the compiler may leave without its execz skip).
// out: (512 threads x 4) acc + bias.
template <bool UNIFORM>
__global__ __launch_bounds__(512) void probe_mfma_exec_kernel(const h16* a, float* out) {
  const int wave = UNIFORM ? wave_id() : (int)(threadIdx.x / WAVE);
  const int lane = threadIdx.x & 63;
  h16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (h16)1.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, bias = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < 4; ++it) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const h16x8 x = *reinterpret_cast<const h16x8*>(a + ((it * 2 + u) * 64 + lane) * 8);
#if MB_FP16
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, acc, 0, 0, 0);
      if ((wave & 1) == u) bias = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, ones, bias, 0, 0, 0);
#else
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, acc, 0, 0, 0);
      if ((wave & 1) == u) bias = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, ones, bias, 0, 0, 0);
#endif
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) out[threadIdx.x * 4 + i] = acc[i] + bias[i];
}

}  // namespace mb

extern "C" int mb_probe_mfma_exec(const void* a, float* out, int uniform, hipStream_t st) {
  if (uniform)
    hipLaunchKernelGGL(mb::probe_mfma_exec_kernel<true>, dim3(1), dim3(512), 0, st, (const h16*)a, out);
  else
    hipLaunchKernelGGL(mb::probe_mfma_exec_kernel<false>, dim3(1), dim3(512), 0, st, (const h16*)a, out);
  return (int)hipGetLastError();
}

extern "C" int mb_probe_lane_xor(const unsigned* in, unsigned* out, hipStream_t st) {
  hipLaunchKernelGGL(mb::probe_lane_xor_kernel, dim3(1), dim3(64), 0, st, in, out);
  return (int)hipGetLastError();
}

extern "C" int mb_probe_mfma16(const void* a, const void* b, float* d, hipStream_t st) {
  hipLaunchKernelGGL(mb::probe_mfma16_kernel, dim3(1), dim3(64), 0, st, (const h16*)a, (const h16*)b, d);
  return (int)hipGetLastError();
}

extern "C" int mb_probe_mfma(const void* a, const void* b, float* d, hipStream_t st) {
  hipLaunchKernelGGL(mb::probe_mfma_kernel, dim3(1), dim3(64), 0, st, (const h16*)a, (const h16*)b, d);
  return (int)hipGetLastError();
}

extern "C" int mb_probe_tr(const void* img, int rows, int stride, int e0, int m0, void* out, hipStream_t st) {
  if (rows * stride > 64 * 136) return -1;
  hipLaunchKernelGGL(mb::probe_tr_kernel, dim3(1), dim3(64), 0, st, (const h16*)img, rows, stride, e0, m0, (h16*)out);
  return (int)hipGetLastError();
}
