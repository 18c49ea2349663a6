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

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
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

DEV f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

DEV int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// accumulator regs 8S..8S+7 -> bf16 operand fragment
template <int S>
DEV bf16x8 acc_frag(const f32x16& c) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)c[8 * S + j];
  return r;
}

DEV void relu_(f32x16& c) {
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = c[i] > 0.f ? c[i] : 0.f;
}

// accumulator init with a per-row bias b[row0 + acc_row(reg,h)] (standard orientation)
DEV f32x16 bias_rows(const float* b, int row0, int h) {
  f32x16 c;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) c[reg] = b[row0 + acc_row(reg, h)];
  return c;
}

// 16-byte fragment load (LDS or global): fragment f, lane l
DEV bf16x8 frag_ld(const bf16* base, int f, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + ((size_t)f * WAVE + lane) * 8);
}

// An opaque scalar zero: adding it to an LDS base inside a loop stops the compiler from
// hoisting every loop-invariant weight-fragment load out of the loop (which would pin
// 100+ VGPRs and spill); the weights stay in LDS and are re-read per tile.
DEV int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}

DEV float shfl_xor32(float v) { return __shfl_xor(v, 32); }

// hi/lo bf16 split of an fp32 value: x ~= hi + lo with ~16 significant bits
DEV void split_bf16(float x, bf16& hi, bf16& lo) {
  hi = (bf16)x;
  lo = (bf16)(x - (float)hi);
}

// wave-local LDS visibility: all prior LDS writes of this wave done before later LDS reads
DEV void lds_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// cooperative copy of `bytes` (multiple of 16) from global to LDS by the whole block
DEV void block_copy16(void* dst, const void* src, int bytes) {
  const u32x4* s = reinterpret_cast<const u32x4*>(src);
  u32x4* d = reinterpret_cast<u32x4*>(dst);
  for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
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
