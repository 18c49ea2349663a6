// MFMA operand precision of the network kernels.
//
// ctrl.hip and cbf.hip are compiled three times (csrc/build.py):
//   bf16 (default)  one v_mfma_f32_32x32x16_bf16 per product, fp32 accumulation
//   fp16 (-DMB_FP16=1) the same with v_mfma_f32_32x32x16_f16 ("fp16 mixed precision")
//   x3   (-DMB_X3=1)   fp32-accurate: every operand is split x = hi + lo into two bf16 planes and
//                      a product is hi*hi + hi*lo + lo*hi (three bf16 MFMAs, fp32 accumulation;
//                      the dropped lo*lo term is ~2^-16 relative) -- the reference-precision
//                      path (`--dtype fp32`). Weight fragments, row-major weight images, LDS
//                      stage images and the pooled / dL/dpooled activations carry a lo plane.
// The kernels, the launch symbols (mb_*, mb_*_f16, mb_*_x3) and the kernel namespaces
// (mb::b16 / mb::f16 / mb::x3) are distinct so the instantiations share one shared object.
#pragma once

#ifndef MB_X3
#define MB_X3 0
#endif

#if MB_X3
typedef __bf16 h16;
#define MB_PREC x3
#define MB_SYM(name) mb_##name##_x3
#elif MB_FP16
typedef _Float16 h16;
#define MB_PREC f16
#define MB_SYM(name) mb_##name##_f16
#else
typedef __bf16 h16;
#define MB_PREC b16
#define MB_SYM(name) mb_##name
#endif
