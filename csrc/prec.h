// 16-bit MFMA element type of the network kernels.
//
// ctrl.hip and cbf.hip are compiled twice (csrc/build.py): bf16 (default) and fp16
// (-DMB_FP16=1, the "fp16 mixed precision" configuration). Both use the same
// v_mfma_f32_32x32x16_{bf16,f16} fragment layouts and fp32 accumulation; the kernels, the
// launch symbols (mb_*_f16) and the kernel namespaces (mb::b16 / mb::f16) are distinct so the
// two instantiations can live in one shared object.
#pragma once

#if MB_FP16
typedef _Float16 h16;
#define MB_PREC f16
#define MB_SYM(name) mb_##name##_f16
#else
typedef __bf16 h16;
#define MB_PREC b16
#define MB_SYM(name) mb_##name
#endif
