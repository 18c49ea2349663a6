"""Static check of the shipped gfx950 code: no v_mfma in an EXEC-masked block that may run with
EXEC = 0 (the compiler drops the s_cbranch_execz skip of short blocks; an MFMA there still updates
its accumulator). Round 4 found one in the 1-pass 16x16x32 edge backward (a wave-parity bias
MFMA under a VGPR condition: db2 90 % wrong); the kernels now branch on wave_id() (csrc/common.h).
scripts/check_mfma_exec.py disassembles build/csrc/*.o; the test also checks that the scan flags
the pre-fix pattern (a kernel with the wave index in a VGPR)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

OBJS = [os.path.join(ROOT, "build", "csrc", f"{k}{p}.o") for k in ("cbf", "ctrl") for p in ("", "_f16", "_x3")]


def _tools():
    import check_mfma_exec as c
    if not os.path.exists(c.OBJDUMP):
        pytest.skip("llvm-objdump not available")
    return c


def test_shipped_kernels_have_no_exec_masked_mfma():
    c = _tools()
    objs = [o for o in OBJS if os.path.exists(o)]
    if not objs:
        pytest.skip("extension not built (python csrc/build.py)")
    assert c.main(objs) == 0


def test_scan_flags_a_masked_bias_mfma(tmp_path):
    """A wave-parity-conditional MFMA with the wave index in a VGPR (the round-4 bug) is flagged;
    the same kernel with wave_id() is not."""
    c = _tools()
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = tmp_path / "k.hip"
    src.write_text(r'''
#include <hip/hip_runtime.h>
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
template <bool UNIFORM>
__global__ __launch_bounds__(512) void k(const bf8* a, float* out) {
  const int wave = UNIFORM ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64)) : (int)(threadIdx.x / 64);
  const int lane = threadIdx.x & 63;
  bf8 ones;
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
  f4 acc = {0.f, 0.f, 0.f, 0.f}, bias = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < 4; ++it) {
    for (int u = 0; u < 2; ++u) {
      const bf8 x = a[(it * 2 + u) * 64 + lane];
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, acc, 0, 0, 0);
      if ((wave & 1) == u) bias = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, ones, bias, 0, 0, 0);
    }
  }
  for (int i = 0; i < 4; ++i) out[(threadIdx.x * 4 + i) * 2] = acc[i] + bias[i];
}
template __global__ void k<true>(const bf8*, float*);
template __global__ void k<false>(const bf8*, float*);
''')
    obj = tmp_path / "k.o"
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-c", str(src), "-o", str(obj)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    (tmp_path / "x").mkdir()
    bad = c.scan(c.code_object(str(obj), str(tmp_path / "x")))
    names = {f for f, _ in bad}
    assert any("ILb0E" in f for f in names), names          # k<false>: flagged
    assert not any("ILb1E" in f for f in names), names      # k<true>: clean
