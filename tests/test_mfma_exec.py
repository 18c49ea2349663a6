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


def test_hazard_scan_follows_the_taken_branch():
    """The round-3 CBF pattern in objdump form: the forward's last MFMA, a runtime stamp branch to a
    label right after the stamp block, and the relu read of the MFMA result at that label. The
    fall-through path has 8 states, the taken path 1: the scan reports the 1."""
    c = _tools()
    text = """
0000000000001000 <k>:
  v_mfma_f32_16x16x32_bf16 v[132:135], v[136:139], v[88:91], v[132:135] // 000000001000: D3B50084 0612B188
  s_cbranch_vccnz 8 // 000000001008: BF870008 <k+0x2c>
  s_memtime s[26:27] // 00000000100C: C0900680 00000000
  s_waitcnt lgkmcnt(0) // 000000001014: BF8CC07F
  s_sub_u32 s1, s26, s94 // 000000001018: 80815E1A
  s_subb_u32 s28, s27, s95 // 00000000101C: 829C5F1B
  s_add_u32 s80, s1, s80 // 000000001020: 80505001
  s_addc_u32 s81, s28, s81 // 000000001024: 8251511C
  s_mov_b64 s[94:95], s[26:27] // 000000001028: BEDE011A
  v_max_i32_e32 v148, 0, v132 // 00000000102C: 1B290880
  s_endpgm // 000000001030: BF810000
"""
    hz = c.hazards_in(text)
    assert [h[1] for h in hz] == [1], hz
    # with the stamp branch compiled out (straight line + the compiler's nops): nothing to report
    text2 = """
0000000000001000 <k>:
  v_mfma_f32_16x16x32_bf16 v[132:135], v[136:139], v[88:91], v[132:135] // 000000001000: D3B50084 0612B188
  s_nop 7 // 000000001008: BF800007
  v_max_i32_e32 v148, 0, v132 // 00000000100C: 1B290880
  s_endpgm // 000000001010: BF810000
"""
    assert c.hazards_in(text2) == []


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
