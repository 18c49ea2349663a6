"""Static check of the built kernels: no v_mfma inside an EXEC-masked region.

A v_mfma in a block the compiler entered with s_and_saveexec (a lane-divergent branch) runs with
a partial or empty EXEC; when the compiler also drops the block's s_cbranch_execz skip (short
blocks), the MFMA still updates its accumulator with operand registers the masked instructions
left stale (csrc/common.h wave_id(), docs/ARCHITECTURE.md "MFMA and EXEC"). The kernels branch on
the wave index through wave_id() (an SGPR: scalar branches), so no MFMA should be EXEC-masked.

Scan: the gfx950 code objects of build/csrc/*.o are disassembled (llvm-objdump --offloading, -d);
per kernel, in layout order, an s_*saveexec / s_*_b64 exec write opens a masked region and the
s_or_b64 exec, exec, s[..] that restores it closes it (the structurizer emits properly nested
regions in layout order); a region whose opening is not followed by s_cbranch_execz may run with
EXEC = 0. Prints every MFMA found inside such a region; exit 1 if any.

    python scripts/check_mfma_exec.py [--all] [OBJ ...]   (default: build/csrc/{cbf,ctrl}{,_f16,_x3}.o;
                                                         --all: every kernel, not only the strict set)
"""
from __future__ import annotations

import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
OPEN = re.compile(r"\bs_(and|andn2|orn2|nand|nor|xnor)_saveexec_b64\b|\bs_(and|andn2)_b64\s+exec,")
SWITCH = re.compile(r"\bs_or_saveexec_b64\b|\bs_xor_saveexec_b64\b|\bs_xor_b64\s+exec,")   # else part of an if
CLOSE = re.compile(r"\bs_or_b64\s+exec,\s*exec,")
FUNC = re.compile(r"^[0-9a-f]+ <([^>]+)>:")


def code_object(obj: str, tmp: str) -> str:
    dst = os.path.join(tmp, os.path.basename(obj))
    shutil.copy(obj, dst)
    subprocess.run([OBJDUMP, "--offloading", dst], check=True, capture_output=True, cwd=tmp)
    cos = glob.glob(dst + ".*gfx950*")
    if not cos:
        raise RuntimeError(f"no gfx950 bundle in {obj}")
    return cos[0]


def scan(co: str):
    """-> [(kernel, instruction)] of MFMAs inside a masked region entered WITHOUT the
    s_cbranch_execz skip (a region the wave may run with EXEC = 0). Regions with the skip (and
    loops, whose back-edge leaves on EXEC = 0) never run an instruction with an empty EXEC."""
    out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout
    lines = [l for l in out.splitlines() if l.strip()]
    bad, fn, stack = [], None, []
    for k, line in enumerate(lines):
        m = FUNC.match(line)
        if m:
            fn, stack = m.group(1), []
            continue
        if fn is None:
            continue
        if CLOSE.search(line):
            if stack:
                stack.pop()
        elif OPEN.search(line) or SWITCH.search(line):
            if SWITCH.search(line) and stack:
                stack.pop()
            # guarded: an s_cbranch_execz among the scalar instructions that follow the opening
            guarded = False
            for x in lines[k + 1:k + 6]:
                op = x.strip().split(" ")[0]
                if op in ("s_cbranch_execz", "s_cbranch_execnz"):    # execnz body; else s_branch past it
                    guarded = True
                    break
                if not op.startswith("s_"):
                    break
            stack.append(guarded)
        elif "v_mfma" in line and any(not g for g in stack):
            bad.append((fn, line.strip()))
    return bad


# the kernels held to the rule (the 16x16x32 backward kernels and every CBF kernel); the 32x32x16
# controller kernels predate wave_id() and are reported only with --all
STRICT = re.compile(r"bwd16_kernel|cbf_")


def main(objs):
    show_all = "--all" in objs
    objs = [o for o in objs if o != "--all"]
    objs = objs or [os.path.join(ROOT, "build", "csrc", f"{k}{p}.o") for k in ("cbf", "ctrl") for p in ("", "_f16", "_x3")]
    total = 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            bad = scan(code_object(obj, tmp))
            if not show_all:
                bad = [(f, l) for f, l in bad if STRICT.search(f)]
            total += len(bad)
            kern = sorted({f for f, _ in bad})
            print(f"{os.path.basename(obj)}: {len(bad)} EXEC-masked MFMA(s)" + (f" in {kern}" if kern else ""))
            for f, l in bad[:8]:
                print(f"   {f}: {l}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
