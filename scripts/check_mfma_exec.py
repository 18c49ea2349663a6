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


# ---- MFMA result -> consumer wait states along every path (a branch between them included)
# gfx950 asks for 8 wait states (instructions or s_nop states) between a v_mfma_f32_16x16x32 / 32x32x16
# result write and a VALU / memory instruction that reads it; the compiler's nops satisfy that in
# straight-line code (measured in these kernels: always 8), but it left 1-2 states on the TAKEN path
# of a runtime branch right after the CBF forward's last MFMA (the round-3 "miscompile": ~20 % wrong
# evaluations with the branch one instruction closer). Checked for reads (RAW) only.
HAZARD_STATES = 8          # v_mfma_f32_16x16x32 (the compiler's straight-line minimum in these kernels)
HAZARD_STATES_32 = 12      # v_mfma_f32_32x32x16 (likewise)
# a taken branch costs more than the one state counted for it (the failing round-3 path had 1,
# its passing barrier variant 2): reads on a path with fewer than FAIL_STATES fail the check, the
# others (4..7) are reported
FAIL_STATES = 4


def _vregs(txt):
    """Typed register set of an operand text: {('v', n), ('a', n)}."""
    used = set()
    for t, a_, b_ in re.findall(r"\b([va])\[(\d+):(\d+)\]", txt):
        used |= {(t, r) for r in range(int(a_), int(b_) + 1)}
    used |= {(t, int(n)) for t, n in re.findall(r"\b([va])(\d+)\b", txt)}
    return used


def _writes(ins):
    """VGPRs an instruction writes: its first operand, unless it is a store / scalar instruction."""
    parts = ins.split(None, 1)
    if len(parts) < 2 or re.match(r"(ds_write|ds_store|global_store|buffer_store|flat_store|scratch_store|s_)", parts[0]):
        return set()
    return _vregs(parts[1].split(",")[0])


def _reads(ins):
    """VGPRs an instruction reads: every operand but the first (the destination), except for stores
    (all operands are sources) and instructions without a VGPR destination."""
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return set()
    op, rest = parts
    ops = [o.strip() for o in rest.split(",")]
    if re.match(r"(ds_write|ds_store|global_store|buffer_store|flat_store|scratch_store|s_)", op):
        return _vregs(rest)
    return _vregs(",".join(ops[1:]))


def hazards(co: str):
    """-> [(kernel, states, mfma, consumer)] where a consumer of an MFMA result is reached along
    some path (fall-through or taken branch, depth <= 4) with fewer than HAZARD_STATES states."""
    out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout
    return hazards_in(out)


def hazards_in(out: str):
    """hazards() on llvm-objdump -d text (functions '<addr> <name>:', branch targets '<label>')."""
    bad = []
    fn_lines, fn = [], None

    def flush():
        if not fn_lines:
            return
        L = [l.split("//")[0].strip() for l in fn_lines]
        at = {}                                    # instruction address -> index
        for i, l in enumerate(fn_lines):
            m = re.search(r"//\s*([0-9A-Fa-f]+):", l)
            if m:
                at[int(m.group(1), 16)] = i
        for i, ins in enumerate(L):
            m = re.match(r"v_mfma\S*\s+([va])\[(\d+):(\d+)\]", ins)
            if not m:
                continue
            regs = {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
            need = HAZARD_STATES_32 if "32x32" in ins else HAZARD_STATES
            stack = [(i + 1, 0, 0)]
            while stack:
                j, st, depth = stack.pop()
                while j < len(L) and st < need:
                    x = L[j]
                    if not x:
                        j += 1
                        continue
                    if x.startswith("s_nop"):
                        st += int(x.split()[1], 0) + 1
                        j += 1
                        continue
                    if x.startswith("s_endpgm") or x.startswith("s_setpc"):
                        break
                    if x.startswith("s_cbranch") or x.startswith("s_branch"):
                        tgt = re.search(r"<[^>+]+\+0x([0-9a-fA-F]+)>", fn_lines[j])
                        k = at.get(fn_addr + int(tgt.group(1), 16)) if tgt else None
                        if k is not None and depth < 4:
                            stack.append((k, st + 1, depth + 1))
                        if x.startswith("s_branch"):
                            break
                        st += 1
                        j += 1
                        continue
                    if x.startswith("v_mfma"):
                        if _vregs(x.split(",")[0]) & regs:
                            break                      # the next MFMA of the chain (srcC forwarding)
                    elif _reads(x) & regs:
                        bad.append((fn, st, ins[:60], x[:60]))
                        break
                    else:
                        regs = regs - _writes(x)       # overwritten: later reads see the new value
                        if not regs:
                            break
                    st += 1
                    j += 1

    fn_addr = 0
    for line in out.splitlines():
        m = FUNC.match(line)
        if m:
            flush()
            fn, fn_lines = m.group(1), []
            fn_addr = int(line.split()[0], 16)
            continue
        if fn is not None and line.strip():
            fn_lines.append(line)
    flush()
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
            co = code_object(obj, tmp)
            bad = scan(co)
            hz = hazards(co)
            if not show_all:
                bad = [(f, l) for f, l in bad if STRICT.search(f)]
                hz = [h for h in hz if STRICT.search(h[0])]
            total += len(bad) + sum(1 for h in hz if h[1] < FAIL_STATES)
            kern = sorted({f for f, _ in bad})
            print(f"{os.path.basename(obj)}: {len(bad)} EXEC-masked MFMA(s)" + (f" in {kern}" if kern else "")
                  + f"; {len(hz)} MFMA result read(s) with < {HAZARD_STATES} wait states on some path")
            for f, l in bad[:8]:
                print(f"   {f}: {l}")
            for f, st, m_, x in hz[:8]:
                print(f"   {f}: {st} states: {m_} -> {x}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
