"""Build the native extension ``macbf_gnn_amd/_C*.so`` for gfx950 with hipcc + ninja.

Each ``csrc/*.hip`` kernel file compiles to its own object in parallel (no libtorch headers:
seconds per file); ``bindings.cpp`` is a pybind11 module taking device pointers + the torch
HIP stream handle. The shared object is linked in-tree so it travels with the repo snapshot
to the GPU box. Usage: ``python csrc/build.py [-j N] [--clean] [--verbose]``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "macbf_gnn_amd")
BUILD = os.path.join(ROOT, "build", "csrc")
ARCH = os.environ.get("MACBF_ARCH", "gfx950")
KERNELS = ["scan", "scenario", "ctrl", "cbf", "dedup", "graph", "optim"]
HALF_KERNELS = {"ctrl", "cbf"}       # compiled per MFMA operand precision (csrc/prec.h)


HOST_SRCS = ["host/scenario_host.cpp", "host/bindings_host.cpp"]   # CPU runtime (plain C++)


def ext_path():
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def probe_ext_path():
    """Layout probes (csrc/probe.hip) for tests/test_gpu_probe.py: a separate extension, not in _C."""
    return os.path.join(PKG, "_probe" + sysconfig.get_config_var("EXT_SUFFIX"))


def host_ext_path():
    return os.path.join(PKG, "_host" + sysconfig.get_config_var("EXT_SUFFIX"))


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def torch_lib():
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib") if spec else "/opt/rocm/lib"


def write_ninja(debug=False):
    import pybind11
    py_inc = sysconfig.get_paths()["include"]
    opt = "-O1 -g" if debug else "-O3"
    kflags = (f"--offload-arch={ARCH} {opt} -fPIC -std=c++17 -mcode-object-version=5 "
              f"-Wno-unused-result -Wno-unused-variable -I{HERE}")
    bflags = f"-O2 -fPIC -std=c++17 -I{HERE} -I{pybind11.get_include()} -I{py_inc}"
    tl = torch_lib()
    lines = [
        f"hipcc = {hipcc()}",
        f"kflags = {kflags}",
        f"bflags = {bflags}",
        f"ldflags = -shared -fPIC --offload-arch={ARCH} -Wl,-rpath,{tl} -Wl,-rpath,/opt/rocm/lib",
        "rule kcc",
        "  command = $hipcc $kflags $kdefs -c $in -o $out -MD -MF $out.d",
        "  depfile = $out.d",
        "  description = HIPCC $in",
        "rule bcc",
        "  command = $hipcc $bflags -c $in -o $out -MD -MF $out.d",
        "  depfile = $out.d",
        "  description = CXX $in",
        f"cxx = {shutil.which('g++') or 'g++'}",
        f"hflags = -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -I{HERE}/host -I{pybind11.get_include()} -I{py_inc}",
        "rule hcc",
        "  command = $cxx $hflags -c $in -o $out -MD -MF $out.d",
        "  depfile = $out.d",
        "  description = CXX $in",
        "rule hlink",
        "  command = $cxx -shared -pthread $in -o $out",
        "  description = LINK $out",
        "rule link",
        "  command = $hipcc $ldflags $in -o $out",
        "  description = LINK $out",
    ]
    objs = []
    for k in KERNELS:
        src = os.path.join(HERE, k + ".hip")
        if not os.path.exists(src):
            continue
        o = os.path.join(BUILD, k + ".o")
        lines.append(f"build {o}: kcc {src}")
        objs.append(o)
        if k in HALF_KERNELS:   # fp16 MFMA inputs and the fp32-accurate 3-term split (csrc/prec.h)
            for suffix, d in (("_f16", "-DMB_FP16=1"), ("_x3", "-DMB_X3=1")):
                o = os.path.join(BUILD, k + suffix + ".o")
                lines.append(f"build {o}: kcc {src}")
                lines.append(f"  kdefs = {d}")
                objs.append(o)
    for b in ("bindings", "runtime"):      # pybind11 layer + native rollout driver (host C++)
        bo = os.path.join(BUILD, b + ".o")
        lines.append(f"build {bo}: bcc {os.path.join(HERE, b + '.cpp')}")
        objs.append(bo)
    lines.append(f"build {ext_path()}: link {' '.join(objs)}")
    po, pb = os.path.join(BUILD, "probe.o"), os.path.join(BUILD, "probe_bindings.o")
    lines.append(f"build {po}: kcc {os.path.join(HERE, 'probe.hip')}")
    lines.append(f"build {pb}: bcc {os.path.join(HERE, 'probe_bindings.cpp')}")
    lines.append(f"build {probe_ext_path()}: link {po} {pb}")
    hobjs = []
    for src in HOST_SRCS:
        o = os.path.join(BUILD, "host_" + os.path.basename(src).replace(".cpp", ".o"))
        lines.append(f"build {o}: hcc {os.path.join(HERE, src)}")
        hobjs.append(o)
    lines.append(f"build {host_ext_path()}: hlink {' '.join(hobjs)}")
    lines.append(f"default {ext_path()} {host_ext_path()} {probe_ext_path()}")
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, "build.ninja"), "w") as f:
        f.write("\n".join(lines) + "\n")


def build(jobs=None, clean=False, verbose=False, debug=False):
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    write_ninja(debug)
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmd = [shutil.which("ninja") or "ninja", "-C", BUILD, f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("native build failed")
    return ext_path()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    print(build(a.j, a.clean, a.verbose, a.debug))


if __name__ == "__main__":
    main()
