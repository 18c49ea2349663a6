"""Profiler checks as tests: rocprofv3 over a fixed, deterministic training workload
(``scripts/prof_workload.py``: fp32 / x3 kernels, 512 agents x 8 envs, fixed horizon), each pass in a
fresh child process with the program itself right after ``--``.

* kernel trace: a training iteration launches only ``mb::`` kernels (no ``at::native`` glue, no
  fills) and at most two copies (the sampled start states and goals);
* PMC counters: per kernel and dispatch, the MFMA instruction count stays within 10 % of the
  recorded baseline (``tests/data/pmc_baseline*.json``; a changed count means a changed kernel
  structure, which must come with a re-recorded baseline) and the LDS bank-conflict share
  (``SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE``) does not regress by more than 5 points. Two
  workloads: 512 x 8 (the fused node + edge BPTT step) and 1024 x 32 (32 K agents per step: the
  16x16x32 node and edge backward kernels of the headline, csrc/node16.h and csrc/ctrl16.h).

Re-record a baseline on an MI355X with ``MACBF_PMC_RECORD=1`` (written to
``gpurun_out/pmc_baseline*.json``; copy it to tests/data/).
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {"512x8": ((), "pmc_baseline.json"),
             "1024x32": (("--agents", "1024", "--envs", "32"), "pmc_baseline_1024x32.json")}
COUNTERS = ["SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVES"]
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def _rocprof(out, args, wl=()):
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        pytest.skip("rocprofv3 not available")
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = ["timeout", "-s", "KILL", "200", exe, *args, "-d", str(out), "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.join(ROOT, "scripts", "prof_workload.py"), "--iters", "2", *wl]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=260)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    return out


def _find(out, suffix):
    fs = glob.glob(os.path.join(str(out), "**", "*" + suffix), recursive=True)
    assert fs, f"no *{suffix} under {out}"
    return fs[0]


def test_iteration_launches_only_native_kernels(tmp_path):
    from iter_kernels import iterations, summary
    _rocprof(tmp_path / "trace", ["--kernel-trace"])
    its = iterations(_find(tmp_path / "trace", "kernel_trace.csv"))
    assert len(its) >= 3
    s = summary(its[-1])
    glue = dict(s["glue"])
    copies = glue.pop("__amd_rocclr_copyBuffer", 0)
    assert copies <= 2, s["glue"]
    assert not glue, f"non-native kernels in the training iteration: {glue}"


@pytest.mark.parametrize("workload", sorted(WORKLOADS))
def test_pmc_mfma_counts_and_lds_conflicts(tmp_path, workload):
    from prof_workload import summarize
    wl, fname = WORKLOADS[workload]
    _rocprof(tmp_path / "pmc", ["--pmc", *COUNTERS], wl)
    got = summarize([_find(tmp_path / "pmc", "counter_collection.csv")])
    got = {k: v for k, v in got.items() if k.startswith("mb::")}
    if os.environ.get("MACBF_PMC_RECORD") == "1":
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", fname), "w") as f:
            json.dump(got, f, indent=1, sort_keys=True)
    baseline = os.path.join(ROOT, "tests", "data", fname)
    if not os.path.exists(baseline):
        pytest.skip("no recorded PMC baseline")
    base = json.load(open(baseline))
    if workload == "1024x32":      # the workload exists to pin these kernels
        for k in ("mb::x3::ctrl_node_bwd16_kernel<2, false>", "mb::x3::ctrl_edge_bwd16_kernel<2, false>",
                  "mb::x3::cbf_bwd16_kernel<2, false>"):
            assert k in base, f"baseline lacks {k}"
    bad = []
    for k, b in base.items():
        if b.get("SQ_INSTS_MFMA", 0) <= 0:
            continue
        g = got.get(k)
        if g is None:
            bad.append(f"{k}: not launched")
            continue
        if abs(g["SQ_INSTS_MFMA"] - b["SQ_INSTS_MFMA"]) > 0.10 * b["SQ_INSTS_MFMA"]:
            bad.append(f"{k}: MFMA {g['SQ_INSTS_MFMA']:.4g} vs baseline {b['SQ_INSTS_MFMA']:.4g}")
        share = lambda r: r.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(r.get("SQ_LDS_IDX_ACTIVE", 0.0), 1.0)
        if share(g) > share(b) + 0.05:
            bad.append(f"{k}: LDS conflict share {share(g):.3f} vs baseline {share(b):.3f}")
    assert not bad, "\n".join(bad)
