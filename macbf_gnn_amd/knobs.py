"""Every environment knob the framework reads (one list, each with its user).

Production runs set none of them. The remaining knobs exist for tests (they force a code path a
test compares against) or for A/B measurement scripts; knobs whose A/B question was settled were
removed (their decision is the code's default, the measurement is in docs/PERF.md).

| knob | default | read by | used by |
|---|---|---|---|
| MACBF_DP_BACKEND | nccl on GPU, gloo on CPU | parallel/dist.py, parallel/launch.py | rehearsal of N ranks on one GPU (gloo) |
| MACBF_DP_FORCE_PG | 0 | parallel/dist.py | RCCL process group at world 1 (tests/test_gpu_dp.py) |
| MACBF_EXT | -- | ops/native.py | load an alternative extension build (scripts/build_variant.sh A/B, no-barrier builds) |
| MACBF_NATIVE_BPTT | 1 | engine/hip_engine.py | Python BPTT launch loop, so tests can spy on the calls |
| MACBF_EB16 | 1 (fp32), 0 (bf16 / fp16) | engine/hip_engine.py | 16x16x32 vs 32x32x16 edge backward (tests and A/B runs) |
| MACBF_NODE16 | 1 | engine/hip_engine.py | 32x32x16 node backward (tests/test_gpu_node16.py; bf16 / fp16 A/B) |
| MACBF_NODE_CHUNK | by size | ops/native.py | agents per node-backward chunk (tests force 128 at small sizes) |
| MACBF_BWD_FUSED | by size | ops/native.py | fused node + edge BPTT step on / off (tests) |
| MACBF_CTRL_APW | by size | ops/native.py | agents per wave of the controller step (tests/test_gpu_fp32.py dense-row equality) |
| MACBF_EDGE_WG_PER_CU | 1 (x3) | ops/native.py | edge-backward workgroups per CU (tests) |
| MACBF_NODE_ACTS | 1 | engine/hip_engine.py | 0: the cooperative node backward recomputes the node MLP instead of reusing the rollout's activations (A/B, tests) |
| MACBF_BWD_GRAPH | 1 | engine/hip_engine.py | small scenes: post-rollout work replayed from per-T HIP graphs (0: eager, tests / A/B) |
| MACBF_KERNEL_SCENARIO | 1 | engine/hip_engine.py | small scenes: the persistent rollout loads the start states and goals itself (0: copy launches, A/B) |
| MACBF_OVERLAP_HFWD | by size | engine/hip_engine.py | 1 / 0: CBF h of each step's main slots on a side stream during the rollout (default: on for fp32 ranks of 12,288-24,576 agents, off otherwise; A/B) |
| MACBF_GRAPH_LAUNCH | 1 | engine/hip_engine.py | small scenes: the rollout driver launches the horizon's backward graph itself (0: replay from Python, A/B) |
| MACBF_PUBLISH | 1 | engine/hip_engine.py | early stop through a queue marker instead of kernel publication (tests) |
| MACBF_SELFCHECK | 1 | ops/selfcheck.py | skip the start-up self-check of the 16x16x32 kernels |
| MACBF_ARCH | gfx950 | csrc/build.py | build target |
"""
from __future__ import annotations

import os


def get_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return default if v is None or v == "" else int(v)
