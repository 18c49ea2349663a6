"""Shared numerics comparison for the GPU kernel tests: relative norm error and cosine
similarity of a HIP result against a PyTorch reference.

Calibration: with MACBF_NUM_LOG=<file> every comparison appends one JSON line (test, tensor,
measured error, bound); MACBF_NUM_NOASSERT=1 additionally turns the bounds off, so one GPU run
collects the measured errors of every case (scripts/gpu_numerics.sh)."""
import json
import os

import torch


def rel_cmp(got, ref, name, rel, cos=None):
    got = got.detach().double().flatten()
    ref = ref.detach().double().flatten()
    rn = ref.norm().item()
    if rn < 1e-12:
        assert got.norm().item() < 1e-6, name
        return 0.0
    err = (got - ref).norm().item() / rn
    c = torch.nn.functional.cosine_similarity(got, ref, dim=0).item()
    log = os.environ.get("MACBF_NUM_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "name": name,
                                "err": err, "cos": c, "bound": rel}) + "\n")
        if os.environ.get("MACBF_NUM_NOASSERT"):
            return err
    cos = 1.0 - rel * rel if cos is None else cos     # |a-b|/|b| = e < rel  =>  cos >= sqrt(1 - e^2)
    assert err < rel and c > cos, f"{name}: rel err {err:.3e} (bound {rel:.1e}), cos {c:.6f}"
    return err


def ctrl_pool_slots(ctrl, s, g, idx, obs=None):
    """The controller kernel's max-pool argmax slots (B, N, 128; 255 = none) and pooled values
    (B, N, 128 fp32; hi + lo for x3) for this input and the module's precision -- ``ctrl_fwd``
    is deterministic, so these are what the module's own forward saved. Tests pin the oracle's
    max-pool subgradient and values to them (``oracle.controller_forward(pool_slots=...,
    pool_values=...)``) and bound how far the slots are from the true max
    (``oracle.pool_slot_gap``): near-ties may legitimately resolve either way."""
    from macbf_gnn_amd.ops import graph, native
    from macbf_gnn_amd.ops import layout as L
    from macbf_gnn_amd.ops.packing import module_pack
    B, N, K = idx.shape
    dev = s.device
    if obs is not None:
        obs = (obs if obs.dim() == 3 else obs.unsqueeze(0)).expand(B, *obs.shape[-2:]).float()
    mp = module_pack("ctrl", ctrl, dev)
    w, v, rm = mp.pack(tuple(ctrl.parameters()))
    S = graph.node_records(s.detach().float(), obs)
    A = torch.empty(B, N, mp.dim, device=dev)
    pooled = torch.empty(B, N, L.pooled_row(mp.prec), dtype=w.dtype, device=dev)
    am = torch.empty(B, N, 128, dtype=torch.uint8, device=dev)
    native.ctrl_fwd(S, g.detach().float().contiguous(), idx.to(torch.int32).contiguous(), w, mp.off["ew1f"],
                    mp.off["nw1f"], v, A, None, None, None, pooled=pooled, argmax=am, prec=mp.prec)
    torch.cuda.synchronize()
    pv = pooled[..., :128].float()
    if mp.prec == "fp32":
        pv = pv + pooled[..., 128:256].float()
    return am, pv
