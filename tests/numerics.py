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


def tie_log(what, ties, total, limit):
    """Tie allowance of a tie-aware comparison: the rows a relu / radius / max-pool tie exempts
    may not exceed `limit` (a per-case bound set at ~2x the measured count).
    With MACBF_NUM_LOG the measured count is logged (calibration runs)."""
    ties, total = int(ties), int(total)
    log = os.environ.get("MACBF_NUM_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "name": what,
                                "ties": ties, "total": total, "frac": ties / max(total, 1), "limit": limit}) + "\n")
        if os.environ.get("MACBF_NUM_NOASSERT"):
            return
    assert ties <= limit, f"{what}: {ties} tie rows of {total} > allowance {limit}"


def _lin64(x, w, b):
    w = w.detach().double()
    w = w.reshape(w.shape[0], -1)
    b = b.detach().double()
    return x @ w.t() + b, x.abs() @ w.abs().t() + b.abs()


def ctrl_tie_nodes(p, s, g, idx, tau=3e-5, nodes=None):
    """(B, N) bool, float64: agents whose dL/ds the x3 kernels may legitimately compute on the other
    side of a branch than the fp32 oracle -- some relu pre-activation of the agent's node MLP or of
    an edge row touching it (as centre or as neighbour) within tau * sum |terms| of zero (tau = 3e-5,
    the x3 products' own error bound), an edge at the radius boundary (|d - R| <= 1e-6), or a
    max-pool feature whose two largest slot values are within tau of each other. Reference op:
    /root/reference/controller.py:31-63."""
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd import oracle as O
    s = s.detach().double()
    g = g.detach().double()
    D = O.sdim(s)
    rel, eye = O.edge_rel(s, idx, None if nodes is None else nodes.double())
    x = torch.cat([rel, eye.unsqueeze(-1)], -1)
    dist = torch.sqrt(O.sq_dist(rel, D))
    etie = (dist - C.OBS_RADIUS).abs() <= 1e-6
    h = x
    for li in (0, 2):
        pre, sc = _lin64(h, p[f"controller_centr_net.{li}.weight"], p[f"controller_centr_net.{li}.bias"])
        etie |= (pre.abs() <= tau * sc).any(-1)
        h = torch.relu(pre)
    hm = h * (dist < C.OBS_RADIUS).double().unsqueeze(-1)
    if hm.shape[-2] >= 2:
        top = hm.topk(2, dim=-2).values
        ptie = ((top[..., 0, :] - top[..., 1, :]) <= tau * top[..., 0, :]) & (top[..., 0, :] > 0)
        etie |= ptie.any(-1, keepdim=True)          # a pool near-tie may route to any slot of the agent
    z = torch.cat([hm.max(dim=-2).values, s[..., :D] - g, s[..., D:2 * D]], -1)
    ntie = torch.zeros(z.shape[:-1], dtype=torch.bool, device=z.device)
    for li in (0, 2, 4):
        pre, sc = _lin64(z, p[f"controller_dec_net.{li}.weight"], p[f"controller_dec_net.{li}.bias"])
        ntie |= (pre.abs() <= tau * sc).any(-1)
        z = torch.relu(pre)
    return ntie | edge_ties_to_nodes(etie, idx, s.shape[-2])


def edge_ties_to_nodes(etie, idx, N):
    """(..., N, K) edge tie flags -> (..., N) node flags: the centre i and the neighbour j of every
    tie edge (an edge gradient is added to s_i and subtracted from s_j)."""
    lead = etie.shape[:-2]
    e = etie.reshape(-1, *etie.shape[-2:])
    ix = idx.long().reshape(-1, *idx.shape[-2:])
    out = e.any(-1).clone()
    for b in range(e.shape[0]):
        j = ix[b][e[b]]
        out[b, j[j < N]] = True
    return out.reshape(*lead, N)


def cmp_nodes_tie(got, ref, tie, name, rel=1e-3, rel_all=2e-2, limit=None):
    """Per-node records (..., W) against a float64 reference, tie-aware (the scheme of the
    16x16x32 row checks, tests/test_gpu_oracle16.py): a node whose error exceeds
    rel * |its row| + 0.1 rel * rms row norm must be a flagged tie node; the untied nodes together
    <= rel of the whole reference norm, everything <= rel_all; and the number of nodes the tie
    flags actually exempt (flagged AND outside the row tolerance) <= limit (~2x measured)."""
    g = got.double().reshape(-1, got.shape[-1])
    r = ref.double().reshape(-1, ref.shape[-1])
    t = tie.reshape(-1)
    rn = max(r.norm().item(), 1e-30)
    rows = r.norm(dim=1)
    tol = rel * rows + 0.1 * rel * rows.pow(2).mean().sqrt()
    over = (g - r).norm(dim=1) > tol
    ek = (g[~t] - r[~t]).norm().item() / rn
    ea = (g - r).norm().item() / rn
    if limit is not None:
        tie_log(name + " exempt tie nodes", int((over & t).sum()), t.numel(), limit)
    assert int((over & ~t).sum()) == 0, f"{name}: {int((over & ~t).sum())} untied nodes outside the row tolerance"
    assert ek <= rel and ea <= rel_all, f"{name}: untied rel err {ek:.3e} (<= {rel:.0e}), all {ea:.3e}, ties {int(t.sum())}"
