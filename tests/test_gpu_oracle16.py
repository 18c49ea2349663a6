"""The 16x16x32 x3 backward kernels pinned to a float64 oracle of the SAME inputs.

* CBF backward (csrc/cbf16.h) over cbf_compact's records of a real training call: each record
  {u, e | pass << 31, j, dh} is re-evaluated in float64 autograd -- the edge features of (i, j) on
  s_{t+pass}, the 6 -> 64 -> 128 -> 64 -> 1 MLP, the radius mask -- and dE[u] = dh * dh/d(s_i - s_j)
  and the weight-gradient slab sums are compared with the kernel's.
* Controller edge backward (csrc/ctrl16.h) of a captured BPTT step: the edge MLP 5 -> 64 -> 128, the
  max-pool routed through the kernel's saved argmax slots, the upstream dL/dpooled -> dL/d(s_i - s_j)
  per edge (dEc) and dW1 / db1 / dW2 / db2, in float64.

Per row, NO deviation is allowed except on a provable relu / radius tie: an evaluation with some
pre-activation |z| <= TAU * sum |terms| (float64), or |d - R| <= 1e-6. TAU = 3e-5 is the x3
arithmetic's own error bound: every product carries <= ~2^-16 relative error (hi*hi + hi*lo + lo*hi
of ~16-bit splits), so the kernel's relu' can differ from the exact one only inside that band.
Everything else must agree to 1e-3 of its row norm (x3 lands at ~1e-5; a schedule miscompile -- the
reason for the sched_barrier in cbf16.h -- moves whole rows by 2-80 %).

Reference ops: /root/reference/cbf.py:13-18,40-43 and /root/reference/controller.py:16-20,43-46,
differentiated by /root/reference/train.py:103.
"""
import pytest
import torch
import torch.nn.functional as F

from macbf_gnn_amd import config as C
from macbf_gnn_amd.engine import Trainer
from macbf_gnn_amd.ops import layout as L
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TAU = 3e-5
ROW_TOL = 1e-3
ABS_TOL = 1e-4


def _params(tr, module):
    return {pn: tr.fp.flat[o:o + n].view(shape).detach().double()
            for m, pn, shape, o, n in tr.fp.specs if m == module}


def _unpack(tr, fn, red):
    offs = {pn: o for (m, pn, shape, o, n) in tr.fp.specs}
    s, d = fn(offs, tr.cfg.dim)
    g = torch.zeros_like(tr.fp.flat, dtype=torch.float64)
    g.index_add_(0, torch.as_tensor(d, device=DEV), red.double().index_select(0, torch.as_tensor(s, device=DEV)))
    return g


def _lin(x, w, b):
    return x @ w.reshape(w.shape[0], -1).t() + b


def _tie(pre, x, w, b):
    """Per row: some unit's |pre-activation| within TAU of the sum of its |terms|."""
    scale = x.abs() @ w.reshape(w.shape[0], -1).abs().t() + b.abs()
    return (pre.abs() <= TAU * scale).any(-1)


def _check_rows(got, ref, tie, what, scale):
    """Per row: |kernel - float64| <= ROW_TOL |ref| + ABS_TOL |scale|, scale = the row's sum of
    |terms| (|W1^T| |dZ1|: the features' gradient is a sum over 64 hidden units that can cancel)."""
    err = (got - ref).norm(dim=1)
    tol = ROW_TOL * ref.norm(dim=1) + ABS_TOL * scale.norm(dim=1) + 1e-30
    bad = (err > tol) & ~tie
    n_bad = int(bad.sum())
    assert n_bad == 0, (what, n_bad, int(tie.sum()), got.shape[0], float((err / tol.clamp(min=1e-30)).max()))


def _abs_scales(pr, ins, dzs, prefix, layers, head=None):
    """Per parameter: the sum over records of |per-record gradient| (float64), the scale the kernels'
    fp32 accumulation of split-bf16 products is accurate against (a weight-gradient sum over
    10^5-10^6 records cancels: its relative error against its own norm is not bounded)."""
    out = {}
    for li, x, dz in zip(layers, ins, dzs):
        dz = dz.detach().abs()
        out[f"{prefix}.{li}.weight"] = (dz.t() @ x.abs()).reshape(pr[f"{prefix}.{li}.weight"].shape)
        out[f"{prefix}.{li}.bias"] = dz.sum(0)
    if head is not None:
        x, dh = head
        out[f"{prefix}.6.weight"] = (dh.abs().unsqueeze(-1) * x.abs()).sum(0).reshape(pr[f"{prefix}.6.weight"].shape)
        out[f"{prefix}.6.bias"] = dh.abs().sum().reshape(1)
    return out


def _check_grads(tr, got, ref_dw, scale, what, tol=1e-4):
    """|kernel - float64| <= tol * ||sum |terms||| per parameter tensor; and <= 2e-3 of the
    reference's own norm (a loose sanity bound that still catches a corrupted section)."""
    for m, pn, shape, o, n in tr.fp.specs:
        if pn not in ref_dw:
            continue
        r = ref_dw[pn].reshape(-1)
        if r.norm() == 0:
            continue
        err = float((got[o:o + n] - r).norm())
        sc = float(scale[pn].norm())
        assert err <= tol * sc, (what, pn, err / sc)
        assert err <= 2e-3 * float(r.norm()), (what, pn, err / float(r.norm()))


# ------------------------------------------------------------------------------------------ CBF
def _capture_cbf(monkeypatch, **cfg):
    tr = Trainer(C.TrainConfig(device="hip", seed=0, dtype="fp32", **cfg), device=DEV)
    assert tr.engine.cbf16
    cap = {}
    orig = native.cbf_bwd

    def spy(*a, **k):
        if k.get("rec") is not None:
            cap["a"], cap["k"] = a, dict(k)
        return orig(*a, **k)

    monkeypatch.setattr(native, "cbf_bwd", spy)
    flat0 = tr.fp.flat.clone()
    tr.train_step()
    torch.cuda.synchronize()
    tr.fp.flat.copy_(flat0)          # the weights of the captured call
    tr.engine.after_update()
    return tr, orig, cap["a"], cap["k"]


def cbf_record_oracle(p, S, rec, T, B, N, K, D):
    """float64 autograd over the records: (dE rows (n, 2D), tie flags (n,), flat dW dict)."""
    Sf = native.from_records(S).double()                        # (T+1, B, Nn, 2D)
    u = rec[:, 1]
    ps = (u < 0).long()
    e = (u & 0x7FFFFFFF).long()
    k = e % K
    i = (e // K) % N
    b = (e // (K * N)) % B
    t = e // (K * N * B)
    j = rec[:, 2].long()
    dh = rec[:, 3].contiguous().view(torch.float32).double()
    ts = t + ps
    si, sj = Sf[ts, b, i], Sf[ts, b, j]
    rel = (si - sj).requires_grad_(True)
    eye = (i == j).double().unsqueeze(-1)
    pr = {n_: v.clone().requires_grad_(True) for n_, v in p.items()}
    d = torch.sqrt((rel[:, :D] ** 2).sum(-1) + C.CBF_DIST_EPS_COORD * D)
    x = torch.cat([rel, eye, (d - C.DIST_MIN_THRES).unsqueeze(-1)], -1)
    mask = (d <= C.OBS_RADIUS).double()
    tie = (d - C.OBS_RADIUS).abs() <= 1e-6
    z = x
    pres, ins = [], []
    for li in (0, 2, 4):
        w, bb = pr[f"cbf_net.{li}.weight"], pr[f"cbf_net.{li}.bias"]
        pre = _lin(z, w, bb)
        tie |= _tie(pre.detach(), z.detach(), w.detach(), bb.detach())
        pres.append(pre)
        ins.append(z.detach())
        z = F.relu(pre)
    h = _lin(z, pr["cbf_net.6.weight"], pr["cbf_net.6.bias"])[:, 0] * mask
    grads = torch.autograd.grad((dh * h).sum(), [rel] + list(pr.values()) + pres)
    notself = (i != j).double().unsqueeze(-1)
    drel = grads[0] * notself                          # self pairs: +i - i cancels, the kernel writes 0
    dws = dict(zip(pr.keys(), grads[1:1 + len(pr)]))
    w1 = pr["cbf_net.0.weight"].detach().reshape(64, -1).abs()
    dz1 = grads[1 + len(pr)].detach().abs()
    rscale = (dz1 @ w1[:, :2 * D] + (dz1 @ w1[:, 2 * D + 1:2 * D + 2])) * notself
    return drel, tie & (mask > 0), dws, _abs_scales(pr, ins, grads[1 + len(pr):], "cbf_net", (0, 2, 4),
                                                    head=(z.detach(), dh * mask)), rscale


@pytest.mark.parametrize("cfg", [
    dict(num_agents=96, num_envs=3, inner_loops=6),
    dict(num_agents=1024, num_envs=4, inner_loops=8),
    dict(num_agents=64, num_envs=2, inner_loops=6, dim=3, num_obstacles=2),
    dict(num_agents=96, num_envs=3, inner_loops=6, reuse_nbr_idx=False),
    dict(num_agents=13, num_envs=5, inner_loops=6),
    dict(num_agents=12, num_envs=3, inner_loops=6),
])
def test_cbf16_matches_fp64_oracle(monkeypatch, cfg):
    tr, orig, a, k = _capture_cbf(monkeypatch, **cfg)
    nact = int(k["nact"][0])
    assert nact > 0
    rec, dE, part = k["rec"][:nact].clone(), k["dE"], k["partial"]
    dE.zero_()
    part.zero_()
    orig(*a, **k)                 # the kernel on exactly the captured inputs
    torch.cuda.synchronize()
    S, idx = a[0], a[1]
    T, B, N, K = idx.shape
    D = tr.cfg.dim
    W = dE.shape[-1]
    ref_rows, tie, ref_dw, scale, rscale = cbf_record_oracle(_params(tr, "cbf"), S, rec, T, B, N, K, D)
    got = native.from_records(dE.view(-1, W)[rec[:, 0].long()]).double()
    _check_rows(got, ref_rows, tie, "cbf dE", rscale)
    assert int(tie.sum()) <= max(8, nact // 20), int(tie.sum())     # ties are rare, not a loophole
    mine = _unpack(tr, L.cbf_grad_map, part.double().sum(0))
    _check_grads(tr, mine, ref_dw, scale, "cbf dW")


# ------------------------------------------------------------------------------- controller edge
def _capture_edge(monkeypatch, **cfg):
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    monkeypatch.setenv("MACBF_NATIVE_BPTT", "0")      # the Python launch loop: the spy sees the calls
    tr = Trainer(C.TrainConfig(device="hip", seed=0, dtype="fp32", **cfg), device=DEV)
    assert tr.engine.eb16_w is not None
    cap = []
    orig = native.ctrl_edge_bwd

    def spy(*a, **k):
        if k.get("w16") is not None and not k.get("_defer"):
            cap.append((a, dict(k)))
        return orig(*a, **k)

    monkeypatch.setattr(native, "ctrl_edge_bwd", spy)
    flat0 = tr.fp.flat.clone()
    tr.train_step()
    torch.cuda.synchronize()
    assert cap, "no 16x16x32 edge backward call"
    # back to the weights the rollout ran with: the saved argmax slots are the max-pool of THAT
    # forward (the backward routes dL/dpooled through them assuming a positive pre-activation)
    tr.fp.flat.copy_(flat0)
    tr.engine.after_update()
    return tr, orig, cap[len(cap) // 2]


def edge_oracle(p, S, idx, argmax, dP, N, D):
    """float64: dL/d(s_i - s_j) (B, N, K, 2D), tie flags (B, N, K), dW dict, for
    L = sum dP * maxpool_{argmax}(mask * relu(W2 relu(W1 [rel, eye] + b1) + b2))."""
    Sf = native.from_records(S).double()                         # (B, Nn, 2D)
    B, _, K = idx.shape
    il = idx.long()
    sj = torch.gather(Sf, 1, il.reshape(B, -1, 1).expand(-1, -1, 2 * D)).reshape(B, N, K, 2 * D)
    rel = (Sf[:, :N].unsqueeze(2) - sj).requires_grad_(True)
    ar = torch.arange(N, device=DEV).view(1, N, 1)
    eye = (il == ar).double().unsqueeze(-1)
    pr = {n_: v.clone().requires_grad_(True) for n_, v in p.items()
          if n_.startswith("controller_centr_net")}
    x = torch.cat([rel, eye], -1)
    d = torch.sqrt((rel[..., :D] ** 2).sum(-1))
    mask = (d < C.OBS_RADIUS).double()
    tie = ((d - C.OBS_RADIUS).abs() <= 1e-6).reshape(-1)
    w1, b1 = pr["controller_centr_net.0.weight"], pr["controller_centr_net.0.bias"]
    w2, b2 = pr["controller_centr_net.2.weight"], pr["controller_centr_net.2.bias"]
    x = x.reshape(-1, x.shape[-1])
    z1 = _lin(x, w1, b1)
    tie |= _tie(z1.detach(), x.detach(), w1.detach(), b1.detach())
    h1 = F.relu(z1)
    z2 = _lin(h1, w2, b2)
    tie |= _tie(z2.detach(), h1.detach(), w2.detach(), b2.detach())
    hm = (F.relu(z2) * mask.reshape(-1, 1)).reshape(B, N, K, -1)
    sl = argmax.long()
    has = (sl < K).double()
    pooled = hm.gather(-2, sl.clamp(max=K - 1).unsqueeze(-2)).squeeze(-2) * has
    dPf = dP[..., :128].double() + dP[..., 128:256].double()          # x3 rows: [hi | lo]
    grads = torch.autograd.grad((dPf * pooled).sum(), [rel] + list(pr.values()) + [z1, z2])
    notself = (il != ar).double().unsqueeze(-1)
    drel = grads[0] * notself                             # self pairs: +i - i cancels, the kernel writes 0
    dws = dict(zip(pr.keys(), grads[1:1 + len(pr)]))
    scale = _abs_scales(pr, [x.detach(), h1.detach()], grads[1 + len(pr):], "controller_centr_net", (0, 2))
    # row scale: |W1^T| (|W2^T| |dZ2| . relu'(Z1)) over the relative-state features
    dz2 = grads[-1].detach().abs()
    s1 = (dz2 @ w2.detach().reshape(128, 64).abs()) * (z1.detach() > 0).double()
    rscale = (s1 @ w1.detach().reshape(64, -1)[:, :2 * D].abs()).reshape(B, N, K, 2 * D) * notself
    return drel, tie.reshape(B, N, K), dws, scale, rscale


@pytest.mark.parametrize("cfg", [
    dict(num_agents=1024, num_envs=4, inner_loops=6),
    dict(num_agents=96, num_envs=3, inner_loops=6),
    dict(num_agents=12, num_envs=3, inner_loops=6),
    dict(num_agents=13, num_envs=5, inner_loops=6),
    dict(num_agents=17, num_envs=3, inner_loops=6),
    dict(num_agents=64, num_envs=2, inner_loops=6, dim=3, num_obstacles=2),
])
def test_eb16_matches_fp64_oracle(monkeypatch, cfg):
    tr, orig, (a, k) = _capture_edge(monkeypatch, **cfg)
    kk = dict(k)
    kk["init"] = True
    kk["partial"] = torch.full_like(k["partial"], float("nan"))    # init must overwrite every row
    kk["dEc"] = torch.zeros_like(k["dEc"])
    orig(*a, **kk)
    torch.cuda.synchronize()
    S, idx, argmax, dP = kk["S"], kk["idx"], kk["argmax"], kk["dP"]
    B, N, K = idx.shape
    D = tr.cfg.dim
    ref_rows, tie, ref_dw, scale, rscale = edge_oracle(_params(tr, "controller"), S, idx, argmax, dP, N, D)
    got = native.from_records(kk["dEc"]).double().reshape(-1, 2 * D)
    _check_rows(got, ref_rows.reshape(-1, 2 * D), tie.reshape(-1), "edge dEc", rscale.reshape(-1, 2 * D))
    assert int(tie.sum()) <= max(8, tie.numel() // 20), int(tie.sum())
    part = kk["partial"].double()
    assert torch.isfinite(part).all()
    mine = _unpack(tr, L.ctrl_edge_grad_map, part.sum(0))
    _check_grads(tr, mine, ref_dw, scale, "edge dW")
