"""Float64 oracles of the 16x16x32 x3 backward kernels, and a start-up self-check.

`cbf_record_oracle` / `edge_oracle` re-evaluate, in float64 autograd, exactly what one call of
csrc/cbf16.h / csrc/ctrl16.h computes from its inputs (tests/test_gpu_oracle16.py pins the kernels
to them on captured training calls). `check(engine)` runs the 16x16x32 kernels the engine uses once
on a small synthetic batch when the engine is built -- CBF and edge (x3) against the oracles, the
node kernel (every precision, csrc/node16.h) against the 32x32x16 node kernel -- and raises
`NativeError` on a disagreement beyond the tolerances below: a toolchain change that miscompiles these schedules (round 3 saw one, see
docs/ARCHITECTURE.md "Scheduling boundary") then stops training instead of corrupting it
(ADVICE r3). MACBF_SELFCHECK=0 skips it.

Tolerances. A row may deviate only on a provable relu / radius tie: some pre-activation
|z| <= TAU * sum |terms| (TAU = 3e-5 is the x3 arithmetic's own bound: each product carries
<= ~2^-16 relative error), or |d - R| <= 1e-6. Otherwise |kernel - float64| <= ROW_TOL |ref| +
ABS_TOL |row scale|, the row scale being the row's sum of |terms| (|W1^T| |dZ1|). Weight gradients:
<= 1e-4 of the per-parameter sum of |per-record gradients|.

Reference ops: /root/reference/cbf.py:13-18,40-43 and /root/reference/controller.py:16-20,43-46,
differentiated by /root/reference/train.py:103.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import config as C
from . import native

TAU = 3e-5
ROW_TOL = 1e-3
ABS_TOL = 1e-4


def _lin(x, w, b):
    return x @ w.reshape(w.shape[0], -1).t() + b


def _tie(pre, x, w, b):
    """Per row: some unit's |pre-activation| within TAU of the sum of its |terms|."""
    scale = x.abs() @ w.reshape(w.shape[0], -1).abs().t() + b.abs()
    return (pre.abs() <= TAU * scale).any(-1)


def bad_rows(got, ref, tie, scale):
    """Rows outside the tolerance that are not ties: (mask, worst err / tol)."""
    err = (got - ref).norm(dim=1)
    tol = ROW_TOL * ref.norm(dim=1) + ABS_TOL * scale.norm(dim=1) + 1e-30
    bad = (err > tol) & ~tie
    return bad, float((err / tol).max()) if err.numel() else 0.0


def abs_scales(pr, ins, dzs, prefix, layers, head=None, tie=None):
    """Per parameter: the sum over records of |per-record gradient| (float64). With a tie mask
    (rows), also "<name>@tie": the same sum over the tie rows only -- a relu / radius flip inside
    the x3 error band may move a weight gradient by up to its tie rows' whole contribution."""
    out = {}
    masks = [("", None)] + ([("@tie", tie.reshape(-1, 1).double())] if tie is not None else [])
    for sfx, m in masks:
        for li, x, dz in zip(layers, ins, dzs):
            dz = dz.detach().abs()
            if m is not None:
                dz = dz * m
            out[f"{prefix}.{li}.weight{sfx}"] = (dz.t() @ x.abs()).reshape(pr[f"{prefix}.{li}.weight"].shape)
            out[f"{prefix}.{li}.bias{sfx}"] = dz.sum(0)
        if head is not None:
            x, dh = head
            dh = dh.abs() if m is None else dh.abs() * m[:, 0]
            out[f"{prefix}.6.weight{sfx}"] = (dh.unsqueeze(-1) * x.abs()).sum(0).reshape(pr[f"{prefix}.6.weight"].shape)
            out[f"{prefix}.6.bias{sfx}"] = dh.sum().reshape(1)
    return out


def cbf_record_oracle(p, S, rec, T, B, N, K, D):
    """Records {u, e | pass << 31, j, dh} of the CBF backward -> float64 (dE rows (n, 2D), tie
    flags (n,), dW dict, |term| scales dict, row scales (n, 2D))."""
    Sf = native.from_records(S).double()                        # (T+1, B, Nn, 2D)
    u = rec[:, 1]
    ps = (u < 0).long()
    e = (u & 0x7FFFFFFF).long()
    i = (e // K) % N
    b = (e // (K * N)) % B
    t = e // (K * N * B)
    j = rec[:, 2].long()
    dh = rec[:, 3].contiguous().view(torch.float32).double()
    ts = t + ps
    rel = (Sf[ts, b, i] - Sf[ts, b, j]).requires_grad_(True)
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
    tie = tie & (mask > 0)
    scales = abs_scales(pr, ins, grads[1 + len(pr):], "cbf_net", (0, 2, 4), head=(z.detach(), dh * mask), tie=tie)
    return drel, tie, dws, scales, rscale


def edge_forward(p, S, idx, N, D):
    """float64 edge MLP of the controller: (rel (B,N,K,2D) leaf, pre-activations, hm (B,N,K,128))."""
    Sf = native.from_records(S).double()                         # (B, Nn, 2D)
    B, _, K = idx.shape
    il = idx.long()
    sj = torch.gather(Sf, 1, il.reshape(B, -1, 1).expand(-1, -1, 2 * D)).reshape(B, N, K, 2 * D)
    rel = (Sf[:, :N].unsqueeze(2) - sj).requires_grad_(True)
    ar = torch.arange(N, device=S.device).view(1, N, 1)
    eye = (il == ar).double().unsqueeze(-1)
    return rel, eye, il, ar


def edge_oracle(p, S, idx, argmax, dP, N, D):
    """float64: dL/d(s_i - s_j) (B, N, K, 2D), tie flags (B, N, K), dW dict, |term| scales, row
    scales, for L = sum dP * maxpool_{argmax}(mask * relu(W2 relu(W1 [rel, eye] + b1) + b2)); the
    max-pool is routed through the given argmax slots (the kernel's saved ones)."""
    B, _, K = idx.shape
    rel, eye, il, ar = edge_forward(p, S, idx, N, D)
    pr = {n_: v.clone().requires_grad_(True) for n_, v in p.items() if n_.startswith("controller_centr_net")}
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
    scales = abs_scales(pr, [x.detach(), h1.detach()], grads[1 + len(pr):], "controller_centr_net", (0, 2),
                        tie=tie)
    dz2 = grads[-1].detach().abs()
    s1 = (dz2 @ w2.detach().reshape(128, 64).abs()) * (z1.detach() > 0).double()
    rscale = (s1 @ w1.detach().reshape(64, -1)[:, :2 * D].abs()).reshape(B, N, K, 2 * D) * notself
    return drel, tie.reshape(B, N, K), dws, scales, rscale


def _params(fp, module):
    return {pn: fp.flat[o:o + n].view(shape).detach().double() for m, pn, shape, o, n in fp.specs if m == module}


def _synthetic_states(B, N, D, T, gen, dev):
    L_ = max(1.0, N / C.AGENT_DENSITY) ** (1.0 / D)
    p = torch.rand(T, B, N, D, generator=gen) * L_
    v = (torch.rand(T, B, N, D, generator=gen) - 0.5) * 1.2
    s = torch.cat([p, v], -1).to(dev)
    return s


@torch.no_grad()
def _knn(s, K, D):
    d2 = ((s[..., :, None, :D] - s[..., None, :, :D]) ** 2).sum(-1)
    return d2.topk(K, dim=-1, largest=False).indices.to(torch.int32).contiguous()


def check(engine) -> dict:
    """Run the 16x16x32 backward kernels this engine uses once on a synthetic batch: the CBF and
    edge kernels (x3) against the float64 oracles, the node kernel (every precision) against the
    independent 32x32x16 node kernel. Raises native.NativeError on a disagreement; returns a small
    report."""
    pw = engine.pw
    dev = engine.dev
    D = engine.D
    gen = torch.Generator().manual_seed(1234)
    B, N, T, K = 2, 48, 2, 12
    rep = {}
    fp = engine.tr.fp
    if engine.node16_w is not None:
        rep["node16"] = _node_check(engine, gen)
    if not pw.x3 or not (engine.dedup and getattr(engine, "cbf16", False)):
        return rep
    # ---- CBF backward over every (pass, t, b, i, k) record, random upstream gradients
    s = _synthetic_states(B, N, D, T + 1, gen, dev)
    S = native.to_records(s).contiguous()                       # (T+1, B, N, W)
    idx = _knn(s[:T], K, D)                                     # (T, B, N, K)
    E = T * B * N * K
    e = torch.arange(E, device=dev, dtype=torch.int64)
    rec = torch.zeros(2 * E, 4, dtype=torch.int32, device=dev)
    j = idx.reshape(-1).to(torch.int64)
    dh = (torch.rand(2 * E, generator=gen) - 0.5).to(dev).float()
    rec[:, 0] = torch.arange(2 * E, device=dev, dtype=torch.int32)
    rec[:E, 1] = e.to(torch.int32)
    rec[E:, 1] = (e - (1 << 31)).to(torch.int32)              # e | pass << 31 as int32 (pass 1: s_{t+1})
    rec[:E, 2] = j.to(torch.int32)
    rec[E:, 2] = j.to(torch.int32)
    # the kernel's contract (cbf_dh / cbf_compact): records carry dh = 0 outside the radius mask (h is
    # masked there, its gradient zero) -- the kernel itself does not re-apply the mask
    Sf = native.from_records(S).double()
    ps = torch.cat([torch.zeros(E, dtype=torch.int64, device=dev), torch.ones(E, dtype=torch.int64, device=dev)])
    ee = torch.cat([e, e])
    ii, bb_, tt = (ee // K) % N, (ee // (K * N)) % B, ee // (K * N * B)
    jj = torch.cat([j, j])
    rel = Sf[tt + ps, bb_, ii, :D] - Sf[tt + ps, bb_, jj, :D]
    dist = torch.sqrt((rel ** 2).sum(-1) + C.CBF_DIST_EPS_COORD * D)
    dh = torch.where(dist <= C.OBS_RADIUS, dh.double(), torch.zeros_like(dist)).float()
    rec[:, 3] = dh.view(torch.int32)
    W = S.shape[-1]
    dE = torch.zeros(2, T, B, N, K, W, dtype=torch.float32, device=dev)
    nbb = native.cbf_bwd_grid(2 * E, dev)
    part = torch.zeros(nbb, native.CBF_PARTIAL, dtype=torch.float32, device=dev)
    src = torch.zeros(2 * E, dtype=torch.int32, device=dev)
    nev = torch.full((1,), 2 * E, dtype=torch.int32, device=dev)
    nact = torch.full((1,), 2 * E, dtype=torch.int32, device=dev)
    native.cbf_bwd(S, idx, torch.zeros(2, T, B, N, K, device=dev), pw.cbf_w, pw.cbf_off["w1f"], pw.cbf_rm, pw.cbf_v,
                   passes=2, dE=dE, partial=part, num_blocks=nbb, idx1=idx, src=src, nev=nev, nact=nact,
                   prec=pw.prec, rec=rec, wrm16=pw.cbf_rm16, w16=pw.cbf_w16)
    torch.cuda.synchronize(dev)
    with torch.enable_grad():
        ref, tie, _, _, rscale = cbf_record_oracle(_params(fp, "cbf"), S, rec, T, B, N, K, D)
    got = native.from_records(dE.view(-1, W)[rec[:, 0].long()]).double()
    bad, worst = bad_rows(got, ref, tie, rscale)
    rep["cbf16"] = {"rows": int(got.shape[0]), "bad": int(bad.sum()), "ties": int(tie.sum()), "worst_err_over_tol": worst}
    if int(bad.sum()):
        raise native.NativeError(f"16x16x32 CBF backward self-check failed: {rep['cbf16']} (toolchain / schedule "
                                 f"miscompile? see docs/ARCHITECTURE.md; MACBF_SELFCHECK=0 skips)")
    # ---- controller edge backward (K = 12), argmax slots = the true masked max-pool
    if engine.eb16_w is not None and pw.x3:
        s1 = s[0]
        S1 = native.to_records(s1).contiguous()
        idx1 = idx[0]
        p = _params(fp, "controller")
        with torch.no_grad():
            rel, eye, il, ar = edge_forward(p, S1, idx1, N, D)
            x = torch.cat([rel, eye], -1)
            d = torch.sqrt((rel[..., :D] ** 2).sum(-1))
            m_ = (d < C.OBS_RADIUS).double().unsqueeze(-1)
            h2 = F.relu(_lin(F.relu(_lin(x, p["controller_centr_net.0.weight"], p["controller_centr_net.0.bias"])),
                             p["controller_centr_net.2.weight"], p["controller_centr_net.2.bias"])) * m_
            mx = h2.max(dim=2)
            am = torch.where(mx.values > 0, mx.indices, torch.full_like(mx.indices, 255)).to(torch.uint8).contiguous()
        dPv = (torch.rand(B, N, 128, generator=gen) - 0.5).to(dev)
        hi = dPv.to(torch.bfloat16)
        lo = (dPv - hi.float()).to(torch.bfloat16)
        dP = torch.cat([hi, lo], -1).contiguous()
        dEc = torch.zeros(B, N, K, W, dtype=torch.float32, device=dev)
        nbe = max(1, min((B * N + 127) // 128, native.num_cu(dev)))
        pe = torch.zeros(nbe, native.CTRL_EDGE_PARTIAL, dtype=torch.float32, device=dev)
        native.ctrl_edge_bwd(S1, idx1, am, dP, pw.ctrl_w, pw.ctrl_off["ew1f"], pw.ctrl_off["ew2tn"], dEc, pe, nbe,
                             prec=pw.prec, init=True, w16=engine.eb16_w)
        torch.cuda.synchronize(dev)
        with torch.enable_grad():
            ref, tie, _, _, rscale = edge_oracle(p, S1, idx1, am, dP, N, D)
        got = native.from_records(dEc).double().reshape(-1, 2 * D)
        bad, worst = bad_rows(got, ref.reshape(-1, 2 * D), tie.reshape(-1), rscale.reshape(-1, 2 * D))
        rep["eb16"] = {"rows": int(got.shape[0]), "bad": int(bad.sum()), "ties": int(tie.sum()), "worst_err_over_tol": worst}
        if int(bad.sum()):
            raise native.NativeError(f"16x16x32 edge backward self-check failed: {rep['eb16']} (toolchain / schedule "
                                     f"miscompile? see docs/ARCHITECTURE.md; MACBF_SELFCHECK=0 skips)")
    return rep


# node16 vs the 32x32x16 node kernel: both fp32-accurate in x3 (different accumulation orders);
# the 1-pass builds round the activations to 16 bits at the same points, so a rounding can flip:
# the bounds of the bf16 / fp16 full-step tests
NODE_TOL = {"fp32": 1e-4, "bf16": 2e-2, "fp16": 2e-2}


def _rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def _node_check(engine, gen, B=2, N=256) -> dict:
    """One reverse step of the controller node backward (dL/dpooled rows, ego terms, weight
    gradients) on synthetic inputs, 16x16x32 kernel (csrc/node16.h) against 32x32x16
    (csrc/ctrl.hip node_bwd_body), 128-agent chunks both (node16 is the default node
    kernel of every precision)."""
    from . import layout as L
    pw = engine.pw
    dev, D = engine.dev, engine.D
    W = native.rec_width(D)
    prow = L.pooled_row(pw.prec)
    s = _synthetic_states(B, N, D, 1, gen, dev)[0]
    S = native.to_records(s).contiguous()
    G = (s[..., :D] + (torch.rand(B, N, D, generator=gen).to(dev) - 0.5)).contiguous()
    A = ((torch.rand(B, N, D, generator=gen) - 0.5) * 2.0).to(dev).contiguous()
    Gn = native.to_records((torch.rand(B, N, 2 * D, generator=gen) - 0.5).to(dev)).contiguous()
    pv = torch.rand(B, N, 128, generator=gen).to(dev) * (torch.rand(B, N, 128, generator=gen).to(dev) > 0.3)
    hi = pv.to(engine.hdt)
    pooled = (torch.cat([hi, (pv - hi.float()).to(engine.hdt)], -1) if prow == 256 else hi).contiguous()
    valid = torch.ones(B, dtype=torch.uint8, device=dev)
    act_cnt = torch.full((1,), float(B * N), dtype=torch.float32, device=dev)
    nb = max(1, min((B * N + 127) // 128, native.num_cu(dev)))
    offs = {pn: o for (m, pn, shape, o, n) in engine.tr.fp.specs}
    out = {}
    for mode, wrm16, gmap in (("16", pw.node_rm16, L.ctrl_node16_grad_map), ("32", None, L.ctrl_node_grad_map)):
        dP = torch.zeros(B, N, prow, dtype=engine.hdt, device=dev)
        ego = torch.zeros(B, N, W, dtype=torch.float32, device=dev)
        part = torch.zeros(nb, native.CTRL_NODE_PARTIAL, dtype=torch.float32, device=dev)
        native.ctrl_node_bwd(pooled, S, G, A, Gn, valid, pw.ctrl_rm, pw.node_rm_off, pw.ctrl_v, 0.37, dP, ego, part, nb,
                             act_cnt=act_cnt, prec=pw.prec, init=True, chunk=128, wrm16=wrm16)
        torch.cuda.synchronize(dev)
        red = part.double().sum(0)
        sm, dm = gmap(offs, D)
        g = torch.zeros(engine.tr.fp.numel, dtype=torch.float64, device=dev)
        g.index_add_(0, torch.as_tensor(dm, device=dev), red[torch.as_tensor(sm, device=dev)])
        dPf = dP[..., :128].double() + (dP[..., 128:].double() if prow == 256 else 0.0)
        out[mode] = (dPf, ego.double(), g)
    tol = NODE_TOL[pw.prec]
    new, old = out["16"], out["32"]
    errs = {"dP": _rel(new[0], old[0]), "ego": _rel(new[1], old[1])}
    for m, pn, shape, o, n in engine.tr.fp.specs:
        if pn.startswith("controller_dec_net"):
            errs[pn] = _rel(new[2][o:o + n], old[2][o:o + n])
    worst = max(errs.items(), key=lambda kv: kv[1])
    finite = all(bool(torch.isfinite(x).all()) for x in new)
    rep = {"agents": B * N, "worst": worst[0], "worst_rel": worst[1], "tol": tol}
    if not finite or worst[1] > tol:
        raise native.NativeError(f"16x16x32 node backward self-check failed: {rep} (toolchain / schedule miscompile? "
                                 f"see docs/ARCHITECTURE.md; MACBF_SELFCHECK=0 skips)")
    return rep


def enabled() -> bool:
    return os.environ.get("MACBF_SELFCHECK", "1") != "0"
