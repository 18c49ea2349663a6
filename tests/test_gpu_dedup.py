"""GPU: the deduplicated CBF path (csrc/dedup.hip + cbf_hfwd + non-fused cbf_bwd on the
evaluation list + node_reduce with map1) against its pure-torch index reference and against
the fused two-evaluation kernel."""
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.ops import native
from macbf_gnn_amd.ops.dedup import match_reference

from test_gpu_backward import _cmp, _states, _trainer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("recomputed", [False, True])
def test_cbf_match_equals_reference(recomputed):
    T, B, N, K = 4, 2, 50, C.TOP_K
    S = _states((T + 1, B), N, seed=4, vscale=1.5).contiguous()
    Tg = T + int(recomputed)
    idx = torch.stack([O.knn_idx(S[t], K) for t in range(Tg)]).to(torch.int32).contiguous()
    E = T * B * N * K
    map1 = torch.full((T, B, N, K), -7, dtype=torch.int32, device=DEV)
    src = torch.full((2 * E,), -7, dtype=torch.int32, device=DEV)
    cnt = torch.zeros(T * B * N, dtype=torch.int32, device=DEV)
    nev = native.cbf_match(idx, T, map1, src, cnt, recomputed=recomputed)
    m_ref, s_ref, n_ref = match_reference(idx, T, recomputed=recomputed)
    torch.cuda.synchronize()
    assert int(nev) == n_ref
    assert torch.equal(map1.cpu().long(), m_ref)
    assert torch.equal(src[:n_ref].cpu().long(), s_ref[:n_ref])
    if not recomputed:
        assert n_ref > E            # the states move: some neighbour sets change


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("reuse", [True, False])
def test_dedup_step_matches_fused_kernel(reuse, prec):
    """One training step: deduplicated evaluation list vs the fused h/h' kernel (same
    semantics, different evaluation order; bf16: the summed upstream grads dh + dh' of a
    shared evaluation are rounded once instead of twice -> a looser bound)."""
    a = _trainer(DEV, N=96, B=3, T=6, reuse_nbr_idx=reuse, cbf_dedup=True, dtype=prec)
    b = _trainer(DEV, N=96, B=3, T=6, reuse_nbr_idx=reuse, cbf_dedup=False, dtype=prec)
    rel = 1e-4 if prec == "fp32" else 2e-2
    assert a.engine.dedup and not b.engine.dedup
    s0, g, _ = a.sample()
    sa = a.engine.step(s0, g)
    ga = a.fp.grad.clone()
    sb = b.engine.step(s0, g)
    gb = b.fp.grad.clone()
    for name in ("controller", "cbf"):
        lo, hi = a.fp.ranges[name]
        _cmp(ga[lo:hi], gb[lo:hi], name, rel=rel)
    for k in ("loss_dang", "loss_safe", "loss_dang_deriv", "loss_safe_deriv", "loss_action",
              "acc_dang_sum", "acc_safe_sum", "acc_dang_deriv_sum", "acc_safe_deriv_sum"):
        x, y = float(sa[k]), float(sb[k])
        assert abs(x - y) <= 2e-3 * abs(y) + 1e-5, (k, x, y)
    # the per-step state gradients (CBF -> dS) agree too
    _cmp(a.engine.dS, b.engine.dS, "dS", rel=rel)


def test_dedup_deterministic():
    tr = _trainer(DEV, N=64, B=3, T=5)
    assert tr.engine.dedup
    s0, g, _ = tr.sample()
    tr.engine.step(s0, g)
    g1 = tr.fp.grad.clone()
    tr.engine.step(s0, g)
    assert torch.equal(g1, tr.fp.grad)
