"""The 16x16x32 x3 controller edge backward (csrc/ctrl16.h: 16 agents per wave, two waves per SIMD)
against the 32x32x16 x3 kernel on the same captured BPTT step: the reduced weight-gradient slab
(dW2, db2, dW1f) and dL/d(s_i - s_j) of every edge. Both are fp32-accurate split-bf16 products with
fp32 accumulation in different orders. Reference op: /root/reference/controller.py:43-50 backward
(train.py:103)."""
import pytest
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd.engine import Trainer
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
SECTIONS = {"dW2": (0, 8192), "db2": (8192, 8320)}


def _capture(monkeypatch, **cfg):
    monkeypatch.setenv("MACBF_EB16", "1")
    monkeypatch.setenv("MACBF_BWD_FUSED", "0")
    monkeypatch.setenv("MACBF_NATIVE_BPTT", "0")      # the Python launch loop: the spy sees the calls
    tr = Trainer(C.TrainConfig(device="hip", seed=0, **cfg), device=DEV)
    assert tr.engine.eb16_w is not None
    cap = []
    orig = native.ctrl_edge_bwd

    def spy(*a, **k):
        if k.get("w16") is not None and not k.get("_defer"):
            cap.append((a, dict(k)))
        return orig(*a, **k)

    monkeypatch.setattr(native, "ctrl_edge_bwd", spy)
    tr.train_step()
    torch.cuda.synchronize()
    assert cap, "no 16x16x32 edge backward call"
    return orig, cap[len(cap) // 2]


@pytest.mark.parametrize("cfg", [
    dict(num_agents=1024, num_envs=4, inner_loops=6),
    dict(num_agents=96, num_envs=3, inner_loops=6),
    dict(num_agents=64, num_envs=2, inner_loops=6, dim=3, num_obstacles=2),
])
def test_eb16_matches_eb32(monkeypatch, cfg):
    orig, (a, k) = _capture(monkeypatch, **cfg)
    outs = {}
    for mode in ("new", "old"):
        kk = dict(k)
        kk["init"] = True
        kk["partial"] = torch.full_like(k["partial"], float("nan"))    # init must overwrite every row
        kk["dEc"] = torch.zeros_like(k["dEc"])
        if mode == "old":
            kk.pop("w16")
        orig(*a, **kk)
        torch.cuda.synchronize()
        outs[mode] = (kk["dEc"], kk["partial"].double())
    pn, po = outs["new"][1], outs["old"][1]
    assert torch.isfinite(pn).all()
    sn, so = pn.sum(0), po.sum(0)
    for name, (lo, hi) in SECTIONS.items():
        err = float((sn[lo:hi] - so[lo:hi]).norm() / so[lo:hi].norm().clamp(min=1e-30))
        assert err < 2e-5, (name, err)
    w1n = sn[8320:10368].view(64, 32)[:, :16]
    w1o = so[8320:10368].view(64, 32)[:, :16]
    assert float((w1n - w1o).norm() / w1o.norm()) < 2e-5
    dn, do = outs["new"][0].flatten(0, -2).double(), outs["old"][0].flatten(0, -2).double()
    assert float((dn - do).norm() / do.norm()) < 1e-4
    bad = ((dn - do).norm(dim=1) > 1e-2 * do.norm(dim=1) + 1e-9).sum().item()
    assert bad <= max(2, dn.shape[0] // 20000), bad
