"""Host-side argument checks of the native wrappers (CPU: they raise before any device work)."""
import pytest
import torch

from macbf_gnn_amd.ops import native


@pytest.mark.parametrize("lanes", [1, 2, 5, 16])
def test_scan_rejects_unsupported_lane_layouts(lanes):
    S = torch.zeros(1, 16, 4)
    idx = torch.zeros(1, 16, 12, dtype=torch.int32)
    with pytest.raises(native.NativeError, match="lanes"):
        native.scan(S, idx, None, None, None, K=12, lanes=lanes)


def test_edge_backward_grid_one_workgroup_per_cu_for_x3(monkeypatch):
    """The x3 edge backward holds one workgroup per CU: its grid is capped at the CU count
    (the 16-bit builds at two per CU); MACBF_EDGE_WG_PER_CU overrides."""
    monkeypatch.setattr(native, "num_cu", lambda device=None: 256)
    monkeypatch.delenv("MACBF_EDGE_WG_PER_CU", raising=False)
    monkeypatch.delenv("MACBF_NODE_CHUNK", raising=False)
    agents = 64 * 1024
    _, e_x3 = native.ctrl_bwd_grids(agents, None, "fp32")
    _, e_bf = native.ctrl_bwd_grids(agents, None, "bf16")
    assert e_x3 == 256 and e_bf == 512
    monkeypatch.setenv("MACBF_EDGE_WG_PER_CU", "2")
    assert native.ctrl_bwd_grids(agents, None, "fp32")[1] == 512


def test_scan_plans_of_the_production_configs():
    """The scan launcher's plan (csrc/scan.hip mb_scan_plan; host logic, no launch) for the
    BASELINE shapes at 256 CUs: the instantiations tests/test_gpu_scan_plans.py pins to the oracle."""
    p = native.scan_plan(64, 1024, 12, prev=True)
    assert (p["bs"], p["lpa"], p["use_cells"], p["cell_g"]) == (1024, 4, 1, 24)
    p = native.scan_plan(64, 1024, 12, Nn=1120, dim=3, prev=True)
    assert (p["bs"], p["lpa"], p["use_cells"], p["cell_g"], p["wave_atomic"]) == (512, 4, 1, 10, 1)
    p = native.scan_plan(8, 1024, 12, prev=True)
    assert (p["bs"], p["lpa"], p["use_cells"], p["cell_g"]) == (256, 8, 1, 16)
    p = native.scan_plan(1, 20000, 12, prev=True)
    assert p["glb"] == 1 and p["cells"] == 0


def test_scan_cell_lds_only_when_searched():
    """Safety-only scans (the rollout's tail) and first steps (no temporal bound) never search
    the cell grid and do not allocate its LDS."""
    base = native.scan_plan(64, 1024, 12, prev=True)
    for kw in (dict(do_knn=False, prev=True), dict(prev=False)):
        p = native.scan_plan(64, 1024, 12, **kw)
        assert p["cells"] == 0 and p["use_cells"] == 0 and p["lds"] < base["lds"], kw
    assert base["cells"] == 1 and base["lds"] <= 160 * 1024
