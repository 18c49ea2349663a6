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
