"""Dump raw v_smfmac_f32_32x32x32_bf16 inputs/outputs (random small integers) for layout analysis."""
import numpy as np
import torch
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from macbf_gnn_amd.ops import native

rng = np.random.default_rng(1)
out = {}
for trial in range(4):
    a = rng.integers(-4, 5, size=(64, 8)).astype(np.float32)
    b = rng.integers(-4, 5, size=(64, 16)).astype(np.float32)
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    idx = np.zeros(64, np.int64)
    for l in range(64):
        v = 0
        for g in range(8):      # 8 nibbles: one valid (i0 < i1) pair each
            i0, i1 = pairs[rng.integers(0, 6)] if trial else pairs[(l + g) % 6]
            v |= (i0 | (i1 << 2)) << (4 * g)
        idx[l] = v
    idx = idx.astype(np.uint32).view(np.int32)
    ta = torch.tensor(a, dtype=torch.bfloat16, device="cuda").contiguous()
    tb = torch.tensor(b, dtype=torch.bfloat16, device="cuda").contiguous()
    ti = torch.tensor(idx, dtype=torch.int32, device="cuda").contiguous()
    d = torch.zeros(64, 16, dtype=torch.float32, device="cuda")
    assert native.lib().probe_smfmac(ta.data_ptr(), tb.data_ptr(), ti.data_ptr(), d.data_ptr(), native.stream_handle()) == 0
    torch.cuda.synchronize()
    out[f"a{trial}"], out[f"b{trial}"], out[f"i{trial}"], out[f"d{trial}"] = a, b, idx, d.cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/smfmac_probe.npz", **out)
print("saved", list(out)[:4])
