"""Device checks of the hardware layouts every fused kernel relies on (MI355X only):
v_mfma_f32_32x32x16_bf16 operand/accumulator maps and ds_read_b64_tr_b16 semantics."""
import numpy as np
import pytest
import torch

from macbf_gnn_amd.ops import layout as L
from macbf_gnn_amd.ops import native

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def test_mfma_layout_exact():
    rng = np.random.default_rng(0)
    A = rng.integers(-4, 5, size=(32, 16)).astype(np.float32)
    B = rng.integers(-4, 5, size=(16, 32)).astype(np.float32)   # asymmetric
    a = np.zeros((64, 8), np.float32)
    b = np.zeros((64, 8), np.float32)
    for l in range(64):
        r, h = l & 31, l >> 5
        a[l] = A[r, 8 * h:8 * h + 8]
        b[l] = B[8 * h:8 * h + 8, r]
    ta = torch.tensor(a, dtype=torch.bfloat16, device=DEV).contiguous()
    tb = torch.tensor(b, dtype=torch.bfloat16, device=DEV).contiguous()
    d = torch.zeros(64, 16, dtype=torch.float32, device=DEV)
    assert native.probe_lib().probe_mfma(ta.data_ptr(), tb.data_ptr(), d.data_ptr(), native.stream_handle()) == 0
    torch.cuda.synchronize()
    d = d.cpu().numpy()
    D = np.zeros((32, 32), np.float32)
    for l in range(64):
        r, h = l & 31, l >> 5
        for reg in range(16):
            D[L.acc_row(reg, h), r] = d[l, reg]
    np.testing.assert_array_equal(D, A @ B)


@pytest.mark.parametrize("stride,e0,m0", [(64, 0, 0), (64, 16, 32), (72, 8, 0), (128, 0, 96)])
def test_tr16_transposed_fragment(stride, e0, m0):
    rows = 32 if stride <= 72 else 40
    img = (np.arange(rows * stride) % 251).astype(np.float32).reshape(rows, stride)
    t = torch.tensor(img, dtype=torch.bfloat16, device=DEV).contiguous()
    out = torch.zeros(64, 8, dtype=torch.bfloat16, device=DEV)
    assert native.probe_lib().probe_tr(t.data_ptr(), rows, stride, e0, m0, out.data_ptr(), native.stream_handle()) == 0
    torch.cuda.synchronize()
    got = out.float().cpu().numpy()
    exp = np.zeros((64, 8), np.float32)
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(8):
            exp[l, j] = img[e0 + 8 * h + j, m0 + r]
    np.testing.assert_array_equal(got, exp)


def test_lane_xor_exchanges_and_reductions():
    """lane_xor<O> (DPP / permlane, common.h) returns lane (l ^ O)'s value for every O, and the wave
    reductions built on it equal the xor-butterfly reference bit for bit (same pairing order)."""
    rng = np.random.default_rng(3)
    vals = rng.standard_normal(64).astype(np.float32)
    vin = torch.tensor(vals.view(np.uint32).astype(np.int64), dtype=torch.int64).to(torch.int32).to(DEV)
    out = torch.zeros(9 * 64, dtype=torch.int32, device=DEV)
    assert native.probe_lib().probe_lane_xor(vin.data_ptr(), out.data_ptr(), native.stream_handle()) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.int64).astype(np.uint32).reshape(9, 64)
    bits = vals.view(np.uint32)
    lanes = np.arange(64)
    for s in range(6):
        np.testing.assert_array_equal(got[s], bits[lanes ^ (1 << s)], err_msg=f"xor {1 << s}")

    def butterfly(x, dists, op):
        x = x.copy()
        for o in dists:
            x = op(x, x[lanes ^ o]).astype(np.float32)
        return x
    ws = butterfly(vals, [32, 16, 8, 4, 2, 1], lambda a, b: a + b)
    wm = butterfly(vals, [32, 16, 8, 4, 2, 1], np.maximum)
    s32 = butterfly(vals, [16, 8, 4, 2, 1], lambda a, b: a + b)
    np.testing.assert_array_equal(got[6], ws.view(np.uint32))
    np.testing.assert_array_equal(got[7], wm.view(np.uint32))
    np.testing.assert_array_equal(got[8], s32.view(np.uint32))


def test_mfma16_layout_exact():
    """v_mfma_f32_16x16x32_bf16 (the x3 CBF backward, csrc/cbf16.h): lane (n = l & 15, g = l >> 4)
    holds A[n][8g + j], B[8g + j][n] and D[4g + i][n] (layout.emu_mfma16)."""
    rng = np.random.default_rng(5)
    a = rng.integers(-4, 5, size=(64, 8)).astype(np.float32)
    b = rng.integers(-4, 5, size=(64, 8)).astype(np.float32)
    ta = torch.tensor(a, dtype=torch.bfloat16, device=DEV).contiguous()
    tb = torch.tensor(b, dtype=torch.bfloat16, device=DEV).contiguous()
    d = torch.zeros(64, 4, dtype=torch.float32, device=DEV)
    assert native.probe_lib().probe_mfma16(ta.data_ptr(), tb.data_ptr(), d.data_ptr(), native.stream_handle()) == 0
    torch.cuda.synchronize()
    d = d.cpu().numpy()
    D = np.zeros((16, 16), np.float32)
    for l in range(64):
        n, g = l & 15, l >> 4
        for i in range(4):
            D[L.acc_row16(i, g), n] = d[l, i]
    np.testing.assert_array_equal(D, L.emu_mfma16(a, b))


def test_mfma_under_wave_condition():
    """The round-4 hazard (csrc/common.h wave_id()): a wave-parity-conditional MFMA. With the
    condition on wave_id() (scalar branch) the result equals the reference for every wave; the
    VGPR-condition build is run too and its deviation recorded (printed), documenting what the
    hardware does with an MFMA in a block the compiler left without its execz skip."""
    rng = np.random.default_rng(3)
    a = rng.integers(-3, 4, size=(4, 2, 64, 8)).astype(np.float32)
    ta = torch.tensor(a, dtype=torch.bfloat16, device=DEV).contiguous()
    outs = {}
    for uniform in (1, 0):
        o = torch.full((512, 4), float("nan"), dtype=torch.float32, device=DEV)
        assert native.probe_lib().probe_mfma_exec(ta.data_ptr(), o.data_ptr(), uniform, native.stream_handle()) == 0
        torch.cuda.synchronize()
        outs[uniform] = o.cpu().numpy()
    # reference: X (16 x 32), X[n][8g + j] = a[lane (n, g)][j]; acc = sum X X^T, bias = row sums
    X = np.zeros((4, 2, 16, 32), np.float32)
    for l in range(64):
        n, g = l & 15, l >> 4
        X[:, :, n, 8 * g:8 * g + 8] = a[:, :, l]
    acc = sum(X[i, u] @ X[i, u].T for i in range(4) for u in range(2))
    ref = np.zeros((512, 4), np.float32)
    for w in range(8):
        bias = sum(X[i, w & 1].sum(1) for i in range(4))          # (16,) per output row
        C = acc + bias[:, None]
        for l in range(64):
            n, g = l & 15, l >> 4
            ref[w * 64 + l] = C[4 * g:4 * g + 4, n]
    np.testing.assert_array_equal(outs[1], ref)
    dev = float(np.nanmax(np.abs(outs[0] - ref)))
    print(f"VGPR-condition build: max |deviation| = {dev} (0: the hardware skipped the masked MFMA)")
