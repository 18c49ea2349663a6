"""CPU checks of the MFMA fragment packing with a lane-level emulator of
v_mfma_f32_32x32x16_bf16 (layouts from the CDNA4 guide). If these pass, the index
arithmetic the HIP kernels rely on is consistent; the GPU tests then check the kernels."""
import numpy as np
import torch

from macbf_gnn_amd.models import CBF, Controller
from macbf_gnn_amd.ops import layout as L
from macbf_gnn_amd.utils.params import FlatParams


def _setup():
    torch.manual_seed(0)
    ctrl, cbf = Controller(4), CBF(4)
    fp = FlatParams({"controller": ctrl, "cbf": cbf})
    offs = {pn: o for (m, pn, shape, o, n) in fp.specs}
    src = np.concatenate([fp.flat.numpy().astype(np.float64), [0.0, 1.0]])
    return ctrl, cbf, fp, offs, src


def _vals(packer, src, nflat):
    return src[L.resolve(packer.index(), nflat)]


def acc_to_mat(c):
    """(64,16) accumulator regs -> (32,32) matrix D[row][col]."""
    D = np.zeros((32, 32))
    for l in range(64):
        r, h = l & 31, l >> 5
        for reg in range(16):
            D[L.acc_row(reg, h), r] = c[l, reg]
    return D


def bias_init(b, mt):
    c = np.zeros((64, 16))
    for l in range(64):
        h = l >> 5
        for reg in range(16):
            c[l, reg] = b[32 * mt + L.acc_row(reg, h)]
    return c


def test_emulated_cbf_chain_matches_mlp():
    ctrl, cbf, fp, offs, src = _setup()
    pk = L.cbf_packer(offs)
    vals = _vals(pk, src, fp.numel)
    fo = pk.offsets()
    rng = np.random.default_rng(1)
    X = rng.normal(size=(32, 6))          # 32 edges x 6 features
    # B operand of layer 1: lane (edge r, h): hi features in h=0 (+const 1 at k=6), zeros in h=1
    Fb = np.zeros((64, 8))
    for l in range(64):
        r, h = l & 31, l >> 5
        if h == 0:
            Fb[l, :6] = X[r]
            Fb[l, 6] = 1.0
    H1 = [np.maximum(L.emu_mfma(L.emu_frag(vals, fo["w1f"] + mt), Fb, np.zeros((64, 16))), 0) for mt in range(2)]
    W2b = cbf.cbf_net[2].bias.detach().numpy()
    H2 = []
    for mt in range(4):
        c = bias_init(W2b, mt)
        for kk in range(4):
            c = L.emu_mfma(L.emu_frag(vals, fo["w2"] + mt * 4 + kk), L.emu_acc_frag(H1[kk >> 1], kk & 1), c)
        H2.append(np.maximum(c, 0))
    b3 = cbf.cbf_net[4].bias.detach().numpy()
    H3 = []
    for mt in range(2):
        c = bias_init(b3, mt)
        for kk in range(8):
            c = L.emu_mfma(L.emu_frag(vals, fo["w3"] + mt * 8 + kk), L.emu_acc_frag(H2[kk >> 1], kk & 1), c)
        H3.append(np.maximum(c, 0))
    got = np.concatenate([acc_to_mat(H3[0]), acc_to_mat(H3[1])], 0)     # (64, 32)
    net = cbf.cbf_net
    with torch.no_grad():
        x = torch.tensor(X, dtype=torch.float32)
        ref = torch.relu(torch.nn.functional.linear(x, net[0].weight[..., 0], net[0].bias))
        ref = torch.relu(torch.nn.functional.linear(ref, net[2].weight[..., 0], net[2].bias))
        ref = torch.relu(torch.nn.functional.linear(ref, net[4].weight[..., 0], net[4].bias))
    np.testing.assert_allclose(got, ref.numpy().T, rtol=1e-4, atol=1e-5)

    # backward data chain: dH2 = W3^T dH3 with w3t packed, dH1 = W2^T dH2 with w2t
    dH3 = [rng.normal(size=(64, 16)) for _ in range(2)]
    dH2 = []
    for mt in range(4):
        c = np.zeros((64, 16))
        for kk in range(4):
            c = L.emu_mfma(L.emu_frag(vals, fo["w3t"] + mt * 4 + kk), L.emu_acc_frag(dH3[kk >> 1], kk & 1), c)
        dH2.append(c)
    W3 = net[4].weight.detach().numpy()[..., 0]
    ref2 = W3.T @ np.concatenate([acc_to_mat(d) for d in dH3], 0)
    np.testing.assert_allclose(np.concatenate([acc_to_mat(d) for d in dH2], 0), ref2, rtol=1e-6, atol=1e-6)
    dH1 = []
    for mt in range(2):
        c = np.zeros((64, 16))
        for kk in range(8):
            c = L.emu_mfma(L.emu_frag(vals, fo["w2t"] + mt * 8 + kk), L.emu_acc_frag(dH2[kk >> 1], kk & 1), c)
        dH1.append(c)
    W2 = net[2].weight.detach().numpy()[..., 0]
    ref1 = W2.T @ ref2
    np.testing.assert_allclose(np.concatenate([acc_to_mat(d) for d in dH1], 0), ref1, rtol=1e-6, atol=1e-6)
    c = np.zeros((64, 16))
    for kk in range(4):
        c = L.emu_mfma(L.emu_frag(vals, fo["w1ft"] + kk), L.emu_acc_frag(dH1[kk >> 1], kk & 1), c)
    W1 = net[0].weight.detach().numpy()[..., 0]
    np.testing.assert_allclose(acc_to_mat(c)[:6], W1.T @ ref1, rtol=1e-6, atol=1e-6)


def test_emulated_transposed_orientation():
    """Z = H1^T W2^T with H1 (accumulator) as the A operand and ew2 as B fragments."""
    ctrl, cbf, fp, offs, src = _setup()
    pk = L.ctrl_packer(offs)
    vals = _vals(pk, src, fp.numel)
    fo = pk.offsets()
    rng = np.random.default_rng(2)
    H1 = rng.normal(size=(64, 32))     # 64 features x 32 edges (standard orientation)
    acc = [np.zeros((64, 16)) for _ in range(2)]
    for t in range(2):
        for l in range(64):
            r, h = l & 31, l >> 5
            for reg in range(16):
                acc[t][l, reg] = H1[32 * t + L.acc_row(reg, h), r]
    W2 = ctrl.controller_centr_net[2].weight.detach().numpy()[..., 0]   # (128, 64)
    for nt in range(4):
        c = np.zeros((64, 16))
        for kk in range(4):
            # A = accumulator regs (Z = X^T B), B = packed ew2 fragment for column tile nt
            c = L.emu_mfma(L.emu_acc_frag(acc[kk >> 1], kk & 1), L.emu_frag(vals, fo["ew2"] + nt * 4 + kk), c)
        Z = acc_to_mat(c)                  # rows = edges, cols = features 32nt..
        np.testing.assert_allclose(Z, (W2 @ H1).T[:, 32 * nt:32 * nt + 32], rtol=1e-6, atol=1e-6)


def test_emulated_node_w1_natural():
    ctrl, cbf, fp, offs, src = _setup()
    pk = L.ctrl_packer(offs)
    vals = _vals(pk, src, fp.numel)
    fo = pk.offsets()
    rng = np.random.default_rng(3)
    P = rng.normal(size=(132, 32))          # node input: pooled 128 + state 4, 32 agents
    Pb = np.zeros((144, 32))
    Pb[:132] = P
    Pb[132] = 1.0
    out = []
    for mt in range(2):
        c = np.zeros((64, 16))
        for kk in range(9):
            b = np.zeros((64, 8))
            for l in range(64):
                r, h = l & 31, l >> 5
                b[l] = Pb[16 * kk + 8 * h: 16 * kk + 8 * h + 8, r]
            c = L.emu_mfma(L.emu_frag(vals, fo["nw1f"] + mt * 9 + kk), b, c)
        out.append(acc_to_mat(c))
    lin = ctrl.controller_dec_net[0]
    ref = lin.weight.detach().numpy() @ P + lin.bias.detach().numpy()[:, None]
    np.testing.assert_allclose(np.concatenate(out, 0), ref, rtol=1e-5, atol=1e-6)


def _rm_images(fp, offs, src):
    pk = L.ctrl_node_rm(offs)
    vals = src[L.resolve(pk.index(), fp.numel)]
    imgs = {}
    for im in pk.images:
        imgs[im.name] = vals[im.offset: im.offset + im.rows * im.stride].reshape(im.rows, im.stride)
    return imgs


def test_emulated_rowmajor_node_forward_backward():
    ctrl, cbf, fp, offs, src = _setup()
    im = _rm_images(fp, offs, src)
    rng = np.random.default_rng(5)
    Pin = np.zeros((160, 32))
    Pin[:132] = rng.normal(size=(132, 32))
    Pin[132] = 1.0
    # forward Y1 = W1f P (natural B from data)
    Y1 = []
    for mt in range(2):
        c = np.zeros((64, 16))
        for kk in range(9):
            b = np.stack([Pin[16 * kk + 8 * (l >> 5): 16 * kk + 8 * (l >> 5) + 8, l & 31] for l in range(64)])
            c = L.emu_mfma(L.emu_wrm_nat(im["w1"], 32 * mt, kk), b, c)
        Y1.append(np.maximum(c, 0))
    net = ctrl.controller_dec_net
    W = [net[i].weight.detach().numpy().astype(np.float64) for i in (0, 2, 4, 6)]
    bb = [net[i].bias.detach().numpy().astype(np.float64) for i in (0, 2, 4, 6)]
    ref1 = np.maximum(W[0] @ Pin[:132] + bb[0][:, None], 0)
    np.testing.assert_allclose(np.concatenate([acc_to_mat(y) for y in Y1]), ref1, rtol=1e-5, atol=1e-6)
    # Y2 = W2 Y1 (accumulator B)
    Y2 = []
    for mt in range(4):
        c = bias_init(bb[1], mt)
        for kk in range(4):
            c = L.emu_mfma(L.emu_wrm_acc(im["w2"], 32 * mt, kk), L.emu_acc_frag(Y1[kk >> 1], kk & 1), c)
        Y2.append(c)
    ref2 = W[1] @ ref1 + bb[1][:, None]
    np.testing.assert_allclose(np.concatenate([acc_to_mat(y) for y in Y2]), ref2, rtol=1e-5, atol=1e-6)
    # backward: dY3 = W4^T dY4 (K=32 from a 32-row accumulator), dY1 = W2^T dY2, dP = W1f^T dY1
    dY4 = np.zeros((64, 16))
    for l in range(32):
        dY4[l, :4] = rng.normal(size=4)       # rows 0..3 live in lanes h=0, regs 0..3
    dY3 = []
    for mt in range(2):
        c = np.zeros((64, 16))
        for kk in range(2):
            c = L.emu_mfma(L.emu_wrmT_acc(im["w4"], 32 * mt, kk), L.emu_acc_frag(dY4, kk & 1), c)
        dY3.append(c)
    D4 = acc_to_mat(dY4)[:4]
    np.testing.assert_allclose(np.concatenate([acc_to_mat(y) for y in dY3]), W[3].T @ D4, rtol=1e-6, atol=1e-7)
    dY2 = [rng.normal(size=(64, 16)) for _ in range(4)]
    dY1 = []
    for mt in range(2):
        c = np.zeros((64, 16))
        for kk in range(8):
            c = L.emu_mfma(L.emu_wrmT_acc(im["w2"], 32 * mt, kk), L.emu_acc_frag(dY2[kk >> 1], kk & 1), c)
        dY1.append(c)
    D2 = np.concatenate([acc_to_mat(d) for d in dY2])
    np.testing.assert_allclose(np.concatenate([acc_to_mat(y) for y in dY1]), W[1].T @ D2, rtol=1e-6, atol=1e-6)
    dP = []
    for mt in range(5):
        c = np.zeros((64, 16))
        for kk in range(4):
            c = L.emu_mfma(L.emu_wrmT_acc(im["w1"], 32 * mt, kk), L.emu_acc_frag(dY1[kk >> 1], kk & 1), c)
        dP.append(c)
    D1 = np.concatenate([acc_to_mat(d) for d in dY1])
    got = np.concatenate([acc_to_mat(d) for d in dP])
    np.testing.assert_allclose(got[:132], W[0].T @ D1, rtol=1e-6, atol=1e-6)
    # natural transposed reader: A = W2^T with natural-k B
    Bn = rng.normal(size=(128, 32))
    for mt in range(2):
        c = np.zeros((64, 16))
        for kk in range(8):
            b = np.stack([Bn[16 * kk + 8 * (l >> 5): 16 * kk + 8 * (l >> 5) + 8, l & 31] for l in range(64)])
            c = L.emu_mfma(L.emu_wrmT_nat(im["w2"], 32 * mt, kk), b, c)
        np.testing.assert_allclose(acc_to_mat(c), (W[1].T @ Bn)[32 * mt:32 * mt + 32], rtol=1e-6, atol=1e-6)


def test_cbf16_permuted_image_chain():
    """16x16x32 data path (csrc/cbf16.h) emulated lane by lane: A = W from the column-permuted
    image (one 16-byte read at col 32s + 8g), A = W^T through the transposed-read addressing, and
    B from packed accumulator tiles (pk4_fr) reproduce W @ X and W^T @ Y."""
    rng = np.random.default_rng(0)
    W = rng.standard_normal((128, 64))
    X = rng.standard_normal((64, 16))
    Y = rng.standard_normal((128, 16))
    img = np.array([[W[r, L.perm32_logical(c)] for c in range(64)] for r in range(128)])

    def tiles(M):     # C-layout tiles: tile t, lane (n, g), reg i = M[16t + 4g + i][n]
        return [[[M[16 * t + 4 * (l >> 4) + i, l & 15] for i in range(4)] for l in range(64)]
                for t in range(M.shape[0] // 16)]

    def bfrag(T, s):  # pk4_fr(T[2s], T[2s + 1])
        return np.array([T[2 * s][l] + T[2 * s + 1][l] for l in range(64)])

    TX, TY = tiles(X), tiles(Y)
    for mt in range(8):
        D = np.zeros((16, 16))
        for s in range(2):
            a = np.array([img[16 * mt + (l & 15), 32 * s + 8 * (l >> 4): 32 * s + 8 * (l >> 4) + 8] for l in range(64)])
            D += L.emu_mfma16(a, bfrag(TX, s))
        np.testing.assert_allclose(D, (W @ X)[16 * mt:16 * mt + 16], rtol=1e-12, atol=1e-12)
    for mt in range(4):                     # W^T: rows = logical columns 16mt.., K over W's rows
        m0 = 16 * mt
        D = np.zeros((16, 16))
        for s in range(4):
            a = np.zeros((64, 8))
            for l in range(64):
                n, g = l & 15, l >> 4
                p, t = n >> 2, n & 3
                col = 32 * (m0 >> 5) + 4 * ((m0 >> 4) & 1) + 8 * p + t
                assert L.perm32_logical(col) == m0 + n
                for j in range(8):
                    a[l, j] = img[32 * s + 4 * g + (j & 3) + 16 * (j >> 2), col]
            D += L.emu_mfma16(a, bfrag(TY, s))
        np.testing.assert_allclose(D, (W.T @ Y)[m0:m0 + 16], rtol=1e-12, atol=1e-12)
