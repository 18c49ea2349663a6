"""MFMA fragment layouts for ``v_mfma_f32_32x32x16_bf16`` and weight packing.

gfx950 lane maps (cdna_hip_programming.md section 3), lane ``l``, ``r = l & 31``, ``h = l >> 5``:

* A fragment (32x16): element j = ``A[r][k(h, j)]``
* B fragment (16x32): element j = ``B[k(h, j)][r]``
* C/D (32x32), 16 regs: ``D[(reg & 3) + 8*(reg >> 2) + 4*h][r]``

``k(h, j)`` is ``8h + j`` ("natural") when the operand is built from data, and
``kacc(s, h, j) = 16s + 8(j >> 2) + 4h + (j & 3)`` when the operand is the bf16 conversion of
accumulator registers ``8s..8s+7`` of a previous 32x32 result (the chain trick: the next
layer consumes the previous layer's accumulator with no lane movement). The *other*
operand must then use the same k permutation, which is baked into the packed weights here.

A weight fragment is stored as 64 lanes x 8 bf16 = 1 KiB, lane-contiguous, so the kernels
read it with one conflict-free ``ds_read_b128`` per lane from an LDS copy.

Packing is a gather ``packed = src[index]`` from ``src = cat(flat_params, [0, 1])``; the
index tensors are built once here (host) and reused every step.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Tuple

import numpy as np

LANES = 64
FRAG = 8          # bf16 elements per lane per fragment


def kacc(s: int, h: int, j: int) -> int:
    return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)


def knat(kk: int, h: int, j: int) -> int:
    return 16 * kk + 8 * h + j


def acc_row(reg: int, h: int) -> int:
    return (reg & 3) + 8 * (reg >> 2) + 4 * h


# A "virtual matrix" maps (row, col) -> index into src (flat params), or ZERO / ONE.
ZERO = -1
ONE = -2


def pack_frags(vm: Callable[[int, int], int], mtiles: int, ksteps: int, kind: str) -> np.ndarray:
    """Index array (mtiles*ksteps*64*8,) for fragments of virtual matrix ``vm``.

    kind = "acc": element j of lane (r,h) at k-step kk=(2t+s) is vm(32mt+r, 32t+kacc(s,h,j))
    kind = "nat": ... vm(32mt+r, 16kk+8h+j)
    """
    out = np.empty((mtiles, ksteps, LANES, FRAG), dtype=np.int64)
    for mt in range(mtiles):
        for kk in range(ksteps):
            t, s = kk >> 1, kk & 1
            for l in range(LANES):
                r, h = l & 31, l >> 5
                for j in range(FRAG):
                    col = 32 * t + kacc(s, h, j) if kind == "acc" else knat(kk, h, j)
                    out[mt, kk, l, j] = vm(32 * mt + r, col)
    return out.reshape(-1)


@dataclass
class Block:
    name: str
    index: np.ndarray      # into src
    frag_offset: int = 0   # in fragments (1 KiB units) within the packed buffer


class Packer:
    """Collects fragment blocks for one kernel family into a single packed buffer."""

    def __init__(self):
        self.blocks: List[Block] = []
        self.nfrag = 0

    def add(self, name, vm, mtiles, ksteps, kind):
        idx = pack_frags(vm, mtiles, ksteps, kind)
        self.blocks.append(Block(name, idx, self.nfrag))
        self.nfrag += mtiles * ksteps
        return self

    def index(self) -> np.ndarray:
        return np.concatenate([b.index for b in self.blocks])

    def offsets(self) -> Dict[str, int]:
        return {b.name: b.frag_offset for b in self.blocks}


def _mat(off: int, rows: int, cols: int):
    """vm for a row-major (rows, cols) parameter starting at flat offset ``off``."""
    def f(r, c):
        if r < rows and c < cols:
            return off + r * cols + c
        return ZERO
    return f


def _matT(off: int, rows: int, cols: int):
    """vm for the transpose of a row-major (rows, cols) parameter."""
    def f(r, c):
        if c < rows and r < cols:
            return off + c * cols + r
        return ZERO
    return f


def cbf_w1_slot(k: int, dim: int = 2):
    """Layer-1 K slot k (0..15) of the CBF edge fragment -> ('w', feature column) | ('b',) | None.

    Edge features (2D + 2 columns): s_i - s_j (0..2D-1), eye (2D), |dp|_eps - r (2D+1); every
    fp32 input is split into a bf16 hi part (lanes h = 0, K 0..7) and its residual (lanes h = 1,
    K 8..15). D = 2: hi [rel 4, eye, dist, 1, 0] / lo [rel 4, eye(0), dist, 0, 0];
    D = 3: hi [rel 6, dist, 1] / lo [rel 6, dist, eye] (eye is exact in bf16)."""
    F = 2 * dim + 2
    if dim == 2:
        if k < F:
            return ("w", k)
        if k == F:
            return ("b",)
        if 8 <= k < 8 + F:
            return ("w", k - 8)
        return None
    if k < 2 * dim:
        return ("w", k)
    if k == 2 * dim:
        return ("w", F - 1)
    if k == 2 * dim + 1:
        return ("b",)
    if 8 <= k < 8 + 2 * dim:
        return ("w", k - 8)
    if k == 8 + 2 * dim:
        return ("w", F - 1)
    if k == 9 + 2 * dim:
        return ("w", 2 * dim)
    return None


def cbf_packer(fp_offsets: Dict[str, int], dim: int = 2) -> Packer:
    """Fragments used by csrc/cbf.hip. Offsets are flat indices of the CBF parameters."""
    W1, b1 = fp_offsets["cbf_net.0.weight"], fp_offsets["cbf_net.0.bias"]
    W2 = fp_offsets["cbf_net.2.weight"]
    W3 = fp_offsets["cbf_net.4.weight"]
    F = 2 * dim + 2

    def w1f(o, k):           # (64 x 16): hi / lo slots of the edge features + bias
        sl = cbf_w1_slot(k, dim) if o < 64 else None
        if sl is None:
            return ZERO
        return b1 + o if sl[0] == "b" else W1 + o * F + sl[1]

    def w1ft(f, o):          # (32 x 64): W1^T, rows = feature columns
        if f < F and o < 64:
            return W1 + o * F + f
        return ZERO

    p = Packer()
    p.add("w1f", w1f, 2, 1, "nat")
    p.add("w2", _mat(W2, 128, 64), 4, 4, "acc")
    p.add("w3", _mat(W3, 64, 128), 2, 8, "acc")
    p.add("w3t", _matT(W3, 64, 128), 4, 4, "acc")
    p.add("w2t", _matT(W2, 128, 64), 2, 8, "acc")
    p.add("w1ft", w1ft, 1, 4, "acc")
    return p


def ctrl_edge_slot(k: int, dim: int = 2):
    """Controller edge layer-1 K slot -> ('w', col) | ('b',) | None. Features (2D + 1):
    s_i - s_j (0..2D-1), eye (2D). hi [rel, eye, 1], lo [rel]."""
    E = 2 * dim + 1
    if k < E:
        return ("w", k)
    if k == E:
        return ("b",)
    if 8 <= k < 8 + 2 * dim:
        return ("w", k - 8)
    return None


def ctrl_node_slot(k: int, dim: int = 2):
    """Node layer-1 K slot (0..143) -> ('w', col) | ('b',) | None. Inputs (128 + 2D): pooled
    (0..127), [p - g, v] (128..128+2D-1); slots 128.. = state hi, 1 (bias); 136.. = state lo."""
    n_in = 128 + 2 * dim
    if k < n_in:
        return ("w", k)
    if k == n_in:
        return ("b",)
    if 136 <= k < 136 + 2 * dim:
        return ("w", 128 + (k - 136))
    return None


def ctrl_packer(fp_offsets: Dict[str, int], dim: int = 2) -> Packer:
    """Fragments used by csrc/ctrl.hip."""
    eW1, eb1 = fp_offsets["controller_centr_net.0.weight"], fp_offsets["controller_centr_net.0.bias"]
    eW2 = fp_offsets["controller_centr_net.2.weight"]
    nW1, nb1 = fp_offsets["controller_dec_net.0.weight"], fp_offsets["controller_dec_net.0.bias"]
    nW2 = fp_offsets["controller_dec_net.2.weight"]
    nW3 = fp_offsets["controller_dec_net.4.weight"]
    nW4 = fp_offsets["controller_dec_net.6.weight"]
    E = 2 * dim + 1
    n_in = 128 + 2 * dim
    SD = 2 * dim

    def ew1f(o, k):          # (64 x 16): [W1 | b1] hi, [W1(rel)] lo
        sl = ctrl_edge_slot(k, dim) if o < 64 else None
        if sl is None:
            return ZERO
        return eb1 + o if sl[0] == "b" else eW1 + o * E + sl[1]

    def ew1ft(f, o):         # (32 x 64): W1^T for the 2D relative-state features
        if f < SD and o < 64:
            return eW1 + o * E + f
        return ZERO

    def ew2tn(m, f):         # (64 x 128) = W2^T, paired with a natural-k B (dZ from LDS)
        if m < 64 and f < 128:
            return eW2 + f * 64 + m
        return ZERO

    def nw1f(o, k):          # (64 x 144): [pooled 128 | state hi 2D | b1 | .. | state lo 2D | ..]
        sl = ctrl_node_slot(k, dim) if o < 64 else None
        if sl is None:
            return ZERO
        return nb1 + o if sl[0] == "b" else nW1 + o * n_in + sl[1]

    def nw1ft(k, o):         # (160 x 64) = nw1f^T restricted to the hi/pooled rows
        if o < 64 and k < n_in:
            return nW1 + o * n_in + k
        return ZERO

    p = Packer()
    p.add("ew1f", ew1f, 2, 1, "nat")
    p.add("ew2", _mat(eW2, 128, 64), 4, 4, "acc")          # also the B frags of Z = H1^T W2^T
    p.add("ew2tn", ew2tn, 2, 8, "nat")
    p.add("ew1ft", ew1ft, 1, 4, "acc")
    p.add("nw1f", nw1f, 2, 9, "nat")
    p.add("nw2", _mat(nW2, 128, 64), 4, 4, "acc")
    p.add("nw3", _mat(nW3, 64, 128), 2, 8, "acc")
    p.add("nw4", _mat(nW4, SD, 64), 1, 4, "acc")
    p.add("nw4t", _matT(nW4, SD, 64), 2, 2, "acc")
    p.add("nw3t", _matT(nW3, 64, 128), 4, 4, "acc")
    p.add("nw2t", _matT(nW2, 128, 64), 2, 8, "acc")
    p.add("nw1ft", nw1ft, 5, 4, "acc")
    return p


# fp32 side-vectors (biases added in accumulator init, last-layer weights, ...)
def cbf_vec_index(fp_offsets) -> Tuple[np.ndarray, Dict[str, int]]:
    parts = [("b2", fp_offsets["cbf_net.2.bias"], 128), ("b3", fp_offsets["cbf_net.4.bias"], 64),
             ("w4", fp_offsets["cbf_net.6.weight"], 64), ("b4", fp_offsets["cbf_net.6.bias"], 1)]
    return _vec(parts)


def ctrl_vec_index(fp_offsets, dim: int = 2) -> Tuple[np.ndarray, Dict[str, int]]:
    parts = [("eb2", fp_offsets["controller_centr_net.2.bias"], 128),
             ("nb2", fp_offsets["controller_dec_net.2.bias"], 128),
             ("nb3", fp_offsets["controller_dec_net.4.bias"], 64),
             ("nb4", fp_offsets["controller_dec_net.6.bias"], 2 * dim, 32)]
    return _vec(parts)


def _vec(parts):
    idx, offs, o = [], {}, 0
    for part in parts:
        name, off, n = part[:3]
        width = part[3] if len(part) > 3 else n
        offs[name] = o
        idx.extend(range(off, off + n))
        idx.extend([ZERO] * (width - n))
        o += width
        pad = (-o) % 4
        idx.extend([ZERO] * pad)
        o += pad
    return np.asarray(idx, dtype=np.int64), offs


def resolve(index: np.ndarray, nflat: int) -> np.ndarray:
    """Map ZERO/ONE sentinels to the two constant slots appended after the flat params."""
    out = index.copy()
    out[out == ZERO] = nflat
    out[out == ONE] = nflat + 1
    return out


# ------------------------------------------------------------------ lane-level emulator
def emu_mfma(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Emulate v_mfma_f32_32x32x16 on per-lane fragments: a,b (64,8), c (64,16) -> (64,16)."""
    A = np.zeros((32, 16))
    B = np.zeros((16, 32))
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(8):
            A[r, 8 * h + j] = a[l, j]
            B[8 * h + j, r] = b[l, j]
    D = A @ B
    out = c.astype(np.float64).copy()
    for l in range(64):
        r, h = l & 31, l >> 5
        for reg in range(16):
            out[l, reg] += D[acc_row(reg, h), r]
    return out


def emu_acc_frag(c: np.ndarray, s: int) -> np.ndarray:
    """Accumulator regs 8s..8s+7 as an operand fragment (64,8)."""
    return c[:, 8 * s: 8 * s + 8].copy()


def emu_frag(packed_vals: np.ndarray, frag: int) -> np.ndarray:
    return packed_vals[frag * 512:(frag + 1) * 512].reshape(64, 8)


# ------------------------------------------------------------------ row-major LDS images
# One padded row-major bf16 copy per weight matrix; the kernels read W fragments with
# ds_read_b64/b128 (wrm_*) and W^T fragments with ds_read_b64_tr_b16 (wrmT_*), so the
# forward and backward chains share one LDS image (csrc/common.h).
@dataclass
class RMImage:
    name: str
    offset: int     # elements
    rows: int
    stride: int


class RMPacker:
    def __init__(self):
        self.images: List[RMImage] = []
        self.parts: List[np.ndarray] = []
        self.size = 0

    def add(self, name, vm, rows, cols, stride):
        assert stride % 4 == 0 and stride >= cols and (rows * stride) % 8 == 0
        idx = np.full((rows, stride), ZERO, dtype=np.int64)
        for r in range(rows):
            for c in range(cols):
                idx[r, c] = vm(r, c)
        self.images.append(RMImage(name, self.size, rows, stride))
        self.parts.append(idx.reshape(-1))
        self.size += rows * stride
        return self

    def index(self):
        return np.concatenate(self.parts)

    def offsets(self):
        return {im.name: im.offset for im in self.images}


NODE_STRIDES = {"w1": 168, "w2": 68, "w3": 132, "w4": 68}


def ctrl_node_rm(fp_offsets, dim: int = 2) -> RMPacker:
    """Row-major node-MLP images for the controller backward kernel (csrc/ctrl.hip)."""
    nW1, nb1 = fp_offsets["controller_dec_net.0.weight"], fp_offsets["controller_dec_net.0.bias"]
    nW2 = fp_offsets["controller_dec_net.2.weight"]
    nW3 = fp_offsets["controller_dec_net.4.weight"]
    nW4 = fp_offsets["controller_dec_net.6.weight"]
    n_in = 128 + 2 * dim

    def w1f(o, k):   # same virtual matrix as ctrl_packer's nw1f, 160 columns (144.. zero)
        sl = ctrl_node_slot(k, dim)
        if sl is None:
            return ZERO
        return nb1 + o if sl[0] == "b" else nW1 + o * n_in + sl[1]

    p = RMPacker()
    p.add("w1", w1f, 64, 160, NODE_STRIDES["w1"])
    p.add("w2", _mat(nW2, 128, 64), 128, 64, NODE_STRIDES["w2"])
    p.add("w3", _mat(nW3, 64, 128), 64, 128, NODE_STRIDES["w3"])
    p.add("w4", _mat(nW4, 2 * dim, 64), 32, 64, NODE_STRIDES["w4"])
    return p


def emu_tr_pair(img, rb1, rb2, c0):
    """ds_read_b64_tr_b16 pair as used by tr_pair(): rb1/rb2 are arrays over h (2,)."""
    out = np.zeros((64, 8))
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(4):
            out[l, j] = img[rb1[h] + j, c0 + r]
            out[l, 4 + j] = img[rb2[h] + j, c0 + r]
    return out


def emu_wrm_nat(img, m0, kk):
    out = np.zeros((64, 8))
    for l in range(64):
        r, h = l & 31, l >> 5
        out[l] = img[m0 + r, 16 * kk + 8 * h: 16 * kk + 8 * h + 8]
    return out


def emu_wrm_acc(img, m0, kk):
    out = np.zeros((64, 8))
    for l in range(64):
        r, h = l & 31, l >> 5
        base = 16 * kk + 4 * h
        out[l, :4] = img[m0 + r, base:base + 4]
        out[l, 4:] = img[m0 + r, base + 8:base + 12]
    return out


def emu_wrmT_acc(img, m0, kk):
    rb = [16 * kk + 4 * h for h in range(2)]
    return emu_tr_pair(img, rb, [x + 8 for x in rb], m0)


def emu_wrmT_nat(img, m0, kk):
    rb = [16 * kk + 8 * h for h in range(2)]
    return emu_tr_pair(img, rb, [x + 4 for x in rb], m0)


# ------------------------------------------------------------------ gradient slab -> flat maps
def _pairs_rowmajor(base_slab, ncols_slab, param_off, rows, cols):
    src, dst = [], []
    for r in range(rows):
        for c in range(cols):
            src.append(base_slab + r * ncols_slab + c)
            dst.append(param_off + r * cols + c)
    return src, dst


def cbf_grad_map(fp_offsets, dim: int = 2):
    """(src in the reduced CBF slab, dst in the flat grad) pairs; src may repeat dst (hi/lo)."""
    W1, b1 = fp_offsets["cbf_net.0.weight"], fp_offsets["cbf_net.0.bias"]
    W2, b2 = fp_offsets["cbf_net.2.weight"], fp_offsets["cbf_net.2.bias"]
    W3, b3 = fp_offsets["cbf_net.4.weight"], fp_offsets["cbf_net.4.bias"]
    W4, b4 = fp_offsets["cbf_net.6.weight"], fp_offsets["cbf_net.6.bias"]
    F = 2 * dim + 2
    S, D = [], []
    for s_, d_ in (_pairs_rowmajor(0, 128, W3, 64, 128), _pairs_rowmajor(8256, 64, W2, 128, 64)):
        S += s_; D += d_
    S += [8192 + m for m in range(64)]; D += [b3 + m for m in range(64)]
    S += [16448 + m for m in range(128)]; D += [b2 + m for m in range(128)]
    for o in range(64):
        for k in range(16):
            sl = cbf_w1_slot(k, dim)
            if sl is None:
                continue
            S.append(16576 + o * 32 + k)
            D.append(b1 + o if sl[0] == "b" else W1 + o * F + sl[1])
    S += [18624 + n for n in range(64)]; D += [W4 + n for n in range(64)]
    S.append(18688); D.append(b4)
    return np.asarray(S, np.int64), np.asarray(D, np.int64)


def ctrl_node_grad_map(fp_offsets, dim: int = 2):
    nW1, nb1 = fp_offsets["controller_dec_net.0.weight"], fp_offsets["controller_dec_net.0.bias"]
    nW2, nb2 = fp_offsets["controller_dec_net.2.weight"], fp_offsets["controller_dec_net.2.bias"]
    nW3, nb3 = fp_offsets["controller_dec_net.4.weight"], fp_offsets["controller_dec_net.4.bias"]
    nW4, nb4 = fp_offsets["controller_dec_net.6.weight"], fp_offsets["controller_dec_net.6.bias"]
    n_in = 128 + 2 * dim
    S, D = [], []
    for o in range(64):
        for k in range(160):
            sl = ctrl_node_slot(k, dim)
            if sl is None:
                continue
            S.append(o * 160 + k)
            D.append(nb1 + o if sl[0] == "b" else nW1 + o * n_in + sl[1])
    for s_, d_ in (_pairs_rowmajor(10240, 64, nW2, 128, 64), _pairs_rowmajor(18560, 128, nW3, 64, 128),
                   _pairs_rowmajor(26816, 64, nW4, 2 * dim, 64)):
        S += s_; D += d_
    S += [18432 + m for m in range(128)]; D += [nb2 + m for m in range(128)]
    S += [26752 + m for m in range(64)]; D += [nb3 + m for m in range(64)]
    S += [28864 + m for m in range(2 * dim)]; D += [nb4 + m for m in range(2 * dim)]
    return np.asarray(S, np.int64), np.asarray(D, np.int64)


def ctrl_node16_grad_map(fp_offsets, dim: int = 2):
    """Slab -> flat grad pairs of the 16x16x32 node backward (csrc/node16.h, tile-major slab):
    a 16x16 tile (M, N) is 64 lanes x 4 floats, lane l = (n = l & 15, g = l >> 4), float q ->
    row 16M + 4g + q, column 16N + n. Wave w owns dW2 tiles (w, u < 4), dW3 tiles (w & 3, 4(w >> 2) + u),
    dW1f slots v < 5 -> tile (w & 3, (w >> 2) + 2v) for tile columns < 9, dW4 tile (0, w) for w < 4;
    then the bias rows b2 (128), b3 (64), b4 (16)."""
    nW1, nb1 = fp_offsets["controller_dec_net.0.weight"], fp_offsets["controller_dec_net.0.bias"]
    nW2, nb2 = fp_offsets["controller_dec_net.2.weight"], fp_offsets["controller_dec_net.2.bias"]
    nW3, nb3 = fp_offsets["controller_dec_net.4.weight"], fp_offsets["controller_dec_net.4.bias"]
    nW4, nb4 = fp_offsets["controller_dec_net.6.weight"], fp_offsets["controller_dec_net.6.bias"]
    n_in = 128 + 2 * dim
    S, D = [], []

    def tile(base, M, Nt, dst):
        for lane in range(64):
            n, g = lane & 15, lane >> 4
            for q in range(4):
                d = dst(16 * M + 4 * g + q, 16 * Nt + n)
                if d is not None:
                    S.append(base + lane * 4 + q)
                    D.append(d)

    for w in range(8):
        for u in range(4):
            tile((w * 4 + u) * 256, w, u, lambda r, c: nW2 + r * 64 + c)
            tile((32 + w * 4 + u) * 256, w & 3, 4 * (w >> 2) + u, lambda r, c: nW3 + r * 128 + c)
        for v in range(5):
            nt = (w >> 2) + 2 * v
            if nt < 9:
                def w1(r, c):
                    sl = ctrl_node_slot(c, dim)
                    if sl is None:
                        return None
                    return nb1 + r if sl[0] == "b" else nW1 + r * n_in + sl[1]
                tile((64 + w * 5 + v) * 256, w & 3, nt, w1)
        if w < 4:
            tile((104 + w) * 256, 0, w, lambda r, c: nW4 + r * 64 + c if r < 2 * dim else None)
    b2 = 108 * 256
    S += [b2 + m for m in range(128)]; D += [nb2 + m for m in range(128)]
    S += [b2 + 128 + m for m in range(64)]; D += [nb3 + m for m in range(64)]
    S += [b2 + 192 + m for m in range(2 * dim)]; D += [nb4 + m for m in range(2 * dim)]
    return np.asarray(S, np.int64), np.asarray(D, np.int64)


def ctrl_edge_grad_map(fp_offsets, dim: int = 2):
    eW1, eb1 = fp_offsets["controller_centr_net.0.weight"], fp_offsets["controller_centr_net.0.bias"]
    eW2, eb2 = fp_offsets["controller_centr_net.2.weight"], fp_offsets["controller_centr_net.2.bias"]
    E = 2 * dim + 1
    S, D = _pairs_rowmajor(0, 64, eW2, 128, 64)
    S += [8192 + m for m in range(128)]; D += [eb2 + m for m in range(128)]
    for o in range(64):
        for k in range(16):
            sl = ctrl_edge_slot(k, dim)
            if sl is None:
                continue
            S.append(8320 + o * 32 + k)
            D.append(eb1 + o if sl[0] == "b" else eW1 + o * E + sl[1])
    return np.asarray(S, np.int64), np.asarray(D, np.int64)


CBF_RM_STRIDES = {"w2": 68, "w3": 148}      # csrc/cbf.hip WS2 / WS3 (bank-conflict-aware)


def cbf_rm(fp_offsets, dim: int = 2) -> RMPacker:
    """Row-major CBF images for the backward kernel: W2 (128x64) and W3 (64x128)."""
    W2 = fp_offsets["cbf_net.2.weight"]
    W3 = fp_offsets["cbf_net.4.weight"]
    p = RMPacker()
    p.add("w2", _mat(W2, 128, 64), 128, 64, CBF_RM_STRIDES["w2"])
    p.add("w3", _mat(W3, 64, 128), 64, 128, CBF_RM_STRIDES["w3"])
    return p


# ------------------------------------------------------------------ 16x16x32 layouts (x3 CBF backward)
# v_mfma_f32_16x16x32_bf16, lane l: n = l & 15, g = l >> 4.
#   A fragment (16x32): element j = A[n][8g + j]     B fragment (32x16): element j = B[8g + j][n]
#   C/D (16x16), 4 regs: reg i = D[4g + i][n]
# The B operand of K-step s built from the packed accumulator tiles 2s, 2s+1 has
# k(8g + j) = 32s + kacc16(g, j): the weight operands use the same permutation.
CBF16_STRIDES = {"w2": 80, "w3": 144}     # csrc/cbf16.h S16_W2 / S16_W3 (conflict-free b128 / tr reads)


def kacc16(g: int, j: int) -> int:
    return 16 * (j >> 2) + 4 * g + (j & 3)


def acc_row16(i: int, g: int) -> int:
    return 4 * g + i


def perm32_logical(c: int) -> int:
    """Column c of a 16x16x32 row-major image -> logical weight column: within every 32-column
    block, physical 8g + j holds logical kacc16(g, j), so an A fragment is one 16-byte read."""
    b, q = divmod(c, 32)
    return 32 * b + kacc16(q >> 3, q & 7)


def cbf_rm16(fp_offsets, dim: int = 2) -> RMPacker:
    """Column-permuted row-major images of W2 (128x64) and W3 (64x128) for the 16x16x32 x3 CBF
    backward (csrc/cbf16.h): rows = output units; read as A = W (one ds_read_b128 per lane) and
    A = W^T (two ds_read_b64_tr_b16 per lane)."""
    W2 = fp_offsets["cbf_net.2.weight"]
    W3 = fp_offsets["cbf_net.4.weight"]
    m2, m3 = _mat(W2, 128, 64), _mat(W3, 64, 128)
    p = RMPacker()
    p.add("w2", lambda r, c: m2(r, perm32_logical(c)), 128, 64, CBF16_STRIDES["w2"])
    p.add("w3", lambda r, c: m3(r, perm32_logical(c)), 64, 128, CBF16_STRIDES["w3"])
    return p


NODE16_STRIDES = {"w1": 176, "w2": 80, "w3": 144, "w4": 80}    # csrc/node16.h N16_S1..S4 (bank model)


def node_rm16(fp_offsets, dim: int = 2) -> RMPacker:
    """Row-major node-MLP images for the 16x16x32 x3 node backward (csrc/node16.h): W1f (64 x 160,
    the layer-1 slots of ctrl_node_slot in natural order: its forward B operand is the pooled row),
    W2 (128x64), W3 (64x128) and W4 (16 x 64: rows >= 2D zero), the last three column-permuted
    (perm32_logical: their forward B operands are packed C-tile pairs). A = W is one 16-byte read
    per lane, A = W^T two ds_read_b64_tr_b16."""
    nW1, nb1 = fp_offsets["controller_dec_net.0.weight"], fp_offsets["controller_dec_net.0.bias"]
    nW2 = fp_offsets["controller_dec_net.2.weight"]
    nW3 = fp_offsets["controller_dec_net.4.weight"]
    nW4 = fp_offsets["controller_dec_net.6.weight"]
    n_in = 128 + 2 * dim

    def w1f(o, k):
        sl = ctrl_node_slot(k, dim)
        if sl is None:
            return ZERO
        return nb1 + o if sl[0] == "b" else nW1 + o * n_in + sl[1]

    m2, m3, m4 = _mat(nW2, 128, 64), _mat(nW3, 64, 128), _mat(nW4, 2 * dim, 64)
    p = RMPacker()
    p.add("w1", w1f, 64, 160, NODE16_STRIDES["w1"])
    p.add("w2", lambda r, c: m2(r, perm32_logical(c)), 128, 64, NODE16_STRIDES["w2"])
    p.add("w3", lambda r, c: m3(r, perm32_logical(c)), 64, 128, NODE16_STRIDES["w3"])
    p.add("w4", lambda r, c: m4(r, perm32_logical(c)) if r < 2 * dim else ZERO, 16, 64, NODE16_STRIDES["w4"])
    return p


def pack_frags16(vm: Callable[[int, int], int], mtiles: int, ksteps: int, kind: str) -> np.ndarray:
    """16x32 A fragments: element j of lane (n, g) at K-step s is vm(16mt + n, k) with
    k = 32s + 8g + j ("nat") or 32s + kacc16(g, j) ("acc"). 64 lanes x 8 per fragment."""
    out = np.empty((mtiles, ksteps, LANES, FRAG), dtype=np.int64)
    for mt in range(mtiles):
        for s in range(ksteps):
            for l in range(LANES):
                n, g = l & 15, l >> 4
                for j in range(FRAG):
                    k = 32 * s + (8 * g + j if kind == "nat" else kacc16(g, j))
                    out[mt, s, l, j] = vm(16 * mt + n, k)
    return out.reshape(-1)


def cbf_packer16(fp_offsets: Dict[str, int], dim: int = 2) -> Packer:
    """Layer-1 fragments of the 16x16x32 x3 CBF backward: w1f16 (64 x 32: the 16 edge-feature
    slots of cbf_w1_slot, slots 16..31 zero; 4 M-tiles) and w1ft16 (16 x 64: W1^T, rows = feature
    columns, accumulator-ordered k; 2 K-steps)."""
    W1, b1 = fp_offsets["cbf_net.0.weight"], fp_offsets["cbf_net.0.bias"]
    F = 2 * dim + 2

    def w1f(o, k):
        sl = cbf_w1_slot(k, dim) if (o < 64 and k < 16) else None
        if sl is None:
            return ZERO
        return b1 + o if sl[0] == "b" else W1 + o * F + sl[1]

    def w1ft(f, o):
        if f < F and o < 64:
            return W1 + o * F + f
        return ZERO

    p = Packer()
    p.blocks.append(Block("w1f16", pack_frags16(w1f, 4, 1, "nat"), 0))
    p.blocks.append(Block("w1ft16", pack_frags16(w1ft, 1, 2, "acc"), 4))
    p.nfrag = 6
    return p


def ctrl_edge_packer16(fp_offsets: Dict[str, int], dim: int = 2) -> Packer:
    """Fragments of the 16x16x32 x3 controller edge backward (csrc/ctrl16.h): ew1f16 (64 x 32:
    the 16 edge-feature slots of ctrl_edge_slot, 4 M-tiles), ew2tn16 (64 x 128 = W2^T with a
    natural-k B read from the dZ image rows: 4 M-tiles x 4 K-steps), ew1ft16 (16 x 64 = W1^T for the
    2D relative-state features, accumulator-ordered k: 2 K-steps)."""
    eW1, eb1 = fp_offsets["controller_centr_net.0.weight"], fp_offsets["controller_centr_net.0.bias"]
    eW2 = fp_offsets["controller_centr_net.2.weight"]
    E = 2 * dim + 1

    def ew1f(o, k):
        sl = ctrl_edge_slot(k, dim) if (o < 64 and k < 16) else None
        if sl is None:
            return ZERO
        return eb1 + o if sl[0] == "b" else eW1 + o * E + sl[1]

    def ew2tn(m, f):
        if m < 64 and f < 128:
            return eW2 + f * 64 + m
        return ZERO

    def ew1ft(f, o):
        if f < 2 * dim and o < 64:
            return eW1 + o * E + f
        return ZERO

    p = Packer()
    p.blocks.append(Block("ew1f16", pack_frags16(ew1f, 4, 1, "nat"), 0))
    p.blocks.append(Block("ew2tn16", pack_frags16(ew2tn, 4, 4, "nat"), 4))
    p.blocks.append(Block("ew1ft16", pack_frags16(ew1ft, 1, 2, "acc"), 20))
    p.nfrag = 22
    return p


def emu_mfma16(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """v_mfma_f32_16x16x32 on per-lane fragments a, b (64, 8) -> D (16, 16)."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for l in range(64):
        n, g = l & 15, l >> 4
        A[n, 8 * g:8 * g + 8] = a[l]
        B[8 * g:8 * g + 8, n] = b[l]
    return A @ B


# ------------------------------------------------------------------ operand precision (csrc/prec.h)
# "bf16" / "fp16": one 16-bit MFMA per product. "fp32": the fp32-accurate 3-term split (x3 kernels):
# every packed weight carries a bf16 residual plane; the pack gathers flag residual entries with
# LO_FLAG (pack_gather computes bf16(v - bf16(v)) for them).
PRECISIONS = ("bf16", "fp16", "fp32")
PREC_CODE = {"bf16": 0, "fp16": 1, "fp32": 2}
LO_FLAG = 1 << 30


def check_prec(prec: str) -> str:
    if prec not in PREC_CODE:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {prec!r}")
    return prec


def pooled_row(prec: str) -> int:
    """h16 elements per pooled / dL/dpooled row: [hi 128 | lo 128] for the x3 kernels."""
    return 256 if prec == "fp32" else 128


def x3_frags(index: np.ndarray) -> np.ndarray:
    """Resolved fragment index (nfrag * 512,) -> per fragment [hi 512 | lo 512] (x3 packing)."""
    a = np.asarray(index, dtype=np.int64).reshape(-1, LANES * FRAG)
    return np.stack([a, a | LO_FLAG], 1).reshape(-1)


def x3_planes(index: np.ndarray) -> np.ndarray:
    """Resolved row-major image index -> [hi plane | lo plane] (x3 packing)."""
    a = np.asarray(index, dtype=np.int64).reshape(-1)
    return np.concatenate([a, a | LO_FLAG])
