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


def cbf_packer(fp_offsets: Dict[str, int]) -> Packer:
    """Fragments used by csrc/cbf.hip. Offsets are flat indices of the CBF parameters."""
    W1, b1 = fp_offsets["cbf_net.0.weight"], fp_offsets["cbf_net.0.bias"]
    W2 = fp_offsets["cbf_net.2.weight"]
    W3 = fp_offsets["cbf_net.4.weight"]

    def w1f(o, k):           # (64 x 16): [W1 | b1 | 0] hi, [W1 | 0] lo
        if o >= 64:
            return ZERO
        if k < 6:
            return W1 + o * 6 + k
        if k == 6:
            return b1 + o
        if 8 <= k < 14:
            return W1 + o * 6 + (k - 8)
        return ZERO

    def w1ft(f, o):          # (32 x 64): W1^T restricted to the 6 input features
        if f < 6 and o < 64:
            return W1 + o * 6 + f
        return ZERO

    p = Packer()
    p.add("w1f", w1f, 2, 1, "nat")
    p.add("w2", _mat(W2, 128, 64), 4, 4, "acc")
    p.add("w3", _mat(W3, 64, 128), 2, 8, "acc")
    p.add("w3t", _matT(W3, 64, 128), 4, 4, "acc")
    p.add("w2t", _matT(W2, 128, 64), 2, 8, "acc")
    p.add("w1ft", w1ft, 1, 4, "acc")
    return p


def ctrl_packer(fp_offsets: Dict[str, int]) -> Packer:
    """Fragments used by csrc/ctrl.hip."""
    eW1, eb1 = fp_offsets["controller_centr_net.0.weight"], fp_offsets["controller_centr_net.0.bias"]
    eW2 = fp_offsets["controller_centr_net.2.weight"]
    nW1, nb1 = fp_offsets["controller_dec_net.0.weight"], fp_offsets["controller_dec_net.0.bias"]
    nW2 = fp_offsets["controller_dec_net.2.weight"]
    nW3 = fp_offsets["controller_dec_net.4.weight"]
    nW4 = fp_offsets["controller_dec_net.6.weight"]

    def ew1f(o, k):          # (64 x 16): [W1(5) | b1 | 0 0] hi, [W1(:4) | 0...] lo
        if o >= 64:
            return ZERO
        if k < 5:
            return eW1 + o * 5 + k
        if k == 5:
            return eb1 + o
        if 8 <= k < 12:
            return eW1 + o * 5 + (k - 8)
        return ZERO

    def ew1ft(f, o):         # (32 x 64): W1^T for the 4 relative-state features
        if f < 4 and o < 64:
            return eW1 + o * 5 + f
        return ZERO

    def ew2tn(m, f):         # (64 x 128) = W2^T, paired with a natural-k B (dZ from LDS)
        if m < 64 and f < 128:
            return eW2 + f * 64 + m
        return ZERO

    def nw1f(o, k):          # (64 x 144): [pooled 128 | state hi 4 | b1 | 0 0 0 | state lo 4 | 0 x4]
        if o >= 64:
            return ZERO
        if k < 132:
            return nW1 + o * 132 + k
        if k == 132:
            return nb1 + o
        if 136 <= k < 140:
            return nW1 + o * 132 + 128 + (k - 136)
        return ZERO

    def nw1ft(k, o):         # (160 x 64) = nw1f^T restricted to the hi/pooled rows
        if o < 64 and k < 132:
            return nW1 + o * 132 + k
        return ZERO

    p = Packer()
    p.add("ew1f", ew1f, 2, 1, "nat")
    p.add("ew2", _mat(eW2, 128, 64), 4, 4, "acc")          # also the B frags of Z = H1^T W2^T
    p.add("ew2tn", ew2tn, 2, 8, "nat")
    p.add("ew1ft", ew1ft, 1, 4, "acc")
    p.add("nw1f", nw1f, 2, 9, "nat")
    p.add("nw2", _mat(nW2, 128, 64), 4, 4, "acc")
    p.add("nw3", _mat(nW3, 64, 128), 2, 8, "acc")
    p.add("nw4", _mat(nW4, 4, 64), 1, 4, "acc")
    p.add("nw4t", _matT(nW4, 4, 64), 2, 2, "acc")
    p.add("nw3t", _matT(nW3, 64, 128), 4, 4, "acc")
    p.add("nw2t", _matT(nW2, 128, 64), 2, 8, "acc")
    p.add("nw1ft", nw1ft, 5, 4, "acc")
    return p


# fp32 side-vectors (biases added in accumulator init, last-layer weights, ...)
def cbf_vec_index(fp_offsets) -> Tuple[np.ndarray, Dict[str, int]]:
    parts = [("b2", fp_offsets["cbf_net.2.bias"], 128), ("b3", fp_offsets["cbf_net.4.bias"], 64),
             ("w4", fp_offsets["cbf_net.6.weight"], 64), ("b4", fp_offsets["cbf_net.6.bias"], 1)]
    return _vec(parts)


def ctrl_vec_index(fp_offsets) -> Tuple[np.ndarray, Dict[str, int]]:
    parts = [("eb2", fp_offsets["controller_centr_net.2.bias"], 128),
             ("nb2", fp_offsets["controller_dec_net.2.bias"], 128),
             ("nb3", fp_offsets["controller_dec_net.4.bias"], 64),
             ("nb4", fp_offsets["controller_dec_net.6.bias"], 4, 32)]
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
