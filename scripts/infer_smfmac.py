"""Infer the v_smfmac_f32_32x32x32_bf16 operand layout from scripts/probe_smfmac.py dumps by
checking candidate maps against every trial (CPU)."""
import itertools
import sys

import numpy as np


def acc_row(reg, h):
    return (reg & 3) + 8 * (reg >> 2) + 4 * h


def kb(layout, h, j):
    """K index of dense B element j (0..15) of a lane in half h."""
    if layout == "B1":
        return 16 * h + j
    if layout == "B2":
        return 8 * h + j if j < 8 else 16 + 8 * h + (j - 8)
    if layout == "B3":
        return 4 * h + (j % 4) + 8 * (j // 4)
    raise ValueError


def ka_groups(layout, h):
    """K start of the 4 groups (of 4) of a lane's compressed A row in half h."""
    if layout == "A1":
        return [16 * h + 4 * g for g in range(4)]
    if layout == "A2":
        return [8 * h, 8 * h + 4, 16 + 8 * h, 16 + 8 * h + 4]
    if layout == "A3":
        return [4 * h + 8 * g for g in range(4)]
    raise ValueError


def dense_A(a, idx, la, ioff):
    A = np.zeros((32, 32), np.float64)
    for l in range(64):
        r, h = l & 31, l >> 5
        iv = int(np.uint32(idx[l]))
        off = ioff(h)
        for g, k0 in enumerate(ka_groups(la, h)):
            nib = (iv >> (off + 4 * g)) & 0xF
            i0, i1 = nib & 3, nib >> 2
            A[r, k0 + i0] += a[l, 2 * g]
            A[r, k0 + i1] += a[l, 2 * g + 1]
    return A


def dense_B(b, lb):
    B = np.zeros((32, 32), np.float64)
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(16):
            B[kb(lb, h, j), r] = b[l, j]
    return B


def D_of(d):
    D = np.zeros((32, 32), np.float64)
    for l in range(64):
        r, h = l & 31, l >> 5
        for reg in range(16):
            D[acc_row(reg, h), r] = d[l, reg]
    return D


def main(path):
    z = np.load(path)
    trials = sorted({k[1:] for k in z.files})
    ioffs = {"same16lo": lambda h: 0, "h*16": lambda h: 16 * h}
    ok = []
    for la, lb, (iname, ioff) in itertools.product(["A1", "A2", "A3"], ["B1", "B2", "B3"], ioffs.items()):
        good = True
        for t in trials:
            A = dense_A(z["a" + t], z["i" + t], la, ioff)
            B = dense_B(z["b" + t], lb)
            if not np.array_equal(A @ B, D_of(z["d" + t])):
                good = False
                break
        print(la, lb, iname, "MATCH" if good else "-")
        if good:
            ok.append((la, lb, iname))
    print("matches:", ok)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/smfmac_probe.npz")
