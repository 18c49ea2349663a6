"""Shared helper of scripts/micro_cbfbwd.py and scripts/stamps_cbf.py."""
import torch


def all_active(a, k, nev, dev):
    """Make every deduplicated evaluation active (index list or records)."""
    if k.get("rec") is None:
        k["act"][:nev] = torch.arange(nev, dtype=torch.int32, device=dev)
    else:
        idx = a[1]
        E = idx.numel()
        idx1 = k["idx1"] if k.get("idx1") is not None else idx
        u = torch.arange(nev, dtype=torch.int64, device=dev)
        p1 = u >= E
        e = torch.where(p1, k["src"][:nev].long(), u)
        j = torch.where(p1, idx1.reshape(-1)[e.clamp(max=E - 1)], idx.reshape(-1)[e.clamp(max=E - 1)])
        dh = a[2].reshape(-1)[:nev].contiguous().view(torch.int32)
        rec = k["rec"]
        rec[:nev, 0] = u.int()
        rec[:nev, 1] = torch.where(p1, e - 2 ** 31, e).int()      # e | pass << 31 as int32
        rec[:nev, 2] = j.int()
        rec[:nev, 3] = dh
    k["nact"].fill_(nev)
