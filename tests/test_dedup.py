"""Deduplicated h / h' evaluations (csrc/dedup.hip, macbf_gnn_amd/ops/dedup.py).

CPU: the identity the deduplication relies on -- h'(s_{t+1}) of slot (t,b,i,k) equals the next
step's h of the slot holding the same neighbour (or the extra evaluation) -- on the oracle,
and the invariants of the reference index maps."""
import torch

from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E
from macbf_gnn_amd import oracle as O
from macbf_gnn_amd.models import CBF, Controller
from macbf_gnn_amd.ops.dedup import extras_fraction, match_reference


def _rollout(B=2, N=40, T=5, seed=0):
    torch.manual_seed(seed)
    ctrl = Controller(4)
    p = {k: v.detach() for k, v in ctrl.state_dict().items()}
    s0, g = E.generate_batch(B, N, seed=seed + 1)
    with torch.no_grad():
        out = O.rollout(p, s0, g, inner_loops=T, early_stop=False, bptt=False)
    return out


def _eval_h(cbfp, S, idx, src, nev, T, recomputed):
    """h of every deduplicated evaluation u < nev (main slot on s_t / extra on s_{t+1})."""
    B, _, N, _ = S.shape
    K = idx.shape[-1]
    E_ = T * B * N * K
    h_main = torch.stack([O.cbf_forward(cbfp, S[:, t], idx[:, t]) for t in range(T)], 0)   # (T,B,N,K)
    idx_tm = idx.permute(1, 0, 2, 3)                                                      # (T',B,N,K)
    out = torch.zeros(nev)
    out[:E_] = h_main.reshape(-1)
    for u in range(E_, nev):
        e = int(src[u])
        t, r = divmod(e, B * N * K)
        b, r = divmod(r, N * K)
        i, k = divmod(r, K)
        nb_idx = idx_tm[t + 1] if recomputed else idx_tm[t]
        one = torch.zeros(1, N, K, dtype=torch.long)
        one[0, i, 0] = nb_idx[b, i, k]            # slot 0 of agent i = the pair (i, j)
        out[u] = O.cbf_forward(cbfp, S[b:b + 1, t + 1], one)[0, i, 0]
    return out


def test_match_reference_invariants():
    out = _rollout()
    idx = out["idx"].permute(1, 0, 2, 3).contiguous()           # (T,B,N,K)
    T = idx.shape[0]
    map1, src, nev = match_reference(idx, T)
    E_ = idx.numel()
    assert E_ <= nev <= 2 * E_
    flat = map1.reshape(-1)
    assert len(set(flat.tolist())) == E_                        # injective
    assert (src[flat] == torch.arange(E_)).all()                # src inverts map1
    assert (src[nev:] == -1).all()
    # first step's main slots have no source
    BNK = idx[0].numel()
    assert (src[:BNK] == -1).all()
    assert abs(extras_fraction(idx, T) - (nev - E_) / E_) < 1e-9


def test_dedup_identity_on_oracle():
    """h'(s_{t+1}, slot e) == h(evaluation map1[e]) for both neighbour modes."""
    torch.manual_seed(3)
    cbfp = {k: v.detach() for k, v in CBF(4).state_dict().items()}
    out = _rollout(B=2, N=30, T=4, seed=2)
    S = out["S"]                                                 # (B,T+1,N,4)
    idx = out["idx"]                                             # (B,T,N,K)
    T = idx.shape[1]
    for recomputed in (False, True):
        if recomputed:
            extra = O.knn_idx(S[:, T], idx.shape[-1]).unsqueeze(1)
            idx_all = torch.cat([idx, extra], 1)
        else:
            idx_all = idx
        map1, src, nev = match_reference(idx_all.permute(1, 0, 2, 3), T, recomputed=recomputed)
        h = _eval_h(cbfp, S, idx_all, src, nev, T, recomputed)
        nb = idx_all[:, 1:T + 1] if recomputed else idx
        hn_ref = torch.stack([O.cbf_forward(cbfp, S[:, t + 1], nb[:, t]) for t in range(T)], 0)
        torch.testing.assert_close(h[map1.reshape(-1)], hn_ref.reshape(-1), rtol=1e-5, atol=1e-6)
