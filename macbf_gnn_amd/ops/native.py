"""Loader and validated launch wrappers for the gfx950 extension ``macbf_gnn_amd._C``.

The extension is built in-tree by ``csrc/build.py`` (``__graft_entry__.build()``). On a HIP
device there is no fallback: if the extension is missing or was built for another arch,
``lib()`` raises. Every wrapper checks device/dtype/contiguity/shape on the host before
passing raw device addresses to the kernels (an out-of-bounds kernel can take the GPU down,
so shapes are never trusted implicitly).
"""
from __future__ import annotations

import functools
import math
import os

import torch

from .. import config as C
from . import layout as L

_LIB = None


class NativeError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        alt = os.environ.get("MACBF_EXT")
        if alt:   # experiment builds (scripts/build_variants.sh) loaded in place of the in-tree .so
            import importlib.util
            import sys
            spec = importlib.util.spec_from_file_location("macbf_gnn_amd._C", alt)
            mod = importlib.util.module_from_spec(spec)
            sys.modules["macbf_gnn_amd._C"] = mod
            spec.loader.exec_module(mod)
        try:
            from .. import _C  # noqa: F401  (in-tree .so)
        except ImportError as e:  # pragma: no cover - exercised on GPU boxes only
            raise NativeError(
                "native extension macbf_gnn_amd._C is not built; run `python csrc/build.py` "
                f"(or __graft_entry__.build()) first: {e}") from e
        _LIB = _C
    return _LIB


_PROBE = None


def probe_lib():
    """The layout-probe extension (csrc/probe.hip, tests only; not part of _C)."""
    global _PROBE
    if _PROBE is None:
        lib()       # HIP runtime + the main extension first
        try:
            from .. import _probe  # noqa: F401
        except ImportError as e:  # pragma: no cover
            raise NativeError(f"probe extension macbf_gnn_amd._probe is not built: {e}") from e
        _PROBE = _probe
    return _PROBE


def available() -> bool:
    try:
        lib()
        return True
    except NativeError:
        return False


def stream_handle(device=None) -> int:
    """Raw hipStream_t of the current stream. Direct C calls (no torch.cuda device-index
    resolution): this runs once per kernel launch and the host issues ~10 launches per rollout
    step, ahead of a GPU that finishes a step in ~0.13 ms."""
    if device is None:
        return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
    return int(torch.cuda.current_stream(device).cuda_stream)


@functools.lru_cache(maxsize=None)
def device_info(index: int = 0) -> dict:
    return dict(lib().device_info(index))


def num_cu(device=None) -> int:
    idx = device.index if isinstance(device, torch.device) and device.index is not None else torch.cuda.current_device()
    return int(device_info(idx).get("cu", 256))


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def check(t, dtype, shape=None, name="tensor"):
    if t is None:
        return
    if not t.is_cuda:
        raise NativeError(f"{name} must be on the HIP device")
    if t.dtype != dtype:
        raise NativeError(f"{name} dtype {t.dtype} != {dtype}")
    if not t.is_contiguous():
        raise NativeError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise NativeError(f"{name} shape {tuple(t.shape)} != {tuple(shape)}")


HALF_DTYPES = (torch.bfloat16, torch.float16)


def _half(t, name, prec=None):
    """Kernel precision variant of a packed-weight tensor (csrc/prec.h): 0 bf16, 1 fp16, 2 the
    fp32-accurate 3-term split ("fp32", bf16 hi/lo planes). prec=None: from the dtype."""
    if t is None or t.dtype not in HALF_DTYPES:
        raise NativeError(f"{name} must be bf16 or fp16")
    if prec is None:
        return int(t.dtype == torch.float16)
    if prec not in L.PREC_CODE:
        raise NativeError(f"unknown precision {prec!r}")
    code = L.PREC_CODE[prec]
    if (code == 1) != (t.dtype == torch.float16):
        raise NativeError(f"{name}: dtype {t.dtype} does not match precision {prec}")
    return code


def _planes(code):
    return 2 if code == 2 else 1


def _prow(code):
    return 256 if code == 2 else 128


def _same_half(t, ref, name):
    if t is not None and t.dtype != ref.dtype:
        raise NativeError(f"{name} dtype {t.dtype} != weight dtype {ref.dtype}")


def _ok(rc, what):
    if rc != 0:
        raise NativeError(f"{what} launch failed: {rc} ({lib().err_str(rc) if rc > 0 else 'bad args'})")


# ----------------------------------------------------------------------------- node records
def rec_width(dim: int) -> int:
    """Floats per node record: D = 2 -> (x, y, vx, vy); D = 3 -> (x, y, z, 0, vx, vy, vz, 0)."""
    return 4 if dim == 2 else 8


def dim_of(S) -> int:
    w = S.shape[-1]
    if w == 4:
        return 2
    if w == 8:
        return 3
    raise NativeError(f"node records must be 4 (2-D) or 8 (3-D) floats wide, got {w}")


def to_records(s: torch.Tensor) -> torch.Tensor:
    """(..., 2D) states -> (..., rec_width(D)) kernel records (identity for D = 2)."""
    D = s.shape[-1] // 2
    if D == 2:
        return s.contiguous()
    z = torch.zeros(*s.shape[:-1], 1, dtype=s.dtype, device=s.device)
    return torch.cat([s[..., :3], z, s[..., 3:6], z], -1).contiguous()


def from_records(r: torch.Tensor) -> torch.Tensor:
    """Inverse of ``to_records``."""
    if r.shape[-1] == 4:
        return r
    return torch.cat([r[..., 0:3], r[..., 4:7]], -1)


# ----------------------------------------------------------------------------- kernels
SMALL_MAXN = 64             # envs up to this many graph nodes: persistent one-launch rollout (ctrl.hip)
SMALL_WAVES = 8


def small_apw(N: int) -> int:
    """Agents per wave of the persistent rollout's edge phase: the env's agents over its 8 waves."""
    a = -(-N // SMALL_WAVES)
    return max(2, min(32, a + (a & 1)))


SCAN_MAX_N = 4096           # envs up to this many graph nodes are staged whole in LDS
SCAN_MAX_NODES = 262144     # beyond SCAN_MAX_N: global staging (csrc/scan.hip scan_stage_kernel); the
                            # culling boxes in LDS up to ~36 K nodes, read from the workspace above


def scan_ws_f4(Nn: int) -> int:
    """float4s of global scan staging per env (0 when the env fits LDS)."""
    if Nn <= SCAN_MAX_N:
        return 0
    Np = (Nn + 7) // 8 * 8
    nch = Np // 8
    nsc = (nch + 7) // 8
    return 2 * Np + 2 * (nch + nsc)


def scan_ws(B: int, Nn: int, device):
    """(workspace tensor or None, float4s per env) for scans of B envs of Nn graph nodes."""
    f4 = scan_ws_f4(Nn)
    if not f4:
        return None, 0
    return _workspace("scan", B * f4 * 16, device), f4
_perm_cache = {}
_perm_sorted = set()      # cached permutation buffers that hold a curve order


def _perm_buf(B, N, device):
    key = (B, N, str(device))
    t = _perm_cache.get(key)
    if t is None:
        t = torch.empty(B, N, dtype=torch.int32, device=device)
        _perm_cache[key] = t
    return t


def scan(S, idx, dang, cnt, safe, *, K, do_knn=True, do_safety=True, perm=None, n_agents=None, prev_idx=None,
         sort=True, lanes=0, stamps=None):
    """K1 over one timestep. S: (B, N, 4) view with env stride (may be a slice of a (B,T+1,N,4)
    buffer); idx/dang: (B, N, K) views; cnt: (B, 2) view; safe: (B,) view.

    Two launches: cell_sort orders each env's agents along a Hilbert curve, then the scan walks
    candidates outward along it (results are order independent; the order only keeps the
    wave-divergent top-K insertion rare). prev_idx (B, N, K): the previous step's kNN of the same
    agents; their current distances bound the K-th distance (tighter culling, same result).
    sort=False reuses the curve order of the previous call on the same perm buffer (the agents
    moved one step: slightly looser culling, identical results). lanes: lanes per agent (0: by
    grid size -- 8 when 4-lane 256-thread blocks leave CUs idle; 4 or 8 forces the layout; the
    lists, bits and counts are identical for either)."""
    if lanes not in (0, 4, 8):
        raise NativeError("lanes must be 0 (auto), 4 or 8")
    B, Nn = S.shape[0], S.shape[1]
    if stamps is not None:   # diagnostics (scripts/stamps_scan.py): [block][wave][16] int64, <= 512 waves per env
        if K != 12 or stamps.dtype != torch.int64 or stamps.numel() < B * 8192 or not stamps.is_contiguous():
            raise NativeError("scan stamps: K = 12 and a contiguous int64 buffer of B * 8192")
    D = dim_of(S)
    W = rec_width(D)
    N = Nn if n_agents is None else int(n_agents)     # centres = the first N nodes
    if Nn > SCAN_MAX_NODES or N > Nn:
        raise NativeError(f"scan: N <= Nn <= {SCAN_MAX_NODES} graph nodes per env (got {N}, {Nn})")
    if S.dtype != torch.float32 or S.stride(2) != 1 or S.stride(1) != W:
        raise NativeError(f"S must be float32 with contiguous (Nn,{W}) rows")
    if K < 1 or K > C.MAX_TOP_K or K > Nn:
        raise NativeError(f"bad K={K} for Nn={Nn}")
    if do_knn:
        if idx.dtype != torch.int32 or tuple(idx.shape) != (B, N, K) or idx.stride(2) != 1 or idx.stride(1) != K:
            raise NativeError("idx must be int32 (B,N,K) with contiguous (N,K)")
        if dang is not None and (dang.dtype != torch.uint8 or tuple(dang.shape) != (B, N, K)
                                 or dang.stride() != idx.stride()):
            raise NativeError("dang must be uint8 (B,N,K) with idx's strides")
        if cnt is not None and (cnt.dtype != torch.float32 or tuple(cnt.shape) != (B, 2) or cnt.stride(1) != 1):
            raise NativeError("cnt must be float32 (B,2)")
    if do_safety and safe is not None and (safe.dtype != torch.float32 or tuple(safe.shape) != (B,)):
        raise NativeError("safe must be float32 (B,)")
    if prev_idx is not None and (not do_knn or prev_idx.dtype != torch.int32 or tuple(prev_idx.shape) != (B, N, K)
                                 or prev_idx.stride(2) != 1 or prev_idx.stride(1) != K):
        raise NativeError("prev_idx must be int32 (B,N,K) with contiguous (N,K)")
    if perm is None:
        perm = _perm_buf(B, Nn, S.device)
        # never scan through a never-sorted (uninitialised) cached permutation: it indexes nodes
        key = (B, Nn, str(S.device))
        if not sort and key not in _perm_sorted:
            sort = True
        _perm_sorted.add(key)
    ws, ws_f4 = scan_ws(B, Nn, S.device)
    if sort:
        L = float(max(1.0, N / C.AGENT_DENSITY) ** (1.0 / D))
        rc = lib().cell_sort(ptr(S), S.stride(0) // W, B, Nn, L, ptr(perm), W // 4, stream_handle())
        _ok(rc, "cell_sort")
    rc = lib().scan(ptr(S), S.stride(0) // W, ptr(perm), B, N, K, ptr(idx) if do_knn else 0,
                    idx.stride(0) if do_knn else 0, ptr(dang) if do_knn else 0,
                    ptr(cnt) if do_knn else 0, cnt.stride(0) if (do_knn and cnt is not None) else 0,
                    ptr(safe) if do_safety else 0, safe.stride(0) if (do_safety and safe is not None) else 0,
                    float(C.DIST_MIN_THRES * C.DIST_MIN_THRES), float(C.TIME_TO_COLLISION),
                    float(C.DIST_MIN_CHECK * C.DIST_MIN_CHECK), float(C.TIME_TO_COLLISION_CHECK),
                    int(do_knn), int(do_safety), Nn, D, ptr(prev_idx),
                    prev_idx.stride(0) if prev_idx is not None else 0, ptr(ws), int(ws_f4), int(lanes),
                    ptr(stamps), stream_handle())
    _ok(rc, "scan")


def scan_plan(B: int, N: int, K: int, *, Nn: int | None = None, dim: int = 2, prev: bool = True, do_knn: bool = True,
              do_safety: bool = True, lanes: int = 0) -> dict:
    """The launch plan ``scan`` picks for a call of this shape, without launching (csrc/scan.hip
    mb_scan_plan): block size ``bs``, lanes per agent ``lpa``, staging mode ``glb`` (0 LDS, 1 global
    records, 2 global boxes), cell-grid LDS allocated ``cells`` / searched ``use_cells``, grid side
    ``cell_g``, per-wave count atomics ``wave_atomic``, ``blocks`` and dynamic ``lds`` bytes. Tests
    use it to assert the instantiation they exercise."""
    Nn = N if Nn is None else int(Nn)
    v = lib().scan_plan(int(B), int(N), int(K), Nn, int(dim), int(bool(prev)), int(bool(do_knn)),
                        int(bool(do_safety)), int(lanes))
    return dict(zip(("bs", "lpa", "glb", "cells", "use_cells", "cell_g", "wave_atomic", "blocks", "lds"), v))


def scenario(S, G, *, seed, L, r=C.DIST_MIN_THRES, spread=C.GOAL_SPREAD, max_rounds=256, status=None, obs=None,
             lds_free=False):
    """S (B, >=N, W) agent records out (velocity 0), G (B, N, D) goals out; obs (B, M, D) static
    obstacle points kept > r from every start and goal. lds_free: the per-env arrays and cell grid
    in a global workspace even when they fit LDS (the large-env path; same results)."""
    B, N, D = G.shape
    W = rec_width(D)
    _records(S, "S", (B, N), W)
    check(G, torch.float32, (B, N, D), "G")
    check(status, torch.int32, (B,), "status")
    M = 0
    if obs is not None:
        M = obs.shape[1]
        check(obs, torch.float32, (B, M, D), "obs")
    base = (3 * N + M) * D * 4 + 5 * N + 16
    ws, ws_env = None, 0
    if lds_free or base + 4 * 2 ** D > 160 * 1024 - 64:
        # env too large for LDS: the sampler's arrays live in a per-env global workspace with a
        # full-resolution cell grid (same results: acceptance does not depend on the grid)
        span = float(L) + 2.0 * (float(spread) + float(r))
        import numpy as _np
        G1 = max(1, int(_np.floor(_np.float32(span) / _np.float32(r))))
        ws_env = (base + 4 * (G1 + 2) ** D + 255) // 256 * 256      # (+2: float rounding slack)
        ws = _workspace("scenario", B * ws_env, S.device)
    rc = lib().scenario(ptr(S), S.stride(0) // W, ptr(G), ptr(obs), M, D, B, N, float(L), float(r), float(spread),
                        int(seed) & 0xFFFFFFFFFFFFFFFF, int(max_rounds), ptr(status), ptr(ws), int(ws_env),
                        stream_handle())
    _ok(rc, "scenario")


_WS = {}


def _workspace(name, nbytes, device):
    """Cached uint8 device scratch, one per (name, device, current stream): grown on demand,
    reused in stream order. Per stream, because launches on different streams may run
    concurrently (the trainer samples the next iteration's scenarios on a side stream while
    the current one is still being sampled / simulated) and must not share scratch."""
    key = (name, str(device), stream_handle(device))
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
        _WS[key] = t
    return t


def _rows(t, last, name, lead):
    """t is a float/bf16 view whose trailing dims are contiguous rows of width `last`."""
    if t is None:
        return
    if tuple(t.shape[:len(lead)]) != tuple(lead) or t.shape[-1] != last or t.stride(-1) != 1 \
            or t.stride(-2) != last:
        raise NativeError(f"{name}: expected {lead}x{last} with contiguous rows, got {tuple(t.shape)} {t.stride()}")


def _records(t, name, lead, W, min_rows=None):
    """(lead..., rows, W) float32 view with contiguous records; rows may exceed lead[-1] (nodes)."""
    if t is None:
        return
    if t.dtype != torch.float32 or t.dim() != len(lead) + 1 or tuple(t.shape[:len(lead) - 1]) != tuple(lead[:-1]) \
            or t.shape[-2] < lead[-1] or t.shape[-1] != W or t.stride(-1) != 1 or t.stride(-2) != W:
        raise NativeError(f"{name}: expected {lead}x{W} float32 records, got {tuple(t.shape)} {t.stride()}")


def ctrl_fwd(S, G, idx, wpack, f_edge, f_node, wvec, A, Sn, dist_sum, act_sum, noise=None, pooled=None, argmax=None,
             prec=None, noise_key=None, noise_prob=0.0, noise_scale=0.0, noise_t=0, stamps=None):
    """Fused controller step on per-step views: S/Sn (B,Nn,W) node records (agents first),
    G (B,N,D), idx (B,N,K), A (B,N,D), dist_sum/act_sum (B,) int64 fixed point (x FX_DIST /
    x FX_ACT: order-independent integer atomics), pooled (B,N,128) bf16
    ((B,N,256) [hi | lo] rows for prec="fp32", required there), argmax (B,N,128) uint8."""
    B, N, K = idx.shape
    D = dim_of(S)
    W = rec_width(D)
    if K < 1 or K > C.MAX_TOP_K:
        raise NativeError("K out of range")
    _records(S, "S", (B, N), W)
    _records(Sn, "Sn", (B, N), W)
    _rows(A, D, "A", (B, N))
    check(G, torch.float32, (B, N, D), "G")
    if idx.dtype != torch.int32 or idx.stride(2) != 1 or idx.stride(1) != K:
        raise NativeError("idx must be int32 (B,N,K)")
    f16 = _half(wpack, "wpack", prec)
    check(wpack, wpack.dtype, None, "wpack")
    check(wvec, torch.float32, None, "wvec")
    if wvec.numel() < 352 or wpack.numel() < (f_node + 54) * 512 * _planes(f16):
        raise NativeError("packed controller weights too small")
    if f16 == 2 and pooled is None:
        raise NativeError("the fp32 (x3) controller step needs the pooled buffer")
    for t, n in ((dist_sum, "dist_sum"), (act_sum, "act_sum")):
        if t is not None and (t.dtype != torch.int64 or tuple(t.shape) != (B,)):
            raise NativeError(f"{n} must be int64 (B,) fixed point")
    _rows(noise, D, "noise", (B, N))
    check(noise_key, torch.int64, (1,), "noise_key")
    if pooled is not None:
        _rows(pooled, _prow(f16), "pooled", (B, N))
        _same_half(pooled, wpack, "pooled")
    if argmax is not None:
        _rows(argmax, 128, "argmax", (B, N))
        if argmax.dtype != torch.uint8:
            raise NativeError("argmax must be uint8")
    if stamps is not None:   # diagnostics (scripts/stamps_ctrl.py): x3 step only, [blocks, 8 waves, 16]
        if f16 != 2 or stamps.dtype != torch.int64 or not stamps.is_contiguous():
            raise NativeError("ctrl_fwd stamps: int64 buffer of the x3 step")
        if stamps.numel() < 16 * 8 * 2 * num_cu(S.device):       # the grid is at most 2 blocks per CU
            raise NativeError("ctrl_fwd stamps buffer too small")
    rc = lib().ctrl_fwd(ptr(S), S.stride(0) // W, ptr(G), ptr(idx), idx.stride(0), B, N, K,
                        ptr(wpack), int(f_edge), int(f_node), ptr(wvec),
                        ptr(A), A.stride(0) // D if A is not None else 0,
                        ptr(Sn), Sn.stride(0) // W if Sn is not None else 0,
                        ptr(dist_sum), dist_sum.stride(0) if dist_sum is not None else 0,
                        ptr(act_sum), act_sum.stride(0) if act_sum is not None else 0,
                        ptr(noise), noise.stride(0) // D if noise is not None else 0,
                        float(C.TIME_STEP), float(C.OBS_RADIUS), float(C.SQRT3),
                        ptr(pooled), pooled.stride(0) if pooled is not None else 0,
                        ptr(argmax), argmax.stride(0) if argmax is not None else 0,
                        D, num_cu(S.device), f16, ctrl_fwd_apw(B * N, S.device, N),
                        ptr(noise_key), float(noise_prob), float(noise_scale), int(noise_t), ptr(stamps),
                        stream_handle())
    _ok(rc, "ctrl_fwd")


def ctrl_fwd_apw(total_agents: int, device, n_agents: int | None = None) -> int:
    """Agents per wave of the controller step's edge phase: 32, halved (down to 4) while the
    scene has fewer groups than eight per CU, so smaller scenes spread the edge phase over more
    waves; scenes of >= 8,192 agents stop at 8. Measured per-rank work of config #3 (fp32,
    interleaved, profiles/r6_runs/r6au/, r6av/, r6ap/): 65,536 agents 32 / 16 / 8 -> 10.08-10.27 /
    10.41-10.43 / 11.02 ms; 32,768: 16 -> 5.79 vs 6.17-6.24 (32) and 6.19 (8); 16,384: 8 -> 3.88-3.90
    vs 3.97-4.27 (16) and 4.17 (4); 8,192: 8 -> 2.80-2.82 vs 2.91-2.98 (4) and 2.91-2.96 (16). Any
    grouping gives the same results (the per-env sums are per-agent fixed-point integers).
    MACBF_CTRL_APW overrides (A/B runs)."""
    env = os.environ.get("MACBF_CTRL_APW")
    if env:
        return int(env)
    apw, cap = 32, 8 * num_cu(device)
    for cand in (16, 8, 4):
        if (total_agents + apw - 1) // apw >= cap or (cand == 4 and total_agents >= 8192):
            break
        apw = cand
    return apw


LOSS_CONSTS = (C.LOSS_EPS_DANG, C.TIME_STEP * C.ALPHA_CBF, C.LOSS_WEIGHTS[0], C.LOSS_WEIGHTS[1],
               C.LOSS_WEIGHTS[2], C.LOSS_WEIGHTS[3], C.LOSS_SCALE)


def _loss_consts(grad_scale=1.0, gscale=None):
    """LOSS_CONSTS with the upstream-gradient scale: a host factor and/or a device loss scale
    (fp16 dynamic scaling: 1-element float32 tensor read by the kernel, no host round trip)."""
    check(gscale, torch.float32, (1,), "gscale")
    return LOSS_CONSTS[:6] + (LOSS_CONSTS[6] * float(grad_scale), ptr(gscale))
CBF_FWD_WAVES = 4
CBF_PARTIAL = 18704
CBF_P_LOSS = 18692          # 10 loss partial sums in the CBF slab (fused mode)
CTRL_NODE_PARTIAL = 28896
CTRL_EDGE_PARTIAL = 10368
NODE_RM_ELEMS = 64 * 168 + 128 * 68 + 64 * 132 + 32 * 68     # csrc/ctrl.hip row-major node images


def cbf_fwd_grid(E: int, device) -> int:
    tiles = (E + 31) // 32
    return max(1, min((tiles + CBF_FWD_WAVES - 1) // CBF_FWD_WAVES, num_cu(device) * 4))


def _time_major_S(S, T, B, N, need):
    """S (>= T+need, B, Nn >= N, W) node records (agents first, then obstacle points)."""
    W = S.shape[-1] if S.dim() == 4 else 0
    if S.dtype != torch.float32 or S.dim() != 4 or S.shape[0] < T + need or S.shape[1] != B \
            or S.shape[2] < N or W not in (4, 8) or S.stride(3) != 1 or S.stride(2) != W:
        raise NativeError(f"S must be float32 (>=T+{need}, B, >=N, 4|8) with contiguous rows")
    return dim_of(S), W


def cbf_fwd(S, idx, wpack, f_fwd, wvec, *, dang=None, valid=None, two=True, h_out=None, hn_out=None,
            dh_out=None, counts=None, partial=None, num_blocks=None, prec=None):
    """Time-major: S (>=T+two, B, N, 4); idx/dang/h (T, B, N, K); valid (T, B); dh (2, T, B, N, K)."""
    T, B, N, K = idx.shape
    check(idx, torch.int32, None, "idx")
    D, W = _time_major_S(S, T, B, N, 1 if two else 0)
    E = B * T * N * K
    check(dang, torch.uint8, (T, B, N, K), "dang")
    check(valid, torch.uint8, (T, B), "valid")
    check(h_out, torch.float32, (T, B, N, K), "h_out")
    check(hn_out, torch.float32, (T, B, N, K), "hn_out")
    check(dh_out, torch.float32, (2, T, B, N, K), "dh_out")
    if dh_out is not None:
        check(counts, torch.float32, None, "counts")
    f16 = _half(wpack, "wpack", prec)
    check(wpack, wpack.dtype, None, "wpack")
    check(wvec, torch.float32, None, "wvec")
    if wpack.numel() < (f_fwd + 34) * 512 * _planes(f16):
        raise NativeError("packed CBF weights too small")
    nb = num_blocks or cbf_fwd_grid(E, S.device)
    check(partial, torch.float32, (nb, 10), "partial")
    rc = lib().cbf_fwd(ptr(S), S.stride(1) // W, S.stride(0) // W, ptr(idx), ptr(dang), ptr(valid),
                       B, T, N, K, int(two), ptr(wpack), int(f_fwd), ptr(wvec), ptr(h_out), ptr(hn_out),
                       ptr(dh_out), ptr(counts), ptr(partial), LOSS_CONSTS,
                       float(C.OBS_RADIUS), float(C.DIST_MIN_THRES), float(C.CBF_DIST_EPS_COORD * D), D, nb,
                       f16, stream_handle())
    _ok(rc, "cbf_fwd")
    return nb


# ----------------------------------------------------------------------------- deduplicated h / h'
MATCH_BLOCK = 256


def cbf_match(idx, T, map1, src, cnt, *, recomputed=False, nev=None):
    """Deduplicate the h / h' evaluations of a rollout (csrc/dedup.hip).

    idx (>= T + recomputed, B, N, K) int32 neighbour slots. Writes map1 (T, B, N, K): the
    evaluation index of each slot's h' partner (< E: the next step's main slot with the same
    neighbour; >= E: an extra evaluation) and src (2E): the slot whose h' evaluation u is, or
    -1. cnt: int32 scratch (>= one entry per 256-row block). Returns the device int32 tensor
    [U] (evaluations; written into `nev` when given). Two launches, the exclusive scan of the
    per-row extras counts runs inside the kernels; stream-ordered, no host synchronisation."""
    _, B, N, K = idx.shape
    if idx.shape[0] < T + int(recomputed):
        raise NativeError("idx has too few steps")
    check(idx, torch.int32, None, "idx")
    E = T * B * N * K
    if 2 * E >= 2 ** 31:
        raise NativeError("too many edge evaluations for 32-bit indexing")
    check(map1, torch.int32, (T, B, N, K), "map1")
    check(src, torch.int32, (2 * E,), "src")
    rows = T * B * N
    nblk = (rows + MATCH_BLOCK - 1) // MATCH_BLOCK
    check(cnt, torch.int32, None, "cnt")
    if cnt.numel() < nblk:
        raise NativeError("cnt too small")
    if nev is None:
        nev = torch.empty(1, dtype=torch.int32, device=idx.device)
    check(nev, torch.int32, (1,), "nev")
    mode = 1 if recomputed else 0
    rowcnt = _workspace("match_rows", rows * 4, idx.device).view(torch.int32)
    # phase 0: match + everything but the extras' offsets; phase 1: the offsets (rows with extras)
    _ok(lib().cbf_match(ptr(idx), T, B, N, K, mode, 0, ptr(rowcnt), 0, ptr(map1), ptr(src), ptr(cnt), 0,
                        stream_handle()), "cbf_match/match")
    _ok(lib().cbf_match(ptr(idx), T, B, N, K, mode, 1, ptr(rowcnt), 0, ptr(map1), ptr(src), ptr(cnt), ptr(nev),
                        stream_handle()), "cbf_match/extras")
    return nev


HFWD_WAVES = 8


def cbf_hfwd_grid(EV: int, device, per_cu: int | None = None) -> int:
    """Workgroups of an h evaluation launch: up to per_cu per CU (default 4)."""
    tiles = (EV + 31) // 32
    if per_cu is None:
        per_cu = 4
    return max(1, min((tiles + HFWD_WAVES - 1) // HFWD_WAVES, num_cu(device) * per_cu))


def cbf_hfwd(S, idx, idx1, src, nev, wpack, f_fwd, wrm, wvec, h_out, mask_out, num_blocks=None,
             u_begin=0, u_end=None, prec=None):
    """h (masked) and the radius mask of every evaluation u_begin <= u < (u_end or nev) of the
    deduplicated list: S (>= T+1, B, N, W); idx / idx1 (T, B, N, K) (idx1 = idx for
    reuse_nbr_idx); src, h_out, mask_out (>= 2E,). Weights: w1f fragments at f_fwd of wpack + the
    row-major W2|W3 image. A host range [u_begin, u_end) within the main slots (u_end <= E) needs
    neither src nor nev contents: the rollout evaluates step t's main slots (idx[:t+1]) while
    later steps are still being simulated."""
    T, B, N, K = idx.shape
    check(idx, torch.int32, None, "idx")
    check(idx1, torch.int32, (T, B, N, K), "idx1")
    D, W = _time_major_S(S, T, B, N, 1)
    E = B * T * N * K
    if 2 * E >= 2 ** 31:
        raise NativeError("too many edge evaluations for 32-bit indexing")
    cap = src.numel() if src is not None else 0
    if u_end is not None and not (0 <= u_begin <= u_end <= E):
        raise NativeError(f"host range [{u_begin}, {u_end}) must lie in the main slots [0, {E})")
    if cap < 2 * E or h_out is None or h_out.numel() < 2 * E or mask_out is None or mask_out.numel() < 2 * E:
        raise NativeError("src / h_out / mask_out must hold >= 2E evaluations")
    check(src, torch.int32, None, "src")
    check(nev, torch.int32, (1,), "nev")
    check(h_out, torch.float32, None, "h_out")
    check(mask_out, torch.uint8, None, "mask_out")
    f16 = _half(wpack, "wpack", prec)
    check(wpack, wpack.dtype, None, "wpack")
    check(wrm, wpack.dtype, (_planes(f16) * (128 * 68 + 64 * 148),), "wrm")
    check(wvec, torch.float32, None, "wvec")
    if wpack.numel() < (f_fwd + 2) * 512 * _planes(f16):
        raise NativeError("packed CBF weights too small")
    if u_end is not None and u_end == u_begin:
        return 0
    nb = num_blocks or cbf_hfwd_grid((u_end if u_end is not None else 2 * E) - u_begin, S.device)
    rc = lib().cbf_hfwd(ptr(S), S.stride(1) // W, S.stride(0) // W, ptr(idx), ptr(idx1), ptr(src), ptr(nev),
                        B, T, N, K, ptr(wpack), int(f_fwd), ptr(wrm), ptr(wvec), ptr(h_out), ptr(mask_out),
                        float(C.OBS_RADIUS), float(C.DIST_MIN_THRES), float(C.CBF_DIST_EPS_COORD * D), D, nb,
                        f16, int(u_begin), int(u_end or 0), stream_handle())
    _ok(rc, "cbf_hfwd")
    return nb


DH_BLOCK = 256
DH_PARTIAL = 12


def cbf_dh_grid(EV: int, device) -> int:
    # >= ~8 evaluations per thread (the loop body is a chain of dependent gathers, map1 -> h),
    # 16 blocks per CU: enough loads in flight, a small partial-sum slab
    return max(1, min((EV + 8 * DH_BLOCK - 1) // (8 * DH_BLOCK), num_cu(device) * 16))


def cbf_dh(h, hmask, map1, src, nev, dang, valid, counts, dh, partial, *, grad_scale=1.0, blk_active=None,
           gscale=None):
    """Upstream dL/dh of every deduplicated evaluation (h-role + h'-role) and the 10 loss
    partial sums per block (slots as CBF_P_LOSS: [0, 0, 8 sums], padded) -> partial (nb, DH_PARTIAL)."""
    T, B, N, K = map1.shape
    E = T * B * N * K
    check(h, torch.float32, (2 * E,), "h")
    check(hmask, torch.uint8, (2 * E,), "hmask")
    check(map1, torch.int32, (T, B, N, K), "map1")
    check(src, torch.int32, (2 * E,), "src")
    check(nev, torch.int32, (1,), "nev")
    check(dang, torch.uint8, (T, B, N, K), "dang")
    check(valid, torch.uint8, (T, B), "valid")
    check(counts, torch.float32, None, "counts")
    check(dh, torch.float32, (2 * E,), "dh")
    if partial is None or partial.dim() != 2 or partial.shape[1] != DH_PARTIAL:
        raise NativeError(f"partial must be (nb, {DH_PARTIAL})")
    check(partial, torch.float32, None, "partial")
    nb = partial.shape[0]
    check(blk_active, torch.int32, (nb,), "blk_active")
    _ok(lib().cbf_dh(ptr(h), ptr(hmask), ptr(map1), ptr(src), ptr(nev), ptr(dang), ptr(valid), B, T, N, K,
                     ptr(counts), _loss_consts(grad_scale, gscale), ptr(dh), ptr(partial),
                     ptr(blk_active), nb, stream_handle()), "cbf_dh")


def cbf_active(dh, nev, blk_active, act, nact=None, *, rec=None, src=None, idx=None, idx1=None):
    """Stable list of the evaluations with dh != 0 (cbf_dh's per-block counts blk_active, same
    grid): act[:nact] in index order. Returns the device int32 tensor [nact] (written into
    `nact` when given; block offsets are scanned in-kernel, one launch). The backward skips the
    rest: their upstream gradient, hence every contribution, is exactly zero.

    rec (int32 (2E, 4), the 16x16x32 x3 backward's input) replaces act: one record per active
    evaluation {u, e | pass << 31, neighbour j, dh bits}, resolved through src (deduplicated
    list) and idx (T,B,N,K) / idx1 (pass-1 neighbours, None = idx)."""
    check(dh, torch.float32, None, "dh")
    check(nev, torch.int32, (1,), "nev")
    check(blk_active, torch.int32, None, "blk_active")
    if rec is None:
        check(act, torch.int32, (dh.numel(),), "act")
    else:
        check(rec, torch.int32, (dh.numel(), 4), "rec")
        check(src, torch.int32, (dh.numel(),), "src")
        check(idx, torch.int32, None, "idx")
        check(idx1, torch.int32, tuple(idx.shape), "idx1")
        if 2 * idx.numel() != dh.numel():
            raise NativeError("rec: dh must cover the two passes of idx")
    if nact is None:
        nact = torch.empty(1, dtype=torch.int32, device=dh.device)
    check(nact, torch.int32, (1,), "nact")
    E = idx.numel() if idx is not None else 0
    _ok(lib().cbf_compact(ptr(dh), ptr(nev), 0, ptr(act) if rec is None else 0, blk_active.numel(),
                          ptr(blk_active), ptr(nact), ptr(src), ptr(idx), ptr(idx1), int(E), ptr(rec),
                          stream_handle()), "cbf_compact")
    return nact


def node_act_bytes(prec) -> int:
    """Bytes per agent and step of the node activations the rollout keeps for the cooperative node
    backward (csrc/ctrl.hip NODE_ACT_BYTES: 1152 x3, 640 in the 16-bit builds)."""
    return int(lib().node_act_bytes(L.PREC_CODE[prec]))


def k16_wg_per_cu(prec, kernel: int) -> int:
    """Workgroups per CU of the 16x16x32 backward kernel `kernel` (0 CBF, 1 edge, 2 node) of the
    build of `prec` (csrc/mfma16.h: x3 one, the 1-pass builds two)."""
    return int(lib().k16_wg_per_cu(L.PREC_CODE[prec], kernel))


def cbf_bwd_grid(EV: int, device, prec=None) -> int:
    """Workgroups of the CBF backward over EV evaluations (128 per chunk): one per CU, or as many
    as the 16x16x32 kernel of `prec` keeps resident per CU when prec is given."""
    per_cu = k16_wg_per_cu(prec, 0) if prec is not None else 1
    return max(1, min((EV + 127) // 128, per_cu * num_cu(device)))


CBF_RM16 = 128 * 80 + 64 * 144     # elements per plane of the 16x16x32 W2 | W3 images (layout.cbf_rm16)


def cbf_bwd(S, idx, dh, wpack, f_bwd, wrm, wvec, *, passes=2, dE=None, partial=None, num_blocks=None,
            fused=False, dang=None, valid=None, counts=None, idx1=None, grad_scale=1.0, src=None, nev=None,
            act=None, nact=None, prec=None, gscale=None, stamps=None, rec=None, wrm16=None, w16=None, dbg=None):
    """dh (passes, T, B, N, K) -> dE (passes, T, B, N, K, 4), per-WG dW slabs (nb, CBF_PARTIAL).

    fused=True (training, passes=2): dh is not read; the kernel evaluates h and h' of every
    edge, forms the hinge-loss upstream gradients from dang (T,B,N,K), valid (T,B) and the
    global counts [n_dang, n_safe], and writes the 10 loss partial sums at CBF_P_LOSS.
    grad_scale multiplies the in-kernel upstream gradients (fp16 loss scaling); the loss sums
    are unscaled.

    src/nev (deduplicated list, non-fused, passes=2): evaluation u < nev is main slot u (u < E)
    or the extra evaluation of slot src[u] on s_{t+1}; dh / dE are indexed by u (sizes 2E)."""
    T, B, N, K = idx.shape
    check(idx, torch.int32, None, "idx")
    D, W = _time_major_S(S, T, B, N, passes - 1)
    if fused:
        if passes != 2:
            raise NativeError("fused CBF backward needs passes=2")
        check(dang, torch.uint8, (T, B, N, K), "dang")
        check(valid, torch.uint8, (T, B), "valid")
        check(counts, torch.float32, None, "counts")
        if dang is None or counts is None or counts.numel() < 2:
            raise NativeError("fused CBF backward needs dang and counts")
    else:
        check(dh, torch.float32, (passes, T, B, N, K), "dh")
    check(dE, torch.float32, (passes, T, B, N, K, W), "dE")
    if src is not None:
        if fused or passes != 2:
            raise NativeError("deduplicated CBF backward is non-fused with passes=2")
        check(src, torch.int32, (2 * B * T * N * K,), "src")
        check(nev, torch.int32, (1,), "nev")
    if act is not None:
        if src is None:
            raise NativeError("the active list needs the deduplicated evaluation list")
        check(act, torch.int32, (2 * B * T * N * K,), "act")
        check(nact, torch.int32, (1,), "nact")
    f16 = _half(wpack, "wpack", prec)
    if rec is not None:
        # 16x16x32 backward over cbf_compact's records (csrc/cbf16.h)
        if fused or src is None:
            raise NativeError("record backward: deduplicated non-fused path only")
        check(rec, torch.int32, (2 * B * T * N * K, 4), "rec")
        check(nact, torch.int32, (1,), "nact")
        check(wrm16, wpack.dtype, (_planes(f16) * CBF_RM16,), "wrm16")
        check(w16, wpack.dtype, (6 * 512 * _planes(f16),), "w16")
    check(wpack, wpack.dtype, None, "wpack")
    check(wvec, torch.float32, None, "wvec")
    if wpack.numel() < (f_bwd + 70) * 512 * _planes(f16):
        raise NativeError("packed CBF weights too small")
    check(wrm, wpack.dtype, (_planes(f16) * (128 * 68 + 64 * 148),), "wrm")
    if idx1 is not None:
        check(idx1, torch.int32, (T, B, N, K), "idx1")
    E = B * T * N * K
    if E * passes >= 2 ** 31:
        raise NativeError("too many edge evaluations for 32-bit indexing")
    nb = num_blocks or cbf_bwd_grid(E * passes, S.device)
    check(partial, torch.float32, (nb, CBF_PARTIAL), "partial")
    check(stamps, torch.int64, (nb, 8 if (rec is not None or f16 != 2) else 4, 8), "stamps")   # phase cycles
    rc = lib().cbf_bwd(ptr(S), S.stride(1) // W, S.stride(0) // W, ptr(idx), B, T, N, K, int(passes),
                       0 if fused else ptr(dh),
                       ptr(wpack), int(f_bwd), ptr(wrm), ptr(wvec), ptr(dE), ptr(partial), float(C.OBS_RADIUS),
                       float(C.DIST_MIN_THRES), float(C.CBF_DIST_EPS_COORD * D), int(fused), ptr(dang) if fused else 0,
                       ptr(valid) if fused else 0, ptr(counts) if fused else 0,
                       _loss_consts(grad_scale, gscale), ptr(idx1), D, nb,
                       f16, ptr(src), ptr(nev) if src is not None else 0, ptr(act), ptr(nact) if (act is not None or rec is not None) else 0,
                       ptr(rec), ptr(wrm16), ptr(w16), ptr(dbg), ptr(stamps), stream_handle())
    _ok(rc, "cbf_bwd")
    return nb


def rev_csr(idx, rptr, redges, n_nodes=None):
    """idx (G, N, K) int32 contiguous -> rptr (G, Nn+1), redges (G, N*K); Nn = n_nodes (agents +
    obstacle points, default N)."""
    Gn, N, K = idx.shape
    Nn = N if n_nodes is None else int(n_nodes)
    check(idx, torch.int32, (Gn, N, K), "idx")
    check(rptr, torch.int32, (Gn, Nn + 1), "rptr")
    check(redges, torch.int32, (Gn, N * K), "redges")
    ws = None
    if (2 * Nn + 1) * 4 > 150 * 1024:         # counters beyond LDS: csrc/graph.hip global path
        ws = _workspace("csr", Gn * Nn * 4, idx.device)
    _ok(lib().rev_csr(ptr(idx), Gn, N, K, ptr(rptr), ptr(redges), Nn, ptr(ws), stream_handle()), "rev_csr")


def node_reduce(dE, rptr, redges, out, *, T, B, N, K, passes=2, accumulate=False, pass_mask=0, shift1=0,
                n_nodes=None, map1=None, gate=None, t_range=None):
    """dE (passes, T, B, N, K, W) -> out[t'] (+)= sum over passes p of the edge->node reduction of
    step t' - p, for the N agents. pass_mask selects passes (0 = all); shift1=1: pass-1 edges live
    in graph t+1 (h' on the recomputed kNN of s_{t+1}), so the CSR arrays must hold T+1 graphs.
    map1 (T, B, N, K): deduplicated evaluations (cbf_match) -- dE is then indexed by evaluation
    and pass 1 reads only the extras map1[e] >= E. t_range=(lo, hi): only output steps
    lo <= t' < hi (the BPTT consumes dS from the last step down: the early steps can be reduced
    on a side stream while it runs)."""
    Nn = N if n_nodes is None else int(n_nodes)
    W = dE.shape[-1]
    D = 2 if W == 4 else 3
    check(dE, torch.float32, (passes, T, B, N, K, W), "dE")
    check(rptr, torch.int32, None, "rptr")
    check(redges, torch.int32, None, "redges")
    if rptr.shape[0] < (T + shift1) * B or redges.shape[0] < (T + shift1) * B or rptr.shape[1] != Nn + 1:
        raise NativeError("reverse CSR too small")
    if out.dtype != torch.float32 or not out.is_contiguous() or out.shape[0] < T + 1 or \
            tuple(out.shape[1:]) != (B, N, W):
        raise NativeError(f"out must be float32 (>=T+1, B, N, {W})")
    if map1 is not None:
        check(map1, torch.int32, (T, B, N, K), "map1")
        if passes != 2:
            raise NativeError("map1 needs passes=2")
    if gate is not None:
        check(gate, torch.float32, (passes * T * B * N * K,), "gate")
    lo, hi = (0, 0) if t_range is None else (int(t_range[0]), int(t_range[1]))
    if t_range is not None and not (0 <= lo < hi <= T + 1):
        raise NativeError(f"t_range must satisfy 0 <= lo < hi <= T+1 (got {t_range}, T={T})")
    _ok(lib().node_reduce(ptr(dE), ptr(rptr), ptr(redges), B, T, N, K, passes, int(accumulate), ptr(out),
                          int(pass_mask), int(shift1), Nn, D, ptr(map1), ptr(gate), int(lo), int(hi),
                          stream_handle()), "node_reduce")


def node_combine(dS_t, ego, dEc, rptr_t, redges_t, Gn, Gout, *, K, dt=C.TIME_STEP):
    """All (B,N,W) record views; dEc (B,N,K,W); rptr_t (B, Nn+1) / redges_t (B, N*K) of graph t."""
    B, N, W = dS_t.shape
    D = 2 if W == 4 else 3
    _records(dS_t, "dS_t", (B, N), W)
    _records(Gout, "Gout", (B, N), W)
    _records(Gn, "Gn", (B, N), W)
    check(ego, torch.float32, (B, N, W), "ego")
    check(dEc, torch.float32, (B, N, K, W), "dEc")
    if dEc is not None:
        if rptr_t.dtype != torch.int32 or rptr_t.shape[0] != B or rptr_t.shape[1] < N + 1 or rptr_t.stride(1) != 1:
            raise NativeError("rptr_t must be int32 (B, Nn+1)")
        if redges_t.dtype != torch.int32 or tuple(redges_t.shape) != (B, N * K) or redges_t.stride(1) != 1:
            raise NativeError("redges_t must be int32 (B, N*K)")
    _ok(lib().node_combine(ptr(dS_t), dS_t.stride(0) // W, ptr(ego), ptr(dEc),
                           ptr(rptr_t), rptr_t.stride(0) if dEc is not None else 0,
                           ptr(redges_t), redges_t.stride(0) if dEc is not None else 0,
                           ptr(Gn), Gn.stride(0) // W if Gn is not None else 0,
                           ptr(Gout), Gout.stride(0) // W, B, N, K, float(dt), D, stream_handle()), "node_combine")


CTRL_EDGE_WAVES = 4          # csrc/ctrl.hip EB_WAVES


def ctrl_edge_qsplit(total_agents: int, device) -> int:
    """Workgroups per 128-agent chunk of the edge backward: small scenes split a chunk's tile
    rounds (K of them with the dense edge rows, csrc/ctrl.hip) over up to 16 workgroups (the tiles
    are independent; a single wave would otherwise run all of them back to back; a part with no
    tile writes a zero slab row); 1 once the chunks alone fill the GPU."""
    che = (total_agents + 32 * CTRL_EDGE_WAVES - 1) // (32 * CTRL_EDGE_WAVES)
    cap = (8 // CTRL_EDGE_WAVES) * num_cu(device)
    p = 1
    while p < 16 and che * p * 2 <= cap:
        p *= 2
    return p


def node_bwd_chunk(total_agents: int, device) -> int:
    """Agents per node-backward workgroup chunk: 128 while the chunks fill half the CUs, else 64
    while they fill the CUs, else 32 (small scenes and strong-scaling slices: more, shorter
    workgroups; a chunk's empty stage turns are skipped). At 16,384 agents (config #3 per rank at
    DP 4) 128 over 64: 3.815-3.853 vs 3.873-3.888 ms interleaved (profiles/r6_runs/r6ax/, r6ay/).
    MACBF_NODE_CHUNK overrides."""
    env = os.environ.get("MACBF_NODE_CHUNK")
    if env:
        return int(env)
    cu = num_cu(device)
    if (total_agents + 127) // 128 >= cu // 2:
        return 128
    if (total_agents + 63) // 64 >= cu:
        return 64
    return 32


def ctrl_bwd_grids(total_agents: int, device, prec=None, eb16=False):
    """(node, edge) backward grids: the node kernel takes node_bwd_chunk-agent chunks, one
    workgroup per CU; the edge kernel 32*CTRL_EDGE_WAVES-agent chunks x ctrl_edge_qsplit tile
    ranges, at most as many workgroups as fit the CUs at once (4 waves: two per CU in the 16-bit
    builds; one in the fp32 (x3) build -- 322 registers, 118 KB of LDS: a grid of one per CU
    loops over two chunks instead of running a second round of workgroups, 142 -> 137 us per
    call at 1024 x 64, profiles/r2_egrid/); eb16: the 8-wave 16x16x32 kernel (same 128-agent
    chunks, k16_wg_per_cu per CU). MACBF_EDGE_WG_PER_CU overrides the cap."""
    ca = node_bwd_chunk(total_agents, device)
    ch = (total_agents + ca - 1) // ca
    che = (total_agents + 32 * CTRL_EDGE_WAVES - 1) // (32 * CTRL_EDGE_WAVES)
    cu = num_cu(device)
    if bwd_step_fused(total_agents, device):      # one fused launch per step: one grid for both
        n = max(1, min(ch, cu))
        return n, n
    if eb16:
        per_cu = k16_wg_per_cu(prec or "bf16", 1)
    else:
        per_cu = 1 if prec == "fp32" else 8 // CTRL_EDGE_WAVES
    per_cu = int(os.environ.get("MACBF_EDGE_WG_PER_CU", per_cu))
    return max(1, min(ch, cu)), max(1, min(che * ctrl_edge_qsplit(total_agents, device), per_cu * cu))


NODE16_RM = 64 * 176 + 128 * 80 + 64 * 144 + 16 * 80    # csrc/node16.h: elements per plane (layout.node_rm16)


def ctrl_node_bwd(pooled, S, G, A, Gn, valid_t, wrm, offs, wvec, act_coef, dP, ego, partial, num_blocks,
                  act_cnt=None, prec=None, init=False, chunk=None, gscale=None, combine=None, stamps=None, _defer=False,
                  wrm16=None):
    """act_cnt: optional 1-element device tensor holding the (all-reduced) action-loss count
    n_act; the action-loss coefficient is then act_coef / max(n_act, 1), read by the kernel (no
    host round trip, no extra launch). init: write the weight-gradient slabs instead of
    accumulating into them (no zero fill needed). stamps: diagnostics only, int64
    (num_blocks, 4, 16) phase clocks of the cooperative 32-agent path (scripts/stamps_node.py)."""
    B, N = G.shape[:2]
    D = dim_of(S)
    W = rec_width(D)
    f16 = _half(wrm, "wrm", prec)
    _rows(pooled, _prow(f16), "pooled", (B, N))
    _records(S, "S", (B, N), W)
    check(G, torch.float32, (B, N, D), "G")
    _rows(A, D, "A", (B, N))
    _records(Gn, "Gn", (B, N), W)
    if valid_t is not None and (valid_t.dtype != torch.uint8 or tuple(valid_t.shape) != (B,)):
        raise NativeError("valid_t must be uint8 (B,)")
    check(wrm, wrm.dtype, None, "wrm")
    if wrm.numel() < _planes(f16) * NODE_RM_ELEMS:
        raise NativeError("node weight images too small")
    check(dP, wrm.dtype, (B, N, _prow(f16)), "dP")
    _same_half(pooled, wrm, "pooled")
    check(ego, torch.float32, (B, N, W), "ego")
    check(partial, torch.float32, (num_blocks, CTRL_NODE_PARTIAL), "partial")
    check(act_cnt, torch.float32, (1,), "act_cnt")
    check(gscale, torch.float32, (1,), "gscale")
    check(stamps, torch.int64, (num_blocks, 8 if wrm16 is not None else 4, 16), "stamps")
    cmb = ()
    if combine is not None:
        # fused BPTT combine: Gn is formed in the kernel from step t+1's records (node_combine's terms)
        c = combine
        K = int(c["K"])
        _records(c["dS"], "combine dS", (B, N), W)
        check(c["ego"], torch.float32, (B, N, W), "combine ego")
        check(c["dEc"], torch.float32, (B, N, K, W), "combine dEc")
        _rows(c["rptr"], c["rptr"].shape[1], "combine rptr", (B,))
        _rows(c["redges"], N * K, "combine redges", (B,))
        _records(c["Gn"], "combine Gn", (B, N), W)
        _records(c["Gout"], "combine Gout", (B, N), W)
        if c["rptr"].dtype != torch.int32 or c["redges"].dtype != torch.int32 or c["rptr"].shape[1] < N + 1:
            raise NativeError("combine rptr / redges must be int32 CSR rows")
        Gn_c = c["Gn"]
        cmb = (ptr(c["dS"]), c["dS"].stride(0) // W, ptr(c["ego"]), ptr(c["dEc"]), ptr(c["rptr"]), c["rptr"].stride(0),
               ptr(c["redges"]), c["redges"].stride(0), ptr(Gn_c), Gn_c.stride(0) // W if Gn_c is not None else 0,
               ptr(c["Gout"]), c["Gout"].stride(0) // W, K)
    args = (ptr(pooled), pooled.stride(0), ptr(S), S.stride(0) // W, ptr(G), ptr(A), A.stride(0) // D,
            ptr(Gn), Gn.stride(0) // W if Gn is not None else 0,
            ptr(valid_t), valid_t.stride(0) if valid_t is not None else 0, B, N,
            ptr(wrm), offs["w1"], offs["w2"], offs["w3"], offs["w4"], ptr(wvec),
            float(act_coef), ptr(act_cnt), float(C.TIME_STEP), float(C.SQRT3), ptr(dP), dP.stride(0),
            ptr(ego), ptr(partial), D, int(num_blocks), f16, int(bool(init)),
            int(chunk or node_bwd_chunk(B * N, S.device)), ptr(gscale), cmb, ptr(stamps))
    if _defer:
        return args
    if wrm16 is not None:
        # 16x16x32 kernel (csrc/node16.h): 128-agent chunks (eight 16-agent waves)
        if args[-4] != 128:
            raise NativeError("16x16x32 node backward: 128-agent chunks only")
        check(wrm16, wrm.dtype, (_planes(f16) * NODE16_RM,), "wrm16")
    _ok(lib().ctrl_node_bwd(*args, ptr(wrm16), stream_handle()), "ctrl_node_bwd")


def ctrl_edge_bwd(S, idx, argmax, dP, wpack, f_ew1f, f_ew2tn, dEc, partial, num_blocks, prec=None, init=False,
                  _defer=False, w16=None, stamps=None):
    """w16 (K = 12): the 16x16x32 fragments (layout.ctrl_edge_packer16) -> the 8-wave 16x16x32 kernel
    (csrc/ctrl16.h); same slabs, same dEc records. stamps (num_blocks, 8, 16) int64 (diagnostics,
    16x16x32 kernel): per wave the shader-clock cycles of each loop phase summed over its tiles
    (slot 15: tiles), scripts/stamps_edge16.py."""
    B, N, K = idx.shape
    D = dim_of(S)
    W = rec_width(D)
    _records(S, "S", (B, N), W)
    if idx.dtype != torch.int32 or idx.stride(2) != 1 or idx.stride(1) != K:
        raise NativeError("idx must be int32 (B,N,K)")
    _rows(argmax, 128, "argmax", (B, N))
    f16 = _half(wpack, "wpack", prec)
    check(dP, wpack.dtype, (B, N, _prow(f16)), "dP")
    if wpack.numel() < (f_ew2tn + 20) * 512 * _planes(f16) or wpack.numel() < (f_ew1f + 2) * 512 * _planes(f16):
        raise NativeError("packed controller weights too small")
    check(dEc, torch.float32, (B, N, K, W), "dEc")
    check(partial, torch.float32, (num_blocks, CTRL_EDGE_PARTIAL), "partial")
    args = (ptr(S), S.stride(0) // W, ptr(idx), idx.stride(0), ptr(argmax), argmax.stride(0),
            ptr(dP), dP.stride(0), B, N, K, ptr(wpack), int(f_ew1f), int(f_ew2tn), ptr(dEc),
            dEc.stride(0) // W if dEc is not None else 0, ptr(partial), D, int(num_blocks),
            f16, ctrl_edge_qsplit(B * N, S.device), int(bool(init)))
    if _defer:
        return args
    if w16 is not None:
        if K != 12:
            raise NativeError("16x16x32 edge backward: K = 12 only")
        check(w16, wpack.dtype, (22 * 512 * _planes(f16),), "w16")
    if stamps is not None:
        if w16 is None:
            raise NativeError("edge backward stamps: 16x16x32 kernel only")
        check(stamps, torch.int64, (num_blocks, 8, 16), "stamps")
    _ok(lib().ctrl_edge_bwd(*args, ptr(w16), ptr(stamps), stream_handle()), "ctrl_edge_bwd")


def ctrl_bwd_step(node: dict, edge: dict, num_blocks: int):
    """One fused BPTT step (csrc/ctrl.hip ctrl_bwd_step_kernel): the node backward of each
    workgroup's 32-agent chunks, then the edge backward of the same agents, in one launch.
    `node` / `edge` are the keyword arguments of ctrl_node_bwd / ctrl_edge_bwd (validated the same
    way); both run on num_blocks workgroups (their slabs need num_blocks rows each)."""
    na = ctrl_node_bwd(**node, num_blocks=num_blocks, chunk=32, _defer=True)
    ea = ctrl_edge_bwd(**edge, num_blocks=num_blocks, _defer=True)
    _ok(lib().ctrl_bwd_step(na, ea, int(num_blocks), na[29], stream_handle()), "ctrl_bwd_step")


BWD_FUSED_DEFAULT = True


def bwd_step_fused(total_agents: int, device) -> bool:
    """Whether the BPTT runs as fused node+edge launches (ctrl_bwd_step): in the cooperative regime
    (32-agent node chunks) with at least half a chunk per CU -- strong-scaling slices. Small scenes
    keep the separate launches: their edge backward splits a chunk over up to 16 workgroups
    (qsplit), which one fused workgroup cannot. MACBF_BWD_FUSED=0/1 forces the choice."""
    env = os.environ.get("MACBF_BWD_FUSED")
    if env is not None:
        return env == "1" and node_bwd_chunk(total_agents, device) == 32
    return BWD_FUSED_DEFAULT and node_bwd_chunk(total_agents, device) == 32 and (total_agents + 31) // 32 >= num_cu(device) // 2


def reduce_multi(jobs):
    """Several reduce_rows in ONE launch: jobs = [(partial (rows, cols), out (cols,), accumulate)]
    (at most 4; the same fixed-order sums as reduce_rows)."""
    if not 1 <= len(jobs) <= 4:
        raise NativeError("reduce_multi takes 1..4 jobs")
    spec = []
    for partial, out, acc in jobs:
        rows, cols = partial.shape
        check(partial, torch.float32, None, "partial")
        check(out, torch.float32, (cols,), "out")
        if cols % 4:
            raise NativeError("cols must be a multiple of 4")
        spec.append((ptr(partial), rows, cols, ptr(out), int(bool(acc))))
    _ok(lib().reduce_multi(spec, stream_handle()), "reduce_multi")


def reduce_rows(partial, out, accumulate=False):
    rows, cols = partial.shape
    check(partial, torch.float32, None, "partial")
    check(out, torch.float32, (cols,), "out")
    if cols % 4:
        raise NativeError("cols must be a multiple of 4")
    _ok(lib().reduce_rows(ptr(partial), rows, cols, ptr(out), int(accumulate), stream_handle()), "reduce_rows")


FX_DIST = 2.0 ** 32           # csrc/args.h: fixed-point scales of the per-env rollout sums
FX_ACT = 2.0 ** 24


def rollout_stats(dist, cnt, safe, act, valid, counts, local, *, N, reset=None):
    """dist/act (T,B), cnt (T,B,2), safe (T+1,B) or None -> valid (T,B) u8, counts[:3] =
    [n_dang, n_safe, n_act] of this rank, local[:3] = [agent-steps, safe agents of s_{t+1},
    action-loss sum]. One launch, deterministic. reset = (dist, cnt, safe, act) full (Tmax, ...)
    buffers whose leading views are the inputs: zeroed after they are read, so the next
    rollout's atomics start from zero without fill kernels."""
    T, B = dist.shape
    reset_T = 0
    if reset is not None:
        zd, zc, zs, za = reset
        reset_T = zd.shape[0]
        check(zd, torch.int64, (reset_T, B), "reset dist")
        check(zc, torch.float32, (reset_T, B, 2), "reset cnt")
        check(zs, torch.float32, (reset_T + 1, B), "reset safe")
        check(za, torch.int64, (reset_T, B), "reset act")
        if (ptr(zd), ptr(zc), ptr(zs), ptr(za)) != (ptr(dist), ptr(cnt), ptr(safe), ptr(act)) or T > reset_T:
            raise NativeError("reset buffers must start at the inputs")
    check(dist, torch.int64, (T, B), "dist")
    check(cnt, torch.float32, (T, B, 2), "cnt")
    check(safe, torch.float32, (T + 1, B), "safe")
    check(act, torch.int64, (T, B), "act")
    check(valid, torch.uint8, (T, B), "valid")
    check(counts, torch.float32, None, "counts")
    check(local, torch.float32, None, "local")
    if counts.numel() < 3 or local.numel() < 3:
        raise NativeError("counts / local need 3 slots")
    _ok(lib().rollout_stats(ptr(dist), ptr(cnt), ptr(safe), ptr(act), T, B, int(N), float(C.DIST_MIN_CHECK),
                            ptr(valid), ptr(counts), ptr(local), int(reset_T), stream_handle()), "rollout_stats")


def adam_multi(param, grad, m, v, groups, lr, b1, b2, eps, wd, ok=None):
    """Fused Adam over several ranges in ONE launch: groups = [(lo, hi, step_dev)] (at most 4; each
    step_dev a 1-element device int32 counter, step = *step_dev + 1); ok as in adam."""
    for t, n in ((param, "param"), (grad, "grad"), (m, "m"), (v, "v")):
        check(t, torch.float32, (param.numel(),), n)
    check(ok, torch.int32, None, "ok")
    if not 1 <= len(groups) <= 4:
        raise NativeError("adam_multi takes 1..4 groups")
    spec = []
    for lo, hi, sd in groups:
        if not (0 <= lo <= hi <= param.numel()):
            raise NativeError("bad Adam range")
        check(sd, torch.int32, (1,), "step_dev")
        spec.append((int(lo), int(hi), ptr(sd)))
    _ok(lib().adam_multi(ptr(param), ptr(grad), ptr(m), ptr(v), spec, float(b1), float(b2), float(eps), float(wd),
                         ptr(ok), float(lr), stream_handle()), "adam_multi")


def adam(param, grad, m, v, lo, hi, lr, b1, b2, eps, wd, step, ok=None, step_dev=None):
    """Fused Adam over param[lo:hi]. step: host step count (bias corrections), or step_dev: a
    1-element device int32 counter (step = *step_dev + 1, read by the kernel); ok: optional
    device int32 guard flag (0 -> the kernel leaves everything untouched)."""
    for t, n in ((param, "param"), (grad, "grad"), (m, "m"), (v, "v")):
        check(t, torch.float32, (param.numel(),), n)
    if not (0 <= lo <= hi <= param.numel()):
        raise NativeError("bad Adam range")
    check(ok, torch.int32, None, "ok")
    check(step_dev, torch.int32, None, "step_dev")
    bc1 = 1.0 - b1 ** max(step, 1)
    bc2 = 1.0 - b2 ** max(step, 1)
    _ok(lib().adam(ptr(param), ptr(grad), ptr(m), ptr(v), int(lo), int(hi), float(b1), float(b2), float(eps),
                   float(wd), float(lr / bc1), float(bc2 ** 0.5), ptr(ok), ptr(step_dev), float(lr),
                   stream_handle()), "adam")


def pack_gather(src, idx16, out16, idx32, out32, commit=None):
    """out16[i] = h16(src'[idx16[i]]), out32[j] = src'[idx32[j]] with src' = [src, 0, 1]: all
    packed weight buffers of both networks in one launch. commit: step_commit_args(...) of the
    optimizer step just enqueued -- its commit then runs in this launch (one launch fewer)."""
    check(src, torch.float32, None, "src")
    check(idx16, torch.int32, None, "idx16")
    check(idx32, torch.int32, None, "idx32")
    check(out32, torch.float32, (idx32.numel(),), "out32")
    if out16.dtype not in HALF_DTYPES or not out16.is_contiguous() or out16.numel() != idx16.numel():
        raise NativeError("out16 must be a contiguous bf16/fp16 buffer matching idx16")
    n = src.numel()    # index range (<= n + 1) is validated once by ops.weights.PackedWeights
    _ok(lib().pack_gather(ptr(src), n, ptr(idx16), idx16.numel(), ptr(out16), int(out16.dtype == torch.float16),
                          ptr(idx32), idx32.numel(), ptr(out32), commit, stream_handle()), "pack_gather")


def grad_assemble(red, ptr_, src, grad, scale=1.0, gscale=None, ok=None, stats=None):
    """grad[p] = scale * sum(red[src[ptr[p]:ptr[p+1]]]) (/ *gscale: the device loss scale) for
    every flat parameter p (one launch, fixed order). ptr (n+1,) / src int32 from a host-built CSR
    (validated by the caller). In the same launch (single-process runs): ok (int32 flag) <- 0 if an
    assembled element is not finite (grad_check's test); stats = (sums, counts, local, row): the
    iteration's statistics row (stats_pack's work)."""
    n = grad.numel()
    check(red, torch.float32, None, "red")
    check(ptr_, torch.int32, (n + 1,), "ptr")
    check(src, torch.int32, None, "src")
    check(grad, torch.float32, None, "grad")
    check(gscale, torch.float32, (1,), "gscale")
    check(ok, torch.int32, (1,), "ok")
    sums = counts = local = row = None
    if stats is not None:
        sums, counts, local, row = stats
        _stats_args(sums, counts, local, row)
    _ok(lib().grad_assemble(ptr(red), ptr(ptr_), ptr(src), n, float(scale), ptr(gscale), ptr(grad), ptr(ok),
                            ptr(sums), ptr(counts), ptr(local), ptr(row), stream_handle()), "grad_assemble")


def _stats_args(sums, counts, local, row):
    check(sums, torch.float32, None, "sums")
    check(counts, torch.float32, None, "counts")
    check(local, torch.float32, None, "local")
    if sums.numel() < 10 or counts.numel() < 3 or local.numel() < 3:
        raise NativeError("stats_pack needs 10 sums, 3 counts, 3 local values")
    if row.dtype != torch.float32 or row.numel() < 18 or not row.is_contiguous():
        raise NativeError("row must be a contiguous float32 row of >= 18")


def grad_check(g, ok):
    """ok (int32, 1 between steps: step_commit resets it) <- 0 if any element of g is not finite.
    No host sync."""
    check(g, torch.float32, None, "g")
    check(ok, torch.int32, None, "ok")
    _ok(lib().grad_check(ptr(g), g.numel(), ptr(ok), stream_handle()), "grad_check")


def _check_stats_src(stats_src, stats_row):
    if stats_src is None:
        return
    if stats_row is None:
        raise NativeError("stats_src needs stats_row")
    if stats_src.dtype != torch.float32 or stats_src.numel() < 16 or not stats_src.is_contiguous():
        raise NativeError("stats_src must be a contiguous float32 row of >= 16")


def step_commit_args(ok, steps, mask, skipped, *, gscale=None, good=None, growth=1000, max_scale=2.0 ** 24,
                     stats_row=None, stats_src=None):
    """Validated step_commit arguments as the tuple pack_gather(commit=...) takes; stats_src: the
    commit first copies stats_row[0:16] from it (the graph-replayed backward's fixed row)."""
    _check_stats_src(stats_src, stats_row)
    check(ok, torch.int32, (1,), "ok")
    check(steps, torch.int32, None, "steps")
    check(skipped, torch.int32, (1,), "skipped")
    check(gscale, torch.float32, (1,), "gscale")
    check(good, torch.int32, (1,), "good")
    if (gscale is None) != (good is None):
        raise NativeError("gscale and good go together")
    if stats_row is not None and (stats_row.dtype != torch.float32 or stats_row.numel() < 18
                                  or not stats_row.is_contiguous()):
        raise NativeError("stats_row must be a contiguous float32 row of >= 18")
    return (ptr(ok), ptr(steps), int(mask), steps.numel(), ptr(skipped), ptr(gscale), ptr(good), int(growth),
            float(max_scale), ptr(stats_row), ptr(stats_src))


def step_commit_raw(args):
    """step_commit from a step_commit_args tuple (its own launch)."""
    _ok(lib().step_commit(*args, stream_handle()), "step_commit")


def step_commit(ok, steps, mask, skipped, *, gscale=None, good=None, growth=1000, max_scale=2.0 ** 24,
                stats_row=None, stats_src=None):
    """End of an optimizer step on the device: steps[g] += 1 for the groups in mask if *ok, else
    skipped += 1; fp16 (gscale, good): the dynamic loss scale halves on a skipped step and doubles
    after `growth` finite ones; stats_row[16:18] = [skipped, loss scale]; *ok reset to 1."""
    check(ok, torch.int32, (1,), "ok")
    check(steps, torch.int32, None, "steps")
    check(skipped, torch.int32, (1,), "skipped")
    check(gscale, torch.float32, (1,), "gscale")
    check(good, torch.int32, (1,), "good")
    if (gscale is None) != (good is None):
        raise NativeError("gscale and good go together")
    if stats_row is not None and (stats_row.dtype != torch.float32 or stats_row.numel() < 18
                                  or not stats_row.is_contiguous()):
        raise NativeError("stats_row must be a contiguous float32 row of >= 18")
    _check_stats_src(stats_src, stats_row)
    _ok(lib().step_commit(ptr(ok), ptr(steps), int(mask), steps.numel(), ptr(skipped), ptr(gscale), ptr(good),
                          int(growth), float(max_scale), ptr(stats_row), ptr(stats_src), stream_handle()), "step_commit")


def stats_pack(sums, counts, local, row):
    """row[:18] = [sums (10) | counts (3) | local (3) | 0 | 1] (one launch; utils.metrics.StepStats)."""
    check(sums, torch.float32, None, "sums")
    check(counts, torch.float32, None, "counts")
    check(local, torch.float32, None, "local")
    if sums.numel() < 10 or counts.numel() < 3 or local.numel() < 3:
        raise NativeError("stats_pack needs 10 sums, 3 counts, 3 local values")
    if row.dtype != torch.float32 or row.numel() < 18 or not row.is_contiguous():
        raise NativeError("row must be a contiguous float32 row of >= 18")
    _ok(lib().stats_pack(ptr(sums), ptr(counts), ptr(local), ptr(row), stream_handle()), "stats_pack")
