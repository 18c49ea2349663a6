"""Loader and validated launch wrappers for the gfx950 extension ``macbf_gnn_amd._C``.

The extension is built in-tree by ``csrc/build.py`` (``__graft_entry__.build()``). On a HIP
device there is no fallback: if the extension is missing or was built for another arch,
``lib()`` raises. Every wrapper checks device/dtype/contiguity/shape on the host before
passing raw device addresses to the kernels (an out-of-bounds kernel can take the GPU down,
so shapes are never trusted implicitly).
"""
from __future__ import annotations

import functools
import os

import torch

from .. import config as C

_LIB = None


class NativeError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        try:
            from .. import _C  # noqa: F401  (in-tree .so)
        except ImportError as e:  # pragma: no cover - exercised on GPU boxes only
            raise NativeError(
                "native extension macbf_gnn_amd._C is not built; run `python csrc/build.py` "
                f"(or __graft_entry__.build()) first: {e}") from e
        _LIB = _C
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except NativeError:
        return False


def stream_handle(device=None) -> int:
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


def _ok(rc, what):
    if rc != 0:
        raise NativeError(f"{what} launch failed: {rc} ({lib().err_str(rc) if rc > 0 else 'bad args'})")


# ----------------------------------------------------------------------------- kernels
def scan(S, idx, dang, cnt, safe, *, K, do_knn=True, do_safety=True):
    """K1 over one timestep. S: (B, N, 4) view with env stride (may be a slice of a (B,T+1,N,4)
    buffer); idx/dang: (B, N, K) views; cnt: (B, 2) view; safe: (B,) view."""
    B, N = S.shape[0], S.shape[1]
    if S.dtype != torch.float32 or S.stride(2) != 1 or S.stride(1) != 4:
        raise NativeError("S must be float32 with contiguous (N,4) rows")
    if K < 1 or K > C.MAX_TOP_K or K > N:
        raise NativeError(f"bad K={K} for N={N}")
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
    rc = lib().scan(ptr(S), S.stride(0) // 4, B, N, K, ptr(idx) if do_knn else 0,
                    idx.stride(0) if do_knn else 0, ptr(dang) if do_knn else 0,
                    ptr(cnt) if do_knn else 0, cnt.stride(0) if (do_knn and cnt is not None) else 0,
                    ptr(safe) if do_safety else 0, safe.stride(0) if (do_safety and safe is not None) else 0,
                    float(C.DIST_MIN_THRES * C.DIST_MIN_THRES), float(C.TIME_TO_COLLISION),
                    float(C.DIST_MIN_CHECK * C.DIST_MIN_CHECK), float(C.TIME_TO_COLLISION_CHECK),
                    int(do_knn), int(do_safety), stream_handle())
    _ok(rc, "scan")


def scenario(S, G, *, seed, L, r=C.DIST_MIN_THRES, spread=C.GOAL_SPREAD, max_rounds=256, status=None):
    B, N = S.shape[0], S.shape[1]
    check(S, torch.float32, (B, N, 4), "S")
    check(G, torch.float32, (B, N, 2), "G")
    check(status, torch.int32, (B,), "status")
    if N * 25 > 160 * 1024 - 64:
        raise NativeError(f"scenario sampler supports N <= 6500 per env (got {N})")
    rc = lib().scenario(ptr(S), ptr(G), B, N, float(L), float(r), float(spread),
                        int(seed) & 0xFFFFFFFFFFFFFFFF, int(max_rounds), ptr(status), stream_handle())
    _ok(rc, "scenario")


def ctrl_fwd(S, G, idx, wpack, f_edge, f_node, wvec, A, Sn, dist_sum, act_sum, noise=None):
    """Fused controller step. S (B,N,4) view (row-contiguous), G (B,N,2) contiguous,
    idx (B,N,K) view, A (B,N,2) view, Sn (B,N,4) view, dist_sum/act_sum (B,) views."""
    B, N = S.shape[0], S.shape[1]
    K = idx.shape[2]
    if K < 1 or K > C.MAX_TOP_K:
        raise NativeError("K out of range")
    for t, n, last in ((S, "S", 4), (Sn, "Sn", 4), (A, "A", 2)):
        if t is not None and (t.dtype != torch.float32 or t.shape[:2] != (B, N) or t.shape[2] != last
                              or t.stride(2) != 1 or t.stride(1) != last):
            raise NativeError(f"{n} must be float32 (B,N,{last}) with contiguous rows")
    check(G, torch.float32, (B, N, 2), "G")
    if idx.dtype != torch.int32 or idx.stride(2) != 1 or idx.stride(1) != K or idx.shape[:2] != (B, N):
        raise NativeError("idx must be int32 (B,N,K)")
    check(wpack, torch.bfloat16, None, "wpack")
    check(wvec, torch.float32, None, "wvec")
    if wvec.numel() < 352 or wpack.numel() < (f_node + 54) * 512:
        raise NativeError("packed controller weights too small")
    for t, n in ((dist_sum, "dist_sum"), (act_sum, "act_sum")):
        if t is not None and (t.dtype != torch.float32 or tuple(t.shape) != (B,)):
            raise NativeError(f"{n} must be float32 (B,)")
    if noise is not None and (noise.dtype != torch.float32 or noise.shape[:2] != (B, N) or noise.stride(1) != 2):
        raise NativeError("noise must be float32 (B,N,2)")
    rc = lib().ctrl_fwd(ptr(S), S.stride(0) // 4, ptr(G), ptr(idx), idx.stride(0), B, N, K,
                        ptr(wpack), int(f_edge), int(f_node), ptr(wvec),
                        ptr(A), A.stride(0) // 2 if A is not None else 0,
                        ptr(Sn), Sn.stride(0) // 4 if Sn is not None else 0,
                        ptr(dist_sum), dist_sum.stride(0) if dist_sum is not None else 0,
                        ptr(act_sum), act_sum.stride(0) if act_sum is not None else 0,
                        ptr(noise), noise.stride(0) // 2 if noise is not None else 0,
                        float(C.TIME_STEP), float(C.OBS_RADIUS), float(C.SQRT3),
                        num_cu(S.device), stream_handle())
    _ok(rc, "ctrl_fwd")


LOSS_CONSTS = (C.LOSS_EPS_DANG, C.TIME_STEP * C.ALPHA_CBF, C.LOSS_WEIGHTS[0], C.LOSS_WEIGHTS[1],
               C.LOSS_WEIGHTS[2], C.LOSS_WEIGHTS[3], C.LOSS_SCALE)
CBF_FWD_WAVES = 4


def cbf_fwd_grid(E: int, device) -> int:
    tiles = (E + 31) // 32
    return max(1, min((tiles + CBF_FWD_WAVES - 1) // CBF_FWD_WAVES, num_cu(device) * 2))


def cbf_fwd(S, idx, wpack, f_fwd, wvec, *, dang=None, valid=None, two=True, h_out=None, hn_out=None,
            dh_out=None, counts=None, partial=None, num_blocks=None):
    """S: (B, T', N, 4) contiguous with T' >= T + two; idx (B,T,N,K) int32 contiguous."""
    B, T, N, K = idx.shape
    check(idx, torch.int32, None, "idx")
    if S.dtype != torch.float32 or not S.is_contiguous() or S.shape[0] != B or S.shape[2] != N \
            or S.shape[1] < T + (1 if two else 0):
        raise NativeError("S must be contiguous float32 (B, >=T+1, N, 4)")
    E = B * T * N * K
    check(dang, torch.uint8, (B, T, N, K), "dang")
    check(valid, torch.uint8, (B, T), "valid")
    check(h_out, torch.float32, (B, T, N, K), "h_out")
    check(hn_out, torch.float32, (B, T, N, K), "hn_out")
    check(dh_out, torch.float32, (2, B, T, N, K), "dh_out")
    if dh_out is not None:
        check(counts, torch.float32, None, "counts")
    check(wpack, torch.bfloat16, None, "wpack")
    check(wvec, torch.float32, None, "wvec")
    nb = num_blocks or cbf_fwd_grid(E, S.device)
    check(partial, torch.float32, (nb, 10), "partial")
    rc = lib().cbf_fwd(ptr(S), S.stride(0) // 4, S.stride(1) // 4, ptr(idx), ptr(dang), ptr(valid),
                       B, T, N, K, int(two), ptr(wpack), int(f_fwd), ptr(wvec), ptr(h_out), ptr(hn_out),
                       ptr(dh_out), ptr(counts), ptr(partial), LOSS_CONSTS,
                       float(C.OBS_RADIUS), float(C.DIST_MIN_THRES), float(C.CBF_DIST_EPS), nb, stream_handle())
    _ok(rc, "cbf_fwd")
    return nb
