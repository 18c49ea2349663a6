"""Data parallelism of the HIP engine on one MI355X: two ranks share the card over the gloo
backend (RCCL cannot place two ranks on one GPU; the collectives, the async count all-reduce
and the global pooled normalisation are the same code path as with RCCL).

* the all-reduced DP gradient equals the single-process gradient on the concatenated env
  batch (per-env early stop: the ranks' horizons differ);
* both ranks hold the bit-identical reduced gradient.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E

pytestmark = pytest.mark.gpu

BTOT, N, T = 4, 32, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(B):
    return C.TrainConfig(num_agents=N, num_envs=B, inner_loops=T, device="hip", seed=5, early_stop=True)


def _worker(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dp = DP(backend="gloo", device=dev)
    s_all, g_all = E.generate_batch(BTOT, N, seed=21)
    B = BTOT // world
    tr = Trainer(_cfg(B), device=dev, dp=dp)
    sl = slice(rank * B, (rank + 1) * B)
    tr.engine.step(s_all[sl].to(dev), g_all[sl].to(dev))
    tr.reduce_grad()
    torch.cuda.synchronize()
    torch.save(tr.fp.grad.cpu(), os.path.join(outdir, f"grad{rank}.pt"))
    dp.shutdown()


@pytest.mark.timeout(300)
def test_hip_dp_grad_equals_single_process(tmp_path):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    g0 = torch.load(tmp_path / "grad0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "grad1.pt", weights_only=True)
    assert torch.equal(g0, g1)
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    dev = torch.device("cuda", 0)
    s_all, g_all = E.generate_batch(BTOT, N, seed=21)
    tr = Trainer(_cfg(BTOT), device=dev, dp=DP(device=dev))
    tr.engine.step(s_all.to(dev), g_all.to(dev))
    ref = tr.fp.grad.cpu()
    assert torch.isfinite(ref).all() and ref.abs().sum() > 0
    # same per-edge arithmetic, different slab partitions: fp32 summation-order differences only
    torch.testing.assert_close(g0, ref, rtol=2e-3, atol=1e-6)


def _forced_worker(rank, outdir, steps):
    """One process, world size 1, MACBF_DP_FORCE_PG=1: the process group is RCCL (nccl) and every
    collective (parameter broadcast, async count all-reduce + wait, gradient all-reduce,
    barrier(device_ids), max_scalar) runs through it."""
    os.environ.update({"MACBF_DP_FORCE_PG": "1", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()),
                       "RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    import torch.distributed as dist
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dp = DP(device=dev)
    assert dist.is_initialized() and dist.get_backend() == "nccl" and dp.enabled
    tr = Trainer(_cfg(BTOT), device=dev, dp=dp)
    for _ in range(steps):
        tr.train_step()
    dp.barrier()
    t = dp.max_scalar(1.5)
    assert t == 1.5
    torch.cuda.synchronize()
    torch.save({"flat": tr.fp.flat.cpu(), "backend": dist.get_backend()}, os.path.join(outdir, "forced.pt"))
    dp.shutdown()


@pytest.mark.timeout(300)
def test_forced_rccl_group_world1_bit_identical(tmp_path):
    """RCCL path at world size 1: parameters after 3 training steps with every
    collective issued through an nccl process group == the no-group run, bit for bit."""
    steps = 3
    mp.start_processes(_forced_worker, args=(str(tmp_path), steps), nprocs=1, join=True, start_method="spawn")
    got = torch.load(tmp_path / "forced.pt", weights_only=True)
    assert got["backend"] == "nccl"
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    dev = torch.device("cuda", 0)
    tr = Trainer(_cfg(BTOT), device=dev, dp=DP(device=dev))
    for _ in range(steps):
        tr.train_step()
    torch.cuda.synchronize()
    assert torch.equal(got["flat"], tr.fp.flat.cpu())
