"""Data parallelism without a cluster: gloo on CPU, world_size 2, 4 and 8.

* the DP all-reduced gradient equals the single-process gradient on the concatenated env
  batch (global pooled loss normalisation);
* parameters stay bit-identical across ranks after k optimizer steps;
* a checkpoint written by a DP run resumes in a run of a different width.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from macbf_gnn_amd import config as C
from macbf_gnn_amd import env as E


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


NE = 8        # envs of the global batch (every world size here divides it)


def _cfg(B, steps=1):
    return C.TrainConfig(num_agents=10, num_envs=B, inner_loops=6, device="cpu", seed=3,
                         early_stop=True, train_steps=steps)


def _worker(rank, world, port, outdir, mode):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    torch.set_num_threads(1)
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    dp = DP(device=torch.device("cpu"))
    s_all, g_all = E.generate_batch(NE, 10, seed=11)
    B = NE // world
    tr = Trainer(_cfg(B), device=torch.device("cpu"), dp=dp)
    sl = slice(rank * B, (rank + 1) * B)
    if mode == "ckpt":
        for it in range(4):
            if it == 2:
                tr.save(os.path.join(outdir, "ck.pt"))
            s, g = E.generate_batch(NE, 10, seed=200 + it)
            tr.train_step(s[sl], g[sl])
        torch.save(tr.fp.flat.clone(), os.path.join(outdir, f"flat{rank}.pt"))
    elif mode == "grad":
        tr.engine.step(s_all[sl], g_all[sl])
        tr.reduce_grad()
        torch.save(tr.fp.grad.clone(), os.path.join(outdir, f"grad{rank}.pt"))
    else:
        for it in range(3):
            s, g = E.generate_batch(NE, 10, seed=100 + it)
            tr.train_step(s[sl], g[sl])
        torch.save(tr.fp.flat.clone(), os.path.join(outdir, f"flat{rank}.pt"))
    dp.shutdown()


def _run(world, outdir, mode):
    mp.start_processes(_worker, args=(world, _free_port(), str(outdir), mode), nprocs=world, join=True,
                       start_method="spawn")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_grad_equals_single_process(tmp_path, world):
    _run(world, tmp_path, "grad")
    g0 = torch.load(tmp_path / "grad0.pt", weights_only=True)
    for r in range(1, world):
        assert torch.equal(g0, torch.load(tmp_path / f"grad{r}.pt", weights_only=True))
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    s_all, g_all = E.generate_batch(NE, 10, seed=11)
    tr = Trainer(_cfg(NE), device=torch.device("cpu"), dp=DP(device=torch.device("cpu")))
    tr.engine.step(s_all, g_all)
    torch.testing.assert_close(g0, tr.fp.grad, rtol=2e-4, atol=1e-7)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 8])
def test_dp_params_identical_across_ranks(tmp_path, world):
    _run(world, tmp_path, "train")
    f0 = torch.load(tmp_path / "flat0.pt", weights_only=True)
    for r in range(1, world):
        assert torch.equal(f0, torch.load(tmp_path / f"flat{r}.pt", weights_only=True))


@pytest.mark.timeout(600)
def test_dp_checkpoint_resumes_at_other_width(tmp_path):
    """DP-2 run saves after 2 of 4 iterations; a 1-process run resumes from that checkpoint on
    the full env batch and must land on the DP-2 run's final parameters."""
    _run(2, tmp_path, "ckpt")
    f0 = torch.load(tmp_path / "flat0.pt", weights_only=True)
    assert torch.equal(f0, torch.load(tmp_path / "flat1.pt", weights_only=True))
    from macbf_gnn_amd.engine import Trainer
    from macbf_gnn_amd.parallel import DP
    from macbf_gnn_amd.utils import ckpt
    tr = Trainer(C.TrainConfig(num_agents=10, num_envs=NE, inner_loops=6, device="cpu", seed=99,
                               early_stop=True, train_steps=1),
                 device=torch.device("cpu"), dp=DP(device=torch.device("cpu")))
    ckpt.load(tr, str(tmp_path / "ck.pt"))
    assert tr.step_count == 2
    for it in range(2, 4):
        s, g = E.generate_batch(NE, 10, seed=200 + it)
        tr.train_step(s, g)
    torch.testing.assert_close(tr.fp.flat, f0, rtol=1e-4, atol=2e-6)
