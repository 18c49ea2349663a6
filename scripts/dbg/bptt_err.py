"""Debug: per-step decomposition of the bf16 BPTT full-step gradient error (N=32, B=2)."""
import sys
import torch
sys.path.insert(0, "tests")
from macbf_gnn_amd import config as C, oracle as O
from macbf_gnn_amd.engine import Trainer
from macbf_gnn_amd.engine.oracle_engine import OracleEngine
from macbf_gnn_amd.parallel import DP

DEV = torch.device("cuda")
for prec in ("bf16", "fp32"):
    for T in (1, 2, 3, 5, 10):
        for cbf_on in (True,):
            cfg = C.TrainConfig(num_agents=32, num_envs=2, inner_loops=T, early_stop=False, seed=0, device="hip",
                                dtype=prec, bptt=True)
            tr = Trainer(cfg, device=DEV, dp=DP(device=DEV))
            if prec == "bf16":
                with torch.no_grad():
                    tr.fp.flat.copy_(tr.fp.flat.bfloat16().float())
                tr.engine.after_update()
            s0, g, _ = tr.sample()
            st = tr.engine.step(s0, g)
            gh = tr.fp.grad.clone()
            with O.emulate_bf16(prec == "bf16"):
                OracleEngine(tr).step(s0, g, forced=tr.engine.trajectory(int(float(st["T"]))))
            gr = tr.fp.grad.clone()
            a_, b_ = tr.fp.ranges["controller"]
            c_, d_ = tr.fp.ranges["cbf"]
            e1 = ((gh[a_:b_] - gr[a_:b_]).norm() / gr[a_:b_].norm()).item()
            e2 = ((gh[c_:d_] - gr[c_:d_]).norm() / gr[c_:d_].norm()).item()
            print(f"{prec} T={T} ctrl {e1:.3e} (|g| {gr[a_:b_].norm().item():.3e})  cbf {e2:.3e}  loss {float(st['loss_total']):.5f}", flush=True)
