"""Does training make the policy safer? (reference ``config.py:17-20``,
``train.py:73-76``.)

Three sub-commands, all writing JSON under ``--out``:

    train  --name NAME [--agents 1024 --envs 64 --steps 6000 --alternate_every 10 --no_bptt]
           trains from random init with the reference CLI semantics, logs JSONL, saves NAME.pt
    eval   --models none,A.pt,B.pt [--agents 1024 --episodes 10]
           evaluate.py metrics with test-time refinement on and off, plus the share of unsafe
           agent-steps whose flagged pair is one of the agent's top-K neighbours
    grads  --models none,A.pt [--agents 1024 --envs 4]
           per-loss-term gradient norms reaching the controller (pure-torch oracle, autograd
           through the BPTT rollout), split into the parts through the CBF terms and the action term

    python scripts/safety_study.py train --name headline --steps 6000 --out gpurun_out/eval
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _out(args, name):
    os.makedirs(args.out, exist_ok=True)
    return os.path.join(args.out, name)


def cmd_train(args):
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine import Trainer
    cfg = C.TrainConfig(num_agents=args.agents, num_envs=args.envs, seed=args.seed, device="auto",
                        dtype=args.dtype, bptt=not args.no_bptt, alternate_every=args.alternate_every,
                        model_path=_out(args, args.name + ".pt"), log_path=_out(args, args.name + ".jsonl"),
                        display_steps=args.display, save_steps=10 ** 9, train_steps=args.steps)
    tr = Trainer(cfg)
    t0 = time.time()
    chunk = max(args.display, 1)
    while tr.step_count < args.steps:
        tr.fit(steps=min(chunk, args.steps - tr.step_count))
        print(f"[{args.name}] step {tr.step_count} {time.time() - t0:.0f}s", flush=True)
    tr.save(cfg.model_path)
    torch.cuda.synchronize() if torch.cuda.is_available() else None


def _load(path, dev):
    import torch
    from macbf_gnn_amd.models import CBF, Controller
    from macbf_gnn_amd.utils import ckpt
    torch.manual_seed(0)
    ctrl, cbf = Controller(4).to(dev), CBF(4).to(dev)
    if path and path != "none":
        ckpt.load_models(path, ctrl, cbf)
    return ctrl, cbf


def cmd_eval(args):
    import torch
    from macbf_gnn_amd.engine.trainer import resolve_device
    from macbf_gnn_amd.evaluate import EvalConfig, evaluate
    dev = resolve_device("auto")
    rows = []
    for m in args.models.split(","):
        for refine in ((False, "actions"), (True, "actions"), (True, "gains")):
            refine, space = refine
            ctrl, cbf = _load(m, dev)
            cfg = EvalConfig(num_agents=args.agents, num_envs=1, episodes=args.episodes, refine=refine,
                             seed=args.seed, diagnose=True, refine_space=space)
            t0 = time.time()
            r = evaluate(ctrl, cbf, cfg, device=dev)
            r.update(model=os.path.basename(m), refine=refine and space, agents=args.agents, episodes=args.episodes,
                     seconds=round(time.time() - t0, 1))
            rows.append(r)
            print(json.dumps(r), flush=True)
            with open(_out(args, args.tag + ".json"), "w") as f:
                json.dump(rows, f, indent=1)


def cmd_grads(args):
    """Gradient of each loss term w.r.t. the controller parameters (autograd through the oracle's
    BPTT rollout, as reference train.py:58-103 with the defect fixes of SURVEY 2.4)."""
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd import oracle
    from macbf_gnn_amd.engine.trainer import resolve_device
    from macbf_gnn_amd.ops import scenario
    dev = resolve_device("auto")
    rows = []
    terms = ("loss_dang", "loss_safe", "loss_dang_deriv", "loss_safe_deriv", "loss_action")
    for m in args.models.split(","):
        ctrl, cbf = _load(m, dev)
        cp, bp = ctrl.params_dict(), cbf.params_dict()
        acc = {t: 0.0 for t in terms}
        acc_bptt = {t: 0.0 for t in terms}
        for it in range(args.iters):
            if dev.type == "cuda":
                s0, g, _ = scenario.generate(args.envs, args.agents, seed=args.seed + 17, iteration=it, rank=0, device=dev)
            else:
                from macbf_gnn_amd import env as E
                s0, g = E.generate_batch(args.envs, args.agents, seed=args.seed * 31 + it)
            for bptt in (True, False):
                traj = oracle.rollout(cp, s0, g, bptt=bptt)
                losses, _, _ = oracle.train_losses(cp, bp, traj, g)
                w = dict(zip(terms, C.LOSS_WEIGHTS))
                for t in terms:
                    gr = torch.autograd.grad(C.LOSS_SCALE * w[t] * losses[t], list(cp.values()), retain_graph=True,
                                             allow_unused=True)
                    n = sum(float((x.float() ** 2).sum()) for x in gr if x is not None) ** 0.5
                    (acc_bptt if bptt else acc)[t] += float(n) / args.iters
        r = {"model": os.path.basename(m), "agents": args.agents, "envs": args.envs, "iters": args.iters,
             "ctrl_grad_norm_bptt": acc_bptt, "ctrl_grad_norm_no_bptt": acc}
        rows.append(r)
        print(json.dumps(r), flush=True)
        with open(_out(args, args.tag + ".json"), "w") as f:
            json.dump(rows, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["train", "eval", "grads"])
    ap.add_argument("--out", default="gpurun_out/eval")
    ap.add_argument("--name", default="headline")
    ap.add_argument("--tag", default="eval")
    ap.add_argument("--models", default="none")
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--episodes", type=int, default=10)
    ap.add_argument("--display", type=int, default=250)
    ap.add_argument("--alternate_every", type=int, default=0)
    ap.add_argument("--no_bptt", action="store_true")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    {"train": cmd_train, "eval": cmd_eval, "grads": cmd_grads}[args.cmd](args)


if __name__ == "__main__":
    main()
