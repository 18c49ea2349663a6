"""Evaluate a trained controller + CBF with test-time action refinement.

    python evaluate.py --num_agents 32 [--model_path ckpt.pt] [--num_envs 4] [--episodes 10]
                       [--max_steps 50] [--no_refine] [--refine_space actions|gains] [--diagnose]
                       [--device auto|cpu|hip] [--gpu 0]

Prints one JSON line: safety rate, reaching rate, mean final goal distance, refinement
iterations. Without --model_path the networks are random-initialised (plumbing check).
--refine_space gains refines only the PD gains of the controller law (what the trained policy
class can express); --diagnose adds the share of unsafe pairs that are top-K neighbours.
"""
from __future__ import annotations

import argparse
import json
import os


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--num_agents", type=int, required=True)
    ap.add_argument("--model_path", type=str, default=None)
    ap.add_argument("--gpu", type=str, default=None)
    ap.add_argument("--num_envs", type=int, default=1)
    ap.add_argument("--episodes", type=int, default=None)
    ap.add_argument("--max_steps", type=int, default=None)
    ap.add_argument("--no_refine", action="store_true")
    ap.add_argument("--refine_loops", type=int, default=None)
    ap.add_argument("--refine_lr", type=float, default=None)
    ap.add_argument("--refine_space", choices=["actions", "gains"], default="actions")
    ap.add_argument("--diagnose", action="store_true")
    ap.add_argument("--device", type=str, default="auto")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    if args.gpu is not None:
        os.environ.setdefault("HIP_VISIBLE_DEVICES", args.gpu)
    import torch
    from macbf_gnn_amd import config as C
    from macbf_gnn_amd.engine.trainer import resolve_device
    from macbf_gnn_amd.evaluate import EvalConfig, evaluate
    from macbf_gnn_amd.models import CBF, Controller
    from macbf_gnn_amd.utils import ckpt

    dev = resolve_device(args.device)
    torch.manual_seed(args.seed)
    ctrl, cbf = Controller(4).to(dev), CBF(4).to(dev)
    if args.model_path:
        ckpt.load_models(args.model_path, ctrl, cbf)
    cfg = EvalConfig(num_agents=args.num_agents, num_envs=args.num_envs, seed=args.seed, refine=not args.no_refine,
                     refine_space=args.refine_space, diagnose=args.diagnose)
    if args.episodes is not None:
        cfg.episodes = args.episodes
    if args.max_steps is not None:
        cfg.max_steps = args.max_steps
    if args.refine_loops is not None:
        cfg.refine_loops = args.refine_loops
    if args.refine_lr is not None:
        cfg.refine_lr = args.refine_lr
    out = evaluate(ctrl, cbf, cfg, device=dev)
    out.update({"num_agents": args.num_agents, "num_envs": args.num_envs, "episodes": cfg.episodes,
                "refine": cfg.refine, "device": str(dev)})
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
