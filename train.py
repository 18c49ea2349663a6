"""Training entry point, reference-compatible CLI (``/root/reference/train.py:17-23``).

    python train.py --num_agents N [--model_path P] [--gpu G]

plus the knobs of SURVEY 5.6. Data parallel: launch one process per GPU with
``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...``;
each rank trains ``--num_envs`` environments and gradients are all-reduced over RCCL.
"""
from __future__ import annotations

import argparse
import os


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="MACBF-GNN trainer (MI355X-native)")
    p.add_argument("--num_agents", type=int, required=True)
    p.add_argument("--model_path", type=str, default=None,
                   help="checkpoint path: resumed from if it exists, saved every SAVE_STEPS")
    p.add_argument("--gpu", type=str, default=None,
                   help="device index (sets HIP_VISIBLE_DEVICES before torch initialises HIP)")
    p.add_argument("--num_envs", type=int, default=1, help="batched environments per rank")
    p.add_argument("--train_steps", type=int, default=None)
    p.add_argument("--inner_loops", type=int, default=None)
    p.add_argument("--top_k", type=int, default=None)
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", type=str, default="auto", choices=["auto", "cpu", "hip"])
    p.add_argument("--dtype", type=str, default="fp32", choices=["fp32", "bf16", "fp16"],
                   help="HIP kernel precision: fp32 (default; fp32-accurate split-bf16 MFMA, the reference's "
                        "precision), bf16 or fp16 (faster; fp16 with dynamic loss scaling); the CPU path is fp32")
    p.add_argument("--no_bptt", action="store_true", help="detach states between rollout steps")
    p.add_argument("--no_reuse_nbr_idx", action="store_true", help="recompute kNN for h(s')")
    p.add_argument("--alternate_every", type=int, default=0)
    p.add_argument("--no_early_stop", action="store_true")
    p.add_argument("--display_steps", type=int, default=None)
    p.add_argument("--save_steps", type=int, default=None)
    p.add_argument("--log_path", type=str, default=None)
    p.add_argument("--noise_prob", type=float, default=None)
    p.add_argument("--dim", type=int, default=2, choices=[2, 3], help="spatial dimension of the double integrator")
    p.add_argument("--num_obstacles", type=int, default=0, help="static point-set obstacles per env")
    p.add_argument("--graph", action="store_true",
                   help="HIP: replay each iteration as captured graphs (launch-bound small configs)")
    return p.parse_args(argv)


def build_config(args):
    from macbf_gnn_amd import config as C
    cfg = C.TrainConfig(num_agents=args.num_agents, num_envs=args.num_envs, seed=args.seed,
                        device=args.device, dtype=args.dtype, bptt=not args.no_bptt,
                        reuse_nbr_idx=not args.no_reuse_nbr_idx,
                        alternate_every=args.alternate_every, early_stop=not args.no_early_stop,
                        model_path=args.model_path, log_path=args.log_path, dim=args.dim,
                        num_obstacles=args.num_obstacles, graph=args.graph)
    for name in ("train_steps", "inner_loops", "top_k", "lr", "display_steps", "save_steps"):
        v = getattr(args, name)
        if v is not None:
            setattr(cfg, name, v)
    if args.noise_prob is not None:
        cfg.add_noise_prob = args.noise_prob
    return cfg


def main(argv=None):
    args = parse_args(argv)
    if args.gpu is not None and "LOCAL_RANK" not in os.environ:
        # must happen before HIP initialises (the reference sets it after import torch, train.py:28)
        os.environ["HIP_VISIBLE_DEVICES"] = args.gpu
    from macbf_gnn_amd.engine import Trainer
    cfg = build_config(args)
    tr = Trainer(cfg)
    tr.fit(progress=True)
    if cfg.model_path:
        tr.save(cfg.model_path)
    tr.dp.shutdown()


if __name__ == "__main__":
    main()
