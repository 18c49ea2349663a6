"""Checkpoint save/resume (absent in the reference: ``--model_path``/``SAVE_STEPS`` unused,
``train.py:20``, ``config.py:24``).

Format (a plain dict, loadable with ``torch.load(..., weights_only=True)``)::

    {'controller': state_dict, 'cbf': state_dict,
     'optim_controller': Adam state_dict, 'optim_cbf': Adam state_dict,
     'step': int, 'config': dict, 'rng': dict, 'format': 'macbf-gnn-amd/1'}

``load`` also accepts a bare ``{'controller':..., 'cbf':...}`` pair or a single module
state_dict (keys prefixed ``controller_`` / ``cbf_net``). Checkpoints are DP-width agnostic:
parameters and Adam moments are replicated on every rank, scenario RNG is counter-based.
"""
from __future__ import annotations

import dataclasses
import os

import torch

FORMAT = "macbf-gnn-amd/1"


def save(trainer, path: str):
    if trainer.dp.rank != 0:
        return
    cfg = dataclasses.asdict(trainer.cfg)
    ck = {
        "format": FORMAT,
        "controller": {k: v.detach().cpu().clone() for k, v in trainer.controller.state_dict().items()},
        "cbf": {k: v.detach().cpu().clone() for k, v in trainer.cbf.state_dict().items()},
        "optim_controller": trainer.opt.torch_state_dict("controller"),
        "optim_cbf": trainer.opt.torch_state_dict("cbf"),
        "step": int(trainer.step_count),
        "config": {k: v for k, v in cfg.items() if isinstance(v, (int, float, str, bool, type(None)))},
        "rng": {"seed": int(trainer.cfg.seed), "iteration": int(trainer.step_count)},
        "grad_scale": float(getattr(trainer, "grad_scale", 1.0)),
    }
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    torch.save(ck, tmp)
    os.replace(tmp, path)


# architecture-defining config entries a resumed checkpoint must agree on
ARCH_KEYS = ("dim", "top_k", "num_obstacles", "obstacle_points")


def load(trainer, path: str, strict: bool = True):
    ck = torch.load(path, map_location="cpu", weights_only=True)
    saved = ck.get("config") if isinstance(ck.get("config"), dict) else {}
    for k in ARCH_KEYS:
        if k in saved and hasattr(trainer.cfg, k) and saved[k] != getattr(trainer.cfg, k):
            raise ValueError(f"checkpoint {path} was written with {k}={saved[k]!r}, "
                             f"the current run has {k}={getattr(trainer.cfg, k)!r}")
    if "controller" in ck or "cbf" in ck:
        if "controller" in ck:
            _load_module(trainer.controller, ck["controller"], strict)
        if "cbf" in ck:
            _load_module(trainer.cbf, ck["cbf"], strict)
    else:
        keys = list(ck.keys())
        if any(k.startswith("controller_") for k in keys):
            _load_module(trainer.controller, ck, strict)
        elif any(k.startswith("cbf_net") for k in keys):
            _load_module(trainer.cbf, ck, strict)
        else:
            raise ValueError(f"unrecognised checkpoint layout in {path}")
    if "optim_controller" in ck:
        trainer.opt.load_torch_state_dict("controller", ck["optim_controller"])
    if "optim_cbf" in ck:
        trainer.opt.load_torch_state_dict("cbf", ck["optim_cbf"])
    if "step" in ck:
        trainer.step_count = int(ck["step"])
    if "grad_scale" in ck and getattr(trainer, "fp16", False):
        trainer.grad_scale = float(ck["grad_scale"])
    trainer.on_params_loaded()
    return ck


def _load_module(mod, sd, strict):
    """Copy a state_dict into `mod`. Shapes must match exactly (a same-size tensor of another
    layout -- transposed, another in_dim -- would load as garbage); strict also rejects missing
    and unexpected keys."""
    with torch.no_grad():
        own = dict(mod.named_parameters())
        missing = [k for k in own if k not in sd]
        if strict and missing:
            raise KeyError(f"missing keys {missing}")
        if strict:
            unexpected = [k for k in sd if k not in own]
            if unexpected:
                raise KeyError(f"unexpected keys {unexpected}")
        for k, p in own.items():
            if k in sd:
                if tuple(sd[k].shape) != tuple(p.shape):
                    raise ValueError(f"{k}: checkpoint shape {tuple(sd[k].shape)} != parameter shape {tuple(p.shape)}")
                p.copy_(sd[k].to(p.dtype))


def load_models(path: str, controller, cbf, strict: bool = True):
    """Load only the network weights of a checkpoint (any format ``load`` accepts) into bare
    modules, e.g. for evaluation without a trainer."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if "controller" in ck or "cbf" in ck:
        if "controller" in ck and controller is not None:
            _load_module(controller, ck["controller"], strict)
        if "cbf" in ck and cbf is not None:
            _load_module(cbf, ck["cbf"], strict)
        return
    keys = list(ck.keys())
    if any(k.startswith("controller_") for k in keys) and controller is not None:
        _load_module(controller, ck, strict)
    elif any(k.startswith("cbf_net") for k in keys) and cbf is not None:
        _load_module(cbf, ck, strict)
