"""Hyper-parameters and physical constants.

The 20 module-level constants keep the exact names and default values of the
reference (``/root/reference/config.py:1-27``) so ``from config import *`` code keeps
working. ``TrainConfig`` adds the knobs the reference hard-codes or lacks
(batched environments, dtype, BPTT, neighbour-index reuse, seeding, ...) -- see
SURVEY.md section 5.6.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

# --- reference constants (config.py:1-27) -------------------------------------
TIME_STEP = 1e-1
WEIGHT_DECAY = 1e-8

ALPHA_CBF = 1.0

DIST_MIN_THRES = 0.07
DIST_MIN_CHECK = 0.07
DIST_MIN_ENLARGED = 0.07

OBS_RADIUS = 1.0
TOP_K = 12

TIME_TO_COLLISION = 2.0
TIME_TO_COLLISION_CHECK = 0.1

TRAIN_STEPS = 70000
EVALUATE_STEPS = 10
INNER_LOOPS = 50
REFINE_LOOPS = 50
REFINE_LEARNING_RATE = 0.3

LEARNING_RATE = 1e-4
DISPLAY_STEPS = 200
SAVE_STEPS = 1000

ADD_NOISE_PROB = 0.0
NOISE_SCALE = 0.3

# --- derived / fixed-by-reference constants -----------------------------------
# eps inside the CBF distance feature: sqrt(sum(x^2 + 1e-4)) over 2 coords (cbf.py:24-25)
CBF_DIST_EPS = 2e-4
CBF_DIST_EPS_COORD = 1e-4          # per coordinate (D = 3: 3e-4)
# loss margins (core.py:113, 155)
LOSS_EPS_DANG = 1e-3
# loss weights (train.py:93) and global scale (train.py:98)
LOSS_WEIGHTS = (2.0, 1.0, 2.0, 1.0, 0.01)
LOSS_SCALE = 10.0
# LQR-like reference gain K_ref = -[[1,0,sqrt3,0],[0,1,0,sqrt3]] (core.py:175-176)
SQRT3 = math.sqrt(3.0)
# agent density used by the scenario sampler: side = sqrt(max(1, N/8)) (core.py:46)
AGENT_DENSITY = 8.0
GOAL_SPREAD = 0.5

# maximum neighbour slots supported by the native kernels (controller tiles pad to 16)
MAX_TOP_K = 16


@dataclasses.dataclass
class TrainConfig:
    """Everything a training run needs. Defaults reproduce the reference."""

    num_agents: int = 8
    num_envs: int = 1                 # batched environments per rank
    train_steps: int = TRAIN_STEPS
    inner_loops: int = INNER_LOOPS
    top_k: int = TOP_K
    lr: float = LEARNING_RATE
    weight_decay: float = WEIGHT_DECAY
    add_noise_prob: float = ADD_NOISE_PROB
    noise_scale: float = NOISE_SCALE
    display_steps: int = DISPLAY_STEPS
    save_steps: int = SAVE_STEPS
    seed: int = 0
    dtype: str = "fp32"               # HIP kernel precision: fp32 (fp32-accurate split kernels, the reference's
                                      # precision) | bf16 | fp16 (faster, reduced precision); CPU: fp32 oracle
    loss_scale_init: float = 4096.0   # fp16: initial dynamic loss scale of the upstream gradients
    loss_scale_growth: int = 1000     # fp16: double the scale after this many finite steps
    bptt: bool = True                 # keep the rollout graph (reference behaviour, train.py:58-81)
    reuse_nbr_idx: bool = True        # h' = CBF(s') on the time-t neighbour set
    alternate_every: int = 0          # 0 = joint stepping (reference); >0 = upstream MACBF alternation
    early_stop: bool = True           # per-env done mask + stop when all envs done (train.py:78-81)
    device: str = "auto"              # auto | cpu | hip
    model_path: Optional[str] = None
    log_path: Optional[str] = None
    compute_safety: bool = True
    nan_guard: bool = True            # skip the optimizer step when the reduced gradient is not finite
    phase_timing: bool = False        # per-phase device-event timings in the step stats
    prefetch_data: bool = True        # HIP: sample iteration i+1 on a side stream during iteration i
    graph: bool = False               # HIP: replay the iteration as captured HIP graphs (Tmax steps,
                                      # done envs masked on the device) -- for launch-bound sizes
    dim: int = 2                      # spatial dimension of the double integrator (2: reference, 3)
    num_obstacles: int = 0            # static point-set obstacles per env (12 points each)
    obstacle_points: int = 12
    cbf_dedup: bool = True            # HIP, BPTT: evaluate h'(s_{t+1}) through the next step's h of the
                                      # same neighbour pair (~1.08 E instead of 2 E CBF evaluations)

    def k_eff(self) -> int:
        return min(self.num_agents, self.top_k)
