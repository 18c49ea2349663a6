"""Reference-compatible constants module (``/root/reference/config.py:1-27``).

``from config import *`` exposes the same 20 names with the same defaults; they are
re-exported from :mod:`macbf_gnn_amd.config`, which also holds ``TrainConfig``.
"""
from macbf_gnn_amd.config import (  # noqa: F401
    TIME_STEP, WEIGHT_DECAY, ALPHA_CBF, DIST_MIN_THRES, DIST_MIN_CHECK, DIST_MIN_ENLARGED,
    OBS_RADIUS, TOP_K, TIME_TO_COLLISION, TIME_TO_COLLISION_CHECK, TRAIN_STEPS, EVALUATE_STEPS,
    INNER_LOOPS, REFINE_LOOPS, REFINE_LEARNING_RATE, LEARNING_RATE, DISPLAY_STEPS, SAVE_STEPS,
    ADD_NOISE_PROB, NOISE_SCALE,
)
