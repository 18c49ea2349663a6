"""Reference-compatible ``cbf`` module: ``cbf.CBF(in_dim)`` (``/root/reference/cbf.py:8-45``)."""
from macbf_gnn_amd.models.cbf import CBF  # noqa: F401
from macbf_gnn_amd.config import *  # noqa: F401,F403
