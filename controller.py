"""Reference-compatible ``controller`` module: ``controller.Controller(in_dim)``
(``/root/reference/controller.py:10-63``)."""
from macbf_gnn_amd.models.controller import Controller  # noqa: F401
from macbf_gnn_amd.config import *  # noqa: F401,F403
