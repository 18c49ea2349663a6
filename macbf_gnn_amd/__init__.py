"""macbf_gnn_amd -- MI355X-native multi-agent control-barrier-function trainer.

Same capabilities and user-facing API as lucaballotta/macbf-gnn (``train.py --num_agents``,
``core.py`` functions, ``config.py`` constants, ``Controller``/``CBF`` state_dict layout),
re-designed for AMD Instinct MI355X (gfx950): hand-written HIP/CDNA4 kernels for the graph
build, GNN message passing, CBF losses and rollout; RCCL data parallelism over xGMI.
"""
from . import config
from .models import CBF, Controller

__version__ = "0.1.0"

__all__ = ["config", "CBF", "Controller", "__version__"]
