from .cbf import CBF
from .controller import Controller

__all__ = ["CBF", "Controller"]
