from .dist import DP, env_world
from . import launch

__all__ = ["DP", "env_world", "launch"]
