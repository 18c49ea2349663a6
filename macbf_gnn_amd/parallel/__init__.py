from .dist import DP, env_world

__all__ = ["DP", "env_world"]
