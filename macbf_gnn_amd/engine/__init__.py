from .trainer import Trainer, resolve_device

__all__ = ["Trainer", "resolve_device"]
