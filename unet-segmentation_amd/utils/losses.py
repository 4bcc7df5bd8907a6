"""Drop-in for the reference module path ``utils.losses`` (utils/losses.py)."""
from unet_amd.modules import WeightedCrossEntropyLoss  # noqa: F401

__all__ = ["WeightedCrossEntropyLoss"]
