"""MI355X-native U-Net hot path (drop-in for SaurabhIndi/unet-segmentation's
models/unet_model.py UNet and utils/losses.py WeightedCrossEntropyLoss)."""
from ._lib import LIB_PATH, load  # noqa: F401
from .modules import UNet, WeightedCrossEntropyLoss, DoubleConv, Down, Up, OutConv  # noqa: F401
from .plan import Plan  # noqa: F401

__all__ = ["UNet", "WeightedCrossEntropyLoss", "DoubleConv", "Down", "Up", "OutConv", "Plan", "load", "LIB_PATH"]
