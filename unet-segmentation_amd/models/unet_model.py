"""Drop-in for the reference module path ``models.unet_model`` (models/unet_model.py).

``sys.path.insert(0, '<repo>/unet-segmentation_amd')`` then
``from models.unet_model import UNet`` -- exactly as scripts/train.py:19 does
with the reference project root.
"""
from unet_amd.modules import DoubleConv, Down, OutConv, UNet, Up  # noqa: F401

__all__ = ["UNet", "DoubleConv", "Down", "Up", "OutConv"]
