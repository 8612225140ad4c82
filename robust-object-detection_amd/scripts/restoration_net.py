"""Drop-in for the reference's scripts/restoration_net.py (same module tree / state_dict keys)."""
from mx_det.unet import ConvBlock, DownBlock, RestorationUNet, UpBlock  # noqa: F401
