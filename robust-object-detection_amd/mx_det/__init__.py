"""mx_det — MI355X-native hot path of ysbbin/Robust-Object-Detection's Faster R-CNN train/eval step.

Host side in Python on PyTorch-ROCm (device memory, streams, torch.distributed); every hot op runs in
libmx_det.so (HIP, gfx950) through the C ABI declared in include/mx_det.h.
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
