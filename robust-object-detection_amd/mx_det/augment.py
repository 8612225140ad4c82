"""Corruption augmentation (drop-in for scripts/augmentations.py) executed by the HIP kernels.

Same constants and call surface as the reference (augmentations.py:14-98):
  NOISE_SIGMA = 15, BLUR_KERNEL = 9, BLUR_ANGLE_DEG = 0, DOWNSCALE_FACTOR = 0.5
  apply_noise / apply_motion_blur / apply_lowres on HxWx3 uint8 numpy arrays (BGR or RGB: the ops
  are per-channel), _apply_random_corruption, RandomCorruption(p) as a PIL transform,
  patch_ultralytics_augmentations().
apply_noise draws its field with np.random.normal(0, sigma, shape) exactly like the reference, so a
seeded numpy stream reproduces the reference output bit for bit; the add/clip/truncate runs on
device. RandomCorruptionGPU is the training-loop form: uint8 HWC device tensors in and out, the noise
field from the on-device Philox generator, never leaving HBM.
"""
import random

import numpy as np
import torch

from . import ops

NOISE_SIGMA = 15
BLUR_KERNEL = 9
BLUR_ANGLE_DEG = 0
DOWNSCALE_FACTOR = 0.5


def _dev():
    if not torch.cuda.is_available():
        raise RuntimeError("mx_det corruption ops run on the GPU (HIP); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _run(img, op, **kw):
    t = torch.from_numpy(np.ascontiguousarray(img, dtype=np.uint8))[None].to(_dev())
    return ops.corrupt_u8(t, [op], **kw)[0].cpu().numpy()


def apply_noise(img_bgr: np.ndarray, sigma: float) -> np.ndarray:
    noise = np.random.normal(0, sigma, img_bgr.shape).astype(np.float32)
    return _run(img_bgr, ops.CORRUPT_NOISE, noise=torch.from_numpy(noise)[None].to(_dev()))


def apply_motion_blur(img_bgr: np.ndarray, k: int, angle_deg: float) -> np.ndarray:
    if k != BLUR_KERNEL or angle_deg % 180 != 0:
        raise NotImplementedError("device motion blur implements the reference setting (k=9, angle 0)")
    return _run(img_bgr, ops.CORRUPT_BLUR)


def apply_lowres(img_bgr: np.ndarray, factor: float) -> np.ndarray:
    return _run(img_bgr, ops.CORRUPT_LOWRES, factor=float(factor))


def _apply_random_corruption(img_bgr: np.ndarray) -> np.ndarray:
    choice = random.choice(["noise", "blur", "lowres"])
    if choice == "noise":
        return apply_noise(img_bgr, NOISE_SIGMA)
    if choice == "blur":
        return apply_motion_blur(img_bgr, BLUR_KERNEL, BLUR_ANGLE_DEG)
    return apply_lowres(img_bgr, DOWNSCALE_FACTOR)


class RandomCorruption:
    """PIL transform: with probability p apply one random corruption (augmentations.py:60-74)."""

    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, img):
        from PIL import Image
        if random.random() > self.p:
            return img
        return Image.fromarray(_apply_random_corruption(np.asarray(img)))


class RandomCorruptionGPU:
    """Device form for uint8 HWC tensors: same decision rule (keep with prob 1-p, else a uniform choice
    of noise / blur / lowres) drawn from Python's `random` like the reference; noise from Philox."""

    CODES = {"noise": ops.CORRUPT_NOISE, "blur": ops.CORRUPT_BLUR, "lowres": ops.CORRUPT_LOWRES}

    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, img):
        if random.random() > self.p:
            return img
        code = self.CODES[random.choice(["noise", "blur", "lowres"])]
        return ops.corrupt_u8(img[None], [code], sigma=NOISE_SIGMA, seed=random.getrandbits(63),
                              factor=DOWNSCALE_FACTOR)[0]


def patch_ultralytics_augmentations():
    """augmentations.py:78-98: wrap Ultralytics' Albumentations.__call__ with a p=0.5 corruption of
    labels["img"] (BGR uint8). Ultralytics itself is not installed here (SURVEY.md §8f 'next')."""
    from ultralytics.data import augment as _augment

    orig = _augment.Albumentations.__call__

    def _patched(self, labels):
        if random.random() < 0.5:
            labels["img"] = _apply_random_corruption(labels["img"])
        return orig(self, labels)

    _augment.Albumentations.__call__ = _patched
    print("[augmentations] Ultralytics Albumentations patched with corruption augmentations")
