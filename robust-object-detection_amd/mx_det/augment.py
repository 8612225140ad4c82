"""Corruption augmentation (drop-in for scripts/augmentations.py) executed by the HIP kernels.

Same constants and call surface as the reference (augmentations.py:14-98):
  NOISE_SIGMA = 15, BLUR_KERNEL = 9, BLUR_ANGLE_DEG = 0, DOWNSCALE_FACTOR = 0.5
  apply_noise / apply_motion_blur (any kernel size and angle) / apply_lowres on HxWx3 uint8 numpy
  arrays, _apply_random_corruption, RandomCorruption(p) as a PIL transform that corrupts the BGR view
  of the RGB image like the reference (augmentations.py:72-74), patch_ultralytics_augmentations().
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


def motion_blur_kernel(k: int, angle_deg: float) -> np.ndarray:
    """_motion_blur_kernel (augmentations.py:21-27) restated without OpenCV: the centre row of ones,
    rotated by cv2.getRotationMatrix2D((k/2 - 0.5, k/2 - 0.5), angle, 1) through cv2.warpAffine's
    INTER_LINEAR / BORDER_CONSTANT path (OpenCV imgwarp.cpp: the matrix inverted in double, source
    coordinates in 1/32-pixel fixed point -- AB_BITS 10, INTER_BITS 5, round_delta 16 -- and the f32
    bilinear table (1-ay)(1-ax), (1-ay)ax, ay(1-ax), ay*ax summed in tap order), then / (sum + 1e-8)
    in f32 (numpy 2 scalar rules). Host-side: k*k values."""
    f32 = np.float32
    src = np.zeros((k, k), f32)
    src[k // 2, :] = 1.0
    cx = cy = k / 2 - 0.5
    a = np.deg2rad(angle_deg)
    alpha, beta = float(np.cos(a)), float(np.sin(a))
    M = [alpha, beta, (1 - alpha) * cx - beta * cy, -beta, alpha, beta * cx + (1 - alpha) * cy]
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[4] * D, M[0] * D
    M[0], M[1], M[3], M[4] = A11, M[1] * -D, M[3] * -D, A22
    M[2], M[5] = -M[0] * M[2] - M[1] * M[5], -M[3] * M[2] - M[4] * M[5]
    rnd = lambda v: int(np.rint(v))  # noqa: E731  (cvRound: half to even)
    out = np.zeros((k, k), f32)

    def tap(yy, xx):
        return src[yy, xx] if 0 <= yy < k and 0 <= xx < k else f32(0)
    for y in range(k):
        X0 = rnd((M[1] * y + M[2]) * 1024) + 16
        Y0 = rnd((M[4] * y + M[5]) * 1024) + 16
        for x in range(k):
            X = (X0 + rnd(M[0] * x * 1024)) >> 5
            Y = (Y0 + rnd(M[3] * x * 1024)) >> 5
            sx, sy = X >> 5, Y >> 5
            ax, ay = f32(X & 31) * f32(1 / 32), f32(Y & 31) * f32(1 / 32)
            w = (f32(1) - ay) * (f32(1) - ax), (f32(1) - ay) * ax, ay * (f32(1) - ax), ay * ax
            if sx >= k or sx + 1 < 0 or sy >= k or sy + 1 < 0:
                continue
            v = tap(sy, sx) * w[0] + tap(sy, sx + 1) * w[1]
            v = v + tap(sy + 1, sx) * w[2]
            out[y, x] = v + tap(sy + 1, sx + 1) * w[3]
    return out / (out.sum() + f32(1e-8))


def kernel_taps(kernel: np.ndarray):
    """Non-zero coefficients of a k x k kernel in row-major order (OpenCV preprocess2DKernel) as
    (dy, dx, coef) relative to the centre anchor."""
    k = kernel.shape[0]
    ys, xs = np.nonzero(kernel)
    return [(int(y) - k // 2, int(x) - k // 2, float(kernel[y, x])) for y, x in zip(ys, xs)]


_DEFAULT_TAPS = None


def apply_motion_blur(img_bgr: np.ndarray, k: int, angle_deg: float) -> np.ndarray:
    global _DEFAULT_TAPS
    taps = kernel_taps(motion_blur_kernel(k, angle_deg))
    if _DEFAULT_TAPS is None:
        _DEFAULT_TAPS = kernel_taps(motion_blur_kernel(BLUR_KERNEL, BLUR_ANGLE_DEG))
    if taps == _DEFAULT_TAPS:  # the reference setting: the fused 1x9 row kernel (same arithmetic)
        return _run(img_bgr, ops.CORRUPT_BLUR)
    t = torch.from_numpy(np.ascontiguousarray(img_bgr, dtype=np.uint8))[None].to(_dev())
    return ops.filter2d_u8(t, taps)[0].cpu().numpy()


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
        bgr = np.ascontiguousarray(np.asarray(img)[..., ::-1])  # cv2.cvtColor(RGB2BGR)
        out = _apply_random_corruption(bgr)
        return Image.fromarray(np.ascontiguousarray(out[..., ::-1]))  # BGR2RGB


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
