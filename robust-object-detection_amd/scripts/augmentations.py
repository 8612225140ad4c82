"""Drop-in for the reference's scripts/augmentations.py; the corruption ops run as HIP kernels."""
from mx_det.augment import (  # noqa: F401
    BLUR_ANGLE_DEG, BLUR_KERNEL, DOWNSCALE_FACTOR, NOISE_SIGMA, RandomCorruption, RandomCorruptionGPU,
    _apply_random_corruption, apply_lowres, apply_motion_blur, apply_noise, patch_ultralytics_augmentations)
