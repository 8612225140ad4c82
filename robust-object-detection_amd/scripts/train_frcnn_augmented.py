"""Faster R-CNN augmented training — `python -m scripts.train_frcnn_augmented`.

Identical to train_frcnn_baseline except RandomCorruption(p=0.5) on the training images (noise / blur /
low-res; here on the GPU, never touching the host) and the output directory (reference
train_frcnn_augmented.py:1-11).
"""
from pathlib import Path

from scripts import train_frcnn_baseline as base

OUT_DIR = Path("experiments/frcnn/augmented")


def main():
    cfg = base.config()
    cfg.update(OUT_DIR=OUT_DIR, AUGMENT=True)
    return base.train_frcnn(cfg)


if __name__ == "__main__":
    main()
