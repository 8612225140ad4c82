"""Faster R-CNN baseline (clean) training — `python -m scripts.train_frcnn_baseline`.

Hyper-parameters and outputs of the reference entry point (train_frcnn_baseline.py:21-36); the step
runs on MI355X through mx_det (HIP kernels). Multi-GPU: `torchrun --nproc-per-node 8 -m scripts.train_frcnn_baseline`.
MX_FRCNN_WEIGHTS may name a local COCO-pretrained state_dict (the reference's weights="DEFAULT"
download is unavailable offline; without it the model starts from random init).
"""
import os
from pathlib import Path

from mx_det.engine import train_frcnn

SEED = 42
EPOCHS = 24
BATCH_SIZE = 2
LR = 0.005
WEIGHT_DECAY = 0.0005
MOMENTUM = 0.9

DATA_ROOT = Path("data/processed/visdrone_coco6")
TRAIN_IMG = DATA_ROOT / "images/train"
VAL_IMG = DATA_ROOT / "images/val"
TRAIN_ANN = DATA_ROOT / "annotations/instances_train.json"
VAL_ANN = DATA_ROOT / "annotations/instances_val.json"
OUT_DIR = Path("experiments/frcnn/baseline_clean")
AUGMENT = False


def config():
    g = globals()
    cfg = {k: g[k] for k in ("SEED", "EPOCHS", "BATCH_SIZE", "LR", "WEIGHT_DECAY", "MOMENTUM", "TRAIN_IMG", "VAL_IMG",
                             "TRAIN_ANN", "VAL_ANN", "OUT_DIR", "AUGMENT")}
    cfg["WEIGHTS"] = os.environ.get("MX_FRCNN_WEIGHTS")
    return cfg


def main():
    return train_frcnn(config())


if __name__ == "__main__":
    main()
