"""Evaluate the baseline Faster R-CNN on U-Net-restored test sets — `python -m scripts.eval_restored`.

Reference: eval_restored.py (FRCNN branch :60-113, :164-184) reads JPEGs written by restore_testsets.py.
Default (MX_RESTORE_ON_DEVICE=0): the reference's pipeline -- pre-restored JPEGs from
data/testsets/coco6_restored (written by `python -m scripts.restore_testsets`, which runs the U-Net
on the device in the reference's fp32 precision and re-encodes JPEG like restore_testsets.py:101),
results in experiments/eval_restored_results.json (reference schema).
MX_RESTORE_ON_DEVICE=1: the fused MI355X pipeline of the north star -- each corrupted test image is
restored by the HIP U-Net on the GPU (reflect pad, /255, U-Net, *255, clip, truncate, crop) and fed
straight to detection, no host round trip and no JPEG re-encode. That skips the reference's JPEG
round trip, so its mAP is not the reference's number: it goes to
experiments/eval_restored_results_fused.json instead.
"""
import os
from pathlib import Path

import torch

from mx_det.unet import RestorationUNet
from scripts import eval_all

VARIANTS = eval_all.VARIANTS
CORRUPTED_ROOT = Path("data/testsets/coco6")
RESTORED_ROOT = Path("data/testsets/coco6_restored")
UNET_CKPT = Path("experiments/restoration/best.pth")
CKPTS = {"FasterRCNN": Path("experiments/frcnn/baseline_clean/best.pth")}
OUT_DIR = Path("experiments")


def load_unet(dev, ckpt=None):
    ckpt = UNET_CKPT if ckpt is None else ckpt
    unet = RestorationUNet(channels=(32, 64, 128, 256))
    sd = torch.load(ckpt, map_location="cpu", weights_only=True)
    unet.load_state_dict(sd.get("model", sd))
    return unet.to(dev).eval()


def main():
    dev, world, rank = eval_all.init_device()
    on_device = os.environ.get("MX_RESTORE_ON_DEVICE", "0") != "0"
    restorer = load_unet(dev) if on_device else None
    root = CORRUPTED_ROOT if on_device else RESTORED_ROOT
    results = {}
    for name, ck in CKPTS.items():
        r = eval_all.eval_model(name, ck, dev, root=root, restorer=restorer)
        if rank == 0:
            results[name] = r
    if rank == 0:
        OUT_DIR.mkdir(parents=True, exist_ok=True)
        name = "eval_restored_results_fused.json" if on_device else "eval_restored_results.json"
        eval_all.save_json(results, OUT_DIR / name)
    return results


if __name__ == "__main__":
    main()
