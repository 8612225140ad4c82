"""Evaluate the baseline Faster R-CNN on U-Net-restored test sets — `python -m scripts.eval_restored`.

Reference: eval_restored.py (FRCNN branch :60-113, :164-184) reads JPEGs written by restore_testsets.py.
Default here (MX_RESTORE_ON_DEVICE=1) is the fused MI355X pipeline of the north star: each corrupted
test image is restored by the HIP U-Net on the GPU (reflect pad, /255, U-Net, *255, clip, truncate,
crop) and fed straight to detection — no host round trip, no JPEG re-encode. Set
MX_RESTORE_ON_DEVICE=0 to evaluate pre-restored images from data/testsets/coco6_restored instead.
Output: experiments/eval_restored_results.json (reference schema).
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
    on_device = os.environ.get("MX_RESTORE_ON_DEVICE", "1") != "0"
    restorer = load_unet(dev) if on_device else None
    root = CORRUPTED_ROOT if on_device else RESTORED_ROOT
    results = {}
    for name, ck in CKPTS.items():
        r = eval_all.eval_model(name, ck, dev, root=root, restorer=restorer)
        if rank == 0:
            results[name] = r
    if rank == 0:
        OUT_DIR.mkdir(parents=True, exist_ok=True)
        eval_all.save_json(results, OUT_DIR / "eval_restored_results.json")
    return results


if __name__ == "__main__":
    main()
