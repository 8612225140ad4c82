"""Write U-Net-restored copies of the corrupted COCO test sets — `python -m scripts.restore_testsets`.

Reference restore_testsets.py:82-159: Noise / Blur / LowRes images restored, annotations copied, Clean
copied unchanged; JPEG output. Here the restoration itself runs on the GPU (mx_det.unet.restore_u8);
decode/encode stay on the host (PIL). The fused eval path (eval_restored.py) skips this step.
"""
import shutil
from pathlib import Path

import numpy as np
import torch
from PIL import Image

from scripts import eval_restored
from mx_det.engine import init_device

COCO_TESTSET_ROOT = Path("data/testsets/coco6")
COCO_OUT_ROOT = Path("data/testsets/coco6_restored")
VARIANTS_TO_RESTORE = ["Test_Noise", "Test_Blur", "Test_LowRes"]


def restore_variant(unet, variant, dev, src_root=None, dst_root=None):
    src_root = COCO_TESTSET_ROOT if src_root is None else src_root
    dst_root = COCO_OUT_ROOT if dst_root is None else dst_root
    src_img, dst_img = src_root / variant / "images" / "val", dst_root / variant / "images" / "val"
    src_ann, dst_ann = src_root / variant / "annotations", dst_root / variant / "annotations"
    dst_img.mkdir(parents=True, exist_ok=True)
    dst_ann.mkdir(parents=True, exist_ok=True)
    for f in src_ann.glob("*.json"):
        shutil.copy2(f, dst_ann / f.name)
    files = sorted(src_img.glob("*.jpg"))
    for i, p in enumerate(files):
        img = torch.from_numpy(np.asarray(Image.open(p).convert("RGB"), dtype=np.uint8).copy()).to(dev)
        out = unet.restore_u8(img[None])[0].cpu().numpy()
        Image.fromarray(out).save(dst_img / p.name, quality=95)
        if (i + 1) % 100 == 0 or i + 1 == len(files):
            print(f"    COCO {variant}: {i + 1}/{len(files)}", flush=True)


def main():
    dev, _, _ = init_device()
    unet = eval_restored.load_unet(dev)
    for v in VARIANTS_TO_RESTORE:
        restore_variant(unet, v, dev)
    clean_src, clean_dst = COCO_TESTSET_ROOT / "Test_Clean", COCO_OUT_ROOT / "Test_Clean"
    if clean_src.exists() and not clean_dst.exists():
        shutil.copytree(clean_src, clean_dst)


if __name__ == "__main__":
    main()
