"""COCO-format detection dataset (drop-in for scripts/coco_detection_dataset.py:8-71).

Same contract as the reference: COCODetectionDataset(img_dir, ann_file, transforms=None) indexes the
COCO json (images sorted by id), __getitem__ -> (image, target) with target boxes f32 [G,4] xyxy
(x, y, x+w, y+h), labels i64 (category ids 1..6), image_id i64[1], area f32 (ann "area" or w*h),
iscrowd i64; annotations with w <= 0 or h <= 0 are dropped; images without boxes get [0,4] / [0]
tensors; collate_fn(batch) = tuple(zip(*batch)). Image = PIL RGB unless a transform is given;
uint8_transform keeps the pixels as a uint8 HWC tensor so scaling/normalisation/corruption run on the
GPU (mx_det kernels) instead of the host.
"""
from pathlib import Path

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

from .coco import get_coco_api


def uint8_transform(img):
    return torch.from_numpy(np.asarray(img, dtype=np.uint8).copy())


class COCODetectionDataset(Dataset):
    """raw=True: __getitem__ returns the file's bytes (uint8 numpy) instead of a decoded image, for the
    device JPEG decoder (mx_det.jpeg via engine.DeviceJpegLoader); transforms are not applied."""

    def __init__(self, img_dir: str, ann_file: str, transforms=None, raw=False):
        self.raw = raw
        COCO, _ = get_coco_api()
        self.img_dir = Path(img_dir)
        self.coco = COCO(ann_file)
        self.ids = sorted(self.coco.imgs.keys())
        self.transforms = transforms

    def __len__(self):
        return len(self.ids)

    def _target(self, img_id):
        anns = self.coco.loadAnns(self.coco.getAnnIds(imgIds=[img_id]))
        rows = [(a["bbox"], a) for a in anns if a["bbox"][2] > 0 and a["bbox"][3] > 0]
        if not rows:
            return {"boxes": torch.zeros((0, 4), dtype=torch.float32), "labels": torch.zeros((0,), dtype=torch.int64),
                    "image_id": torch.tensor([img_id]), "area": torch.zeros((0,), dtype=torch.float32),
                    "iscrowd": torch.zeros((0,), dtype=torch.int64)}
        xyxy = [[x, y, x + w, y + h] for (x, y, w, h), _ in rows]
        return {
            "boxes": torch.tensor(xyxy, dtype=torch.float32),
            "labels": torch.tensor([int(a["category_id"]) for _, a in rows], dtype=torch.int64),
            "image_id": torch.tensor([img_id]),
            "area": torch.tensor([float(a.get("area", b[2] * b[3])) for b, a in rows], dtype=torch.float32),
            "iscrowd": torch.tensor([int(a.get("iscrowd", 0)) for _, a in rows], dtype=torch.int64),
        }

    def __getitem__(self, idx: int):
        img_id = self.ids[idx]
        info = self.coco.loadImgs(img_id)[0]
        if self.raw:
            return np.fromfile(self.img_dir / info["file_name"], dtype=np.uint8), self._target(img_id)
        img = Image.open(self.img_dir / info["file_name"]).convert("RGB")
        target = self._target(img_id)
        if self.transforms is not None:
            img = self.transforms(img)
        return img, target


def collate_fn(batch):
    return tuple(zip(*batch))
