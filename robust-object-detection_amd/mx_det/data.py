"""Synthetic VisDrone-shaped inputs (there is no dataset offline).

Images: uint8 [H, W, 3] (default 800 x 1333), seed 1000 + i: a blocky low-pass field plus uniform
detail, so blur / low-res corruption is non-trivial.
Targets: G ~ Poisson(55) clipped to [1, 300]; centres uniform; w, h log-normal (median 24 px,
sigma 0.8) clipped to >= 2 px and to the image; labels 1..6 with p = (0.30, 0.40, 0.07, 0.04,
0.02, 0.17) (VisDrone-like skew; an assumption); seed 42. Target dicts follow
coco_detection_dataset.py:55-61 (boxes f32 xyxy, labels i64, image_id, area, iscrowd).
"""
import numpy as np
import torch

CLASS_P = (0.30, 0.40, 0.07, 0.04, 0.02, 0.17)


def synth_image(i, H=800, W=1333):
    rng = np.random.default_rng(1000 + i)
    base = rng.integers(0, 256, (H // 16 + 1, W // 16 + 1, 3)).astype(np.uint8)
    low = np.repeat(np.repeat(base, 16, 0), 16, 1)[:H, :W]
    detail = rng.integers(0, 64, (H, W, 3), dtype=np.uint8)
    return (low // 4 * 3 + detail).astype(np.uint8)


def synth_target(i, H=800, W=1333, seed=42, max_boxes=300, mean_boxes=55):
    rng = np.random.default_rng(seed * 100003 + i)
    G = int(np.clip(rng.poisson(mean_boxes), 1, max_boxes))
    w = np.clip(rng.lognormal(np.log(24.0), 0.8, G), 2, W - 1)
    h = np.clip(rng.lognormal(np.log(24.0), 0.8, G), 2, H - 1)
    cx = rng.uniform(0, W, G)
    cy = rng.uniform(0, H, G)
    x1 = np.clip(cx - w / 2, 0, W - 2)
    y1 = np.clip(cy - h / 2, 0, H - 2)
    x2 = np.minimum(x1 + w, W)
    y2 = np.minimum(y1 + h, H)
    boxes = np.stack([x1, y1, x2, y2], 1).astype(np.float32)
    labels = rng.choice(np.arange(1, 7), size=G, p=CLASS_P).astype(np.int64)
    return {
        "boxes": torch.from_numpy(boxes),
        "labels": torch.from_numpy(labels),
        "image_id": torch.tensor([i]),
        "area": torch.from_numpy(((x2 - x1) * (y2 - y1)).astype(np.float32)),
        "iscrowd": torch.zeros(G, dtype=torch.int64),
    }


def synth_batch(start, n, H=800, W=1333, device="cpu"):
    imgs = torch.from_numpy(np.stack([synth_image(start + k, H, W) for k in range(n)])).to(device)
    tg = [{k: v.to(device) for k, v in synth_target(start + k, H, W).items()} for k in range(n)]
    return imgs, tg


VISDRONE_CATEGORIES = ["pedestrian", "car", "van", "truck", "bus", "motor"]  # convert_visdrone_to_coco.py:24-31


def write_coco_split(root, split, start, n, H=800, W=1333, mean_boxes=55, quality=95):
    """A synthetic VisDrone-COCO split on disk in the layout the reference's scripts read
    (data/processed/visdrone_coco6: images/<split>/*.jpg as PIL JPEG q95 and
    annotations/instances_<split>.json, bbox xywh, the six VisDrone categories). Returns the json path."""
    import json
    from pathlib import Path
    from PIL import Image
    root = Path(root)
    img_dir = root / "images" / split
    img_dir.mkdir(parents=True, exist_ok=True)
    images, anns, aid = [], [], 1
    for i in range(n):
        name = f"{start + i:05d}.jpg"
        Image.fromarray(synth_image(start + i, H, W)).save(img_dir / name, quality=quality)
        images.append({"id": start + i, "file_name": name, "width": W, "height": H})
        t = synth_target(start + i, H, W, mean_boxes=mean_boxes)
        for b, lab in zip(t["boxes"].tolist(), t["labels"].tolist()):
            anns.append({"id": aid, "image_id": start + i, "category_id": lab,
                         "bbox": [b[0], b[1], b[2] - b[0], b[3] - b[1]], "area": (b[2] - b[0]) * (b[3] - b[1]),
                         "iscrowd": 0})
            aid += 1
    cats = [{"id": k, "name": nm} for k, nm in enumerate(VISDRONE_CATEGORIES, 1)]
    (root / "annotations").mkdir(parents=True, exist_ok=True)
    ann = root / "annotations" / f"instances_{split}.json"
    with open(ann, "w") as f:
        json.dump({"images": images, "annotations": anns, "categories": cats}, f)
    return ann
