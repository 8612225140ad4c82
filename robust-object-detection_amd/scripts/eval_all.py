"""Evaluate Faster R-CNN checkpoints on the Clean / Noise / Blur / LowRes test sets —
`python -m scripts.eval_all`.

FRCNN branch of the reference's eval_all.py (:79-156, :198-213) on MI355X; the Ultralytics RT-DETR /
YOLO branches are outside this build's scope and are reported as skipped.
Outputs keep the reference schema: experiments/eval_results.json ({model: {variant: {mAP50_95, mAP50,
per_class_ap50}}}) and experiments/eval_results.csv. torchrun shards the images per rank.
"""
import csv
import json
import time
from pathlib import Path

import torch

from mx_det.engine import dist_info, eval_frcnn_variant, init_device, load_frcnn_checkpoint

VARIANTS = ["Test_Clean", "Test_Noise", "Test_Blur", "Test_LowRes"]
SHORT = {"Test_Clean": "Clean", "Test_Noise": "Noise", "Test_Blur": "Blur", "Test_LowRes": "LowRes"}
CLASS_NAMES = ["pedestrian", "car", "van", "truck", "bus", "motor"]
COCO_TESTSET_ROOT = Path("data/testsets/coco6")
CKPTS = {
    "FasterRCNN": Path("experiments/frcnn/baseline_clean/best.pth"),
    "FasterRCNN_aug": Path("experiments/frcnn/augmented/best.pth"),
}
MODEL_ORDER = ["FasterRCNN", "FasterRCNN_aug", "RT-DETR-L", "RT-DETR-L_aug", "YOLOv8m", "YOLOv8m_aug"]
BASELINE_PAIRS = [("FasterRCNN", "FasterRCNN_aug"), ("RT-DETR-L", "RT-DETR-L_aug"), ("YOLOv8m", "YOLOv8m_aug")]
OUT_DIR = Path("experiments")


def variant_paths(root, v):
    return str(root / v / "images" / "val"), str(root / v / "annotations" / "instances_val.json")


def eval_model(name, ckpt, dev, root=None, restorer=None, variants=None):
    rank = dist_info()[1]
    root = COCO_TESTSET_ROOT if root is None else root
    variants = VARIANTS if variants is None else variants
    if rank == 0:
        print("=" * 60 + f"\n  {name}  (COCOeval bbox)\n" + "=" * 60, flush=True)
    model = load_frcnn_checkpoint(ckpt, dev)
    res = {}
    for v in variants:
        img_dir, ann = variant_paths(root, v)
        m = eval_frcnn_variant(model, img_dir, ann, dev, restorer=restorer if v != "Test_Clean" else None)
        if rank == 0:
            res[v] = m
            print(f"  [{SHORT[v]}] mAP50={m['mAP50']:.4f}  mAP50-95={m['mAP50_95']:.4f}", flush=True)
    del model
    torch.cuda.empty_cache()
    return res


def save_json(all_results, path):
    with open(path, "w", encoding="utf-8") as f:
        json.dump(all_results, f, indent=2, ensure_ascii=False)
    print(f"\nJSON saved: {Path(path).resolve()}")


def save_csv(all_results, path, variants=None, pairs=None):
    variants = VARIANTS if variants is None else variants
    pairs = BASELINE_PAIRS if pairs is None else pairs
    models = [m for m in MODEL_ORDER if m in all_results]
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["Model", "Metric"] + [SHORT[v] for v in variants])
        for m in models:
            w.writerow([m, "mAP@50"] + [f"{all_results[m][v]['mAP50']:.4f}" for v in variants])
            w.writerow([m, "mAP@50-95"] + [f"{all_results[m][v]['mAP50_95']:.4f}" for v in variants])
        w.writerow([])
        w.writerow(["Model", "Metric"] + [SHORT[v] for v in variants[1:]])
        for m in models:
            clean = all_results[m]["Test_Clean"]["mAP50"]
            w.writerow([m, "Deg%_mAP50"] + [f"{((all_results[m][v]['mAP50'] - clean) / clean * 100 if clean > 0 else 0.0):.1f}%"
                                            for v in variants[1:]])
        w.writerow([])
        w.writerow(["Model", "Metric"] + [SHORT[v] for v in variants])
        for base, aug in pairs:
            if base in all_results and aug in all_results:
                w.writerow([base, "Aug-Base_mAP50"] + [f"{all_results[aug][v]['mAP50'] - all_results[base][v]['mAP50']:+.4f}"
                                                       for v in variants])
    print(f"CSV  saved: {Path(path).resolve()}")


def main():
    dev, world, rank = init_device()
    t0 = time.time()
    all_results = {}
    for name, ck in CKPTS.items():
        r = eval_model(name, ck, dev)
        if rank == 0:
            all_results[name] = r
    if rank == 0:
        print("\n  RT-DETR-L / YOLOv8m: Ultralytics branches not part of this build (skipped)")
        print(f"\nTotal evaluation time: {(time.time() - t0) / 60:.1f} min")
        OUT_DIR.mkdir(parents=True, exist_ok=True)
        save_json(all_results, OUT_DIR / "eval_results.json")
        save_csv(all_results, OUT_DIR / "eval_results.csv")
    return all_results


if __name__ == "__main__":
    main()
