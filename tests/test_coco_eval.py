"""COCOeval (bbox) restatement: known-answer tests (pycocotools is absent here: parity unpinned
against pycocotools itself; these cases are hand-computable from its published algorithm)."""
import numpy as np

from mx_det.coco import COCO, COCOeval


def _gt(boxes, cats=None, crowd=None, img_ids=None):
    imgs = sorted(set(img_ids or [1] * len(boxes))) or [1]
    anns = []
    for i, b in enumerate(boxes):
        anns.append({"id": i + 1, "image_id": (img_ids or [1] * len(boxes))[i], "category_id": (cats or [1] * len(boxes))[i],
                     "bbox": list(b), "area": b[2] * b[3], "iscrowd": (crowd or [0] * len(boxes))[i]})
    return COCO({"images": [{"id": i} for i in imgs], "annotations": anns,
                 "categories": [{"id": c, "name": f"c{c}"} for c in (1, 2)]})


def _eval(gt, dets):
    ev = COCOeval(gt, gt.loadRes(dets), "bbox")
    ev.evaluate()
    ev.accumulate()
    ev.summarize()
    return ev


def test_perfect_detections():
    gt = _gt([[10, 10, 50, 40], [100, 80, 30, 30]], cats=[1, 2])
    ev = _eval(gt, [{"image_id": 1, "category_id": 1, "bbox": [10, 10, 50, 40], "score": 0.9},
                    {"image_id": 1, "category_id": 2, "bbox": [100, 80, 30, 30], "score": 0.8}])
    assert abs(ev.stats[0] - 1.0) < 1e-12 and abs(ev.stats[1] - 1.0) < 1e-12


def test_false_positive_ranked_first_halves_ap():
    gt = _gt([[10, 10, 50, 40]])
    ev = _eval(gt, [{"image_id": 1, "category_id": 1, "bbox": [300, 300, 20, 20], "score": 0.95},
                    {"image_id": 1, "category_id": 1, "bbox": [10, 10, 50, 40], "score": 0.5}])
    assert abs(ev.stats[1] - 0.5) < 1e-12


def test_partial_iou_thresholds():
    gt = _gt([[0, 0, 10, 10]])
    ev = _eval(gt, [{"image_id": 1, "category_id": 1, "bbox": [0, 0, 10, 6.2], "score": 0.9}])  # IoU 0.62
    assert abs(ev.stats[0] - 0.3) < 1e-12 and abs(ev.stats[1] - 1.0) < 1e-12
    # per-class AP50 as eval_all.py:146-156 extracts it
    ap50 = ev.eval["precision"][0, :, 0, 0, 2]
    assert abs(np.mean(ap50[ap50 > -1]) - 1.0) < 1e-12


def test_crowd_gt_is_ignored():
    gt = _gt([[0, 0, 100, 100], [200, 200, 20, 20]], crowd=[1, 0])
    ev = _eval(gt, [{"image_id": 1, "category_id": 1, "bbox": [10, 10, 20, 20], "score": 0.9},  # inside crowd
                    {"image_id": 1, "category_id": 1, "bbox": [200, 200, 20, 20], "score": 0.5}])
    assert abs(ev.stats[1] - 1.0) < 1e-12
