"""COCO Dataset API parity with the reference scripts/coco_detection_dataset.py, pinned by
tests/golden/dataset_target.json (produced by importing the reference module, make_golden.py)."""
import json
import os

from PIL import Image


def test_dataset_targets_match_reference_golden(tmp_path):
    from mx_det.dataset import COCODetectionDataset, collate_fn
    g = json.load(open("tests/golden/dataset_target.json"))
    ann = tmp_path / "ann.json"
    cats = [{"id": i, "name": n} for i, n in enumerate(["pedestrian", "car", "van", "truck", "bus", "motor"], 1)]
    json.dump({"images": g["coco"]["images"], "annotations": g["coco"]["annotations"], "categories": cats}, open(ann, "w"))
    for im in g["coco"]["images"]:
        Image.new("RGB", (im["width"], im["height"]), (im["id"], 2, 3)).save(os.path.join(tmp_path, im["file_name"]))
    ds = COCODetectionDataset(str(tmp_path), str(ann))
    assert ds.ids == g["ids"] and len(ds) == len(g["items"])
    for i, item in enumerate(g["items"]):
        img, t = ds[i]
        assert list(img.size) == item["size"] and img.mode == item["mode"]
        assert set(t) == set(item["target"])
        for k, ref in item["target"].items():
            assert str(t[k].dtype) == ref["dtype"], k
            assert list(t[k].shape) == ref["shape"], k
            assert t[k].tolist() == ref["data"], k
    imgs, tgs = collate_fn([ds[0], ds[1]])
    assert type(imgs).__name__ == g["collate"]["type"] and len(imgs) == g["collate"]["len"]
