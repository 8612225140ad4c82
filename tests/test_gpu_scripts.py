"""Drop-in entry points end to end on a tiny synthetic VisDrone-COCO dataset written to disk
(the reference's config #1 plumbing case, on MI355X): train_frcnn_baseline / _augmented (1 epoch),
eval_all (4 variants) and eval_restored (reference pipeline, and the fused device U-Net) with the
reference's output schemas."""
import json

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


def _write_split(root, split, start, n, H=200, W=280):
    from mx_det.data import write_coco_split
    return write_coco_split(root, split, start, n, H, W, mean_boxes=8)


def test_train_eval_scripts(dev, tmp_path, monkeypatch):
    from scripts import eval_all, eval_restored, train_frcnn_augmented, train_frcnn_baseline as base
    data = tmp_path / "visdrone_coco6"
    _write_split(data, "train", 0, 4)
    _write_split(data, "val", 100, 2)
    monkeypatch.setattr(base, "EPOCHS", 1)
    monkeypatch.setattr(base, "TRAIN_IMG", data / "images/train")
    monkeypatch.setattr(base, "VAL_IMG", data / "images/val")
    monkeypatch.setattr(base, "TRAIN_ANN", data / "annotations/instances_train.json")
    monkeypatch.setattr(base, "VAL_ANN", data / "annotations/instances_val.json")
    monkeypatch.setattr(base, "OUT_DIR", tmp_path / "frcnn/baseline_clean")
    m = base.main()
    assert set(m) == {"mAP50", "mAP50_95"}
    hist = [json.loads(l) for l in open(tmp_path / "frcnn/baseline_clean/history.jsonl")]
    assert [h["epoch"] for h in hist] == [1, "final"]
    assert set(hist[0]) == {"epoch", "train_loss_sum", "lr", "mAP50", "mAP50_95", "elapsed_sec"}
    ck = torch.load(tmp_path / "frcnn/baseline_clean/best.pth", weights_only=True)
    assert set(ck) == {"model", "epoch", "metrics"} and ck["epoch"] == "final"
    assert set(torch.load(tmp_path / "frcnn/baseline_clean/last.pth", weights_only=True)) == {"model", "epoch"}
    monkeypatch.setattr(train_frcnn_augmented, "OUT_DIR", tmp_path / "frcnn/augmented")
    train_frcnn_augmented.main()
    assert (tmp_path / "frcnn/augmented/best.pth").exists()

    # test sets: the val split under four variant names (corruption is not needed for plumbing)
    ts = tmp_path / "testsets/coco6"
    for v in eval_all.VARIANTS:
        _write_split(ts / v, "val", 100, 2)
    monkeypatch.setattr(eval_all, "COCO_TESTSET_ROOT", ts)
    monkeypatch.setattr(eval_all, "OUT_DIR", tmp_path / "experiments")
    monkeypatch.setattr(eval_all, "CKPTS", {"FasterRCNN": tmp_path / "frcnn/baseline_clean/best.pth",
                                            "FasterRCNN_aug": tmp_path / "frcnn/augmented/best.pth"})
    res = eval_all.main()
    assert set(res) == {"FasterRCNN", "FasterRCNN_aug"}
    assert set(res["FasterRCNN"]["Test_Blur"]) == {"mAP50_95", "mAP50", "per_class_ap50"}
    rows = list(open(tmp_path / "experiments/eval_results.csv"))
    assert rows[0].startswith("Model,Metric,Clean,Noise,Blur,LowRes")

    from mx_det.unet import RestorationUNet
    torch.save({"model": RestorationUNet().state_dict()}, tmp_path / "unet.pth")
    monkeypatch.setattr(eval_restored, "UNET_CKPT", tmp_path / "unet.pth")
    monkeypatch.setattr(eval_restored, "CORRUPTED_ROOT", ts)
    monkeypatch.setattr(eval_restored, "OUT_DIR", tmp_path / "experiments")
    monkeypatch.setattr(eval_restored, "CKPTS", {"FasterRCNN": tmp_path / "frcnn/baseline_clean/best.pth"})
    # default: the reference's pipeline (pre-restored images; here the plumbing test set itself)
    monkeypatch.setattr(eval_restored, "RESTORED_ROOT", ts)
    eval_restored.main()
    out = json.load(open(tmp_path / "experiments/eval_restored_results.json"))
    assert set(out["FasterRCNN"]) == set(eval_all.VARIANTS)
    # fused on-device restoration: reported separately (not the reference's JPEG round trip)
    monkeypatch.setenv("MX_RESTORE_ON_DEVICE", "1")
    eval_restored.main()
    out = json.load(open(tmp_path / "experiments/eval_restored_results_fused.json"))
    assert set(out["FasterRCNN"]) == set(eval_all.VARIANTS)


def test_augmentations_api_on_device(dev):
    """augmentations.py API: seeded apply_noise reproduces the reference exactly (same numpy stream
    and arithmetic: golden from make_golden.py); blur / lowres equal the oracle restatement."""
    from scripts import augmentations as aug
    from oracle import oracle as orc
    d = np.load("tests/golden/noise.npz")
    np.random.seed(42)
    assert np.array_equal(aug.apply_noise(d["img"], aug.NOISE_SIGMA), d["out"])
    img = np.random.default_rng(1).integers(0, 256, (31, 47, 3)).astype(np.uint8)
    assert np.array_equal(aug.apply_motion_blur(img, aug.BLUR_KERNEL, aug.BLUR_ANGLE_DEG), orc.blur_u8(img))
    assert np.array_equal(aug.apply_lowres(img, aug.DOWNSCALE_FACTOR), orc.lowres_u8(img, 0.5))
    rc = aug.RandomCorruption(p=1.0)
    out = rc(Image.fromarray(img))
    assert np.asarray(out).shape == img.shape
