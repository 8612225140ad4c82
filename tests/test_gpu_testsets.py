"""scripts.build_corrupted_testsets end to end on a tiny synthetic YOLO6 + COCO6 source (reference
build_corrupted_testsets.py:129-166): layout, copied labels / annotations, data.yaml, and the pixels.
The noise stream: one np.random stream seeded 42 consumed YOLO first, then COCO, image by image in glob
order -- replayed here through the oracle's apply_noise restatement (numpy add/clip/truncate) and
compared with the device output BEFORE the JPEG encode (bit-exact); the written file is byte-equal
to the quality-95 JPEG of those pixels. Blur / low-res outputs are bit-exact against the oracle's OpenCV
restatements (oracle.filter2d / oracle.lowres)."""
import json

import numpy as np
import pytest
from PIL import Image

pytestmark = pytest.mark.gpu


def _src(root, n=3):
    from mx_det.data import synth_image
    for kind in ("yolo6", "coco6"):
        img = root / kind / "images" / "val"
        img.mkdir(parents=True)
        for i in range(n):
            Image.fromarray(synth_image(i, 120 + 2 * i, 160 + 3 * i)).save(img / f"{i:03d}.jpg", quality=95)
    lbl = root / "yolo6" / "labels" / "val"
    lbl.mkdir(parents=True)
    for i in range(n):
        (lbl / f"{i:03d}.txt").write_text("0 0.5 0.5 0.1 0.1\n")
    (root / "coco6" / "annotations").mkdir(parents=True)
    json.dump({"images": [], "annotations": [], "categories": []}, open(root / "coco6/annotations/instances_val.json", "w"))


def test_build_corrupted_testsets(dev, tmp_path, monkeypatch):
    from oracle import oracle as orc
    from scripts import build_corrupted_testsets as b
    _src(tmp_path / "src")
    written = {}
    orig = b._write_bgr

    def spy(path, img):  # keep the pre-encode pixels
        written[str(path)] = img.cpu().numpy() if hasattr(img, "cpu") else img.copy()
        orig(path, img)
    monkeypatch.setattr(b, "_write_bgr", spy)
    b.main(tmp_path / "src/yolo6", tmp_path / "src/coco6", tmp_path / "out")
    out = tmp_path / "out"
    for kind in ("yolo6", "coco6"):
        for v in b.VARIANTS:
            assert len(list((out / kind / v / "images/val").glob("*.jpg"))) == 3
    assert len(list((out / "yolo6/Test_Noise/labels/val").glob("*.txt"))) == 3
    assert (out / "yolo6/Test_Blur/data.yaml").read_text().splitlines()[5] == "  0: pedestrian"
    assert (out / "coco6/Test_LowRes/annotations/instances_val.json").exists()
    # replay the reference's single noise stream: YOLO (glob order) then COCO
    rng = np.random.RandomState(42)
    for kind in ("yolo6", "coco6"):
        for p in (tmp_path / "src" / kind / "images" / "val").glob("*.*"):
            bgr = np.ascontiguousarray(np.asarray(Image.open(p).convert("RGB"))[..., ::-1])
            noise = rng.normal(0, 15, bgr.shape).astype(np.float32)
            exp = np.clip(bgr.astype(np.float32) + noise, 0, 255).astype(np.uint8)
            got = written[str(tmp_path / "out" / kind / "Test_Noise/images/val" / p.name)]
            assert np.array_equal(got, exp), (kind, p.name)
            import io
            buf = io.BytesIO()  # the file is the quality-95 JPEG of exactly those pixels
            Image.fromarray(np.ascontiguousarray(exp[..., ::-1])).save(buf, format="JPEG", quality=95)
            assert (tmp_path / "out" / kind / "Test_Noise/images/val" / p.name).read_bytes() == buf.getvalue()
            blur = written[str(tmp_path / "out" / kind / "Test_Blur/images/val" / p.name)]
            assert np.array_equal(blur, orc.motion_blur_u8(bgr, 9, 0.0))
            low = written[str(tmp_path / "out" / kind / "Test_LowRes/images/val" / p.name)]
            assert np.array_equal(low, orc.lowres_u8(bgr, 0.5))
            assert np.array_equal(written[str(tmp_path / "out" / kind / "Test_Clean/images/val" / p.name)], bgr)
