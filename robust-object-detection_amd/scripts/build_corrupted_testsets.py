"""Build the corrupted test sets — `python -m scripts.build_corrupted_testsets` (reference
build_corrupted_testsets.py).

Same constants (SEED 42, sigma 15, 1x9 motion blur at 0 deg, 0.5 down/up-scale), the same sources
(data/processed/visdrone_yolo6 and visdrone_coco6 val), the same outputs under data/testsets/{yolo6,coco6}/
Test_{Clean,Noise,Blur,LowRes} (labels / instances_val.json copied, YOLO data.yaml written), in the
same order: YOLO first, then COCO, variants and images in the reference's glob order -- so the single
np.random stream seeded with 42 hands every Test_Noise image the reference's noise field. The pixel
work runs on the device (mx_det.augment: noise add/clip/truncate, cv2.filter2D motion blur, INTER_AREA
down + INTER_LINEAR up; bit-exact against the reference's apply_noise golden and the OpenCV
restatements in oracle/). Each source JPEG is decoded on the device (mx_det.jpeg: host entropy decode,
device IDCT / upsampling / colour, bit-identical to cv2.imread's libjpeg-turbo decode, in BGR like
cv2.imread; PIL decodes the formats it does not handle), corrupted there, and copied back once for the
JPEG encode (PIL / libjpeg-turbo, cv2.imwrite's default quality 95).
"""
import shutil
from pathlib import Path

import numpy as np
import torch
from PIL import Image

from mx_det import augment, jpeg, ops

YOLO_SRC = Path("data/processed/visdrone_yolo6")
COCO_SRC = Path("data/processed/visdrone_coco6")
OUT_ROOT = Path("data/testsets")
SEED = 42
NOISE_SIGMA = 15
BLUR_KERNEL = 9
BLUR_ANGLE_DEG = 0
DOWNSCALE_FACTOR = 0.5
VARIANTS = ["Test_Clean", "Test_Noise", "Test_Blur", "Test_LowRes"]
NAMES = ["pedestrian", "car", "van", "truck", "bus", "motor"]


def set_seed(seed):
    np.random.seed(seed)


def ensure_dir(p):
    Path(p).mkdir(parents=True, exist_ok=True)


def corrupt(img_bgr, variant):
    """One variant of build_corrupted_testsets.py:140-150 on a BGR uint8 image, a device tensor
    [H, W, 3] (returned on the device) or a numpy array (returned as numpy)."""
    if not torch.is_tensor(img_bgr):
        if variant == "Test_Noise":
            return augment.apply_noise(img_bgr, NOISE_SIGMA)
        if variant == "Test_Blur":
            return augment.apply_motion_blur(img_bgr, BLUR_KERNEL, BLUR_ANGLE_DEG)
        if variant == "Test_LowRes":
            return augment.apply_lowres(img_bgr, DOWNSCALE_FACTOR)
        return img_bgr
    x = img_bgr[None]
    if variant == "Test_Noise":  # the reference's numpy stream, added / clipped / truncated on the device
        noise = np.random.normal(0, NOISE_SIGMA, tuple(img_bgr.shape)).astype(np.float32)
        return ops.corrupt_u8(x, [ops.CORRUPT_NOISE], noise=torch.from_numpy(noise).to(x.device))[0]
    if variant == "Test_Blur":
        taps = augment.kernel_taps(augment.motion_blur_kernel(BLUR_KERNEL, BLUR_ANGLE_DEG))
        return ops.filter2d_u8(x, taps)[0]
    if variant == "Test_LowRes":
        return ops.corrupt_u8(x, [ops.CORRUPT_LOWRES], factor=float(DOWNSCALE_FACTOR))[0]
    return img_bgr


def _read_bgr(path):
    """cv2.imread(path) on the device: BGR uint8 [H, W, 3]; None for unreadable files (skipped, like
    cv2.imread's None)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    try:
        data = Path(path).read_bytes()
        try:
            return jpeg.decode(data, dev, bgr=True)
        except (jpeg.JpegUnsupported, ValueError):
            with Image.open(path) as im:
                rgb = np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])
            return torch.from_numpy(rgb).to(dev)
    except OSError:
        return None


def _write_bgr(path, img_bgr):
    if torch.is_tensor(img_bgr):
        img_bgr = img_bgr.cpu().numpy()
    Image.fromarray(np.ascontiguousarray(img_bgr[..., ::-1])).save(path, quality=95)


def _build_images(src_img_dir, dst_img_dir, variant):
    for img_path in src_img_dir.glob("*.*"):
        img = _read_bgr(img_path)
        if img is None:
            continue
        _write_bgr(dst_img_dir / img_path.name, corrupt(img, variant))


def write_yolo_valonly_yaml(dst_root):
    lines = [f"path: {Path(dst_root).as_posix()}", "train: images/val", "val: images/val", "", "names:"]
    lines += [f"  {i}: {n}" for i, n in enumerate(NAMES)]
    (Path(dst_root) / "data.yaml").write_text("\n".join(lines), encoding="utf-8")


def build_yolo_testsets(src=None, out_root=None):
    src, out_root = Path(src or YOLO_SRC), Path(out_root or OUT_ROOT)
    src_img_dir, src_lbl_dir = src / "images" / "val", src / "labels" / "val"
    if not src_img_dir.exists() or not src_lbl_dir.exists():
        raise FileNotFoundError("YOLO val images/labels not found. Check YOLO_SRC path.")
    for v in VARIANTS:
        dst_root = out_root / "yolo6" / v
        dst_img_dir, dst_lbl_dir = dst_root / "images" / "val", dst_root / "labels" / "val"
        ensure_dir(dst_img_dir)
        ensure_dir(dst_lbl_dir)
        for lbl in src_lbl_dir.glob("*.txt"):
            shutil.copy2(lbl, dst_lbl_dir / lbl.name)
        write_yolo_valonly_yaml(dst_root)
        _build_images(src_img_dir, dst_img_dir, v)
    print("YOLO Test sets created:", (out_root / "yolo6").resolve())


def build_coco_testsets(src=None, out_root=None):
    src, out_root = Path(src or COCO_SRC), Path(out_root or OUT_ROOT)
    src_img_dir, src_ann = src / "images" / "val", src / "annotations" / "instances_val.json"
    if not src_img_dir.exists() or not src_ann.exists():
        raise FileNotFoundError("COCO val images or instances_val.json not found. Check COCO_SRC path.")
    for v in VARIANTS:
        dst_root = out_root / "coco6" / v
        dst_img_dir, dst_ann_dir = dst_root / "images" / "val", dst_root / "annotations"
        ensure_dir(dst_img_dir)
        ensure_dir(dst_ann_dir)
        shutil.copy2(src_ann, dst_ann_dir / "instances_val.json")
        _build_images(src_img_dir, dst_img_dir, v)
    print("COCO Test sets created:", (out_root / "coco6").resolve())


def main(yolo_src=None, coco_src=None, out_root=None):
    set_seed(SEED)
    build_yolo_testsets(yolo_src, out_root)
    build_coco_testsets(coco_src, out_root)
    print("\nAll corrupted test sets are ready under:", Path(out_root or OUT_ROOT).resolve())


if __name__ == "__main__":
    main()
