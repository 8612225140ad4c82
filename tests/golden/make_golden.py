"""Generate golden fixtures by importing the reference's own Python modules.

Run here (the container that holds /root/reference), never on the GPU box:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is pinned, and by which reference code:
  * unet_small.npz   - scripts/restoration_net.py:60-106 RestorationUNet forward (eval mode) with
                       channels (8,16,32,64), seeded weights and randomised BN running stats/affine,
                       on [1,3,48,64] and on odd [1,3,50,66] (exercises the bilinear fix-up :53-55).
  * unet_keys.json   - state_dict key -> shape list of the full-size RestorationUNet(32,64,128,256)
                       and its parameter count (restoration_net.py:60-86).
  * noise.npz        - scripts/augmentations.py:30-33 apply_noise with np.random.seed(42), and the
                       noise field it drew (so the restatement can be fed the same field).
  * dataset_target.json - scripts/coco_detection_dataset.py:18-67 target construction for a small
                       COCO json with a zero-width box, a zero-height box and an image with no boxes.
  * random_corruption.npz - scripts/augmentations.py:60-74 RandomCorruption(p=0.5) on a PIL RGB image
                       under random.seed(s) / np.random.seed(s): the keep decision, the choice and,
                       for the seeds whose choice is noise (or keep), the output image -- the noise
                       field lands on the BGR view (cvtColor RGB2BGR, :72) and the result is flipped
                       back (:74).

cv2 and pycocotools are not installed here; they are stubbed only where the pinned function never
calls them (apply_noise uses numpy alone; the dataset uses COCO as a plain index) or with exact
equivalents (cv2.cvtColor RGB2BGR / BGR2RGB on HxWx3 uint8 is the channel reversal). A seed whose
choice is blur or low-res needs real cv2 and is recorded without an output.
"""
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    cv2 = types.ModuleType("cv2")
    cv2.__stub__ = True
    cv2.COLOR_RGB2BGR, cv2.COLOR_BGR2RGB = 4, 4

    def cvtColor(a, code):  # RGB <-> BGR for 3-channel uint8: the channel reversal
        assert code == 4 and a.ndim == 3 and a.shape[2] == 3
        return np.ascontiguousarray(a[..., ::-1])
    cv2.cvtColor = cvtColor
    sys.modules.setdefault("cv2", cv2)

    class COCO:  # minimal index with the calls coco_detection_dataset.py:11-26 makes
        def __init__(self, ann_file):
            with open(ann_file) as f:
                d = json.load(f)
            self.imgs = {im["id"]: im for im in d["images"]}
            self.anns = {a["id"]: a for a in d["annotations"]}
            self._by_img = {}
            for a in d["annotations"]:
                self._by_img.setdefault(a["image_id"], []).append(a["id"])

        def loadImgs(self, ids):
            ids = ids if isinstance(ids, (list, tuple)) else [ids]
            return [self.imgs[i] for i in ids]

        def getAnnIds(self, imgIds):
            out = []
            for i in imgIds:
                out += self._by_img.get(i, [])
            return out

        def loadAnns(self, ids):
            return [self.anns[i] for i in ids]

    pc = types.ModuleType("pycocotools")
    pcc = types.ModuleType("pycocotools.coco")
    pcc.COCO = COCO
    pc.coco = pcc
    sys.modules.setdefault("pycocotools", pc)
    sys.modules.setdefault("pycocotools.coco", pcc)


def make_unet():
    from scripts.restoration_net import RestorationUNet

    full = RestorationUNet(channels=(32, 64, 128, 256))
    keys = [[k, list(v.shape)] for k, v in full.state_dict().items()]
    nparam = sum(p.numel() for p in full.parameters())
    with open(os.path.join(OUT, "unet_keys.json"), "w") as f:
        json.dump({"n_params": nparam, "state_dict": keys}, f, indent=0)

    torch.manual_seed(1234)
    m = RestorationUNet(channels=(8, 16, 32, 64))
    g = torch.Generator().manual_seed(99)
    with torch.no_grad():
        for name, mod in m.named_modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                c = mod.num_features
                mod.running_mean.copy_(torch.randn(c, generator=g) * 0.2)
                mod.running_var.copy_(torch.rand(c, generator=g) * 1.5 + 0.25)
                mod.weight.copy_(torch.rand(c, generator=g) + 0.5)
                mod.bias.copy_(torch.randn(c, generator=g) * 0.1)
    m.eval()
    arrays = {}
    for k, v in m.state_dict().items():
        arrays["sd/" + k] = v.numpy()
    for tag, shape in (("a", (1, 3, 48, 64)), ("b", (1, 3, 50, 66))):
        x = torch.rand(shape, generator=g)
        with torch.no_grad():
            y = m(x)
        arrays["x_" + tag] = x.numpy()
        arrays["y_" + tag] = y.numpy()
    np.savez_compressed(os.path.join(OUT, "unet_small.npz"), **arrays)
    print("unet: full params", nparam, "small keys", len(m.state_dict()))


def make_noise():
    from scripts import augmentations as aug

    rng = np.random.RandomState(7)
    img = rng.randint(0, 256, size=(37, 53, 3)).astype(np.uint8)
    img[0, :5] = 0
    img[1, :5] = 255
    np.random.seed(42)
    field = np.random.normal(0, aug.NOISE_SIGMA, img.shape).astype(np.float32)
    np.random.seed(42)
    out = aug.apply_noise(img, aug.NOISE_SIGMA)
    np.savez_compressed(os.path.join(OUT, "noise.npz"), img=img, noise=field, out=out,
                        sigma=np.float32(aug.NOISE_SIGMA))
    consts = {"NOISE_SIGMA": aug.NOISE_SIGMA, "BLUR_KERNEL": aug.BLUR_KERNEL,
              "BLUR_ANGLE_DEG": aug.BLUR_ANGLE_DEG, "DOWNSCALE_FACTOR": aug.DOWNSCALE_FACTOR}
    with open(os.path.join(OUT, "augment_constants.json"), "w") as f:
        json.dump(consts, f)
    print("noise: changed px", int((out != img).sum()))


def make_random_corruption():
    import random

    from PIL import Image
    from scripts import augmentations as aug

    rng = np.random.RandomState(11)
    img = rng.randint(0, 256, size=(23, 31, 3)).astype(np.uint8)
    seeds, ops, outs = [], [], []
    for s in range(40):
        chosen = []
        orig = {n: getattr(aug, n) for n in ("apply_noise", "apply_motion_blur", "apply_lowres")}

        def spy(name):
            def f(*a, **k):
                chosen.append(name)
                return orig[name](*a, **k)
            return f
        for n in orig:
            setattr(aug, n, spy(n))
        random.seed(s)
        np.random.seed(s)
        try:
            out = np.asarray(aug.RandomCorruption(p=0.5)(Image.fromarray(img)))
        except AttributeError:  # blur / low-res: real cv2 needed
            out = None
        finally:
            for n, f in orig.items():
                setattr(aug, n, f)
        op = chosen[0] if chosen else "keep"
        seeds.append(s)
        ops.append(op)
        outs.append(out if out is not None else np.zeros_like(img))
    ops_a = np.array(ops)
    np.savez_compressed(os.path.join(OUT, "random_corruption.npz"), img=img, seeds=np.array(seeds), ops=ops_a,
                        outs=np.stack(outs), pinned=np.isin(ops_a, ["keep", "apply_noise"]))
    print("random_corruption:", {o: int((ops_a == o).sum()) for o in set(ops)})


def make_dataset():
    from PIL import Image
    from scripts.coco_detection_dataset import COCODetectionDataset, collate_fn

    tmp = tempfile.mkdtemp()
    imgs = [
        {"id": 3, "file_name": "c.png", "width": 8, "height": 6},
        {"id": 1, "file_name": "a.png", "width": 7, "height": 5},
        {"id": 2, "file_name": "b.png", "width": 9, "height": 4},
    ]
    anns = [
        {"id": 10, "image_id": 1, "category_id": 2, "bbox": [1, 1, 3, 2], "area": 6.0, "iscrowd": 0},
        {"id": 11, "image_id": 1, "category_id": 5, "bbox": [2.5, 0.5, 0, 3], "area": 0.0, "iscrowd": 0},
        {"id": 12, "image_id": 1, "category_id": 6, "bbox": [0.25, 1.5, 4.5, 2.25]},
        {"id": 13, "image_id": 3, "category_id": 1, "bbox": [4, 2, 3, -1], "area": 3.0},
        {"id": 14, "image_id": 3, "category_id": 3, "bbox": [0, 0, 8, 6], "area": 48.0, "iscrowd": 1},
    ]
    ann_file = os.path.join(tmp, "ann.json")
    with open(ann_file, "w") as f:
        json.dump({"images": imgs, "annotations": anns,
                   "categories": [{"id": i, "name": n} for i, n in enumerate(
                       ["pedestrian", "car", "van", "truck", "bus", "motor"], 1)]}, f)
    for im in imgs:
        Image.new("RGB", (im["width"], im["height"]), (im["id"], 2, 3)).save(
            os.path.join(tmp, im["file_name"]))
    ds = COCODetectionDataset(tmp, ann_file, transforms=None)
    out = {"coco": {"images": imgs, "annotations": anns}, "ids": ds.ids, "items": []}
    for i in range(len(ds)):
        img, t = ds[i]
        out["items"].append({
            "size": list(img.size),
            "mode": img.mode,
            "target": {k: {"dtype": str(v.dtype), "shape": list(v.shape), "data": v.tolist()}
                       for k, v in t.items()},
        })
    imgs_b, tg_b = collate_fn([ds[0], ds[1]])
    out["collate"] = {"type": type(imgs_b).__name__, "len": len(imgs_b)}
    with open(os.path.join(OUT, "dataset_target.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("dataset: items", len(out["items"]))


if __name__ == "__main__":
    sys.path.insert(0, REF)
    _stub_modules()
    make_unet()
    make_noise()
    make_random_corruption()
    make_dataset()
