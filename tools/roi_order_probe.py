"""RoIAlign forward: does the block -> RoI order matter (L2 per XCD)? Times the forward on one real
train step's RoIs, caches cold (bench.time_cold), in three orders of the same RoIs:
  given   -- the sampler's order (image, then sampled index)
  xcd     -- sorted by (level, image, Z-order cell of the level map) and dealt so that each XCD
             (blocks b, b+8, ...) gets one contiguous run of the sorted list
  shuffle -- random
    python tools/roi_order_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mx_det import ops  # noqa: E402
from mx_det.backend import HipBackend  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def morton(y, x):
    z = 0
    for b in range(10):
        z |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
    return z


def main():
    dev = torch.device("cuda")
    cap = {}
    orig = HipBackend.multiscale_roi_align

    def hook(self, feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
        cap.update(feats=[f.detach() for f in feats], rois=rois.detach().clone(), scales=list(scales), k_min=k_min)
        return orig(self, feats, rois, scales, k_min, output_size, sampling_ratio)

    HipBackend.multiscale_roi_align = hook
    torch.manual_seed(42)
    model = bench.build_model(dev, precision=os.environ.get("MX_PRECISION", "f32")).train()
    opt = bench.make_optimizer(model)
    imgs, tg = synth_batch(0, 2, device=dev)
    os.environ["MX_GRAPHS"] = "0"
    for _ in range(2):
        bench.train_step(model, opt, imgs, tg)
    HipBackend.multiscale_roi_align = orig
    feats, rois, scales, k_min = cap["feats"], cap["rois"], cap["scales"], cap["k_min"]
    K = rois.shape[0]
    r = rois.cpu().numpy()
    b = r[:, 1:]
    s = np.sqrt(np.maximum(b[:, 2] - b[:, 0], 0) * np.maximum(b[:, 3] - b[:, 1], 0))
    lv = np.clip(np.floor(4 + np.log2(s / 224 + 1e-30) + 1e-6), k_min, k_min + len(feats) - 1).astype(int) - k_min
    sc = np.array(scales)[lv]
    cy = ((b[:, 1] + b[:, 3]) * 0.5 * sc / 16).astype(int).clip(0, 1023)
    cx = ((b[:, 0] + b[:, 2]) * 0.5 * sc / 16).astype(int).clip(0, 1023)
    key = [(int(l), int(img), morton(int(y), int(x)), k) for k, (l, img, y, x) in enumerate(zip(lv, r[:, 0], cy, cx))]
    srt = [k for *_, k in sorted(key)]
    # block b runs on XCD b % 8; XCD x takes sorted positions [x*q, (x+1)*q)
    q = (K + 7) // 8
    blk = np.empty(K, np.int64)
    pos = 0
    for x in range(8):
        for j in range(q):
            bidx = j * 8 + x
            if pos < K and bidx < K:
                blk[bidx] = srt[pos]
                pos += 1
    assert pos == K, (pos, K)
    orders = {"given": np.arange(K), "xcd": blk, "shuffle": np.random.default_rng(0).permutation(K)}
    with torch.no_grad():
        for name, perm in orders.items():
            rp = rois[torch.from_numpy(perm).to(dev)]
            us = bench.time_cold(lambda: ops.multiscale_roi_align(feats, rp, scales, k_min), reps=10)
            warm = bench.time_cold(lambda: ops.multiscale_roi_align(feats, rp, scales, k_min), reps=10, scrub_mb=4)
            print(f"{name:8s} cold {us:7.1f} us   warm-ish {warm:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
