"""MultiScaleRoIAlign backward micro-benchmark on the RoIs of a real train step.

    python tools/bench_roialign.py
Captures the (features, rois) of one bench.py train step, prints the RoI level / footprint
distribution, and times the forward and every backward form on exactly those inputs.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mx_det import ops  # noqa: E402
from mx_det.backend import HipBackend  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda")
    cap = {}
    orig = HipBackend.multiscale_roi_align

    def hook(self, feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
        cap.update(feats=[f.detach() for f in feats], rois=rois.detach().clone(), scales=list(scales), k_min=k_min)
        return orig(self, feats, rois, scales, k_min, output_size, sampling_ratio)

    HipBackend.multiscale_roi_align = hook
    if os.environ.get("MX_ROI_SPLIT"):
        from mx_det import _lib
        _lib.call("mx_roi_fwd_set_split", int(os.environ["MX_ROI_SPLIT"]))
    if os.environ.get("MX_ROI_STRIP"):
        from mx_det import _lib
        _lib.call("mx_roi_bwd_set_strip", int(os.environ["MX_ROI_STRIP"]))
    torch.manual_seed(42)
    precision = os.environ.get("MX_PRECISION", "f32")
    model = bench.build_model(dev, precision=precision).train()
    opt = bench.make_optimizer(model)
    imgs, tg = synth_batch(0, 2, device=dev)
    os.environ["MX_GRAPHS"] = "0"  # eager, so the hook sees the call
    for _ in range(int(os.environ.get("MX_PROBE_STEPS", "2"))):  # RoIs concentrate as the RPN trains
        bench.train_step(model, opt, imgs, tg)
    HipBackend.multiscale_roi_align = orig
    feats, rois, scales, k_min = cap["feats"], cap["rois"], cap["scales"], cap["k_min"]
    K = rois.shape[0]
    print("K", K, "levels", [tuple(f.shape) for f in feats], feats[0].dtype)
    b = rois[:, 1:].float()
    s = torch.sqrt((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]))
    lv = torch.clamp(torch.floor(4 + torch.log2(s / 224) + 1e-6), k_min, k_min + len(feats) - 1).long() - k_min
    for l in range(len(feats)):
        m = lv == l
        if m.any():
            cells = torch.maximum(b[m, 2] - b[m, 0], b[m, 3] - b[m, 1]) * scales[l]
            print(f"level {l}: {int(m.sum())} rois, footprint side cells median {cells.median():.1f} max {cells.max():.1f}")
    # RoIs overlapping each 8x8 tile of their level map (the deterministic gather's serial chain)
    import numpy as np
    rb = rois.float().cpu().numpy()
    lvn = lv.cpu().numpy()
    for l in range(len(feats)):
        H, W = feats[l].shape[1], feats[l].shape[2]
        cntt = np.zeros((2, (H + 7) // 8, (W + 7) // 8), np.int64)
        for r, ll in zip(rb, lvn):
            if ll != l:
                continue
            x1, y1, x2, y2 = r[1:] * scales[l]
            ys, ye = max(int(np.floor(y1)) - 1, 0), min(int(np.floor(max(y2, y1 + 1))) + 1, H - 1)
            xs, xe = max(int(np.floor(x1)) - 1, 0), min(int(np.floor(max(x2, x1 + 1))) + 1, W - 1)
            cntt[int(r[0]), ys // 8:ye // 8 + 1, xs // 8:xe // 8 + 1] += 1
        nz = cntt[cntt > 0]
        if nz.size:
            print(f"level {l}: tiles {cntt.size}, touched {nz.size}, RoIs per touched tile mean {nz.mean():.1f} "
                  f"p90 {np.percentile(nz, 90):.0f} max {nz.max()}")
    fs = [f.clone().requires_grad_(True) for f in feats]
    out = ops.multiscale_roi_align(fs, rois, scales, k_min)
    g = torch.randn_like(out)
    print(f"fwd {timeit(lambda: ops.multiscale_roi_align(feats, rois, scales, k_min)) * 1000:.1f} us")
    res = {}
    for det in ("1", "0"):
        os.environ["MX_ROI_DETERMINISTIC"] = det
        t = timeit(lambda: torch.autograd.grad(out, fs, g, retain_graph=True)) * 1000
        res[det] = [torch.autograd.grad(out, fs, g, retain_graph=True) for _ in range(2)]
        same = all(torch.equal(a, b) for a, b in zip(*res[det]))
        print(f"bwd deterministic={det}: {t:.1f} us (incl. map allocation{'' if det == '1' else ' + zero fill'}); "
              f"run-twice bitwise equal: {same}")
    d = max(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item() for a, b in zip(res["1"][0], res["0"][0]))
    print(f"max |det - atomic| / max|atomic| over levels: {d:.2e}")
    maps = sum(f.numel() for f in feats) * 4
    print(f"level-map bytes {maps / 1e6:.1f} MB, gout {g.numel() * g.element_size() / 1e6:.1f} MB")
    zero_only = timeit(lambda: [torch.zeros(f.shape, dtype=torch.float32, device=dev) for f in feats])
    print(f"zero-filled map allocation alone {zero_only * 1000:.1f} us")


if __name__ == "__main__":
    main()
