"""Where the deterministic RoIAlign backward spends its time: the gather kernel timed (HIP graph replay)
on the RoIs of a real train step, then on subsets -- one RoI (the level maps' zero fill), and the RoIs
of each pyramid level alone.

    python tools/roi_bwd_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]
os.environ["MX_GRAPHS"] = "0"

import torch  # noqa: E402

import bench  # noqa: E402
from mx_det import ops  # noqa: E402
from mx_det.backend import HipBackend  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda")
    torch.manual_seed(42)
    model = bench.build_model(dev, precision="f32").train()
    opt = bench.make_optimizer(model)
    imgs, tg = synth_batch(0, 2, device=dev)
    cap = {}
    o_ra = HipBackend.multiscale_roi_align

    def ra(self, feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
        cap["ra"] = ([f.detach() for f in feats], rois.detach().clone(), list(scales), k_min)
        return o_ra(self, feats, rois, scales, k_min, output_size, sampling_ratio)

    HipBackend.multiscale_roi_align = ra
    bench.train_step(model, opt, imgs, tg)
    HipBackend.multiscale_roi_align = o_ra
    feats, rois, scales, k_min = cap["ra"]
    shapes = [tuple(f.shape) for f in feats]
    fs = [f.clone().requires_grad_(True) for f in feats]
    out = ops.multiscale_roi_align(fs, rois, scales, k_min)
    r_saved, lv_saved = out.grad_fn.saved_tensors
    g = torch.randn_like(out)
    print("levels", [s[1:3] for s in shapes], "RoIs per level", torch.bincount(lv_saved.long(), minlength=len(shapes)).tolist())

    def run(idx):
        return lambda: ops.multiscale_roi_align_backward(g[idx], r_saved[idx], lv_saved[idx], shapes, list(scales))

    allk = torch.arange(rois.shape[0], device=dev)
    print(f"all RoIs: {timed(run(allk)):8.1f} us")
    print(f"one RoI (zero fill + scan): {timed(run(allk[:1])):8.1f} us")
    for lv in range(len(shapes)):
        idx = (lv_saved == lv).nonzero().flatten()
        if idx.numel():
            print(f"level {lv} only ({idx.numel()} RoIs): {timed(run(idx)):8.1f} us")


if __name__ == "__main__":
    main()
