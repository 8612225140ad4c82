"""Capture probe: build the model, run one eager step, then capture _Graphs for one RoI-head part.

    python tools/graph_probe.py {conv1|head|pred|full|step}
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mx_det import frcnn  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def main():
    part = sys.argv[1]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = bench.build_model(dev).train()
    opt = bench.make_optimizer(m)
    imgs, tg = synth_batch(0, 2, device=dev)
    if part == "step":
        for i in range(3):
            print("step", i, bench.train_step(m, opt, imgs, tg), flush=True)
        return
    os.environ["MX_GRAPHS"] = "0"
    bench.train_step(m, opt, imgs, tg)
    be = m.be
    rh = m.roi_heads
    x = torch.randn(1024, 7, 7, 256, device=dev).bfloat16()
    if part == "conv1":
        mod = rh.box_head[0]
        fn = lambda t: (mod(t, be),)  # noqa: E731
        params = list(mod.parameters())
    elif part == "head":
        fn = lambda t: (rh.box_head(t, be),)  # noqa: E731
        params = list(rh.box_head.parameters())
    elif part == "pred":
        x = torch.randn(1024, 1, 1, 1024, device=dev).bfloat16()
        fn = lambda t: rh.box_predictor(t, be)  # noqa: E731
        params = list(rh.box_predictor.parameters())
    else:
        h = frcnn._Head(rh, be)
        fn, params = h, list(h.parameters())
    print("capturing", part, flush=True)
    g = frcnn._Graphs(fn, params, rh, x, input_grad=True)
    outs = g(x.requires_grad_(True))
    sum(o.float().sum() for o in outs).backward()
    torch.cuda.synchronize()
    print("ok", part, flush=True)


if __name__ == "__main__":
    main()
