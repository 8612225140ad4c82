"""Probe of the host crash inside hipGraphLaunch (r06a / r06b): a second model whose trunk is captured
as _SegGraphs in one process. Runs model A for 3 steps, then -- per --mode -- keeps A alive, or deletes
it (gc + empty_cache), or keeps only A's captured graphs alive, then runs model B for 3 steps.
Usage: python tools/seg_probe.py --mode keep|del|graphs [--seg-a 1] [--seg-b 1]"""
import argparse
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402


def model(dev):
    from mx_det import frcnn
    torch.manual_seed(0)
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(1024, 7)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    return m.to(dev).train()


def run(m, dev, tag):
    from mx_det.data import synth_batch
    imgs, tg = synth_batch(41, 6, H=512, W=672, device=dev)
    for step in range(3):
        losses = m(imgs[2 * step:2 * step + 2], tg[2 * step:2 * step + 2])
        for p in m.parameters():
            p.grad = None
        sum(losses.values()).backward()
        torch.cuda.synchronize()
        print(tag, "step", step, "ok", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="keep")
    ap.add_argument("--seg-a", default="1")
    ap.add_argument("--seg-b", default="1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    os.environ["MX_SEG_GRAPHS"] = args.seg_a
    a = model(dev)
    run(a, dev, "A")
    keep = []
    if args.mode == "keep":
        keep.append(a)
    elif args.mode == "graphs":
        keep.append(a.__dict__.get("_mx_graphs"))
        keep.append(a.roi_heads.__dict__.get("_mx_graphs"))
    del a
    gc.collect()
    torch.cuda.synchronize()
    if args.mode != "keep":
        torch.cuda.empty_cache()
    print("A released:", args.mode, flush=True)
    os.environ["MX_SEG_GRAPHS"] = args.seg_b
    b = model(dev)
    run(b, dev, "B")
    print("probe ok", args.mode, flush=True)


if __name__ == "__main__":
    main()
