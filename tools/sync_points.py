"""Every host-synchronising CUDA/HIP operation of one steady-state train step (bench.py's headline
workload), with the Python stack that issued it: torch.cuda.set_sync_debug_mode("warn") after the
warmup steps (the graphs are captured by then). Expected: the RPN's per-image count read, the RoI
sampler's, the degenerate-box flag read and loss.item(); anything else is a GPU bubble.
    python tools/sync_points.py"""
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(42)
    model = bench.build_model(dev).train()
    opt = bench.make_optimizer(model)
    imgs, tg = synth_batch(0, 2, device=dev)
    for _ in range(4):
        bench.train_step(model, opt, imgs, tg)
    torch.cuda.synchronize()
    seen = []

    def show(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.extract_stack()[:-1] if "warnings.py" not in f.filename]
        here = [f"{os.path.relpath(f.filename, ROOT)}:{f.lineno} {f.name}" for f in stack
                if ROOT in f.filename][-4:]
        seen.append((str(message).split("\n")[0][:80], here))

    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    try:
        bench.train_step(model, opt, imgs, tg)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    print(f"{len(seen)} synchronising calls in one step")
    for msg, here in seen:
        print(msg)
        for h in here:
            print("    ", h)


if __name__ == "__main__":
    main()
