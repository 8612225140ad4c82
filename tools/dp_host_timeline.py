"""Host timeline of the data-parallel train step (one-rank nccl group, mx_det.dp.DataParallel) against the
plain step: per phase host time (forward, backward, sync_gradients, optimizer, loss.item()) and, inside the
backward, the time of each hand-off hook and of each all_reduce call. Where the GPU idles in the DP step
(tools/step_concurrency.py) is where the host is inside one of these.

    python tools/dp_host_timeline.py [--steps 10]
"""
import argparse
import os
import socket
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def run(model, opt, imgs, tg, steps, acc):
    ph = defaultdict(float)
    for i in range(steps + 3):
        t0 = time.perf_counter()
        ld = model(imgs, tg)
        loss = sum(ld.values())
        t1 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        t2 = time.perf_counter()
        if hasattr(model, "sync_gradients"):
            model.sync_gradients()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        float(loss.item())
        t5 = time.perf_counter()
        if i == 2:
            acc.clear()
        if i >= 3:
            for k, v in (("forward", t1 - t0), ("backward", t2 - t1), ("sync_gradients", t3 - t2), ("opt.step", t4 - t3),
                         ("loss.item", t5 - t4), ("step", t5 - t0)):
                ph[k] += v
    return {k: 1000 * v / steps for k, v in ph.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    imgs, tg = synth_batch(0, 2, device=dev)
    torch.manual_seed(42)
    model = bench.build_model(dev).train()
    opt = bench.make_optimizer(model)
    plain = run(model, opt, imgs, tg, args.steps, {})
    del model, opt
    torch.cuda.empty_cache()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from mx_det.dp import DataParallel
    torch.manual_seed(42)
    model = bench.build_model(dev).train()
    ddp = DataParallel(model)
    opt = bench.make_optimizer(model)
    acc = defaultdict(lambda: [0, 0.0])
    ar = dist.all_reduce

    class TimedWork:
        def __init__(self, w):
            self.w = w

        def wait(self):
            t = time.perf_counter()
            try:
                return self.w.wait()
            finally:
                acc["work.wait"][0] += 1
                acc["work.wait"][1] += time.perf_counter() - t

    def timed_all_reduce(*a, **k):
        t = time.perf_counter()
        try:
            w = ar(*a, **k)
            return TimedWork(w) if w is not None else w
        finally:
            acc["all_reduce"][0] += 1
            acc["all_reduce"][1] += time.perf_counter() - t

    dist.all_reduce = timed_all_reduce
    for name in ("_start", "_early_reduce", "_segment_reduce", "_check_flag"):
        f = getattr(ddp, name)

        def wrap(*a, _f=f, _n=name, **k):
            t = time.perf_counter()
            try:
                return _f(*a, **k)
            finally:
                acc[_n][0] += 1
                acc[_n][1] += time.perf_counter() - t
        setattr(ddp, name, wrap)
    rh = model.roi_heads
    rh.__dict__["_mx_grads_ready"] = ddp._early_reduce
    model.__dict__["_mx_seg_ready"] = ddp._segment_reduce
    sg = ddp.sync_gradients

    def timed_sync():
        t = time.perf_counter()
        try:
            return sg()
        finally:
            acc["sync_gradients"][0] += 1
            acc["sync_gradients"][1] += time.perf_counter() - t
    ddp.sync_gradients = timed_sync
    st = opt.step

    def timed_step(*a, **k):
        torch.cuda.synchronize()  # (diagnostic) the optimizer's own host time, GPU drained first
        t = time.perf_counter()
        try:
            return st(*a, **k)
        finally:
            acc["opt.step (drained)"][0] += 1
            acc["opt.step (drained)"][1] += time.perf_counter() - t
    dp = run(ddp, opt, imgs, tg, args.steps, acc)
    opt.step = timed_step
    run(ddp, opt, imgs, tg, 3, {})
    ddp.close()
    dist.destroy_process_group()
    print("phase             plain ms   dp ms")
    for k in ("forward", "backward", "sync_gradients", "opt.step", "loss.item", "step"):
        print(f"{k:16s} {plain.get(k, 0):9.3f} {dp.get(k, 0):9.3f}")
    print("inside the DP step (host ms per step, calls per step):")
    for k, (n, t) in sorted(acc.items()):
        print(f"  {k:16s} {1000 * t / args.steps:8.3f}  {n / args.steps:5.1f}")


if __name__ == "__main__":
    main()
