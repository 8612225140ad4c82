"""Host time of the optimizer step (mx_det.optim.SGD._pack_step) on the headline model, GPU drained
before each call, with a cProfile breakdown: the optimizer's issue time is exposed GPU idle when the
backward's graph launch returns late.

    python tools/opt_host_profile.py
"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = bench.build_model(dev).train()
    opt = bench.make_optimizer(m)
    imgs, tg = synth_batch(0, 2, device=dev)
    for _ in range(4):
        bench.train_step(m, opt, imgs, tg)
    ts = []
    pr = cProfile.Profile()
    for i in range(12):
        ld = m(imgs, tg)
        loss = sum(ld.values())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        t = time.perf_counter()
        if i >= 2:
            pr.enable()
        opt.step()
        if i >= 2:
            pr.disable()
        ts.append(time.perf_counter() - t)
        float(loss.item())
    print(f"opt.step host time (GPU drained, cProfile on): {1e3 * sum(ts[2:]) / len(ts[2:]):.3f} ms")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(s.getvalue())


if __name__ == "__main__":
    main()
