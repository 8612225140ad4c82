"""Time mx_level_topk on the training step's two shapes: the RPN's per-level pre-NMS top-k (bs=2 at
1344x800, k=2000) and the RoI sampler's stacked draw (4 rows of ~2k keys, k=512, most keys tied at
the fill value). Prints one line per (case, MX_TOPK_SLICED)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "robust-object-detection_amd"))
from mx_det import ops  # noqa: E402


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    rng = np.random.default_rng(0)
    dev = torch.device("cuda:0")
    levels = [201600, 50400, 12600, 3150, 819]
    rpn = torch.from_numpy((0.01 * rng.standard_normal((2, sum(levels)))).astype(np.float32)).to(dev)
    L = 2048
    r = rng.random((4, L)).astype(np.float32)
    keys = np.where(rng.random((4, L)) < 0.1, -r, -2.0).astype(np.float32)
    samp = torch.from_numpy(keys).to(dev)
    for sliced in ("0", "1"):
        os.environ["MX_TOPK_SLICED"] = sliced
        t_rpn = timeit(lambda: ops.level_topk(rpn, levels, 2000))
        t_s = timeit(lambda: ops.level_topk(samp, [L], 512))
        print(f"sliced={sliced} rpn_topk_us={t_rpn:.1f} sampler_topk_us={t_s:.1f}", flush=True)


if __name__ == "__main__":
    main()
