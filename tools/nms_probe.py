"""Per-kernel timing probe of the proposal NMS (run under rocprofv3 --kernel-trace --stats): the
training call's shape (2 images x levels [2000, 2000, 2000, 2000, 819], presorted per level, boxes
clustered like RPN proposals around objects), REPS calls of the sort-free path and of the general
grouped path (two radix sorts).

    rocprofv3 --kernel-trace --stats -d gpurun_out/nms -o nms -- python3 tools/nms_probe.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

from mx_det import ops  # noqa: E402


def candidates(rng, G=2, runs=(2000, 2000, 2000, 2000, 819)):
    b, s, lv, gr = [], [], [], []
    for g in range(G):
        ctr = rng.uniform([0, 0], [1333, 800], (60, 2))
        for l, k in enumerate(runs):
            c = ctr[rng.integers(0, 60, k)] + rng.normal(0, 20 * 2 ** l, (k, 2))
            wh = rng.lognormal(np.log(24 * 2 ** l), 0.5, (k, 2))
            b.append(np.concatenate([c - wh / 2, c + wh / 2], 1))
            s.append(np.sort(rng.random(k))[::-1])
            lv.append(np.full(k, l))
            gr.append(np.full(k, g))
    cat = np.concatenate
    return (cat(b).astype(np.float32), cat(s).astype(np.float32), cat(lv).astype(np.int64), cat(gr).astype(np.int32))


def main():
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    b, s, lv, gr = [torch.from_numpy(a).to(dev) for a in candidates(rng)]
    reps = int(os.environ.get("REPS", "20"))
    for _ in range(reps):
        ops.batched_nms_grouped_sorted(b, s, lv, gr, 2, 5, 0.7, 2000, post=2000)
    torch.cuda.synchronize()
    for _ in range(reps):
        ops.batched_nms_grouped(b, s, lv, gr, 2, 5, 0.7, 2000)
    torch.cuda.synchronize()
    k1, n1 = ops.batched_nms_grouped_sorted(b, s, lv, gr, 2, 5, 0.7, 2000)
    k0, n0 = ops.batched_nms_grouped(b, s, lv, gr, 2, 5, 0.7, 2000)
    n = int(n0.item())
    assert int(n1.item()) == n and torch.equal(k0[:n], k1[:n])
    print("survivors", n)


if __name__ == "__main__":
    main()
