"""RPN per-level top-k micro-benchmark at the bench workload's shape (bs=2, 1344x800, pre=2000):
mx_level_topk (one launch) vs the per-level torch.topk loop it replaces. HIP-event timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

from mx_det import ops  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def torch_loop(ob, levels, k):
    tops, off = [], 0
    for n in levels:
        tops.append(ob[:, off:off + n].topk(min(k, n), dim=1)[1] + off)
        off += n
    return torch.cat(tops, 1)


def main():
    levels, k = [201600, 50400, 12600, 3150, 819], 2000
    ob = torch.randn(2, sum(levels), device="cuda")
    dists = {"randn": ob, "logits(0.01+-0.001)": 0.01 + 0.001 * torch.randn_like(ob),
             "uniform": torch.rand_like(ob)}
    for name, t in dists.items():
        print(f"{name:20s} proposals k=2000: {timeit(lambda: ops.level_topk(t, levels, k)):6.1f} us"
              f"   sampler k=256 one level: {timeit(lambda: ops.level_topk(t, [sum(levels)], 256)):6.1f} us",
              flush=True)
    print(f"mx_level_topk {timeit(lambda: ops.level_topk(ob, levels, k)):.1f} us")
    print(f"torch.topk loop {timeit(lambda: torch_loop(ob, levels, k)):.1f} us")
    for lv in ([201600], [50400], [3150]):
        o = ob[:, :lv[0]].contiguous()
        print(f"  level n={lv[0]}: mx {timeit(lambda: ops.level_topk(o, lv, k)):.1f} us")


if __name__ == "__main__":
    main()
