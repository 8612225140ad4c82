"""torch.profiler op table of one steady-state train step (which torch-level ops still run per step).

    python tools/torch_ops_profile.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

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
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        bench.train_step(m, opt, imgs, tg)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="count", row_limit=40))
    print(prof.key_averages(group_by_stack_n=4).table(sort_by="count", row_limit=25))
    # where the device copies come from (aten::copy_ / to / contiguous call sites, 6 frames)
    for ev in prof.key_averages(group_by_stack_n=6):
        if ev.key in ("aten::copy_", "aten::clone", "aten::_to_copy", "aten::cat", "aten::index", "aten::nonzero",
                      "aten::item", "aten::_local_scalar_dense", "aten::mul", "aten::mul_", "aten::add_",
                      "aten::add"):
            print(f"{ev.key} x{ev.count}")
            for fr in ev.stack[:6]:
                print("    ", fr)


if __name__ == "__main__":
    main()
