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
                      "aten::add", "aten::fill_", "aten::zero_", "aten::arange", "aten::where", "aten::lt",
                      "aten::uniform_", "aten::sum", "aten::scatter_", "aten::index_put_", "aten::stack",
                      "aten::sigmoid", "aten::_foreach_add_", "aten::div", "aten::sub"):
            print(f"{ev.key} x{ev.count}")
            for fr in ev.stack[:6]:
                print("    ", fr)


def call_sites():
    """Every device-launching aten op of one steady-state train step with the framework frames that
    issued it (a TorchDispatchMode records the Python stack at dispatch)."""
    import traceback
    from collections import Counter
    from torch.utils._python_dispatch import TorchDispatchMode
    skip = ("aten::view", "aten::detach", "aten::empty", "aten::as_strided", "aten::reshape", "aten::_unsafe_view",
            "aten::expand", "aten::select", "aten::slice", "aten::unsqueeze", "aten::t", "aten::alias",
            "aten::empty_strided", "aten::empty_like", "aten::narrow", "aten::squeeze", "aten::permute",
            "aten::transpose", "aten::lift_fresh", "aten::_to_copy", "aten::is_nonzero", "aten::set_")
    seen = Counter()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket).replace("aten.", "aten::")
            if name not in skip:
                fr = [f for f in traceback.extract_stack()[:-1] if "mx_det" in f.filename or "bench.py" in f.filename]
                where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:][::-1])
                if name in ("aten::copy_", "aten::zero_", "aten::fill_", "aten::zeros", "aten::cat") and args:
                    a0 = args[0][0] if isinstance(args[0], (list, tuple)) and args[0] else args[0]
                    if isinstance(a0, torch.Tensor):
                        where += f"  {tuple(a0.shape)} {str(a0.dtype).replace('torch.', '')}"
                seen[(name, where)] += 1
            return func(*args, **(kwargs or {}))

    dev = torch.device("cuda")
    torch.manual_seed(0)
    from mx_det import conv as mc
    orig_split = mc.split_planes
    splits = Counter()

    def logged_split(t, *a, **k):  # captured graphs replay these: log them while the steps capture
        fr = [f for f in traceback.extract_stack()[:-1] if "mx_det" in f.filename or "bench.py" in f.filename]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-4:][::-1])
        splits[(where, tuple(t.shape), torch.cuda.is_current_stream_capturing())] += 1
        return orig_split(t, *a, **k)
    mc.split_planes = logged_split
    m = bench.build_model(dev).train()
    opt = bench.make_optimizer(m)
    imgs, tg = synth_batch(0, 2, device=dev)
    for _ in range(4):
        bench.train_step(m, opt, imgs, tg)
    torch.cuda.synchronize()
    print("mx_split_planes calls during the warm-up steps (site, shape, inside a capture):")
    for (where, shp, cap), n in sorted(splits.items()):
        print(f"  {n:3d}  {'graph' if cap else 'eager'}  {shp}  {where}")
    with Log():
        bench.train_step(m, opt, imgs, tg)
    torch.cuda.synchronize()
    mc.split_planes = orig_split
    print("aten ops dispatched in one step (count, op, call site):")
    for (name, where), n in sorted(seen.items(), key=lambda kv: kv[0][1]):
        print(f"  {n:3d}  {name:28s} {where}")


if __name__ == "__main__":
    if "--sites" in sys.argv:
        call_sites()
    else:
        main()
