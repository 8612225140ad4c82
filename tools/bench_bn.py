"""BatchNorm kernel micro-benchmark (train-mode fwd apply, bwd reduce + apply) on the step's shapes.

    python tools/bench_bn.py
Prints per shape the time per launch and the achieved algorithmic HBM GB/s (peak ~8000).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

from mx_det import _lib  # noqa: E402
from mx_det.conv import _p, _s  # noqa: E402

SHAPES = [(134400, 256), (33600, 512), (33600, 128), (8400, 1024), (8400, 256), (2100, 2048), (2100, 512),
          (50176, 256)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda")
    call = _lib.call
    for M, K in SHAPES:
        z = torch.randn(M, K, device=dev).bfloat16()
        y = torch.relu(z)
        dy = torch.randn(M, K, device=dev).bfloat16()
        mean = torch.zeros(K, device=dev)
        invstd = torch.ones(K, device=dev)
        gamma = torch.ones(K, device=dev)
        sums = torch.zeros(2, K, device=dev)
        out = torch.empty_like(z)
        out2 = torch.empty_like(z)
        res = []
        t = timeit(lambda: call("mx_bn_apply", _p(z), 1, M, K, _p(invstd), _p(mean), None, 1, _p(out), 1, _s()))
        res.append(("apply", t, M * K * 4))
        wsb = _lib.load().mx_bn_bwd_workspace(M, K)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
        coef = torch.empty(3, K, device=dev)
        t = timeit(lambda: call("mx_bn_bwd_reduce_ex", _p(dy), _p(y), _p(z), 1, M, K, 1, _p(mean), _p(invstd),
                                _p(gamma), _p(ws), wsb, _p(sums), _p(coef), _s()))
        res.append(("bwd_reduce", t, M * K * 6))
        t = timeit(lambda: call("mx_bn_bwd_apply_ex", _p(dy), _p(y), _p(z), 1, M, K, 1, _p(coef), _p(out), _p(out2),
                                _s()))
        res.append(("bwd_apply", t, M * K * 10))
        mb = (M + 63) // 64
        st = torch.randn(2, mb, K, device=dev).abs()
        fwb = _lib.load().mx_bn_finalize_workspace(mb, K)
        fws = torch.zeros(fwb, dtype=torch.uint8, device=dev)
        outs = [torch.empty(K, device=dev) for _ in range(4)]
        t = timeit(lambda: call("mx_bn_finalize_ex", _p(st), mb, K, M, _p(gamma), _p(mean), 1e-5, 0.1, None, None,
                                *[_p(o) for o in outs], _p(fws), fwb, _s()))
        res.append(("finalize", t, mb * K * 8))
        from mx_det import conv as mc
        t = timeit(lambda: mc.act_bias_bwd(dy, y, 1, K, True))
        res.append(("act_bias", t, M * K * 6))
        print(f"{M:7d}x{K:<5d} " + " | ".join(f"{n} {ms * 1000:6.1f}us {by / ms / 1e6:6.0f}GB/s" for n, ms, by in res),
              flush=True)


if __name__ == "__main__":
    main()
