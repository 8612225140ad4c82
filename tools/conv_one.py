"""Run one conv shape/pass repeatedly (for rocprofv3 --pmc passes).

    python tools/conv_one.py --shape 2,200,336,256,256,3,1,1 --pass fwd --reps 20 [--variant 7]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

from mx_det import _lib, conv as mc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="2,200,336,256,256,3,1,1")
    ap.add_argument("--pass", dest="kind", default="fwd")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "f32"))
    a = ap.parse_args()
    if a.variant >= 0:
        _lib.call("mx_conv_set_variant", a.variant)
    N, H, W, C, K, k, st, pd = [int(v) for v in a.shape.split(",")]
    dev = torch.device("cuda")
    dt = torch.float32 if a.dtype == "f32" else torch.bfloat16
    x = torch.randn(N, H, W, C, device=dev).to(dt)
    w = torch.randn(K, C, k, k, device=dev) * 0.05
    wk, wt = mc.pack_weight(w, C, (st, st), (pd, pd), dgrad=True, split=a.dtype == "f32")
    Ho, Wo = mc.out_hw(H, W, k, k, (st, st), (pd, pd))
    dy = torch.randn(N, Ho, Wo, K, device=dev).to(dt)
    fn = {"fwd": lambda: mc.conv_fwd(x, wk, (st, st), (pd, pd), stats=True),
          "dgrad": lambda: mc.conv_dgrad(dy, wt, x.shape, k, k, (st, st), (pd, pd)),
          "wgrad": lambda: mc.conv_wgrad(dy, x, K, k, k, (st, st), (pd, pd))}[a.kind]
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    print("done", a.kind, a.shape)


if __name__ == "__main__":
    main()
