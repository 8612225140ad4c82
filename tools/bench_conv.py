"""Conv kernel micro-benchmark on the shapes that dominate the FRCNN train step (bs=2, 800x1344).

    python tools/bench_conv.py [--reps 20]
Prints per shape and pass (fwd / dgrad / wgrad) the time per launch and TFLOP/s (bf16 MFMA peak 2500).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

os.environ.setdefault("MX_CONV_TUNE", "0")  # the forced launch settings below, not the tuner's picks

import torch  # noqa: E402

from mx_det import conv as mc  # noqa: E402

SHAPES = [  # name, N, H, W, C, K, k, stride, pad
    ("L3 1x1 256->1024 (M 8400)", 2, 50, 84, 256, 1024, 1, 1, 0),
    ("L4 3x3 256->256 (FPN P5, M 2100)", 2, 25, 42, 256, 256, 3, 1, 1),
    ("P6-ish 3x3 256->256 (M 546)", 2, 13, 21, 256, 256, 3, 1, 1),
    ("P2 3x3 256->256 (RPN/FPN)", 2, 200, 336, 256, 256, 3, 1, 1),
    ("P2 1x1 256->256 (FPN inner)", 2, 200, 336, 256, 256, 1, 1, 0),
    ("L2 1x1 128->512", 2, 100, 168, 128, 512, 1, 1, 0),
    ("L2 3x3 128->128", 2, 100, 168, 128, 128, 3, 1, 1),
    ("L3 3x3 256->256", 2, 50, 84, 256, 256, 3, 1, 1),
    ("L3 1x1 1024->256", 2, 50, 84, 1024, 256, 1, 1, 0),
    ("L4 1x1 2048->512", 2, 25, 42, 2048, 512, 1, 1, 0),
    ("box head 3x3 on 1024 RoIs", 1024, 7, 7, 256, 256, 3, 1, 1),
    ("FC6 as 7x7 valid conv (12544->1024)", 1024, 7, 7, 256, 1024, 7, 1, 0),
    ("L4 3x3 512->512", 2, 25, 42, 512, 512, 3, 1, 1),
    ("L3 1x1 256->1024", 2, 50, 84, 256, 1024, 1, 1, 0),
    ("stem 7x7 s2 (8->64)", 2, 800, 1344, 8, 64, 7, 2, 3),
    ("L3.0 3x3 s2 128->256 (dgrad s2)", 2, 100, 168, 256, 256, 3, 2, 1),
    # thin (memory-bound) 1x1 convs of the f32 step
    ("thin L1 1x1 64->256", 2, 200, 336, 64, 256, 1, 1, 0),
    ("thin L1 1x1 256->64", 2, 200, 336, 256, 64, 1, 1, 0),
    ("thin L2 1x1 512->128", 2, 100, 168, 512, 128, 1, 1, 0),
    ("thin L3 1x1 1024->256", 2, 50, 84, 1024, 256, 1, 1, 0),
    ("thin predictor 1024->40", 1024, 1, 1, 1024, 40, 1, 1, 0),
    ("thin RPN P2 cls+box 256->16", 2, 200, 336, 256, 16, 1, 1, 0),
]


GRAPH = False


def timeit(fn, reps):
    for _ in range(3):
        fn()
    if GRAPH:  # replay reps launches from one HIP graph: kernel time without host launch cost
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="7")
    ap.add_argument("--wgrad", default="0")
    ap.add_argument("--wtarget", default="0")
    ap.add_argument("--loaders", default="1")
    ap.add_argument("--tiles", default="0x0", help="comma list of BMTxBN overrides, 0x0 = auto")
    ap.add_argument("--splits", default="0", help="comma list of fwd/dgrad split-K caps, 0 = auto")
    ap.add_argument("--stages", default="0", help="comma list of buffer-kernel ring depths, 0 = auto")
    ap.add_argument("--korder", default="1", help="comma list of buffer-kernel K-tile orders (0 tap-, 1 channel-major)")
    ap.add_argument("--debug", default="0", help="comma list of mx_conv_set_debug values (1: no epilogue)")
    ap.add_argument("--graph", action="store_true", help="time launches replayed from a HIP graph")
    ap.add_argument("--planes", action="store_true",
                    help="f32: also time the pre-split (x3p) forms and the split passes they need")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "f32"),
                    help="f32: the precision-faithful bf16x3 kernels (TFLOP/s are f32-equivalent, peak 833)")
    args = ap.parse_args()
    global GRAPH
    GRAPH = args.graph
    import itertools
    from mx_det import _lib
    ints = lambda v: [int(x) for x in v.split(",")]  # noqa: E731
    for dbg, ko, ld, v, wv, wt, stg, sp, tl in itertools.product(ints(args.debug), ints(args.korder), ints(args.loaders), ints(args.variants),
                                                             ints(args.wgrad), ints(args.wtarget), ints(args.stages),
                                                             ints(args.splits), args.tiles.split(",")):
        bm, bn = [int(x) for x in tl.split("x")]
        _lib.call("mx_conv_set_tile", bm, bn)
        _lib.call("mx_conv_set_max_splits", sp)
        _lib.call("mx_conv_set_stages", stg)
        _lib.call("mx_conv_set_korder", ko)
        _lib.call("mx_conv_set_debug", dbg)
        _lib.call("mx_conv_set_loader", ld)
        _lib.call("mx_conv_set_variant", v)
        _lib.call("mx_conv_set_wgrad_variant", wv)
        _lib.call("mx_conv_set_wgrad_target", wt)
        print(f"== loader {ld} tile {tl} conv variant {v} wgrad variant {wv} wgrad target {wt} "
              f"max splits {sp} stages {stg} korder {ko} debug {dbg}", flush=True)
        run(args)


def run(args):
    dev = torch.device("cuda")
    tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
    for name, N, H, W, C, K, k, st, pd in SHAPES:
        if args.only and args.only not in name:
            continue
        dt = torch.float32 if args.dtype == "f32" else torch.bfloat16
        x = torch.randn(N, H, W, C, device=dev).to(dt)
        w = (torch.randn(K, C, k, k, device=dev) * 0.05)
        wk, wt = mc.pack_weight(w, C, (st, st), (pd, pd), dgrad=True, split=args.dtype == "f32")
        Ho, Wo = mc.out_hw(H, W, k, k, (st, st), (pd, pd))
        dy = torch.randn(N, Ho, Wo, K, device=dev).to(dt)
        fl = 2.0 * N * Ho * Wo * K * k * k * C
        es = 4 if args.dtype == "f32" else 2
        nb = {"fwd": es * (x.numel() + dy.numel()), "dgrad": es * (x.numel() + dy.numel()),
              "wgrad": es * (x.numel() + dy.numel()) + 4 * w.numel()}  # operands read once, output written once
        res = []
        cases = [("fwd", lambda: mc.conv_fwd(x, wk, (st, st), (pd, pd), stats=True)),
                 ("dgrad", lambda: mc.conv_dgrad(dy, wt, x.shape, k, k, (st, st), (pd, pd))),
                 ("wgrad", lambda: mc.conv_wgrad(dy, x, K, k, k, (st, st), (pd, pd)))]
        if args.planes and args.dtype == "f32" and C % 32 == 0 and K % 32 == 0:
            xp, dyp = mc.split_planes(x), mc.split_planes(dy)
            cases += [("split_x", lambda: mc.split_planes(x)), ("split_dy", lambda: mc.split_planes(dy)),
                      ("fwd_p", lambda: mc.conv_fwd(x, wk, (st, st), (pd, pd), stats=True, xp=xp)),
                      ("dgrad_p", lambda: mc.conv_dgrad(dy, wt, x.shape, k, k, (st, st), (pd, pd), dyp=dyp)),
                      ("wgrad_p", lambda: mc.wgrad_launch(mc.wgrad_prepare(dy, x, K, k, k, (st, st), (pd, pd),
                                                                          dyp=dyp, xp=xp)))]
        for kind, fn in cases:
            if kind not in tot:
                tot[kind] = [0, 0]
            ms = timeit(fn, args.reps)
            tot[kind][0] += fl
            tot[kind][1] += ms
            nbk = nb.get(kind.replace("_p", ""), 8 * (x.numel() if kind == "split_x" else dy.numel()))
            res.append(f"{kind} {ms * 1000:8.1f}us {fl / ms / 1e9:7.1f}TF {nbk / ms / 1e6:6.0f}GB/s")
        print(f"{name:34s} {fl / 1e9:7.1f} GF | " + " | ".join(res), flush=True)
    print("aggregate: " + " | ".join(f"{k} {v[0] / v[1] / 1e9:.1f} TF/s" for k, v in tot.items() if v[1]))


if __name__ == "__main__":
    main()
