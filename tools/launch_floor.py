"""Fixed per-launch cost in HIP-graph replay: a 1-block conv vs a tiny torch op (both replayed x50)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

from mx_det import conv as mc  # noqa: E402


def graph_time(fn, reps=50):
    for _ in range(3):
        fn()
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
    return a.elapsed_time(b) / reps * 1000


def main():
    dev = torch.device("cuda")
    t = torch.zeros(256, device=dev)
    print(f"torch add_ (1 block):        {graph_time(lambda: t.add_(1.0)):.2f} us")
    for (N, H, W, C, K, k) in [(1, 8, 8, 32, 64, 1), (1, 8, 8, 256, 64, 1), (1, 16, 16, 256, 128, 3),
                               (2, 13, 21, 256, 256, 3)]:
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = torch.randn(K, C, k, k, device=dev) * 0.05
        wk, wt = mc.pack_weight(w, C, (1, 1), (k // 2, k // 2), dgrad=True)
        f = lambda: mc.conv_fwd(x, wk, (1, 1), (k // 2, k // 2), stats=True)  # noqa: E731
        g = lambda: mc.conv_fwd(x, wk, (1, 1), (k // 2, k // 2))  # noqa: E731
        print(f"conv fwd M={N*H*W} N={K} K={C*k*k}: stats {graph_time(f):.2f} us, plain {graph_time(g):.2f} us")


if __name__ == "__main__":
    main()
