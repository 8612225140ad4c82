"""Time the ResNet stem at the headline shape (bs=2, 1344x800 padded image, 3 real channels padded to 8):
mx_conv2d_stem_x3 vs the generic x3 conv (MX_STEM_KERNEL=0), and the frozen-stem BN apply + max pool
fused (mx_bn_act_maxpool) vs bn_apply + maxpool."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "robust-object-detection_amd"))
from mx_det import conv as mc  # noqa: E402
from mx_det.backend import _MaxPool  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
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
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.zeros(2, 800, 1344, 8, device=dev)
    x[..., :3] = torch.randn(2, 800, 1344, 3, device=dev)
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.05
    wk, _ = mc.pack_weight(w, 8, (2, 2), (3, 3), split=True)
    for v in ("0", "1"):
        os.environ["MX_STEM_KERNEL"] = v
        t = timeit(lambda: mc.conv_fwd(x, wk, (2, 2), (3, 3), stats=True, cin=3))
        print(f"MX_STEM_KERNEL={v} stem_conv_us={t:.1f}", flush=True)
    os.environ["MX_STEM_KERNEL"] = "1"
    conv = mc.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    bn = mc.BatchNorm2d(64).to(dev)
    for p in list(conv.parameters()) + list(bn.parameters()):
        p.requires_grad_(False)
    t1 = timeit(lambda: mc.conv_bn_act_maxpool(x, conv, bn, mc.ACT_RELU, 3, 2, 1))
    t0 = timeit(lambda: _MaxPool.apply(mc.conv_bn(x, conv, bn, mc.ACT_RELU), 3, 2, 1))
    print(f"stem_total_us fused={t1:.1f} unfused={t0:.1f}", flush=True)


if __name__ == "__main__":
    main()
