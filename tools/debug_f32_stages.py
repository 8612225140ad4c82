"""Per-stage error of the HipBackend("f32") trunk vs the CPU restatement (train-mode BN): each stage
fed the SAME input (local error) and the chained run (accumulated error)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]
os.environ.setdefault("MX_GRAPHS", "0")

import torch  # noqa: E402

from tests.test_gpu_model_f32 import _pair  # noqa: E402
from mx_det.conv import ACT_RELU  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    dev = torch.device("cuda:0")
    m, mc = _pair(dev, 1, float(os.environ.get("DAMP", "1")))
    m.train()
    mc.train()
    imgs, _ = synth_batch(30, 2, H=512, W=672)
    with torch.no_grad():
        il, _ = m.transform(list(imgs.to(dev)), None, m.be)
        ilc, _ = mc.transform(list(imgs), None, mc.be)
        print("input", rel(il.tensors[..., :3], ilc.tensors))
        bg, bc = m.backbone.body, mc.backbone.body
        xh = m.be.conv_bn(il.tensors, bg.conv1, bg.bn1, ACT_RELU)
        xc = mc.be.conv_bn(ilc.tensors, bc.conv1, bc.bn1, ACT_RELU)
        print("stem conv+bn+relu", rel(xh, xc))
        xh, xc = m.be.maxpool(xh, 3, 2, 1), mc.be.maxpool(xc, 3, 2, 1)
        print("maxpool", rel(xh, xc))
        for name in ("layer1", "layer2", "layer3", "layer4"):
            for i, (b1, b2) in enumerate(zip(getattr(bg, name), getattr(bc, name))):
                loc = rel(b1(xc.to(dev).contiguous(), m.be), b2(xc, mc.be))
                xh, xc = b1(xh, m.be), b2(xc, mc.be)
                print(f"{name}.{i}: local {loc:.3g}  chained {rel(xh, xc):.3g}  |x| {xc.abs().mean():.3g}")
        # BN statistics of the last block: compare batch mean/var of the pre-BN conv output
        blk_h, blk_c = bg.layer1[0], bc.layer1[0]
        from mx_det import conv as mc_
        x0 = xc
        import torch.nn.functional as F
        z = F.conv2d(ilc.tensors.permute(0, 3, 1, 2), bc.conv1.weight, None, 2, 3)
        print("stem pre-BN channel mean/std ratio max", (z.mean((0, 2, 3)).abs() / z.std((0, 2, 3))).max().item())


if __name__ == "__main__":
    main()
