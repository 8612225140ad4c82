"""Per-step weight pack (mx_conv_pack_batched) micro-benchmark on the bench model's conv weights.

    python tools/bench_pack.py
Prints the time per launch and the algorithmic HBM rate: f32 reads (once per tile kind that is
packed) + bf16 writes of both operand layouts.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402
from torch.autograd.graph import increment_version  # noqa: E402

from mx_det import frcnn  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    m = m.to(dev).train()
    imgs, tg = synth_batch(0, 2, device=dev)
    sum(m(imgs, tg).values()).backward()
    pk = m.__dict__["_mx_packer_" + m.be.precision]
    es = [pk.entries[k] for k in pk.order]
    ws = [e.w for e in es]
    nbytes = sum(e.w.numel() * 4 + e.wk.numel() * 2 + (e.wt.numel() * 2 + e.w.numel() * 4 if e.wt is not None else 0)
                 for e in es)

    def step():
        increment_version(ws)
        pk.refresh()

    for _ in range(3):
        step()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    a.record()
    for _ in range(reps):
        step()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"pack: {len(es)} weights, {nbytes / 1e6:.1f} MB algorithmic, {ms * 1e3:.1f} us/launch, "
          f"{nbytes / ms / 1e6:.0f} GB/s")


if __name__ == "__main__":
    main()
