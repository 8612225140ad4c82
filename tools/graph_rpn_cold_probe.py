"""Probe: capture the RPN proposal chain with cold per-shape caches (no eager warm-up), then replay
and compare with eager. Prints what happens at capture and at each replay."""
import sys
import os
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]
import torch  # noqa: E402
from mx_det import frcnn  # noqa: E402
from mx_det.backend import HipBackend  # noqa: E402

dev = torch.device("cuda")
be = HipBackend("f32")
rpn = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None).rpn.to(dev).train()
N, pad = 2, (800, 1344)
grid = [(200, 336), (100, 168), (50, 84), (25, 42), (13, 21)]
npl = [h * w * 3 for h, w in grid]
A = sum(npl)
sizes = [(800, 1333), (750, 1333)]
g = torch.Generator(device=dev).manual_seed(1)
obj = torch.randn(N, A, device=dev, generator=g)
dl = torch.randn(N, A, 4, device=dev, generator=g) * 0.2


def chain(o, d):
    anchors = rpn.anchor_generator(pad, grid, dev, be)
    props = be.box_decode(d.reshape(-1, 4), anchors.repeat(N, 1), frcnn.RPN_WEIGHTS).view(N, A, 4)
    return rpn.filter_proposals_padded(props, o, sizes, npl, be)


graph = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(graph):
        out = chain(obj, dl)
    print("cold capture: ok", flush=True)
except Exception:
    print("cold capture raised:\n" + "\n".join(traceback.format_exc().splitlines()[-12:]), flush=True)
    sys.exit(0)
for i in range(2):
    obj.copy_(torch.randn(N, A, device=dev, generator=g))
    graph.replay()
    ref = chain(obj, dl)
    torch.cuda.synchronize()
    print(f"replay {i}: equal {all(torch.equal(a, b) for a, b in zip(out, ref))}", flush=True)
