"""Diagnostic: the captured proposal stage step by step with a device sync after each (fault localisation)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]
import torch  # noqa: E402


def step(msg, fn):
    t = time.time()
    out = fn()
    torch.cuda.synchronize()
    print(f"ok {msg} ({time.time() - t:.2f}s)", flush=True)
    return out


def main():
    from mx_det import frcnn
    from mx_det.data import synth_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(1024, 7)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    m = m.to(dev).train()
    imgs, tg = synth_batch(7, 2, H=448, W=640, device=dev)
    ld = step("forward 1 (captures)", lambda: m(imgs, tg))
    print({k: float(v) for k, v in ld.items()}, flush=True)
    step("backward 1", lambda: sum(ld.values()).backward())
    g = next(iter(m.__dict__["_mx_stage_graphs"].values()))
    obj, dl = g.static[0].clone(), g.static[1].clone()
    gt = [t.clone() for t in g.static[2:]]
    step("replay", lambda: g(obj, dl, gt))
    step("eager stage", lambda: g._run())
    for p in m.parameters():
        p.grad = None
    ld = step("forward 2", lambda: m(imgs, tg))
    step("backward 2", lambda: sum(ld.values()).backward())
    print("diag done", flush=True)


if __name__ == "__main__":
    main()
