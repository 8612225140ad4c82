"""Rank body of tests/test_gpu_dp2.py (launched by torch.distributed.run, two ranks sharing cuda:0 over
gloo). configs[2]'s augmented train step (train_frcnn_augmented.py:159-177: on-GPU RandomCorruption,
forward, loss sum, backward) through mx_det.dp.DataParallel with the segmented trunk graphs, for three
steps. Rank 1 runs its RoI head eagerly (MX_HEAD_GRAPHS=0) while rank 0 replays the head graph, the
case where the two ranks' hooks fire in different orders. Each rank also runs the same step on an
unwrapped copy of the model (its single-process gradient); after sync_gradients every trainable
gradient must equal the mean over ranks of those single-process gradients. Writes one JSON result
per rank to argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _keys(seed):
    g = torch.Generator().manual_seed(seed)
    return lambda shape, device: torch.rand(shape, generator=g).to(device)


def _model(dev):
    from mx_det import frcnn
    torch.manual_seed(0)
    m = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    m.roi_heads.box_predictor = frcnn.FastRCNNPredictor(m.roi_heads.box_predictor.cls_score.in_features, 7)
    frcnn.set_trainable_layers(m.backbone.body, 3)
    return m.to(dev).train()


def main():
    out_dir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if rank == 1:
        os.environ["MX_HEAD_GRAPHS"] = "0"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    from mx_det import ops, frcnn
    from mx_det.data import synth_batch
    from mx_det.dp import DataParallel
    ref = _model(dev)
    m = _model(dev)
    m.load_state_dict(ref.state_dict())
    dp = DataParallel(m)
    imgs, tg = synth_batch(40 + 10 * rank, 6, H=512, W=672, device=dev)
    res = {"rank": rank, "worst_grad": 0.0, "worst_loss": 0.0, "issued": [], "steps": 0}
    for step in range(3):
        i, t = imgs[2 * step:2 * step + 2], tg[2 * step:2 * step + 2]
        # RandomCorruption(p=0.5) on the device: a fixed per-rank/step draw of one op per image
        codes = [(rank + step + k) % 4 for k in range(2)]
        i = ops.corrupt_u8(i, codes, seed=1000 * rank + step)
        for mod in (ref, m):
            mod.rpn.fg_bg_sampler.rand = _keys(7 + 100 * rank + step)
            mod.roi_heads.fg_bg_sampler.rand = _keys(8 + 100 * rank + step)
        lr = ref(i, t)
        ld = dp(i, t)
        for p in list(ref.parameters()) + list(m.parameters()):
            p.grad = None
        sum(lr.values()).backward()
        sum(ld.values()).backward()
        dp.sync_gradients()
        res["issued"].append(list(dp.last_issued))
        for k in lr:
            a, b = float(ld[k]), float(lr[k])
            res["worst_loss"] = max(res["worst_loss"], abs(a - b) / max(abs(b), 1e-30))
        avg = {}
        for (n, p), q in zip(m.named_parameters(), ref.parameters()):
            if not p.requires_grad:
                continue
            local = q.grad.detach().cpu()
            gl = [torch.zeros_like(local) for _ in range(world)]
            dist.all_gather(gl, local)
            avg[n] = (sum(gl) / world).to(dev)
            e = ((p.grad - avg[n]).norm() / avg[n].norm().clamp_min(1e-30)).item()
            if e > res["worst_grad"]:
                res["worst_grad"], res["worst_param"] = e, n
        with torch.no_grad():  # one identical update on every rank and both copies: weights stay equal
            for (n, p), q in zip(m.named_parameters(), ref.parameters()):
                if n in avg:
                    p.sub_(1e-3 * avg[n])
                    q.sub_(1e-3 * avg[n])
        res["steps"] += 1
        print(f"rank {rank} step {step} worst_grad {res['worst_grad']:.3e}", flush=True)
    res["head_graphs"] = len(m.roi_heads.__dict__.get("_mx_graphs", {}))
    res["trunk_seg_graphs"] = sum(isinstance(g, frcnn._SegGraphs) for g in m.__dict__.get("_mx_graphs", {}).values())
    torch.cuda.synchronize()
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
