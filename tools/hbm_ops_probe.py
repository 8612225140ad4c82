"""bench.py's hbm_ops section alone (RoIAlign fwd / bwd, proposal NMS on a real step's inputs), for a
rocprofv3 --kernel-trace run that checks the per-call figures against the kernels' own durations.

    rocprofv3 --kernel-trace --stats -d out -- python3 tools/hbm_ops_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "robust-object-detection_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mx_det.data import synth_batch  # noqa: E402


def main():
    dev = torch.device("cuda")
    if os.environ.get("MX_ROI_SPLIT"):
        from mx_det import _lib
        _lib.call("mx_roi_fwd_set_split", int(os.environ["MX_ROI_SPLIT"]))
    torch.manual_seed(42)
    model = bench.build_model(dev, precision="f32").train()
    opt = bench.make_optimizer(model)
    imgs, tg = synth_batch(0, 2, device=dev)
    for _ in range(2):
        bench.train_step(model, opt, imgs, tg)
    print(json.dumps(bench.hbm_ops_roofline(model, opt, imgs, tg), indent=1))


if __name__ == "__main__":
    main()
