"""The RCCL path (torch.distributed backend "nccl" on ROCm) on one MI355X, each case in a fresh child
process (no test had ever used the nccl backend; configs[2]'s 8-GPU run depends on it).

* tests/_rccl_worker.py: a world-size-1 nccl group with device_id, mx_det.dp.DataParallel with the
  segmented backward graphs for three augmented steps (train_frcnn_augmented.py:159-177): the hand-off
  hooks fire in backward order, the collectives are issued in the canonical order, RCCL's AVG is used,
  losses and gradients equal the unwrapped model's (same segmented graphs) to 1e-6, the conv weight
  gradients are born in their bucket slots (only the small remainder is copied).
* bench.py --gpus 1 with MX_BENCH_DP=1: the bench's data-parallel leg (nccl group + DataParallel, every
  measurement leg through the wrapper) prints its usual JSON line.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
               PYTHONUNBUFFERED="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    return env


@pytest.mark.timeout(300)
def test_data_parallel_over_rccl(tmp_path):
    out = tmp_path / "rccl.json"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "_rccl_worker.py"), str(out)], env=_env(),
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = json.loads(out.read_text())
    assert r["backend"] == "nccl" and r["steps"] == 3
    assert "AVG" in r["reduce_op"], r["reduce_op"]
    assert r["trunk_seg_graphs"] == 1 and r["head_graphs"] >= 1, r
    # default segment boundaries (MX_DP_BOUNDS=23): FPN + RPN head + layer4 + layer3, then layer2; the
    # collectives still go out one per group, in the canonical order
    segs = ["fpn+rpn_head", "layer4", "layer3", "layer2"]
    assert r["order"] == ["layer3", "layer2"] * 3, r["order"]
    assert all(i == ["roi_heads"] + segs for i in r["issued"]), r["issued"]
    assert r["worst_loss"] <= 1e-6 and r["worst_grad"] <= 1e-6, r
    # every conv weight gradient written into its slot by its wgrad kernel; copied: BatchNorm affine,
    # biases, the RPN head's shared weights and the predictor -- a small remainder
    assert r["slot_grads"] + r["copied"][-1] == r["trainable"], r
    assert r["slot_grads"] >= 50, r


@pytest.mark.timeout(360)
def test_bench_line_under_nccl_group():
    env = _env()
    env["MX_BENCH_DP"] = "1"
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", "2", "--warmup", "2", "--precision", "f32",
                        "--no-eval-variant", "--no-augment-variant", "--no-cpu-baseline"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert rec["config"]["parallelism"] == "dp1 (nccl group, DataParallel)"
    assert "roofline" in rec and "hbm_ops" in rec


@pytest.mark.timeout(360)
def test_bench_line_carries_dp_variant():
    """The default N=1 line times the headline step a second time through DataParallel in a one-rank
    nccl group (dp_variant: the N-GPU code path's per-rank cost), then leaves the group."""
    env = _env()
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", "2", "--warmup", "2", "--precision", "f32",
                        "--no-eval-variant", "--no-augment-variant", "--no-cpu-baseline", "--no-roofline"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["config"]["parallelism"] == "dp1"
    dv = rec["dp_variant"]
    assert dv["parallelism"] == "dp1 (nccl group, DataParallel)" and dv["value"] > 0 and dv["ratio_to_headline"] > 0
