"""configs[2]'s multi-rank train path on one MI355X: two ranks (torch.distributed.run, gloo, both on
cuda:0) run three augmented train steps (train_frcnn_augmented.py:120-216, on-GPU corruption) through
mx_det.dp.DataParallel with the segmented trunk graphs. Rank 1's RoI head runs eagerly
(MX_HEAD_GRAPHS=0) while rank 0's replays its graph, so their hand-off hooks fire in different orders:
both must still issue the collectives in the same canonical order, and every trainable gradient after
sync_gradients must equal the mean of the ranks' single-process gradients (rel 2e-4, the
tests/test_gpu_dp.py bar: only summation order differs). The launcher is a child process; this
process makes no GPU call before it."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(170)
def test_two_rank_augmented_step_mixed_head_graphs(tmp_path):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    env.pop("MX_HEAD_GRAPHS", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(HERE, "_dp2_worker.py"),
           str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=160)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(2)]
    canonical = ["roi_heads", "fpn+rpn_head", "layer4", "layer3", "layer2"]
    assert res[0]["issued"] == res[1]["issued"], res  # same collectives, same order, every step
    for d in res:
        assert d["steps"] == 3
        for issued in d["issued"]:
            assert issued[:5] == canonical and set(issued[5:]) <= {"bucket"}, (d["rank"], issued)
        assert d["worst_loss"] <= 1e-5, d
        assert d["worst_grad"] < 2e-4, d
        assert d["trunk_seg_graphs"] == 1, d
    assert res[0]["head_graphs"] >= 1 and res[1]["head_graphs"] == 0, res
