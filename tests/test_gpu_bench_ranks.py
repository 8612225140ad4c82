"""bench.py's N>1 entry with its DEFAULT legs (headline, roofline + hbm_ops, bf16 variant, augment
variant, eval variants, CPU baseline) on one MI355X: `bench.py --gpus 2` run directly starts the
torch.distributed.run child itself, both ranks on cuda:0 over gloo (MX_BENCH_REHEARSE=1; the real
N>1 run is one rank per GPU over RCCL). Every leg that all-reduces gradients must run on every rank,
or the ranks' collectives pair wrongly and the run hangs: the test asserts the run ends, with one JSON
line from rank 0 carrying n_gpus=2, roofline, hbm_ops and cpu_baseline. This process makes no GPU
call (the launcher is a child process). Reference: train_frcnn_augmented.py:120-216."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(560)
def test_bench_two_ranks_default_flags():
    # the launching shell's OMP_NUM_THREADS (16 on the GPU boxes) is left as it is: the CPU baseline must
    # pick its thread count itself (bench.host_threads), not inherit torchrun's per-rank default of 1
    env = dict(os.environ, MX_BENCH_REHEARSE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "2"], env=env, cwd=ROOT, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 4
    assert rec["value"] > 0 and rec["steps"] == 2 and rec["warmup"] == 2
    for key in ("roofline", "hbm_ops", "cpu_baseline", "bf16_variant", "augment_variant", "eval_variant",
                "eval_restored_variant"):
        assert key in rec, key
    assert rec["roofline"]["frac"] > 0 and "roi_align_fwd" in rec["hbm_ops"]
    assert rec["cpu_baseline"]["value"] > 0 and rec["cpu_baseline"]["kind"] == "port"
    assert rec["cpu_baseline"]["cores"] > 1, rec["cpu_baseline"]
    assert "roofline" in rec["bf16_variant"]
