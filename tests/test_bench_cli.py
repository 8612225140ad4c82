"""bench.py's rank plumbing without a GPU: `--gpus N` with no WORLD_SIZE starts exactly one
torch.distributed.run child (same arguments, 127.0.0.1 rendezvous) and exits with its code before any
HIP call; a WORLD_SIZE that disagrees with --gpus is refused."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_world_size_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_gpus_n_spawns_launcher(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    def no_cuda():
        raise AssertionError("HIP touched before the launcher")

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(bench.torch.cuda, "is_available", no_cuda)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3", "--warmup", "1"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-6:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]
    assert cmd[cmd.index("--nnodes=1") + 4].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_cpu_baseline_threads_ignore_torchrun_default(monkeypatch):
    """torch.distributed.run sets OMP_NUM_THREADS=1 in every rank when the variable was unset,
    so a CPU baseline reading torch.get_num_threads() at N>1 timed ONE thread. bench.host_threads()
    picks the host's cores itself."""
    import bench
    for k in ("MX_CPU_THREADS", "MX_HOST_THREADS", "OMP_NUM_THREADS", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    ncpu = len(os.sched_getaffinity(0))
    assert bench.host_threads() == ncpu
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("OMP_NUM_THREADS", "1")  # torchrun's default: not a request
    assert bench.host_threads() == ncpu
    monkeypatch.setenv("MX_HOST_THREADS", "16")  # the launching shell's setting, passed on by _launch_ranks
    assert bench.host_threads() == 16
    monkeypatch.setenv("MX_CPU_THREADS", "6")
    assert bench.host_threads() == 6
    monkeypatch.delenv("MX_CPU_THREADS")
    monkeypatch.delenv("MX_HOST_THREADS")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.host_threads() == 3
    with bench._threads(2) as n:
        assert n == 2
    assert bench.torch.get_num_threads() != 2 or ncpu == 2


def test_launcher_passes_the_shell_thread_count(monkeypatch):
    import bench
    seen = {}
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: seen.update(env=env) or 0)
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    monkeypatch.delenv("MX_HOST_THREADS", raising=False)
    bench._launch_ranks(2)
    assert seen["env"]["MX_HOST_THREADS"] == "16"
