"""Host -> HBM copy probe (run under rocprofv3 --kernel-trace --stats to count the blit dispatches per
copy): the JPEG coefficient copy of one 1333x800 4:2:0 image (1.6 M int16, pinned by torch's caching
host allocator) and the target tensors' small pinned copies, each timed on the host (issue cost) and
end to end.

    rocprofv3 --kernel-trace --stats -d gpurun_out/h2d -o h2d -- python3 tools/h2d_probe.py
"""
import time

import torch


def main():
    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    for n, label in ((1_600_000, "coefficients 3.2 MB"), (64, "target 256 B")):
        host = torch.empty(n, dtype=torch.int16, pin_memory=True)
        host.fill_(1)
        for _ in range(3):
            host.to(dev, non_blocking=True)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            host.to(dev, non_blocking=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{label}: issue {1e6 * (t1 - t0) / reps:.1f} us/copy, end-to-end {1e6 * (t2 - t0) / reps:.1f} us/copy",
              f"pinned={host.is_pinned()}", flush=True)


if __name__ == "__main__":
    main()
