import os, sys, warnings, traceback
sys.path[:0] = ["/root/repo", "/root/repo/robust-object-detection_amd"]
import torch, bench
from mx_det.data import synth_batch
dev = torch.device("cuda")
torch.manual_seed(42)
m = bench.build_model(dev, precision="f32").train()
opt = bench.make_optimizer(m)
imgs, tg = synth_batch(0, 2, device=dev)
for _ in range(3):
    bench.train_step(m, opt, imgs, tg)
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("warn")
seen = []
def hook(message, category, filename, lineno, file=None, line=None):
    st = [f for f in traceback.extract_stack() if "robust-object-detection_amd" in f.filename or "bench.py" in f.filename]
    seen.append((str(message)[:60], [f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:]]))
warnings.showwarning = hook
warnings.simplefilter("always")
bench.train_step(m, opt, imgs, tg)
torch.cuda.set_sync_debug_mode(0)
for s in seen:
    print(s)
print(len(seen), "syncs")
