import sys, collections
sys.path[:0] = ["/root/repo", "/root/repo/robust-object-detection_amd"]
import torch, bench
from mx_det import conv as mc
from mx_det.data import synth_batch
dev = torch.device("cuda")
torch.manual_seed(42)
m = bench.build_model(dev, precision="f32").train()
opt = bench.make_optimizer(m)
imgs, tg = synth_batch(0, 2, device=dev)
for _ in range(2):
    bench.train_step(m, opt, imgs, tg)
cnt = collections.Counter()
for k, v in mc._tune_cache.items():
    cnt[(k[0], v)] += 1
for (kind, v), n in sorted(cnt.items(), key=lambda kv: (kv[0][0], -kv[1])):
    print(kind, v, n)
