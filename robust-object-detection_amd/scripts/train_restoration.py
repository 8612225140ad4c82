"""Train the restoration U-Net — `python -m scripts.train_restoration` (reference train_restoration.py).

Same constants (SEED 42, 60 epochs, batch 8, 256x256 patches, AdamW lr 1e-3 wd 1e-4, cosine to 1e-6,
L1 + 0.3 (1 - SSIM)), the same data roots, and the same outputs: experiments/restoration/history.jsonl
({epoch, train_loss, lr, val_psnr, val_ssim, elapsed_sec}; validation every 5 epochs and the last),
best.pth ({"model", "epoch", "psnr", "ssim"}) and last.pth ({"model", "epoch"}), so eval_restored /
restore_testsets load them unchanged. The U-Net forward/backward runs on the HIP kernels (f32 with
bf16x3 conv products by default, MX_PRECISION=bf16 for bf16); the corruption of each batch runs on
the device (mx_det.restoration.RestorationBatcher).
"""
import json
import os
import time
from pathlib import Path

import torch

from mx_det.engine import init_device, set_seed
from mx_det.restoration import (CombinedLoss, RestorationBatcher, RestorationDataset, collate_u8, train_epoch,
                                validate)
from mx_det.unet import RestorationUNet

SEED = 42
EPOCHS = int(os.environ.get("MX_EPOCHS", 60))
BATCH_SIZE = 8
PATCH_SIZE = 256
LR = 1e-3
NUM_WORKERS = 0
DATA_ROOT = Path("data/processed/visdrone_coco6")
TRAIN_IMG_DIR = DATA_ROOT / "images" / "train"
VAL_IMG_DIR = DATA_ROOT / "images" / "val"
OUT_DIR = Path("experiments/restoration")


def save_jsonl(path, record):
    with Path(path).open("a", encoding="utf-8") as f:
        f.write(json.dumps(record, ensure_ascii=False) + "\n")


def main(train_dir=TRAIN_IMG_DIR, val_dir=VAL_IMG_DIR, out_dir=OUT_DIR, epochs=EPOCHS):
    set_seed(SEED)
    dev, _, _ = init_device()
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    print(f"Device: {dev}\nTraining image restoration model (U-Net)", flush=True)
    train_ds = RestorationDataset(train_dir, PATCH_SIZE, is_train=True)
    val_ds = RestorationDataset(val_dir, PATCH_SIZE, is_train=False)
    train_loader = torch.utils.data.DataLoader(train_ds, batch_size=BATCH_SIZE, shuffle=True, num_workers=NUM_WORKERS,
                                               pin_memory=True, drop_last=True, collate_fn=collate_u8)
    val_loader = torch.utils.data.DataLoader(val_ds, batch_size=BATCH_SIZE, shuffle=False, num_workers=NUM_WORKERS,
                                             pin_memory=True, collate_fn=collate_u8)
    print(f"Train: {len(train_ds)} images, Val: {len(val_ds)} images", flush=True)
    model = RestorationUNet(channels=(32, 64, 128, 256)).to(dev)
    print(f"Model parameters: {sum(p.numel() for p in model.parameters()) / 1e6:.2f}M\n", flush=True)
    optimizer = torch.optim.AdamW(model.parameters(), lr=LR, weight_decay=1e-4)
    scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=epochs, eta_min=1e-6)
    criterion = CombinedLoss(ssim_weight=0.3)
    batcher = RestorationBatcher(dev)
    history, best_ckpt, last_ckpt = out_dir / "history.jsonl", out_dir / "best.pth", out_dir / "last.pth"
    best_psnr, t0 = 0.0, time.time()
    for epoch in range(1, epochs + 1):
        avg = train_epoch(model, train_loader, batcher, optimizer, criterion, epoch=epoch)
        scheduler.step()
        vp = vs = 0.0
        if epoch % 5 == 0 or epoch == epochs:
            vp, vs = validate(model, val_loader, batcher)
            print(f"[Epoch {epoch:03d}/{epochs}] loss={avg:.4f}  val_PSNR={vp:.2f}dB  val_SSIM={vs:.4f}", flush=True)
            if vp > best_psnr:
                best_psnr = vp
                torch.save({"model": model.state_dict(), "epoch": epoch, "psnr": vp, "ssim": vs}, best_ckpt)
                print(f"  -> New best PSNR: {vp:.2f}dB", flush=True)
        else:
            print(f"[Epoch {epoch:03d}/{epochs}] loss={avg:.4f}", flush=True)
        save_jsonl(history, {"epoch": epoch, "train_loss": avg, "lr": float(optimizer.param_groups[0]["lr"]),
                             "val_psnr": vp if vp > 0 else None, "val_ssim": vs if vs > 0 else None,
                             "elapsed_sec": int(time.time() - t0)})
        torch.save({"model": model.state_dict(), "epoch": epoch}, last_ckpt)
    print(f"\nTraining done. Total time: {(time.time() - t0) / 60:.1f} min\nBest PSNR: {best_psnr:.2f}dB", flush=True)
    return best_psnr


if __name__ == "__main__":
    main()
