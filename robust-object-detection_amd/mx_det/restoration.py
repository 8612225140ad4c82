"""U-Net restoration training (reference scripts/train_restoration.py) on the HIP U-Net.

Drop-in pieces with the reference's names and semantics:
  ssim(pred, target, window_size=11)      train_restoration.py:142-164 (11x11 Gaussian sigma 1.5, C1/C2)
  CombinedLoss(ssim_weight=0.3)           :167-178  L1 + 0.3 * (1 - SSIM)
  compute_psnr(pred, target)              :185-190
  RestorationDataset(img_dir, patch, is_train)  :54-111 -- (corrupted, clean) f32 CHW patches; here the
      host only decodes, crops and flips (uint8) and the corruption of a whole batch runs on the device
      (ops.corrupt_u8: noise / motion blur / low-res, one random choice per patch) via RestorationBatcher
  train_epoch / validate                  :199-215 / :161-175
The loss runs as the fused HIP SSIM kernels (mx_ssim.hip: window sums, SSIM map, its derivative maps
and the L1 term in one forward launch + a finish block; one backward launch); the U-Net
forward/backward is the HIP path (mx_det.unet).
"""
import math
import random
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

from . import ops

NOISE, BLUR, LOWRES = ops.CORRUPT_NOISE, ops.CORRUPT_BLUR, ops.CORRUPT_LOWRES  # augmentations.py ops


def ssim(pred, target, window_size=11):
    """Mean SSIM of NCHW f32 images in [0, 1] (train_restoration.py:142-164 semantics: Gaussian window
    σ 1.5, zero-padded 'same' window sums, C1 = 0.01², C2 = 0.03², no clipping), computed by the fused
    device kernel mx_ssim_l1_fwd; differentiable in `pred`."""
    return ops.ssim(pred, target, window_size)


class CombinedLoss(nn.Module):
    """The reference's restoration loss, mean absolute error + ssim_weight · (1 − SSIM)
    (train_restoration.py:167-178), as one fused forward launch and one fused backward launch."""

    def __init__(self, ssim_weight=0.3):
        super().__init__()
        self.ssim_weight = ssim_weight

    def forward(self, pred, target):
        return ops.ssim_l1_loss(pred, target, self.ssim_weight)


@torch.no_grad()
def compute_psnr(pred, target):
    """Peak signal-to-noise ratio in dB for images in [0, 1] (train_restoration.py:185-190); identical
    images report 100 dB as the reference does."""
    err = float(torch.mean(torch.square(pred.float() - target.float())))
    return 100.0 if err == 0.0 else -10.0 * math.log10(err)


def _read_rgb(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


def _resize_up(img, size):
    """cv2.resize(img, (max(w, size), max(h, size))) (bilinear) for images smaller than the patch."""
    h, w = img.shape[:2]
    if h >= size and w >= size:
        return img
    from PIL import Image
    return np.asarray(Image.fromarray(img).resize((max(w, size), max(h, size)), Image.BILINEAR))


class RestorationDataset(torch.utils.data.Dataset):
    """Clean uint8 RGB patches (H, W, 3) of the reference's crops; the corruption happens per batch on
    the device (RestorationBatcher). Train: random crop + 50 % horizontal flip; val: centre crop."""

    def __init__(self, img_dir, patch_size=256, is_train=True):
        self.img_paths = sorted(Path(img_dir).glob("*.jpg"))
        self.patch_size = patch_size
        self.is_train = is_train

    def __len__(self):
        return len(self.img_paths)

    def crop(self, img):
        img = _resize_up(img, self.patch_size)
        h, w = img.shape[:2]
        s = self.patch_size
        if self.is_train:
            y, x = random.randint(0, h - s), random.randint(0, w - s)
            p = img[y:y + s, x:x + s]
            if random.random() > 0.5:
                p = p[:, ::-1]
        else:
            y, x = (h - s) // 2, (w - s) // 2
            p = img[y:y + s, x:x + s]
        return np.ascontiguousarray(p)

    def __getitem__(self, idx):
        return torch.from_numpy(self.crop(_read_rgb(self.img_paths[idx])))


def collate_u8(batch):
    return torch.stack(batch)


class RestorationBatcher:
    """uint8 clean patches [B,S,S,3] (host) -> (corrupted, clean) f32 NCHW in [0, 1] on the device;
    each patch gets random.choice(noise, blur, lowres) as in _apply_random_corruption (:92-100)."""

    def __init__(self, dev):
        self.dev = dev

    def __call__(self, clean_u8):
        x = clean_u8.to(self.dev, non_blocking=True)
        codes = [random.choice((NOISE, BLUR, LOWRES)) for _ in range(x.shape[0])]
        cor = ops.corrupt_u8(x, codes, seed=random.getrandbits(62))
        to = lambda t: t.permute(0, 3, 1, 2).float().div_(255.0)  # noqa: E731
        return to(cor), to(x)


def train_epoch(model, loader, batcher, optimizer, criterion, log_every=200, epoch=0):
    model.train()
    total, n = 0.0, len(loader)
    for i, clean in enumerate(loader):
        corrupted, target = batcher(clean)
        restored = model(corrupted)
        loss = criterion(restored, target)
        optimizer.zero_grad(set_to_none=True)
        loss.backward()
        optimizer.step()
        v = float(loss.item())
        total += v
        if (i + 1) % log_every == 0 or (i + 1) == n:
            print(f"  [Epoch {epoch:03d}] batch {i + 1}/{n}  loss={v:.4f}", flush=True)
    return total / max(n, 1)


@torch.no_grad()
def validate(model, loader, batcher):
    model.eval()
    tp, ts, n = 0.0, 0.0, 0
    for clean in loader:
        corrupted, target = batcher(clean)
        restored = model(corrupted)
        b = corrupted.size(0)
        tp += compute_psnr(restored, target) * b
        ts += float(ssim(restored, target)) * b
        n += b
    return tp / max(n, 1), ts / max(n, 1)
