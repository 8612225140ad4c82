"""Restoration U-Net (scripts/restoration_net.py) on the libmx_det HIP kernels: eval forward and
training (train_restoration.py:199-205).

Same module tree and state_dict keys as the reference (down1.conv.block.{0,1,3,4}.*, up4.up.*,
out_conv.*; 118 entries incl. BN buffers), so experiments/restoration/best.pth loads unchanged.
Eval forward, NHWC activations: f32 with bf16x3 conv products (precision "f32", the default: the
reference runs the U-Net in fp32, restore_testsets.py:64-68) or bf16 ("bf16"):
  ConvBlock  = 2 x [conv3x3 with eval-BN folded into weights+bias, LeakyReLU(0.2) fused in the epilogue]
  MaxPool2d(2), ConvTranspose2d(2, s2) as a 1x1 MFMA conv to 4*Cout channels + fused pixel-shuffle/concat,
  out_conv 1x1 (f32 out) + clamp(x + residual, 0, 1).
Training (module in train mode, grad enabled): the same kernels as the detector's trunk --
  ConvBlock  = 2 x ConvBNAct (batch-statistics BN + LeakyReLU(0.2) fused, running stats updated),
  MaxPool2d(2) with argmax backward, ConvTranspose2d(2, s2) = ConvAct 1x1 GEMM to (i, j, co) channels
  whose weight view keeps autograd to up.weight / up.bias, up_concat with its HIP backward,
  out_conv ConvAct (f32 out); weights of all 3x3 / 1x1 convs repacked in one launch per step.
restore_u8() is restore_testsets.py:53-79 on device: reflect-pad to /16, /255, U-Net, *255, clip,
truncate, crop — uint8 in, uint8 out, no host round trip.
"""
import ctypes

import torch
import torch.nn.functional as F
from torch import nn

from . import conv as mc
from . import ops
from . import _lib
from ._lib import call


def _s():
    return _lib.stream()


def _p(t):
    return t.data_ptr() if t is not None else None


def _wk(w, cin, x):
    """The conv operand of an f32 [K,C,R,S] weight for activations like x: hi/lo split planes
    (device pack kernel) for f32 x, a KRSC bf16 copy for bf16 x."""
    if mc.is_x3(x):
        return mc.pack_weight(w.contiguous(), cin, split=True)[0]
    return mc.weight_krsc(w, cin)


def _training(mod):
    return mod.training and torch.is_grad_enabled()


class _UpConcat(torch.autograd.Function):
    """up [N,H,W,4*Cu] (ConvTranspose2d as a 1x1 conv, channel = (i, j, co)) + skip -> [N,2H,2W,Cu+Cs]."""

    @staticmethod
    def forward(ctx, u, skip, cu):
        N, H, W, _ = u.shape
        skip = skip.contiguous()
        cs = skip.shape[3]
        cat = torch.empty((N, 2 * H, 2 * W, cu + cs), dtype=u.dtype, device=u.device)
        call("mx_up_concat", _p(u.contiguous()), _p(skip), mc.dcode(u), N, H, W, cu, cs, _p(cat), _s())
        ctx.cfg = (N, H, W, cu, cs)
        return cat

    @staticmethod
    def backward(ctx, g):
        N, H, W, cu, cs = ctx.cfg
        g = g.contiguous()
        gu = torch.empty((N, H, W, 4 * cu), dtype=g.dtype, device=g.device)
        gs = torch.empty((N, 2 * H, 2 * W, cs), dtype=g.dtype, device=g.device) if ctx.needs_input_grad[1] else None
        call("mx_up_concat_bwd", _p(g), mc.dcode(g), N, H, W, cu, cs, _p(gu), _p(gs), _s())
        return gu, gs, None


class ConvBlock(nn.Module):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv2d(in_ch, out_ch, 3, padding=1, bias=False), nn.BatchNorm2d(out_ch), nn.LeakyReLU(0.2, inplace=True),
            nn.Conv2d(out_ch, out_ch, 3, padding=1, bias=False), nn.BatchNorm2d(out_ch), nn.LeakyReLU(0.2, inplace=True))

    def forward(self, x):
        if _training(self):  # batch-statistics BN, fused LeakyReLU, autograd through the HIP kernels
            for ci, bi in ((0, 1), (3, 4)):
                x = mc.conv_bn(x, self.block[ci], self.block[bi], mc.ACT_LEAKY)
            return x
        for ci, bi in ((0, 1), (3, 4)):
            c, b = self.block[ci], self.block[bi]

            def make(c=c, b=b, x=x):
                w, bias = mc.fold_bn(c, b)
                return _wk(w, x.shape[3], x), bias
            wk, bias = mc.cached_operand(c, ("fold", id(b), x.shape[3], x.dtype), mc._fold_tensors(c, b), make)
            x = mc.conv_fwd(x, wk, c.stride, c.padding, bias=bias, act=mc.ACT_LEAKY)
        return x


def _maxpool2(x):
    N, H, W, C = x.shape
    y = torch.empty((N, H // 2, W // 2, C), dtype=x.dtype, device=x.device)
    call("mx_maxpool_fwd", _p(x.contiguous()), mc.dcode(x), N, H, W, C, 2, 2, 0, _p(y), None, _s())
    return y


class DownBlock(nn.Module):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = ConvBlock(in_ch, out_ch)
        self.pool = nn.MaxPool2d(2)

    def forward(self, x):
        feat = self.conv(x)
        if _training(self):
            from .backend import _MaxPool
            return _MaxPool.apply(feat, 2, 2, 0), feat
        return _maxpool2(feat), feat


class UpBlock(nn.Module):
    def __init__(self, in_ch, skip_ch, out_ch):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_ch, in_ch, 2, stride=2)
        self.conv = ConvBlock(in_ch + skip_ch, out_ch)

    def forward(self, x, skip):
        N, H, W, C = x.shape
        if _training(self):
            wt = self.up.weight                                   # [Cin, Cout, 2, 2]
            Cout = wt.shape[1]
            w1 = wt.permute(2, 3, 1, 0).reshape(4 * Cout, C, 1, 1)   # output channel = (i, j, co)
            u = mc.ConvAct.apply(x, w1, self.up.bias.repeat(4), (1, 1), (0, 0), mc.ACT_NONE, None)
            if (2 * H, 2 * W) == (skip.shape[1], skip.shape[2]):
                return self.conv(_UpConcat.apply(u, skip, Cout))
            up = u.view(N, H, W, 2, 2, Cout).permute(0, 1, 3, 2, 4, 5).reshape(N, 2 * H, 2 * W, Cout)
            up = F.interpolate(up.permute(0, 3, 1, 2), size=tuple(skip.shape[1:3]), mode="bilinear",
                               align_corners=False).permute(0, 2, 3, 1)
            return self.conv(torch.cat([up, skip], dim=3).contiguous())
        Cout = self.up.weight.shape[1]

        def make():  # the transposed conv as one 1x1 GEMM: weight rows = (i, j, co)
            wt = self.up.weight.detach()                 # [Cin, Cout, 2, 2]
            w1 = wt.permute(2, 3, 1, 0).reshape(4 * Cout, C, 1, 1)
            return _wk(w1, C, x), self.up.bias.detach().repeat(4).float().contiguous()
        wk1, b1 = mc.cached_operand(self.up, ("up", C, x.dtype), [self.up.weight, self.up.bias], make)
        u = mc.conv_fwd(x, wk1, (1, 1), (0, 0), bias=b1)   # [N, H, W, 4*Cout]
        if (2 * H, 2 * W) == (skip.shape[1], skip.shape[2]):
            cat = torch.empty((N, 2 * H, 2 * W, Cout + skip.shape[3]), dtype=x.dtype, device=x.device)
            call("mx_up_concat", _p(u), _p(skip.contiguous()), mc.dcode(x), N, H, W, Cout, skip.shape[3], _p(cat),
                 _s())
        else:
            # odd spatial size (restoration_net.py:53-55): bilinear fix-up of the upsampled map
            up = u.view(N, H, W, 2, 2, Cout).permute(0, 1, 3, 2, 4, 5).reshape(N, 2 * H, 2 * W, Cout)
            up = F.interpolate(up.permute(0, 3, 1, 2).float(), size=tuple(skip.shape[1:3]), mode="bilinear",
                               align_corners=False).permute(0, 2, 3, 1).to(x.dtype)
            cat = torch.cat([up, skip], dim=3).contiguous()
        return self.conv(cat)


class RestorationUNet(nn.Module):
    def __init__(self, channels=(32, 64, 128, 256), precision=None):
        super().__init__()
        from .backend import default_precision
        self.precision = precision or default_precision()
        self.act_dtype = torch.float32 if self.precision == "f32" else torch.bfloat16
        c1, c2, c3, c4 = channels
        self.down1 = DownBlock(3, c1)
        self.down2 = DownBlock(c1, c2)
        self.down3 = DownBlock(c2, c3)
        self.down4 = DownBlock(c3, c4)
        self.bottleneck = ConvBlock(c4, c4)
        self.up4 = UpBlock(c4, c4, c3)
        self.up3 = UpBlock(c3, c3, c2)
        self.up2 = UpBlock(c2, c2, c1)
        self.up1 = UpBlock(c1, c1, c1)
        self.out_conv = nn.Conv2d(c1, 3, 1)

    def residual_nhwc(self, x8):
        """x8: NHWC [N,H,W,8] of the activation dtype (image in [0,1] in channels 0..2) -> residual f32
        [N,H,W,3]."""
        d1, s1 = self.down1(x8)
        d2, s2 = self.down2(d1)
        d3, s3 = self.down3(d2)
        d4, s4 = self.down4(d3)
        b = self.bottleneck(d4)
        u = self.up1(self.up2(self.up3(self.up4(b, s4), s3), s2), s1)
        oc = self.out_conv
        if _training(self):
            return mc.ConvAct.apply(u, oc.weight, oc.bias, (1, 1), (0, 0), mc.ACT_NONE, torch.float32)
        wk, b = mc.cached_operand(oc, ("out", u.shape[3], u.dtype), [oc.weight, oc.bias],
                                  lambda: (_wk(oc.weight.detach(), u.shape[3], u), oc.bias.detach().float()))
        return mc.conv_fwd(u, wk, (1, 1), (0, 0), bias=b, out_dtype=torch.float32)

    def _prepare(self):
        """Training: every 3x3 / 1x1 conv weight repacked (hi/lo planes in f32 mode) in one launch."""
        pk = self.__dict__.get("_mx_packer")
        if pk is None:
            pk = self.__dict__["_mx_packer"] = mc.WeightPacker()
            for m in self.modules():
                if isinstance(m, nn.Conv2d):
                    pk.register(m.weight, m.stride, m.padding, True, split=self.precision == "f32")
        mc.set_packer(pk)
        pk.refresh()

    def forward(self, x):
        """Reference contract: x [N,3,H,W] f32 in [0,1] -> clamp(x + residual, 0, 1) [N,3,H,W] f32.
        In train mode with grad enabled the output carries autograd through the HIP kernels."""
        if not _training(self):
            with torch.no_grad():
                x8 = F.pad(x.permute(0, 2, 3, 1), (0, 5)).to(self.act_dtype).contiguous()
                r = self.residual_nhwc(x8)
                return torch.clamp(x + r.permute(0, 3, 1, 2), 0.0, 1.0)
        if not x.is_cuda:
            raise RuntimeError("RestorationUNet training runs on the HIP device (no CPU path)")
        self._prepare()
        x8 = F.pad(x.detach().permute(0, 2, 3, 1), (0, 5)).to(self.act_dtype).contiguous()
        r = self.residual_nhwc(x8)
        return torch.clamp(x + r.permute(0, 3, 1, 2), 0.0, 1.0)

    @torch.no_grad()
    def restore_u8(self, img_u8):
        """restore_testsets.py:53-79 on device. img_u8 [B,H,W,3] uint8 (RGB) -> restored uint8 [B,H,W,3]."""
        B, H, W, _ = img_u8.shape
        ph, pw = (16 - H % 16) % 16, (16 - W % 16) % 16
        Hp, Wp = H + ph, W + pw
        src = img_u8.contiguous()
        if ph or pw:
            pad = torch.empty((B, Hp, Wp, 3), dtype=torch.uint8, device=img_u8.device)
            call("mx_reflect_pad_u8", _p(src), B, H, W, 3, Hp, Wp, _p(pad), _s())
            src = pad
        x8 = ops.normalize_pad(src, (Hp, Wp), channels=8, dtype=self.act_dtype, mean=(0.0, 0.0, 0.0),
                               std=(1.0, 1.0, 1.0))
        r = self.residual_nhwc(x8)
        out = torch.empty((B, H, W, 3), dtype=torch.uint8, device=img_u8.device)
        call("mx_restore_finish", _p(src), B, Hp, Wp, _p(r), H, W, _p(out), _s())
        return out
