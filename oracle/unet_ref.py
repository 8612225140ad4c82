"""CPU restatement of the reference's restoration U-Net and its restore_image pipeline.

TEST INFRASTRUCTURE ONLY: used by tests/test_unet.py (checker of the HIP U-Net) and bench.py's
cpu_baseline leg of the restored-eval line. The product never imports it.
Follows restoration_net.py:17-106 (ConvBlock / DownBlock / UpBlock / RestorationUNet: residual output
clamp(x + out_conv(u), 0, 1)) and restore_testsets.py:53-79 (reflect pad to /16, /255, U-Net, *255,
clip, uint8 truncate, crop); pinned by tests/golden/unet_small.npz (outputs of the reference module).
"""
import numpy as np
import torch


def restore_cpu(model_ref, img_u8):
    """restore_testsets.py:53-79 restated on CPU with the reference U-Net golden model semantics
    (torch CPU fp32 eval forward of the same weights) and the oracle reflect pad."""
    from oracle import oracle as orc
    H, W, _ = img_u8.shape
    ph, pw = (16 - H % 16) % 16, (16 - W % 16) % 16
    p = orc.reflect_pad_u8(img_u8, ph, pw) if (ph or pw) else img_u8
    x = torch.from_numpy(p.astype(np.float32) / 255.0).permute(2, 0, 1)[None]
    with torch.no_grad():
        y = model_ref(x)[0].permute(1, 2, 0).numpy()
    y = (y * 255.0).clip(0, 255).astype(np.uint8)
    return y[:H, :W]


def torch_reference_unet(sd, channels):
    """Plain-torch CPU module with the reference layer structure (for the host-side restatement)."""
    import torch.nn as nn

    class CB(nn.Module):
        def __init__(s, i, o):
            super().__init__()
            s.block = nn.Sequential(nn.Conv2d(i, o, 3, padding=1, bias=False), nn.BatchNorm2d(o), nn.LeakyReLU(0.2),
                                    nn.Conv2d(o, o, 3, padding=1, bias=False), nn.BatchNorm2d(o), nn.LeakyReLU(0.2))

        def forward(s, x):
            return s.block(x)

    class Down(nn.Module):
        def __init__(s, i, o):
            super().__init__()
            s.conv, s.pool = CB(i, o), nn.MaxPool2d(2)

        def forward(s, x):
            f = s.conv(x)
            return s.pool(f), f

    class Up(nn.Module):
        def __init__(s, i, sk, o):
            super().__init__()
            s.up, s.conv = nn.ConvTranspose2d(i, i, 2, stride=2), CB(i + sk, o)

        def forward(s, x, skip):
            x = s.up(x)
            if x.shape[2:] != skip.shape[2:]:
                x = nn.functional.interpolate(x, size=skip.shape[2:], mode="bilinear", align_corners=False)
            return s.conv(torch.cat([x, skip], 1))

    class U(nn.Module):
        def __init__(s, c):
            super().__init__()
            c1, c2, c3, c4 = c
            s.down1, s.down2, s.down3, s.down4 = Down(3, c1), Down(c1, c2), Down(c2, c3), Down(c3, c4)
            s.bottleneck = CB(c4, c4)
            s.up4, s.up3, s.up2, s.up1 = Up(c4, c4, c3), Up(c3, c3, c2), Up(c2, c2, c1), Up(c1, c1, c1)
            s.out_conv = nn.Conv2d(c1, 3, 1)

        def forward(s, x):
            d1, s1 = s.down1(x)
            d2, s2 = s.down2(d1)
            d3, s3 = s.down3(d2)
            d4, s4 = s.down4(d3)
            b = s.bottleneck(d4)
            u = s.up1(s.up2(s.up3(s.up4(b, s4), s3), s2), s1)
            return torch.clamp(x + s.out_conv(u), 0.0, 1.0)

    u = U(channels)
    u.load_state_dict(sd)
    return u.eval()
