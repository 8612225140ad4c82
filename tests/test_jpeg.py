"""Hybrid baseline-JPEG decode (mx_det.jpeg) against libjpeg-turbo itself (PIL's
decoder, the one behind coco_detection_dataset.py:23 Image.open().convert("RGB"); cv2.imread uses the
same library): bit-exact pixels.
CPU: the host entropy decoder of libmx_det (mx_jpeg_decode_coefs) + the oracle's libjpeg restatement of
the pixel stage (oracle/mx_oracle.c orc_jpeg_reconstruct) == PIL, over 4:2:0 / 4:2:2 / 4:4:4 / grey,
qualities 50..100, odd sizes, restart intervals, 16-bit quantisation tables, tiny images; unsupported
files (progressive) raise. GPU: mx_jpeg_reconstruct on the device == PIL on the same files."""
import io

import numpy as np
import pytest
from PIL import Image

CASES = [  # (H, W, quality, subsampling (PIL: 0 4:4:4, 1 4:2:2, 2 4:2:0), mode, restart MCUs or 0)
    (120, 160, 95, 2, "RGB", 0),
    (121, 163, 95, 2, "RGB", 0),
    (97, 131, 75, 1, "RGB", 0),
    (64, 80, 90, 0, "RGB", 0),
    (75, 93, 100, 2, "RGB", 0),
    (50, 66, 50, 2, "RGB", 0),
    (83, 57, 95, 2, "RGB", 4),
    (41, 29, 90, 1, "RGB", 3),
    (33, 47, 85, 0, "L", 0),
    (9, 5, 95, 2, "RGB", 0),
    (16, 3, 95, 2, "RGB", 0),
    (256, 384, 95, 2, "RGB", 0),
]


def _image(H, W, seed):
    from mx_det.data import synth_image
    img = synth_image(seed, max(H, 32), max(W, 32))[:H, :W]
    g = np.random.default_rng(seed)
    return np.clip(img.astype(np.int16) + g.integers(-40, 40, img.shape), 0, 255).astype(np.uint8)


def _encode(case, seed):
    H, W, q, sub, mode, rst = case
    im = Image.fromarray(_image(H, W, seed))
    if mode == "L":
        im = im.convert("L")
    b = io.BytesIO()
    kw = {"quality": q}
    if mode == "RGB":
        kw["subsampling"] = sub
    im.save(b, format="JPEG", **kw)
    data = b.getvalue()
    if rst:
        data = _with_restarts(data, rst)
    return data


def _with_restarts(data, interval):
    """Re-encode with restart markers through PIL's restart_marker_blocks when available; otherwise
    skip (older Pillow)."""
    im = Image.open(io.BytesIO(data))
    b = io.BytesIO()
    try:
        im.save(b, format="JPEG", quality=90, restart_marker_blocks=interval)
    except TypeError:
        pytest.skip("Pillow without restart_marker_blocks")
    out = b.getvalue()
    if b"\xff\xdd" not in out:
        pytest.skip("no DRI written")
    return out


def _pil(data):
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


@pytest.mark.parametrize("i", range(len(CASES)))
def test_entropy_decode_and_oracle_match_libjpeg(i):
    from mx_det import jpeg
    from oracle import oracle as orc
    data = _encode(CASES[i], i)
    info, coefs = jpeg.decode_coefs(data)
    assert (info.height, info.width) == CASES[i][:2]
    got = orc.jpeg_reconstruct(coefs, info)
    ref = _pil(data)
    assert np.array_equal(got, ref), (np.abs(got.astype(int) - ref).max(), (got != ref).mean())
    assert np.array_equal(orc.jpeg_reconstruct(coefs, info, bgr=True), ref[..., ::-1])


def test_unsupported_raises():
    from mx_det import jpeg
    b = io.BytesIO()
    Image.fromarray(_image(64, 64, 1)).save(b, format="JPEG", progressive=True)
    with pytest.raises(jpeg.JpegUnsupported):
        jpeg.parse(b.getvalue())
    with pytest.raises(ValueError):
        jpeg.parse(b"\x00\x01\x02\x03")


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(len(CASES)))
def test_device_decode_matches_libjpeg(dev, i):
    from mx_det import jpeg
    data = _encode(CASES[i], i)
    ref = _pil(data)
    assert np.array_equal(jpeg.decode(data, dev).cpu().numpy(), ref)
    assert np.array_equal(jpeg.decode(data, dev, bgr=True).cpu().numpy(), ref[..., ::-1])
