"""Hybrid baseline-JPEG decode (mx_det.jpeg) against libjpeg-turbo itself (PIL's
decoder, the one behind coco_detection_dataset.py:23 Image.open().convert("RGB"); cv2.imread uses the
same library): bit-exact pixels.
CPU: the host entropy decoder of libmx_det (mx_jpeg_decode_coefs) + the oracle's libjpeg restatement of
the pixel stage (oracle/mx_oracle.c orc_jpeg_reconstruct) == PIL, over 4:2:0 / 4:2:2 / 4:4:4 / grey,
qualities 50..100, odd sizes, restart intervals, 16-bit quantisation tables, tiny images; unsupported
files (progressive) raise. GPU: mx_jpeg_reconstruct on the device == PIL on the same files."""
import io

import numpy as np
import torch
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


# ------------------------------------------------------------------ malformed / unusual streams
def _segs(data):
    """[(marker, offset of 0xFF, segment end)] of the header segments up to and including SOS."""
    out, i = [], 2
    while i + 4 <= len(data):
        m = data[i + 1]
        ln = (data[i + 2] << 8) | data[i + 3]
        out.append((m, i, i + 2 + ln))
        if m == 0xDA:
            break
        i += 2 + ln
    return out


def _base():
    b = io.BytesIO()
    Image.fromarray(_image(48, 64, 3)).save(b, format="JPEG", quality=90)
    return bytearray(b.getvalue())


def test_oversubscribed_dht_rejected_before_table_writes():
    from mx_det import jpeg
    d = _base()
    m, o, e = next(s for s in _segs(d) if s[0] == 0xC4)
    bits = o + 5  # first table's 16 counts start after FF C4, length, Tc/Th
    k = next(l for l in range(16) if d[bits + l] >= 3 and l > 0)
    d[bits + 0] += 3          # three more 1-bit codes (only two exist)...
    d[bits + k] -= 3          # ...same total, so only the code-space check can catch it
    with pytest.raises(ValueError):  # checked where a scan uses the table, as libjpeg does
        jpeg.decode_coefs(bytes(d))
    with pytest.raises(OSError):
        _pil(bytes(d))
    # the entropy decoder's own table builder refuses it too (a caller handing it a crafted info)
    good = _base()
    info = jpeg.parse(bytes(good))
    for t in range(8):
        info.hbits[t][1] = 255
    with pytest.raises(ValueError):
        jpeg.decode_coefs(bytes(good), info)


def test_complete_code_space_dht_rejected_like_libjpeg():
    """A table whose codes fill the whole code space (Kraft sum 1: the last code is all ones) is legal
    prefix code but libjpeg's jpeg_make_d_derived_tbl rejects it (`code >= 1 << si`): so must we."""
    from mx_det import jpeg
    d = _base()
    m, o, e = next(s for s in _segs(d) if s[0] == 0xC4)
    bits = o + 5
    counts = list(d[bits:bits + 16])
    assert counts == [0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], counts  # T.81 K.3 DC luminance
    assert sum(c / 2 ** (l + 1) for l, c in enumerate(counts)) == 1 - 2 ** -9
    d[bits + 7] += 1  # one 9-bit code becomes an 8-bit one: Kraft sum exactly 1, same total
    d[bits + 8] -= 1
    with pytest.raises(OSError):
        _pil(bytes(d))
    with pytest.raises(ValueError):
        jpeg.decode_coefs(bytes(d))


def test_short_sos_and_undefined_quant_table_rejected():
    from mx_det import jpeg
    d = _base()
    m, o, e = next(s for s in _segs(d) if s[0] == 0xDA)
    bad = bytes(d[:o + 2]) + b"\x00\x02" + bytes(d[o + 4:])
    with pytest.raises((ValueError, jpeg.JpegUnsupported)):
        jpeg.parse(bad)
    d = _base()
    m, o, e = next(s for s in _segs(d) if s[0] in (0xC0, 0xC1))
    d[o + 4 + 6 + 2] = 3  # component 0 -> quant table 3, never defined
    with pytest.raises(ValueError):
        jpeg.parse(bytes(d))


def test_huge_header_goes_to_host_and_truncated_stream_does_not_crash():
    from mx_det import jpeg
    d = _base()
    m, o, e = next(s for s in _segs(d) if s[0] in (0xC0, 0xC1))
    d[o + 5:o + 9] = b"\xff\xff\xff\xff"  # 65535 x 65535
    with pytest.raises(jpeg.JpegUnsupported):
        jpeg.parse(bytes(d))
    d = bytes(_base())
    for cut in (len(d) // 2, len(d) - 40, _segs(d)[-1][2] + 3):
        try:
            jpeg.decode_coefs(d[:cut])
        except ValueError:
            pass


def _without_jfif(d):
    m, o, e = next(s for s in _segs(d) if s[0] == 0xE0)
    return d[:o] + d[e:]


def test_rgb_coded_frames_go_to_host():
    """libjpeg default_decompress_parms: no JFIF + Adobe transform 0, or no marker + component IDs
    'R','G','B' -> RGB (no colour transform). Those are left to PIL; JFIF + Adobe stays YCbCr."""
    from mx_det import jpeg
    adobe0 = b"\xff\xee\x00\x0eAdobe\x00\x64\x00\x00\x00\x00\x00"
    d = bytes(_base())
    nj = _without_jfif(d)
    with pytest.raises(jpeg.JpegUnsupported):
        jpeg.parse(nj[:2] + adobe0 + nj[2:])
    rgb = bytearray(nj)
    m, o, e = next(s for s in _segs(rgb) if s[0] in (0xC0, 0xC1))
    for c, cid in enumerate((82, 71, 66)):
        rgb[o + 4 + 6 + 3 * c] = cid
    m, o, e = next(s for s in _segs(rgb) if s[0] == 0xDA)
    for c, cid in enumerate((82, 71, 66)):
        rgb[o + 5 + 2 * c] = cid
    with pytest.raises(jpeg.JpegUnsupported):
        jpeg.parse(bytes(rgb))
    # JFIF present: YCbCr whatever the Adobe flag says -> decoded here, equal to libjpeg
    both = d[:2] + adobe0 + d[2:]
    from oracle import oracle as orc
    info, coefs = jpeg.decode_coefs(both)
    assert np.array_equal(orc.jpeg_reconstruct(coefs, info), _pil(both))


def test_extraneous_bytes_before_marker_skipped_like_libjpeg():
    from mx_det import jpeg
    from oracle import oracle as orc
    d = bytes(_base())
    m, o, e = next(s for s in _segs(d) if s[0] == 0xDB)
    junk = d[:o] + b"\x00\x12\x34" + d[o:]
    info, coefs = jpeg.decode_coefs(junk)
    assert np.array_equal(orc.jpeg_reconstruct(coefs, info), _pil(d))


@pytest.mark.gpu
def test_prefetch_loader_matches_pil(dev, tmp_path):
    """engine.PrefetchJpegLoader (producer thread, threaded host entropy decode, device pixel stage,
    pinned targets) over an on-disk COCO split: every image bit-identical to PIL's decode, targets
    identical to the reference dataset's, batches in the loader's order."""
    from torch.utils.data import DataLoader
    from mx_det.data import write_coco_split
    from mx_det.dataset import COCODetectionDataset, collate_fn, uint8_transform
    from mx_det.engine import PrefetchJpegLoader
    ann = write_coco_split(tmp_path, "train", 0, 5, H=120, W=176, mean_boxes=6)
    raw = COCODetectionDataset(str(tmp_path / "images/train"), str(ann), transforms=uint8_transform, raw=True)
    ref = COCODetectionDataset(str(tmp_path / "images/train"), str(ann), transforms=uint8_transform)
    for kicked in (False, True):  # staging when the consumer runs dry / on the training loop's kick
        loader = PrefetchJpegLoader(DataLoader(raw, batch_size=2, shuffle=False, collate_fn=collate_fn), dev,
                                    workers=3)
        seen = 0
        for images, targets in loader:
            for im, t in zip(images, targets):
                r_img, r_t = ref[seen]
                assert im.device.type == "cuda" and torch.equal(im.cpu(), r_img)
                assert sorted(t) == sorted(r_t)
                for k in r_t:
                    assert t[k].dtype == r_t[k].dtype and torch.equal(t[k].cpu(), r_t[k]), k
                seen += 1
            if kicked:
                loader.kick()
        assert seen == 5


def test_pack_targets_roundtrip():
    """engine._pack_targets / _unpack_targets: one byte buffer per batch, views with the loader's keys,
    dtypes, shapes and values (empty targets included)."""
    from mx_det.engine import _pack_targets, _unpack_targets
    t = [{"boxes": torch.rand(3, 4), "labels": torch.tensor([1, 2, 3]), "image_id": torch.tensor([7]),
          "area": torch.rand(3), "iscrowd": torch.zeros(3, dtype=torch.int64)},
         {"boxes": torch.zeros((0, 4)), "labels": torch.zeros((0,), dtype=torch.int64),
          "image_id": torch.tensor([8]), "area": torch.zeros(0), "iscrowd": torch.zeros(0, dtype=torch.int64)}]
    buf, layout = _pack_targets(t, pin=False)
    assert buf.dtype == torch.uint8 and buf.dim() == 1
    out = _unpack_targets(buf.clone(), layout)
    for a, b in zip(t, out):
        assert list(a) == list(b)
        for k in a:
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape and torch.equal(a[k], b[k]), k
