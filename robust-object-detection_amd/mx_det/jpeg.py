"""Baseline-JPEG decode onto the device, hybrid like a host-entropy /
device-pixel decoder: the Huffman-coded bitstream is decoded on the host (libmx_det
mx_jpeg_decode_coefs: the sequential prefix code has no parallel structure without restart markers),
the quantised coefficients (int16, ~1.5 B per pixel at 4:2:0) are copied to HBM, and the device
dequantises, runs the libjpeg islow IDCT, upsamples the chroma and converts YCbCr -> RGB
(mx_jpeg_reconstruct). Output: uint8 [H, W, 3] on the device, bit-identical to libjpeg-turbo's default
decode -- PIL Image.open(p).convert("RGB") (coco_detection_dataset.py:23), or with bgr=True
cv2.imread (restore_testsets.py:99). Progressive / arithmetic / CMYK / 4:4:0 files raise
NotImplementedError (MX_EUNSUPPORTED); callers that must accept them decode those on the host.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import JpegInfo


class JpegUnsupported(NotImplementedError):
    pass


def parse(data):
    """Marker parse of the bytes `data` -> JpegInfo (host)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    info = JpegInfo()
    rc = _lib.load().mx_jpeg_parse(buf.ctypes.data, buf.size, ctypes.byref(info))
    if rc == -2:
        raise JpegUnsupported(_lib.load().mx_last_error().decode())
    if rc != 0:
        raise ValueError(_lib.load().mx_last_error().decode())
    return info


def decode_coefs(data, info=None, out=None):
    """Host entropy decode -> (info, int16 [coef_total]) of quantised natural-order coefficients: a numpy
    array, or `out` (an int16 CPU tensor of >= coef_total elements, e.g. pinned) filled in place. The
    decoder is a ctypes call into libmx_det, which releases the GIL: threads decode in parallel."""
    info = parse(data) if info is None else info
    buf = np.frombuffer(data, dtype=np.uint8)
    if out is None:
        coefs = np.empty(info.coef_total, dtype=np.int16)
        ptr = coefs.ctypes.data
    else:
        if not (out.dtype == torch.int16 and out.device.type == "cpu" and out.is_contiguous()
                and out.numel() >= info.coef_total):
            raise ValueError("decode_coefs: out must be a contiguous int16 CPU tensor of coef_total elements")
        coefs, ptr = out, out.data_ptr()
    rc = _lib.load().mx_jpeg_decode_coefs(buf.ctypes.data, buf.size, ctypes.byref(info), ptr)
    if rc != 0:
        raise ValueError(_lib.load().mx_last_error().decode())
    return info, coefs


def host_stage(data):
    """The host half of decode(): marker parse + entropy decode straight into pinned memory ->
    (info, pinned int16 tensor), ready for an asynchronous copy (device_stage). Thread-safe."""
    from .conv import capture_lock
    info = parse(data)
    # pinned allocations (cudaHostAlloc on a cache miss) are prohibited while another thread has a graph
    # capture open in global mode: the training thread's captures (frcnn._Graphs) hold capture_lock
    with capture_lock:
        host = torch.empty(info.coef_total, dtype=torch.int16, pin_memory=True)
    return decode_coefs(data, info, out=host)


def device_stage(info, host, device, bgr=False):
    """The device half: coefficients to HBM (non-blocking from pinned memory), then dequantise + islow
    IDCT + chroma upsampling + YCbCr -> RGB in mx_jpeg_reconstruct on the current stream."""
    dev = host.to(device, non_blocking=True)
    ws = torch.empty(_lib.load().mx_jpeg_workspace(ctypes.byref(info)), dtype=torch.uint8, device=device)
    out = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device=device)
    _lib.call("mx_jpeg_reconstruct", dev.data_ptr(), ctypes.byref(info), ws.data_ptr(), ws.numel(), out.data_ptr(),
              int(bool(bgr)), _lib.stream())
    return out


def decode(data, device, bgr=False, pin=True):
    """JPEG bytes -> uint8 [H, W, 3] tensor on `device` (RGB, or BGR with bgr=True)."""
    if pin:
        return device_stage(*host_stage(data), device, bgr)
    info, coefs = decode_coefs(data)
    dev = torch.from_numpy(coefs).to(device)
    ws = torch.empty(_lib.load().mx_jpeg_workspace(ctypes.byref(info)), dtype=torch.uint8, device=device)
    out = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device=device)
    _lib.call("mx_jpeg_reconstruct", dev.data_ptr(), ctypes.byref(info), ws.data_ptr(), ws.numel(), out.data_ptr(),
              int(bool(bgr)), _lib.stream())
    return out


def read_file(path, device, bgr=False):
    with open(path, "rb") as f:
        return decode(f.read(), device, bgr=bgr)
