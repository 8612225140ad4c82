"""Split-K tail of the bf16x3 buffer conv kernel, checked on the CPU through the library's host-side
queries (mx_conv_x3_geometry, mx_conv_tail_map -- the kernel's own block mapping, compiled
__host__ __device__): for the model's GEMM shapes and random ones, the blocks of the launched grid
cover every (tile, K-tile) pair exactly once, the unsplit tiles are exactly the rows below m_base (the
fused epilogue writes them and their BatchNorm statistics rows), the split tiles are whole block rows
from m_base on (the reduce kernel's rows, 128-row aligned), and the workspace query covers the tail's
slab planes. The outputs themselves are compared on the GPU (tests/test_gpu_x3.py::test_x3_tail_split)."""
import ctypes
import random

import pytest

from mx_det import _lib


def _geo(M, Ncol, Kdim):
    out = (ctypes.c_int64 * 7)()
    assert _lib.load().mx_conv_x3_geometry(M, Ncol, Kdim, out) == 0
    return dict(zip(("bmt", "bn", "tiles", "splits", "tail_tile", "m_base", "tail_splits"), list(out)))


def _map(tail_tile, splits, gid):
    out = (ctypes.c_int64 * 3)()
    assert _lib.load().mx_conv_tail_map(tail_tile, splits, gid, out) == 0
    return tuple(out)


def _cdiv(a, b):
    return -(-a // b)


def _check_cover(M, Ncol, Kdim):
    g = _geo(M, Ncol, Kdim)
    nk = _cdiv(Kdim, 32)
    ntn = _cdiv(Ncol, g["bn"])
    assert g["tiles"] == _cdiv(M, g["bmt"]) * ntn
    if g["tail_splits"] <= 1:
        assert g["tail_tile"] == 0 and g["m_base"] == 0
        return g
    assert g["splits"] == 1 and g["bmt"] == 128
    assert 0 < g["tail_tile"] < g["tiles"] and g["tail_tile"] % ntn == 0
    assert g["m_base"] == g["tail_tile"] // ntn * 128 and g["m_base"] % 128 == 0 and g["m_base"] < M
    kps = _cdiv(nk, g["tail_splits"])
    splits = _cdiv(nk, kps)  # as launch_igemm_x3 sets p.splits
    blocks = g["tail_tile"] + (g["tiles"] - g["tail_tile"]) * splits
    cover = {}
    for gid in range(blocks):
        bid, split, partial = _map(g["tail_tile"], splits, gid)
        assert 0 <= bid < g["tiles"]
        assert bool(partial) == (bid >= g["tail_tile"])
        k0, k1 = (split * kps, min(nk, (split + 1) * kps)) if partial else (0, nk)
        assert k0 < k1
        cover.setdefault(bid, []).append((k0, k1))
    assert sorted(cover) == list(range(g["tiles"]))
    for bid, ranges in cover.items():
        ranges.sort()
        assert ranges[0][0] == 0 and ranges[-1][1] == nk
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:])), (bid, ranges)
        # unsplit tiles hold rows below m_base, split ones rows from m_base on
        m0 = bid // ntn * 128
        assert (m0 >= g["m_base"]) == (len(ranges) > 1 or bid >= g["tail_tile"])
    return g


def test_plain_split_k_mapping_unchanged():
    for splits in (1, 2, 5, 16):
        for gid in range(64):
            assert _map(0, splits, gid) == (gid // splits, gid % splits, 1)


# fwd / dgrad GEMMs (M, Ncol, Kdim) of the f32 headline step: P2 3x3 convs (FPN output, RPN head),
# the box head's 3x3 on 1024 RoIs, layer2 / layer3 convs, the dgrads' stride-parity classes
MODEL = [(134400, 256, 2304), (50176, 256, 2304), (33600, 128, 1152), (33600, 512, 128), (8400, 256, 2304),
         (134400, 64, 576), (33600, 128, 512), (8400, 1024, 256), (134400, 256, 64), (33600, 256, 2304)]


@pytest.mark.parametrize("gemm", MODEL)
def test_tail_cover_model_shapes(gemm):
    _check_cover(*gemm)


def test_p2_3x3_takes_the_tail():
    g = _check_cover(134400, 256, 2304)  # 2,100 tiles on 512 slots: a fifth round 10 % full
    assert g["tail_splits"] >= 2 and g["tiles"] - g["tail_tile"] <= 128, g


def test_tail_cover_random_shapes():
    rnd = random.Random(5)
    seen = 0
    for _ in range(300):
        M = rnd.randrange(1, 300000)
        Ncol = 8 * rnd.randrange(1, 96)
        Kdim = 32 * rnd.randrange(1, 160)
        seen += _check_cover(M, Ncol, Kdim)["tail_splits"] > 1
    assert seen > 10  # the random set does exercise the tail


def test_tail_switch_and_workspace():
    lib = _lib.load()
    from mx_det.conv import shape
    import torch
    x = torch.empty((2, 200, 336, 256))
    sh = shape(x, 256, 3, 3, (1, 1), (1, 1))
    g = _geo(134400, 256, 2304)
    ws = lib.mx_conv_workspace_x3(ctypes.byref(sh), 0)
    assert ws >= 4 * g["tail_splits"] * (134400 - g["m_base"]) * 256
    assert lib.mx_conv_set_tail(0) == 0
    try:
        assert _geo(134400, 256, 2304)["tail_splits"] == 1
        assert lib.mx_conv_workspace_x3(ctypes.byref(sh), 0) == 0
    finally:
        lib.mx_conv_set_tail(1)
