"""CPU checks of the corruption restatements (oracle/mx_oracle.c) and of the reference-pinned
RandomCorruption stream (tests/golden/random_corruption.npz, make_golden.py).

- _motion_blur_kernel (augmentations.py:21-27): the reference setting k=9, angle 0 is the centre row of
  float32(1/9) (the restatement's warpAffine is exactly the identity there); 90 / 180 / 270 degrees are
  the column / row; every kernel sums to 1 (f32); the product's numpy restatement equals the C oracle.
- cv2.resize INTER_AREA at an exact x2 scale (apply_lowres on even x even frames such as 1920x1080):
  (a+b+c+d+2)>>2 in the vectorised part of each row, round-half-even of sum*0.25 in the scalar tail.
- RandomCorruption: the keep decision, the choice and the noise field follow the reference's random /
  numpy streams, and the noise lands on the BGR view (cvtColor RGB2BGR, augmentations.py:72-74).
cv2 is not installed: the OpenCV arithmetic is restated from its source (parity unpinned beyond
the seeds whose reference output needs no OpenCV, which the golden pins)."""
import random

import numpy as np

from oracle import oracle as orc


def test_motion_blur_kernel_known_answers():
    k0 = orc.motion_blur_kernel(9, 0)
    row = np.zeros((9, 9), np.float32)
    row[4] = np.float32(1.0) / np.float32(9.0)
    assert np.array_equal(k0, row)
    assert np.array_equal(orc.motion_blur_kernel(9, 180), row)
    col = row.T.copy()
    assert np.array_equal(orc.motion_blur_kernel(9, 90), col)
    assert np.array_equal(orc.motion_blur_kernel(9, 270), col)
    for k in (5, 9, 11):
        for a in (15, 45, 60, 137):
            kk = orc.motion_blur_kernel(k, a)
            assert abs(float(kk.sum()) - 1.0) < 1e-6
            assert (kk >= 0).all()


def test_motion_blur_kernel_product_restatement_matches_oracle():
    import sys
    sys.path.insert(0, "robust-object-detection_amd")
    from mx_det.augment import motion_blur_kernel
    for k in (3, 5, 7, 9, 11, 15):
        for a in (0, 10, 30, 45, 90, 135, -20, 180, 17.5, 300):
            assert np.array_equal(motion_blur_kernel(k, a), orc.motion_blur_kernel(k, a)), (k, a)


def test_filter2d_angle0_is_the_box_row():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (21, 34, 3)).astype(np.uint8)
    assert np.array_equal(orc.motion_blur_u8(img, 9, 0), orc.blur_u8(img))


def test_area_fast2_rounding():
    # dw = 18 -> 54 elements per row: 48 in the vector loop ((s + 2) >> 2: ties round up), the last 6 in
    # the scalar tail (rint(s * 0.25): ties to even)
    img = np.zeros((4, 36, 3), np.uint8)
    img[0::2, :, :] = 1  # every 2x2 block sums to 2 -> 0.5
    out = orc.resize_area_fast2_u8(img)
    assert out.shape == (2, 18, 3)
    flat = out.reshape(2, -1)
    assert (flat[:, :48] == 1).all() and (flat[:, 48:] == 0).all()
    img[0::2] = 3  # sum 6 -> 1.5: vector 2, tail rint(1.5) = 2
    flat = orc.resize_area_fast2_u8(img).reshape(2, -1)
    assert (flat == 2).all()
    # lowres takes the fast path exactly when W == 2*nw and H == 2*nh
    rng = np.random.default_rng(4)
    even = rng.integers(0, 256, (40, 62, 3)).astype(np.uint8)
    small = orc.resize_area_fast2_u8(even)
    assert np.array_equal(orc.lowres_u8(even, 0.5), orc.resize_linear_u8(small, 40, 62))


def test_random_corruption_stream_matches_reference_golden():
    d = np.load("tests/golden/random_corruption.npz")
    img = d["img"]
    n = 0
    for s, op, out, pinned in zip(d["seeds"], d["ops"], d["outs"], d["pinned"]):
        random.seed(int(s))
        np.random.seed(int(s))
        if random.random() > 0.5:
            assert op == "keep"
            assert np.array_equal(out, img)
            n += 1
            continue
        choice = random.choice(["noise", "blur", "lowres"])
        assert op == {"noise": "apply_noise", "blur": "apply_motion_blur", "lowres": "apply_lowres"}[choice]
        if not pinned:
            continue
        bgr = np.ascontiguousarray(img[..., ::-1])
        field = np.random.normal(0, 15, bgr.shape).astype(np.float32)
        got = orc.noise_u8(bgr, field)[..., ::-1]
        assert np.array_equal(got, out), s
        n += 1
    assert n >= 20
