"""mx_sample_draw, the fused BalancedPositiveNegativeSampler draw: bit-exact masks and counts against
oracle.balanced_sample (stable sort of each class's keys) on the RPN's float32 1 / 0 / -1 rows at the
headline anchor count (the sliced three-launch form, checked against the one-workgroup kernel too) and the RoI head's int64 class / 0 / -1 rows, with key ties, classes short of
their quota, empty classes, rows shorter than one tile and row lengths off the 1,024 grid; and the
sampler class on both paths (MX_FUSED_SAMPLER=1 / 0) drawing the same masks from the same keys."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _rows(g, N, L, p_pos, p_neg, int_labels, classes=7):
    u = torch.rand(N, L, generator=g)
    lab = torch.full((N, L), -1.0)
    lab[u < p_pos + p_neg] = 0.0
    lab[u < p_pos] = 1.0
    if int_labels:
        lab = lab.to(torch.int64)
        c = torch.randint(1, classes, (N, L), generator=g)
        lab = torch.where(lab == 1, c, lab)
    return lab


CASES = [  # N, L, p_pos, p_neg, int labels, key levels (0: continuous), batch, frac
    (2, 268569, 0.002, 0.7, False, 0, 256, 0.5),       # configs[1]'s RPN rows (800 x 1344, 15 anchors/loc)
    (2, 268569, 0.002, 0.7, False, 4096, 256, 0.5),    # many ties at the threshold
    (2, 2011, 0.05, 0.9, True, 0, 512, 0.25),          # RoI rows (2000 proposals + GT)
    (3, 2011, 0.4, 0.5, True, 64, 512, 0.25),          # positives over quota, heavy ties
    (2, 1000, 0.0, 0.9, True, 0, 512, 0.25),           # no positives
    (2, 777, 0.01, 0.0, False, 0, 256, 0.5),           # no negatives, short row
    (4, 100, 0.1, 0.2, False, 8, 256, 0.5),            # every candidate drawn
    (1, 1025, 0.3, 0.3, True, 2, 512, 0.25),           # two key values only
    (2, 0, 0.0, 0.0, True, 0, 512, 0.25),              # empty rows
    (1, 70001, 1.0, 0.0, False, 0, 256, 0.5),          # all positives
    (2, 50000, 0.3, 0.6, True, 2, 512, 0.25),          # long rows, two key values: whole classes tie
    (1, 16385, 0.01, 0.5, False, 1, 256, 0.5),         # just past the sliced threshold, every key equal
    (3, 40000, 0.0, 0.0, False, 0, 256, 0.5),          # long rows without candidates
]


@pytest.mark.parametrize("case", CASES)
def test_sample_draw_matches_oracle(dev, case):
    from mx_det import ops
    N, L, pp, pn, il, lv, B, fr = case
    g = torch.Generator().manual_seed(L + N + lv)
    lab = _rows(g, N, L, pp, pn, il)
    keys = torch.rand(N, L, generator=g)
    if lv:
        keys = torch.floor(keys * lv) / lv
    pos, neg, un, nums = ops.sample_draw(lab.to(dev), keys.to(dev), B, fr, with_union=True)
    rp, rn, rnums = orc.balanced_sample(lab.numpy(), keys.numpy(), B, fr)
    assert np.array_equal(nums.cpu().numpy(), rnums)
    assert np.array_equal(pos.cpu().numpy(), rp)
    assert np.array_equal(neg.cpu().numpy(), rn)
    assert np.array_equal(un.cpu().numpy(), rp | rn)
    p2, n2, u2, nums2 = ops.sample_draw(lab.to(dev), keys.to(dev), B, fr)
    assert u2 is None and torch.equal(p2, pos) and torch.equal(n2, neg) and torch.equal(nums2, nums)
    if L > ops.SAMPLE_SLICED_MIN:  # the one-workgroup-per-row kernel on the same long rows
        p3, n3, u3, nums3 = ops.sample_draw(lab.to(dev), keys.to(dev), B, fr, with_union=True, sliced=False)
        assert torch.equal(p3, pos) and torch.equal(n3, neg) and torch.equal(u3, un) and torch.equal(nums3, nums)


def test_sample_draw_negative_zero_ties_positive_zero(dev):
    from mx_det import ops
    lab = torch.zeros(1, 3000)
    keys = torch.rand(1, 3000, generator=torch.Generator().manual_seed(3)) + 0.5
    keys[0, 100:400:2] = -0.0
    keys[0, 101:400:2] = 0.0
    pos, neg, _, nums = ops.sample_draw(lab.to(dev), keys.to(dev), 256, 0.5)
    want = torch.zeros(1, 3000, dtype=torch.bool)
    want[0, 100:356] = True
    assert nums.tolist() == [[0, 256]] and not pos.any() and torch.equal(neg.cpu(), want)


@pytest.mark.parametrize("int_labels", [False, True])
def test_sampler_paths_agree(dev, monkeypatch, int_labels):
    """The sampler class with injected distinct keys: the fused draw and the pre-fusion paths (the RPN's
    torch.topk with be=None, the RoI head's mx_level_topk) mark the same anchors / proposals."""
    from mx_det import frcnn
    from mx_det.backend import default_backend
    be = default_backend()
    N, L = (2, 268569) if not int_labels else (2, 2011)
    B, fr = (256, 0.5) if not int_labels else (512, 0.25)
    g = torch.Generator().manual_seed(11)
    lab = _rows(g, N, L, 0.003 if not int_labels else 0.05, 0.8, int_labels).to(dev)
    keys = (torch.randperm(N * L, generator=g).float() / (N * L)).reshape(N, L).to(dev)  # distinct
    s = frcnn.BalancedPositiveNegativeSampler(B, fr)
    s.rand = lambda shape, device: keys
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("MX_FUSED_SAMPLER", fused)
        use = be if (fused == "1" or int_labels) else None
        out[fused] = s(lab, use)
    assert torch.equal(out["1"][0], out["0"][0]) and torch.equal(out["1"][1], out["0"][1])


@pytest.mark.parametrize("L", [2011, 40000])
def test_sample_draw_valid_mask_is_label_masking(dev, L):
    """valid=False entries belong to neither class: the same draw as on labels set to -1 there (both
    kernel forms: the RoI rows' one-workgroup kernel and the sliced one)."""
    from mx_det import ops
    g = torch.Generator().manual_seed(L)
    lab = _rows(g, 2, L, 0.1, 0.8, True)
    keys = torch.rand(2, L, generator=g)
    valid = torch.rand(2, L, generator=g) < 0.7
    masked = torch.where(valid, lab, -1)
    p0, n0, u0, c0 = ops.sample_draw(masked.to(dev), keys.to(dev), 512, 0.25, with_union=True)
    p1, n1, u1, c1 = ops.sample_draw(lab.to(dev), keys.to(dev), 512, 0.25, with_union=True, valid=valid.to(dev))
    rp, rn, rnums = orc.balanced_sample(masked.numpy(), keys.numpy(), 512, 0.25)
    assert np.array_equal(p1.cpu().numpy(), rp) and np.array_equal(n1.cpu().numpy(), rn)
    assert np.array_equal(c1.cpu().numpy(), rnums)
    assert torch.equal(p0, p1) and torch.equal(n0, n1) and torch.equal(u0, u1) and torch.equal(c0, c1)


@pytest.mark.parametrize("gm,counts", [(32, [5, 0]), (64, [64, 33]), (0, [0, 0])])
def test_roi_candidates_matches_cat(dev, gm, counts):
    """mx_roi_candidates = torchvision's cat([proposals, gt]) on the padded rows, with the validity the
    sampler masks by: proposals valid where pvalid, GT slots below the per-image count."""
    from mx_det import ops
    g = torch.Generator().manual_seed(gm + 1)
    N, post = 2, 2000
    pb = torch.rand(N, post, 4, generator=g) * 800
    pvalid = torch.arange(post)[None, :] < torch.tensor([1500, 2000])[:, None]
    gtp = torch.rand(N, gm, 4, generator=g) * 800
    gcnt = torch.tensor(counts, dtype=torch.int32)
    box, valid = ops.roi_candidates(pb.to(dev), pvalid.to(dev), gtp.to(dev), gcnt.to(dev))
    want_box = torch.cat([pb, gtp], 1)
    want_valid = torch.cat([pvalid, torch.arange(gm)[None, :] < gcnt[:, None].long()], 1)
    assert torch.equal(box.cpu(), want_box) and torch.equal(valid.cpu(), want_valid)
