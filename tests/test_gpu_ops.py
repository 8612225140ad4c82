"""GPU parity of the libmx_det HIP ops against the CPU oracle (oracle/mx_oracle.c).

Bar: bit-exact for index work (matches, NMS keep lists, anchors) and for f32 RoIAlign forward
(same op order per element); IoU values bit-exact; exp/log-based coder outputs within 1e-5
relative (device expf/logf vs libm may differ in the last ulp; north_star tolerance is 1e-3).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _rand_boxes(rng, n, H=800, W=1333, med=24.0):
    cx = rng.uniform(0, W, n)
    cy = rng.uniform(0, H, n)
    w = np.clip(rng.lognormal(np.log(med), 0.8, n), 2, W)
    h = np.clip(rng.lognormal(np.log(med), 0.8, n), 2, H)
    b = np.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1)
    b[:, 0::2] = np.clip(b[:, 0::2], 0, W)
    b[:, 1::2] = np.clip(b[:, 1::2], 0, H)
    return b.astype(np.float32)


def _anchors_np(H=800, W=1344):
    lv = []
    for i, s in enumerate((32, 64, 128, 256, 512)):
        st = 4 * 2 ** i
        gh, gw = -(-H // st), -(-W // st)
        if i == 4:  # P6 = max_pool(P5, 1, 2)
            gh, gw = (-(-H // 32) + 1) // 2, (-(-W // 32) + 1) // 2
        sh, sw = H // gh, W // gw
        lv.append(orc.anchors_level(s, [0.5, 1.0, 2.0], gh, gw, sh, sw))
    return np.concatenate(lv)


def test_anchors_bitexact(dev):
    from mx_det import ops
    ref = _anchors_np()
    assert ref.shape[0] == 268569
    got = []
    for i, s in enumerate((32, 64, 128, 256, 512)):
        st = 4 * 2 ** i
        gh, gw = -(-800 // st), -(-1344 // st)
        if i == 4:
            gh, gw = 13, 21
        got.append(ops.anchors_level(s, [0.5, 1.0, 2.0], gh, gw, 800 // gh, 1344 // gw, dev))
    got = torch.cat(got).cpu().numpy()
    assert np.array_equal(got, ref)


def test_box_iou_bitexact(dev):
    from mx_det import ops
    rng = np.random.default_rng(0)
    a, b = _rand_boxes(rng, 77), _rand_boxes(rng, 1500)
    b[:10] = a[:10]  # exact duplicates -> IoU 1
    got = ops.box_iou(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), orc.box_iou(a, b).view(np.uint32))


@pytest.mark.parametrize("G", [0, 1, 55, 300])
def test_rpn_matcher_bitexact(dev, G):
    """RPN: Matcher(0.7, 0.3, allow_low_quality=True) over the real 800x1344 anchor set."""
    from mx_det import ops
    rng = np.random.default_rng(G + 1)
    anchors = _anchors_np()
    gt = _rand_boxes(rng, G)
    if G > 3:
        gt[1] = gt[0]  # duplicate gt -> argmax tie must pick the first index
    m, lab, tgt = ops.match_assign(torch.from_numpy(gt).to(dev), torch.from_numpy(anchors).to(dev), 0.7, 0.3, True,
                                   mode=1, weights=(1.0, 1.0, 1.0, 1.0))
    m = m.cpu().numpy()
    if G == 0:
        assert (m == -1).all() and (lab.cpu().numpy() == 0).all()
        return
    ref = orc.matcher(orc.box_iou(gt, anchors), 0.7, 0.3, True)
    assert np.array_equal(m, ref)
    reflab = np.where(ref >= 0, 1.0, np.where(ref == -1, 0.0, -1.0)).astype(np.float32)
    assert np.array_equal(lab.cpu().numpy(), reflab)
    pos = ref >= 0
    reft = orc.box_encode(gt[np.clip(ref, 0, None)][pos], anchors[pos], [1, 1, 1, 1])
    np.testing.assert_allclose(tgt.cpu().numpy()[pos], reft, rtol=1e-5, atol=1e-5)


def test_roi_matcher_labels(dev):
    """RoIHeads: proposals + gt appended, Matcher(0.5, 0.5, False), labels from gt labels."""
    from mx_det import ops
    rng = np.random.default_rng(5)
    gt = _rand_boxes(rng, 40)
    props = np.concatenate([_rand_boxes(rng, 2000, med=40), gt])
    glab = rng.integers(1, 7, 40).astype(np.int64)
    m, lab, tgt = ops.match_assign(torch.from_numpy(gt).to(dev), torch.from_numpy(props).to(dev), 0.5, 0.5, False,
                                   mode=2, gt_labels=torch.from_numpy(glab).to(dev), weights=(10., 10., 5., 5.))
    ref = orc.matcher(orc.box_iou(gt, props), 0.5, 0.5, False)
    assert np.array_equal(m.cpu().numpy(), ref)
    reflab = np.where(ref >= 0, glab[np.clip(ref, 0, None)], 0)
    assert np.array_equal(lab.cpu().numpy(), reflab)
    reft = orc.box_encode(gt[np.clip(ref, 0, None)], props, [10, 10, 5, 5])
    np.testing.assert_allclose(tgt.cpu().numpy(), reft, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("counts", [(0, 3), (55, 300), (33, 1), (0, 0)])
def test_batched_matcher_equals_per_image(dev, counts):
    """One launch pair over zero-padded GT (frcnn's RPN and RoI target path) == the per-image matcher,
    bit for bit: RPN mode over shared anchors, RoI mode over per-image [B, A, 4] candidates."""
    from mx_det import ops
    rng = np.random.default_rng(sum(counts) + 7)
    anchors = torch.from_numpy(_anchors_np()).to(dev)
    targets = [{"boxes": torch.from_numpy(_rand_boxes(rng, g)).to(dev),
                "labels": torch.from_numpy(rng.integers(1, 7, g).astype(np.int64)).to(dev)} for g in counts]
    if counts[1] > 3:
        targets[1]["boxes"][2] = targets[1]["boxes"][0]  # duplicate gt -> first index wins
    gtp, glp, gc = ops.pad_gt(targets, dev)
    assert gtp.shape[1] % 32 == 0 and gtp.shape[1] >= max(counts)
    m, lab, tg, cnt = ops.match_assign_batched(gtp, gc, anchors, 0.7, 0.3, True, 1, weights=(1., 1., 1., 1.),
                                               with_counts=True)
    assert torch.equal(cnt.long(), torch.stack([(lab == 1).sum(1), (lab == 0).sum(1)], 1))
    for i, t in enumerate(targets):
        mi, li, ti = ops.match_assign(t["boxes"], anchors, 0.7, 0.3, True, mode=1, weights=(1., 1., 1., 1.))
        assert torch.equal(m[i], mi) and torch.equal(lab[i], li)
        pos = mi >= 0
        assert torch.equal(tg[i][pos], ti[pos])
    props = torch.stack([torch.from_numpy(_rand_boxes(rng, 2000, med=40)).to(dev) for _ in counts])
    cand = torch.cat([props, gtp], 1)
    m, lab, tg, cnt = ops.match_assign_batched(gtp, gc, cand, 0.5, 0.5, False, 2, gt_labels=glp,
                                               weights=(10., 10., 5., 5.), with_counts=True)
    assert torch.equal(cnt.long(), torch.stack([(lab >= 1).sum(1), (lab == 0).sum(1)], 1))
    for i, t in enumerate(targets):
        mi, li, ti = ops.match_assign(t["boxes"], cand[i], 0.5, 0.5, False, mode=2, gt_labels=t["labels"],
                                      weights=(10., 10., 5., 5.))
        real = slice(0, 2000 + counts[i])  # padded candidate rows are masked out by the caller
        assert torch.equal(m[i][real], mi[real]) and torch.equal(lab[i][real], li[real])
        pos = mi[real] >= 0
        assert torch.equal(tg[i][real][pos], ti[real][pos])


@pytest.mark.parametrize("n,thr", [(1, 0.7), (50, 0.7), (999, 0.5), (2000, 0.7), (6000, 0.5), (7200, 0.7)])
def test_nms_bitexact(dev, n, thr):
    from mx_det import ops
    rng = np.random.default_rng(n)
    b = _rand_boxes(rng, n, med=60)
    b[n // 2:] = b[: n - n // 2] + rng.normal(0, 3, (n - n // 2, 4)).astype(np.float32)  # dense clusters
    s = rng.random(n).astype(np.float32)
    s[::7] = s[0]  # score ties -> stable order by index
    got = ops.nms(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev), thr).cpu().numpy()
    assert np.array_equal(got, orc.nms(b, s, thr))


@pytest.mark.parametrize("chain", [3, 40, 1500])
def test_nms_suppression_chains(dev, chain):
    """Boxes on a line where each suppresses the next but not the one after (keep every other one):
    chains longer than the tile resolver's Jacobi steps take its survivor-walk fallback; short ones
    converge in the Jacobi steps. Mixed with random boxes; bit-exact vs the oracle."""
    from mx_det import ops
    rng = np.random.default_rng(chain)
    x = np.arange(chain, dtype=np.float32) * 7.0
    line = np.stack([x, np.zeros_like(x), x + 30, np.full_like(x, 20)], 1)  # IoU(i, i+1) .62, (i, i+2) .36
    b = np.concatenate([line, _rand_boxes(rng, 1900 - chain if chain < 1900 else 0, med=40)]).astype(np.float32)
    s = rng.random(len(b)).astype(np.float32) * 0.5
    s[:chain] = 1.0 - np.arange(chain, dtype=np.float32) / (4 * chain)  # the chain first, in line order
    got = ops.nms(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev), 0.5).cpu().numpy()
    ref = orc.nms(b, s, 0.5)
    assert np.array_equal(got, ref)
    assert np.array_equal(ref[: (chain + 1) // 2], np.arange(0, chain, 2))


@pytest.mark.parametrize("n,ncls", [(700, 6), (1000, 5), (1001, 5), (8819, 5), (5000, 6)])
def test_batched_nms_paths(dev, n, ncls):
    """CPU dispatch: 4n > 4000 -> per-class loop; else coordinate trick (both bit-exact)."""
    from mx_det import ops
    rng = np.random.default_rng(n + ncls)
    b = _rand_boxes(rng, n, med=50)
    s = rng.random(n).astype(np.float32)
    idx = rng.integers(0, ncls, n).astype(np.int64)
    got = ops.batched_nms(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev), torch.from_numpy(idx).to(dev),
                          0.7).cpu().numpy()
    assert np.array_equal(got, orc.batched_nms(b, s, idx, 0.7))


def test_batched_nms_grouped(dev):
    """Two images in one call: output ordered by (image, score desc) == per-image calls."""
    from mx_det import ops
    rng = np.random.default_rng(9)
    n = 3000
    b = _rand_boxes(rng, n, med=50)
    s = rng.random(n).astype(np.float32)
    lvl = rng.integers(0, 5, n)
    img = (np.arange(n) >= 1700).astype(np.int64)
    idx = img * 5 + lvl
    got = ops.batched_nms(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev), torch.from_numpy(idx).to(dev),
                          0.7, group=torch.from_numpy(img).to(dev), mode=1).cpu().numpy()
    ref = []
    for i in (0, 1):
        sel = np.where(img == i)[0]
        k = orc.batched_nms(b[sel], s[sel], lvl[sel], 0.7)
        ref.append(sel[k])
    assert np.array_equal(got, np.concatenate(ref))


def _presorted(rng, G, runs, dead_frac, ties):
    """filter_proposals-shaped candidates: per image, per level a run of `runs[l]` slots with scores
    descending (ties every `ties` slots), a fraction of slots dead (group G), boxes random."""
    b, s, lv, gr = [], [], [], []
    for g in range(G):
        for l, k in enumerate(runs):
            sc = np.sort(rng.random(k).astype(np.float32))[::-1].copy()
            if ties:
                sc[1::ties] = sc[0::ties][:len(sc[1::ties])]
            b.append(_rand_boxes(rng, k, med=40))
            s.append(sc)
            lv.append(np.full(k, l))
            gg = np.full(k, g, np.int32)
            gg[rng.random(k) < dead_frac] = G
            gr.append(gg)
    return (np.concatenate(b).astype(np.float32), np.concatenate(s), np.concatenate(lv).astype(np.int64),
            np.concatenate(gr))


@pytest.mark.parametrize("G,runs,dead,ties,shuffle", [
    (2, [2000, 2000, 2000, 2000, 819], 0.0, 0, False),   # the bs=2 training call: per-level NMS
    (2, [2000, 2000, 2000, 2000, 819], 0.1, 5, False),   # dead slots + score ties
    (3, [200, 100, 60, 30, 9], 0.2, 3, False),           # <= 1000 live per image: coordinate trick
    (2, [900, 500, 200, 60, 20], 0.5, 0, False),         # one image per level, one trick (mixed)
    (1, [1000, 1000, 1000, 1000, 273], 0.0, 0, False),   # eval: one image
    (2, [700, 600, 300, 50, 10], 0.05, 0, True),         # runs NOT sorted: exact by the counting path
    (2, [300, 200, 100, 20, 5], 0.05, 0, True),          # unsorted trick images
    (2, [3, 0, 2, 0, 1], 0.0, 0, False),                 # tiny, empty levels
])
def test_batched_nms_grouped_sorted(dev, G, runs, dead, ties, shuffle):
    """The sort-free grouped NMS on presorted candidates == the general grouped NMS (two radix sorts)
    == per-image torchvision batched_nms (oracle): keep[:num_keep] bit-exact, and the padded
    per-image selection equals the survivors' prefix. Shuffled runs break the presorted order: the
    counting fallback must still give the exact stable order."""
    from mx_det import ops
    rng = np.random.default_rng(sum(runs) + G)
    b, s, lv, gr = _presorted(rng, G, runs, dead, ties)
    if shuffle:
        perm = np.arange(len(s))
        o = 0
        for _ in range(G):
            for k in runs:
                perm[o:o + k] = o + rng.permutation(k)
                o += k
        b, s, lv, gr = b[perm], s[perm], lv[perm], gr[perm]
    t = [torch.from_numpy(a).to(dev) for a in (b, s, lv, gr)]
    L = len(runs)
    k0, n0 = ops.batched_nms_grouped(*t, G, L, 0.7, 2000)
    k1, n1, sel, valid = ops.batched_nms_grouped_sorted(*t, G, L, 0.7, 2000, post=1500)
    nk = int(n0.item())
    assert int(n1.item()) == nk
    got = k1[:nk].cpu().numpy()
    assert np.array_equal(got, k0[:nk].cpu().numpy())
    ref = []
    for g in range(G):
        idx = np.where(gr == g)[0]
        if idx.size:
            ref.append(idx[orc.batched_nms(b[idx], s[idx], lv[idx], 0.7)])
    assert np.array_equal(got, np.concatenate(ref) if ref else np.zeros(0, np.int64))
    sel, valid = sel.cpu().numpy(), valid.cpu().numpy()
    o = 0
    for g in range(G):
        c = len(ref[g]) if g < len(ref) else 0
        assert valid[g].sum() == min(c, 1500) and valid[g][:min(c, 1500)].all()
        assert np.array_equal(sel[g][:min(c, 1500)], got[o:o + min(c, 1500)])
        o += c


def test_batched_nms_grouped_sorted_layout_violation(dev):
    """Levels not contiguous within an image (outside the presorted contract): num_keep = -2 and an
    empty selection -- reported, never an out-of-range index."""
    from mx_det import ops
    rng = np.random.default_rng(3)
    b, s, lv, gr = _presorted(rng, 2, [300, 300, 300], 0.0, 0)
    lv = lv.copy()
    lv[:600] = np.tile([0, 1], 300)  # image 0's first two runs interleaved
    t = [torch.from_numpy(a).to(dev) for a in (b, s, lv, gr)]
    k, nk, sel, valid = ops.batched_nms_grouped_sorted(*t, 2, 3, 0.7, 2000, post=100)
    assert int(nk.item()) == -2 and not valid.any()
    assert int(k.min()) >= 0 and int(k.max()) < len(s)


def test_batched_nms_grouped_sorted_empty(dev):
    from mx_det import ops
    z = torch.zeros((0, 4), device=dev)
    k, nk, sel, valid = ops.batched_nms_grouped_sorted(z, torch.zeros(0, device=dev),
                                                       torch.zeros(0, dtype=torch.int64, device=dev),
                                                       torch.zeros(0, dtype=torch.int32, device=dev), 2, 5, 0.7, 2000,
                                                       post=10)
    assert int(nk.item()) == 0 and not valid.any() and (sel == 0).all()


def test_nms_empty(dev):
    from mx_det import ops
    k = ops.nms(torch.zeros((0, 4), device=dev), torch.zeros(0, device=dev), 0.5)
    assert k.shape == (0,) and k.dtype == torch.int64


def _rois(rng, K, N, H, W, scale):
    b = _rand_boxes(rng, K, H=H / scale, W=W / scale, med=60)
    b[0] = [-20, -30, 5, 5]  # partially outside the map
    b[1] = [3, 3, 3.2, 3.1]  # smaller than one pixel -> size clamped to 1
    bi = rng.integers(0, N, K).astype(np.float32)[:, None]
    return np.concatenate([bi, b], 1).astype(np.float32)


def test_roi_align_fwd_f32_bitexact(dev):
    from mx_det import ops
    rng = np.random.default_rng(3)
    N, C, H, W, scale = 2, 96, 50, 84, 1 / 16
    feat = rng.standard_normal((N, C, H, W)).astype(np.float32)
    rois = _rois(rng, 300, N, H, W, scale)
    ref = orc.roi_align(feat, rois, scale, (7, 7), 2, False)
    f = torch.from_numpy(feat).to(dev).permute(0, 2, 3, 1).contiguous()
    got = ops.roi_align(f, torch.from_numpy(rois).to(dev), (7, 7), scale, 2, False)
    got = got.permute(0, 3, 1, 2).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_roi_align_aligned_and_bf16(dev):
    from mx_det import ops
    rng = np.random.default_rng(4)
    N, C, H, W, scale = 1, 256, 40, 40, 0.25
    feat = rng.standard_normal((N, C, H, W)).astype(np.float32)
    rois = _rois(rng, 64, N, H, W, scale)
    ref = orc.roi_align(feat, rois, scale, (7, 7), 2, True)
    f = torch.from_numpy(feat).to(dev).permute(0, 2, 3, 1).contiguous()
    got = ops.roi_align(f, torch.from_numpy(rois).to(dev), 7, scale, 2, True).permute(0, 3, 1, 2).cpu().numpy()
    assert np.array_equal(got, ref)
    fb = f.bfloat16()
    ref_b = orc.roi_align(fb.float().permute(0, 3, 1, 2).cpu().numpy(), rois, scale, (7, 7), 2, False)
    got_b = ops.roi_align(fb, torch.from_numpy(rois).to(dev), 7, scale, 2, False).float().permute(0, 3, 1, 2)
    np.testing.assert_allclose(got_b.cpu().numpy(), ref_b, rtol=8e-3, atol=8e-3)


def test_roi_align_backward(dev):
    from mx_det import ops
    rng = np.random.default_rng(6)
    N, C, H, W, scale = 2, 64, 30, 41, 0.125
    feat = rng.standard_normal((N, C, H, W)).astype(np.float32)
    rois = _rois(rng, 120, N, H, W, scale)
    rois[2, 1:] = [0, 0, W / scale, H / scale]  # footprint > the LDS tile: direct-atomic fallback
    rois[3, 1:] = [8, 8, 8 + 20 / scale, 8 + 17 / scale]  # 21x18 cells: just over the tile
    gout = rng.standard_normal((120, C, 7, 7)).astype(np.float32)
    ref = orc.roi_align_backward(gout, rois, scale, (N, C, H, W), 2, False)
    f = torch.from_numpy(feat).to(dev).permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    out = ops.roi_align(f, torch.from_numpy(rois).to(dev), 7, scale, 2, False)
    out.backward(torch.from_numpy(gout).to(dev).permute(0, 2, 3, 1))
    got = f.grad.permute(0, 3, 1, 2).cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("C,gdt", [(256, torch.float32), (64, torch.float32), (32, torch.bfloat16), (12, torch.float32)])
def test_multiscale_roi_align_backward_deterministic(dev, monkeypatch, C, gdt):
    """Atomic-free gather backward: BIT-EXACT against the oracle (torchvision's CPU loop order: RoI,
    bin, sample, corner, each contribution g * w / count added in turn), bitwise identical run to run,
    equal to the atomic form up to summation order, and every level-map element written (the maps
    come from torch.empty)."""
    from mx_det import ops
    rng = np.random.default_rng(C + 1)
    N = 2
    shapes = [(60, 101), (30, 51), (15, 26), (8, 13)]
    scales = [0.25, 0.125, 0.0625, 0.03125]
    feats = [torch.from_numpy(rng.standard_normal((N, h, w, C)).astype(np.float32)) for h, w in shapes]
    boxes = np.concatenate([_rand_boxes(rng, 120, H=240, W=404, med=16), _rand_boxes(rng, 80, H=240, W=404, med=150)])
    boxes[0] = [-30, -30, 430, 260]  # overhangs every edge
    boxes[1] = [3, 3, 3.2, 3.1]      # sub-pixel
    bi = rng.integers(0, N, len(boxes)).astype(np.float32)[:, None]
    rois = np.concatenate([bi, boxes], 1).astype(np.float32)
    lv = _level_mapper_np(boxes)
    g = torch.from_numpy(rng.standard_normal((len(rois), 7, 7, C)).astype(np.float32)).to(gdt)
    rt = torch.from_numpy(rois).to(dev)

    def run(det):
        monkeypatch.setenv("MX_ROI_DETERMINISTIC", "1" if det else "0")
        ft = [f.to(dev).to(gdt).requires_grad_(True) for f in feats]
        out = ops.multiscale_roi_align(ft, rt, scales, 2)
        return torch.autograd.grad(out, ft, g.to(dev))
    a, b, c = run(True), run(True), run(False)
    gn = g.float().permute(0, 3, 1, 2).numpy()
    for l in range(4):
        assert torch.equal(a[l], b[l]), l
        tol = 1e-5 if gdt == torch.float32 else 1e-2
        torch.testing.assert_close(a[l].float(), c[l].float(), rtol=tol, atol=tol)
        sel = np.where(lv == l)[0]
        r = orc.roi_align_backward(gn[sel], rois[sel], scales[l], (N, C) + shapes[l], 2, False)
        r = torch.from_numpy(r).to(gdt).float().numpy()  # the returned grad is in the feature dtype
        assert np.array_equal(a[l].float().permute(0, 3, 1, 2).cpu().numpy(), r), l


def test_multiscale_roi_align_backward_heavy_overlap(dev, monkeypatch):
    """Deterministic gather on a tile that ~1,100 RoIs overlap (more than one 1,024-RoI list chunk;
    the pipelined walk crosses RoI and batch boundaries with prefetched groups): still BIT-EXACT vs
    the oracle's loop order, and bitwise reproducible."""
    from mx_det import ops
    monkeypatch.setenv("MX_ROI_DETERMINISTIC", "1")
    rng = np.random.default_rng(77)
    N, C = 1, 256
    shapes = [(60, 101), (30, 51), (15, 26), (8, 13)]
    scales = [0.25, 0.125, 0.0625, 0.03125]
    feats = [torch.from_numpy(rng.standard_normal((N, h, w, C)).astype(np.float32)) for h, w in shapes]
    K = 1100
    ctr = rng.uniform(90, 110, (K, 2))
    wh = rng.uniform(20, 90, (K, 2))
    boxes = np.concatenate([ctr - wh / 2, ctr + wh / 2], 1).astype(np.float32)
    rois = np.concatenate([np.zeros((K, 1), np.float32), boxes], 1)
    lv = _level_mapper_np(boxes)
    g = torch.from_numpy(rng.standard_normal((K, 7, 7, C)).astype(np.float32))
    rt = torch.from_numpy(rois).to(dev)

    def run():
        ft = [f.to(dev).requires_grad_(True) for f in feats]
        out = ops.multiscale_roi_align(ft, rt, scales, 2)
        return torch.autograd.grad(out, ft, g.to(dev))
    a, b = run(), run()
    gn = g.permute(0, 3, 1, 2).numpy()
    assert (lv == 0).sum() > 1000
    for l in range(4):
        assert torch.equal(a[l], b[l]), l
        sel = np.where(lv == l)[0]
        r = orc.roi_align_backward(gn[sel], rois[sel], scales[l], (N, C) + shapes[l], 2, False)
        assert np.array_equal(a[l].permute(0, 3, 1, 2).cpu().numpy(), r), l


def test_roi_align_backward_no_rois_writes_zeros(dev):
    """K = 0: the gather still writes every element of the (torch.empty) gradient map."""
    from mx_det import ops
    f = torch.randn(1, 20, 30, 64, device=dev).requires_grad_(True)
    out = ops.roi_align(f, torch.zeros((0, 5), device=dev), 7, 0.25, 2, False)
    (gf,) = torch.autograd.grad(out, f, torch.zeros_like(out))
    assert gf.shape == f.shape and (gf == 0).all()


def _level_mapper_np(boxes, k_min=2, k_max=5):
    # torchvision poolers.LevelMapper in f32 (CPU path)
    b = torch.from_numpy(boxes)
    s = torch.sqrt((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]))
    t = torch.floor(4 + torch.log2(s / 224) + torch.tensor(1e-6, dtype=s.dtype))
    t = torch.clamp(t, min=k_min, max=k_max)
    return (t.to(torch.int64) - k_min).numpy()


def test_multiscale_roi_align(dev):
    from mx_det import ops
    rng = np.random.default_rng(8)
    N, C = 2, 32
    shapes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    scales = [0.25, 0.125, 0.0625, 0.03125]
    feats = [rng.standard_normal((N, C, h, w)).astype(np.float32) for h, w in shapes]
    boxes = np.concatenate([_rand_boxes(rng, 200, med=30), _rand_boxes(rng, 200, med=200)])
    bi = rng.integers(0, N, len(boxes)).astype(np.float32)[:, None]
    rois = np.concatenate([bi, boxes], 1)
    lv = _level_mapper_np(boxes)
    ref = np.zeros((len(rois), C, 7, 7), np.float32)
    for l in range(4):
        sel = np.where(lv == l)[0]
        if len(sel):
            ref[sel] = orc.roi_align(feats[l], rois[sel], scales[l], (7, 7), 2, False)
    ft = [torch.from_numpy(f).to(dev).permute(0, 2, 3, 1).contiguous().requires_grad_(True) for f in feats]
    got = ops.multiscale_roi_align(ft, torch.from_numpy(rois).to(dev), scales, 2)
    assert np.array_equal(got.permute(0, 3, 1, 2).detach().cpu().numpy(), ref)
    g = rng.standard_normal(got.shape).astype(np.float32)
    got.backward(torch.from_numpy(g).to(dev))
    gn = torch.from_numpy(g).permute(0, 3, 1, 2).numpy()
    for l in range(4):
        sel = np.where(lv == l)[0]
        r = orc.roi_align_backward(gn[sel], rois[sel], scales[l], feats[l].shape, 2, False)
        np.testing.assert_allclose(ft[l].grad.permute(0, 3, 1, 2).cpu().numpy(), r, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_proposal_clip_filter_matches_torch(dev):
    """mx_proposal_clip_filter == filter_proposals' torch formulation (gather by the top-k indices,
    clamp(min=0) + minimum against (w, h), min-size and score masks, dead group N): bit-identical boxes
    incl. NaN / negative / out-of-image coordinates, identical groups."""
    from mx_det import ops
    rng = np.random.default_rng(5)
    N, A, T = 2, 5000, 3000
    props = rng.normal(600, 500, (N, A, 4)).astype(np.float32)
    props[0, :50] = np.nan
    props[1, 50:80, 2] = props[1, 50:80, 0] + 1e-4  # narrower than min_size
    pt = torch.from_numpy(props).to(dev)
    top = torch.from_numpy(np.stack([rng.choice(A, T, replace=False) for _ in range(N)])).to(dev)
    top[0, :60] = torch.arange(60, device=dev)
    prob = torch.from_numpy(rng.random((N, T)).astype(np.float32)).to(dev)
    hw = torch.tensor([[800.0, 1333.0], [768.0, 1344.0]], device=dev)
    for min_size, thr in ((1e-3, 0.0), (8.0, 0.3)):
        boxes, grp = ops.proposal_clip_filter(pt, top, prob, hw, min_size, thr)
        bi = torch.arange(N, device=dev)[:, None]
        rb = pt[bi, top]
        x = torch.minimum(rb[..., 0::2].clamp(min=0), hw[:, 1, None, None])
        y = torch.minimum(rb[..., 1::2].clamp(min=0), hw[:, 0, None, None])
        rb = torch.stack((x[..., 0], y[..., 0], x[..., 1], y[..., 1]), dim=-1)
        keep = (rb[..., 2] - rb[..., 0] >= min_size) & (rb[..., 3] - rb[..., 1] >= min_size) & (prob >= thr)
        rg = torch.where(keep, bi, N).reshape(-1)
        assert torch.equal(torch.isnan(boxes), torch.isnan(rb))
        assert torch.equal(torch.nan_to_num(boxes, nan=-7.0), torch.nan_to_num(rb, nan=-7.0))
        assert torch.equal(grp.long(), rg)


@pytest.mark.gpu
def test_roi_compact_matches_torch(dev):
    """mx_roi_compact == the torch formulation after the RoI sampler (ascending selected entries,
    rois = (entry // cm, box), labels / targets gathered): bit-identical, incl. an empty image row
    and a fully selected one."""
    from mx_det import ops
    from mx_det.frcnn import _compact
    rng = np.random.default_rng(9)
    N, cm = 3, 2064
    mask = torch.from_numpy(rng.random((N, cm)) < 0.25).to(dev)
    mask[1] = False
    mask[2, :700] = True
    box = torch.from_numpy(rng.normal(500, 300, (N * cm, 4)).astype(np.float32)).to(dev)
    lab = torch.from_numpy(rng.integers(-1, 8, N * cm)).to(dev)
    tg = torch.from_numpy(rng.normal(0, 1, (N * cm, 4)).astype(np.float32)).to(dev)
    sm = mask.flatten()
    total = int(sm.sum())
    rois, lo, to = ops.roi_compact(sm, total, cm, box, lab, tg)
    idx = _compact(sm, total)
    ref = torch.cat([(idx // cm).to(torch.float32)[:, None], box[idx]], 1)
    assert torch.equal(rois, ref) and torch.equal(lo, lab[idx]) and torch.equal(to, tg[idx])


@pytest.mark.gpu
def test_boxes_degenerate_flag(dev):
    """mx_boxes_degenerate == any((b[:, 2:] <= b[:, :2]).any()) over the target tensors (empty sets,
    zero-width / -height, NaN coordinates, more than 8 sets)."""
    from mx_det import ops
    rng = np.random.default_rng(2)

    def sets(n, bad=None):
        out = []
        for i in range(n):
            b = rng.uniform(0, 500, (int(rng.integers(0, 60)), 2)).astype(np.float32)
            b = np.concatenate([b, b + rng.uniform(1, 50, b.shape).astype(np.float32)], 1)
            out.append(torch.from_numpy(b).to(dev))
        if bad is not None:
            i, kind = bad
            b = torch.tensor([[10.0, 10.0, 10.0, 20.0]] if kind == "w" else
                             [[10.0, 10.0, 20.0, 5.0]] if kind == "h" else [[float("nan"), 1.0, 2.0, 3.0]], device=dev)
            out[i] = torch.cat([out[i], b])
        return out
    for n, bad in ((2, None), (2, (1, "w")), (3, (0, "h")), (2, (0, "nan")), (11, None), (11, (9, "w")), (1, None)):
        bl = sets(n, bad)
        ref = any(bool((b[:, 2:] <= b[:, :2]).any()) for b in bl)
        assert bool(ops.boxes_degenerate(bl)) == ref, (n, bad)


def test_box_decode(dev):
    from mx_det import ops
    rng = np.random.default_rng(11)
    boxes = _rand_boxes(rng, 4000, med=80)
    rel = rng.normal(0, 1.5, (4000, 28)).astype(np.float32)
    rel[0, 2] = 50.0  # exercises the dw clamp
    ref = orc.box_decode(rel, boxes, [10, 10, 5, 5])
    got = ops.box_decode(torch.from_numpy(rel).to(dev), torch.from_numpy(boxes).to(dev), (10., 10., 5., 5.))
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-5, atol=1e-3)


def _img(rng, H=800, W=1333):
    base = rng.integers(0, 256, (H // 8 + 1, W // 8 + 1, 3)).astype(np.float32)
    low = np.kron(base, np.ones((8, 8, 1)))[:H, :W]
    return np.clip(low + rng.normal(0, 25, (H, W, 3)), 0, 255).astype(np.uint8)


def test_corruption_ops(dev):
    from mx_det import ops
    rng = np.random.default_rng(12)
    img = np.stack([_img(rng, 96, 133), _img(rng, 96, 133), _img(rng, 96, 133)])
    noise = rng.normal(0, 15, img.shape).astype(np.float32)
    t = torch.from_numpy(img).to(dev)
    got = ops.corrupt_u8(t, [1, 2, 3], noise=torch.from_numpy(noise).to(dev)).cpu().numpy()
    assert np.array_equal(got[0], orc.noise_u8(img[0], noise[0]))
    assert np.array_equal(got[1], orc.blur_u8(img[1]))
    assert np.array_equal(got[2], orc.lowres_u8(img[2], 0.5))


def test_noise_golden_from_reference(dev):
    """apply_noise pinned by the reference itself (tests/golden/noise.npz, make_golden.py)."""
    from mx_det import ops
    d = np.load("tests/golden/noise.npz")
    got = ops.corrupt_u8(torch.from_numpy(d["img"][None]).to(dev), [1],
                         noise=torch.from_numpy(d["noise"][None]).to(dev)).cpu().numpy()[0]
    assert np.array_equal(got, d["out"])


def test_corruption_full_size_properties(dev):
    """Full 1333x800: device Philox noise statistics; blur/lowres idempotent on flat images."""
    from mx_det import ops
    flat = torch.full((1, 800, 1333, 3), 117, dtype=torch.uint8, device=dev)
    for op in (2, 3):
        assert torch.equal(ops.corrupt_u8(flat, [op]), flat)
    z = torch.full((1, 800, 1333, 3), 128, dtype=torch.uint8, device=dev)
    n = ops.corrupt_u8(z, [1], sigma=15.0, seed=123).float() - 128
    # astype(uint8) truncates: floor(128 + N(0,15)) has mean -0.5, std sqrt(225 + 1/12)
    assert abs(n.mean().item() + 0.5) < 0.05 and abs(n.std().item() - 15.0) < 0.1


def test_normalize_pad(dev):
    from mx_det import ops
    rng = np.random.default_rng(13)
    img = np.stack([_img(rng, 50, 61), _img(rng, 50, 61)])
    got = ops.normalize_pad(torch.from_numpy(img).to(dev), (64, 64), channels=8).cpu()
    x = torch.from_numpy(img).float().mul_(1.0 / 255)
    ref = (x - torch.tensor(ops.IMAGE_MEAN)) / torch.tensor(ops.IMAGE_STD)
    assert torch.equal(got[:, :50, :61, :3], ref)
    assert got[:, 50:].abs().sum() == 0 and got[:, :, 61:].abs().sum() == 0 and got[..., 3:].abs().sum() == 0


@pytest.mark.parametrize("C", [256, 64])
def test_multiscale_roi_align_bf16_tiled(dev, C):
    """bf16 hot path: vectorised forward bit-exact vs the oracle on the bf16 feature values (rounded
    once); tiled gather backward (bf16 level grads, no atomics) vs the oracle scatter within bf16."""
    from mx_det import ops
    rng = np.random.default_rng(C)
    N = 2
    shapes = [(100, 168), (50, 84), (25, 42), (13, 21)]
    scales = [0.25, 0.125, 0.0625, 0.03125]
    feats = [torch.from_numpy(rng.standard_normal((N, h, w, C)).astype(np.float32)).bfloat16() for h, w in shapes]
    boxes = np.concatenate([_rand_boxes(rng, 150, H=400, W=672, med=20), _rand_boxes(rng, 150, H=400, W=672, med=150)])
    boxes[0] = [-30, -30, 700, 420]  # overhangs every edge
    bi = rng.integers(0, N, len(boxes)).astype(np.float32)[:, None]
    rois = np.concatenate([bi, boxes], 1).astype(np.float32)
    lv = _level_mapper_np(boxes)
    fn = [f.float().permute(0, 3, 1, 2).contiguous().numpy() for f in feats]
    ref = np.zeros((len(rois), C, 7, 7), np.float32)
    for l in range(4):
        sel = np.where(lv == l)[0]
        if len(sel):
            ref[sel] = orc.roi_align(fn[l], rois[sel], scales[l], (7, 7), 2, False)
    ft = [f.to(dev).requires_grad_(True) for f in feats]
    got = ops.multiscale_roi_align(ft, torch.from_numpy(rois).to(dev), scales, 2)
    assert got.dtype == torch.bfloat16
    refb = torch.from_numpy(ref).bfloat16().permute(0, 2, 3, 1)
    assert torch.equal(got.detach().cpu(), refb)
    g = torch.from_numpy(rng.standard_normal(got.shape).astype(np.float32)).bfloat16()
    got.backward(g.to(dev))
    gn = g.float().permute(0, 3, 1, 2).numpy()
    for l in range(4):
        sel = np.where(lv == l)[0]
        r = orc.roi_align_backward(gn[sel], rois[sel], scales[l], fn[l].shape, 2, False)
        gg = ft[l].grad.float().permute(0, 3, 1, 2).cpu().numpy()
        np.testing.assert_allclose(gg, r, rtol=1e-2, atol=1e-2)


def test_rpn_loss_fused_matches_torch(dev):
    """mx_rpn_loss_fwd / _bwd == torchvision's compute_loss formulation (BCE-with-logits mean over the
    sampled anchors, smooth-L1 beta 1/9 over positives / number sampled) and its autograd gradients."""
    import torch.nn.functional as F
    from mx_det import ops
    g = torch.Generator().manual_seed(5)
    N, A = 2, 70001
    x = (torch.randn(N, A, generator=g) * 3).to(dev).requires_grad_(True)
    d = torch.randn(N, A, 4, generator=g).to(dev).requires_grad_(True)
    t = torch.randn(N, A, 4, generator=g).to(dev)
    lab = (torch.randint(-1, 2, (N, A), generator=g)).float().to(dev)
    r = torch.rand(N, A, generator=g).to(dev)
    pm = (lab == 1) & (r < 0.01)
    nm = (lab == 0) & (r < 0.02)
    lo, lb = ops.rpn_loss(x, d, lab, t, pm, nm, 1.0 / 9)
    (lo * 1.5 + lb * 0.5).backward()
    gx, gd = x.grad.clone(), d.grad.clone()
    x.grad = d.grad = None
    sm = pm | nm
    cnt = sm.sum()
    ro = torch.where(sm, F.binary_cross_entropy_with_logits(x, lab.clamp(min=0), reduction="none"), 0.0).sum() / cnt
    rb = torch.where(pm, F.smooth_l1_loss(d, t, beta=1.0 / 9, reduction="none").sum(-1), 0.0).sum() / cnt
    (ro * 1.5 + rb * 0.5).backward()
    torch.testing.assert_close(lo, ro, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lb, rb, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gx, x.grad, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(gd, d.grad, rtol=1e-4, atol=1e-8)


def test_roi_loss_fused_matches_torch(dev):
    """mx_roi_loss_fwd / _bwd == fastrcnn_loss (cross-entropy mean; class-indexed smooth-L1 beta 1/9
    over positives / R) and its gradients, on strided views of one predictor output as in the model."""
    import torch.nn.functional as F
    from mx_det import ops
    g = torch.Generator().manual_seed(6)
    R, C = 1000, 7
    o = torch.randn(R, 5 * C, generator=g).to(dev).requires_grad_(True)
    lab = torch.randint(0, C, (R,), generator=g).to(dev)
    lab[torch.rand(R, generator=g).to(dev) < 0.7] = 0
    t = torch.randn(R, 4, generator=g).to(dev)
    lc, lb = ops.roi_loss(o[:, :C], o[:, C:], lab, t, 1.0 / 9)
    (lc * 0.7 + lb * 1.3).backward()
    go = o.grad.clone()
    o.grad = None
    cl, br = o[:, :C], o[:, C:]
    rc = F.cross_entropy(cl, lab)
    reg = br.reshape(R, -1, 4)[torch.arange(R, device=dev), lab]
    rb = torch.where(lab > 0, F.smooth_l1_loss(reg, t, beta=1.0 / 9, reduction="none").sum(-1), 0.0).sum() / R
    (rc * 0.7 + rb * 1.3).backward()
    torch.testing.assert_close(lc, rc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lb, rb, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(go, o.grad, rtol=1e-4, atol=1e-7)


def _level_topk_np(scores, num_per_level, k):
    """_get_top_n_idx by definition: per level the min(k, n) largest, value descending, ties by
    index ascending (the set at a tied threshold takes the lowest indices), + level offset."""
    out, off = [], 0
    for n in num_per_level:
        seg = scores[:, off:off + n]
        rows = []
        for r in seg:
            o = np.lexsort((np.arange(n), -r.astype(np.float64)))[:min(k, n)]
            rows.append(o + off)
        out.append(np.stack(rows) if rows else np.zeros((scores.shape[0], 0), np.int64))
        off += n
    return np.concatenate(out, 1)


@pytest.mark.parametrize("case", ["train", "logits", "uniform", "ties", "edges", "flat"])
def test_level_topk(dev, case):
    """mx_level_topk == the per-level topk of RegionProposalNetwork._get_top_n_idx: exact indices vs
    the definition (value desc, index asc) and exact values vs torch.topk on the CPU. "logits" (one
    exponent band, an untrained RPN's objectness) and "uniform" (the samplers' keys) put most lanes of
    a wave on a few first-digit bins of the radix select."""
    from mx_det import ops
    rng = np.random.default_rng(21)
    if case == "train":  # bs=2 at 1344x800: P2..P6 anchors per level, pre_nms_top_n=2000
        levels, k = [201600, 50400, 12600, 3150, 819], 2000
        s = rng.standard_normal((2, sum(levels))).astype(np.float32)
    elif case == "logits":
        levels, k = [201600, 50400, 12600, 3150, 819], 2000
        s = (0.01 + 0.001 * rng.standard_normal((2, sum(levels)))).astype(np.float32)
    elif case == "uniform":
        levels, k = [268569], 256
        s = rng.random((2, sum(levels))).astype(np.float32)
    elif case == "ties":  # heavy ties at every threshold (quantised logits), eval k=1000
        levels, k = [40000, 10000, 2500, 700], 1000
        s = (np.round(rng.standard_normal((3, sum(levels))) * 4) / 4).astype(np.float32)
        s[1, :] = 0.5  # a row of one value: every level is one tie
        s[2, ::7] = -0.0  # -0.0 and +0.0 compare equal: ties
    elif case == "flat":  # sliced levels whose slices tie at the threshold (merge's many-ties path)
        levels, k = [201600, 24577, 60000], 2000
        s = (np.round(rng.standard_normal((3, sum(levels))) * 2) / 2).astype(np.float32)
        s[1, :] = 0.25  # one value: 9 slices x 2000 ties reach the merge
        s[2, 100000:] = 7.0  # the top 2000 ties sit in later slices only
    else:  # tiny / empty levels, k=1, infinities, k > n
        levels, k = [5, 0, 3000, 1, 64], 1
        s = rng.standard_normal((2, sum(levels))).astype(np.float32)
        s[0, 10:20] = np.inf
        s[1, 5:3005] = -np.inf
        s[1, 7] = -3.0
    ref = _level_topk_np(s, levels, k)
    st = torch.from_numpy(s)
    got = ops.level_topk(st.to(dev), levels, k).cpu().numpy()
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
    tv, off = [], 0
    for n in levels:
        tv.append(st[:, off:off + n].topk(min(k, n), dim=1).values)
        off += n
    assert torch.equal(torch.gather(st, 1, torch.from_numpy(got)), torch.cat(tv, 1))
    if case == "edges":
        got2 = ops.level_topk(st.to(dev), levels, 5000).cpu().numpy()  # k >= every n: full sorts
        assert np.array_equal(got2, _level_topk_np(s, levels, 5000))


def test_level_topk_sliced_matches_single_workgroup(dev, monkeypatch):
    """Slicing long levels over many workgroups (+ the merge launch) returns exactly the indices of
    the one-workgroup-per-level path, on the RPN's training shape."""
    from mx_det import ops
    rng = np.random.default_rng(5)
    levels, k = [201600, 50400, 12600, 3150, 819], 2000
    st = torch.from_numpy((0.01 + 0.001 * rng.standard_normal((2, sum(levels)))).astype(np.float32)).to(dev)
    monkeypatch.setenv("MX_TOPK_SLICED", "1")
    a = ops.level_topk(st, levels, k)
    monkeypatch.setenv("MX_TOPK_SLICED", "0")
    b = ops.level_topk(st, levels, k)
    assert torch.equal(a, b)


def test_sampler_draw_via_level_topk(dev):
    """BalancedPositiveNegativeSampler with the HIP backend (RoI-head rows: the k smallest uniform
    keys drawn with mx_level_topk): per image exactly min(#pos, 128) positives and min(#neg,
    512 - pos) negatives, each a subset of its candidates; a fresh draw differs; rows with fewer
    candidates than k (the non-candidate key ties) included."""
    from mx_det.backend import HipBackend
    from mx_det.frcnn import BalancedPositiveNegativeSampler
    torch.manual_seed(3)
    L = 2100
    lab = torch.full((3, L), -1, dtype=torch.int64)
    lab[0, torch.randperm(L)[:40]] = 1            # fewer positives than k=128
    lab[0, torch.randperm(L)[:1500]] = 0
    lab[1, :700] = 1
    lab[1, 700:] = 0
    lab[2, :100] = 0                              # fewer negatives than 512 - 0
    lab = lab.to(dev)
    s = BalancedPositiveNegativeSampler(512, 0.25)
    be = HipBackend()
    pm, nm = s(lab, be)
    pos, neg = lab >= 1, lab == 0
    npos = pos.sum(1).clamp(max=128)
    nneg = torch.minimum(neg.sum(1), 512 - npos)
    assert torch.equal(pm.sum(1), npos) and torch.equal(nm.sum(1), nneg)
    assert not (pm & ~pos).any() and not (nm & ~neg).any()
    pm2, _ = s(lab, be)
    assert not torch.equal(pm2[1], pm[1])  # 128 of 700 positives redrawn


def test_sampler_picks_equal_topk_on_same_keys_and_are_uniform(dev):
    """The level_topk draw picks exactly the candidates torch.topk(largest=False) picks on the same
    injected keys (the k smallest keys: randperm[:k] semantics), and over 400 fresh draws every
    candidate is picked with frequency k / #candidates (+-5 sigma), non-candidates never: no bias
    from filler-key ties or index order."""
    from mx_det.backend import HipBackend
    from mx_det.frcnn import BalancedPositiveNegativeSampler
    torch.manual_seed(4)
    L = 2100
    lab = torch.full((2, L), -1, dtype=torch.int64)
    lab[0, :700] = 1
    lab[0, 700:1900] = 0
    lab[1, torch.randperm(L)[:300]] = 1
    lab[1, torch.randperm(L)[:900]] = 0
    lab = lab.to(dev)
    s = BalancedPositiveNegativeSampler(512, 0.25)
    g = torch.Generator().manual_seed(11)
    keys = torch.rand(lab.shape, generator=g).to(dev)
    s.rand = lambda shape, device: keys
    pm, nm = s(lab, HipBackend())
    pt, nt = s(lab, None)
    assert torch.equal(pm, pt) and torch.equal(nm, nt)
    s.rand = None
    cnt = torch.zeros(lab.shape, device=dev)
    n = 400
    for _ in range(n):
        p, _ = s(lab, HipBackend())
        cnt += p
    pos = lab >= 1
    for r in range(2):
        c = int(pos[r].sum())
        k = min(128, c)
        f = cnt[r][pos[r]] / n
        sd = (k / c * (1 - k / c) / n) ** 0.5
        assert (f - k / c).abs().max().item() < 5 * sd + 1e-6, (r, f.min().item(), f.max().item(), k / c)
        assert cnt[r][~pos[r]].sum().item() == 0


@pytest.mark.parametrize("k,angle", [(9, 0), (9, 45), (9, 90), (7, 30), (11, 135), (5, -20)])
def test_motion_blur_any_angle(dev, k, angle):
    """apply_motion_blur at any kernel size / angle (augmentations.py:21-38): the device filter2D on
    the restated kernel equals the oracle's filter2D restatement bit for bit."""
    from mx_det import augment as aug
    rng = np.random.default_rng(k * 100 + angle % 360)
    img = _img(rng, 61, 87)
    got = aug.apply_motion_blur(img, k, angle)
    assert np.array_equal(got, orc.motion_blur_u8(img, k, angle))


@pytest.mark.parametrize("H,W", [(96, 134), (80, 132), (64, 2 * 81)])
def test_lowres_even_frames_take_the_area_fast_path(dev, H, W):
    """Even x even frames (VisDrone 1920x1080, 2000x1500) take OpenCV's exact-x2 INTER_AREA path."""
    from mx_det import ops
    rng = np.random.default_rng(H + W)
    img = np.stack([_img(rng, H, W), _img(rng, H, W)])
    got = ops.corrupt_u8(torch.from_numpy(img).to(dev), [3, 3]).cpu().numpy()
    for b in range(2):
        small = orc.resize_area_fast2_u8(img[b])
        assert np.array_equal(got[b], orc.resize_linear_u8(small, H, W))
        assert np.array_equal(got[b], orc.lowres_u8(img[b], 0.5))


def test_random_corruption_matches_reference_golden(dev):
    """RandomCorruption(p=0.5) (PIL transform) under the reference's seeded random / numpy streams:
    identical output to the reference for every seed whose reference output needs no OpenCV
    (keep or noise on the BGR view; tests/golden/random_corruption.npz)."""
    import random
    from PIL import Image
    from mx_det import augment as aug
    d = np.load("tests/golden/random_corruption.npz")
    img = Image.fromarray(d["img"])
    for s, out, pinned in zip(d["seeds"], d["outs"], d["pinned"]):
        if not pinned:
            continue
        random.seed(int(s))
        np.random.seed(int(s))
        got = np.asarray(aug.RandomCorruption(p=0.5)(img))
        assert np.array_equal(got, out), int(s)


def test_rpn_head_split_merge_equals_torch_slicing(dev):
    """ops.rpn_head_split (one gather) / its backward (one scatter writing every element, frame pixels
    0) == torchvision's per-level permute / reshape / cat over the level map and the canvas slices."""
    from mx_det import frcnn, ops
    torch.manual_seed(3)
    A, N = 3, 2
    hws = [(25, 42), (13, 21), (7, 11), (4, 6)]
    pos, Hc, Wc = frcnn.RPNHead.canvas_layout(hws)
    rects = [(y, x, h, w) for (y, x), (h, w) in zip(pos, hws)]
    o0 = torch.randn(N, 50, 84, 5 * A, device=dev, requires_grad=True)
    ocv = torch.randn(N, Hc, Wc, 5 * A, device=dev, requires_grad=True)
    obj, dl = ops.rpn_head_split(o0, ocv, rects, A)
    outs = [o0] + [ocv[:, y:y + h, x:x + w] for y, x, h, w in rects]
    robj = torch.cat([o[..., :A].reshape(N, -1) for o in outs], 1)
    rdl = torch.cat([o[..., A:].reshape(N, -1, 4) for o in outs], 1)
    assert torch.equal(obj, robj) and torch.equal(dl, rdl)
    go, gd = torch.randn_like(obj), torch.randn_like(dl)
    g0, gcv = torch.autograd.grad((obj, dl), (o0, ocv), (go, gd))
    r0, rcv = torch.autograd.grad((robj, rdl), (o0, ocv), (go, gd))
    assert torch.equal(g0, r0) and torch.equal(gcv, rcv)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_canvas_pack_unpack_equals_torch(dev, dtype):
    """ops.canvas_pack: the zero-framed canvas of the small levels (frcnn.RPNHead) == zeros + slice
    copies; its backward == the slices of the canvas gradient, plus the absorbed root gradients
    (conv.GradSlot) when given."""
    from mx_det import conv as mc, frcnn, ops
    torch.manual_seed(5)
    hws = [(25, 42), (13, 21), (7, 11), (4, 6)]
    pos, Hc, Wc = frcnn.RPNHead.canvas_layout(hws)
    rects = [(y, x, h, w) for (y, x), (h, w) in zip(pos, hws)]
    maps = [torch.randn(2, h, w, 256, device=dev).to(dtype).requires_grad_(True) for h, w in hws]
    slots = [mc.GradSlot() for _ in hws]
    for s, (h, w) in zip(slots[::2], hws[::2]):
        s.buf = torch.randn(2, h, w, 256, device=dev).to(dtype)
    cv = ops.canvas_pack(maps, rects, Hc, Wc, slots)
    ref = torch.zeros(2, Hc, Wc, 256, device=dev, dtype=dtype)
    for m, (y, x, h, w) in zip(maps, rects):
        ref[:, y:y + h, x:x + w] = m.detach()
    assert torch.equal(cv, ref)
    g = torch.randn_like(cv)
    grads = torch.autograd.grad(cv, maps, g)
    for gr, s, (y, x, h, w) in zip(grads, slots, rects):
        want = g[:, y:y + h, x:x + w]
        if s.buf is not None:
            want = (want.float() + s.buf.float()).to(dtype)
        assert torch.equal(gr, want)


@pytest.mark.parametrize("C", [64, 256])
def test_roi_align_fwd_wide_channels_bitexact(dev, C):
    """The 8-channel-vector forward (roi_align_fwd_v8_kernel) at C = 64 / 256 over small and large RoIs,
    RoIs partly or wholly outside the map: bit-identical to the oracle (same per-element op order)."""
    from mx_det import ops
    rng = np.random.default_rng(C)
    N, H, W, scale = 2, 100, 168, 1 / 8
    feat = rng.standard_normal((N, C, H, W)).astype(np.float32)
    small = _rand_boxes(rng, 150, H=H / scale, W=W / scale, med=40)
    large = _rand_boxes(rng, 40, H=H / scale, W=W / scale, med=400)
    b = np.concatenate([small, large])
    b[0] = [-20, -30, 5, 5]
    b[1] = [3, 3, 3.2, 3.1]
    b[2] = [-400, -400, -300, -300]  # no sample inside the map: zeros
    bi = rng.integers(0, N, len(b)).astype(np.float32)[:, None]
    rois = np.concatenate([bi, b], 1).astype(np.float32)
    ref = orc.roi_align(feat, rois, scale, (7, 7), 2, False)
    f = torch.from_numpy(feat).to(dev).permute(0, 2, 3, 1).contiguous()
    got = ops.roi_align(f, torch.from_numpy(rois).to(dev), (7, 7), scale, 2, False).permute(0, 3, 1, 2).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
