"""BalancedPositiveNegativeSampler's host paths (CPU, no GPU): the torch.topk draw agrees with the
oracle's stable-sort restatement (oracle.balanced_sample) on distinct keys, and a validity mask means
exactly "label -1 there" -- the contract mx_sample_draw's valid operand implements on the device
(tests/test_gpu_sample.py)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc


def _sampler(batch, frac, keys):
    from mx_det import frcnn
    s = frcnn.BalancedPositiveNegativeSampler(batch, frac)
    s.rand = lambda shape, device: keys
    return s


@pytest.mark.parametrize("N,L,batch,frac,int_labels", [(2, 3000, 256, 0.5, False), (3, 700, 512, 0.25, True),
                                                       (1, 50, 256, 0.5, True)])
def test_cpu_draw_matches_oracle(N, L, batch, frac, int_labels):
    g = torch.Generator().manual_seed(L)
    u = torch.rand(N, L, generator=g)
    lab = torch.full((N, L), -1.0)
    lab[u < 0.8] = 0.0
    lab[u < 0.05] = 1.0
    if int_labels:
        lab = torch.where(lab == 1, torch.randint(1, 7, (N, L), generator=g).float(), lab).long()
    keys = (torch.randperm(N * L, generator=g).float() / (N * L)).reshape(N, L)  # distinct keys
    pos, neg = _sampler(batch, frac, keys)(lab)
    rp, rn, _ = orc.balanced_sample(lab.numpy(), keys.numpy(), batch, frac)
    assert np.array_equal(pos.numpy(), rp) and np.array_equal(neg.numpy(), rn)


def test_valid_mask_is_label_masking():
    g = torch.Generator().manual_seed(3)
    lab = torch.randint(-1, 3, (2, 900), generator=g)
    valid = torch.rand(2, 900, generator=g) < 0.6
    keys = (torch.randperm(1800, generator=g).float() / 1800).reshape(2, 900)
    p0, n0 = _sampler(512, 0.25, keys)(torch.where(valid, lab, -1))
    p1, n1 = _sampler(512, 0.25, keys)(lab, valid=valid)
    assert torch.equal(p0, p1) and torch.equal(n0, n1)
    assert not (p1 & ~valid).any() and not (n1 & ~valid).any()
