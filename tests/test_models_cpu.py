"""CPU checks of model-level loss forms."""

import torch


def test_ssd_loss_reference_matches_argsort_form():
    """ops.ssd_loss_reference (stable, positives never mined) equals the
    double-argsort form of tcb's loss when no mined value ties."""
    import torch.nn.functional as tF
    from kf_benchmarks_amd.ops import nn as F_ops
    B, A, C = 3, 500, 11
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(B, A, 4 + C, generator=g)
    gt_loc = torch.randn(B, A, 4, generator=g)
    lab = torch.where(torch.rand(B, A, generator=g) < 0.05,
                      torch.randint(1, C, (B, A), generator=g), torch.zeros(B, A).long())
    nm = (lab > 0).sum(1).float().clamp(min=1)
    ce = tF.cross_entropy(logits[..., 4:].reshape(-1, C), lab.reshape(-1),
                          reduction="none").reshape(B, A)
    pos = (lab > 0).float()
    rank = (ce * (1 - pos)).argsort(1, descending=True).argsort(1)
    neg = (rank < (nm.long() * 3)[:, None]).float()
    cls = ((ce * (pos + neg)).sum(1) / nm).mean()
    sl1 = tF.smooth_l1_loss(logits[..., :4], gt_loc, reduction="none").sum(2)
    loc = ((sl1 * pos).sum(1) / nm).mean()
    got = F_ops.ssd_loss(logits, gt_loc, lab.float(), nm)
    torch.testing.assert_close(got, cls + loc)
