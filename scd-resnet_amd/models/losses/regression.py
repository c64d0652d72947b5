"""Masked regression losses (models/losses/regression.py:28-44 of the reference).

``L1LossMask`` keeps the reference signature; CenterNetLoss recognises it and runs the
fused gather + L1 kernel (scd_l1_gather_fwd) instead.  ``smoothL1LossMask`` is API-only
(unused by the benchmarked plugins).
"""
import torch.nn.functional as F


def smoothL1LossMask(regression, groundTruth, mask):
    num = mask.float().sum()
    m = mask.bool().unsqueeze(2).expand_as(groundTruth)
    return F.smooth_l1_loss(regression[m], groundTruth[m], reduction="sum") / (num + 1e-4)


def L1LossMask(regression, groundTruth, mask):
    num = mask.float().sum()
    m = mask.bool().unsqueeze(2).expand_as(groundTruth)
    return F.l1_loss(regression[m], groundTruth[m], reduction="sum") / (num + 1e-4)
