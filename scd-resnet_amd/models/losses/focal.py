"""Penalty-reduced focal loss (models/losses/focal.py:25-53 of the reference).

``focalLoss`` keeps the reference signature for user code; CenterNetLoss/CornerNetLoss
recognise it and run the fused device kernel (scd_focal_fwd: per-element gradient,
fp64 posL/negL/#pos accumulators, normaliser applied on device) instead.
"""
import torch


def focalLoss(prediction, groundTruth, alpha=2, beta=4):
    pos = groundTruth.eq(1)
    neg = groundTruth.lt(1)
    negw = torch.pow(1 - groundTruth[neg], beta)
    loss = 0
    for pred in prediction:
        pp, npred = pred[pos], pred[neg]
        posl = (torch.log(pp) * torch.pow(1 - pp, alpha)).sum()
        negl = (torch.log(1 - npred) * torch.pow(npred, alpha) * negw).sum()
        if pp.nelement() == 0:
            loss = loss - negl
        else:
            loss = loss - (posl + negl) / pos.float().sum()
    return loss
