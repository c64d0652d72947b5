"""Penalty-reduced focal loss (models/losses/focal.py:25-53 of the reference).

``focalLoss`` keeps the reference signature for user code and runs on libscdhip (scdhip.api.focal_loss:
scd_focal_prob_fwd writes the per-element gradient and the posL / negL / #pos sums, the normaliser stays on the
device).  CenterNetLoss/CornerNetLoss recognise it and run the fused logits kernel (scd_focal_fwd, sigmoid and
clamp folded in) instead.
"""
from scdhip import api


def focalLoss(prediction, groundTruth, alpha=2, beta=4):
    if (alpha, beta) != (2, 4):
        raise NotImplementedError("focalLoss: the reference's alpha=2, beta=4 only")
    return api.focal_loss(list(prediction), groundTruth)
