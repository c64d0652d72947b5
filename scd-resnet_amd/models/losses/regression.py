"""Masked regression losses (models/losses/regression.py:28-44 of the reference).

``L1LossMask`` / ``smoothL1LossMask`` keep the reference signatures and run on libscdhip (scdhip.api.masked_l1:
scd_masked_l1_fwd, normaliser #mask + 1e-4 kept on the device).  CenterNetLoss recognises L1LossMask and runs the
fused gather + L1 kernel (scd_l1_gather_fwd) instead.
"""
from scdhip import api


def smoothL1LossMask(regression, groundTruth, mask):
    return api.masked_l1(regression, groundTruth, mask, smooth=True)


def L1LossMask(regression, groundTruth, mask):
    return api.masked_l1(regression, groundTruth, mask, smooth=False)
