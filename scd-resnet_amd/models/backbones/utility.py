"""Backbone utilities (models/backbones/utility.py of the reference).

``convolution3x3`` builds the module used by BasicBlock.  The functional helpers keep the
reference API for user code and evaluation and run on libscdhip (scdhip.api: scd_nms, scd_topk);
on the training/decode path the fused kernels take their place: gather + clampSigmoid inside
scdhip.loss.CenterNetLossFn, NMS + top-K + gather inside scdhip.ops.decode_topk.
"""
import torch

from scdhip import api, ops


def convolution3x3(inputDimension, outputDimension, stride=1):
    """utility.py:125-127"""
    return torch.nn.Conv2d(inputDimension, outputDimension, kernel_size=3, stride=stride, padding=1, bias=False)


def gatherFeatures(feature, indices, mask=None):
    """utility.py:76-84: (B, HW, C) gathered at (B, K) -> (B, K, C)."""
    dimension = feature.size(2)
    indices = indices.unsqueeze(2).expand(indices.size(0), indices.size(1), dimension)
    feature = feature.gather(1, indices)
    if mask is not None:
        mask = mask.unsqueeze(2).expand_as(feature)
        feature = feature[mask].view(-1, dimension)
    return feature


def reshapeGatherFeatures(feat, ind):
    """utility.py:94-98"""
    feat = feat.permute(0, 2, 3, 1).contiguous()
    feat = feat.view(feat.size(0), -1, feat.size(3))
    return gatherFeatures(feat, ind)


def nonMaximumSuppression(heat, kernelSize=3):
    """utility.py:87-92: heat * (maxpool_kxk(heat) == heat) (scd_nms)."""
    return api.nms(heat, kernelSize)


def extractTopK(scores, K=20):
    """utility.py:106-118 (returns scores, inds, categories, ys, xs; scd_topk, ties by ascending index)."""
    return api.topk(scores, K)


def clampSigmoid(x):
    """utility.py:120-122 (in place, as the reference)."""
    return torch.clamp(x.sigmoid_(), min=1e-4, max=1 - 1e-4)


def decodeTopK(heat, offset=None, regr=None, K=100):
    """Fused sigmoid -> 3x3 NMS -> top-K -> gather on device (libscdhip)."""
    return ops.decode_topk(heat, offset, regr, K)
