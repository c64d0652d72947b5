"""The reference's functional helpers on libscdhip (api.hip), for user code that calls them directly.

nonMaximumSuppression / extractTopK (models/backbones/utility.py:87-118), focalLoss (models/losses/focal.py:25-53),
L1LossMask / smoothL1LossMask (models/losses/regression.py:28-44).  The losses are autograd Functions: the forward
kernel writes the per-element gradient, the normaliser stays on the device (scd_centernet_loss_finalize factors) and
the backward scales the saved gradient by it -- no host synchronisation, as in the fused training loss (loss.py).
"""
import ctypes

import torch

from . import lib as L
from . import ops


def nms(heat, kernel=3):
    """heat * (maxpool_kxk(heat) == heat) on (..., H, W) fp32 (utility.py:87-92)."""
    ops._need_gpu(heat)
    h = heat.float().contiguous()
    H, W = h.shape[-2], h.shape[-1]
    out = torch.empty_like(h)
    L.call("scd_nms", ops.ptr(h), h.numel() // (H * W), H, W, int(kernel), ops.ptr(out), ops.stream())
    return out


def topk(scores, K):
    """(B, C, H, W) scores -> topKScores, topKIndices (% H*W), topKCategories (int32), ys, xs (float) as
    utility.py:106-118 returns them; ties by ascending flat index (torch.topk leaves tie order open)."""
    ops._need_gpu(scores)
    B, C, H, W = scores.shape
    s = scores.float().contiguous()
    dev = s.device
    out = torch.empty(B, K, device=dev)
    inds = torch.empty(B, K, dtype=torch.int64, device=dev)
    cats = torch.empty(B, K, dtype=torch.int32, device=dev)
    ys = torch.empty(B, K, device=dev)
    xs = torch.empty(B, K, device=dev)
    L.call("scd_topk", ops.ptr(s), B, C * H * W, int(K), H * W, W, ops.ptr(out), ops.ptr(inds), ops.ptr(cats),
           ops.ptr(ys), ops.ptr(xs), ops.stream())
    return out, inds, cats, ys, xs


def _finalize(facc, nfocal, lacc, nl1, weights):
    dev = (facc if facc is not None else lacc).device
    out = torch.empty(1 + nfocal + nl1, device=dev)
    factors = torch.empty(max(1, nfocal + nl1), device=dev)
    w = (ctypes.c_float * max(1, nl1))(*weights)
    L.call("scd_centernet_loss_finalize", ops.ptr(facc), nfocal, ops.ptr(lacc), nl1, w, ops.ptr(out),
           ops.ptr(factors), ops.stream())
    return out, factors


class FocalLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gt, *preds):
        gt = gt.float().contiguous()
        dev = gt.device
        facc = torch.zeros(len(preds) * L.STAT_REPLICAS * 4, dtype=torch.float64, device=dev)
        grads = []
        for f, p in enumerate(preds):
            if p.shape != gt.shape:
                raise RuntimeError("focalLoss: prediction and ground truth shapes differ")
            p = p.float().contiguous()
            g = torch.empty_like(p)
            L.call("scd_focal_prob_fwd", ops.ptr(p), ops.ptr(gt), p.numel(), ops.ptr(g),
                   ops.ptr(facc[f * L.STAT_REPLICAS * 4:]), ops.stream())
            grads.append(g)
        out, factors = _finalize(facc, len(preds), None, 0, [])
        ctx.save_for_backward(factors, *grads)
        return out[0:1].reshape(())

    @staticmethod
    def backward(ctx, go):
        factors, *grads = ctx.saved_tensors
        res = []
        for f, g in enumerate(grads):
            g = g.clone()
            L.call("scd_scale_by_device", ops.ptr(g), g.numel(), ops.ptr(factors), f, ops.ptr(go.reshape(1)),
                   ops.stream())
            res.append(g)
        return (None, *res)


def focal_loss(prediction, groundTruth):
    """focal.py:25-53 (alpha 2, beta 4): prediction is a list of probability maps shaped like groundTruth."""
    ops._need_gpu(groundTruth, *prediction)
    return FocalLossFn.apply(groundTruth, *prediction)


class MaskedL1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, t, mask, smooth):
        if r.shape != t.shape or tuple(mask.shape) != tuple(r.shape[:-1]):
            raise RuntimeError("L1LossMask: regression (B, K, C), groundTruth (B, K, C), mask (B, K) expected")
        rr = r.float().contiguous()
        tt = t.float().contiguous()
        m = mask.contiguous()
        m = m.view(torch.uint8) if m.dtype == torch.bool else (m != 0).to(torch.uint8)
        lacc = torch.zeros(2, dtype=torch.float64, device=r.device)
        g = torch.empty_like(rr)
        L.call("scd_masked_l1_fwd", ops.ptr(rr), ops.ptr(tt), ops.ptr(m), m.numel(), rr.shape[-1], int(smooth),
               ops.ptr(g), ops.ptr(lacc), ops.stream())
        out, factors = _finalize(None, 0, lacc, 1, [1.0])
        ctx.save_for_backward(factors, g)
        return out[0:1].reshape(())

    @staticmethod
    def backward(ctx, go):
        factors, g = ctx.saved_tensors
        g = g.clone()
        L.call("scd_scale_by_device", ops.ptr(g), g.numel(), ops.ptr(factors), 0, ops.ptr(go.reshape(1)), ops.stream())
        return g, None, None, None


def masked_l1(regression, groundTruth, mask, smooth=False):
    ops._need_gpu(regression, groundTruth, mask)
    return MaskedL1Fn.apply(regression, groundTruth, mask, bool(smooth))
