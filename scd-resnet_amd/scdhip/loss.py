"""Fused device-side CenterNet / CornerNet losses (no host syncs).

CenterNetLoss.forward (centerNetOffset.py:182-217) =
    focal(clampSigmoid(heatmap), gt)                       focal.py:25-53
  + wr * L1LossMask(gather(regr, inds), gt[..., 2:6], mask)  regression.py:37-44
  + wo * L1LossMask(gather(offset, inds), gt[..., 0:2], mask)
The reference's boolean-mask indexing (a `nonzero` host sync per call) and the Python
`#pos == 0` branch are replaced by device accumulators and a finalize kernel; the
normalisers stay on device and scale the saved per-element gradients in backward.
"""
import torch

from . import lib as L
from . import ops


_ONES = {}


def mean_backward(loss):
    """``loss = loss.mean(); loss.backward()`` of the reference step (networkFactory.py:257-263) without ATen launches
    when the loss is one element (the fused losses return out[0:1]): the mean is then a view, and the seed gradient a
    persistent 0-dim one (backward() would fill a fresh ones tensor and MeanBackward divide it by numel: three
    small kernels on the critical path between the loss and the heads' backward).  Returns the 0-dim mean."""
    if loss.numel() != 1:
        m = loss.mean()
        m.backward()
        return m
    m = loss.reshape(())
    key = (m.device, m.dtype)
    one = _ONES.get(key)
    if one is None:
        one = torch.ones((), dtype=m.dtype, device=m.device)
        _ONES[key] = one
    m.backward(one)
    return m


class CenterNetLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, heat, regr, off, gt_heat, mask, regr_t, inds, wr, wo):
        ops._need_gpu(heat, gt_heat)
        heat, regr, off = heat.contiguous(), regr.contiguous(), off.contiguous()
        N, _, H, W = heat.shape
        HW = H * W
        K = inds.shape[1]
        dev = heat.device
        mask_u8 = mask.contiguous()
        mask_u8 = mask_u8.view(torch.uint8) if mask_u8.dtype == torch.bool else mask_u8.to(torch.uint8)
        inds = ops.hinted_inds(inds)
        regr_t = regr_t.float().contiguous()
        gt_heat = gt_heat.float().contiguous()
        s = ops.stream()
        g_heat = torch.empty_like(heat)
        facc = _acc_buffer(dev, "focal", L.STAT_REPLICAS * 4)
        # one buffer for both scattered L1 gradients (zero-filled by the first launch)
        g_both = torch.empty(regr.numel() + off.numel(), dtype=regr.dtype, device=dev)
        g_regr = g_both[:regr.numel()].view(regr.shape)
        g_off = g_both[regr.numel():].view(off.shape)
        out = torch.empty(4, device=dev)
        factors = torch.empty(3, device=dev)
        L.call("scd_centernet_loss_fwd", ops.ptr(heat), ops.ptr(gt_heat), heat.numel(), ops.ptr(regr), regr.shape[1],
               ops.ptr(off), off.shape[1], N, HW, ops.ptr(inds), ops.ptr(mask_u8), ops.ptr(regr_t), K,
               regr_t.shape[2], 2, 0, ctypes_float2(wr, wo), ops.ptr(g_heat), ops.ptr(g_regr), ops.ptr(g_off),
               ops.ptr(facc), ops.ptr(out), ops.ptr(factors), s)
        ctx.save_for_backward(g_heat, g_regr, g_off, factors)
        ctx.inds = inds
        ops.clear_sparse_grads()          # a new loss: earlier certificates are consumed or stale
        loss = out[0:1]
        stats = out[1:4]
        ctx.mark_non_differentiable(stats)
        # the statistics never carry a gradient: without this autograd fills a zeros tensor for them (one ATen launch
        # between the loss and the heads' backward)
        ctx.set_materialize_grads(False)
        return loss, stats

    @staticmethod
    def backward(ctx, gl, gstats):
        g_heat, g_regr, g_off, factors = ctx.saved_tensors
        gl = gl.contiguous() if gl is not None else torch.ones(1, device=g_heat.device)
        N, Cr, H, W = g_regr.shape
        L.call("scd_centernet_loss_bwd_scale", ops.ptr(g_heat), g_heat.numel(), N, H * W, ops.ptr(ctx.inds),
               ctx.inds.shape[1], ops.ptr(g_regr), Cr, ops.ptr(g_off), g_off.shape[1], ops.ptr(factors), ops.ptr(gl),
               ops.stream())
        # the L1 terms reach the size / offset outputs only at the gathered pixels (g_regr, g_off share one buffer)
        ops.certify_sparse_grad(g_regr, ctx.inds)
        return g_heat, g_regr, g_off, None, None, None, None, None, None


class FocalOnlyLossFn(torch.autograd.Function):
    """CornerNetLoss.forward (cornerNetCPool.py:244-272): sum of focal losses on several maps."""

    @staticmethod
    def forward(ctx, *args):
        n = len(args) // 2
        heats, gts = args[:n], args[n:]
        dev = heats[0].device
        s = ops.stream()
        facc = _acc_buffer(dev, "focal%d" % n, n * L.STAT_REPLICAS * 4)
        grads = []
        for i, (h, g) in enumerate(zip(heats, gts)):
            h = h.contiguous()
            gh = torch.empty_like(h)
            L.call("scd_focal_fwd", ops.ptr(h), ops.ptr(g.float().contiguous()), h.numel(), ops.ptr(gh),
                   ops.ptr(facc[i * L.STAT_REPLICAS * 4:]), s)
            grads.append(gh)
        out = torch.empty(1 + n, device=dev)
        factors = torch.empty(n, device=dev)
        L.call("scd_centernet_loss_finalize", ops.ptr(facc), n, 0, 0, ctypes_float2(0.0, 0.0), ops.ptr(out),
               ops.ptr(factors), s)
        ctx.save_for_backward(factors, *grads)
        stats = out[1:]
        ctx.mark_non_differentiable(stats)
        # the statistics never carry a gradient: without this autograd fills a zeros tensor for them (one ATen launch
        # between the loss and the heads' backward)
        ctx.set_materialize_grads(False)
        return out[0:1], stats

    @staticmethod
    def backward(ctx, gl, gstats):
        factors, *grads = ctx.saved_tensors
        gl = gl.contiguous() if gl is not None else torch.ones(1, device=factors.device)
        s = ops.stream()
        for i, g in enumerate(grads):
            L.call("scd_scale_by_device", ops.ptr(g), g.numel(), ops.ptr(factors), i, ops.ptr(gl), s)
        return tuple(grads) + (None,) * len(grads)


_ACC = {}


def _acc_buffer(dev, kind, numel):
    """Persistent fp64 loss accumulators per device: zero when created, re-zeroed by the finalize kernel
    that consumes them (scd_centernet_loss_finalize), so the loss needs no memset launches."""
    key = (str(dev), kind, numel)
    buf = _ACC.get(key)
    if buf is None:
        buf = torch.zeros(numel, dtype=torch.float64, device=dev)
        _ACC[key] = buf
    return buf


def ctypes_float2(a, b):
    import ctypes
    arr = (ctypes.c_float * 2)(float(a), float(b))
    return ctypes.cast(arr, ctypes.c_void_p)
