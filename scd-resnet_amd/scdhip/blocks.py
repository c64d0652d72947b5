"""Block-granular autograd Functions of the CenterNet/CornerNet ResNet training path.

Each Function runs one reference module group entirely on libscdhip kernels:
  StemFn        preprocess: Conv2d(1,64,7,s2,p3)+BN+ReLU+MaxPool(3,2,1)   residuals.py:209-216
  BasicBlockFn  BasicBlock (+downsample)                                  residuals.py:84-120, 256-271
  BottleneckFn  Bottleneck (+downsample)                                  residuals.py:122-165
  DeconvBNFn    ConvTranspose2d(k4,s2,p1,no bias)+BN+ReLU                 residuals.py:286-310
  ConvBNFn      Convolution (conv+BN+ReLU) / conv+BN                      convolutions.py:25-49
  HeadsFn       all CenterNet terminals fused: one 3x3 GEMM with N = sum of
                hidden widths (+bias+ReLU epilogue) and the per-head 1x1s  centerNetOffset.py:103-122

Parameter gradients are accumulated straight into ``param.grad`` (created on demand;
with FlatAdam/FlatDDP they are views of one flat buffer), so the Functions return None
for parameter inputs.  Activations between Functions are NHWC in the model's compute dtype.
"""
import os

import torch

from . import ops
from .flat import grads_ready


def _c(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


# stem backward as one pass (ops.stem_backward_fused); SCD_STEM_FUSED_BWD=0: pool backward + fused-apply weight gradient
_STEM_FUSED_BWD = os.environ.get("SCD_STEM_FUSED_BWD", "1") != "0"


def _conv_ld(w):
    """dst strides of an OIHW conv weight (Co, Ci, kh, kw) for scd_wgrad_reduce: [co][ci][tap]."""
    T = w.shape[2] * w.shape[3]
    return (w.shape[1] * T, T, 1)


def _conv_stats(x, conv, bn, stride, pad, training, timer=None):
    """conv (no bias) -> raw y, with the BN statistics accumulated in the GEMM epilogue (training)."""
    C = conv.weight.shape[0]
    kh, kw = conv.weight.shape[2], conv.weight.shape[3]
    wp = ops.pack_weight(conv.weight, x.dtype, 0)
    stats = ops.bn_stats(bn, "fwd") if training else None
    t0 = ops.LaunchTimer.record(timer) if timer else None
    y = ops.conv_fwd(x, wp, C, kh, kw, stride, pad, stats=stats)
    if timer:
        ops.LaunchTimer.close(timer, t0)
    return y, stats


def _train_bn_conv(x, conv, bn, stride, pad, training, timer=None):
    """conv (no bias) -> raw y + BN statistics -> BNState.  timer: LaunchTimer name for the GEMM (bench.py)."""
    C = conv.weight.shape[0]
    y, stats = _conv_stats(x, conv, bn, stride, pad, training, timer)
    return y, ops.bn_finalize(bn, stats, C, y.numel() // C, training)


def _conv1_and_downsample(x, blk, conv1, bn1, s1, pad1, sd):
    """A block's first conv and its downsample conv (both read only the block input; residuals.py:99-120,
    145-165), then both BN finalizes together: with SyncBN one all-reduce for the two layers."""
    bnd = blk.downsample[1]
    C1, Cd = conv1.weight.shape[0], blk.downsample[0].weight.shape[0]
    y1, s1st = _conv_stats(x, conv1, bn1, s1, pad1, True)
    yd, sdst = _conv_stats(x, blk.downsample[0], bnd, sd, 0, True)
    st1, std = ops.bn_finalize_pair(bn1, s1st, C1, y1.numel() // C1, bnd, sdst, Cd, yd.numel() // Cd)
    return y1, st1, yd, std


def _dgrad_bn_relu_bwd(dy, wpack_t, C, Hc, Wc, kh, kw, stride, pad, bn, st, y):
    """Input gradient of a conv whose input is a BN+ReLU layer's output (bn, st, pre-BN y), then that layer's
    backward.  In bf16 the dgrad GEMM's epilogue accumulates the BN backward sums (scd_conv_gemm_bnbwd; shapes
    outside the ping-pong kernel run GEMM + reduce inside the same entry point), so the BN backward is only the
    finalize + apply."""
    if dy.dtype in ops.HALF and ops.BNFusion.enabled:
        stats = ops.bn_stats(bn, "bwdf")
        da = ops.conv_dgrad(dy, wpack_t, C, Hc, Wc, kh, kw, stride, pad, bn_bwd=(st, y, stats))
        return ops.bn_backward(bn, st, da, y, relu=True, stats=stats)
    da = ops.conv_dgrad(dy, wpack_t, C, Hc, Wc, kh, kw, stride, pad)
    return ops.bn_backward(bn, st, da, y, relu=True)


class StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, conv, bn, dtype):
        training = bn.training
        C = conv.weight.shape[0]
        stats = ops.bn_stats(bn, "fwd") if training else None
        ref_geom = tuple(conv.weight.shape) == (64, 1, 7, 7) and conv.stride[0] == 2 and conv.padding[0] == 3
        direct = ops.stem_direct_ok(x, dtype) and ref_geom
        if direct:
            # direct 7x7/s2 conv: the tap tile is built in LDS from the input patch (no column tensor)
            x = _c(x)
            wpk = ops.pack_weight(conv.weight, dtype, 0, ldp=64)
            y = ops.stem_conv_fwd(x, wpk, stats=stats)
            cols = x
        else:
            cols = ops.im2col_stem(x, dtype, kh=conv.weight.shape[2], kw=conv.weight.shape[3],
                                   stride=conv.stride[0], pad=conv.padding[0])
            wp = ops.pack_weight(conv.weight, dtype, 0, ldp=cols.shape[-1])
            y = ops.conv_fwd(cols, wp, C, 1, 1, 1, 0, stats=stats)
        st = ops.bn_finalize(bn, stats, C, y.numel() // C, training)
        out, am = ops.stem_pool_fwd(y, st)
        ctx.save_for_backward(cols, y, am)
        ctx.st, ctx.conv, ctx.bn, ctx.direct = st, conv, bn, direct
        ctx.wpk = wpk if direct else None
        return out

    @staticmethod
    def backward(ctx, dout):
        conv, bn, st = ctx.conv, ctx.bn, ctx.st
        cols, y, am = ctx.saved_tensors
        if ctx.direct and _STEM_FUSED_BWD:
            # pool / ReLU / BN / weight-gradient backward in one pass over the pooled gradient (dz stays on chip)
            ops.stem_backward_fused(bn, _c(dout), am, y, st, cols, ctx.wpk, ops.grad_of(conv.weight))
        elif ctx.direct:
            # pool/ReLU backward + BN reduction in one pass; the BN apply runs inside the weight gradient
            dz, coef = ops.stem_pool_bwd_bn(bn, _c(dout), am, y, st)
            ops.stem_conv_wgrad(dz, cols, ops.grad_of(conv.weight), ybn=y, coef=coef)
        else:
            dz = ops.stem_pool_bwd(_c(dout), am, y, st)
            dy = ops.bn_backward(bn, st, dz, y)
            T = conv.weight.shape[2] * conv.weight.shape[3]
            ops.conv_wgrad(dy, cols, 1, 1, 1, 0, ops.grad_of(conv.weight), (T, 1, 0), cvalid=T)
        grads_ready(conv, bn)
        return None, None, None, None, None


class BasicBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, blk):
        tr = blk.training
        s = blk.stride
        yd = std = None
        if tr and blk.downsample is not None:
            y1, st1, yd, std = _conv1_and_downsample(x, blk, blk.conv1, blk.bn1, s, 1, s)
        else:
            y1, st1 = _train_bn_conv(x, blk.conv1, blk.bn1, s, 1, tr)
        a1 = ops.bn_apply(y1, st1, True)
        y2, st2 = _train_bn_conv(a1, blk.conv2, blk.bn2, 1, 1, tr)
        if blk.downsample is not None:
            if yd is None:                      # eval: the downsample conv after the main branch
                yd, std = _train_bn_conv(x, blk.downsample[0], blk.downsample[1], s, 0, tr)
            out = ops.bn_apply(y2, st2, True, res=yd, rst=std)
        else:
            out = ops.bn_apply(y2, st2, True, res=x)
        ctx.save_for_backward(x, y1, a1, y2, yd, out)
        ctx.sts = (st1, st2, std)
        ctx.blk = blk
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y1, a1, y2, yd, out = ctx.saved_tensors
        st1, st2, std = ctx.sts
        blk = ctx.blk
        dout = _c(dout)
        s = blk.stride
        N, H, W, Cin = x.shape
        C = blk.conv1.weight.shape[0]
        dx = dyd = None
        w2 = blk.conv2.weight
        if blk.downsample is not None:
            dy2, dyd = ops.bn_backward_pair(blk.bn2, st2, y2, blk.downsample[1], std, yd, dout, out)
            wd = blk.downsample[0].weight
            gd, g2 = ops.grad_of(wd), ops.grad_of(w2)      # (before the ordering: may zero-fill on this stream)
            with ops.side_batch():          # both weight gradients behind one side-stream ordering
                ops.conv_wgrad(dyd, x, 1, 1, s, 0, gd, _conv_ld(wd))
                ops.conv_wgrad(dy2, a1, 3, 3, 1, 1, g2, _conv_ld(w2))
        else:
            dx = torch.empty_like(x)
            dy2 = ops.bn_backward(blk.bn2, st2, dout, y2, mask=out, dz_out=dx)
            ops.conv_wgrad(dy2, a1, 3, 3, 1, 1, ops.grad_of(w2), _conv_ld(w2))
        dy1 = _dgrad_bn_relu_bwd(dy2, ops.pack_weight(w2, x.dtype, 1), C, a1.shape[1], a1.shape[2], 3, 3, 1, 1,
                                 blk.bn1, st1, y1)
        w1 = blk.conv1.weight
        ops.conv_wgrad(dy1, x, 3, 3, s, 1, ops.grad_of(w1), _conv_ld(w1))
        dx = ops.conv_dgrad_w(dy1, w1, H, W, s, 1, out=dx, accumulate=dx is not None)
        if dyd is not None:
            # the downsample's input gradient last: += over the pixels its 1x1 taps reach only (one in four at stride 2)
            ops.conv_dgrad(dyd, ops.pack_weight(blk.downsample[0].weight, x.dtype, 1), Cin, H, W, 1, 1, s, 0, out=dx,
                           accumulate=True)
        grads_ready(blk)
        return dx, None, None


class BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, blk):
        tr = blk.training
        s = blk.stride
        yd = std = None
        if tr and blk.downsample is not None:
            y1, st1, yd, std = _conv1_and_downsample(x, blk, blk.conv1, blk.bn1, 1, 0, s)
        else:
            y1, st1 = _train_bn_conv(x, blk.conv1, blk.bn1, 1, 0, tr)
        a1 = ops.bn_apply(y1, st1, True)
        y2, st2 = _train_bn_conv(a1, blk.conv2, blk.bn2, s, 1, tr)
        a2 = ops.bn_apply(y2, st2, True)
        y3, st3 = _train_bn_conv(a2, blk.conv3, blk.bn3, 1, 0, tr)
        if blk.downsample is not None:
            if yd is None:                      # eval: the downsample conv after the main branch
                yd, std = _train_bn_conv(x, blk.downsample[0], blk.downsample[1], s, 0, tr)
            out = ops.bn_apply(y3, st3, True, res=yd, rst=std)
        else:
            out = ops.bn_apply(y3, st3, True, res=x)
        ctx.save_for_backward(x, y1, a1, y2, a2, y3, yd, out)
        ctx.sts = (st1, st2, st3, std)
        ctx.blk = blk
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y1, a1, y2, a2, y3, yd, out = ctx.saved_tensors
        st1, st2, st3, std = ctx.sts
        blk = ctx.blk
        dout = _c(dout)
        s = blk.stride
        N, H, W, Cin = x.shape
        P = blk.conv1.weight.shape[0]
        dx = dyd = None
        w3 = blk.conv3.weight
        if blk.downsample is not None:
            dy3, dyd = ops.bn_backward_pair(blk.bn3, st3, y3, blk.downsample[1], std, yd, dout, out)
            wd = blk.downsample[0].weight
            gd, g3 = ops.grad_of(wd), ops.grad_of(w3)      # (before the ordering: may zero-fill on this stream)
            with ops.side_batch():          # both weight gradients behind one side-stream ordering
                ops.conv_wgrad(dyd, x, 1, 1, s, 0, gd, _conv_ld(wd))
                ops.conv_wgrad(dy3, a2, 1, 1, 1, 0, g3, _conv_ld(w3))
        else:
            dx = torch.empty_like(x)
            dy3 = ops.bn_backward(blk.bn3, st3, dout, y3, mask=out, dz_out=dx)
            ops.conv_wgrad(dy3, a2, 1, 1, 1, 0, ops.grad_of(w3), _conv_ld(w3))
        dy2 = _dgrad_bn_relu_bwd(dy3, ops.pack_weight(w3, x.dtype, 1), P, a2.shape[1], a2.shape[2], 1, 1, 1, 0,
                                 blk.bn2, st2, y2)
        w2 = blk.conv2.weight
        ops.conv_wgrad(dy2, a1, 3, 3, s, 1, ops.grad_of(w2), _conv_ld(w2))
        dy1 = _dgrad_bn_relu_bwd(dy2, ops.pack_weight(w2, x.dtype, 1), P, a1.shape[1], a1.shape[2], 3, 3, s, 1,
                                 blk.bn1, st1, y1)
        w1 = blk.conv1.weight
        ops.conv_wgrad(dy1, x, 1, 1, 1, 0, ops.grad_of(w1), _conv_ld(w1))
        dx = ops.conv_dgrad(dy1, ops.pack_weight(w1, x.dtype, 1), Cin, H, W, 1, 1, 1, 0, out=dx,
                            accumulate=dx is not None)
        if dyd is not None:
            ops.conv_dgrad(dyd, ops.pack_weight(blk.downsample[0].weight, x.dtype, 1), Cin, H, W, 1, 1, s, 0, out=dx,
                           accumulate=True)
        grads_ready(blk)
        return dx, None, None


class DeconvBNFn(torch.autograd.Function):
    """ConvTranspose2d(k, s=2, p, op=0, bias=False) -> BN -> ReLU.  The deconv forward is the
    input-gradient of the Conv2d whose weight is W_t (4 sub-pixel phases of 2x2 taps each)."""

    @staticmethod
    def forward(ctx, x, w, deconv, bn):
        k = w.shape[2]
        s, p = deconv.stride[0], deconv.padding[0]
        Cout = w.shape[1]
        stats = ops.bn_stats(bn, "fwd") if bn.training else None
        y = ops.deconv_fwd(x, ops.pack_weight(w, x.dtype, 1), Cout, k, s, p, stats=stats)
        st = ops.bn_finalize(bn, stats, Cout, y.numel() // Cout, bn.training)
        out = ops.bn_apply(y, st, True)
        ctx.save_for_backward(x, y, out)
        ctx.st, ctx.deconv, ctx.bn = st, deconv, bn
        ctx.prod = ops.bn_producer(x)           # a BN+ReLU layer before this one: its sums come from our dgrad
        ops.set_bn_producer(out, bn, st, y)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y, out = ctx.saved_tensors
        deconv, bn, st = ctx.deconv, ctx.bn, ctx.st
        w = deconv.weight
        k = w.shape[2]
        s, p = deconv.stride[0], deconv.padding[0]
        dout = _c(dout)
        dy = ops.bn_backward(bn, st, dout, y, relu=True, stats=ops.take_bn_bwd_fused(bn, dout))
        # dW_t[i][o][r][s] = sum x[i at q] * dy[o at s*q + r - p]: weight-gradient GEMM with G = x
        T = k * k
        ops.conv_wgrad(x, dy, k, k, s, p, ops.grad_of(w), (w.shape[1] * T, T, 1))
        fuse = ctx.prod is not None and x.dtype in ops.HALF
        dx = ops.deconv_dgrad(dy, ops.pack_weight(w, x.dtype, 0), w.shape[0], k, s, p,
                              bn_bwd=ops.fused_bn_bwd_args(ctx.prod) if fuse else None)
        if fuse:
            ops.mark_bn_bwd_fused(ctx.prod[0], dx)
        grads_ready(deconv, bn)
        return dx, None, None, None


class ConvBNFn(torch.autograd.Function):
    """Conv2d(no bias, 'same' padding) -> BN -> [ReLU] (Convolution, convolutions.py:25-49)."""

    @staticmethod
    def forward(ctx, x, w, conv, bn, relu):
        s, p = conv.stride[0], conv.padding[0]
        y, st = _train_bn_conv(x, conv, bn, s, p, bn.training)
        out = ops.bn_apply(y, st, relu)
        ctx.save_for_backward(x, y, out)
        ctx.st, ctx.conv, ctx.bn, ctx.relu = st, conv, bn, relu
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y, out = ctx.saved_tensors
        conv, bn, st = ctx.conv, ctx.bn, ctx.st
        w = conv.weight
        kh, kw = w.shape[2], w.shape[3]
        s, p = conv.stride[0], conv.padding[0]
        dy = ops.bn_backward(bn, st, _c(dout), y, relu=ctx.relu)
        ops.conv_wgrad(dy, x, kh, kw, s, p, ops.grad_of(w), _conv_ld(w))
        dx = ops.conv_dgrad(dy, ops.pack_weight(w, x.dtype, 1), x.shape[3], x.shape[1], x.shape[2], kh, kw, s, p)
        grads_ready(conv, bn)
        return dx, None, None, None, None


class HeadsFn(torch.autograd.Function):
    """All CenterNet terminals (Conv2d 3x3 +bias -> ReLU -> Conv2d 1x1 +bias) fused:
    hidden = relu(conv3x3(feat, W0cat) + b0cat) with N = sum of hidden widths, then the
    block-diagonal 1x1 tails.  Outputs are NCHW fp32, one tensor per head."""

    @staticmethod
    def forward(ctx, feat, w0_first, heads):
        N, H, W, Cin = feat.shape
        w0s = [h[0].weight for h in heads]
        b0 = torch.cat([h[0].bias for h in heads], 0)
        Hd = heads[0][0].weight.shape[0]
        Ct = sum(w.shape[0] for w in w0s)
        od = [h[2].weight.shape[0] for h in heads]
        outs = [torch.empty(N, o, H, W, device=feat.device, dtype=torch.float32) for o in od]
        wp = ops.pack_concat(w0s, feat.dtype, 0)
        w1s = ops.L.ptr_array([h[2].weight.data_ptr() for h in heads])
        b1s = ops.L.ptr_array([h[2].bias.data_ptr() for h in heads])
        optrs = ops.L.ptr_array([o.data_ptr() for o in outs])
        odarr = ops.L.int_array(od)
        hint = ops.take_sparse_hint()
        ctx.keep = None
        if Hd == 128 and len(heads) <= 4 and max(od) <= 4:
            # tails fused into the GEMM epilogue (one launch, hidden tensor read once)
            hid = torch.empty(N, H, W, Ct, device=feat.device, dtype=feat.dtype)
            keep = None
            if (hint is not None and len(heads) >= 2 and Cin <= 256 and (len(heads) - 1) * Hd <= 256
                    and hint.dim() == 2 and hint.shape[0] == N):
                # the loss gathers the size / offset outputs at `hint` only: their hidden channels are stored there
                keep = ops.heads_keep_map(hint, N, H * W)
                ctx.keep = (hint, hint._version)
            args = (ops.dt(feat), ops.ptr(feat), ops.ptr(wp), ops.ptr(hid), ops.ptr(b0), N, H, W, Cin, len(heads),
                    odarr, w1s, b1s)
            t0 = ops.LaunchTimer.record("heads_gemm")
            ops.L.call("scd_conv_gemm_heads_keep", *args, optrs, ops.ptr(keep) if keep is not None else None, Hd,
                       ops.stream())
            ops.LaunchTimer.close("heads_gemm", t0)
            if keep is not None:
                # everything needed to store the whole hidden tensor again (a dense backward after all)
                scratch = [torch.empty_like(o) for o in outs]
                ctx.refill = (args, ops.L.ptr_array([o.data_ptr() for o in scratch]), wp, b0, scratch)
        else:
            hid = ops.conv_fwd(feat, wp, Ct, 3, 3, 1, 1, bias=b0, relu=True)
            ops.L.call("scd_heads_fwd", ops.dt(hid), ops.ptr(hid), N, H * W, len(heads), Hd, odarr, w1s, b1s, optrs,
                       ops.stream())
        ctx.save_for_backward(feat, hid)
        ctx.w0s = w0s
        ctx.heads, ctx.od, ctx.Hd = heads, od, Hd
        ctx.prod = ops.bn_producer(feat)        # the deconv BN+ReLU: its backward sums come from our dgrad
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        feat, hid = ctx.saved_tensors
        w0s = ctx.w0s
        heads, od, Hd = ctx.heads, ctx.od, ctx.Hd
        N, H, W, Cin = feat.shape
        nh = len(heads)
        douts = [(_c(d) if d is not None else torch.zeros(N, o, H, W, device=feat.device))
                 for d, o in zip(douts, od)]
        # fp16: the backward below runs on loss-scaled gradients (ops.LossScale: the repack multiplies the head
        # gradients by S), unscaled into every .grad
        S = ops.begin_loss_scale(feat.dtype)
        dptrs = ops.L.ptr_array([d.data_ptr() for d in douts])
        odarr = ops.L.int_array(od)
        nd = HeadsFn._dense_prefix(douts, Hd, Cin)
        if ctx.keep is not None:
            inds = ops.sparse_grad_inds(douts[-1]) if nd == 1 else None
            if inds is None or inds is not ctx.keep[0] or inds._version != ctx.keep[1]:
                # the forward kept the size / offset hidden channels at other pixels only: store them all
                args, optrs, _, _, _ = ctx.refill
                ops.L.call("scd_conv_gemm_heads_keep", *args, optrs, None, 0, ops.stream())
            ctx.refill = None
        if nd < nh:
            return HeadsFn._backward_sparse(ctx, douts, dptrs, odarr, nd, S)
        dhid = torch.empty_like(hid)
        acc = ops.persistent_zeros(heads[0][2].weight, "_scd_heads_acc",
                                   ops.L.lib().scd_heads_bwd_accsize(nh, Hd, odarr) // 8, torch.float64)
        packed = torch.empty(N * H * W * nh * 4, device=feat.device)
        ops.L.call("scd_heads_bwd_packed", ops.dt(hid), ops.ptr(hid), N, H * W, nh, Hd, odarr,
                   ops.L.ptr_array([h[2].weight.data_ptr() for h in heads]), dptrs, float(S), ops.ptr(packed),
                   ops.ptr(dhid), ops.ptr(acc), ops.stream())
        ops.L.call("scd_heads_bwd_weight_finalize", ops.ptr(acc), nh, Hd, odarr,
                   ops.L.ptr_array([ops.grad_of(h[2].weight).data_ptr() for h in heads]),
                   ops.L.ptr_array([ops.grad_of(h[2].bias).data_ptr() for h in heads]),
                   ops.L.ptr_array([ops.grad_of(h[0].bias).data_ptr() for h in heads]), 1, 1.0 / S, ops.stream())
        ld = (Cin * 9, 9, 1)
        rows = [(i * Hd, (i + 1) * Hd, ops.grad_of(h[0].weight), ld) for i, h in enumerate(heads)]
        ops.conv_wgrad(dhid, feat, 3, 3, 1, 1, None, None, rows=rows)
        slot = ops.shared_grad_slot(feat)
        if slot is not None:
            # feat's gradient is shared with other consumers (ops.share_grad): write into / start the one buffer
            # (no BN-backward sums from this epilogue: they would cover this consumer's part only)
            dfeat = ops.conv_dgrad(dhid, ops.pack_concat(w0s, feat.dtype, 1), Cin, H, W, 3, 3, 1, 1, out=slot[1],
                                   accumulate=slot[1] is not None)
            grads_ready(*[m for h in heads for m in h if isinstance(m, torch.nn.Module)])
            return ops.shared_grad_out(feat, slot, dfeat if slot[1] is None else None), None, None
        fuse = ctx.prod is not None and feat.dtype in ops.HALF
        dfeat = ops.conv_dgrad(dhid, ops.pack_concat(w0s, feat.dtype, 1), Cin, H, W, 3, 3, 1, 1,
                               bn_bwd=ops.fused_bn_bwd_args(ctx.prod) if fuse else None)
        if fuse:
            ops.mark_bn_bwd_fused(ctx.prod[0], dfeat)
        grads_ready(*[m for h in heads for m in h if isinstance(m, torch.nn.Module)])
        return dfeat, None, None

    @staticmethod
    def _dense_prefix(douts, Hd, Cin):
        """Number of leading heads that need the dense backward: the rest must carry the loss's sparse-support
        certificate (one index tensor for all of them; ops.certify_sparse_grad)."""
        nh = len(douts)
        if nh < 2 or Cin > 256:
            return nh
        certs = [ops.sparse_grad_inds(d) for d in douts]
        nd = nh
        while nd > 1 and certs[nd - 1] is not None and certs[nd - 1] is certs[-1]:
            nd -= 1
        return nd if (nh - nd) * Hd <= 256 else nh

    @staticmethod
    def _backward_sparse(ctx, douts, dptrs, odarr, nd, S):
        """Heads [0, nd): the dense tail backward and 3x3 GEMMs over their nd*Hd hidden channels.  Heads [nd, nh):
        their output gradient lives on the certified pixels inds[b][k] only, so the tail backward, the 3x3 weight
        gradient (a GEMM over those pixels' im2col rows) and the 3x3 input gradient (a small GEMM then a gather
        into the dense input gradient) run over that pixel set (scd_heads_sparse_bwd / scd_heads_sparse_fixup)."""
        feat, hid = ctx.saved_tensors
        w0s, heads, od, Hd = ctx.w0s, ctx.heads, ctx.od, ctx.Hd
        N, H, W, Cin = feat.shape
        nh = len(heads)
        dev, dt = feat.device, feat.dtype
        inds = ops.sparse_grad_inds(douts[-1])
        K = inds.shape[1]
        Sl = N * K                                     # slots
        Cs = (nh - nd) * Hd
        w1s = ops.L.ptr_array([h[2].weight.data_ptr() for h in heads])
        acc = ops.persistent_zeros(heads[0][2].weight, "_scd_heads_acc",
                                   ops.L.lib().scd_heads_bwd_accsize(nh, Hd, odarr) // 8, torch.float64)
        dh_dense = torch.empty(N, H, W, nd * Hd, device=dev, dtype=dt)
        packed = torch.empty(N * H * W * nd * 4, device=dev)
        ops.L.call("scd_heads_bwd_packed_split", ops.dt(hid), ops.ptr(hid), N, H * W, nh, Hd, odarr, nd, w1s, dptrs,
                   float(S), ops.ptr(packed), ops.ptr(dh_dense), ops.ptr(acc), ops.stream())
        dhid_s = torch.empty(Sl, Cs, device=dev, dtype=dt)
        xcol = torch.empty(Sl, Cin * 9, device=dev, dtype=dt)
        slotmap, ownermap = ops.sparse_maps(dev, N * H * W)
        ops.L.call("scd_heads_sparse_bwd", ops.dt(hid), ops.ptr(hid), ops.ptr(feat), N, H, W, Cin, nh, Hd, odarr, nd,
                   w1s, dptrs, float(S), ops.ptr(inds), K, ops.ptr(dhid_s), ops.ptr(xcol), ops.ptr(acc),
                   ops.ptr(slotmap), ops.ptr(ownermap), ops.stream())
        ops.L.call("scd_heads_bwd_weight_finalize", ops.ptr(acc), nh, Hd, odarr,
                   ops.L.ptr_array([ops.grad_of(h[2].weight).data_ptr() for h in heads]),
                   ops.L.ptr_array([ops.grad_of(h[2].bias).data_ptr() for h in heads]),
                   ops.L.ptr_array([ops.grad_of(h[0].bias).data_ptr() for h in heads]), 1, 1.0 / S, ops.stream())
        # weight gradients: dense heads over every pixel, sparse heads over the slots' im2col rows (a 1x1 GEMM whose
        # Cin*9 columns are the OIHW rows of their 3x3 weights)
        ld = (Cin * 9, 9, 1)

        def wgrads():
            # (the gradient views first -- they may zero-fill on this stream -- then both GEMMs behind one
            # side-stream ordering)
            rd = [(i * Hd, (i + 1) * Hd, ops.grad_of(heads[i][0].weight), ld) for i in range(nd)]
            rs = [((i - nd) * Hd, (i - nd + 1) * Hd, ops.grad_of(heads[i][0].weight), ld) for i in range(nd, nh)]
            with ops.side_batch():
                ops.conv_wgrad(dh_dense, feat, 3, 3, 1, 1, None, None, rows=rd)
                # (a 1x1 GEMM over the slots; its 9*Cin columns are reduced as 9 taps x Cin into the OIHW rows)
                ops.conv_wgrad(dhid_s.view(1, 1, Sl, Cs), xcol.view(1, 1, Sl, 9 * Cin), 1, 1, 1, 0, None, None,
                               rows=rs, red_taps=9)
        # input gradient: dense heads' GEMM (+ the deconv BN's backward sums), then the sparse heads' part
        fuse = ctx.prod is not None and dt in ops.HALF
        bn_args = ops.fused_bn_bwd_args(ctx.prod) if fuse else None
        dfeat = ops.conv_dgrad(dh_dense, ops.pack_concat(w0s[:nd], dt, 1), Cin, H, W, 3, 3, 1, 1, bn_bwd=bn_args)
        wt_s = ops.pack_concat(w0s[nd:], dt, 2)          # [tap][ci][c] rows: W0^T of the sparse heads, tap-major
        cols = ops.conv_fwd(dhid_s.view(1, 1, Sl, Cs), wt_s, 9 * Cin, 1, 1, 1, 0)
        if fuse:
            st, ybn, bstats = bn_args
            bn_ptrs = (ops.ptr(ybn), ops.ptr(st.mean), ops.ptr(st.invstd), ops.ptr(st.scale), ops.ptr(st.shift),
                       ops.ptr(bstats))
        else:
            bn_ptrs = (None,) * 6
        ops.L.call("scd_heads_sparse_fixup", ops.dt(dfeat), ops.ptr(dfeat), ops.ptr(cols), N, H, W, Cin, ops.ptr(inds),
                   K, ops.ptr(slotmap), ops.ptr(ownermap), *bn_ptrs, ops.stream())
        mods = [m for h in heads for m in h if isinstance(m, torch.nn.Module)]
        if fuse:
            ops.mark_bn_bwd_fused(ctx.prod[0], dfeat)
        wgrads()                 # side stream ordered after the input gradient: it overlaps the deconv backward
        grads_ready(*mods)
        return dfeat, None, None


class CornerPoolFn(torch.autograd.Function):
    """CornerPool module (cornerNetCPool.py:83-122) on NHWC activations:
    a_i = relu(bn(conv3x3(x)))  (branch1/2, Convolution);  s = pool1(a1) + pool2(a2)
    r = relu(bn(conv3x3(s)) + bn(conv1x1(x)));  out = relu(bn(conv3x3(r)))  (lastConv)."""

    @staticmethod
    def forward(ctx, x, w_anchor, mod, dirs):
        tr = mod.branchMergeBn.training
        b1, b2, lc = mod.branch1, mod.branch2, mod.lastConv
        if tr:
            # both branch convs read x: their BN finalizes together (one SyncBN all-reduce for the two)
            y1, s1 = _conv_stats(x, b1.conv, b1.bn, 1, 1, tr)
            y2, s2 = _conv_stats(x, b2.conv, b2.bn, 1, 1, tr)
            C1, C2 = b1.conv.weight.shape[0], b2.conv.weight.shape[0]
            st1, st2 = ops.bn_finalize_pair(b1.bn, s1, C1, y1.numel() // C1, b2.bn, s2, C2, y2.numel() // C2)
        else:
            y1, st1 = _train_bn_conv(x, b1.conv, b1.bn, 1, 1, tr)
            y2, st2 = _train_bn_conv(x, b2.conv, b2.bn, 1, 1, tr)
        a1 = ops.bn_apply(y1, st1, True)
        a2 = ops.bn_apply(y2, st2, True)
        p1 = ops.cpool_fwd(a1, dirs[0])
        t0 = ops.LaunchTimer.record("cpool_fwd_add")
        s = ops.cpool_fwd(a2, dirs[1], addend=p1)
        ops.LaunchTimer.close("cpool_fwd_add", t0)
        del p1
        if tr:
            ym, sm = _conv_stats(s, mod.branchMerge, mod.branchMergeBn, 1, 1, tr)
            ysc, ss = _conv_stats(x, mod.shortcutConv, mod.shortcutBn, 1, 0, tr)
            Cm, Cs = mod.branchMerge.weight.shape[0], mod.shortcutConv.weight.shape[0]
            stm, sts = ops.bn_finalize_pair(mod.branchMergeBn, sm, Cm, ym.numel() // Cm, mod.shortcutBn, ss, Cs,
                                            ysc.numel() // Cs)
        else:
            ym, stm = _train_bn_conv(s, mod.branchMerge, mod.branchMergeBn, 1, 1, tr)
            ysc, sts = _train_bn_conv(x, mod.shortcutConv, mod.shortcutBn, 1, 0, tr)
        r = ops.bn_apply(ym, stm, True, res=ysc, rst=sts)
        yl, stl = _train_bn_conv(r, lc.conv, lc.bn, 1, 1, tr, timer="cpool_lastconv")
        out = ops.bn_apply(yl, stl, True)
        ctx.save_for_backward(x, y1, a1, y2, a2, s, ym, ysc, r, yl, out)
        ctx.sts = (st1, st2, stm, sts, stl)
        ctx.mod, ctx.dirs = mod, dirs
        return out

    @staticmethod
    def backward(ctx, dout):
        x, y1, a1, y2, a2, s, ym, ysc, r, yl, out = ctx.saved_tensors
        st1, st2, stm, sts, stl = ctx.sts
        mod, dirs = ctx.mod, ctx.dirs
        N, H, W, C = x.shape
        lc = mod.lastConv
        dyl = ops.bn_backward(lc.bn, stl, _c(dout), yl, relu=True)
        ops.conv_wgrad(dyl, r, 3, 3, 1, 1, ops.grad_of(lc.conv.weight), _conv_ld(lc.conv.weight))
        dr = ops.conv_dgrad(dyl, ops.pack_weight(lc.conv.weight, x.dtype, 1), C, H, W, 3, 3, 1, 1)
        dym, dys = ops.bn_backward_pair(mod.branchMergeBn, stm, ym, mod.shortcutBn, sts, ysc, dr, r)
        wsc = mod.shortcutConv.weight
        ops.conv_wgrad(dys, x, 1, 1, 1, 0, ops.grad_of(wsc), _conv_ld(wsc))
        slot = ops.shared_grad_slot(x)          # x's gradient shared with the other heads (ops.share_grad)
        prev = slot[1] if slot is not None else None
        dx = ops.conv_dgrad(dys, ops.pack_weight(wsc, x.dtype, 1), C, H, W, 1, 1, 1, 0, out=prev,
                            accumulate=prev is not None)
        wm = mod.branchMerge.weight
        ops.conv_wgrad(dym, s, 3, 3, 1, 1, ops.grad_of(wm), _conv_ld(wm))
        Cb = wm.shape[1]
        ds = ops.conv_dgrad(dym, ops.pack_weight(wm, x.dtype, 1), Cb, H, W, 3, 3, 1, 1)
        for (a, y, st, br), d in zip(((a1, y1, st1, mod.branch1), (a2, y2, st2, mod.branch2)), dirs):
            da = ops.cpool_bwd(a, ds, d)
            dy = ops.bn_backward(br.bn, st, da, y, relu=True)
            ops.conv_wgrad(dy, x, 3, 3, 1, 1, ops.grad_of(br.conv.weight), _conv_ld(br.conv.weight))
            ops.conv_dgrad(dy, ops.pack_weight(br.conv.weight, x.dtype, 1), C, H, W, 3, 3, 1, 1, out=dx,
                           accumulate=True)
        grads_ready(mod)
        if slot is not None:
            return ops.shared_grad_out(x, slot, dx if prev is None else None), None, None, None
        return dx, None, None, None


class CPoolFn(torch.autograd.Function):
    """Directional corner pool (TopPoolFunction etc., cornerPooling/__init__.py:8-58) on NHWC."""

    @staticmethod
    def forward(ctx, x, direction):
        ctx.save_for_backward(x)
        ctx.direction = direction
        return ops.cpool_fwd(x, direction)


    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return ops.cpool_bwd(x, _c(dy), ctx.direction), None


class NCHWToNHWC(torch.autograd.Function):
    """Layout boundary for callers that hand NCHW activations to a block (tests, custom heads)."""

    @staticmethod
    def forward(ctx, x, dtype):
        ctx.dtype_in = x.dtype
        return x.permute(0, 2, 3, 1).to(dtype).contiguous()

    @staticmethod
    def backward(ctx, g):
        return g.permute(0, 3, 1, 2).to(ctx.dtype_in).contiguous(), None
