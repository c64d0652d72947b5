"""Sparse-support backward of the CenterNet size / offset heads (scd_heads_sparse_bwd / scd_heads_sparse_fixup).

CenterNetLoss reaches the regression and offset outputs only through L1LossMask(gather(out, inds), ...)
(centerNetOffset.py:199-214, regression.py:37-44), so their output gradients vanish outside the gathered pixels.
The HIP backward then runs those heads' tail, 3x3 weight gradient and 3x3 input gradient over that pixel set.
These tests run one training-mode forward + loss + backward twice on the same inputs, with the sparse path and
with the dense path (SCD_SPARSE_HEADS off), and compare every parameter gradient:
  fp32 parity mode: 1e-5 relative to each gradient's scale (the two paths only sum in a different order);
  bf16: 2e-2 relative (the sparse input-gradient part is rounded to bf16 once more before it is added).
Targets include repeated indices, masked-out slots (index 0), and objects on the image border."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _targets(B, Hh, K, dev, seed):
    g = torch.Generator().manual_seed(seed)
    heat = (torch.rand(B, 1, Hh, Hh, generator=g) > 0.995).float()
    mask = torch.arange(K)[None, :] < torch.randint(K // 3, K, (B, 1), generator=g)
    regr = torch.rand(B, K, 6, generator=g) * 4
    inds = torch.randint(0, Hh * Hh, (B, K), generator=g)
    inds[:, 1] = inds[:, 0]                              # a pixel named twice
    inds[:, 2] = 0                                       # image corner
    inds[:, 3] = Hh * Hh - 1
    inds[:, 4] = Hh - 1                                  # right border, top row
    inds[:, 5] = inds[:, 4] + Hh                         # its neighbour below: overlapping 3x3 reach
    inds = inds * mask                                   # masked slots point at pixel 0, as the dataset does
    heat.view(B, -1).scatter_(1, inds[:, :3], 1.0)
    return [heat.to(dev), mask.to(dev), regr.to(dev), inds.to(dev)]


def _grads(model, lossfn, x, ys, sparse, hint=None):
    from scdhip import ops
    prev = ops.SparseHeads.enabled
    ops.SparseHeads.enabled = sparse
    try:
        model.zero_grad(set_to_none=False)
        if hint is not None:
            lossfn.prepare(hint)
        loss, _ = lossfn(model(x, decode=False), ys)
        loss.mean().backward()
        torch.cuda.synchronize()
    finally:
        ops.SparseHeads.enabled = prev
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}, loss.item()


def _setup(dtype, B, S):
    import importlib
    plugin = importlib.import_module("trainer.model.centerOffsetRes10")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = plugin.model(**plugin.modelParams).to(dev).set_compute_dtype(dtype).train()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, 1, S, S, generator=g).to(dev)
    ys = _targets(B, S // 4, 30, dev, 11)
    return plugin, model, x, ys


def _rel(a, b):
    a, b = a.float(), b.float()
    return (a - b).abs().max().item() / max(1e-12, b.abs().max().item())


def test_sparse_heads_match_dense_fp32():
    plugin, model, x, ys = _setup(torch.float32, 2, 128)
    # BN running statistics move on every training forward: restore them between the two runs
    state = {k: v.clone() for k, v in model.state_dict().items()}
    gs, ls = _grads(model, plugin.loss, x, ys, True)
    model.load_state_dict(state)
    gd, ld = _grads(model, plugin.loss, x, ys, False)
    assert abs(ls - ld) <= 1e-6 * max(1.0, abs(ld))
    assert gs.keys() == gd.keys()
    worst = max((_rel(gs[n], gd[n]), n) for n in gd)
    print("fp32: worst relative gradient difference sparse vs dense %.2e (%s)" % worst)
    assert worst[0] < 1e-5, worst


@pytest.mark.parametrize("B,S", [(4, 256), (32, 512)])
def test_sparse_heads_bf16_error_as_dense(B, S):
    """bf16: the sparse path's gradients are as close to the fp32 gradients of the same weights and inputs as the
    dense bf16 path's are (per parameter: e_sparse <= 1.5 e_dense + 2e-3, e = max-abs difference relative to the
    fp32 gradient's scale); the two bf16 paths round differently, and a deep layer's small summed gradient
    (e.g. the stem BN bias) carries the whole backward chain's rounding."""
    plugin, model, x, ys = _setup(torch.bfloat16, B, S)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    gs, _ = _grads(model, plugin.loss, x, ys, True)
    model.load_state_dict(state)
    gd, _ = _grads(model, plugin.loss, x, ys, False)
    model.load_state_dict(state)
    model.set_compute_dtype(torch.float32)
    gf, _ = _grads(model, plugin.loss, x, ys, False)
    rows = []
    for n in gf:
        assert torch.isfinite(gs[n]).all(), n
        es, ed = _rel(gs[n], gf[n]), _rel(gd[n], gf[n])
        rows.append((es - 1.5 * ed, es, ed, n))
    rows.sort(reverse=True)
    for r in rows[:5]:
        print("sparse %.3e dense %.3e  %s" % r[1:])
    for _, es, ed, n in rows:
        assert es <= 1.5 * ed + 2e-3, (n, es, ed)


def test_sparse_path_taken_and_maps_restored():
    """The certificate reaches HeadsFn (the dense tail is launched for the heatmap head only) and both pixel maps
    are back at their idle values after the backward."""
    import importlib
    from scdhip import ops
    plugin = importlib.import_module("trainer.model.centerOffsetRes10")
    dev = torch.device("cuda")
    model = plugin.model(**plugin.modelParams).to(dev).set_compute_dtype(torch.bfloat16).train()
    x = torch.randn(2, 1, 128, 128, device=dev)
    ys = _targets(2, 32, 30, dev, 3)
    from scdhip import blocks
    taken = []
    orig = blocks.HeadsFn._backward_sparse

    def spy(*a, **k):
        taken.append(a[4])
        return orig(*a, **k)
    blocks.HeadsFn._backward_sparse = staticmethod(spy)
    try:
        _grads(model, plugin.loss, x, ys, True)
    finally:
        blocks.HeadsFn._backward_sparse = staticmethod(orig)
    assert taken == [1]
    slotmap, ownermap = ops.sparse_maps(dev, 2 * 32 * 32)
    assert (slotmap == -1).all() and (ownermap == 0x7fffffff).all()


@pytest.mark.parametrize("B,S", [(4, 256), (8, 512)])
def test_heads_keep_map_gradients_identical(B, S):
    """CenterNetLoss.prepare before the forward: the heads GEMM stores the size / offset hidden channels only at the
    gathered pixels (scd_conv_gemm_heads_keep) and the sparse backward reads nothing else, so loss and every
    gradient are bit-identical to the run without the hint; the keep map names exactly the gathered pixels."""
    from scdhip import ops
    plugin, model, x, ys = _setup(torch.bfloat16, B, S)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    ga, la = _grads(model, plugin.loss, x, ys, True)
    model.load_state_dict(state)
    gb, lb = _grads(model, plugin.loss, x, ys, True, hint=ys)
    assert la == lb
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n
    HW = (S // 4) ** 2
    keep = ops._KEEP_MAPS[(str(x.device), B * HW, ys[3].shape[1])][0].view(B, HW)
    ref = torch.zeros(B, HW, dtype=torch.uint8, device=x.device).scatter_(1, ys[3], 1)
    assert torch.equal(keep, ref)


def test_heads_keep_map_fallbacks():
    """A hint that does not match the backward's gradients makes HeadsFn store the whole hidden tensor again:
    (1) the loss gathers at other indices than the hinted ones, (2) a loss without the sparse certificate (dense
    backward).  Gradients equal the runs without any hint."""
    plugin, model, x, ys = _setup(torch.bfloat16, 4, 256)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    other = list(ys)
    other[3] = (torch.flip(ys[3], (1,)) + 1) % (64 * 64)
    ga, _ = _grads(model, plugin.loss, x, other, True)
    model.load_state_dict(state)
    gb, _ = _grads(model, plugin.loss, x, other, True, hint=ys)
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n

    def dense_loss(outs, ys_):
        o = outs[0]
        return (o["heatmap"].float().square().mean() + o["regr"].float().square().mean()
                + o["offset"].float().square().mean()).reshape(1), None
    dense_loss.prepare = plugin.loss.prepare
    model.load_state_dict(state)
    gc, _ = _grads(model, dense_loss, x, ys, True)
    model.load_state_dict(state)
    gd, _ = _grads(model, dense_loss, x, ys, True, hint=ys)
    for n in gc:
        assert torch.equal(gc[n], gd[n]), n
