"""The reference's functional helpers on libscdhip (scdhip/api.py, csrc/api.hip) against the oracle's
restatements of utility.py / focal.py / regression.py (oracle/centernet.py), which tests/test_oracle_golden.py
pins to the reference's own outputs.

NMS and top-K are exact (values, indices, categories, coordinates bit-for-bit wherever the top-K order is strict;
torch.topk leaves tie order open, the HIP kernel takes the lowest index); the losses are fp32 reductions in a
different order: loss 1e-5 relative, gradients 1e-5 relative to their max.  Edge cases from the reference's
branches: no positive in the focal map (the -negL branch), an all-zero mask (the 1e-4 normaliser), ties in the
top-K, negative scores, multi-channel maps (categories) and several focal predictions (CornerNet's list form)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import centernet as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / max(1e-30, b.abs().max().item())


@pytest.mark.parametrize("shape,k", [((2, 1, 128, 128), 3), ((3, 2, 37, 45), 3), ((1, 1, 9, 11), 5)])
def test_nms_matches_reference(shape, k):
    from models.backbones.utility import nonMaximumSuppression
    g = torch.Generator().manual_seed(3)
    heat = torch.rand(shape, generator=g)
    heat[..., 4, 4] = heat[..., 4, 5]            # plateaus: both positions survive (== max)
    got = nonMaximumSuppression(heat.to(DEV), k).cpu()
    assert torch.equal(got, O.nms(heat, k))


@pytest.mark.parametrize("shape,K", [((2, 1, 128, 128), 100), ((3, 4, 20, 30), 50), ((2, 1, 16, 16), 256)])
def test_extract_topk_matches_reference(shape, K):
    from models.backbones.utility import extractTopK
    g = torch.Generator().manual_seed(5)
    s = torch.randn(shape, generator=g)                      # negative scores too
    s.view(shape[0], -1)[:, 10:20] = 0.75                    # a block of ties
    got = [t.cpu() for t in extractTopK(s.to(DEV), K)]
    B, C, H, W = shape
    rs, ri = torch.topk(s.view(B, -1), K)
    np.testing.assert_array_equal(got[0].numpy(), rs.numpy())   # the sorted values are unique whatever the ties
    for b in range(B):
        vals = rs[b].numpy()
        strict = np.ones(K, dtype=bool)
        gap = np.diff(vals) != 0
        strict[1:] &= gap
        strict[:-1] &= gap
        idx = ri[b].numpy()
        np.testing.assert_array_equal(got[1][b].numpy()[strict], (idx % (H * W))[strict])
        np.testing.assert_array_equal(got[2][b].numpy()[strict], (idx // (H * W))[strict])
        np.testing.assert_array_equal(got[3][b].numpy()[strict], ((idx % (H * W)) // W)[strict].astype(np.float32))
        np.testing.assert_array_equal(got[4][b].numpy()[strict], ((idx % (H * W)) % W)[strict].astype(np.float32))
        # tied runs: the HIP kernel lists the lowest flat indices, ascending
        for v in np.unique(vals[~strict]):
            sel = vals == v
            full = np.nonzero(s[b].view(-1).numpy() == v)[0]
            flat = got[2][b].numpy()[sel].astype(np.int64) * H * W + got[1][b].numpy()[sel]
            np.testing.assert_array_equal(flat, full[:sel.sum()])
    assert got[2].dtype == torch.int32 and got[3].dtype == torch.float32


@pytest.mark.parametrize("case", ["pos", "nopos", "list"])
def test_focal_loss_matches_reference(case):
    from models.losses.focal import focalLoss
    g = torch.Generator().manual_seed(7)
    gt = torch.rand(2, 1, 64, 64, generator=g) ** 4
    if case != "nopos":
        gt.view(-1)[torch.randint(0, gt.numel(), (25,), generator=g)] = 1.0
    gt.view(-1)[:5] = 1.5                               # > 1: neither positive nor negative (eq(1) / lt(1))
    n = 2 if case == "list" else 1
    preds = [O.clamp_sigmoid(torch.randn(gt.shape, generator=g)) for _ in range(n)]
    ref_in = [p.clone().requires_grad_(True) for p in preds]
    ref = O.focal_loss(ref_in, gt)
    ref.backward()
    hip_in = [p.to(DEV).requires_grad_(True) for p in preds]
    loss = focalLoss(hip_in, gt.to(DEV))
    (loss * 0.5).backward()
    assert loss.shape == ()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    for a, b in zip(hip_in, ref_in):
        assert _rel(a.grad, 0.5 * b.grad) < 1e-5


@pytest.mark.parametrize("smooth", [False, True])
@pytest.mark.parametrize("empty", [False, True])
def test_masked_l1_matches_reference(smooth, empty):
    from models.losses.regression import L1LossMask, smoothL1LossMask
    g = torch.Generator().manual_seed(11)
    B, K, C = 4, 30, 4
    r = torch.randn(B, K, C, generator=g) * 2
    t = torch.randn(B, K, C, generator=g) * 2
    mask = torch.rand(B, K, generator=g) > (1.0 if empty else 0.4)
    rr = r.clone().requires_grad_(True)
    num = mask.float().sum()
    m = mask.unsqueeze(2).expand_as(t)
    fn = F.smooth_l1_loss if smooth else F.l1_loss
    ref = fn(rr[m], t[m], reduction="sum") / (num + 1e-4)         # regression.py:28-44
    ref.backward()
    rh = r.to(DEV).requires_grad_(True)
    loss = (smoothL1LossMask if smooth else L1LossMask)(rh, t.to(DEV), mask.to(DEV))
    loss.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5, atol=1e-7)
    assert _rel(rh.grad, rr.grad) < 1e-5 or (empty and rh.grad.abs().max().item() == 0.0)


def test_helpers_refuse_cpu_tensors():
    from models.backbones.utility import nonMaximumSuppression
    with pytest.raises(RuntimeError, match="MI355X"):
        nonMaximumSuppression(torch.rand(1, 1, 8, 8))
