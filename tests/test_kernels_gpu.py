"""Per-kernel parity of libscdhip against PyTorch fp32 CPU references (floating-point ops).

Tolerances: fp32 parity mode (exact-f32 MFMA) 1e-4 relative to the output scale; bf16 mode
3e-2 relative (8-bit mantissa operands, fp32 accumulation)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel_err(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return (a - b).abs().max().item() / max(1e-6, b.abs().max().item())


def nhwc(t, dtype):
    return t.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)


def nchw(t):
    return t.float().permute(0, 3, 1, 2).cpu()


TOL = {torch.float32: 1e-4, torch.bfloat16: 3e-2, torch.float16: 1e-2}
CONV_CASES = [  # N, Cin, H, W, Cout, k, stride, pad
    (2, 64, 16, 16, 64, 3, 1, 1),
    (2, 64, 16, 16, 128, 3, 2, 1),
    (2, 64, 15, 13, 128, 1, 2, 0),
    (1, 128, 9, 11, 256, 3, 1, 1),
    (2, 64, 20, 20, 384, 3, 1, 1),
    (1, 256, 8, 8, 512, 3, 2, 1),
    (4, 128, 32, 32, 256, 3, 1, 1),     # large enough for the LDS-DMA ring kernels by default
    (3, 64, 41, 37, 192, 3, 2, 1),      # ragged pixels / channels on the ring kernels
    (2, 192, 11, 13, 256, 3, 1, 1),     # 27 K stages (odd) over the intra-workgroup split-K kernel, ragged M
    (4, 512, 16, 16, 512, 3, 1, 1),     # layer4 conv2 shape at batch 4: split K, 72 stages
    (4, 256, 128, 128, 64, 1, 1, 0),    # 1x1 into 64 channels over 256 tiles: the ring kernel, half-empty tiles
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case, dtype):
    from scdhip import ops
    N, Cin, H, W, Cout, k, s, p = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    if dtype != torch.float32:        # compare on operands representable in the 16-bit type
        x, w = x.to(dtype).float(), w.to(dtype).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    dy = torch.randn(yr.shape, generator=g)
    if dtype != torch.float32:
        dy = dy.to(dtype).float()
    yr.backward(dy)
    wd = w.to(DEV)
    xg = nhwc(x, dtype)
    stats = ops.new_stats(Cout, DEV)
    y = ops.conv_fwd(xg, ops.pack_weight(wd, dtype, 0), Cout, k, k, s, p, stats=stats)
    assert rel_err(nchw(y), yr) < TOL[dtype]
    # BN statistics from the epilogue
    st = stats.view(-1, 2, Cout).sum(0).cpu()
    yd = yr.detach().double()
    np.testing.assert_allclose(st[0].numpy(), yd.sum((0, 2, 3)).numpy(), rtol=1e-3, atol=1e-2 * yd.numel() ** 0.5)
    dyg = nhwc(dy, dtype)
    dx = ops.conv_dgrad(dyg, ops.pack_weight(wd, dtype, 1), Cin, H, W, k, k, s, p)
    assert rel_err(nchw(dx), xr.grad) < TOL[dtype]
    dw = torch.zeros_like(wd)
    ops.conv_wgrad(dyg, xg, k, k, s, p, dw, (Cin * k * k, k * k, 1), accumulate=False)
    assert rel_err(dw, wr.grad) < TOL[dtype] * 3


# shapes large enough (>= 256 tiles of 256 pixels) for the bf16 ping-pong kernels: halo variant (3x3 s1,
# width % 16 == 0; BN 256/192, 32- and 16-wide tiles, ragged tile rows, fwd and dgrad) and gather variant
LARGE_CONV_CASES = [
    (4, 256, 128, 128, 256, 3, 1, 1),     # halo BN 256 (fwd and dgrad), 8x32 tiles
    (12, 128, 64, 48, 384, 3, 1, 1),      # halo BN 192, 16x16 tiles
    (10, 64, 100, 64, 192, 3, 1, 1),      # halo BN 192 fwd, last tile row ragged
    (10, 192, 100, 64, 64, 3, 1, 1),      # halo BN 192 dgrad, ragged
    (2, 64, 181, 179, 384, 3, 1, 1),      # gather ping-pong (odd width), ragged M
    (2, 64, 128, 128, 384, 3, 1, 1),      # weight gradient: 256-channel ping-pong window + 128-channel remainder
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", LARGE_CONV_CASES)
def test_conv_large_bf16(case, dtype):
    test_conv_fwd_dgrad_wgrad(case, dtype)


# weight gradients on the ping-pong kernel with stages of several output rows (Wo = 16, 32: the layer3/4 shapes),
# the linear split map (split counts not a multiple of 8) and a 192-channel window
PP2_ROWS_CASES = [
    (16, 512, 16, 16, 512, 3, 1, 1),      # layer4 conv2, Wo 16
    (16, 256, 32, 32, 512, 3, 2, 1),      # layer4 conv1 (stride 2)
    (8, 256, 32, 32, 256, 3, 1, 1),       # layer3 conv2, Wo 32
    (16, 256, 32, 32, 512, 1, 2, 0),      # layer4 downsample 1x1 s2 (half-empty column tile)
    (12, 128, 32, 32, 384, 3, 1, 1),      # 192-channel windows, Wo 32
    (8, 64, 64, 64, 128, 3, 1, 1),        # 128-channel window (NQ 2): layer2 conv2 shape, Wo 64
    (8, 64, 128, 128, 128, 3, 2, 1),      # NQ 2, stride 2 (layer2 conv1)
    (16, 128, 32, 32, 128, 3, 1, 1),      # NQ 2, Wo 32
    (2, 256, 128, 128, 128, 3, 1, 1),     # NQ 2: the heatmap head's 3x3 weight gradient, Wo 128
    (4, 64, 32, 32, 320, 3, 1, 1),        # 256-channel window + a 64-channel remainder on the register-staged kernel
    (32, 64, 128, 128, 128, 1, 2, 0),     # NQ 2, 1x1 stride 2 (layer2 downsample; 256 splits of 8 stages)
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", PP2_ROWS_CASES)
def test_conv_wgrad_pp2_rows(case, dtype):
    test_conv_fwd_dgrad_wgrad(case, dtype)


@pytest.mark.parametrize("case", [(32, 64, 128, 128, 128, 1, 2, 0), (4, 256, 128, 128, 128, 3, 1, 1)])
def test_conv_wgrad_pp2_repeatable(case):
    """The 128-channel window kernel's stages are filled by both wave groups: the same weight gradient ten times
    over a workspace that held NaNs must come out bit-identical and finite every time (a group reading the other's
    half of a stage before it has landed shows as NaN or drift)."""
    from scdhip import ops
    N, Cin, H, W, Cout, k, s, p = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, H, W, Cin, generator=g).to(DEV, torch.bfloat16)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, Ho, Wo, Cout, generator=g).to(DEV, torch.bfloat16)
    outs = []
    for _ in range(10):
        junk = torch.full((64 << 20,), float("nan"), device=DEV)    # poison the caching allocator's free blocks
        del junk
        dw = torch.zeros(Cout, Cin, k, k, device=DEV)
        ops.conv_wgrad(dy, x, k, k, s, p, dw, (Cin * k * k, k * k, 1), accumulate=False)
        outs.append(dw)
    assert torch.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [(2, 128, 5, 7, 64), (1, 256, 8, 8, 256), (2, 64, 16, 16, 128),
                                  (8, 256, 64, 64, 256), (8, 256, 32, 32, 256), (16, 512, 16, 16, 256)])
def test_deconv_fwd_dgrad_wgrad(case, dtype):
    from scdhip import ops
    N, Cin, H, W, Cout = case
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cin, Cout, 4, 4, generator=g) / (Cin * 4) ** 0.5
    if dtype != torch.float32:
        x, w = x.to(dtype).float(), w.to(dtype).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, stride=2, padding=1)
    dy = torch.randn(yr.shape, generator=g)
    if dtype != torch.float32:
        dy = dy.to(dtype).float()
    yr.backward(dy)
    wd = w.to(DEV)
    xg = nhwc(x, dtype)
    y = ops.deconv_fwd(xg, ops.pack_weight(wd, dtype, 1), Cout)
    assert y.shape == (N, 2 * H, 2 * W, Cout)
    assert rel_err(nchw(y), yr) < TOL[dtype]
    dyg = nhwc(dy, dtype)
    dx = ops.deconv_dgrad(dyg, ops.pack_weight(wd, dtype, 0), Cin)
    assert rel_err(nchw(dx), xr.grad) < TOL[dtype]
    dw = torch.zeros_like(wd)
    ops.conv_wgrad(xg, dyg, 4, 4, 2, 1, dw, (Cout * 16, 16, 1), accumulate=False)
    assert rel_err(dw, wr.grad) < TOL[dtype] * 3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W", [(1, 128, 128), (2, 128, 128), (3, 37, 45)])
def test_heads_fused_gemm(N, H, W, dtype):
    """scd_conv_gemm_heads (3x3 conv + bias + ReLU with the three 1x1 tails in the epilogue) against
    torch fp32, hidden activation and head outputs; bf16 runs conv_gemm_heads384_kernel (one 192 x 384 tile
    per 192 pixels; 3x37x45 ends in a ragged tile and has image borders inside tiles)."""
    from scdhip import ops
    L = ops.L
    g = torch.Generator().manual_seed(31 + N)
    Cin, od = 256, [1, 4, 2]
    x = torch.randn(N, Cin, H, W, generator=g)
    w0 = [torch.randn(128, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5 for _ in od]
    b0 = [0.1 * torch.randn(128, generator=g) for _ in od]
    w1 = [torch.randn(o, 128, 1, 1, generator=g) / 128 ** 0.5 for o in od]
    b1 = [0.1 * torch.randn(o, generator=g) for o in od]
    if dtype != torch.float32:
        x = x.to(dtype).float()
        w0 = [w.to(dtype).float() for w in w0]
    refs = [F.conv2d(F.relu(F.conv2d(x, a, b, padding=1)), c, d) for a, b, c, d in zip(w0, b0, w1, b1)]
    xg = nhwc(x, dtype)
    w0c = torch.cat(w0, 0).to(DEV)
    wp = ops.pack_weight(w0c, dtype, 0)
    b0c = torch.cat(b0, 0).to(DEV)
    w1d = [w.to(DEV).contiguous() for w in w1]
    b1d = [b.to(DEV) for b in b1]
    outs = [torch.full((N, o, H, W), float("nan"), device=DEV) for o in od]
    hid = torch.empty(N, H, W, 128 * len(od), device=DEV, dtype=dtype)
    L.call("scd_conv_gemm_heads", ops.dt(xg), ops.ptr(xg), ops.ptr(wp), ops.ptr(hid), ops.ptr(b0c), N, H, W, Cin,
           len(od), L.int_array(od), L.ptr_array([w.data_ptr() for w in w1d]),
           L.ptr_array([b.data_ptr() for b in b1d]), L.ptr_array([o.data_ptr() for o in outs]), ops.stream())
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.isfinite(o).all()
        assert rel_err(o, r) < TOL[dtype] * (10 if dtype == torch.float32 else 3)
    hid_ref = torch.cat([F.relu(F.conv2d(x, a, b, padding=1)) for a, b in zip(w0, b0)], 1)
    assert rel_err(nchw(hid), hid_ref) < TOL[dtype] * 2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_heads_serpentine_k_order(dtype, monkeypatch):
    """conv_gemm_heads384_kernel walks K backwards on odd rounds of 256 workgroups (SCD_HEADS_SERP, weight reuse in
    L2): 4 x 128^2 pixels = 342 tiles, so tiles 256.. take the reversed order.  Same hidden activation and head
    outputs as the forward order up to fp32 summation order, and the same bits on every run."""
    from scdhip import ops
    L = ops.L
    g = torch.Generator().manual_seed(77)
    N, H, W, Cin, od = 4, 128, 128, 256, [1, 4, 2]
    xg = nhwc(torch.randn(N, Cin, H, W, generator=g), dtype)
    w0c = (torch.randn(384, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5).to(DEV)
    wp = ops.pack_weight(w0c, dtype, 0)
    b0c = (0.1 * torch.randn(384, generator=g)).to(DEV)
    w1d = [(torch.randn(o, 128, 1, 1, generator=g) / 128 ** 0.5).to(DEV) for o in od]
    b1d = [(0.1 * torch.randn(o, generator=g)).to(DEV) for o in od]

    def run(serp):
        monkeypatch.setenv("SCD_HEADS_SERP", str(serp))
        outs = [torch.full((N, o, H, W), float("nan"), device=DEV) for o in od]
        hid = torch.empty(N, H, W, 384, device=DEV, dtype=dtype)
        L.call("scd_conv_gemm_heads", ops.dt(xg), ops.ptr(xg), ops.ptr(wp), ops.ptr(hid), ops.ptr(b0c), N, H, W,
               Cin, len(od), L.int_array(od), L.ptr_array([w.data_ptr() for w in w1d]),
               L.ptr_array([b.data_ptr() for b in b1d]), L.ptr_array([o.data_ptr() for o in outs]), ops.stream())
        torch.cuda.synchronize()
        return hid, outs

    h0, o0 = run(0)
    h1, o1 = run(1)
    h2, o2 = run(1)
    assert torch.equal(h1, h2) and all(torch.equal(a, b) for a, b in zip(o1, o2))
    # workgroups 0..255 keep the forward order: their tiles (XCD-contiguous tile map of the kernel) have the same bits
    nwg = (N * H * W + 191) // 192
    q, r = nwg >> 3, nwg & 7
    fwd_tiles = [(x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + (b >> 3) for b in range(256) for x in [b & 7]]
    rows = torch.cat([torch.arange(t * 192, t * 192 + 192) for t in fwd_tiles]).to(DEV)
    assert torch.equal(h1.view(-1, 384)[rows], h0.view(-1, 384)[rows])
    assert rel_err(h1, h0) < 1e-2 and not torch.equal(h1, h0)
    # the 1x1 tails read the hidden activation rounded to the 16-bit type, so a summation-order change in the 3x3 GEMM
    # moves a head output by up to one rounding of the hidden value (measured 8.3e-4 bf16, 1.4e-4 fp16, normwise)
    tol = 2e-3 if dtype == torch.bfloat16 else 3e-4
    for a, b in zip(o1, o0):
        assert rel_err(a, b) < tol


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("HW", [(128, 128), (9, 11)])
def test_heads_tail_backward(HW, dtype, packed):
    """scd_heads_bwd + finalize (CenterNet tails, centerNetOffset.py:108-110): dhid = relu'(hid) * W1^T dout,
    dW1 = sum dout x hid, db1 = sum dout, db0 = sum dhid against torch fp32 on the same hidden tensor
    (128x128: whole 4-pixel unrolled steps; 9x11: ragged tail)."""
    from scdhip import ops
    L = ops.L
    g = torch.Generator().manual_seed(77)
    N, (H, W), Hd, od = 2, HW, 128, [1, 4, 2]
    P = N * H * W
    hid = F.relu(torch.randn(N, H, W, Hd * 3, generator=g))
    if dtype != torch.float32:
        hid = hid.to(dtype).float()
    w1 = [torch.randn(o, Hd, generator=g) / Hd ** 0.5 for o in od]
    douts = [torch.randn(N, o, H, W, generator=g) for o in od]
    hd = hid.to(DEV, dtype).contiguous()
    dhid = torch.empty_like(hd)
    odarr = L.int_array(od)
    acc = torch.zeros(L.lib().scd_heads_bwd_accsize(3, Hd, odarr) // 8, dtype=torch.float64, device=DEV)
    w1d = [w.to(DEV).contiguous() for w in w1]
    dd = [d.to(DEV).contiguous() for d in douts]
    dw1 = [torch.zeros(o, Hd, device=DEV) for o in od]
    db1 = [torch.zeros(o, device=DEV) for o in od]
    db0 = [torch.zeros(Hd, device=DEV) for o in od]
    if packed:        # gradients repacked pixel-major (x 0.5, undone below: the dscale path of the fp16 loss scale)
        pk = torch.empty(P * 3 * 4, device=DEV)
        L.call("scd_heads_bwd_packed", ops.dt(hd), ops.ptr(hd), N, H * W, 3, Hd, odarr,
               L.ptr_array([w.data_ptr() for w in w1d]), L.ptr_array([d.data_ptr() for d in dd]), 0.5, ops.ptr(pk),
               ops.ptr(dhid), ops.ptr(acc), ops.stream())
        dhid.mul_(2)
    else:
        L.call("scd_heads_bwd", ops.dt(hd), ops.ptr(hd), N, H * W, 3, Hd, odarr,
               L.ptr_array([w.data_ptr() for w in w1d]), L.ptr_array([d.data_ptr() for d in dd]), ops.ptr(dhid),
               ops.ptr(acc), ops.stream())
    L.call("scd_heads_bwd_weight_finalize", ops.ptr(acc), 3, Hd, odarr, L.ptr_array([t.data_ptr() for t in dw1]),
           L.ptr_array([t.data_ptr() for t in db1]), L.ptr_array([t.data_ptr() for t in db0]), 0,
           2.0 if packed else 1.0, ops.stream())
    torch.cuda.synchronize()
    hp = hid.reshape(P, 3 * Hd)
    tol = TOL[dtype] if dtype != torch.float32 else 1e-5
    for h, o in enumerate(od):
        hh = hp[:, h * Hd:(h + 1) * Hd]
        dh = douts[h].permute(0, 2, 3, 1).reshape(P, o)
        ref = (dh @ w1[h]) * (hh > 0)
        got = dhid.float().cpu().reshape(P, 3 * Hd)[:, h * Hd:(h + 1) * Hd]
        assert rel_err(got, ref) < tol
        assert rel_err(dw1[h], dh.t() @ hh) < 1e-5
        assert rel_err(db1[h], dh.sum(0)) < 1e-5
        assert rel_err(db0[h], ref.sum(0)) < 1e-5
    assert torch.count_nonzero(acc) == 0          # the finalize re-zeroes the persistent accumulators


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_im2col_gemm_pool(dtype):
    from scdhip import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 1, 64, 48, generator=g)
    w = torch.randn(64, 1, 7, 7, generator=g) / 7.0
    if dtype == torch.bfloat16:
        x, w = x.bfloat16().float(), w.bfloat16().float()
    cols = ops.im2col_stem(x.to(DEV), dtype)
    y = ops.conv_fwd(cols, ops.pack_weight(w.to(DEV), dtype, 0, ldp=64), 64, 1, 1, 1, 0)
    yr = F.conv2d(x, w, stride=2, padding=3)
    assert rel_err(nchw(y), yr) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 512, 512), (1, 260, 256)])
def test_stem_direct_bf16(shape, dtype):
    """Direct stem conv (tap tile built in LDS) forward + BN sums and its weight gradient vs torch fp32."""
    from scdhip import ops
    N, H, W = shape
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, 1, H, W, generator=g).to(dtype).float()
    w = (torch.randn(64, 1, 7, 7, generator=g) / 7.0).to(dtype).float()
    xr = x.clone()
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=2, padding=3)
    dy = torch.randn(yr.shape, generator=g).to(dtype).float()
    yr.backward(dy)
    xd = x.to(DEV)
    assert ops.stem_direct_ok(xd, dtype)
    stats = ops.new_stats(64, DEV)
    y = ops.stem_conv_fwd(xd, ops.pack_weight(w.to(DEV), dtype, 0, ldp=64), stats=stats)
    assert rel_err(nchw(y), yr) < TOL[dtype]
    st = stats.view(-1, 2, 64).sum(0).cpu()
    yd = yr.detach().double()
    np.testing.assert_allclose(st[0].numpy(), yd.sum((0, 2, 3)).numpy(), rtol=1e-3, atol=1e-2 * yd.numel() ** 0.5)
    dw = torch.full((64, 1, 7, 7), 0.25, device=DEV)
    ops.stem_conv_wgrad(nhwc(dy, dtype), xd, dw, accumulate=True)
    assert rel_err(dw - 0.25, wr.grad) < TOL[dtype] * 3


def test_stem_fused_backward_matches_unfused():
    """Stem backward: pool/ReLU backward fused with the BN reduction and the BN apply fused into the weight
    gradient give the unfused chain's dz (bit-exact), BN parameter gradients and conv weight gradient."""
    from scdhip import ops
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 1, 512, 512, generator=g).to(DEV)
    w = (torch.randn(64, 1, 7, 7, generator=g) / 7.0).to(DEV)
    bns = [torch.nn.BatchNorm2d(64).to(DEV) for _ in range(2)]
    for b in bns:
        with torch.no_grad():
            b.weight.uniform_(0.5, 1.5, generator=None)
            b.bias.normal_()
        b.bias.data.copy_(bns[0].bias.data)
        b.weight.data.copy_(bns[0].weight.data)
    stats = ops.new_stats(64, DEV)
    y = ops.stem_conv_fwd(x, ops.pack_weight(w, torch.bfloat16, 0, ldp=64), stats=stats)
    st = ops.bn_finalize(bns[0], stats, 64, y.numel() // 64)
    out, am = ops.stem_pool_fwd(y, st)
    dout = torch.randn(out.shape, generator=g).to(DEV, torch.bfloat16)
    dz = ops.stem_pool_bwd(dout, am, y, st)
    dy = ops.bn_backward(bns[0], st, dz, y)
    dwa = torch.zeros_like(w)
    ops.stem_conv_wgrad(dy, x, dwa)
    dz2, coef = ops.stem_pool_bwd_bn(bns[1], dout, am, y, st)
    dwb = torch.zeros_like(w)
    ops.stem_conv_wgrad(dz2, x, dwb, ybn=y, coef=coef)
    torch.cuda.synchronize()
    assert torch.equal(dz, dz2)
    for a, b in ((bns[0].weight.grad, bns[1].weight.grad), (bns[0].bias.grad, bns[1].bias.grad)):
        assert rel_err(b, a) < 1e-5
    assert rel_err(dwb, dwa) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 128, 128), (3, 130, 96), (1, 7, 9)])
def test_stem_pool_forward_matches_torch(shape, dtype):
    """scd_stem_pool_fwd (BN apply + ReLU + MaxPool(3, 2, 1), residuals.py:212-214; four pooled rows per thread) against
    float64 torch on the same 16-bit / fp32 conv output: the pooled value within one rounding of the output dtype, the
    argmax byte the window index of the first maximum wherever the window's top two differ clearly; pooled heights
    33 / 65 / 4 (ragged against the four rows per thread)."""
    from scdhip import ops
    N, H, W = shape
    C = 64
    g = torch.Generator().manual_seed(29)
    y = torch.randn(N, H, W, C, generator=g).to(dtype).to(DEV)
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    st = ops.BNState()
    st.scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
    st.shift = torch.randn(C, generator=g).to(DEV)
    out, am = ops.stem_pool_fwd(y, st)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    assert out.shape == (N, Ho, Wo, C) and am.shape == (N, Ho, Wo, C)
    z = torch.relu(y.double() * st.scale.double() + st.shift.double()).permute(0, 3, 1, 2)
    zp = torch.nn.functional.pad(z, (1, 1, 1, 1), value=float("-inf"))
    win = zp.unfold(2, 3, 2).unfold(3, 3, 2).reshape(N, C, Ho, Wo, 9)
    ref, arg = win.max(-1)
    got = out.double().permute(0, 3, 1, 2)
    ulp = {torch.bfloat16: 2.0 ** -7, torch.float16: 2.0 ** -10, torch.float32: 2.0 ** -23}[dtype]
    # one rounding of the output dtype, plus the fp32 rounding of y * scale + shift (values of a few units here)
    assert ((got - ref).abs() <= ulp * ref.abs() + 4e-6).all()
    top2 = win.topk(2, -1).values
    clear = (top2[..., 0] - top2[..., 1]) > 1e-3 * top2[..., 0].abs() + 1e-4    # (ReLU zeros tie: not checked)
    ga = am.long().permute(0, 3, 1, 2)
    assert clear.float().mean() > 0.7
    assert torch.equal(ga[clear], arg[clear])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 512, 512), (3, 260, 256)])
def test_stem_one_pass_backward(shape, dtype):
    """scd_stem_bwd_fused + combine (pool / ReLU / BN backward sums and the weight gradient as a T1 + b W G + c s,
    dz never stored) against the same backward in float64 from the same 16-bit y, dz, x and weights: the weight
    gradient within 2e-3 (the unfused kernels round dy to 16 bits: 2e-2), BN parameter gradients as the unfused
    reduction's (fp32 summation order).  (3, 260, 256): an odd pooled height (the last block row has no pooled row
    below it)."""
    from scdhip import ops
    N, H, W = shape
    g = torch.Generator().manual_seed(19)
    x = torch.randn(N, 1, H, W, generator=g).to(dtype).float().to(DEV)
    w = (torch.randn(64, 1, 7, 7, generator=g) / 7.0).to(dtype).float().to(DEV)
    bns = [torch.nn.BatchNorm2d(64).to(DEV) for _ in range(2)]
    with torch.no_grad():
        bns[0].weight.uniform_(0.5, 1.5)
        bns[0].bias.normal_()
    for b in bns[1:]:
        b.weight.data.copy_(bns[0].weight.data)
        b.bias.data.copy_(bns[0].bias.data)
    wpk = ops.pack_weight(w, dtype, 0, ldp=64)
    stats = ops.new_stats(64, DEV)
    y = ops.stem_conv_fwd(x, wpk, stats=stats)
    st = ops.bn_finalize(bns[0], stats, 64, y.numel() // 64)
    out, am = ops.stem_pool_fwd(y, st)
    dout = torch.randn(out.shape, generator=g).to(DEV, dtype)
    # unfused: dz (16-bit), BN backward sums, dy
    dz = ops.stem_pool_bwd(dout, am, y, st)
    dy = ops.bn_backward(bns[0], st, dz, y)
    dwa = torch.zeros_like(w)
    ops.stem_conv_wgrad(dy, x, dwa)
    dwb = torch.full_like(w, 0.5)
    ops.stem_backward_fused(bns[1], dout, am, y, st, x, wpk, dwb)
    torch.cuda.synchronize()
    for a, b in ((bns[0].weight.grad, bns[1].weight.grad), (bns[0].bias.grad, bns[1].bias.grad)):
        assert rel_err(b, a) < 1e-5
    # float64 backward from the same operands
    zd = dz.double()
    yd = y.double()
    mu, iv = st.mean.double(), st.invstd.double()
    xh = (yd - mu) * iv
    cnt = zd.numel() // 64
    k1 = zd.sum((0, 1, 2)) / cnt
    k2 = (zd * xh).sum((0, 1, 2)) / cnt
    dyd = (bns[0].weight.double() * iv) * (zd - k1 - xh * k2)
    xr = x.double()
    ref = torch.nn.grad.conv2d_weight(xr, (64, 1, 7, 7), dyd.permute(0, 3, 1, 2), stride=2, padding=3)
    assert rel_err(dwb - 0.5, ref) < 2e-3
    assert rel_err(dwa, ref) < 2e-2


def test_cpool_fwd_bwd_fp32():
    from scdhip import ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 8, 9, 12, generator=g)
    x[0, 0, 3, :] = x[0, 0, 5, :]          # ties along H
    x[1, 2, :, 4] = 0.5                    # constant lines
    dy = torch.randn(x.shape, generator=g)
    from oracle import cpool as CP
    for d in range(4):
        y = ops.cpool_fwd(nhwc(x, torch.float32), d)
        np.testing.assert_allclose(nchw(y).numpy(), CP.forward(x, d).numpy(), rtol=0, atol=0)
        dx = ops.cpool_bwd(nhwc(x, torch.float32), nhwc(dy, torch.float32), d)
        np.testing.assert_allclose(nchw(dx).numpy(), CP.backward(x, dy, d).numpy(), rtol=1e-6, atol=1e-6)


def test_adam_matches_torch():
    from scdhip import ops
    g = torch.Generator().manual_seed(9)
    p0 = torch.randn(10007, generator=g)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=1e-3)
    p = p0.clone().to(DEV)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step in range(1, 4):
        gr = torch.randn(10007, generator=g)
        pt.grad = gr.clone()
        opt.step()
        ops.adam_step(p, gr.to(DEV), m, v, 1e-3, 0.9, 0.999, 1e-8, step)
    np.testing.assert_allclose(p.cpu().numpy(), pt.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_adam_device_state_matches_torch():
    """scd_adam_step_dev: {lr, step} in device memory (the step-graph form), step advanced on the stream; an lr
    change between steps is picked up."""
    from scdhip import ops
    g = torch.Generator().manual_seed(10)
    p0 = torch.randn(10007, generator=g)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=1e-3)
    p = p0.clone().to(DEV)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    hyper = torch.tensor([1e-3, 0.0], dtype=torch.float64, device=DEV)
    for step in range(1, 7):
        if step == 4:
            opt.param_groups[0]["lr"] = 2.5e-4
            hyper[0].fill_(2.5e-4)
        gr = torch.randn(10007, generator=g)
        pt.grad = gr.clone()
        opt.step()
        ops.adam_step_dev(p, gr.to(DEV), m, v, hyper, 0.9, 0.999, 1e-8)
    assert hyper[1].item() == 6.0
    np.testing.assert_allclose(p.cpu().numpy(), pt.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_optimizer_skip_word_and_nan_bn_finalize():
    """after a failed peer-memory SyncBN call (its error word set, statistics NaN) the Adam / SGD step
    changes nothing (parameters, moments, step count) and the BN finalize keeps running_mean / running_var AND
    num_batches_tracked; with the word clear, both update as usual."""
    from scdhip import ops
    p0 = torch.randn(5003, device=DEV)
    gr = torch.randn(5003, device=DEV)
    bad = torch.ones(1, dtype=torch.int64, device=DEV)
    ok = torch.zeros(1, dtype=torch.int64, device=DEV)
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    hyper = torch.tensor([1e-3, 0.0], dtype=torch.float64, device=DEV)
    ops.adam_step_dev(p, gr, m, v, hyper, 0.9, 0.999, 1e-8, skip=bad)
    torch.cuda.synchronize()
    assert torch.equal(p, p0) and not m.any() and not v.any() and hyper[1].item() == 0.0
    ops.adam_step_dev(p, gr, m, v, hyper, 0.9, 0.999, 1e-8, skip=ok)
    torch.cuda.synchronize()
    assert not torch.equal(p, p0) and hyper[1].item() == 1.0
    buf = torch.zeros_like(p0)
    p = p0.clone()
    sh = torch.tensor([0.1, 0.0, 0.0, 0.0], dtype=torch.float64, device=DEV)
    ops.sgd_step_dev(p, gr, buf, sh, 0.9, 0.0, 1e-4, False, skip=bad)
    torch.cuda.synchronize()
    assert torch.equal(p, p0) and not buf.any() and sh[1].item() == 0.0
    # BN finalize on NaN-poisoned (collapsed, nrep 1) statistics
    C = 96
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    bn.running_mean.normal_()
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    nb = int(bn.num_batches_tracked.item())
    stats = torch.full((2 * C,), float("nan"), dtype=torch.float64, device=DEV)
    st = ops._bn_state(C, DEV)
    ops._bn_finalize_launch(bn, st, stats, 1, C, 100.0)
    torch.cuda.synchronize()
    assert torch.equal(bn.running_mean, rm) and torch.equal(bn.running_var, rv)
    assert int(bn.num_batches_tracked.item()) == nb
    stats = torch.cat([torch.full((C,), 5.0), torch.full((C,), 100.0)]).double().to(DEV)
    ops._bn_finalize_launch(bn, st, stats, 1, C, 100.0)
    torch.cuda.synchronize()
    assert int(bn.num_batches_tracked.item()) == nb + 1 and not torch.equal(bn.running_mean, rm)


@pytest.mark.parametrize("nesterov,damp", [(False, 0.0), (True, 0.0), (False, 0.25)])
def test_flat_sgd_matches_torch(nesterov, damp):
    """FlatSGD (scd_sgd_step_dev) against torch.optim.SGD with the reference's settings (networkFactory.py:84-89:
    momentum 0.9, weight_decay 1e-4): first step clones d into the momentum buffer; an lr change (setLearningRate)
    between steps is picked up; momentum state survives state_dict round trips."""
    from scdhip.flat import FlatSGD
    g = torch.Generator().manual_seed(11)
    shapes = [(64, 3, 3, 3), (64,), (1000,)]
    p0 = [torch.randn(*s, generator=g) for s in shapes]
    pt = [x.clone().requires_grad_(True) for x in p0]
    opt_t = torch.optim.SGD(pt, lr=2.5e-4, momentum=0.9, weight_decay=1e-4, nesterov=nesterov, dampening=damp)
    pd = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    opt = FlatSGD(pd, lr=2.5e-4, momentum=0.9, weight_decay=1e-4, nesterov=nesterov, dampening=damp)
    for step in range(1, 7):
        if step == 4:
            for o in (opt_t, opt):
                o.param_groups[0]["lr"] = 2.5e-5
        opt.zero_grad()
        for a, b in zip(pt, pd):
            gr = torch.randn(a.shape, generator=g)
            a.grad = gr.clone()
            b.grad.copy_(gr.to(DEV))
        opt_t.step()
        opt.step()
        if step == 2:
            sd = opt.state_dict()
            opt2 = FlatSGD(pd, lr=2.5e-4, momentum=0.9, weight_decay=1e-4, nesterov=nesterov, dampening=damp)
            opt2.load_state_dict(sd)
            opt = opt2
    for a, b in zip(pt, pd):
        np.testing.assert_allclose(b.detach().cpu().numpy(), a.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_flat_sgd_buffer_reset_matches_torch():
    """A momentum buffer re-created mid-training starts as torch's does (clone of d on its first update), also with
    dampening != 0 where the global step count would give (1-dampening)*d (ADVICE r3 flat.py:219): the state is
    loaded without a momentum_buffer on both sides after two steps."""
    from scdhip.flat import FlatSGD
    g = torch.Generator().manual_seed(13)
    p0 = [torch.randn(64, 3, 3, 3, generator=g), torch.randn(1000, generator=g)]
    pt = [x.clone().requires_grad_(True) for x in p0]
    kw = dict(lr=2.5e-4, momentum=0.9, weight_decay=1e-4, dampening=0.25)
    opt_t = torch.optim.SGD(pt, **kw)
    pd = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    opt = FlatSGD(pd, **kw)
    for step in range(1, 6):
        if step == 3:
            opt_t.state.clear()                         # torch: no momentum_buffer -> the next step clones d
            sd = opt.state_dict()
            sd["momentum_buffer"] = None
            opt.load_state_dict(sd)
        opt.zero_grad()
        for a, b in zip(pt, pd):
            gr = torch.randn(a.shape, generator=g)
            a.grad = gr.clone()
            b.grad.copy_(gr.to(DEV))
        opt_t.step()
        opt.step()
    for a, b in zip(pt, pd):
        np.testing.assert_allclose(b.detach().cpu().numpy(), a.detach().numpy(), rtol=1e-6, atol=1e-7)
    with pytest.raises(ValueError):
        FlatSGD(pd, lr=1e-3).load_state_dict({"step": 1, "param_groups": [{"lr": 1e-3}],
                                              "momentum_buffer": torch.zeros(64 * 27 + 1000)})


def test_flat_sgd_state_before_first_step_matches_torch():
    """A FlatSGD state saved before any step (the flat buffer and its zero momentum buffer exist from zero_grad on)
    carries no momentum_buffer, as torch's does, so a run resumed from it clones d on its first update also with
    dampening != 0 (ADVICE r4 flat.py:227)."""
    from scdhip.flat import FlatSGD
    g = torch.Generator().manual_seed(17)
    p0 = [torch.randn(64, 3, 3, 3, generator=g), torch.randn(1000, generator=g)]
    pt = [x.clone().requires_grad_(True) for x in p0]
    kw = dict(lr=2.5e-4, momentum=0.9, weight_decay=1e-4, dampening=0.25)
    opt_t = torch.optim.SGD(pt, **kw)
    pd = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    opt = FlatSGD(pd, **kw)
    opt.zero_grad()
    sd = opt.state_dict()
    assert sd["momentum_buffer"] is None and "momentum_buffer" not in opt_t.state_dict()["state"].get(0, {})
    opt = FlatSGD(pd, **kw)
    opt.load_state_dict(sd)
    for _ in range(3):
        opt.zero_grad()
        for a, b in zip(pt, pd):
            gr = torch.randn(a.shape, generator=g)
            a.grad = gr.clone()
            b.grad.copy_(gr.to(DEV))
        opt_t.step()
        opt.step()
    assert opt.state_dict()["momentum_buffer"] is not None
    for a, b in zip(pt, pd):
        np.testing.assert_allclose(b.detach().cpu().numpy(), a.detach().numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_batched_pack_matches_single(dtype):
    """PackPlan's one-launch batched packing (mode 0 rows, mode 1 LDS-tiled transposes, mode 2 tap-major
    transposes, concatenated head operands) reproduces the per-weight scd_pack_weight layouts bit for bit, and
    mode 2 is out[t*B + b][a] = w[a][b][t]."""
    from scdhip import ops
    g = torch.Generator().manual_seed(12)
    shapes = [(64, 64, 3, 3), (128, 64, 3, 3), (128, 64, 1, 1), (512, 256, 3, 3), (256, 256, 4, 4), (64, 1, 7, 7),
              (96, 40, 3, 3), (200, 72, 4, 4)]
    ws = [torch.nn.Parameter((torch.randn(*s, generator=g)).to(DEV)) for s in shapes]
    heads = [torch.nn.Parameter(torch.randn(128, 256, 3, 3, generator=g).to(DEV)) for _ in range(3)]
    plan = ops.PackPlan()
    ops.pack_begin(plan)                       # first step: records and packs on demand
    first = [ops.pack_weight(w, dtype, m) for w in ws for m in (0, 1)]
    first += [ops.pack_concat(heads, dtype, m) for m in (0, 1, 2)]
    first += [ops.pack_concat(heads[1:], dtype, 2)]
    first = [f.clone() for f in first]
    ops.pack_end()
    # scribble over the cached operands, then repack everything in one batched launch
    for e in plan.entries.values():
        e[0].fill_(float("nan"))
    ops.pack_begin(plan)
    again = [ops.pack_weight(w, dtype, m) for w in ws for m in (0, 1)]
    again += [ops.pack_concat(heads, dtype, m) for m in (0, 1, 2)]
    again += [ops.pack_concat(heads[1:], dtype, 2)]
    torch.cuda.synchronize()
    ops.pack_end()
    for a, b in zip(first, again):
        assert torch.equal(a, b)
    cat = torch.cat([h.detach() for h in heads[1:]], 0)                     # (A=256, B=256, 3, 3)
    want = cat.reshape(256, 256, 9).permute(2, 1, 0).reshape(9 * 256, 256).to(dtype)
    assert torch.equal(first[-1], want)


def _pp_taken(N, phases, Cout):
    """The ping-pong (fused BN-sum epilogue) rule of conv_gemm_launch: bf16, Cout % 256 or % 192 == 0 and at
    least 256 tiles of 256 pixels over all sub-pixel phases."""
    bn = 256 if Cout % 256 == 0 else (192 if Cout % 192 == 0 else 0)
    if not bn:
        return False
    return sum(-(-(N * ph.Qh * ph.Qw) // 256) for ph in phases) * (Cout // bn) >= 256


# (N, Hc, Wc, Co = dy channels, Ci = input-gradient channels, k, stride, pad, fused?)
BNBWD_CASES = [
    (4, 128, 128, 384, 256, 3, 1, 1, True),      # heads / deconv shapes: one 3x3 phase
    (2, 40, 36, 384, 256, 3, 1, 1, False),       # too few tiles: GEMM + separate reduce
    (4, 128, 128, 64, 256, 1, 1, 0, True),       # Bottleneck conv1 1x1 (256 -> 64) dgrad
    (4, 128, 128, 256, 64, 1, 1, 0, False),      # Bottleneck conv3 1x1 (64 -> 256) dgrad into 64 channels: ring
    (4, 128, 128, 256, 256, 3, 2, 1, True),      # Bottleneck stride-2 3x3: 4 sub-pixel phases, out_stride 2
    (4, 128, 128, 512, 256, 1, 2, 0, True),      # downsample 1x1 stride 2: one phase with taps, three empty
    (16, 66, 70, 128, 192, 3, 2, 1, True),       # ragged phases (odd/even extents), 192-wide tiles
    # the shared epilogue of the ring / register-staged kernels (BasicBlock layer1/layer2 bn1 shapes)
    (4, 128, 128, 64, 64, 3, 1, 1, False),       # 64 channels: 256 x 64 register-staged kernel
    (16, 64, 64, 128, 128, 3, 1, 1, False),      # 128 channels, >= 256 tiles: LDS-DMA ring kernel
    (4, 64, 64, 128, 128, 3, 1, 1, False),       # 128 channels, few tiles: 128 x 128 register-staged kernel
    (8, 64, 64, 128, 64, 3, 2, 1, False),        # stride-2 3x3 into 64 channels: 4 phases, narrow kernel
    (3, 33, 35, 64, 128, 3, 2, 1, False),        # ragged odd extents, 128 x 128 kernel
]


@pytest.mark.parametrize("case", BNBWD_CASES)
def test_dgrad_with_bn_backward_sums(case):
    """scd_conv_gemm_bnbwd (input-gradient GEMM whose epilogue adds the following BN+ReLU layer's backward sums)
    against scd_conv_gemm + scd_bn_bwd_reduce: identical gradient, sums within fp32 summation-order noise.
    The multi-phase cases check the epilogue's pixel / sub-pixel (rho) mapping of the BN sums on the shapes the
    Bottleneck blocks send through it; `fused` states which path the launch rule takes."""
    from scdhip import ops
    N, H, W, Co, Ci, k, stride, pad, fused = case
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    assert _pp_taken(N, ops._dgrad_phases(k, k, stride, pad, H, W), Ci) == fused
    g = torch.Generator().manual_seed(41)
    dy = (torch.randn(N, Ho, Wo, Co, generator=g) * 0.1).to(DEV, torch.bfloat16)
    w = (torch.randn(Co, Ci, k, k, generator=g) / (Ci * k * k) ** 0.5).to(DEV)
    ybn = torch.randn(N, H, W, Ci, generator=g).to(DEV, torch.bfloat16)

    class St:
        pass
    st = St()
    st.mean = (torch.randn(Ci, generator=g) * 0.1).to(DEV)
    st.invstd = (torch.rand(Ci, generator=g) + 0.5).to(DEV)
    st.scale = (torch.rand(Ci, generator=g) + 0.5).to(DEV)
    st.shift = (torch.randn(Ci, generator=g) * 0.2).to(DEV)
    wt = ops.pack_weight(w, torch.bfloat16, 1)
    s1 = torch.zeros(64 * 2 * Ci, dtype=torch.float64, device=DEV)
    s2 = torch.zeros_like(s1)
    dx1 = ops.conv_dgrad(dy, wt, Ci, H, W, k, k, stride, pad, bn_bwd=(st, ybn, s1))
    dx2 = ops.conv_dgrad(dy, wt, Ci, H, W, k, k, stride, pad)
    separate = 256 % (Ci // 8) == 0           # scd_bn_bwd_reduce takes channel counts whose 16-B chunks divide 256
    if separate:
        ops.L.call("scd_bn_bwd_reduce", ops.dt(dx2), ops.ptr(dx2), 0, ops.ptr(ybn), ops.ptr(st.scale),
                   ops.ptr(st.shift), ops.ptr(st.mean), ops.ptr(st.invstd), Ci, dx2.numel(), ops.ptr(s2), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx2)
    # independent fp64 check of the sums from the GEMM output (dz = relu-masked gradient, xhat from ybn)
    yf = ybn.double()
    xhat = (yf - st.mean.double()) * st.invstd.double()
    act = (yf * st.scale.double() + st.shift.double()) > 0
    dz = torch.where(act, dx2.double(), torch.zeros((), dtype=torch.float64, device=DEV))
    ref = torch.stack([dz.sum((0, 1, 2)), (dz * xhat).sum((0, 1, 2))]).cpu()
    a = s1.view(64, 2, Ci).sum(0).cpu()
    b = s2.view(64, 2, Ci).sum(0).cpu()
    for i in range(2):
        if separate:
            assert (a[i] - b[i]).abs().max().item() <= 1e-5 * b[i].abs().max().item() + 1e-9, i
        assert (a[i] - ref[i]).abs().max().item() <= 1e-4 * ref[i].abs().max().item() + 1e-9, i


# 64 -> 64 channel 3x3 stride-1 convs (layer1 shapes) on every width the Res10/18/34 stacks and ragged sizes give
LAYER1_CASES = [
    (4, 64, 128, 128, 64, 3, 1, 1),
    (8, 64, 128, 128, 64, 3, 1, 1),
    (3, 64, 64, 64, 64, 3, 1, 1),
    (2, 64, 32, 128, 64, 3, 1, 1),
    (40, 64, 16, 16, 64, 3, 1, 1),
    (5, 64, 24, 16, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", LAYER1_CASES)
def test_conv_layer1_bf16(case):
    test_conv_fwd_dgrad_wgrad(case, torch.bfloat16)


# the layer1 weight gradient (conv_wgrad_l1_kernel: 64 x 576 per workgroup, halo-staged input): widths 64 (a stage is
# a whole row, both borders in it), 128, 192 (a middle stage with in-image neighbours on both sides), ragged splits
L1_WGRAD_CASES = [
    (3, 64, 64, 64, 64, 3, 1, 1),
    (4, 64, 128, 128, 64, 3, 1, 1),
    (2, 64, 32, 192, 64, 3, 1, 1),
    (1, 64, 7, 64, 64, 3, 1, 1),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", L1_WGRAD_CASES)
def test_conv_wgrad_layer1(case, dtype):
    test_conv_fwd_dgrad_wgrad(case, dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
# (tiles of 256 px >= 2 x CUs give runs of 2..16 tiles per workgroup: the row ring is reused; fewer: one tile each)
@pytest.mark.parametrize("N,H,W", [(4, 128, 128), (3, 64, 64), (2, 32, 128), (16, 128, 128), (64, 64, 64),
                                   (32, 128, 128), (2, 32, 256), (8, 128, 256)])
def test_conv_l1p_matches_register_staged(N, H, W, dtype, monkeypatch):
    """conv_gemm_l1p_kernel (layer1 3x3 64 -> 64: a persistent ring of input rows in LDS, every tap read at a
    constant displacement) runs the same MFMA sequence
    per output as the register-staged 256 x 64 kernel (tap-major, two K halves per tap): forward, input gradient
    (+= accumulate) and the BN-backward-sum variant's gradient are bit-identical; the BN sums agree to fp32
    summation-order noise."""
    from scdhip import ops
    g = torch.Generator().manual_seed(71)
    C = 64
    x = nhwc(torch.randn(N, C, H, W, generator=g), dtype)
    w = (torch.randn(C, C, 3, 3, generator=g) / 24).to(DEV)
    base = nhwc(torch.randn(N, C, H, W, generator=g), dtype)
    ybn = nhwc(torch.randn(N, C, H, W, generator=g), dtype)

    class St:
        pass
    st = St()
    st.mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
    st.invstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    st.scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
    st.shift = (torch.randn(C, generator=g) * 0.2).to(DEV)
    outs = {}
    for mode in ("1", "0"):               # persistent row-ring kernel, register-staged kernel
        monkeypatch.setenv("SCD_GEMM_HALO64", mode)
        wp, wt = ops.pack_weight(w, dtype, 0), ops.pack_weight(w, dtype, 1)
        stats = torch.zeros(64 * 2 * C, dtype=torch.float64, device=DEV)
        y = ops.conv_fwd(x, wp, C, 3, 3, 1, 1, stats=stats)
        dx = base.clone()
        ops.conv_dgrad(x, wt, C, H, W, 3, 3, 1, 1, out=dx, accumulate=True)
        bst = torch.zeros(64 * 2 * C, dtype=torch.float64, device=DEV)
        dxb = ops.conv_dgrad(x, wt, C, H, W, 3, 3, 1, 1, bn_bwd=(st, ybn, bst))
        torch.cuda.synchronize()
        outs[mode] = (y, stats.view(64, 2, C).sum(0), dx, dxb, bst.view(64, 2, C).sum(0))
    for m in ("1",):
        for i in (0, 2, 3):                                  # y, dx (+=), dx of the BN-backward-sum variant
            assert torch.equal(outs[m][i], outs["0"][i]), (m, i)
        for i in (1, 4):                                     # BN sums: fp32 partials over other pixel groups
            d = (outs[m][i] - outs["0"][i]).abs().max().item()
            assert d <= 1e-5 * outs["0"][i].abs().max().item(), (m, i, d)
    xr = nchw(x).float().requires_grad_(True)
    ref = F.conv2d(xr, w.cpu().to(dtype).float(), padding=1)
    assert rel_err(nchw(outs["1"][0]), ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K,C,N", [(64, 64, 2), (128, 64, 2), (256, 64, 2), (64, 128, 2), (256, 128, 2), (64, 256, 2),
                                   (128, 256, 2), (128, 512, 2), (512, 128, 2), (256, 256, 2), (256, 1024, 2),
                                   (1024, 256, 2), (64, 256, 3), (256, 256, 3)])
def test_conv1x1_stream_matches_tiled(K, C, N, dtype, monkeypatch):
    """conv1x1_stream_kernel (HBM-bound stride-1 1x1 GEMMs: weights resident in LDS, operands streamed into the MFMA
    fragments; the Res50 layer1 1x1 convs, residuals.py:122-165) against the tiled kernels on the same shapes: the
    forward K -> C with its BN statistics, the input gradient C -> K, its += form and the BN-backward-sum form, each
    where the stream kernel is built for the GEMM shape (K_gemm, N_gemm).  Outputs are bit-identical (same MFMA chain
    per output); statistics and BN sums agree to fp32 summation-order noise.  SCD_GEMM_STREAM1X1=2 fails any GEMM the
    stream kernel does not take, so the "2" results are its own.  The pixel runs per workgroup follow the instance's
    residency (launch_stream1x1 in conv_gemm.hip); N = 3 gives 1,536 chunks of 128 pixels."""
    from scdhip import ops
    # (K_gemm, N_gemm) built into the stream kernel; N = 1024 runs as four 256-channel slices
    sums = {(64, 64), (128, 64), (256, 64), (64, 128), (128, 128), (256, 128), (64, 256), (128, 256), (128, 512),
            (512, 128), (256, 256), (256, 1024)}
    plain = sums
    accum = {(64, 64), (128, 64), (256, 64), (64, 128), (128, 128), (256, 128), (64, 256), (128, 512), (512, 128),
             (256, 256), (256, 1024)}
    bnbwd = {(64, 64), (128, 64), (256, 64), (64, 128), (128, 128), (256, 128), (512, 128), (256, 256), (256, 1024)}
    g = torch.Generator().manual_seed(113)
    H, W = 256, 256                                          # M = 131,072 pixels (N = 3: 196,608, a grid that is no
    #                                                          power of two of 128-pixel chunks)
    x = nhwc(torch.randn(N, K, H, W, generator=g), dtype)
    w = (torch.randn(C, K, 1, 1, generator=g) / K ** 0.5).to(DEV)
    dy = nhwc(torch.randn(N, C, H, W, generator=g), dtype)
    base = nhwc(torch.randn(N, K, H, W, generator=g), dtype)
    ybn = nhwc(torch.randn(N, K, H, W, generator=g), dtype)

    class St:
        pass
    st = St()
    st.mean = (torch.randn(K, generator=g) * 0.1).to(DEV)
    st.invstd = (torch.rand(K, generator=g) + 0.5).to(DEV)
    st.scale = (torch.rand(K, generator=g) + 0.5).to(DEV)
    st.shift = (torch.randn(K, generator=g) * 0.2).to(DEV)
    outs = {}
    for mode in ("2", "0"):                  # the stream kernel only, the tiled kernels
        monkeypatch.setenv("SCD_GEMM_STREAM1X1", mode)
        wp, wt = ops.pack_weight(w, dtype, 0), ops.pack_weight(w, dtype, 1)
        r = {}
        if (K, C) in sums:
            stats = torch.zeros(64 * 2 * C, dtype=torch.float64, device=DEV)
            r["y"] = ops.conv_fwd(x, wp, C, 1, 1, 1, 0, stats=stats)
            r["stats"] = stats.view(64, 2, C).sum(0)
        if (C, K) in plain:
            r["dx"] = ops.conv_dgrad(dy, wt, K, H, W, 1, 1, 1, 0)
        if (C, K) in accum:
            r["dx+"] = base.clone()
            ops.conv_dgrad(dy, wt, K, H, W, 1, 1, 1, 0, out=r["dx+"], accumulate=True)
        if (C, K) in bnbwd:
            bst = torch.zeros(64 * 2 * K, dtype=torch.float64, device=DEV)
            r["dxb"] = ops.conv_dgrad(dy, wt, K, H, W, 1, 1, 1, 0, bn_bwd=(st, ybn, bst))
            r["bsums"] = bst.view(64, 2, K).sum(0)
        torch.cuda.synchronize()
        outs[mode] = r
    assert outs["0"], "no GEMM of this case is built into the stream kernel"
    for k, v in outs["0"].items():
        if k in ("stats", "bsums"):
            d = (outs["2"][k] - v).abs().max().item()
            assert d <= 1e-5 * v.abs().max().item(), (k, d)
        else:
            assert torch.equal(outs["2"][k], v), k
    if "y" in outs["2"]:
        ref = F.conv2d(nchw(x).float(), w.cpu().to(dtype).float())
        assert rel_err(nchw(outs["2"]["y"]), ref) < TOL[dtype]
        yf = outs["2"]["y"].float().view(-1, C)
        ref_s = torch.stack([yf.sum(0), (yf * yf).sum(0)]).double()
        assert (outs["2"]["stats"] - ref_s).abs().max().item() <= 2e-2 * ref_s.abs().max().item()
    if "dx" in outs["2"]:
        dref = F.conv_transpose2d(nchw(dy).float(), w.cpu().to(dtype).float())
        assert rel_err(nchw(outs["2"]["dx"]), dref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,Hq,Cg,Cin,taken", [(32, 64, 128, 64, True), (32, 32, 256, 128, True),
                                               (4, 16, 512, 256, False), (3, 17, 128, 64, False)])
def test_conv_dgrad_s2_phase_gemm(N, Hq, Cg, Cin, taken, dtype):
    """Input gradient of a 3x3 / stride 2 / pad 1 conv as one 2x2-tap GEMM with the four sub-pixel phases as output
    channels (scd_conv_dgrad_s2, pack mode 3) against torch fp32 and the phase-decomposed gather-GEMM; `taken`:
    whether the shape goes to the ping-pong kernel (otherwise ops.conv_dgrad_w falls back), plus += accumulation."""
    from scdhip import ops
    g = torch.Generator().manual_seed(23)
    dy = torch.randn(N, Cg, Hq, Hq, generator=g).to(dtype).float()
    w = (torch.randn(Cg, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5).to(dtype).float()
    base = torch.randn(N, Cin, 2 * Hq, 2 * Hq, generator=g).to(dtype).float()
    x = torch.zeros(N, Cin, 2 * Hq, 2 * Hq, requires_grad=True)
    F.conv2d(x, w, stride=2, padding=1).backward(dy)
    dyd = nhwc(dy, dtype)
    out = torch.empty(N, 2 * Hq, 2 * Hq, Cin, dtype=dtype, device=DEV)
    rc = ops.L.lib().scd_conv_dgrad_s2(ops.dt(dyd), ops.ptr(dyd), ops.ptr(ops.pack_weight(w.to(DEV), dtype, 3)),
                                       ops.ptr(out), N, Hq, Hq, Cg, Cin, 0, ops.stream())
    assert (rc == 0) == taken and rc in (0, 9001)
    dx = ops.conv_dgrad_w(dyd, w.to(DEV), 2 * Hq, 2 * Hq, 2, 1)
    ref_gather = ops.conv_dgrad(dyd, ops.pack_weight(w.to(DEV), dtype, 1), Cin, 2 * Hq, 2 * Hq, 3, 3, 2, 1)
    acc = nhwc(base, dtype)
    ops.conv_dgrad_w(dyd, w.to(DEV), 2 * Hq, 2 * Hq, 2, 1, out=acc, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(nchw(dx), x.grad) < TOL[dtype]
    assert rel_err(nchw(dx), nchw(ref_gather)) < TOL[dtype]
    if taken:
        assert torch.equal(dx, out)
    assert rel_err(nchw(acc), base + x.grad) < TOL[dtype]


def test_conv_layer1_accumulate_and_bias_relu():
    """Epilogue paths the block code uses on the layer1 shapes: dgrad += into an existing gradient, and a
    forward with bias + ReLU."""
    from scdhip import ops
    g = torch.Generator().manual_seed(7)
    N, C, H, W = 4, 64, 128, 128
    x = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    w = (torch.randn(C, C, 3, 3, generator=g) / 24).bfloat16().float()
    b = torch.randn(C, generator=g)
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    y = ops.conv_fwd(nhwc(x, torch.bfloat16), ops.pack_weight(w.to(DEV), torch.bfloat16, 0), C, 3, 3, 1, 1,
                     bias=b.to(DEV), relu=True)
    assert rel_err(nchw(y), ref) < 3e-2
    dy = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    base = torch.randn(N, C, H, W, generator=g).bfloat16().float()
    dx = nhwc(base, torch.bfloat16)
    ops.conv_dgrad(nhwc(dy, torch.bfloat16), ops.pack_weight(w.to(DEV), torch.bfloat16, 1), C, H, W, 3, 3, 1, 1,
                   out=dx, accumulate=True)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, padding=1).backward(dy)
    assert rel_err(nchw(dx), base + xr.grad) < 3e-2


@pytest.mark.parametrize("dtype,C,Cp", [(torch.bfloat16, 32, 64), (torch.bfloat16, 16, 64), (torch.float32, 16, 32),
                                        (torch.bfloat16, 64, 128)])
def test_pad_channels(dtype, C, Cp):
    """scd_pad_channels: zero-extension of the innermost dimension (narrow-layer GEMM operands)."""
    from scdhip import ops
    x = torch.randn(37, 5, C, device=DEV).to(dtype)
    y = ops.pad_channels(x, C, Cp, 37 * 5)
    ref = F.pad(x.float(), (0, Cp - C)).reshape(-1, Cp)
    assert torch.equal(y.float(), ref)


@pytest.mark.parametrize("B,H,W", [(1, 1, 4), (2, 3, 12)])
def test_augment_tiny_tiles(B, H, W):
    from scdhip import ops
    x = torch.randn(B, 1, H, W)
    got = ops.augment_tiles(x.to(DEV)).cpu()
    for b in range(B):
        t = x[b].double()
        ref = ((t - t.mean()) / ((t - t.mean()) ** 2).mean().sqrt()).float()
        np.testing.assert_allclose(got[b].numpy(), ref.numpy(), rtol=0, atol=2e-5)


@pytest.mark.parametrize("ns,Cg,T,Ci,taps_fast", [(1, 64, 9, 64, True), (7, 64, 9, 64, True), (17, 64, 1, 64, True),
                                                  (56, 384, 9, 256, True), (200, 128, 9, 128, True),
                                                  (64, 8, 3, 4, True), (9, 32, 16, 260, True), (5, 24, 9, 132, False)])
def test_wgrad_reduce_rows(ns, Cg, T, Ci, taps_fast):
    """scd_wgrad_reduce_rows (split-slab sum into 1..4 row slices, per (row, 128-channel chunk) workgroup, written in
    the destination's order: OIHW with taps fastest, or a [tap][channel] layout) against a float64 sum of the same
    slabs: fp32 accumulation of ns terms, 1e-5 relative; ragged channel chunks (260 = 2 x 128 + 4)."""
    from scdhip import lib as L
    from scdhip.ops import ptr, stream
    g = torch.Generator().manual_seed(ns * 1000 + Cg)
    ws = torch.randn(ns, Cg, T * Ci, generator=g)
    ref = ws.double().sum(0)                      # (Cg, T*Ci), column = t*Ci + ci
    wsd = ws.to(DEV)
    cuts = sorted({0, Cg // 3 // 4 * 4, Cg // 2, Cg})
    slices = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    cvalid = Ci - 1 if Ci > 4 else Ci
    alpha = 0.5
    if taps_fast:
        dst = [torch.randn(b - a, Ci, T, generator=g).to(DEV) for a, b in slices]   # OIHW-flattened rows
    else:
        dst = [torch.randn(b - a, T, Ci, generator=g).to(DEV) for a, b in slices]   # [row][tap][channel]
    ldc, ldt = (T, 1) if taps_fast else (1, Ci)
    before = [d.clone() for d in dst]
    for accumulate in (1, 0):
        d_in = [d.clone() for d in before]
        wsd = ws.to(DEV)
        L.call("scd_wgrad_reduce_rows", ptr(wsd), ns, Cg, T, Ci, len(slices),
               L.int_array([a for a, _ in slices]), L.int_array([b for _, b in slices]),
               L.long_array([Ci * T] * len(slices)), L.long_array([ldc] * len(slices)),
               L.long_array([ldt] * len(slices)), L.ptr_array([ptr(d) for d in d_in]), cvalid, accumulate, alpha,
               stream())
        torch.cuda.synchronize()
        for (a, b), d, d0 in zip(slices, d_in, before):
            exp = ref[a:b].view(b - a, T, Ci).permute(0, 2, 1) * alpha      # (rows, Ci, T)
            if not taps_fast:
                d, d0 = d.permute(0, 2, 1), d0.permute(0, 2, 1)
            want = d0.cpu().double().clone()
            want[:, :cvalid] = exp[:, :cvalid] + (want[:, :cvalid] if accumulate else 0)
            err = (d.cpu().double() - want).abs().max().item() / max(1e-6, want.abs().max().item())
            assert err < 1e-5, (a, b, accumulate, err)


@pytest.mark.parametrize("dtype,C", [(torch.bfloat16, 128), (torch.bfloat16, 512), (torch.float32, 64)])
def test_bn_backward_pair_matches_two_passes(dtype, C):
    """Residual join out = relu(bn_a(y_a) + bn_b(y_b)) (BasicBlock bn2 + downsample BN, residuals.py:110-120; CornerPool
    merge + shortcut): scd_bn_bwd_reduce2 / scd_bn_bwd_apply2 against two scd_bn_bwd_reduce / scd_bn_bwd_apply passes
    with the same dout and mask -- BN parameter gradients to fp64-summation-order level (1e-6), input gradients equal
    up to one rounding of the 16-bit output where a coefficient differs in its last float bit."""
    from scdhip import ops
    g = torch.Generator().manual_seed(C)
    N, H, W = 4, 32, 32
    ya = torch.randn(N, H, W, C, generator=g).to(DEV, dtype)
    yb = (torch.randn(N, H, W, C, generator=g) * 2 + 0.5).to(DEV, dtype)
    dout = torch.randn(N, H, W, C, generator=g).to(DEV, dtype)
    res = {}
    for pair in (False, True):
        bns = [torch.nn.BatchNorm2d(C).to(DEV) for _ in range(2)]
        sts = []
        for bn, y in zip(bns, (ya, yb)):
            with torch.no_grad():
                bn.weight.copy_(torch.linspace(0.5, 1.5, C))
                bn.bias.copy_(torch.linspace(-0.3, 0.3, C))
            stats = ops.new_stats(C, DEV)
            # the forward statistics of y (as the producing GEMM epilogue would accumulate them)
            yd = y.double().reshape(-1, C)
            stats[:C] = yd.sum(0)
            stats[C:2 * C] = (yd * yd).sum(0)
            sts.append(ops.bn_finalize(bn, stats, C, yd.shape[0]))
        out = torch.relu(ya.float() * sts[0].scale + sts[0].shift + yb.float() * sts[1].scale + sts[1].shift).to(dtype)
        old = ops.BNPair.enabled
        ops.BNPair.enabled = pair
        try:
            dya, dyb = ops.bn_backward_pair(bns[0], sts[0], ya, bns[1], sts[1], yb, dout, out)
        finally:
            ops.BNPair.enabled = old
        torch.cuda.synchronize()
        res[pair] = (dya.float(), dyb.float(), [t.grad.clone() for bn in bns for t in (bn.weight, bn.bias)])
    (a0, b0, g0), (a1, b1, g1) = res[False], res[True]
    for x, y in zip(g0, g1):
        assert rel_err(y, x) < 1e-6
    ulp = 2.0 ** -7 if dtype == torch.bfloat16 else 1e-6
    for x, y in ((a0, a1), (b0, b1)):
        d = (x - y).abs()
        assert (d <= ulp * x.abs().clamp_min(1e-3) + 1e-6).all(), d.max().item()
        if dtype != torch.float32:      # fp32 shows every last-bit coefficient difference; 16-bit rounding hides most
            assert (d > 0).float().mean().item() < 1e-3


@pytest.mark.gpu
def test_raw_stream_handle_follows_torch_current_stream():
    """ops.stream() (the raw-handle fast path every launch uses) names torch's current stream, inside and outside a
    stream context."""
    from scdhip import ops
    assert ops.stream() == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert ops.stream() == s.cuda_stream == torch.cuda.current_stream().cuda_stream
    assert ops.stream() == torch.cuda.current_stream().cuda_stream


def _bnst(C, g):
    class St:
        pass
    st = St()
    st.mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
    st.invstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    st.scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
    st.shift = (torch.randn(C, generator=g) * 0.2).to(DEV)
    return st


@pytest.mark.parametrize("case", ["fwd_stats", "fwd_bias_relu_384", "fwd_ragged", "heads_dgrad_bnbwd", "dgrad_accum",
                                  "deconv_fwd_stats", "deconv_dgrad_bnbwd", "dgrad_s2"])
def test_duo_matches_pingpong(case, monkeypatch):
    """conv_gemm_duo_kernel (two 4-wave 256 x 128 workgroups per CU, BK = 32 K-steps in a 3-slot ring, round 6) against
    the ping-pong kernel on the shapes it replaces: its K order (64-channel chunk, tap, 32-channel half) gives every
    output the ping-pong kernel's MFMA sequence, so outputs are bit-identical; BN statistics / backward sums agree to
    fp64 summation-order noise (the tiles' fp32 partials are the same, their replica slots differ).  SCD_GEMM_DUO=1
    routes the ping-pong shapes to it (read per call)."""
    from scdhip import ops
    g = torch.Generator().manual_seed(29)
    bf = torch.bfloat16
    st = _bnst(256, g)

    def run():
        r = {}
        if case == "fwd_stats":               # 3x3 256 -> 256 with BN statistics (layer4-like, 4 x 128^2 pixels)
            x = nhwc(torch.randn(4, 256, 128, 128, generator=g), bf)
            w = (torch.randn(256, 256, 3, 3, generator=g) / 48).to(DEV)
            stats = torch.zeros(64 * 2 * 256, dtype=torch.float64, device=DEV)
            r["y"] = ops.conv_fwd(x, ops.pack_weight(w, bf, 0), 256, 3, 3, 1, 1, stats=stats)
            r["stats"] = stats.view(64, 2, 256).sum(0)
        elif case == "fwd_bias_relu_384":      # the heads' N = 384 without tails, bias + ReLU
            x = nhwc(torch.randn(4, 256, 128, 128, generator=g), bf)
            w = (torch.randn(384, 256, 3, 3, generator=g) / 48).to(DEV)
            b = torch.randn(384, generator=g).to(DEV)
            r["y"] = ops.conv_fwd(x, ops.pack_weight(w, bf, 0), 384, 3, 3, 1, 1, bias=b, relu=True)
        elif case == "fwd_ragged":             # M = 5 x 127^2 (not a multiple of 256), stride 2 input
            x = nhwc(torch.randn(5, 128, 254, 254, generator=g), bf)
            w = (torch.randn(256, 128, 3, 3, generator=g) / 34).to(DEV)
            stats = torch.zeros(64 * 2 * 256, dtype=torch.float64, device=DEV)
            r["y"] = ops.conv_fwd(x, ops.pack_weight(w, bf, 0), 256, 3, 3, 2, 1, stats=stats)
            r["stats"] = stats.view(64, 2, 256).sum(0)
        elif case == "heads_dgrad_bnbwd":      # dhid (128 ch) -> dfeat (256 ch), 3x3, with the next BN's backward sums
            dy = nhwc(torch.randn(4, 128, 128, 128, generator=g), bf)
            w = (torch.randn(128, 256, 3, 3, generator=g) / 30).to(DEV)
            y = nhwc(torch.randn(4, 256, 128, 128, generator=g), bf)
            bst = torch.zeros(64 * 2 * 256, dtype=torch.float64, device=DEV)
            r["dx"] = ops.conv_dgrad(dy, ops.pack_weight(w, bf, 1), 256, 128, 128, 3, 3, 1, 1, bn_bwd=(st, y, bst))
            r["bsums"] = bst.view(64, 2, 256).sum(0)
        elif case == "dgrad_accum":
            dy = nhwc(torch.randn(4, 256, 128, 128, generator=g), bf)
            w = (torch.randn(256, 256, 3, 3, generator=g) / 48).to(DEV)
            base = nhwc(torch.randn(4, 256, 128, 128, generator=g), bf)
            r["dx+"] = base.clone()
            ops.conv_dgrad(dy, ops.pack_weight(w, bf, 1), 256, 128, 128, 3, 3, 1, 1, out=r["dx+"], accumulate=True)
        elif case == "deconv_fwd_stats":       # ConvTranspose2d(256, 256, 4, 2, 1): 4 sub-pixel phases
            x = nhwc(torch.randn(4, 256, 64, 64, generator=g), bf)
            w = (torch.randn(256, 256, 4, 4, generator=g) / 60).to(DEV)
            stats = torch.zeros(64 * 2 * 256, dtype=torch.float64, device=DEV)
            r["y"] = ops.deconv_fwd(x, ops.pack_weight(w, bf, 1), 256, stats=stats)
            r["stats"] = stats.view(64, 2, 256).sum(0)
        elif case == "deconv_dgrad_bnbwd":     # its input gradient (16 taps, stride 2) with the BN-backward sums
            dy = nhwc(torch.randn(16, 256, 128, 128, generator=g), bf)
            w = (torch.randn(256, 256, 4, 4, generator=g) / 60).to(DEV)
            y = nhwc(torch.randn(16, 256, 64, 64, generator=g), bf)
            bst = torch.zeros(64 * 2 * 256, dtype=torch.float64, device=DEV)
            r["dx"] = ops.deconv_dgrad(dy, ops.pack_weight(w, bf, 0), 256, 4, 2, 1, bn_bwd=(st, y, bst))
            r["bsums"] = bst.view(64, 2, 256).sum(0)
        else:                                  # 3x3 / stride 2 input gradient as one GEMM with phase columns (shuf)
            dy = nhwc(torch.randn(32, 256, 32, 32, generator=g), bf)
            w = torch.randn(256, 128, 3, 3, generator=g).to(DEV) / 34
            r["dx"] = ops.conv_dgrad_w(dy, w, 64, 64, 2, 1)
        torch.cuda.synchronize()
        return r

    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SCD_GEMM_DUO", mode)
        g.manual_seed(29)
        st = _bnst(256, g)
        outs[mode] = run()
    for k, v in outs["0"].items():
        if k in ("stats", "bsums"):
            d = (outs["1"][k] - v).abs().max().item()
            assert d <= 1e-9 * max(v.abs().max().item(), 1.0), (k, d)
        else:
            assert torch.equal(outs["1"][k], v), (k, (outs["1"][k].float() - v.float()).abs().max().item())
