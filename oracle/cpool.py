"""Corner pooling restatement (TEST INFRASTRUCTURE ONLY).

models/backbones/cornerPooling/source/topPool.cpp:5-31 (forward) and :33-74 (backward), and the
bottom/left/right siblings: NCHW fp32 on CPU.  dir 0 top (max over k>=h), 1 bottom (k<=h),
2 left (k>=w), 3 right (k<=w).  Backward routes dy[h] to the running argmax of the scan that
starts at the far end; the argmax moves only on a strict '>' (topPool.cpp:61-65), so ties keep
the first-scanned position.
"""
import torch


def _scan_dim_rev(direction):
    dim = 2 if direction in (0, 1) else 3
    reverse = direction in (0, 2)
    return dim, reverse


def forward(x, direction):
    dim, reverse = _scan_dim_rev(direction)
    t = x.flip(dim) if reverse else x
    out = torch.cummax(t, dim=dim).values
    return out.flip(dim) if reverse else out


def backward(x, dy, direction):
    dim, reverse = _scan_dim_rev(direction)
    xs = x.flip(dim) if reverse else x
    gs = dy.flip(dim) if reverse else dy
    xs = xs.movedim(dim, -1)
    gs = gs.movedim(dim, -1)
    L = xs.shape[-1]
    out = torch.zeros_like(xs)
    maxv = xs[..., 0].clone()
    maxi = torch.zeros(xs.shape[:-1], dtype=torch.long)
    for k in range(L):
        if k > 0:
            gt = xs[..., k] > maxv
            maxv = torch.where(gt, xs[..., k], maxv)
            maxi = torch.where(gt, torch.full_like(maxi, k), maxi)
        out.scatter_add_(-1, maxi.unsqueeze(-1), gs[..., k:k + 1])
    out = out.movedim(-1, dim)
    return out.flip(dim) if reverse else out
