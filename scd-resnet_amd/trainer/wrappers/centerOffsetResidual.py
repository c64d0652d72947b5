"""Inference wrapper (trainer/wrappers/centerOffsetResidual.py:4-23 of the reference).

Output: one (10, B, K) float32 tensor, rows in the order slide.py / test.py unpack them --
scores, inds, ys, xs, major-axis x, major-axis y, minor length, halo radius, offset x, offset y (the integer rows
are promoted to float32, as the reference's torch.stack does).  The decode underneath is scd_decode_topk
(models/centerNetOffset.decodeCenterNet)."""
import torch

# (position in the decode list, column of that tensor or None for a (B, K) row)
_ROWS = ((0, None), (1, None), (2, None), (3, None), (5, 0), (5, 1), (5, 2), (5, 3), (4, 0), (4, 1))


class Wrapper(torch.nn.Module):
    """model(inp, decode=True) -> stacked detections; `model` is any CenterNet plugin model."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, inp):
        dec = self.model(inp, decode=True)       # [scores, inds, ys, xs, offset, regr, outputDict]
        picked = [dec[i] if col is None else dec[i][..., col] for i, col in _ROWS]
        return torch.stack([t.to(torch.float32) for t in picked], 0)
