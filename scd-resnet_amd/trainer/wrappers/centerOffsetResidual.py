"""Inference wrapper (trainer/wrappers/centerOffsetResidual.py:4-23 of the reference): the decoded detections
as one (10, B, K) tensor, rows [scores, inds, ys, xs, majx, majy, minl, halo, offx, offy] (torch.stack promotes
the integer rows to float32).  The decode itself is scd_decode_topk (models/centerNetOffset.decodeCenterNet)."""
import torch
import torch.nn


class Wrapper(torch.nn.Module):

    def __init__(self, model):
        super(Wrapper, self).__init__()
        self.model = model

    def forward(self, inp):
        scores, inds, ys, xs, offset, regression, _ = self.model(inp, decode=True)
        rows = [scores, inds, ys, xs] + [regression[:, :, i] for i in range(4)] + [offset[:, :, 0], offset[:, :, 1]]
        return torch.stack([r.float() for r in rows])
