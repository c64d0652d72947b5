"""Synthetic corner dataset plugin for CornerNet (config 4).  The reference ships no dataset
with corner targets (cornerNetCPool.py:43 imports a module that does not exist); its loss reads
ys[0] = centre heatmap, ys[3] = top-left heatmap, ys[4] = bottom-right heatmap
(cornerNetCPool.py:244-272).  Samples come from syntheticSCD; the corner of each object is its
centre -/+ (round |major_x|, round minor) clipped to the map, rendered with the same Gaussian
rule as the centre (tests/golden/make_golden_corner.py:corner_targets builds F8 the same way).

  __getitem__ -> {"xs": [tile (1,512,512) f32], "ys": [heat, mask (30,), regr (30,6), tl, br]}
"""
import numpy as np
import torch

from trainer.dataset.syntheticSCD import HEATMAPSIZE, SCD, encode_targets


def corner_locs(locs, size=HEATMAPSIZE):
    tl, br = locs.copy(), locs.copy()
    dx = np.round(np.abs(locs[:, 4])).astype(np.float32)
    dy = np.round(locs[:, 6]).astype(np.float32)
    tl[:, 0] = np.clip(locs[:, 0] - dx, 0, size - 1)
    tl[:, 1] = np.clip(locs[:, 1] - dy, 0, size - 1)
    br[:, 0] = np.clip(locs[:, 0] + dx, 0, size - 1)
    br[:, 1] = np.clip(locs[:, 1] + dy, 0, size - 1)
    return tl, br


class CornerSCD(SCD):
    def item(self, index, base):
        tile, locs, ys = super().item(index, base)
        tl, br = corner_locs(locs, self.heat)
        return tile, locs, ys[:3] + [torch.from_numpy(encode_targets(tl, self.heat)[0]),
                                     torch.from_numpy(encode_targets(br, self.heat)[0])]

    def getValidationSet(self, batch=None):
        from configuration import defaultConfig
        from trainer.dataset.syntheticSCD import VALID_SAMPLES
        batch = batch or min(VALID_SAMPLES, defaultConfig.validationBatchSize)
        out = []
        for b0 in range(0, VALID_SAMPLES, batch):
            items = [self.item(i, self.seed + 7919 * 1000003) for i in range(b0, min(VALID_SAMPLES, b0 + batch))]
            out.append({"xs": [torch.stack([it[0] for it in items])],
                        "ys": [torch.stack([it[2][k] for it in items]) for k in range(5)]})
        return out


dataset = CornerSCD
