"""Synthetic SCD dataset plugin (the real presets trainer/dataset/scdx*.py need `.d` archives
that are not distributed).  Same constructor and sample format as datasets/scds/scdx16p100.py:
  __getitem__ -> {"xs": [tile (1,512,512) f32], "ys": [heat (1,128,128) f32, mask (30,) bool,
                                                       regr (30,6) f32, inds (30,) i64]}   (:376-379)
  getValidationSet() -> [{"xs": [tiles], "ys": [heat, mask, regr, locs (b,30,8), objnum, inds]}]  (:381-414)
Tiles are N(0,1) (the post-`normalize` distribution); 5-20 objects per tile; heatmaps are
rendered with the reference's Gaussian radius / splat rules (intersection.py:46-63,
scdx16p100.py:575-591).  Everything is a deterministic function of (seed, index).
"""
import math

import numpy as np
import torch
from torch.utils.data import Dataset

MAXTAGLEN = 30
TARGETSIZE = 512
HEATMAPSIZE = 128
THRESHOLDIOU = 0.5
TRAIN_SAMPLES = 1024
VALID_SAMPLES = 64


def gaussian_radius(width, height, threshold):
    """Smallest of the three quadratic-root radii keeping IoU >= threshold (intersection.py:46-63);
    evaluated in the reference's operation order so the rendered maps match bit for bit."""
    roots = []
    for a, b, c in ((1, height + width, width * height * (1 - threshold) / (1 + threshold)),
                    (4, 2 * (height + width), (1 - threshold) * width * height),
                    (4 * threshold, -2 * threshold * (height + width), (threshold - 1) * width * height)):
        roots.append((b + np.sqrt(b ** 2 - 4 * a * c)) / 2)
    return min(roots)


def splat(heat, x, y, radius):
    """Add exp(-d^2 / (2 (r/3)^2)) over a (2*ceil(2r)+1)^2 window clipped at the border, then clip at 1."""
    h, w = heat.shape
    roi = math.ceil(radius * 2)
    left, right = min(roi, x), min(roi, w - x - 1)
    top, bottom = min(roi, y), min(roi, h - y - 1)
    sigma = radius / 3
    dy = np.arange(-top, bottom + 1, dtype=np.float64)[:, None]
    dx = np.arange(-left, right + 1, dtype=np.float64)[None, :]
    win = heat[y - top:y + bottom + 1, x - left:x + right + 1]
    heat[y - top:y + bottom + 1, x - left:x + right + 1] = (np.exp(-(dx * dx + dy * dy) / (2 * sigma * sigma))
                                                            + win.astype(np.float64)).astype(np.float32)
    np.minimum(heat, 1, out=heat)


def sample_objects(rs, size=HEATMAPSIZE):
    """[ctx, cty, offx, offy, majx, majy, minl, halo] rows, 5-20 objects."""
    n = int(rs.randint(5, 21))
    locs = np.zeros((n, 8), dtype=np.float32)
    locs[:, 0] = rs.randint(0, size, n)
    locs[:, 1] = rs.randint(0, size, n)
    locs[:, 2:4] = rs.uniform(0, 4, (n, 2))
    length, ang = rs.uniform(2, 6, n), rs.uniform(0, np.pi, n)
    locs[:, 4], locs[:, 5] = length * np.cos(ang), length * np.sin(ang)
    locs[:, 6] = rs.uniform(1, 3, n)
    locs[:, 7] = locs[:, 6] + rs.uniform(0, 4, n)
    return locs


def encode_targets(locs, size=HEATMAPSIZE):
    heat = np.zeros((size, size), dtype=np.float32)
    mask = np.zeros(MAXTAGLEN, dtype=bool)
    inds = np.zeros(MAXTAGLEN, dtype=np.int64)
    regr = np.zeros((MAXTAGLEN, 6), dtype=np.float32)
    for i, loc in enumerate(locs[:MAXTAGLEN]):
        x, y = int(loc[0]), int(loc[1])
        inside = 0 <= x < size and 0 <= y < size
        if inside:
            major2 = np.float32(np.float32(loc[4]) ** 2 + np.float32(loc[5]) ** 2)
            splat(heat, x, y, gaussian_radius(2 * math.sqrt(float(major2)), 2 * float(loc[6]), THRESHOLDIOU))
            inds[i] = int(math.floor(loc[1])) * size + int(math.floor(loc[0]))
        mask[i] = inside
        regr[i] = loc[2:8]
    return heat[None], mask, regr, inds


class SCD(Dataset):
    def __init__(self, zipPath, useGPU, dataSplit=None, seed=1234, count=TRAIN_SAMPLES,
                 size=TARGETSIZE, heat=HEATMAPSIZE):
        self.zipPath, self.useGPU, self.seed = zipPath, useGPU, seed
        self.count, self.size, self.heat = count, size, heat

    def __len__(self):
        return self.count

    def item(self, index, base):
        rs = np.random.RandomState((base + index) & 0x7FFFFFFF)
        locs = sample_objects(rs, self.heat)
        tile = torch.from_numpy(rs.standard_normal((1, self.size, self.size)).astype(np.float32))
        heat, mask, regr, inds = encode_targets(locs, self.heat)
        return tile, locs, [torch.from_numpy(heat), torch.from_numpy(mask), torch.from_numpy(regr),
                            torch.from_numpy(inds)]

    def __getitem__(self, index):
        tile, _, ys = self.item(index, self.seed)
        return {"xs": [tile], "ys": ys}

    def gpu_batch(self, indices, device):
        """A training batch with its targets rendered on the GPU (scdhip.ops.render_center_targets, one launch
        for the whole batch) instead of per sample on the host: {"xs": [(B,1,S,S)], "ys": [heat, mask, regr,
        inds]} on `device`, equal to stacking __getitem__(i) for i in indices (tests/test_targets_gpu.py)."""
        from scdhip import ops
        tiles, locs = [], np.zeros((len(indices), MAXTAGLEN, 8), dtype=np.float32)
        counts = np.zeros(len(indices), dtype=np.int32)
        for b, i in enumerate(indices):
            rs = np.random.RandomState((self.seed + i) & 0x7FFFFFFF)
            objs = sample_objects(rs, self.heat)
            tiles.append(torch.from_numpy(rs.standard_normal((1, self.size, self.size)).astype(np.float32)))
            n = min(len(objs), MAXTAGLEN)
            locs[b, :n] = objs[:n]
            counts[b] = n
        ys = ops.render_center_targets(torch.from_numpy(locs).to(device), torch.from_numpy(counts).to(device),
                                       self.heat, THRESHOLDIOU)
        return {"xs": [torch.stack(tiles).to(device)], "ys": ys}

    def getValidationSet(self, batch=None):
        from configuration import defaultConfig
        batch = batch or min(VALID_SAMPLES, defaultConfig.validationBatchSize)
        out = []
        for b0 in range(0, VALID_SAMPLES, batch):
            items = [self.item(i, self.seed + 7919 * 1000003) for i in range(b0, min(VALID_SAMPLES, b0 + batch))]
            locs = torch.zeros(len(items), MAXTAGLEN, 8)
            for j, (_, l, _) in enumerate(items):
                locs[j, :min(len(l), MAXTAGLEN)] = torch.from_numpy(l[:MAXTAGLEN])
            ys = [torch.stack([it[2][k] for it in items]) for k in range(4)]
            out.append({"xs": [torch.stack([it[0] for it in items])],
                        "ys": [ys[0], ys[1], ys[2], locs, [min(len(it[1]), MAXTAGLEN) for it in items], ys[3]]})
        return out


dataset = SCD
