"""Synthetic SCD targets, restating the reference target rendering (TEST INFRASTRUCTURE ONLY).

  * object parameters: SURVEY §8d synthetic distribution (5-20 objects/tile)
  * radius:   centerThresholdRadius           evaluations/intersection.py:46-63
  * splat:    SCD.drawGaussian                datasets/scds/scdx16p100.py:575-591
              gaussianMargin2D                datasets/utility.py:11-15
  * heat/mask/regr/inds packing               datasets/scds/scdx16p100.py:304-379, :514-531
"""
import math

import numpy as np
import torch

MAXTAGLEN = 30          # scdx16p100.py:45
HEATMAPSIZE = 128       # scdx16p100.py:49
THRESHOLDIOU = 0.5      # scdx16p100.py:52


def center_threshold_radius(width, height, threshold=0.7):
    """intersection.py:46-63 (float64, numpy sqrt)."""
    a1, b1 = 1, height + width
    c1 = width * height * (1 - threshold) / (1 + threshold)
    r1 = (b1 + np.sqrt(b1 ** 2 - 4 * a1 * c1)) / 2
    a2, b2 = 4, 2 * (height + width)
    c2 = (1 - threshold) * width * height
    r2 = (b2 + np.sqrt(b2 ** 2 - 4 * a2 * c2)) / 2
    a3, b3 = 4 * threshold, -2 * threshold * (height + width)
    c3 = (threshold - 1) * width * height
    r3 = (b3 + np.sqrt(b3 ** 2 - 4 * a3 * c3)) / 2
    return min(r1, r2, r3)


def draw_gaussian(x, y, heat, radius):
    """scdx16p100.py:575-591: float64 splat added onto the float32 map, clipped at 1."""
    roi = math.ceil(radius * 2)
    top = left = bottom = right = roi
    h, w = heat.shape
    if x - left < 0:
        left = x
    if x + right >= w:
        right = w - x - 1
    if y - top < 0:
        top = y
    if y + bottom >= h:
        bottom = h - y - 1
    sigma = radius / 3
    yy, xx = np.ogrid[-top:bottom + 1, -left:right + 1]
    g = np.exp(-(xx * xx + yy * yy) / (2 * sigma * sigma))
    region = heat[y - top:y + bottom + 1, x - left:x + right + 1]
    heat[y - top:y + bottom + 1, x - left:x + right + 1] = (g + region.astype(np.float64)).astype(np.float32)
    heat[heat > 1] = 1


def random_locs(rs, n_min=5, n_max=20, size=HEATMAPSIZE):
    """centres U{0..127}, offsets U[0,4), major axis length U[2,6) at a random
    angle, minor U[1,3), halo = minor + U[0,4).  Row = [ctx,cty,offx,offy,majx,majy,minl,halo]."""
    n = int(rs.randint(n_min, n_max + 1))
    locs = np.zeros((n, 8), dtype=np.float32)
    locs[:, 0] = rs.randint(0, size, n)
    locs[:, 1] = rs.randint(0, size, n)
    locs[:, 2:4] = rs.uniform(0, 4, (n, 2))
    length = rs.uniform(2, 6, n)
    ang = rs.uniform(0, np.pi, n)
    locs[:, 4] = length * np.cos(ang)
    locs[:, 5] = length * np.sin(ang)
    locs[:, 6] = rs.uniform(1, 3, n)
    locs[:, 7] = locs[:, 6] + rs.uniform(0, 4, n)
    return locs


def render(locs, size=HEATMAPSIZE):
    """argumentation heat rendering + __getitem__ packing (scdx16p100.py:514-531, :320-355).
    Returns heat (1,S,S) f32, mask (30,) bool, regr (30,6) f32, inds (30,) i64."""
    heat = np.zeros((size, size), dtype=np.float32)
    for loc in locs:
        x, y = int(loc[0]), int(loc[1])
        if x < 0 or x >= size or y < 0 or y >= size:
            continue
        maj2 = np.float32(loc[4]) * np.float32(loc[4]) + np.float32(loc[5]) * np.float32(loc[5])
        radius = center_threshold_radius(2 * math.sqrt(float(np.float32(maj2))), 2 * float(loc[6]), THRESHOLDIOU)
        draw_gaussian(x, y, heat, radius)
    n = min(len(locs), MAXTAGLEN)
    mask = np.zeros(MAXTAGLEN, dtype=bool)
    mask[:n] = True
    inds = np.zeros(MAXTAGLEN, dtype=np.int64)
    regr = np.zeros((MAXTAGLEN, 6), dtype=np.float32)
    for i in range(n):
        lx, ly = locs[i, 0], locs[i, 1]
        if lx < 0 or lx >= size or ly < 0 or ly >= size:
            mask[i] = False
        else:
            inds[i] = int(math.floor(ly)) * size + int(math.floor(lx))
        regr[i] = locs[i, 2:8]
    inds[~mask] = 0
    return heat[None], mask, regr, inds


def batch_targets(seed, batch, size=HEATMAPSIZE):
    """A seeded batch of targets: list [heat (B,1,S,S), mask (B,30), regr (B,30,6), inds (B,30)]."""
    rs = np.random.RandomState(seed)
    cols = [render(random_locs(rs, size=size), size) for _ in range(batch)]
    return [torch.from_numpy(np.stack([c[i] for c in cols])) for i in range(4)]


def batch_inputs(seed, batch, size=512):
    """N(0,1) fp32 tiles, (B,1,S,S) -- the post-`normalize` distribution (argumentations.py:40-44)."""
    rs = np.random.RandomState(seed)
    return torch.from_numpy(rs.standard_normal((batch, 1, size, size)).astype(np.float32))


def corner_targets(seed, batch, size=HEATMAPSIZE):
    """[heat, mask, regr, tl, br] for CornerNetLoss (ys[0], ys[3], ys[4]; cornerNetCPool.py:252-254).
    The reference has no corner target encoder; the rule used for F8 and the synthetic corner
    dataset: corners at centre -/+ (round |major_x|, round minor), clipped, Gaussian as the centre."""
    rs = np.random.RandomState(seed)
    cols = []
    for _ in range(batch):
        locs = random_locs(rs, size=size)
        h, m, rg, _ = render(locs, size)
        tl, br = locs.copy(), locs.copy()
        dx = np.round(np.abs(locs[:, 4])).astype(np.float32)
        dy = np.round(locs[:, 6]).astype(np.float32)
        tl[:, 0] = np.clip(locs[:, 0] - dx, 0, size - 1)
        tl[:, 1] = np.clip(locs[:, 1] - dy, 0, size - 1)
        br[:, 0] = np.clip(locs[:, 0] + dx, 0, size - 1)
        br[:, 1] = np.clip(locs[:, 1] + dy, 0, size - 1)
        cols.append((h, m, rg, render(tl, size)[0], render(br, size)[0]))
    return [torch.from_numpy(np.stack([c[i] for c in cols])) for i in range(5)]
