"""CPU restatement of the reference's CenterNet validation metrics -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the product
path (scdhip.ops.center_eval / center_eval_summary -> libscdhip) never does.

Follows:
  models/centerNetOffset.py:253-354      centerNetEvaluation (boxes, validMask = score >= 0.3)
  evaluations/detection.py:11-46         IoU
  evaluations/detection.py:52-97         Orthogonity
  evaluations/detection.py:101-146       MAE
  evaluations/detection.py:149-180       IoUConfidence
  evaluations/detection.py:183-230       averagePrecisionPlots / averagePrecisionAll
  trainer/model/centerOffsetRes10.py:18-106   expression (means, AP30/50/70/90)
numpy float32 arithmetic, one rounding per torch op as in the reference; square roots go through torch.sqrt
(the reference's own CPU kernel: it is not always correctly rounded -- e.g. sqrt(12.603475570678711f) --
so numpy's sqrt would not reproduce the reference bit for bit).  Pinned by tests/golden/eval.npz
(tests/golden/make_golden_eval.py runs the reference functions on the same seeded inputs).
"""
import numpy as np
import torch

from . import targets as T

F = np.float32
EPS = F(1e-5)
STREAMS = ("iou", "score", "ortho", "ioucenter", "iouoffsetwo", "iouoffset", "aemaj", "aemin", "aerad")


def _sqrt(x):
    return torch.sqrt(torch.from_numpy(np.ascontiguousarray(x, F))).numpy()


def _boxes_det(ctY, ctX, offset, regr):
    ml = _sqrt(regr[:, :, 0] * regr[:, :, 0] + regr[:, :, 1] * regr[:, :, 1])
    o0, o1 = offset[:, :, 0] / F(4), offset[:, :, 1] / F(4)
    fx, fy = ctX.astype(F), ctY.astype(F)
    b = np.stack([(fx - ml) + o0, (fy - regr[:, :, 2]) + o1, (fx + ml) + o0, (fy + regr[:, :, 2]) + o1], -1)
    c = np.stack([(ctX - 2), (ctY - 2), (ctX + 2), (ctY + 2)], -1).astype(F)
    o = np.stack([c[..., 0] + o0, c[..., 1] + o1, c[..., 2] + o0, c[..., 3] + o1], -1)
    return b, c, o, ml


def _boxes_gt(ys2, ys3, H):
    if ys3.ndim == 2:
        cy = ys3 // H
        cx = ys3 - (ys3 // H) * H
        c = np.stack([cx - 2, cy - 2, cx + 2, cy + 2], -1).astype(F)
        cx, cy = cx.astype(F), cy.astype(F)
    else:
        cx, cy = ys3[:, :, 0].astype(F), ys3[:, :, 1].astype(F)
        c = np.stack([cx - F(2), cy - F(2), cx + F(2), cy + F(2)], -1)
    ml = _sqrt(ys2[:, :, 2] * ys2[:, :, 2] + ys2[:, :, 3] * ys2[:, :, 3])
    o0, o1 = ys2[:, :, 0] / F(4), ys2[:, :, 1] / F(4)
    b = np.stack([(cx - ml) + o0, (cy - ys2[:, :, 4]) + o1, (cx + ml) + o0, (cy + ys2[:, :, 4]) + o1], -1)
    o = np.stack([c[..., 0] + o0, c[..., 1] + o1, c[..., 2] + o0, c[..., 3] + o1], -1)
    return b, c, o, ml


def _pairs(d, g, valid):
    """(N,K,4) x (N,L,4) -> mask, iou (N,K,L) (detection.py:27-46)."""
    d = d[:, :, None, :]
    g = g[:, None, :, :]
    darea = (d[..., 2] - d[..., 0]) * (d[..., 3] - d[..., 1])
    garea = (g[..., 2] - g[..., 0]) * (g[..., 3] - g[..., 1])
    dx = np.minimum(d[..., 2], g[..., 2]) - np.maximum(d[..., 0], g[..., 0])
    dy = np.minimum(d[..., 3], g[..., 3]) - np.maximum(d[..., 1], g[..., 1])
    mask = (dx > EPS) & (dy > EPS) & (garea > EPS) & valid[:, :, None]
    inter = dx * dy
    with np.errstate(divide="ignore", invalid="ignore"):
        iou = inter / ((darea + garea) - inter)
    return mask, iou


def center_eval(scores, ctY, ctX, offset, regr, ys2, ys3, H=128, thr=0.3):
    """The nine masked_select streams of centerNetEvaluation, in STREAMS order (float32 arrays)."""
    scores, offset, regr, ys2 = (np.asarray(a, F) for a in (scores, offset, regr, ys2))
    ctY, ctX = np.asarray(ctY, np.int64), np.asarray(ctX, np.int64)
    ys3 = np.asarray(ys3)
    ys3 = ys3.astype(np.int64) if ys3.ndim == 2 else ys3.astype(F)
    db, dc, do, dml = _boxes_det(ctY, ctX, offset, regr)
    gb, gc, go, gml = _boxes_gt(ys2, ys3, H)
    valid = scores >= F(thr)
    mb, iou_b = _pairs(db, gb, valid)
    mb2 = mb & (gml[:, None, :] > EPS)
    mcc, iou_cc = _pairs(dc, gc, valid)
    mco, iou_co = _pairs(dc, go, valid)
    moo, iou_oo = _pairs(do, go, valid)
    N, K = scores.shape
    L = ys2.shape[1]
    with np.errstate(divide="ignore", invalid="ignore"):
        cs = ((regr[:, :, None, 0] * ys2[:, None, :, 2]) + (regr[:, :, None, 1] * ys2[:, None, :, 3])) / \
             (dml[:, :, None] * gml[:, None, :])
        sn = _sqrt(F(1) - cs * cs)
    sc = np.broadcast_to(scores[:, :, None], (N, K, L))
    aemaj = np.abs(dml[:, :, None] - gml[:, None, :])
    aemin = np.abs(regr[:, :, None, 2] - ys2[:, None, :, 4])
    aerad = np.abs(regr[:, :, None, 3] - ys2[:, None, :, 5])
    pick = [(iou_b, mb), (sc, mb), (sn, mb2), (iou_cc, mcc), (iou_co, mco), (iou_oo, moo), (aemaj, mb2),
            (aemin, mb2), (aerad, mb2)]
    return [np.ascontiguousarray(v[m]).astype(F) for v, m in pick]


def ap_plots(ious, scores, objnum, threshold, ties="desc"):
    """averagePrecisionPlots (detection.py:183-206) with an explicit tie rule: the reference sorts with
    torch.sort (unstable on CPU above 16 elements) then flips; 'desc' = ties by descending index (what a
    stable sort + flip gives, and what the GPU kernel does), 'asc' = ascending."""
    ious = np.asarray(ious, F)
    scores = np.asarray(scores, F)
    idx = np.arange(len(scores))
    order = np.lexsort((-idx if ties == "desc" else idx, -scores.astype(np.float64)))
    plots = []
    tp = fp = 0
    for i in order:
        if ious[i] < F(threshold):
            fp += 1
        else:
            tp += 1
        plots.append([tp / objnum, tp / (tp + fp)])
    return plots


def ap_all(plots):
    """averagePrecisionAll (detection.py:208-230), verbatim arithmetic in Python floats."""
    x1 = x2 = 1
    y = 0
    ap = 0
    for recall, precision in reversed(plots):
        if precision > y:
            ap += (x2 - x1) * y
            x2 = recall
            x1 = recall
            y = precision
        else:
            x1 = recall
    ap += x2 * y
    return ap


def summary(streams, objnum, thresholds=(0.3, 0.5, 0.7, 0.9), ties="desc"):
    """expression()'s numbers (centerOffsetRes10.py:62-88): means of the nine streams (orthogonity over its
    non-NaN values; 0 for an empty stream) and AP at each threshold."""
    means = []
    for s, v in zip(STREAMS, streams):
        v = np.asarray(v, np.float64)
        if s == "ortho":
            v = v[~np.isnan(v)]
        means.append(float(v.mean()) if len(v) else 0.0)
    n = max(int(objnum), len(streams[0]))
    aps = [ap_all(ap_plots(streams[0], streams[1], n, t, ties)) for t in thresholds]
    return means, aps


def eval_case(seed, N=4, K=100, L=30, H=128, n_near=12):
    """Seeded decoded-detection / ground-truth batch: targets from oracle.targets.random_locs; the first
    n_near detections of each image sit on ground-truth objects with jittered centre / axes / offsets, the
    rest are random.  Scores are distinct (a random permutation of a grid), some below the 0.3 threshold."""
    rs = np.random.RandomState(seed)
    ys2 = np.zeros((N, L, 6), F)
    locs8 = np.zeros((N, L, 8), F)
    inds = np.zeros((N, L), np.int64)
    mask = np.zeros((N, L), bool)
    for n in range(N):
        locs = T.random_locs(rs, size=H)[:L]
        m = len(locs)
        locs8[n, :m] = locs
        locs8[n, :m, :2] = np.floor(locs[:, :2])
        ys2[n, :m] = locs[:, 2:8]
        inds[n, :m] = (np.floor(locs[:, 1]) * H + np.floor(locs[:, 0])).astype(np.int64)
        mask[n, :m] = True
    ctX = rs.randint(0, H, (N, K)).astype(np.int64)
    ctY = rs.randint(0, H, (N, K)).astype(np.int64)
    regr = np.concatenate([rs.uniform(-6, 6, (N, K, 2)), rs.uniform(0.5, 4, (N, K, 2))], -1).astype(F)
    offset = rs.uniform(0, 4, (N, K, 2)).astype(F)
    for n in range(N):
        m = int(mask[n].sum())
        for k in range(min(n_near, m)):
            j = rs.randint(0, m)
            ctX[n, k] = np.clip(locs8[n, j, 0] + rs.randint(-1, 2), 0, H - 1)
            ctY[n, k] = np.clip(locs8[n, j, 1] + rs.randint(-1, 2), 0, H - 1)
            a = rs.uniform(-0.3, 0.3)   # never exactly parallel: orthogonity at cos = 1 is a knife edge (NaN or 0)
            ca, sa = np.cos(a), np.sin(a)
            mx, my = float(ys2[n, j, 2]), float(ys2[n, j, 3])
            regr[n, k, :2] = np.array([ca * mx - sa * my, sa * mx + ca * my]) * rs.uniform(0.7, 1.3)
            regr[n, k, 2] = ys2[n, j, 4] * F(rs.uniform(0.7, 1.3))
            regr[n, k, 3] = ys2[n, j, 5] + F(rs.uniform(-0.5, 0.5))
            offset[n, k] = ys2[n, j, :2] + rs.uniform(-0.5, 0.5, 2).astype(F)
    scores = (rs.permutation(N * K).reshape(N, K).astype(np.float64) / (N * K)).astype(F)
    scores[:, :n_near] = F(0.35) + F(0.6) * scores[:, :n_near]
    return dict(scores=scores, ctY=ctY, ctX=ctX, offset=offset, regr=regr, ys2=ys2, inds=inds, locs=locs8,
                mask=mask)
