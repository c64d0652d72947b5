"""Golden fixture for the validation metrics, from the REAL reference (build container only).

Run:  python tests/golden/make_golden_eval.py      (needs /root/reference; never runs on the GPU box)

Runs the reference's centerNetEvaluation (models/centerNetOffset.py:253-354; evaluations/detection.py) on the
seeded decoded batches of oracle.metrics.eval_case and its expression() reductions
(trainer/model/centerOffsetRes10.py:18-106: torch.mean of the concatenated streams, averagePrecisionPlots +
averagePrecisionAll at 0.3/0.5/0.7/0.9).  Writes tests/golden/eval.npz:
  <case>_<stream>     the nine masked_select streams (float32, reference order)
  <case>_means        expression's nine means (mIoU, avgScore, orthogonity, mIoUC, mIoUwoO, mIoUO, maj/min/radMAE)
  <case>_aps          AP30/50/70/90 (float64)
  <case>_objs         per-image object counts
  <case>_expr         the expression() string (uint8 bytes)
Cases: 'inds' (ys[3] = heat indices, the training batches' format), 'locs' (ys[3] = (N,30,8) locs rows, the
validation set's format), 'empty' (no detection above the 0.3 score threshold).  Each case is checked to be
tie-safe (the AP is the same under either order of equal scores, which torch's unstable CPU sort leaves open).
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True
for _n in ["torchvision", "torchvision.transforms", "torchvision.transforms.functional"]:
    sys.modules[_n] = types.ModuleType(_n)
sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
sys.path.insert(0, REF)
sys.path.insert(1, REPO)

import torch  # noqa: E402

import trainer.model.centerOffsetRes10 as plugin  # noqa: E402  (reference plugin: evaluation, expression)
from evaluations.detection import averagePrecisionAll, averagePrecisionPlots  # noqa: E402

from oracle import metrics as M  # noqa: E402

KEYS = ("iouscore", "ortho", "ioucenter", "iouoffsetwo", "iouoffset", "maes")


def ref_case(c, loc_key):
    ys = [torch.zeros(c["scores"].shape[0], 1, 128, 128), torch.from_numpy(c["mask"]),
          torch.from_numpy(c["ys2"]), torch.from_numpy(c[loc_key])]
    ev, _ = plugin.evaluation(None, ys, torch.from_numpy(c["scores"]), None, torch.from_numpy(c["ctY"]),
                              torch.from_numpy(c["ctX"]), torch.from_numpy(c["offset"]), torch.from_numpy(c["regr"]),
                              {})
    iou, score = ev["iouscore"]
    aemaj, aemin, aerad = ev["maes"]
    streams = [iou, score, ev["ortho"], ev["ioucenter"], ev["iouoffsetwo"], ev["iouoffset"], aemaj, aemin, aerad]
    streams = [s.numpy().astype(np.float32) for s in streams]
    expr = plugin.expression([ev])
    # expression's numbers (centerOffsetRes10.py:62-88), recomputed from the reference functions
    ortho = torch.from_numpy(streams[2])
    ortho = ortho[~torch.isnan(ortho)]
    means = []
    for i, s in enumerate(streams):
        t = ortho if i == 2 else torch.from_numpy(s)
        means.append(float(torch.mean(t if len(t) > 0 else torch.zeros(1))))
    objnum = max(int(sum(ev["objs"])), len(streams[0]))
    aps = [averagePrecisionAll(averagePrecisionPlots(torch.from_numpy(streams[0]), torch.from_numpy(streams[1]),
                                                     objnum, t)) for t in (0.3, 0.5, 0.7, 0.9)]
    return streams, np.array(means), np.array(aps, np.float64), np.array(ev["objs"], np.int64), expr


def main():
    out = {}
    cases = [("inds", 21, "inds", {}), ("locs", 22, "locs", {}), ("empty", 23, "inds", {})]
    for name, seed, loc_key, kw in cases:
        for attempt in range(50):   # first tie-safe seed at or after `seed` (steps of 1000)
            c = M.eval_case(seed + 1000 * attempt, **kw)
            if name == "empty":
                c["scores"] = c["scores"] * np.float32(0.25)
            streams, means, aps, objs, expr = ref_case(c, loc_key)
            _, a1 = M.summary(streams, int(objs.sum()), ties="asc")
            _, a2 = M.summary(streams, int(objs.sum()), ties="desc")
            if np.allclose(a1, a2, rtol=0, atol=1e-12):
                break
        else:
            raise RuntimeError("no tie-safe case for " + name)
        out[name + "_seed"] = np.array(seed + 1000 * attempt)
        for s, v in zip(M.STREAMS, streams):
            out["%s_%s" % (name, s)] = v
        out[name + "_means"] = means
        out[name + "_aps"] = aps
        out[name + "_objs"] = objs
        out[name + "_expr"] = np.frombuffer(expr.encode(), np.uint8)
        print(name, [len(s) for s in streams], aps, expr)
    np.savez_compressed(os.path.join(HERE, "eval.npz"), **out)


def time_reference(N=32):
    """CPU time of the reference's evaluation + expression for one N-image batch (build container)."""
    import time
    c = M.eval_case(99, N=N)
    t0 = time.perf_counter()
    for _ in range(3):
        ref_case(c, "inds")
    print("reference centerNetEvaluation + expression, N=%d: %.1f ms per batch (%d threads)"
          % (N, (time.perf_counter() - t0) / 3 * 1e3, torch.get_num_threads()))


if __name__ == "__main__":
    if "--time" in sys.argv:
        time_reference(32)
        time_reference(256)
    else:
        main()
