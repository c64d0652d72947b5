"""GPU validation metrics: scd_ceval_count/emit (centerNetEvaluation's pair streams) and
scd_ceval_summary (expression's means and AP) against the reference's outputs (tests/golden/eval.npz, made by
tests/golden/make_golden_eval.py from the real reference) and the CPU restatement oracle/metrics.py.

Tolerances.  The streams are float32 values from one rounding per op on both sides; the only op whose result
can differ is sqrt: the device's is correctly rounded, the reference's torch CPU kernel is not always (see
oracle/metrics.py), so values agree to a few ulp: rtol 2e-5 (one ulp of a box coordinate near 128 px, 7.6e-6, over an
intersection side of ~1 px); orthogonity = sqrt(1 - cos^2) is compared through its square (one ulp
of cos near 1 moves it by up to 5e-4) and may be NaN on one side where it is ~0; stream lengths (the masks) are exact on these cases.  The AP walk is checked
exactly (1e-12) against the oracle on the device's own streams, and against the reference's APs.  Means are
fp64 on the device, fp32 torch.mean in the reference: rtol 1e-5."""
import re

import numpy as np
import pytest
import torch

from oracle import metrics as M

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gpu_streams(c, loc_key, H=128):
    from scdhip import ops
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    s = ops.center_eval(t(c["scores"]), t(c["ctY"]), t(c["ctX"]), t(c["offset"]), t(c["regr"]), t(c["ys2"]),
                        t(c[loc_key]), heatmap_size=H)
    torch.cuda.synchronize()
    return s


def _cmp_streams(got, want):
    for name, g, w in zip(M.STREAMS, got, want):
        g = g.cpu().numpy() if torch.is_tensor(g) else g
        assert g.shape == w.shape, (name, g.shape, w.shape)
        if name == "ortho":
            # sqrt(1 - cos^2) is ill-conditioned near cos = 1 (one ulp of cos moves it by up to 5e-4): compare
            # 1 - cos^2 = ortho^2 to a few ulp of 1; NaN (1 - cos^2 rounded below 0) only opposite ~0
            both = ~np.isnan(g) & ~np.isnan(w)
            np.testing.assert_allclose(g[both].astype(np.float64) ** 2, w[both].astype(np.float64) ** 2, rtol=1e-5,
                                       atol=1e-6, err_msg=name)
            assert np.all(np.nan_to_num(g[~both], nan=0.0) ** 2 < 1e-6)
            assert np.all(np.nan_to_num(w[~both], nan=0.0) ** 2 < 1e-6)
        else:
            np.testing.assert_allclose(g, w, rtol=2e-5, atol=2e-6, err_msg=name)


@pytest.mark.parametrize("case,loc_key", [("inds", "inds"), ("locs", "locs"), ("empty", "inds")])
def test_eval_streams_and_summary_vs_reference(golden, case, loc_key):
    from scdhip import ops
    g = golden("eval")
    c = M.eval_case(int(g[case + "_seed"]))
    if case == "empty":
        c["scores"] = c["scores"] * np.float32(0.25)
    s = _gpu_streams(c, loc_key)
    _cmp_streams(s, [g["%s_%s" % (case, n)] for n in M.STREAMS])
    objnum = int(g[case + "_objs"].sum())
    means, aps = ops.center_eval_summary(s, objnum)
    gm = g[case + "_means"]
    keep = [i for i in range(9) if i != 2]
    np.testing.assert_allclose(np.array(means)[keep], gm[keep], rtol=1e-5, atol=1e-7)
    assert abs(means[2] - gm[2]) < 1e-4    # orthogonity: see the module docstring
    np.testing.assert_allclose(aps, g[case + "_aps"], rtol=0, atol=1e-9)
    _, aps_o = M.summary([x.cpu().numpy() for x in s], objnum)
    np.testing.assert_allclose(aps, aps_o, rtol=0, atol=1e-12)


def test_plugin_evaluation_and_expression(golden):
    """The plugin surface: centerNetEvaluation's dict and expression()'s string (numbers at printed precision)."""
    import trainer.model.centerOffsetRes10 as plugin
    g = golden("eval")
    c = M.eval_case(int(g["inds_seed"]))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    ys = [torch.zeros(4, 1, 128, 128, device=DEV), t(c["mask"]), t(c["ys2"]), t(c["inds"])]
    ev, od = plugin.evaluation(None, ys, t(c["scores"]), None, t(c["ctY"]), t(c["ctX"]), t(c["offset"]),
                               t(c["regr"]), {})
    assert set(ev) == {"iouscore", "ortho", "ioucenter", "iouoffsetwo", "iouoffset", "maes", "objs"}
    assert ev["objs"] == g["inds_objs"].tolist()
    expr = plugin.expression([ev, ev])  # two batches: streams concatenated, objects summed
    ref = bytes(g["inds_expr"]).decode()
    tags = re.findall(r"\[(\w+)\]", ref)
    assert re.findall(r"\[(\w+)\]", expr) == tags
    got_v = [float(v) for v in re.findall(r"\]\s+(-?[\d.]+)", expr)]
    ref_v = [float(v) for v in re.findall(r"\]\s+(-?[\d.]+)", ref)]
    # duplicating every batch leaves the means unchanged; AP changes (ties between the copies), so only the
    # means are compared on the doubled set, and the single-batch string is compared in full below
    for tag, a, b in zip(tags, got_v, ref_v):
        if not tag.startswith("AP"):
            assert abs(a - b) <= 2e-6 * max(1.0, abs(b)) + 1e-6 + (1e-4 if tag == "Orth" else 0), (tag, a, b)
    expr1 = plugin.expression([ev])
    got1 = [float(v) for v in re.findall(r"\]\s+(-?[\d.]+)", expr1)]
    for tag, a, b in zip(tags, got1, ref_v):
        slack = 0.0051 if tag.startswith("AP") else (1e-4 if tag == "Orth" else 0)
        assert abs(a - b) <= 2e-6 * max(1.0, abs(b)) + 1e-6 + slack, (tag, a, b)


@pytest.mark.parametrize("seed,K,L", [(5, 100, 30), (6, 256, 64), (7, 1, 1), (8, 37, 5)])
def test_eval_streams_vs_oracle_shapes(seed, K, L):
    c = M.eval_case(seed, N=9, K=K, L=L, n_near=min(K, 40))
    s = _gpu_streams(c, "inds")
    _cmp_streams(s, M.center_eval(c["scores"], c["ctY"], c["ctX"], c["offset"], c["regr"], c["ys2"], c["inds"]))


@pytest.mark.parametrize("n,levels", [(0, 0), (1, 0), (1023, 0), (1024, 7), (1025, 0), (5000, 13), (40000, 50)])
def test_summary_ap_vs_oracle(n, levels):
    """AP over many detections (multi-chunk scans, 2^16-key bitonic sort), with and without tied scores
    (levels > 0: scores quantised to `levels` values, ties ranked by descending index on both sides)."""
    from scdhip import ops
    rs = np.random.RandomState(n + levels)
    iou = rs.uniform(0, 1, n).astype(np.float32)
    sc = rs.uniform(0.3, 1, n).astype(np.float32)
    if levels:
        sc = (np.floor(sc * levels) / levels).astype(np.float32)
    streams = [iou, sc] + [rs.uniform(0, 1, rs.randint(0, 50)).astype(np.float32) for _ in range(7)]
    if len(streams[2]) >= 3:
        streams[2][:3] = np.nan
    objnum = int(n * 0.8) + 3
    means, aps = ops.center_eval_summary([torch.from_numpy(x).to(DEV) for x in streams], objnum)
    m_o, aps_o = M.summary(streams, objnum)
    np.testing.assert_allclose(aps, aps_o, rtol=0, atol=1e-12)
    np.testing.assert_allclose(means, m_o, rtol=1e-12, atol=1e-15)


def test_eval_rejects_oversized_shapes():
    from scdhip import ops
    c = M.eval_case(3, N=1, K=257, L=30, n_near=5)
    with pytest.raises(RuntimeError):
        _gpu_streams(c, "inds")
    with pytest.raises(RuntimeError):
        ops.center_eval(torch.zeros(1, 4), torch.zeros(1, 4, dtype=torch.long), torch.zeros(1, 4, dtype=torch.long),
                        torch.zeros(1, 4, 2), torch.zeros(1, 4, 4), torch.zeros(1, 3, 6),
                        torch.zeros(1, 3, dtype=torch.long))  # CPU tensors: no fallback


def test_eval_streams_many_images():
    """600 images: output offsets from the workgroup-wide sum of the earlier images' counts."""
    c = M.eval_case(31, N=600, K=100, L=30, n_near=20)
    s = _gpu_streams(c, "inds")
    _cmp_streams(s, M.center_eval(c["scores"], c["ctY"], c["ctX"], c["offset"], c["regr"], c["ys2"], c["inds"]))
