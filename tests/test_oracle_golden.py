"""Pin the CPU oracle against golden vectors produced by the real reference
(tests/golden/make_golden.py).  CPU only."""
import zlib

import numpy as np
import pytest
import torch

from oracle import centernet as O
from oracle import targets as T


def _pos(name, numel, k):
    return np.random.RandomState(zlib.crc32(name.encode()) & 0xFFFFFFFF).randint(0, numel, k)


@pytest.fixture(scope="module")
def spec():
    return O.model_spec(10)


@pytest.fixture(scope="module")
def f1_run(spec):
    entries, topo = spec
    P, Bf = O.split_state(O.hash_weights(entries))
    x = T.batch_inputs(1, 2, 512)
    with torch.no_grad():
        out = O.forward(P, Bf, x, topo)
    return out, Bf


def test_param_count(spec, golden):
    entries, _ = spec
    n = sum(int(np.prod(s)) for k, s in entries
            if not (k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked")))
    assert n == int(golden("init")["param_count"]) == 9981383


def test_state_keys_match_reference(spec, golden):
    entries, _ = spec
    g = golden("init")
    keys = sorted({k.split("|")[0] for k in g.files if "|" in k})
    assert keys == sorted(k for k, _ in entries)


def test_f1_forward(f1_run, golden):
    out, Bf = f1_run
    g = golden("fwd")
    for k in ("heatmap", "regr", "offset"):
        np.testing.assert_allclose(out[k].numpy(), g[k], rtol=1e-4, atol=1e-4)
    for k in g.files:
        if k.startswith("rs|"):
            np.testing.assert_allclose(Bf[k[3:]].numpy(), g[k], rtol=1e-4, atol=1e-5)


def test_f4_decode(f1_run, golden):
    out, _ = f1_run
    g = golden("decode")
    dec = O.decode({k: v.clone() for k, v in out.items()})
    names = ["scores", "inds", "ys", "xs", "offset", "regr"]
    np.testing.assert_allclose(dec[0].numpy(), g["f1|scores"], rtol=1e-4, atol=1e-5)
    rs = np.random.RandomState(7)
    syn = {"heatmap": torch.from_numpy((rs.standard_normal((2, 1, 128, 128)) * 3).astype(np.float32)),
           "regr": torch.from_numpy(rs.standard_normal((2, 4, 128, 128)).astype(np.float32)),
           "offset": torch.from_numpy(rs.standard_normal((2, 2, 128, 128)).astype(np.float32))}
    dec = O.decode(syn)
    for i, n in enumerate(names):
        if n in ("offset", "regr", "scores"):
            np.testing.assert_allclose(dec[i].numpy(), g["syn|" + n], rtol=0, atol=0)
        else:
            np.testing.assert_array_equal(dec[i].numpy(), g["syn|" + n])


def test_f2_targets_render(golden):
    g = golden("loss")
    ys = T.batch_targets(2, 2, 128)
    for i, n in enumerate(["heat", "mask", "regr", "inds"]):
        np.testing.assert_array_equal(ys[i].numpy(), g["ys|" + n])


@pytest.mark.parametrize("case", ["a", "b", "c", "d"])
def test_f2_loss_and_grads(case, golden):
    g = golden("loss")
    f = golden("fwd")
    ys = [torch.from_numpy(g["ys|" + n]) for n in ["heat", "mask", "regr", "inds"]]
    preds = {k: torch.from_numpy(f[k]) for k in ("heatmap", "regr", "offset")}
    if case == "b":
        ys[0] = ys[0] * 0.9
    if case == "c":
        ys[3] = torch.from_numpy(g["c|inds"])
    if case == "d":
        h = preds["heatmap"]
        preds["heatmap"] = torch.where(h > h.median(), torch.full_like(h, 20.0), torch.full_like(h, -20.0))
    leaves = {k: v.clone().requires_grad_(True) for k, v in preds.items()}
    loss, stats = O.centernet_loss(leaves, ys)
    loss.mean().backward()
    np.testing.assert_allclose(loss.detach().numpy(), g[case + "|loss"], rtol=1e-5)
    np.testing.assert_allclose([s.item() for s in stats], g[case + "|stats"], rtol=1e-5, atol=1e-7)
    gh = leaves["heatmap"].grad
    if case == "a":
        np.testing.assert_allclose(gh.numpy(), g["a|dheatmap"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(gh.double().abs().sum().item(), g[case + "|dheatmap_abs"], rtol=1e-5)
    for k in ("regr", "offset"):
        np.testing.assert_allclose(O.gather_feat(leaves[k].grad, ys[3]).numpy(), g[case + "|d" + k], rtol=1e-6)


def test_f3_train_step(spec, golden):
    entries, topo = spec
    g = golden("step")
    st = O.TrainState(O.hash_weights(entries))
    x = T.batch_inputs(3, 2, 512)
    ys = T.batch_targets(4, 2, 128)
    pre = {k: v.detach().clone() for k, v in st.P.items()}
    st.opt.zero_grad()
    outs = O.forward(st.P, st.B, x, topo)
    loss, stats = O.centernet_loss(outs, ys)
    loss.mean().backward()
    grads = {k: v.grad.detach().clone() for k, v in st.P.items()}
    st.opt.step()
    np.testing.assert_allclose(loss.detach().numpy(), g["loss"], rtol=1e-4)
    for k, v in st.P.items():
        pos = _pos(k, v.numel(), 16)
        np.testing.assert_allclose(grads[k].double().norm().item(), g["gnorm|" + k], rtol=2e-3, atol=1e-7)
        np.testing.assert_allclose(pre[k].reshape(-1)[pos].numpy(), g["p0samp|" + k], rtol=0, atol=0)
        np.testing.assert_allclose(v.detach().reshape(-1)[pos].numpy(), g["psamp|" + k], rtol=1e-5, atol=2e-6)
        gmax = max(grads[k].abs().max().item(), 1e-30)
        np.testing.assert_allclose(grads[k].reshape(-1)[pos].numpy(), g["gsamp|" + k], rtol=0, atol=1e-4 * gmax,
                                   err_msg=k)


def test_f6_layer_stats(spec, golden):
    entries, topo = spec
    g = golden("layers")
    P, Bf = O.split_state(O.hash_weights(entries))
    taps = {}
    with torch.no_grad():
        O.forward(P, Bf, T.batch_inputs(6, 2, 128), topo, taps=taps)
    for name, t in taps.items():
        if name + "|samp" not in g.files:
            continue
        pos = _pos(name, t.numel(), 32)
        assert tuple(t.shape) == tuple(g[name + "|shape"])
        np.testing.assert_allclose(t.reshape(-1)[pos].numpy(), g[name + "|samp"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name,world,per,seeds", [("ddp", 2, 2, (8, 9)), ("ddp4", 4, 2, (31, 32))])
def test_f7_ddp_syncbn(spec, golden, name, world, per, seeds):
    """Global-batch BN == SyncBN; averaging per-shard losses == DDP gradient averaging (F7 at W=2, F7b at W=4)."""
    entries, topo = spec
    g = golden(name)
    P, Bf = O.split_state(O.hash_weights(entries))
    P = {k: v.requires_grad_(True) for k, v in P.items()}
    x = T.batch_inputs(seeds[0], world * per, 128)
    ys = T.batch_targets(seeds[1], world * per, 32)
    outs = O.forward(P, Bf, x, topo)
    losses = []
    for r in range(world):
        sl = slice(per * r, per * r + per)
        l, _ = O.centernet_loss({k: v[sl] for k, v in outs.items()}, [y[sl] for y in ys])
        losses.append(l.mean())
    (sum(losses) / world).backward()
    for r in range(world):
        np.testing.assert_allclose(losses[r].item(), g["loss_r%d" % r], rtol=1e-4)
    for k, v in P.items():
        np.testing.assert_allclose(v.grad.double().norm().item(), g["gnorm|" + k], rtol=2e-3, atol=1e-7)
        gmax = max(v.grad.abs().max().item(), 1e-30)
        np.testing.assert_allclose(v.grad.reshape(-1)[_pos(k, v.numel(), 16)].numpy(), g["gsamp|" + k], rtol=0,
                                   atol=1e-4 * gmax, err_msg=k)
    for k in g.files:
        if k.startswith("rs|"):
            np.testing.assert_allclose(Bf[k[3:]].numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=k)


# ---------------------------------------------------------------- CornerNet (F5, F8)

def test_f5_cpool_forward_matches_reference_cpp(golden):
    from oracle import cpool
    g = golden("cpool")
    for d in range(4):
        np.testing.assert_array_equal(cpool.forward(torch.from_numpy(g["x"]), d).numpy(), g["y%d" % d])
        np.testing.assert_array_equal(cpool.forward(torch.from_numpy(g["xt"]), d).numpy(), g["yt%d" % d])


def test_cpool_backward_restatement_matches_autograd_when_tie_free():
    from oracle import cpool
    x = torch.randn(2, 3, 9, 7, dtype=torch.float64)
    dy = torch.randn_like(x)
    for d in range(4):
        xr = x.clone().requires_grad_(True)
        cpool.forward(xr, d).backward(dy)
        np.testing.assert_allclose(cpool.backward(x, dy, d).numpy(), xr.grad.numpy(), rtol=1e-12, atol=1e-12)


def test_cpool_backward_tie_rule():
    """ties keep the first-scanned position (strict '>' update, topPool.cpp:61-65)."""
    from oracle import cpool
    x = torch.tensor([[[[1.0], [2.0], [2.0], [0.0]]]])     # H=4, W=1
    dy = torch.ones_like(x)
    # top pool scans h = 3,2,1,0: the max 2.0 is first seen at h=2 -> h=2 collects rows 0,1,2
    np.testing.assert_array_equal(cpool.backward(x, dy, 0).reshape(-1).numpy(), [0, 0, 3, 1])
    # bottom pool scans h = 0,1,2,3: first seen at h=1 -> h=1 collects rows 1,2,3
    np.testing.assert_array_equal(cpool.backward(x, dy, 1).reshape(-1).numpy(), [1, 3, 0, 0])


def test_f8_cornernet_forward_and_loss(golden):
    from oracle import cornernet as OC
    g = golden("corner")
    entries, topo = OC.model_spec(10)
    P, Bf = O.split_state(OC.hash_weights(entries))
    with torch.no_grad():
        out = OC.forward(P, Bf, T.batch_inputs(31, 2, 128), topo)
    for k in ("heatmap", "tl", "br"):
        np.testing.assert_allclose(out[k].numpy(), g[k], rtol=1e-4, atol=1e-4, err_msg=k)
    ys = [torch.from_numpy(g["ys|" + n]) for n in ["heat", "mask", "regr", "tl", "br"]]
    np.testing.assert_allclose(OC.cornernet_loss(out, ys).numpy(), g["loss"], rtol=1e-4)
    for k in g.files:
        if k.startswith("rs|"):
            np.testing.assert_allclose(Bf[k[3:]].numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=k)


def test_f8_corner_targets_rule(golden):
    g = golden("corner")
    ys = T.corner_targets(32, 2, 32)
    for i, n in enumerate(["heat", "mask", "regr", "tl", "br"]):
        np.testing.assert_array_equal(ys[i].numpy(), g["ys|" + n])


def test_f9_res50_bottleneck_step(golden):
    """Oracle Bottleneck path (residuals.py:122-165, ResNetSpec[50]) against the reference's Res50 forward,
    CenterNetLoss and gradients (F9, make_golden_res50.py): pins the oracle for the a3 row."""
    g = golden("res50")
    entries, topo = O.model_spec(50, [64, 64, 128, 256, 512, 256, 256, 256])
    st = O.TrainState(O.hash_weights(entries))
    x = T.batch_inputs(9, 2, 128)
    ys = T.batch_targets(10, 2, 32)
    outs = O.forward(st.P, st.B, x, topo)
    for k in ("heatmap", "regr", "offset"):
        np.testing.assert_allclose(outs[k].detach().numpy(), g[k], rtol=1e-4, atol=1e-4, err_msg=k)
    loss, stats = O.centernet_loss(outs, ys)
    loss.mean().backward()
    np.testing.assert_allclose(loss.detach().numpy(), g["loss"], rtol=1e-4)
    np.testing.assert_allclose([s.item() for s in stats], g["stats"], rtol=1e-4, atol=1e-6)
    for k, v in st.P.items():
        np.testing.assert_allclose(v.grad.double().norm().item(), g["gnorm|" + k], rtol=2e-3, atol=1e-7, err_msg=k)
        gmax = max(v.grad.abs().max().item(), 1e-30)
        np.testing.assert_allclose(v.grad.reshape(-1)[_pos(k, v.numel(), 8)].numpy(), g["gsamp|" + k], rtol=0,
                                   atol=1e-3 * gmax, err_msg=k)
    for k in g.files:
        if k.startswith("rs|"):
            np.testing.assert_allclose(st.B[k[3:]].numpy(), g[k], rtol=1e-4, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("case,loc_key", [("inds", "inds"), ("locs", "locs"), ("empty", "inds")])
def test_f10_eval_metrics(golden, case, loc_key):
    """oracle.metrics vs the reference's centerNetEvaluation + expression numbers (tests/golden/eval.npz)."""
    from oracle import metrics as M
    g = golden("eval")
    c = M.eval_case(int(g[case + "_seed"]))
    if case == "empty":
        c["scores"] = c["scores"] * np.float32(0.25)
    streams = M.center_eval(c["scores"], c["ctY"], c["ctX"], c["offset"], c["regr"], c["ys2"], c[loc_key])
    for s, v in zip(M.STREAMS, streams):
        np.testing.assert_array_equal(v, g["%s_%s" % (case, s)], err_msg=s)
    np.testing.assert_array_equal(c["mask"].sum(1), g[case + "_objs"])
    means, aps = M.summary(streams, int(g[case + "_objs"].sum()))
    np.testing.assert_allclose(means, g[case + "_means"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(aps, g[case + "_aps"], rtol=0, atol=1e-12)


def test_f10_ap_walk_small_cases():
    """averagePrecisionAll restated: hand-checked plots (detection.py:208-230)."""
    from oracle import metrics as M
    assert M.ap_all([]) == 0
    # one true positive of two objects: recall 0.5 at precision 1
    assert M.ap_all([[0.5, 1.0]]) == 0.5
    # FP then TP: precision 0 then 0.5 at recall 1 -> 0.5
    assert M.ap_all([[0.0, 0.0], [1.0, 0.5]]) == 0.5
    # TP, FP, TP over 2 objects: (0.5,1), (0.5,0.5), (1,2/3) -> 1*(2/3) record at the end, then (0.5-0.5)*... + 0.5*1
    plots = [[0.5, 1.0], [0.5, 0.5], [1.0, 2 / 3]]
    assert abs(M.ap_all(plots) - ((1.0 - 0.5) * (2 / 3) + 0.5 * 1.0)) < 1e-15


NARROW = {"centerOffsetRes10q": [16, 16, 32, 64, 128, 64, 64, 64],
          "centerOffsetRes10h": [32, 32, 64, 128, 256, 128, 128, 128]}


@pytest.mark.parametrize("name", sorted(NARROW))
def test_f11_narrow_plugins(golden, name):
    """Oracle on the 16/32-channel plugins with 64-wide heads (centerNetOffseth.py) vs the reference (F11)."""
    g = golden("narrow")
    entries, topo = O.model_spec(10, NARROW[name], head_dim=64)
    st = O.TrainState(O.hash_weights(entries))
    outs = O.forward(st.P, st.B, T.batch_inputs(21, 2, 256), topo)
    for k in ("heatmap", "regr", "offset"):
        np.testing.assert_allclose(outs[k].detach().numpy(), g["%s|%s" % (name, k)], rtol=1e-4, atol=1e-4, err_msg=k)
    loss, stats = O.centernet_loss(outs, T.batch_targets(22, 2, 64))
    loss.mean().backward()
    np.testing.assert_allclose(loss.detach().numpy(), g[name + "|loss"], rtol=1e-4)
    for k, v in st.P.items():
        np.testing.assert_allclose(v.grad.double().norm().item(), g["%s|gnorm|%s" % (name, k)], rtol=2e-3, atol=1e-7,
                                   err_msg=k)
