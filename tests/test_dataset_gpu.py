"""`.d` dataset plugin on the GPU (tile augmentation scd_augment_tiles + targets
scd_render_center_targets) against the reference's SCD run on the same canonical synthetic archive
(tests/golden/scd.npz, tests/golden/make_golden_scd.py).

Tolerances: split / ids / object counts / mask / regr / locs / inds exact; validation tiles and the augmented
item 2e-5 absolute on unit-variance values (mean and variance are fp64 sums here, fp32 torch reductions in the
reference); heatmaps within one float32 ulp (tests/test_targets_gpu.py)."""
import json
import random

import numpy as np
import pytest
import torch

from oracle import scd_archive

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    from configuration import defaultConfig
    from trainer.dataset import scdx16p100 as D
    d = tmp_path_factory.mktemp("scd")
    path = str(d / "synthetic.d")
    scd_archive.write(path)
    old = dict(defaultConfig.config)
    defaultConfig.config["dirTemp"] = str(d / "temp") + "/"
    defaultConfig.config["dirDataSplitProfile"] = str(d / "split.json")
    try:
        random.seed(77)
        ds = D.SCD(path, True, None)
        split = open(defaultConfig.dirDataSplitProfile).read()
    finally:
        defaultConfig.config.clear()
        defaultConfig.config.update(old)
    return ds, split


def test_validation_set_vs_reference(built, golden):
    ds, split = built
    g = golden("scd")
    assert json.loads(split) == json.loads(bytes(g["split_json"]).decode())
    np.testing.assert_array_equal(ds.order, g["train_ids"])
    v = ds.validation
    np.testing.assert_allclose(v["xs"][0].cpu().numpy(), g["valid_xs"], rtol=0, atol=2e-5)
    heat = v["ys"][0].cpu()
    np.testing.assert_allclose(heat.double().sum((1, 2, 3)).numpy(), g["valid_heat_sum"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(heat[:8].numpy(), g["valid_heat0"], rtol=0, atol=1.2e-7)
    np.testing.assert_array_equal(v["ys"][1][:512].cpu().numpy(), g["valid_mask"])
    np.testing.assert_array_equal(v["ys"][2][:512].cpu().numpy(), g["valid_regr"])
    np.testing.assert_array_equal(v["ys"][3][:512].cpu().numpy(), g["valid_locs"])
    np.testing.assert_array_equal(v["xs"][1][:512].cpu().numpy(), g["valid_inds"])
    assert v["ys"][4] == g["valid_objnum"].tolist()


def test_validation_batches(built):
    from configuration import defaultConfig
    ds, _ = built
    bs = ds.getValidationSet()
    size = defaultConfig.validationBatchSize
    assert len(bs) == 5760 // size
    for b in bs:
        assert b["xs"][0].shape == (size, 1, 8, 8) and len(b["ys"]) == 6 and b["ys"][5].dtype == torch.int64


def test_training_item_with_reference_draws(built, golden):
    """The reference's __getitem__ output, reproduced from its own random draws (flips, jitter, noise)."""
    from scdhip import ops
    from trainer.dataset import scdx16p100 as D
    ds, _ = built
    g = golden("scd")
    i = int(g["item_id"])
    flips = g["item_flips"]
    jit = np.float32(1) + np.float32(0.05) * g["item_g"].astype(np.float32)
    xs = ops.augment_tiles(ds.samples[i][None].to(DEV), torch.from_numpy(flips[None]).to(DEV),
                           torch.from_numpy(jit).to(DEV), torch.from_numpy(g["item_noise"]).to(DEV), 0.05)
    np.testing.assert_allclose(xs[0].cpu().numpy(), g["item_xs"], rtol=0, atol=2e-5)
    l, n = D._pack_locs([D.SCD.flipLocs(ds.bounds[i], flips[0], flips[1])], trunc=True)
    heat, mask, regr, inds = ops.render_center_targets(torch.from_numpy(l).to(DEV), torch.from_numpy(n).to(DEV))
    np.testing.assert_allclose(heat[0].cpu().numpy(), g["item_heat"], rtol=0, atol=1.2e-7)
    np.testing.assert_array_equal(mask[0].cpu().numpy(), g["item_mask"])
    np.testing.assert_array_equal(regr[0].cpu().numpy(), g["item_regr"])
    np.testing.assert_array_equal(inds[0].cpu().numpy(), g["item_inds"])


def test_gpu_batch_and_getitem(built):
    ds, _ = built
    b = ds.gpu_batch(list(range(32)))
    x = b["xs"][0]
    assert x.shape == (32, 1, 8, 8) and x.is_cuda and torch.isfinite(x).all()
    assert [tuple(y.shape) for y in b["ys"]] == [(32, 1, 128, 128), (32, 30), (32, 30, 6), (32, 30)]
    it = ds[1]
    assert it["xs"][0].shape == (1, 8, 8) and it["ys"][0].shape == (1, 128, 128)


@pytest.mark.parametrize("B,H,W", [(4, 512, 512), (3, 6, 8), (1, 1024, 1024)])
def test_augment_tiles_vs_torch(B, H, W):
    """flip / normalize / jitter / given noise vs the reference's PyTorch ops on the CPU (argumentations.py)."""
    from scdhip import ops
    rs = np.random.RandomState(B * 7 + H)
    x = torch.from_numpy((rs.standard_normal((B, 1, H, W)) * 30 + 100).astype(np.float32))
    flips = torch.from_numpy(rs.randint(0, 2, (B, 2)).astype(np.uint8))
    g = torch.from_numpy(rs.standard_normal(B).astype(np.float32))
    noise = torch.from_numpy(rs.standard_normal((B, H, W)).astype(np.float32))
    jit = 1 + 0.05 * g
    got = ops.augment_tiles(x.to(DEV), flips.to(DEV), jit.to(DEV), noise.to(DEV), 0.05).cpu()
    for b in range(B):
        t = x[b]
        if flips[b, 0]:
            t = torch.flip(t, [2])
        if flips[b, 1]:
            t = torch.flip(t, [1])
        m = torch.mean(t)
        t = (t - m) / torch.sqrt(torch.mean(torch.square(t - m)))
        t = t * (1 + 0.05 * g[b]) + noise[b][None] * 0.05
        np.testing.assert_allclose(got[b].numpy(), t.numpy(), rtol=0, atol=2e-5)


def test_augment_device_noise_statistics():
    from scdhip import ops
    x = torch.randn(4, 1, 512, 512, device=DEV)
    clean = ops.augment_tiles(x)
    noisy = ops.augment_tiles(x, noise_sv=0.05, seed=123)
    n = ((noisy - clean) / 0.05).double()
    assert abs(n.mean().item()) < 5e-3 and abs(n.std().item() - 1) < 5e-3
    assert abs(torch.corrcoef(torch.stack([n[0].flatten(), n[1].flatten()]))[0, 1].item()) < 5e-3
    again = ops.augment_tiles(x, noise_sv=0.05, seed=123)
    assert torch.equal(noisy, again)
    assert not torch.equal(noisy, ops.augment_tiles(x, noise_sv=0.05, seed=124))
    with pytest.raises(RuntimeError):
        ops.augment_tiles(torch.zeros(1, 1, 8, 6, device=DEV))   # W % 4 != 0


@pytest.mark.parametrize("graph", [False, True])
def test_train_loop_on_d_archive(tmp_path, graph):
    """NetworkFactory end to end on a `.d` archive: split profile from disk, batches through gpu_batch
    (GPUBatchLoader), bf16 steps, validation through evaluation / expression, evals file written.  graph: the
    stepGraph mode -- two eager steps, capture on the third, replays after; validation (eager forwards of the same
    model) runs between replays."""
    from configuration import defaultConfig
    from models.networkFactory import NetworkFactory
    names, samples, locs = scd_archive.archive_content(seed=5, count=48, size=512)
    from trainer.dataset.scdx16p100 import writeArchive
    path = str(tmp_path / "tiny.d")
    writeArchive(path, names, samples, locs)
    split = tmp_path / "tiny.split.json"
    split.write_text(json.dumps({"validation": list(range(8))}))
    old = dict(defaultConfig.config)
    try:
        defaultConfig.updateConfig({"modelName": "centerOffsetRes10", "datasetName": "tiny", "trainName": "dtest",
                                    "iterations": 5 if graph else 2, "validation": 2, "snapshot": 1000,
                                    "batchSize": 16, "stepGraph": graph,
                                    "dirData": "trainer.dataset.scdx16p100", "dirDatafile": path,
                                    "dirDataSplitProfile": str(split), "dirTemp": str(tmp_path / "t") + "/",
                                    "dirResult": str(tmp_path / "r") + "/", "currentIter": 0})
        f = NetworkFactory(True)
        assert len(f.dataset) == 40
        f.beginTraining(0)
        text = open(str(tmp_path / "r" / "evals.dtest.txt")).read()
        if graph:
            assert f.stepGraph is not None and len(f.stepGraph.graphs) == 1 and f.stepGraph.calls == 5
            assert f.optimizer.state_dict()["step"] == 5
    finally:
        defaultConfig.config.clear()
        defaultConfig.config.update(old)
    assert "[mIoU]" in text and "[AP50]" in text and "[Tr]" in text
