"""GPU CenterNet target rendering (scd_render_center_targets) against the CPU renderer of the
dataset plugin (trainer/dataset/syntheticSCD.encode_targets), which follows the reference's drawGaussian /
centerThresholdRadius and is itself pinned to the reference by the F2 target fixtures
(tests/test_oracle_golden.py::test_f2_targets_render).

Heatmaps: the float64 Gaussian is added to the float32 map and rounded back per splat on both sides; the only
possible difference is a last-ulp one from the device's double exp (numpy calls libm), so the bound is one
float32 ulp with nearly every pixel bit-identical.  mask / regr / inds are exact."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cpu(locs_list, size):
    from trainer.dataset.syntheticSCD import encode_targets
    outs = [encode_targets(np.asarray(l, dtype=np.float32).reshape(-1, 8), size) for l in locs_list]
    return [np.stack([o[i] for o in outs]) for i in range(4)]


def _pack(locs_list, K=30):
    B = len(locs_list)
    locs = np.zeros((B, K, 8), dtype=np.float32)
    counts = np.zeros(B, dtype=np.int32)
    for b, l in enumerate(locs_list):
        l = np.asarray(l, dtype=np.float32).reshape(-1, 8)[:K]
        locs[b, :len(l)] = l
        counts[b] = len(l)
    return torch.from_numpy(locs), torch.from_numpy(counts)


def _check(locs_list, size=128):
    from scdhip import ops
    locs, counts = _pack(locs_list)
    heat, mask, regr, inds = ops.render_center_targets(locs.to(DEV), counts.to(DEV), size)
    torch.cuda.synchronize()
    ch, cm, cr, ci = _cpu(locs_list, size)
    gh = heat.cpu().numpy()
    assert gh.shape == ch.shape
    nan = np.isnan(ch)
    np.testing.assert_array_equal(np.isnan(gh), nan)          # degenerate radius 0: NaN on both sides
    diff = np.abs(gh - ch)[~nan]
    assert diff.size == 0 or diff.max() <= 6e-8, diff.max()
    assert diff.size == 0 or (diff == 0).mean() > 0.9999
    np.testing.assert_array_equal(mask.cpu().numpy(), cm)
    np.testing.assert_array_equal(inds.cpu().numpy(), ci)
    np.testing.assert_array_equal(regr.cpu().numpy(), cr)
    return gh


def test_render_matches_dataset_random_tiles():
    from trainer.dataset.syntheticSCD import sample_objects
    locs = [sample_objects(np.random.RandomState(100 + i)) for i in range(32)]
    heat = _check(locs)
    assert (heat == 1.0).sum() >= 32          # every centre pixel is a positive


def test_render_edge_cases():
    row = lambda x, y, mx=3.0, my=1.0, mn=1.5: [x, y, 0.5, 0.25, mx, my, mn, mn + 1.0]   # noqa: E731
    cases = [
        [],                                                                   # no objects
        [row(0, 0), row(127, 127), row(0, 127), row(127, 0)],                 # corners: clipped windows
        [row(64, 64)] * 5 + [row(65, 64, 5.0, 0.0, 2.5)],                      # overlaps: clip at 1 per splat
        [row(-1, 5), row(128, 5), row(5, -0.5), row(5.7, 9.2)],               # outside / truncation / floor
        [row(4 * i + 1, 3 * i + 2, 2 + 0.1 * i, 0.3 * i, 1 + 0.05 * i) for i in range(30)],   # 30 slots
        [row(10, 10, 0.0, 0.0, 1.0), row(20, 20)],                             # zero-length major axis: NaN splat
    ]
    _check(cases)


def test_render_other_map_size():
    from trainer.dataset.syntheticSCD import sample_objects
    locs = [sample_objects(np.random.RandomState(7 + i), size=256) for i in range(4)]
    _check(locs, size=256)


def test_dataset_gpu_batch_equals_per_sample_items():
    """The dataset plugin's GPU batch path returns what stacking __getitem__ gives (tiles exactly, targets as above)."""
    from trainer.dataset.syntheticSCD import SCD
    ds = SCD(None, True, seed=77)
    idx = list(range(8))
    gb = ds.gpu_batch(idx, DEV)
    items = [ds[i] for i in idx]
    assert torch.equal(gb["xs"][0].cpu(), torch.stack([it["xs"][0] for it in items]))
    ref = [torch.stack([it["ys"][k] for it in items]) for k in range(4)]
    assert (gb["ys"][0].cpu() - ref[0]).abs().max().item() <= 6e-8
    for k in (1, 2, 3):
        assert torch.equal(gb["ys"][k].cpu(), ref[k]), k
