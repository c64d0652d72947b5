"""`.d` dataset plugin host logic, CPU only: the archive writer/reader and the split rule
against the reference's own split (tests/golden/scd.npz, tests/golden/make_golden_scd.py)."""
import json
import random

import numpy as np

from oracle import scd_archive
from trainer.dataset import scdx16p100 as D


def test_archive_roundtrip(tmp_path):
    names, samples, locs = scd_archive.archive_content(seed=3, count=50, size=12)
    path = str(tmp_path / "a.d")
    D.writeArchive(path, names, samples, locs)
    n2, counts, s2, b2 = D.readArchive(path, str(tmp_path / "no-such-dir") + "/")
    assert n2 == names
    assert counts == {"count": {n: len(l) for n, l in zip(names, locs)}}
    for a, b in zip(samples, s2):
        assert tuple(b.shape) == (1, 12, 12)
        np.testing.assert_array_equal(b[0].numpy(), a)
    for a, b in zip(locs, b2):
        assert tuple(b.shape) == (len(a), 8)
        np.testing.assert_array_equal(b.numpy(), a)


def test_archive_reads_extracted_cache(tmp_path):
    import zipfile
    names, samples, locs = scd_archive.archive_content(seed=4, count=10, size=8)
    path = str(tmp_path / "a.d")
    D.writeArchive(path, names, samples, locs)
    cache = tmp_path / "confocalCenter"
    zipfile.ZipFile(path).extractall(cache)
    n2, _, s2, _ = D.readArchive(str(tmp_path / "missing.d"), str(cache) + "/")
    assert n2 == names and len(s2) == 10


def test_split_matches_reference(golden):
    g = golden("scd")
    random.seed(77)
    order, profile = D.splitOrder(scd_archive.CANONICAL, None)
    np.testing.assert_array_equal(profile["validation"], g["valid_ids"])
    np.testing.assert_array_equal(order, g["train_ids"])
    ref = json.loads(bytes(g["split_json"]).decode())
    assert ref == json.loads(json.dumps(profile))


def test_split_from_profile():
    g_valid = list(range(0, 49920, 7))[:5760]
    random.seed(1)
    order, profile = D.splitOrder(scd_archive.CANONICAL, {"validation": g_valid})
    assert len(order) == 49920 - len(g_valid) and not set(order) & set(g_valid)
    assert profile[D.TRAINSUBSET] is order
    order2, _ = D.splitOrder(scd_archive.CANONICAL, {"validation": g_valid, D.TRAINSUBSET: [5, 3, 1]})
    assert order2 == [5, 3, 1]


def test_flip_locs_rule():
    l = np.array([[10.5, 20.25, 1, 2, 3, 4, 5, 6]], np.float32)
    f = D.SCD.flipLocs(l, True, True)
    np.testing.assert_array_equal(f, [[117 - 0.5, 107 - 0.25, -1, -2, -3, -4, 5, 6]])
    np.testing.assert_array_equal(l[0, 0], 10.5)   # stored bounds are not mutated
    locs, counts = D._pack_locs([f, np.zeros((0, 8), np.float32)], trunc=True)
    assert counts.tolist() == [1, 0] and locs[0, 0, 0] == 116 and locs[0, 0, 1] == 106


def test_gpu_batch_loader_visits_dataloader_order():
    """networkFactory.GPUBatchLoader asks gpu_batch for exactly the index batches DataLoader would build."""
    import torch.utils.data.distributed as dd
    from torch.utils.data import DataLoader

    from models.networkFactory import GPUBatchLoader

    class Fake:
        def __init__(self):
            self.seen = []

        def __len__(self):
            return 70

        def __getitem__(self, i):
            return i

        def gpu_batch(self, idx, device):
            self.seen.append(idx)
            return idx

    ds = Fake()
    assert list(GPUBatchLoader(ds, None, 16, "cpu")) == [b.tolist() for b in DataLoader(ds, 16, drop_last=True)]
    for rank in range(2):
        s = dd.DistributedSampler(ds, num_replicas=2, rank=rank, drop_last=True, shuffle=False)
        want = [b.tolist() for b in DataLoader(ds, 8, sampler=s, drop_last=True)]
        assert list(GPUBatchLoader(ds, s, 8, "cpu")) == want


def test_slide_restatement_matches_reference(golden):
    """oracle.slide_case (test.py restated) against the reference's own clips and detections (slide.npz)."""
    from oracle import slide_case as S
    g = golden("slide")
    img = S.slide()
    geo = S.geometry(*img.shape[:2])
    assert (geo["clipH"], geo["clipV"], geo["padLR"], geo["padTB"]) == (8, 6, 54, 188)
    c0 = S.clip(img, geo, 0, 0)
    np.testing.assert_allclose(c0[:64, :64], g["win_first"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(c0[::8, ::8], g["clip_sub"][0], rtol=0, atol=1e-6)
    last = S.clip(img, geo, geo["clipH"] - 1, geo["clipV"] - 1)
    np.testing.assert_allclose(last[448:, 448:], g["win_last"], rtol=0, atol=1e-6)
    det = S.detections(g["decoded"], geo)
    np.testing.assert_array_equal(det[:, :2], g["detections"][:, :2])
    np.testing.assert_allclose(det[:, 2], g["detections"][:, 2], rtol=1e-12)
