"""`.d` archive dataset plugin `scdx16p100` (datasets/scds/scdx16p100.py of the reference).

The on-disk format is the reference's (scdx16p100.py:64-93; written by preprocess.py:78-109 through a profile's
generateArchieve): a zip holding
    dataset.json          {"names": [name, ...]}
    object-count.json     {"count": {name: n, ...}}
    samples/<name>.npy    (H, W) grayscale tile
    locs/<name>.npy       (n, 8) float rows [ctx, cty, offx, offy, majx, majy, minl, halo] (heatmap units)
Constructor, split rules and sample format are the reference's:
  * samples index FSI x ARGUM x CLIP = 130 x 16 x 24 raw positions, kept when argum < ARGUMENTRATIO, shuffled with
    Python's `random` (unseeded, as the reference), cut to PARTITION (:143-158);
  * no split profile: the first TESTSET shuffled positions become the validation set, the rest `train16p100`;
    with a profile: its `train16p100` list, or everything not in its `validation` list (:160-180); the profile
    is written back to defaultConfig.dirDataSplitProfile (:264-266);
  * validation set: normalize (no augmentation), heat / mask / regr / locs / inds with the objects' centres
    truncated to integers (:188-262), served in validationBatchSize slices by getValidationSet (:381-414);
  * __getitem__(i): reshuffle at i == 0, x / y flips (numpy.random.uniform() > 0.5), normalize, variance jitter
    and Gaussian noise (0.05 each), targets (:300-379).
MI355X-native differences: the archive is read straight from the zip (no extraction into dirTemp; an already
extracted dirTemp/confocalCenter/ is still used when present); the tile augmentation runs as scd_augment_tiles
and the targets as scd_render_center_targets, batched over a whole training batch by gpu_batch() -- the
reference does both per sample in PyTorch.  Stored bounds are never mutated (the reference's CPU path flips
and truncates them in place, :424-429, :523-525).  A smaller-than-canonical archive (tests) indexes only the
positions it holds.  The reference's CUDA path pins cuda:0 (:316-356); here the device is the caller's.
"""
import io
import json
import os
import zipfile
from random import shuffle

import numpy as np
import torch
from torch.utils.data import Dataset

MAXTAGLEN = 30
TARGETSIZE = 512
HEATMAPSIZE = 128
THRESHOLDIOU = 0.5
TESTSET = 5760
REALTIMETEST = 5760
ARGUMENTRATIO = 16
PARTITION = 1.00
TRAINSUBSET = 'train16p100'
FSI, ARGUM, CLIP = 130, 16, 24
NOISESV, JITTERSV = 0.05, 0.05

__all__ = ["SCD", "dataset", "writeArchive", "readArchive", "splitOrder"]


def writeArchive(path, names, samples, locs):
    """Write a `.d` archive in the reference's layout (the generateArchieve contract of preprocess.py:99-105)."""
    with zipfile.ZipFile(path, "w", zipfile.ZIP_STORED) as z:
        z.writestr("dataset.json", json.dumps({"names": list(names)}))
        z.writestr("object-count.json", json.dumps({"count": {n: int(len(l)) for n, l in zip(names, locs)}}))
        for n, s, l in zip(names, samples, locs):
            for sub, arr in (("samples", s), ("locs", np.asarray(l, np.float32).reshape(-1, 8))):
                buf = io.BytesIO()
                np.save(buf, arr, allow_pickle=False)
                z.writestr("%s/%s.npy" % (sub, n), buf.getvalue())


def readArchive(zipPath, tempDir=None):
    """-> (names, objectCounts, samples [(1,H,W) f32 tensors], bounds [(n,8) f32 tensors]) (scdx16p100.py:98-135).
    Reads an extracted tempDir when it exists (the reference's cache), else the zip members directly."""
    if tempDir is not None and os.path.exists(tempDir):
        def read(name):
            with open(os.path.join(tempDir, name), "rb") as f:
                return f.read()
        z = None
    else:
        z = zipfile.ZipFile(zipPath)
        read = z.read
    try:
        names = json.loads(read("dataset.json"))["names"]
        counts = json.loads(read("object-count.json"))
        samples, bounds = [], []
        for n in names:
            s = np.load(io.BytesIO(read("samples/%s.npy" % n)), allow_pickle=False)
            l = np.load(io.BytesIO(read("locs/%s.npy" % n)), allow_pickle=False)
            samples.append(torch.from_numpy(np.ascontiguousarray(s)).unsqueeze(0).float())
            bounds.append(torch.from_numpy(np.ascontiguousarray(l, dtype=np.float32)).reshape(-1, 8))
    finally:
        if z is not None:
            z.close()
    return names, counts, samples, bounds


def _log(msg):
    try:
        from logger import Logger
        Logger.log(msg)
    except Exception:  # logging is cosmetic
        pass


def _device(useGPU):
    if not torch.cuda.is_available():
        raise RuntimeError("scdx16p100: the augmentation and target kernels run on MI355X only (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _pack_locs(bounds_list, trunc):
    """(B, MAXTAGLEN, 8) rows + per-tile counts; trunc: centres truncated toward zero, as the reference's
    `loc[0] = int(loc[0])` before drawing (scdx16p100.py:201-202, :523-525)."""
    B = len(bounds_list)
    locs = np.zeros((B, MAXTAGLEN, 8), np.float32)
    counts = np.zeros(B, np.int32)
    for b, l in enumerate(bounds_list):
        l = (l.numpy() if torch.is_tensor(l) else np.asarray(l)).astype(np.float32)[:MAXTAGLEN]
        locs[b, :len(l)] = l
        counts[b] = len(l)
    if trunc:
        locs[:, :, :2] = np.trunc(locs[:, :, :2])
    return locs, counts


def splitOrder(count, dataSplit=None):
    """Training order and split profile (scdx16p100.py:143-180): FSI x ARGUM x CLIP positions (only the first
    `count` of a smaller test archive) kept when argum < ARGUMENTRATIO, shuffled with Python's global `random`,
    cut to PARTITION; then the split.  Returns (order, dataProfile)."""
    total = min(FSI * ARGUM * CLIP, count)
    order = [i for i in range(total) if (i // CLIP) % ARGUM < ARGUMENTRATIO]
    shuffle(order)
    order = order[0: int(len(order) * PARTITION)]
    if dataSplit is None:
        _log("The Data Split Profile Do Not Exist, We Randomly Select 10 pct. of Samples as Validation Set.")
        shuffle(order)
        numValidation = round(TESTSET)
        profile = {'validation': order[0:numValidation]}
        order = order[numValidation:]
        profile[TRAINSUBSET] = order
    else:
        _log("Extracting Validation Set from Data Split Profile ...")
        profile = dataSplit
        if TRAINSUBSET in profile.keys():
            order = profile[TRAINSUBSET]
        else:
            valid = set(profile['validation'])
            order = [x for x in order if x not in valid]
            profile[TRAINSUBSET] = order
    return order, profile


class SCD(Dataset):

    def __init__(self, zipPath, useGPU, dataSplit=None):
        from configuration import defaultConfig
        tempDir = defaultConfig.dirTemp + 'confocalCenter' + "/"
        self.names, self.objectCounts, self.samples, self.bounds = readArchive(zipPath, tempDir)
        self.count = len(self.names)
        self.useGPU = useGPU
        self.device = _device(useGPU)

        self.order, self.dataProfile = splitOrder(len(self.names), dataSplit)
        self.count = len(self.order)

        self._buildValidation()
        with open(defaultConfig.dirDataSplitProfile, "w+") as f:
            f.write(json.dumps(self.dataProfile))
        _log("Building Validation Set Completely with {} Samples".format(len(self.validObjNum)))

    # ------------------------------------------------------------------ validation (scdx16p100.py:185-262)
    def _buildValidation(self, chunk=256):
        from scdhip import ops
        ids = self.dataProfile['validation'][:REALTIMETEST]
        xs, heat, mask, regr, locs, inds = [], [], [], [], [], []
        self.validObjNum = [int(len(self.bounds[i])) for i in ids]
        for c0 in range(0, len(ids), chunk):
            part = ids[c0:c0 + chunk]
            tiles = torch.stack([self.samples[i] for i in part]).to(self.device)
            xs.append(ops.augment_tiles(tiles))
            l, n = _pack_locs([self.bounds[i] for i in part], trunc=True)
            L = torch.from_numpy(l).to(self.device)
            h, m, r, ind = ops.render_center_targets(L, torch.from_numpy(n).to(self.device), HEATMAPSIZE,
                                                     THRESHOLDIOU)
            # validation masks every stored object (scdx16p100.py:219-220)
            m = torch.arange(MAXTAGLEN, device=self.device)[None, :] < torch.from_numpy(n).to(self.device)[:, None]
            heat.append(h); mask.append(m); regr.append(r); locs.append(L); inds.append(ind)
        cat = (lambda ts, shape: torch.cat(ts) if ts else torch.zeros(shape, device=self.device))
        self.validation = {
            "xs": [cat(xs, (0, 1, 1, 1)), cat(inds, (0, MAXTAGLEN)).long()],
            "ys": [cat(heat, (0, 1, HEATMAPSIZE, HEATMAPSIZE)), cat(mask, (0, MAXTAGLEN)).bool(),
                   cat(regr, (0, MAXTAGLEN, 6)), cat(locs, (0, MAXTAGLEN, 8)), self.validObjNum]}

    def getValidationSet(self):
        """scdx16p100.py:381-414 (REALTIMETEST positions in validationBatchSize slices; empty slices of a small
        archive are dropped)."""
        from configuration import defaultConfig
        v = self.validation
        length = REALTIMETEST
        size = defaultConfig.validationBatchSize
        if length > size:
            out = []
            for k in range(length // size):
                s = slice(int(k * size), int((k + 1) * size))
                if len(v['ys'][4][s]) == 0:
                    continue
                out.append({'xs': [v['xs'][0][s]],
                            'ys': [v['ys'][0][s], v['ys'][1][s], v['ys'][2][s], v['ys'][3][s], v['ys'][4][s],
                                   v['xs'][1][s]]})
            return out
        return [{'xs': [v['xs'][0]], 'ys': [v['ys'][0], v['ys'][1], v['ys'][2], v['ys'][3], v['ys'][4], v['xs'][1]]}]

    # ------------------------------------------------------------------ training samples (scdx16p100.py:300-379)
    def __len__(self):
        return self.count

    @staticmethod
    def flipLocs(locs, fx, fy):
        """scdx16p100.py:424-436: mirrored centre, offset and major-axis components."""
        locs = (locs.numpy() if torch.is_tensor(locs) else np.asarray(locs)).astype(np.float32).reshape(-1, 8)
        if fx and len(locs):
            locs[:, 0] = HEATMAPSIZE - 1 - locs[:, 0]
            locs[:, 2] = -locs[:, 2]
            locs[:, 4] = -locs[:, 4]
        if fy and len(locs):
            locs[:, 1] = HEATMAPSIZE - 1 - locs[:, 1]
            locs[:, 3] = -locs[:, 3]
            locs[:, 5] = -locs[:, 5]
        return locs

    def _draws(self, B):
        """The reference's random draws per sample, in its order: two numpy uniforms (flips), one torch normal
        (jitter); the per-pixel noise comes from the device generator keyed by one torch-drawn seed."""
        flips = np.zeros((B, 2), np.uint8)
        jit = np.zeros(B, np.float32)
        for b in range(B):
            flips[b, 0] = np.random.uniform() > 0.5
            flips[b, 1] = np.random.uniform() > 0.5
            jit[b] = np.float32(1) + np.float32(JITTERSV) * torch.randn(1).numpy()[0]
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return flips, jit, seed

    def gpu_batch(self, indices, device=None):
        """A training batch augmented and target-rendered on the GPU in two launches each (scd_augment_tiles,
        scd_render_center_targets): {"xs": [(B,1,S,S)], "ys": [heat, mask, regr, inds]} on the device, the
        reference's __getitem__ stacked over `indices` (positions in the shuffled order)."""
        from scdhip import ops
        dev = device or self.device
        if 0 in indices:
            shuffle(self.order)      # the reference reshuffles when index 0 is fetched (scdx16p100.py:302-305)
        ids = [self.order[i] for i in indices]
        B = len(ids)
        flips, jit, seed = self._draws(B)
        tiles = torch.stack([self.samples[i] for i in ids]).to(dev)
        xs = ops.augment_tiles(tiles, torch.from_numpy(flips).to(dev), torch.from_numpy(jit).to(dev), None,
                               NOISESV, seed)
        l, n = _pack_locs([self.flipLocs(self.bounds[i], flips[b, 0], flips[b, 1]) for b, i in enumerate(ids)],
                          trunc=True)
        ys = ops.render_center_targets(torch.from_numpy(l).to(dev), torch.from_numpy(n).to(dev), HEATMAPSIZE,
                                       THRESHOLDIOU)
        return {"xs": [xs], "ys": ys}

    def __getitem__(self, index):
        b = self.gpu_batch([index])
        return {"xs": [b["xs"][0][0]], "ys": [y[0] for y in b["ys"]]}


dataset = SCD
