"""Golden fixture for the `.d` dataset plugin, from the REAL reference (build container only).

Run:  python tests/golden/make_golden_scd.py      (needs /root/reference; never runs on the GPU box; ~2 min)

1. Writes the canonical-size synthetic archive of oracle/scd_archive.py (49,920 tiles of 8 x 8) with the
   product's writer (trainer/dataset/scdx16p100.writeArchive, loaded by file path).
2. Constructs the reference's datasets.scds.scdx16p100.SCD(zipPath, useGPU=False, dataSplit=None) after
   random.seed(77) (its shuffles use Python's global `random`), with dirTemp / dirDataSplitProfile pointed
   at /tmp: this pins the reader, the FSI/ARGUM/CLIP order rule, the split and the validation set.
3. Calls its __getitem__(3) after numpy.random.seed(5) / torch.manual_seed(6) and replays the same draws
   (two numpy uniforms, torch.randn(1), torch.randn(1,H,W)) so the GPU augmentation can be fed the
   reference's random numbers.
Writes tests/golden/scd.npz:
  valid_ids / train_ids (all), split_json (the profile file the reference wrote, bytes),
  valid_xs (all validation tiles, normalised), valid_heat_sum (per tile, float64), valid_heat0 (first 8 maps),
  valid_mask / valid_regr / valid_locs / valid_inds (first 512 tiles), valid_objnum (all),
  item_id, item_flips, item_g, item_noise, item_xs, item_heat, item_mask, item_regr, item_inds.
"""
import importlib.util
import json
import os
import random
import shutil
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
WORK = "/tmp/scd_golden"

sys.dont_write_bytecode = True
for _n in ["torchvision", "torchvision.transforms", "torchvision.transforms.functional"]:
    sys.modules[_n] = types.ModuleType(_n)
sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
sys.path.insert(0, REF)
sys.path.insert(1, REPO)

import torch  # noqa: E402

from configuration import defaultConfig  # noqa: E402  (reference)
from datasets.scds.scdx16p100 import SCD  # noqa: E402  (reference)

from oracle import scd_archive  # noqa: E402


def product_writer():
    spec = importlib.util.spec_from_file_location(
        "_scd_plugin", os.path.join(REPO, "scd-resnet_amd", "trainer", "dataset", "scdx16p100.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.writeArchive


def main():
    shutil.rmtree(WORK, ignore_errors=True)
    os.makedirs(WORK)
    path = os.path.join(WORK, "synthetic.d")
    names, samples, locs = scd_archive.archive_content()
    product_writer()(path, names, samples, locs)
    defaultConfig.config["dirTemp"] = os.path.join(WORK, "temp") + "/"
    defaultConfig.config["dirDataSplitProfile"] = os.path.join(WORK, "split.json")
    random.seed(77)
    ds = SCD(path, False, None)
    v = ds.validation
    out = {
        "valid_ids": np.array(ds.dataProfile["validation"], np.int64),
        "train_ids": np.array(ds.order, np.int64),
        "split_json": np.frombuffer(open(defaultConfig.config["dirDataSplitProfile"], "rb").read(), np.uint8),
        "valid_xs": v["xs"][0].numpy().astype(np.float32),
        "valid_heat_sum": v["ys"][0].double().sum((1, 2, 3)).numpy(),
        "valid_heat0": v["ys"][0][:8].numpy(),
        "valid_mask": v["ys"][1][:512].numpy(),
        "valid_regr": v["ys"][2][:512].numpy(),
        "valid_locs": v["ys"][3][:512].numpy(),
        "valid_inds": v["xs"][1][:512].numpy(),
        "valid_objnum": np.array(v["ys"][4], np.int64),
    }
    # one training item with its random draws replayed
    idx = 3
    item_id = ds.order[idx]
    H, W = samples[0].shape
    np.random.seed(5)
    torch.manual_seed(6)
    item = ds[idx]
    np.random.seed(5)
    torch.manual_seed(6)
    flips = np.array([np.random.uniform() > 0.5, np.random.uniform() > 0.5], np.uint8)
    g = torch.randn(1).numpy()
    noise = torch.randn(1, H, W).numpy()
    out.update({"item_id": np.array(item_id), "item_flips": flips, "item_g": g.astype(np.float32),
                "item_noise": noise.astype(np.float32), "item_xs": item["xs"][0].numpy(),
                "item_heat": item["ys"][0].numpy(), "item_mask": item["ys"][1].numpy(),
                "item_regr": item["ys"][2].numpy(), "item_inds": item["ys"][3].numpy()})
    np.savez_compressed(os.path.join(HERE, "scd.npz"), **out)
    print("validation %d, train %d, item %d flips %s objs %d" % (len(out["valid_ids"]), len(out["train_ids"]), item_id,
                                                                 flips, int(out["item_mask"].sum())))
    shutil.rmtree(WORK, ignore_errors=True)


if __name__ == "__main__":
    main()
