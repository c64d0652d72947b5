"""Golden vectors for the CornerNet-with-corner-pooling path, from the REAL reference
(build container only; needs /root/reference and oracle/build_ref_cpool.py's modules).

models/cornerNetCPool.py is not importable as shipped (:43, :45 import symbols that do not
exist); two names are provided so the module loads: DOWNSAMPLE (used only by its dataset-side
code) and two evaluation helpers (used only by cornerNetEvaluation).  The pools are the
reference's own C++ ops, compiled from their sources into oracle/_ref.

  F5 cpool.npz   top/bottom/left/right forward on random and tie-heavy inputs (C++ reference)
  F8 corner.npz  CornerNetResidual(10) forward (B=2, 128^2, train-mode BN) + CornerNetLoss
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
for _n in ["torchvision", "torchvision.transforms", "torchvision.transforms.functional"]:
    sys.modules[_n] = types.ModuleType(_n)
sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
sys.path.insert(0, "/root/reference")
sys.path.insert(1, REPO)

import torch  # noqa: E402

from oracle import build_ref_cpool  # noqa: E402
from oracle import cornernet as OC  # noqa: E402
from oracle import targets as T  # noqa: E402

mods = build_ref_cpool.build()
sys.modules.update(mods)
cc = types.ModuleType("datasets.confocalCenters")
ccc = types.ModuleType("datasets.confocalCenters.confocalCenter")
ccc.DOWNSAMPLE = 4
sys.modules["datasets.confocalCenters"] = cc
sys.modules["datasets.confocalCenters.confocalCenter"] = ccc
import evaluations.detection as det  # noqa: E402

det.averageIoU = lambda *a, **k: 0.0
det.averagePrecision = lambda *a, **k: 0.0
import models.cornerNetCPool as ref  # noqa: E402


def main():
    # ---- F5: pools forward (reference C++), random + ties
    rs = np.random.RandomState(3)
    x = torch.from_numpy(rs.standard_normal((2, 4, 16, 16)).astype(np.float32))
    xt = torch.from_numpy(rs.randint(0, 3, (2, 4, 16, 16)).astype(np.float32))   # heavy ties
    f5 = {"x": x.numpy(), "xt": xt.numpy()}
    for d, name in enumerate(["topPool", "bottomPool", "leftPool", "rightPool"]):
        f5["y%d" % d] = mods[name].forward(x)[0].numpy()
        f5["yt%d" % d] = mods[name].forward(xt)[0].numpy()
    np.savez_compressed(os.path.join(HERE, "cpool.npz"), **f5)

    # ---- F8: CornerNetResidual(10) forward + loss
    entries, topo = OC.model_spec(10)
    torch.manual_seed(0)
    m = ref.CornerNetResidual(10)
    assert [k for k, _ in entries] == list(m.state_dict().keys()), "state_dict layout mismatch"
    m.load_state_dict(OC.hash_weights(entries))
    m.train()
    x8 = T.batch_inputs(31, 2, 128)
    ys = T.corner_targets(32, 2, 32)
    outs = m(x8, decode=False)
    f8 = {k: v.detach().clone().numpy() for k, v in outs[0].items()}   # before the in-place sigmoid_
    loss, _ = ref.CornerNetLoss()(outs, ys)
    f8["loss"] = loss.detach().numpy()
    for i, n in enumerate(["heat", "mask", "regr", "tl", "br"]):
        f8["ys|" + n] = ys[i].numpy()
    for k, v in m.state_dict().items():
        if k.startswith(("tl.", "br.")) and (k.endswith("running_mean") or k.endswith("running_var")):
            f8["rs|" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "corner.npz"), **f8)
    print("corner fixtures written")


if __name__ == "__main__":
    main()
