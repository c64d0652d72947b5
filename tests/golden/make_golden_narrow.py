"""Golden fixture F11 for the narrow-channel plugins (`*q`, `*h`), from the REAL reference (build container only).

Run:  python tests/golden/make_golden_narrow.py      (needs /root/reference; never runs on the GPU box)

The reference's centerOffsetRes10q / centerOffsetRes10h plugins build models.centerNetOffseth.CenterNetResidual
(64-wide head terminals, centerNetOffseth.py:146-148) with dims [16, 16, 32, 64, 128, 64, 64, 64] and
[32, 32, 64, 128, 256, 128, 128, 128] (trainer/model/centerOffsetRes10q.py, centerOffsetRes10h.py).  As for F9,
weights come from the crc32 hash rule and inputs / targets from seeds; one training-mode forward +
CenterNetLoss + backward at B=2, 256^2 input (heads at 64^2).
  F11 narrow.npz   <plugin>|heatmap/regr/offset, <plugin>|loss, <plugin>|stats, <plugin>|gnorm|<param>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as G  # noqa: E402  (stubs torchvision, puts the reference on sys.path)
from models.centerNetOffseth import CenterNetLoss, CenterNetResidual  # noqa: E402
from models.losses.focal import focalLoss  # noqa: E402
from models.losses.regression import L1LossMask  # noqa: E402

from oracle import centernet as O  # noqa: E402
from oracle import targets as T  # noqa: E402

PLUGINS = {"centerOffsetRes10q": {'numLayers': 10, 'dims': [16, 16, 32, 64, 128, 64, 64, 64]},
           "centerOffsetRes10h": {'numLayers': 10, 'dims': [32, 32, 64, 128, 256, 128, 128, 128]}}


def main():
    out = {}
    for name, params in PLUGINS.items():
        entries, topo = O.model_spec(10, params["dims"], head_dim=64)
        state = O.hash_weights(entries)
        m = CenterNetResidual(**params)
        m.load_state_dict(state)
        m.train()
        loss_fn = CenterNetLoss(0.1, 0.1, focal=focalLoss, regression=L1LossMask)
        x = T.batch_inputs(21, 2, 256)
        ys = G.ref_targets(22, 2, 64)
        o = m(x, decode=False)
        for k in ("heatmap", "regr", "offset"):
            out["%s|%s" % (name, k)] = o[0][k].detach().clone().numpy()
        loss, stats = loss_fn(o, ys)
        loss.mean().backward()
        out[name + "|loss"] = loss.detach().numpy()
        out[name + "|stats"] = np.array([s.item() for s in stats])
        for k, p in m.named_parameters():
            out["%s|gnorm|%s" % (name, k)] = np.array(p.grad.double().norm().item())
        print(name, float(loss.detach()))
    np.savez_compressed(os.path.join(HERE, "narrow.npz"), **out)


if __name__ == "__main__":
    main()
