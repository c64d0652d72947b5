"""Generate the Res50 (Bottleneck) golden fixture F9 by running the REAL reference (build container only).

Run:  python tests/golden/make_golden_res50.py      (needs /root/reference; never runs on the GPU box)

The reference's centerOffsetRes50 plugin pulls in evaluation helpers that are not on the hot path, so
the fixture builds what the plugin exports directly: CenterNetResidual(numLayers=50, dims=[64, 64, 128,
256, 512, 256, 256, 256]) and CenterNetLoss(0.1, 0.1, focalLoss, L1LossMask)
(trainer/model/centerOffsetRes50.py of the reference).  Weights come from the crc32 hash rule
(oracle.centernet.hash_weights), inputs/targets from seeds, as in make_golden.py.

  F9 res50.npz   one training-mode forward + CenterNetLoss + backward at B=2, 128^2 input (heads at
                 32^2): head outputs, loss and its three terms, every parameter's gradient norm and 8
                 sampled gradient values, and the post-forward running statistics of four BN layers
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as G  # noqa: E402  (stubs torchvision, puts the reference on sys.path)
from models.centerNetOffset import CenterNetLoss, CenterNetResidual  # noqa: E402
from models.losses.focal import focalLoss  # noqa: E402
from models.losses.regression import L1LossMask  # noqa: E402

from oracle import centernet as O  # noqa: E402
from oracle import targets as T  # noqa: E402

PARAMS = {'numLayers': 50, 'dims': [64, 64, 128, 256, 512, 256, 256, 256]}
BN_KEYS = ["preprocess.1", "layer1.0.bn3", "layer3.5.bn2", "layer4.2.bn3"]


def main():
    entries, topo = O.model_spec(50, PARAMS["dims"])
    state = O.hash_weights(entries)
    torch.manual_seed(0)
    m = CenterNetResidual(**PARAMS)
    m.load_state_dict(state)
    m.train()
    loss_fn = CenterNetLoss(0.1, 0.1, focal=focalLoss, regression=L1LossMask)
    x = T.batch_inputs(9, 2, 128)
    ys = G.ref_targets(10, 2, 32)
    out = m(x, decode=False)
    # copies: the reference's loss applies clampSigmoid to the heatmap in place (utility.py:120-122)
    f9 = {k: out[0][k].detach().clone().numpy() for k in ("heatmap", "regr", "offset")}
    loss, stats = loss_fn(out, ys)
    loss.mean().backward()
    f9["loss"] = loss.detach().numpy()
    f9["stats"] = np.array([s.item() for s in stats])
    for k, p in m.named_parameters():
        pos = G.sample_positions(k, p.numel(), 8)
        f9["gnorm|" + k] = np.array(p.grad.double().norm().item())
        f9["gsamp|" + k] = p.grad.reshape(-1)[pos].numpy()
    sd = m.state_dict()
    for b in BN_KEYS:
        f9["rs|" + b + ".running_mean"] = sd[b + ".running_mean"].numpy()
        f9["rs|" + b + ".running_var"] = sd[b + ".running_var"].numpy()
    np.savez_compressed(os.path.join(HERE, "res50.npz"), **f9)
    print("F9 res50.npz:", len(f9), "arrays, loss", float(loss.detach()))


if __name__ == "__main__":
    main()
