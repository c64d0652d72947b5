"""Golden fixtures F7b / F7c: DDP + SyncBN semantics at world size 4 / 8, from the REAL reference (build container
only).

Run:  python tests/golden/make_golden_ddp4.py [8]    (needs /root/reference; never runs on the GPU box)

The reference trains multi-GPU runs as DistributedDataParallel over SyncBatchNorm (networkFactory.py:126-136): every
BN layer normalises with the statistics of the GLOBAL batch, each rank's loss is CenterNetLoss over its own shard,
and the gradients are averaged over the ranks.  That is exactly one training-mode forward of the reference model on
the global batch (train-mode BN over all of it), the per-shard losses, and the backward of their mean -- which is
what this script runs (SyncBatchNorm itself refuses CPU tensors).  W = 4 (or 8) ranks x 2 images at 128^2 (heads at
32^2); weights from the crc32 hash rule, inputs / targets from seeds 31 / 32 (W = 8: 51 / 52).
  F7b ddp4.npz, F7c ddp8.npz   loss_r<k>, gnorm|<param>, gsamp|<param>, rs|<running stat>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import make_golden as G  # noqa: E402  (stubs torchvision, puts the reference on sys.path)

from oracle import centernet as O  # noqa: E402
from oracle import targets as T  # noqa: E402

WORLD = int(sys.argv[1]) if len(sys.argv) > 1 else 4
PER_RANK, SIZE = 2, 128
SEEDS = {4: (31, 32), 8: (51, 52)}[WORLD]


def main():
    entries, _ = O.model_spec(10)
    state = O.hash_weights(entries)
    x = T.batch_inputs(SEEDS[0], WORLD * PER_RANK, SIZE)
    ys = G.ref_targets(SEEDS[1], WORLD * PER_RANK, SIZE // 4)
    m = G.ref_model(state)
    outs = m(x, decode=False)[0]
    losses = []
    for r in range(WORLD):
        sl = slice(PER_RANK * r, PER_RANK * (r + 1))
        shard = {k: v[sl].clone() for k, v in outs.items()}
        l, _ = G.plugin.loss([shard], [y[sl] for y in ys])
        losses.append(l.mean())
    total = sum(losses) / WORLD
    total.backward()
    f = {"loss_r%d" % r: np.array(losses[r].item()) for r in range(WORLD)}
    for k, v in m.named_parameters():
        pos = G.sample_positions(k, v.numel(), 16)
        f["gnorm|" + k] = np.array(v.grad.double().norm().item())
        f["gsamp|" + k] = v.grad.reshape(-1)[pos].numpy()
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            f["rs|" + k] = v.numpy()
    name = "ddp%d.npz" % WORLD
    np.savez_compressed(os.path.join(HERE, name), **f)
    print(name, [round(float(l), 5) for l in losses])


if __name__ == "__main__":
    main()
