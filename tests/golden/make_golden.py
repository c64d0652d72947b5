"""Generate the golden fixtures by running the REAL reference (build container only).

Run:  python tests/golden/make_golden.py        (needs /root/reference; never runs on the GPU box)

The reference is imported read-only (no bytecode written) with a stub
``torchvision`` (the hot path never calls it: only argumentations.rotate does,
argumentations.py:158).  Outputs are small .npz fixtures in tests/golden/; the
oracle (oracle/) is then pinned against them by tests/test_oracle_golden.py.
Inputs are regenerated from seeds (numpy legacy RandomState) and weights from
the crc32 hash rule (oracle.centernet.hash_weights), so no 40 MB checkpoint
is stored.

Fixtures:
  F0 init.npz     reference init under the import-order seed 42: per-key sum/sumsq/first values
  F1 fwd.npz      Res10 forward, train-mode BN, B=2 512^2 (seed 1): heads + post-fwd running stats
  F2 loss*.npz    CenterNetLoss + d/d{heatmap,regr,offset} for targets rendered by the reference
  F3 step.npz     one NetworkFactory.train step (fwd, loss, bwd, Adam lr 1e-3): grad norms/samples
  F4 decode.npz   decodeCenterNet on F1 outputs and on a tie-free synthetic map
  F6 layers.npz   per-module outputs at 128^2 input (stats + 32 sampled values)
  F7 ddp.npz      DDP-avg + SyncBN semantics for W=2 (global-batch BN, per-shard loss averaged)
"""
import os
import sys
import types
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True
for _n in ["torchvision", "torchvision.transforms", "torchvision.transforms.functional"]:
    sys.modules[_n] = types.ModuleType(_n)
sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
sys.path.insert(0, REF)
sys.path.insert(1, REPO)

import torch  # noqa: E402

torch.set_num_threads(os.cpu_count() or 8)

import trainer.model.centerOffsetRes10 as plugin  # noqa: E402  (reference plugin)
from datasets.scds.scdx16p100 import SCD  # noqa: E402
from evaluations.intersection import centerThresholdRadius  # noqa: E402
from models.centerNetOffset import decodeCenterNet  # noqa: E402

from oracle import centernet as O  # noqa: E402
from oracle import targets as T  # noqa: E402


def sample_positions(name, numel, k):
    rs = np.random.RandomState(zlib.crc32(name.encode()) & 0xFFFFFFFF)
    return rs.randint(0, numel, k)


def ref_targets(seed, batch, size):
    """Targets rendered with the REFERENCE drawGaussian/centerThresholdRadius on
    the oracle's seeded object list (pins oracle.targets.render)."""
    rs = np.random.RandomState(seed)
    heats, masks, regrs, inds = [], [], [], []
    for _ in range(batch):
        locs = torch.from_numpy(T.random_locs(rs, size=size))
        heat = torch.zeros(size, size)
        for loc in locs.clone():
            loc[0] = int(loc[0]); loc[1] = int(loc[1])
            import math
            radius = centerThresholdRadius(2 * math.sqrt(loc[4] ** 2 + loc[5] ** 2), 2 * loc[6].item(), 0.5)
            SCD.drawGaussian((loc[0], loc[1]), heat, radius)
        m = torch.zeros(30).bool(); m[:len(locs)] = 1
        ind = torch.zeros(30).long()
        ind[:len(locs)] = (torch.floor(locs[:, 1]) * size + torch.floor(locs[:, 0])).long()
        ind[m == 0] = 0
        rg = torch.zeros(30, 6); rg[:len(locs)] = locs[:, 2:8]
        heats.append(heat[None]); masks.append(m); regrs.append(rg); inds.append(ind)
    return [torch.stack(heats), torch.stack(masks), torch.stack(regrs), torch.stack(inds)]


def ref_model(state):
    torch.manual_seed(0)
    m = plugin.model(**plugin.modelParams)
    m.load_state_dict(state)
    m.train()
    return m


def main():
    entries, topo = O.model_spec(10)
    state = O.hash_weights(entries)
    save = {}

    # ---- F0: reference init under the import-order seed (networkFactory.py:34, scdx16p100.py:43)
    torch.random.manual_seed(42)
    m0 = plugin.model(**plugin.modelParams)
    sd = m0.state_dict()
    assert [k for k, _ in entries] == list(sd.keys())
    f0 = {}
    for k, v in sd.items():
        v = v.detach().double()
        f0[k + "|sum"] = np.array(v.sum().item())
        f0[k + "|sumsq"] = np.array((v * v).sum().item())
        f0[k + "|head"] = v.reshape(-1)[:4].numpy().astype(np.float32)
    f0["param_count"] = np.array(sum(p.numel() for p in m0.parameters()))
    np.savez_compressed(os.path.join(HERE, "init.npz"), **f0)

    # ---- F1: forward
    x = T.batch_inputs(1, 2, 512)
    m = ref_model(state)
    with torch.no_grad():
        out = m(x, decode=False)[0]
    f1 = {k: out[k].numpy() for k in ("heatmap", "regr", "offset")}
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            f1["rs|" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "fwd.npz"), **f1)

    # ---- F4: decode on F1 outputs + tie-free synthetic map
    f4 = {}
    dec = decodeCenterNet({k: out[k].clone() for k in ("heatmap", "regr", "offset")})
    for name, t in zip(["scores", "inds", "ys", "xs", "offset", "regr"], dec[:6]):
        f4["f1|" + name] = t.numpy()
    rs = np.random.RandomState(7)
    syn = {"heatmap": torch.from_numpy((rs.standard_normal((2, 1, 128, 128)) * 3).astype(np.float32)),
           "regr": torch.from_numpy(rs.standard_normal((2, 4, 128, 128)).astype(np.float32)),
           "offset": torch.from_numpy(rs.standard_normal((2, 2, 128, 128)).astype(np.float32))}
    dec = decodeCenterNet({k: v.clone() for k, v in syn.items()})
    for name, t in zip(["scores", "inds", "ys", "xs", "offset", "regr"], dec[:6]):
        f4["syn|" + name] = t.numpy()
    np.savez_compressed(os.path.join(HERE, "decode.npz"), **f4)

    # ---- F2: loss + head-output grads (reference CenterNetLoss(0.1, 0.1))
    def loss_case(preds, ys, tag, full):
        leaves = {k: v.clone().requires_grad_(True) for k, v in preds.items()}
        outs = {k: v * 1 for k, v in leaves.items()}       # non-leaf: sigmoid_ is in-place
        loss, stats = plugin.loss([outs], ys)
        loss.mean().backward()
        d = {tag + "|loss": loss.detach().numpy(),
             tag + "|stats": np.array([s.item() for s in stats], dtype=np.float64)}
        gh = leaves["heatmap"].grad
        if full:
            d[tag + "|dheatmap"] = gh.numpy()
        d[tag + "|dheatmap_sum"] = np.array(gh.double().sum().item())
        d[tag + "|dheatmap_abs"] = np.array(gh.double().abs().sum().item())
        for k in ("regr", "offset"):
            g = leaves[k].grad
            d[tag + "|d" + k] = O.gather_feat(g, ys[3]).numpy()
            d[tag + "|d" + k + "_abs"] = np.array(g.double().abs().sum().item())
        return d

    f2 = {}
    ys = ref_targets(2, 2, 128)
    for i, n in enumerate(["heat", "mask", "regr", "inds"]):
        f2["ys|" + n] = ys[i].numpy()
    preds = {k: out[k] for k in ("heatmap", "regr", "offset")}
    f2.update(loss_case(preds, ys, "a", True))
    ys_b = [ys[0] * 0.9, ys[1], ys[2], ys[3]]                         # zero positives
    f2.update(loss_case(preds, ys_b, "b", False))
    ys_c = [y.clone() for y in ys]                                     # duplicate indices
    ys_c[3][:, 1] = ys_c[3][:, 0]
    f2.update(loss_case(preds, ys_c, "c", False))
    f2["c|inds"] = ys_c[3].numpy()
    sat = {k: v.clone() for k, v in preds.items()}                     # saturated logits
    sat["heatmap"] = torch.where(sat["heatmap"] > sat["heatmap"].median(), torch.full_like(sat["heatmap"], 20.0),
                                 torch.full_like(sat["heatmap"], -20.0))
    f2.update(loss_case(sat, ys, "d", False))
    np.savez_compressed(os.path.join(HERE, "loss.npz"), **f2)

    # ---- F3: one training step (NetworkFactory.train, networkFactory.py:257-263)
    x3 = T.batch_inputs(3, 2, 512)
    ys3 = ref_targets(4, 2, 128)
    m = ref_model(state)
    opt = torch.optim.Adam(filter(lambda p: p.requires_grad, m.parameters()))
    opt.zero_grad()
    loss, stats = plugin.loss(m(x3, decode=False), ys3)
    loss.mean().backward()
    f3 = {"loss": loss.detach().numpy(), "stats": np.array([s.item() for s in stats])}
    pre = {k: v.detach().clone() for k, v in m.named_parameters()}
    grads = {k: v.grad.detach().clone() for k, v in m.named_parameters()}
    opt.step()
    for k, v in m.named_parameters():
        pos = sample_positions(k, v.numel(), 16)
        f3["gnorm|" + k] = np.array(grads[k].double().norm().item())
        f3["gsamp|" + k] = grads[k].reshape(-1)[pos].numpy()
        f3["psamp|" + k] = v.detach().reshape(-1)[pos].numpy()
        f3["p0samp|" + k] = pre[k].reshape(-1)[pos].numpy()
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            f3["rs|" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "step.npz"), **f3)

    # ---- F6: per-module outputs at 128^2 input
    x6 = T.batch_inputs(6, 2, 128)
    m = ref_model(state)
    f6 = {}
    hooks = []

    def mk(name):
        def hook(mod, inp, outp):
            t = outp.detach().double()
            pos = sample_positions(name, t.numel(), 32)
            f6[name + "|mean"] = np.array(t.mean().item())
            f6[name + "|std"] = np.array(t.std().item())
            f6[name + "|samp"] = t.reshape(-1)[pos].float().numpy()
            f6[name + "|shape"] = np.array(t.shape)
        return hook
    names = ["preprocess.0", "preprocess.2", "preprocess.3", "layer1.0", "layer2.0", "layer3.0", "layer4.0",
             "deconvolutionLayers.0", "deconvolutionLayers.1", "deconvolutionLayers.3", "deconvolutionLayers.4",
             "deconvolutionLayers.6", "deconvolutionLayers.7", "heatmap.1", "regr.1", "offset.1",
             "heatmap.2", "regr.2", "offset.2"]
    mods = dict(m.named_modules())
    for n in names:
        hooks.append(mods[n].register_forward_hook(mk(n)))
    with torch.no_grad():
        m(x6, decode=False)
    for h in hooks:
        h.remove()
    np.savez_compressed(os.path.join(HERE, "layers.npz"), **f6)

    # ---- F7: DDP (grad average over ranks) + SyncBN (BN over the global batch), W=2
    x7 = T.batch_inputs(8, 4, 128)
    ys7 = ref_targets(9, 4, 32)
    m = ref_model(state)
    outs = m(x7, decode=False)[0]
    losses = []
    for r in range(2):
        sl = slice(2 * r, 2 * r + 2)
        shard = {k: v[sl].clone() for k, v in outs.items()}
        l, _ = plugin.loss([shard], [y[sl] for y in ys7])
        losses.append(l.mean())
    total = (losses[0] + losses[1]) / 2
    total.backward()
    f7 = {"loss_r0": np.array(losses[0].item()), "loss_r1": np.array(losses[1].item())}
    for k, v in m.named_parameters():
        pos = sample_positions(k, v.numel(), 16)
        f7["gnorm|" + k] = np.array(v.grad.double().norm().item())
        f7["gsamp|" + k] = v.grad.reshape(-1)[pos].numpy()
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            f7["rs|" + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "ddp.npz"), **f7)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
