"""CPU restatement of the reference CornerNet-with-corner-pooling model (TEST INFRASTRUCTURE ONLY).

models/cornerNetCPool.py: CornerPool (:83-122), TopLeftPool/BottomRightPool (:124-136),
terminals (:163-217), CornerNetResidual (:219-234), CornerNetLoss (:236-272),
decodeCornerNet (:274-306); Convolution = conv+BN+ReLU (backbones/convolutions.py:25-49);
pools per oracle/cpool.py.  Pinned by tests/golden/corner.npz (reference forward with the
compiled reference pool ops, oracle/build_ref_cpool.py).
"""
import torch
import torch.nn.functional as F

from . import centernet as C
from . import cpool

POOLS = {"tl": (0, 2), "br": (1, 3)}      # TopLeftPool = (TopPool, LeftPool); BottomRightPool = (Bottom, Right)


def model_spec(num_layers=10, dims=None):
    """state_dict layout of CornerNetResidual(numLayers) (default dims, residuals.py:201)."""
    entries, topo = C.model_spec(num_layers, dims, heads=[("heatmap", 1)])
    d = (dims or C.DEFAULT_DIMS)[7]

    def conv(k, co, ci, ks):
        entries.append((k + ".weight", (co, ci, ks, ks)))

    def bn(k, c):
        entries.extend([(k + ".weight", (c,)), (k + ".bias", (c,)), (k + ".running_mean", (c,)),
                        (k + ".running_var", (c,)), (k + ".num_batches_tracked", ())])
    for name in ("tl", "br"):
        p = name + ".0"
        conv(p + ".branch1.conv", 128, d, 3); bn(p + ".branch1.bn", 128)
        conv(p + ".branch2.conv", 128, d, 3); bn(p + ".branch2.bn", 128)
        conv(p + ".branchMerge", d, 128, 3); bn(p + ".branchMergeBn", d)
        conv(p + ".shortcutConv", d, d, 1); bn(p + ".shortcutBn", d)
        conv(p + ".lastConv.conv", d, d, 3); bn(p + ".lastConv.bn", d)
        entries.append((name + ".1.weight", (128, d, 3, 3)))
        entries.append((name + ".1.bias", (128,)))
        entries.append((name + ".3.weight", (1, 128, 1, 1)))
        entries.append((name + ".3.bias", (1,)))
    topo["corner_heads"] = ["tl", "br"]
    return entries, topo


def hash_weights(entries):
    st = C.hash_weights(entries)
    for k in ("tl.3.bias", "br.3.bias"):           # heatmapInitializerRes on the 1-channel tails
        st[k] = torch.full_like(st[k], -2.19)
    return st


def _convbn(h, P, Bf, p, relu=True, stride=1):
    o = F.conv2d(h, P[p + ".conv.weight"], stride=stride, padding=P[p + ".conv.weight"].shape[2] // 2)
    o = C._bn(o, P, Bf, p + ".bn", True)
    return F.relu(o) if relu else o


def corner_pool(x, P, Bf, p, dirs):
    """CornerPool.forward (cornerNetCPool.py:103-122)."""
    p1 = cpool.forward(_convbn(x, P, Bf, p + ".branch1"), dirs[0])
    p2 = cpool.forward(_convbn(x, P, Bf, p + ".branch2"), dirs[1])
    m = C._bn(F.conv2d(p1 + p2, P[p + ".branchMerge.weight"], padding=1), P, Bf, p + ".branchMergeBn", True)
    s = C._bn(F.conv2d(x, P[p + ".shortcutConv.weight"]), P, Bf, p + ".shortcutBn", True)
    return _convbn(F.relu(m + s), P, Bf, p + ".lastConv")


def forward(P, Bf, x, topo):
    feat = C.backbone(P, Bf, x, topo)
    out = C.heads_forward(P, feat, [("heatmap", 1)])
    for name in topo["corner_heads"]:
        h = corner_pool(feat, P, Bf, name + ".0", POOLS[name])
        h = F.relu(F.conv2d(h, P[name + ".1.weight"], P[name + ".1.bias"], padding=1))
        out[name] = F.conv2d(h, P[name + ".3.weight"], P[name + ".3.bias"])
    return out


def cornernet_loss(outs, ys):
    """CornerNetLoss.forward (cornerNetCPool.py:244-272): three focal losses, /1."""
    f = C.focal_loss([C.clamp_sigmoid(outs["heatmap"])], ys[0])
    f = f + C.focal_loss([C.clamp_sigmoid(outs["tl"])], ys[3])
    f = f + C.focal_loss([C.clamp_sigmoid(outs["br"])], ys[4])
    return (f / 1).unsqueeze(0)
