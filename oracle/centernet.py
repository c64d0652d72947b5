"""CPU restatement of the reference CenterNet-on-ResNet training step (TEST INFRASTRUCTURE ONLY).

Functional PyTorch-fp32 restatement of:
  * ResNet backbone + deconv upsampler + terminals   models/backbones/residuals.py:84-353
  * CenterNet heads                                   models/centerNetOffset.py:103-168
  * CenterNetLoss (focal + masked L1)                 models/centerNetOffset.py:170-217,
                                                      models/losses/focal.py:25-53,
                                                      models/losses/regression.py:37-44,
                                                      models/backbones/utility.py:76-122
  * decodeCenterNet (sigmoid, NMS, top-K, gather)     models/centerNetOffset.py:219-251
  * one training iteration (zero_grad/fwd/loss/bwd/   models/networkFactory.py:79-82, 252-263
    Adam with torch defaults, lr=1e-3)

Parameters live in a flat dict keyed exactly like the reference state_dict so
fixtures and checkpoints interchange.  Pinned by tests/golden (see
tests/test_oracle_golden.py).
"""
import math
import zlib

import numpy as np
import torch
import torch.nn.functional as F

BN_MOMENTUM = 0.1          # residuals.py:32 BNMOMENTUM
BN_EPS = 1e-5              # torch.nn.BatchNorm2d default (residuals.py:92)

# ResNetSpec, residuals.py:355-365: depth -> (block, layers)
RESNET_SPEC = {
    18: ("basic", [2, 2, 2, 2]),
    34: ("basic", [3, 4, 6, 3]),
    50: ("bottleneck", [3, 4, 6, 3]),
    101: ("bottleneck", [3, 4, 23, 3]),
    152: ("bottleneck", [3, 8, 36, 3]),
    16: ("basic", [1, 2, 2, 2]),
    14: ("basic", [1, 2, 2, 1]),
    12: ("basic", [1, 1, 2, 1]),
    10: ("basic", [1, 1, 1, 1]),
}
EXPANSION = {"basic": 1, "bottleneck": 4}   # residuals.py:86, :126
DEFAULT_DIMS = [64, 64, 128, 256, 512, 256, 256, 256]   # residuals.py:201
CENTER_HEADS = [("heatmap", 1), ("regr", 4), ("offset", 2)]   # centerNetOffset.py:146-148
HEAD_DIM = 128                                                # centerNetOffset.py:146 terminalDimension


def model_spec(num_layers=10, dims=None, heads=CENTER_HEADS, head_dim=HEAD_DIM, in_dim=1):
    """Structural description of CenterNetResidual(numLayers, dims).

    Returns (entries, blocks): entries is the ordered list of (key, shape) of
    the reference state_dict (registration order of ResNet.__init__,
    residuals.py:200-253); blocks is the per-block topology used by forward().
    """
    dims = list(dims or DEFAULT_DIMS)
    block, layers = RESNET_SPEC[num_layers]
    exp = EXPANSION[block]
    entries = []

    def conv(key, cout, cin, k):
        entries.append((key + ".weight", (cout, cin, k, k)))

    def bn(key, c):
        entries.extend([(key + ".weight", (c,)), (key + ".bias", (c,)),
                        (key + ".running_mean", (c,)), (key + ".running_var", (c,)),
                        (key + ".num_batches_tracked", ())])

    conv("preprocess.0", dims[0], in_dim, 7)
    bn("preprocess.1", dims[0])
    inplanes = dims[0]
    blocks = []
    for li in range(4):
        planes = dims[li + 1]
        stride = 1 if li == 0 else 2
        for bi in range(layers[li]):
            p = "layer%d.%d" % (li + 1, bi)
            s = stride if bi == 0 else 1
            ds = bi == 0 and (s != 1 or inplanes != planes * exp)     # residuals.py:257
            if block == "basic":
                conv(p + ".conv1", planes, inplanes, 3); bn(p + ".bn1", planes)
                conv(p + ".conv2", planes, planes, 3); bn(p + ".bn2", planes)
            else:
                conv(p + ".conv1", planes, inplanes, 1); bn(p + ".bn1", planes)
                conv(p + ".conv2", planes, planes, 3); bn(p + ".bn2", planes)
                conv(p + ".conv3", planes * exp, planes, 1); bn(p + ".bn3", planes * exp)
            if ds:
                conv(p + ".downsample.0", planes * exp, inplanes, 1)
                bn(p + ".downsample.1", planes * exp)
            blocks.append(dict(prefix=p, kind=block, stride=s, downsample=ds,
                               cin=inplanes, planes=planes, cout=planes * exp))
            inplanes = planes * exp
    deconvs = []
    for i in range(3):                                   # makeDeconvLayer residuals.py:286-310
        cout = dims[5 + i]
        entries.append(("deconvolutionLayers.%d.weight" % (3 * i), (inplanes, cout, 4, 4)))
        bn("deconvolutionLayers.%d" % (3 * i + 1), cout)
        deconvs.append(("deconvolutionLayers.%d" % (3 * i), "deconvolutionLayers.%d" % (3 * i + 1)))
        inplanes = cout
    for name, odim in heads:                             # makeResnetTerminal centerNetOffset.py:103-122
        entries.append((name + ".0.weight", (head_dim, inplanes, 3, 3)))
        entries.append((name + ".0.bias", (head_dim,)))
        entries.append((name + ".2.weight", (odim, head_dim, 1, 1)))
        entries.append((name + ".2.bias", (odim,)))
    return entries, dict(blocks=blocks, deconvs=deconvs, heads=list(heads))


def hash_weights(entries):
    """Deterministic, platform-independent weights for fixtures (documented rule).

    conv/deconv weight : RandomState(crc32(key)).standard_normal(shape) / sqrt(prod(shape[1:]))
    BN gamma / beta    : 1 + 0.1 N  /  0.1 N
    BN running mean/var: 0.1 N      /  1 + 0.1 |N|
    conv bias          : 0.05 N, except heatmap.2.bias = -2.19 (centerNetOffset.py:124-125)
    """
    keys = {k for k, _ in entries}
    out = {}
    for key, shape in entries:
        rs = np.random.RandomState(zlib.crc32(key.encode()) & 0xFFFFFFFF)
        prefix, leaf = key.rsplit(".", 1)
        is_bn = (prefix + ".running_mean") in keys
        if leaf == "num_batches_tracked":
            out[key] = torch.zeros((), dtype=torch.int64)
            continue
        n = rs.standard_normal(shape if shape else ())
        if len(shape) == 4:
            v = n / math.sqrt(float(np.prod(shape[1:])))
        elif is_bn and leaf == "weight":
            v = 1.0 + 0.1 * n
        elif is_bn and leaf == "bias":
            v = 0.1 * n
        elif leaf == "running_mean":
            v = 0.1 * n
        elif leaf == "running_var":
            v = 1.0 + 0.1 * np.abs(n)
        elif key == "heatmap.2.bias":
            v = np.full(shape, -2.19)
        else:
            v = 0.05 * n
        out[key] = torch.from_numpy(np.asarray(v, dtype=np.float32).reshape(shape))
    return out


def split_state(state):
    """Split a state_dict into (params, buffers) the way nn.Module does."""
    params, buffers = {}, {}
    for k, v in state.items():
        if k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"):
            buffers[k] = v
        else:
            params[k] = v
    return params, buffers


def _bn(h, P, Bf, p, train):
    """BatchNorm2d(momentum=0.1) in train mode: batch stats (biased var) normalise,
    running stats updated with unbiased var (residuals.py:92,95,212,262,306)."""
    out = F.batch_norm(h, Bf[p + ".running_mean"], Bf[p + ".running_var"],
                       P[p + ".weight"], P[p + ".bias"], training=train,
                       momentum=BN_MOMENTUM, eps=BN_EPS)
    if train:
        Bf[p + ".num_batches_tracked"] += 1
    return out


def backbone(P, Bf, x, topo, train=True, taps=None):
    """ResNet.forward up to and including the deconv stack (residuals.py:312-325)."""
    def tap(name, t):
        if taps is not None:
            taps[name] = t
    h = F.conv2d(x, P["preprocess.0.weight"], stride=2, padding=3)           # residuals.py:211
    tap("preprocess.0", h)
    h = F.relu(_bn(h, P, Bf, "preprocess.1", train))
    tap("preprocess.2", h)
    h = F.max_pool2d(h, 3, stride=2, padding=1)                             # residuals.py:214
    tap("preprocess.3", h)
    for blk in topo["blocks"]:
        p, s = blk["prefix"], blk["stride"]
        idn = h
        if blk["kind"] == "basic":                                          # BasicBlock.forward :99-120
            o = F.conv2d(h, P[p + ".conv1.weight"], stride=s, padding=1)
            o = F.relu(_bn(o, P, Bf, p + ".bn1", train))
            o = F.conv2d(o, P[p + ".conv2.weight"], stride=1, padding=1)
            o = _bn(o, P, Bf, p + ".bn2", train)
        else:                                                               # Bottleneck.forward :145-165
            o = F.conv2d(h, P[p + ".conv1.weight"])
            o = F.relu(_bn(o, P, Bf, p + ".bn1", train))
            o = F.conv2d(o, P[p + ".conv2.weight"], stride=s, padding=1)
            o = F.relu(_bn(o, P, Bf, p + ".bn2", train))
            o = F.conv2d(o, P[p + ".conv3.weight"])
            o = _bn(o, P, Bf, p + ".bn3", train)
        if blk["downsample"]:
            idn = F.conv2d(h, P[p + ".downsample.0.weight"], stride=s)
            idn = _bn(idn, P, Bf, p + ".downsample.1", train)
        h = F.relu(o + idn)
        tap(p, h)
    for wk, bk in topo["deconvs"]:                                          # makeDeconvLayer :286-310
        h = F.conv_transpose2d(h, P[wk + ".weight"], stride=2, padding=1, output_padding=0)
        tap(wk, h)
        h = _bn(h, P, Bf, bk, train)
        tap(bk, h)
        h = F.relu(h)
    return h


def heads_forward(P, feat, heads, taps=None):
    """Terminal heads: conv3x3+bias -> ReLU -> conv1x1+bias (centerNetOffset.py:106-110)."""
    out = {}
    for name, _ in heads:
        hid = F.relu(F.conv2d(feat, P[name + ".0.weight"], P[name + ".0.bias"], padding=1))
        if taps is not None:
            taps[name + ".1"] = hid
        out[name] = F.conv2d(hid, P[name + ".2.weight"], P[name + ".2.bias"])
    return out


def forward(P, Bf, x, topo, train=True, taps=None):
    """CenterNetResidual.forward(x, decode=False)[0] (residuals.py:312-334)."""
    return heads_forward(P, backbone(P, Bf, x, topo, train, taps), topo["heads"], taps)


# ----------------------------------------------------------------------------- loss

def clamp_sigmoid(x):
    """clampSigmoid utility.py:120-122 (the reference applies sigmoid_ in place;
    here out-of-place, the value is identical)."""
    return torch.clamp(torch.sigmoid(x), min=1e-4, max=1 - 1e-4)


def focal_loss(preds, gt, alpha=2, beta=4):
    """Penalty-reduced focal loss, focal.py:25-53 (normaliser = batch-total #pos)."""
    pos = gt.eq(1)
    neg = gt.lt(1)
    negw = torch.pow(1 - gt[neg], beta)
    loss = 0
    for pred in preds:
        pp = pred[pos]
        npred = pred[neg]
        posl = (torch.log(pp) * torch.pow(1 - pp, alpha)).sum()
        negl = (torch.log(1 - npred) * torch.pow(npred, alpha) * negw).sum()
        npos = pos.float().sum()
        if pp.nelement() == 0:
            loss = loss - negl
        else:
            loss = loss - (posl + negl) / npos
    return loss


def gather_feat(feat, ind):
    """reshapeGatherFeatures, utility.py:76-84 + :94-98: (B,C,H,W),(B,K) -> (B,K,C)."""
    b, c = feat.shape[:2]
    f = feat.permute(0, 2, 3, 1).reshape(b, -1, c)
    return f.gather(1, ind.unsqueeze(2).expand(ind.shape[0], ind.shape[1], c))


def l1_loss_mask(regr, gt, mask):
    """L1LossMask, regression.py:37-44."""
    num = mask.float().sum()
    m = mask.bool().unsqueeze(2).expand_as(gt)
    return F.l1_loss(regr[m], gt[m], reduction="sum") / (num + 1e-4)


def centernet_loss(outs, ys, regr_w=0.1, off_w=0.1):
    """CenterNetLoss.forward, centerNetOffset.py:182-217 with the plugin weights
    0.1/0.1 (trainer/model/centerOffsetRes10.py:11).  Returns (loss(1,), [focal,size,offset])."""
    heat, mask, regr_t, inds = ys[0], ys[1], ys[2], ys[3]
    focal = focal_loss([clamp_sigmoid(outs["heatmap"])], heat)
    size = regr_w * l1_loss_mask(gather_feat(outs["regr"], inds), regr_t[:, :, 2:6], mask)
    off = off_w * l1_loss_mask(gather_feat(outs["offset"], inds), regr_t[:, :, 0:2], mask)
    loss = (focal + size + off) / 1
    return loss.unsqueeze(0), [focal, size, off]


# ----------------------------------------------------------------------------- decode

def nms(heat, k=3):
    """nonMaximumSuppression, utility.py:87-92."""
    hmax = F.max_pool2d(heat, (k, k), stride=1, padding=(k - 1) // 2)
    return heat * (hmax == heat).float()


def decode(outs, K=100, nms_k=3):
    """decodeCenterNet, centerNetOffset.py:219-251 + extractTopK utility.py:106-118.
    Returns [scores, inds, ys, xs, offset(B,K,2), regr(B,K,4)]."""
    heat = nms(torch.sigmoid(outs["heatmap"]), nms_k)
    b, c, h, w = heat.shape
    scores, inds = torch.topk(heat.view(b, -1), K)
    inds = inds % (h * w)
    ys = (inds // w).long()
    xs = (inds % w).long()
    return [scores, inds.long(), ys, xs, gather_feat(outs["offset"], inds), gather_feat(outs["regr"], inds)]


# ----------------------------------------------------------------------------- train step

class TrainState:
    """Leaf parameters + buffers + torch.optim.Adam with defaults (networkFactory.py:79-82:
    the reference passes no lr, so lr = 1e-3)."""

    def __init__(self, state, lr=1e-3):
        p, b = split_state({k: v.clone() for k, v in state.items()})
        self.P = {k: v.requires_grad_(True) for k, v in p.items()}
        self.B = b
        self.opt = torch.optim.Adam(list(self.P.values()), lr=lr)

    def step(self, x, ys, topo, world=1):
        """NetworkFactory.train (networkFactory.py:257-263)."""
        self.opt.zero_grad()
        outs = forward(self.P, self.B, x, topo)
        loss, stats = centernet_loss(outs, ys)
        loss.mean().backward()
        self.opt.step()
        return loss.detach(), [s.detach() for s in stats], outs
