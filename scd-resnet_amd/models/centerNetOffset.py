"""CenterNet-with-offset on a ResNet backbone (models/centerNetOffset.py of the reference).

CenterNetResidual (:150-168), CenterNetLoss (:170-217), decodeCenterNet (:219-251) keep the
reference names, constructor arguments, return formats and state_dict keys; the compute runs
on libscdhip (scdhip.blocks / scdhip.loss / scdhip.ops.decode_topk).
"""
import torch

from models.backbones.residuals import BNMOMENTUM, ResNet, ResNetSpec, ResNetTerminal  # noqa: F401
from models.losses.focal import focalLoss
from models.losses.regression import L1LossMask
from scdhip import ops
from scdhip.loss import CenterNetLossFn

CLASSDIMENSION = 1
SIZEREGRFACTOR = 10
DOWNSAMPLE = 4
HEATMAPSIZE = 128


def process(inp, module, *xs, **kwargs):
    return module(inp)


def makeResnetTerminal(prediction, current, output):
    """centerNetOffset.py:103-122 (built on the host; the model is moved to the GPU as a whole)."""
    if current > 0:
        return torch.nn.Sequential(
            torch.nn.Conv2d(prediction, current, kernel_size=3, padding=1, bias=True),
            torch.nn.ReLU(inplace=True),
            torch.nn.Conv2d(current, output, kernel_size=1, stride=1, padding=0))
    return torch.nn.Conv2d(in_channels=prediction, out_channels=output, kernel_size=1, stride=1, padding=0)


def heatmapInitializerRes(m):
    torch.nn.init.constant_(m.bias, -2.19)


def regressionInitializerRes(m):
    torch.nn.init.normal_(m.weight, std=0.001)
    torch.nn.init.constant_(m.bias, 0)


def make_terminals(head_dim=128):
    return [ResNetTerminal("heatmap", CLASSDIMENSION, head_dim, heatmapInitializerRes, makeResnetTerminal, process),
            ResNetTerminal("regr", 4, head_dim, regressionInitializerRes, makeResnetTerminal, process),
            ResNetTerminal("offset", 2, head_dim, regressionInitializerRes, makeResnetTerminal, process)]


resnetHeatmapTerminal, resnetSizeTerminal, resnetOffsetTerminal = make_terminals(128)


class CenterNetResidual(ResNet):
    """CenterNetResidual(numLayers, dims) -- centerNetOffset.py:150-168."""

    HEAD_DIM = 128

    def __init__(self, numLayers, dims=[64, 64, 128, 256, 512, 256, 256, 256]):
        blockType, layers = ResNetSpec[numLayers]
        super(CenterNetResidual, self).__init__(1, blockType, layers, terminals=make_terminals(self.HEAD_DIM),
                                                decoder=decodeCenterNet, dimensions=dims)
        self.initialize(numLayers)


class CenterNetLoss(torch.nn.Module):
    """CenterNetLoss(regressionWeight, offsetWeight, focal, regression) -- centerNetOffset.py:170-217.

    Returns (loss (1,), [focalL, sizeL, offsetL]) like the reference.  Differences: no
    in-place sigmoid on the heatmap output (utility.py:121 mutates it; nothing reads it
    after the loss on the training path) and no host synchronisation.
    """

    def __init__(self, regressionWeight=1, offsetWeight=0.5, focal=focalLoss, regression=L1LossMask):
        super(CenterNetLoss, self).__init__()
        self.regressionWeight = regressionWeight
        self.offsetWeight = offsetWeight
        self.focal = focal
        self.regression = regression

    def forward(self, outs, targets):
        if self.focal is not focalLoss or self.regression is not L1LossMask:
            raise NotImplementedError("only focalLoss + L1LossMask run on the fused HIP loss")
        if len(outs) != 1:
            raise NotImplementedError("one output stack (ResNet) expected")
        out = outs[0]
        loss, stats = CenterNetLossFn.apply(out["heatmap"], out["regr"], out["offset"], targets[0], targets[1],
                                            targets[2], targets[3], float(self.regressionWeight),
                                            float(self.offsetWeight))
        return loss, [stats[0], stats[1], stats[2]]


def decodeCenterNet(outputDictionary, K=100, nmsKernelSize=3, **kwargs):
    """centerNetOffset.py:219-251: [scores, inds, ys, xs, offset(B,K,2), regr(B,K,4), outputDictionary].
    Top-K ties are ordered by ascending index (torch.topk leaves them unspecified)."""
    if nmsKernelSize != 3:
        raise NotImplementedError("decode kernel implements the 3x3 NMS of the reference")
    scores, inds, ys, xs, off, regr = ops.decode_topk(outputDictionary["heatmap"], outputDictionary.get("offset"),
                                                      outputDictionary.get("regr"), K)
    return [scores, inds, ys, xs, off, regr, outputDictionary]


def centerNetEvaluation(xs, ys, ctScores, ctIndices, ctY, ctX, offset, regression, outputDictionary):
    """Validation metrics hook (centerNetOffset.py:253-354).  The reference's IoU/AP/MAE
    metrics are outside the accelerated path; this returns the decoded
    detections' score statistics and object counts with the same dict shape."""
    objNum = [int(m.sum().item()) for m in ys[1]]
    valid = ctScores >= 0.3
    return {"objs": objNum, "scores": ctScores.detach(), "valid": valid.detach()}, outputDictionary


def expression(batches):
    objs = sum(sum(b["objs"]) for b in batches)
    scores = torch.cat([b["scores"].reshape(-1).float().cpu() for b in batches]) if batches else torch.zeros(1)
    valid = torch.cat([b["valid"].reshape(-1).cpu() for b in batches]) if batches else torch.zeros(1, dtype=bool)
    return "[objs] {}    [det>=0.3] {}    [avgS] {}".format(objs, int(valid.sum()),
                                                             format(float(scores.mean()), '-6.4f'))
