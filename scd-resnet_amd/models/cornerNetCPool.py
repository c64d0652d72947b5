"""CornerNet with corner pooling on a ResNet backbone (models/cornerNetCPool.py of the reference).

CornerPool (:83-122), TopLeftPool / BottomRightPool (:124-136), terminals (:163-217),
CornerNetResidual (:219-234), CornerNetLoss (:236-272), decodeCornerNet (:274-306), with the
reference's module tree and state_dict keys.  Runs on libscdhip: the CornerPool module is one
autograd Function (scdhip.blocks.CornerPoolFn: MFMA convolutions, training BN, the four
directional scan kernels), the tails reuse the fused head GEMM.  The reference file is not
importable as shipped (:43, :45); this one is, and ships a plugin (trainer/model/cornerNetCPool.py).
"""
import torch

from models.backbones.convolutions import Convolution
from models.backbones.residuals import ResNet, ResNetSpec, ResNetTerminal
from models.losses.focal import focalLoss
from scdhip import blocks, ops
from scdhip.loss import FocalOnlyLossFn

CLASSDIMENSION = 1
TOP, BOTTOM, LEFT, RIGHT = 0, 1, 2, 3


class _Pool(torch.nn.Module):
    """TopPool / BottomPool / LeftPool / RightPool (cornerPooling/__init__.py:60-73) on NHWC."""
    direction = None

    def forward(self, x):
        return blocks.CPoolFn.apply(x, self.direction)


class TopPool(_Pool):
    direction = TOP


class BottomPool(_Pool):
    direction = BOTTOM


class LeftPool(_Pool):
    direction = LEFT


class RightPool(_Pool):
    direction = RIGHT


class CornerPool(torch.nn.Module):
    def __init__(self, predictionDimension, pool1, pool2):
        super(CornerPool, self).__init__()
        self.branch1 = Convolution(3, predictionDimension, 128)
        self.branch2 = Convolution(3, predictionDimension, 128)
        self.branchMerge = torch.nn.Conv2d(128, predictionDimension, (3, 3), padding=(1, 1), bias=False)
        self.branchMergeBn = torch.nn.BatchNorm2d(predictionDimension)
        self.shortcutConv = torch.nn.Conv2d(predictionDimension, predictionDimension, (1, 1), bias=False)
        self.shortcutBn = torch.nn.BatchNorm2d(predictionDimension)
        self.mixReLU = torch.nn.ReLU(inplace=True)
        self.lastConv = Convolution(3, predictionDimension, predictionDimension)
        self.branchPooling1 = pool1()
        self.branchPooling2 = pool2()
        self.dirs = (self.branchPooling1.direction, self.branchPooling2.direction)

    def forward(self, x):
        """x: NHWC activation in the compute dtype."""
        return blocks.CornerPoolFn.apply(x, self.branch1.conv.weight, self, self.dirs)


class TopLeftPool(CornerPool):
    def __init__(self, dim):
        super(TopLeftPool, self).__init__(dim, TopPool, LeftPool)


class BottomRightPool(CornerPool):
    def __init__(self, dim):
        super(BottomRightPool, self).__init__(dim, BottomPool, RightPool)


def process(inp, module, *xs, **kwargs):
    return module(inp)


def _tail(prediction, current, output, pool=None):
    layers = [] if pool is None else [pool(prediction)]
    layers += [torch.nn.Conv2d(prediction, current, kernel_size=3, padding=1, bias=True), torch.nn.ReLU(inplace=True),
               torch.nn.Conv2d(current, output, kernel_size=1, stride=1, padding=0)]
    return torch.nn.Sequential(*layers)


def makeResnetTerminal(prediction, current, output):
    return _tail(prediction, current, output)


def makeTopLeftTerminal(prediction, current, output):
    return _tail(prediction, current, output, TopLeftPool)


def makeBottomRightTerminal(prediction, current, output):
    return _tail(prediction, current, output, BottomRightPool)


def heatmapInitializerRes(m):
    torch.nn.init.constant_(m.bias, -2.19)


resnetHeatmapTerminal = ResNetTerminal("heatmap", CLASSDIMENSION, 128, heatmapInitializerRes, makeResnetTerminal,
                                       process)
resnetTLTerminal = ResNetTerminal("tl", CLASSDIMENSION, 128, heatmapInitializerRes, makeTopLeftTerminal, process)
resnetBRTerminal = ResNetTerminal("br", CLASSDIMENSION, 128, heatmapInitializerRes, makeBottomRightTerminal, process)


class CornerNetResidual(ResNet):
    def __init__(self, numLayers):
        blockType, layers = ResNetSpec[numLayers]
        super(CornerNetResidual, self).__init__(1, blockType, layers,
                                                terminals=[resnetHeatmapTerminal, resnetTLTerminal, resnetBRTerminal],
                                                decoder=decodeCornerNet)
        self.initialize(numLayers)


class CornerNetLoss(torch.nn.Module):
    """focal(heatmap, ys[0]) + focal(tl, ys[3]) + focal(br, ys[4])  (cornerNetCPool.py:244-272)."""

    def __init__(self, focal=focalLoss):
        super(CornerNetLoss, self).__init__()
        self.focal = focal

    def forward(self, outs, targets):
        if self.focal is not focalLoss or len(outs) != 1:
            raise NotImplementedError("fused HIP focal loss over one output stack")
        o = outs[0]
        loss, _ = FocalOnlyLossFn.apply(o["heatmap"], o["tl"], o["br"], targets[0], targets[3], targets[4])
        return loss, {}


def decodeCornerNet(outputDictionary, K=100, nmsKernelSize=3, **kwargs):
    """[ct scores/inds/ys/xs, tl ..., br ..., outputDictionary] (cornerNetCPool.py:274-306)."""
    if nmsKernelSize != 3:
        raise NotImplementedError("3x3 NMS")
    res = []
    for key in ("heatmap", "tl", "br"):
        s, i, y, x, _, _ = ops.decode_topk(outputDictionary[key], None, None, K)
        res += [s, i, y, x]
    return res + [outputDictionary]


def cornerNetEvaluation(xs, ys, *decoded):
    """Validation metrics hook (cornerNetCPool.py:308-322): object counts and score statistics
    (the reference's AP metrics are SURVEY §8f row 3)."""
    outputDictionary = decoded[-1]
    return {"objs": [int(m.sum().item()) for m in ys[1]], "scores": decoded[0].detach(),
            "valid": (decoded[0] >= 0.3).detach()}, outputDictionary
