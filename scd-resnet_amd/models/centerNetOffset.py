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

    def prepare(self, targets):
        """Called by the training step before the model forward: the heads' forward then keeps the size / offset
        hidden activations only where this loss will gather them (targets[3] = inds; ops.hint_sparse_support)."""
        ops.hint_sparse_support(targets[3])

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
    """Validation metrics hook (centerNetOffset.py:253-354) on the GPU: the reference's predicted / ground-truth
    boxes, validMask = score >= 0.3 and the IoUConfidence / Orthogonity / IoU x3 / MAE pair tests
    (evaluations/detection.py:11-180) run as scd_ceval_count + scd_ceval_emit, one workgroup per image.  Same
    dict as the reference, every value the reference's masked_select stream in the same (n, k, l) order.
    ys = [heat, mask, regr (N,L,6), inds (N,L) or locs (N,L,8), ...]."""
    objNum = [int(v) for v in ys[1].reshape(ys[1].shape[0], -1).sum(1).tolist()]
    heat = outputDictionary.get("heatmap") if isinstance(outputDictionary, dict) else None
    size = heat.shape[-1] if heat is not None else HEATMAPSIZE
    s = ops.center_eval(ctScores, ctY, ctX, offset, regression, ys[2], ys[3], heatmap_size=size, threshold=0.3)
    return {'iouscore': [s[0], s[1]],
            'ortho': s[2],
            'ioucenter': s[3],
            'iouoffsetwo': s[4],
            'iouoffset': s[5],
            'maes': [s[6], s[7], s[8]],
            'objs': objNum}, outputDictionary


def expression(batches):
    """trainer/model/centerOffsetRes10.py:18-106: the per-batch streams are concatenated on the device and
    reduced by scd_ceval_summary (fp64 means, the reference's interpolated AP at 0.3/0.5/0.7/0.9; detections
    ranked by score, ties by descending pair index).  Same output string."""
    objNum = 0
    cols = [[] for _ in range(9)]
    for b in batches:
        objNum += int(sum(b['objs']))
        iou, score = b['iouscore']
        aemaj, aemin, aerad = b['maes']
        for c, v in zip(cols, (iou, score, b['ortho'], b['ioucenter'], b['iouoffsetwo'], b['iouoffset'],
                                aemaj, aemin, aerad)):
            c.append(v.reshape(-1))
    if batches:
        streams = [torch.cat(c) for c in cols]
    else:
        streams = [torch.zeros(0, device=torch.device("cuda", torch.cuda.current_device())) for _ in cols]
    m, ap = ops.center_eval_summary(streams, objNum, (0.3, 0.5, 0.7, 0.9))
    ev = {'mIoU': m[0], 'mIoUC': m[3], 'mIoUwoO': m[4], 'mIoUO': m[5], 'ap30': ap[0], 'ap50': ap[1], 'ap70': ap[2],
          'ap90': ap[3], 'orthogonity': m[2], 'majMAE': m[6], 'minMAE': m[7], 'radMAE': m[8], 'avgScore': m[1]}
    return ("[mIoU] {}    [mIoUC] {}    [mIoUwoO] {}    [mIoUO] {}    [AP30] {}    [AP50] {}    [AP70] {}    "
            "[AP90] {}    [Orth] {}    [majMAE] {}    [minMAE] {}    [radMAE] {}    [avgS] {}").format(
        format(ev['mIoU'] * 100, '-10.8f'),
        format(ev['mIoUC'] * 100, '-10.8f'),
        format(ev['mIoUwoO'] * 100, '-10.8f'),
        format(ev['mIoUO'] * 100, '-10.8f'),
        format(ev['ap30'] * 100, '-5.2f'),
        format(ev['ap50'] * 100, '-5.2f'),
        format(ev['ap70'] * 100, '-5.2f'),
        format(ev['ap90'] * 100, '-5.2f'),
        format(ev['orthogonity'], '-8.6f'),
        format(ev['majMAE'], '-8.6f'),
        format(ev['minMAE'], '-8.6f'),
        format(ev['radMAE'], '-8.6f'),
        format(ev['avgScore'], '-6.4f'))
