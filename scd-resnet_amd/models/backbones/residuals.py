"""ResNet backbone + transposed-conv upsampler + terminal wiring, executed on libscdhip.

Mirrors models/backbones/residuals.py of the reference (BasicBlock :84-120, Bottleneck
:122-165, ResNetTerminal :167-182, ResNet :184-353, ResNetSpec :355-365): the same module
tree is registered in the same order, so state_dict keys, parameter counts and the default
initialisation (including the RNG draw order of ResNet.initialize) are identical.  The
forward pass is different: it runs block-granular HIP autograd Functions (scdhip.blocks)
on NHWC activations in the model's compute dtype (bf16 by default, fp32 for parity).
"""
import sys

import torch

from logger import Logger
from models.backbones.terminal import BackboneTerminal
from models.backbones.utility import convolution3x3
from scdhip import blocks, ops

BNMOMENTUM = 0.1


class BasicBlock(torch.nn.Module):
    expansion = 1

    def __init__(self, inputDimension, outputDimension, stride=1, downsample=None):
        super(BasicBlock, self).__init__()
        self.conv1 = convolution3x3(inputDimension, outputDimension, stride)
        self.bn1 = torch.nn.BatchNorm2d(outputDimension, momentum=BNMOMENTUM)
        self.relu = torch.nn.ReLU(inplace=True)
        self.conv2 = convolution3x3(outputDimension, outputDimension)
        self.bn2 = torch.nn.BatchNorm2d(outputDimension, momentum=BNMOMENTUM)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        """x: NHWC activation (compute dtype) -> NHWC activation."""
        return blocks.BasicBlockFn.apply(x, self.conv1.weight, self)


class Bottleneck(torch.nn.Module):
    expansion = 4

    def __init__(self, inputDimension, outputDimension, stride=1, downsample=None):
        super(Bottleneck, self).__init__()
        self.conv1 = torch.nn.Conv2d(inputDimension, outputDimension, kernel_size=1, bias=False)
        self.bn1 = torch.nn.BatchNorm2d(outputDimension, momentum=BNMOMENTUM)
        self.conv2 = torch.nn.Conv2d(outputDimension, outputDimension, kernel_size=3, stride=stride, padding=1,
                                     bias=False)
        self.bn2 = torch.nn.BatchNorm2d(outputDimension, momentum=BNMOMENTUM)
        self.conv3 = torch.nn.Conv2d(outputDimension, outputDimension * self.expansion, kernel_size=1, bias=False)
        self.bn3 = torch.nn.BatchNorm2d(outputDimension * self.expansion, momentum=BNMOMENTUM)
        self.relu = torch.nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        return blocks.BottleneckFn.apply(x, self.conv1.weight, self)


class ResNetTerminal(BackboneTerminal):
    """Head descriptor (residuals.py:167-182): name, output dims, hidden dims, init, make, process."""

    def __init__(self, name, outputDimension, terminalDimension=0, initializerFunction=None,
                 makeLayerFunction=None, process=None):
        super(ResNetTerminal, self).__init__(name, initializerFunction, makeLayerFunction, process)
        self.outputDimension = outputDimension
        self.terminalDimension = terminalDimension


def _is_plain_head(m):
    """Conv2d(3x3,bias) -> ReLU -> Conv2d(1x1,bias): the CenterNet terminal (centerNetOffset.py:106-110)."""
    return (isinstance(m, torch.nn.Sequential) and len(m) == 3 and isinstance(m[0], torch.nn.Conv2d)
            and isinstance(m[1], torch.nn.ReLU) and isinstance(m[2], torch.nn.Conv2d)
            and m[0].kernel_size == (3, 3) and m[0].bias is not None and m[2].kernel_size == (1, 1))


def _is_corner_head(m):
    """Sequential(CornerPool, Conv2d 3x3 +bias, ReLU, Conv2d 1x1): the CornerNet TL/BR terminal."""
    return (isinstance(m, torch.nn.Sequential) and len(m) == 4 and hasattr(m[0], "dirs")
            and _is_plain_head(torch.nn.Sequential(m[1], m[2], m[3])))


class ResNet(torch.nn.Module):
    """ResNet(inputDimension, block, layers, preprocess, terminals, decoder, dimensions) -- residuals.py:184-353.

    ``compute_dtype`` (torch.bfloat16 default, torch.float16 with a static loss scale, torch.float32 for parity)
    selects the MFMA
    path: bf16 v_mfma_f32_16x16x32_bf16 or exact-f32 v_mfma_f32_16x16x4_f32.
    """

    def __init__(self, inputDimension, block, layers, preprocess=None, terminals=[], decoder=None,
                 dimensions=[64, 64, 128, 256, 512, 256, 256, 256], **kwargs):
        self.inputDimension = dimensions[0]
        self.deconvolutionWithBias = False
        self.terminals = {}
        self.decoder = decoder
        super(ResNet, self).__init__()
        self.compute_dtype = torch.bfloat16
        if preprocess is None:
            self.preprocess = torch.nn.Sequential(
                torch.nn.Conv2d(inputDimension, dimensions[0], kernel_size=7, stride=2, padding=3, bias=False),
                torch.nn.BatchNorm2d(dimensions[0], momentum=BNMOMENTUM),
                torch.nn.ReLU(inplace=True),
                torch.nn.MaxPool2d(kernel_size=3, stride=2, padding=1))
        else:
            self.preprocess = preprocess(inputDimension)
        self.layer1 = self.makeLayer(block, dimensions[1], layers[0])
        self.layer2 = self.makeLayer(block, dimensions[2], layers[1], stride=2)
        self.layer3 = self.makeLayer(block, dimensions[3], layers[2], stride=2)
        self.layer4 = self.makeLayer(block, dimensions[4], layers[3], stride=2)
        self.prediction = dimensions[7]
        self.deconvolutionLayers = self.makeDeconvLayer(3, [dimensions[5], dimensions[6], self.prediction],
                                                        [4, 4, 4])
        self.terminalLayers = {}
        for terminal in terminals:
            outputDim = terminal.outputDimension
            terminalDim = terminal.terminalDimension
            if terminal.makeLayer is not None:
                terminalLayer = terminal.makeLayer(self.prediction, terminalDim, outputDim)
            else:
                terminalLayer = torch.nn.Conv2d(in_channels=self.prediction, out_channels=outputDim,
                                                kernel_size=1, stride=1, padding=0)
            self.terminals[terminal.name] = terminal
            self.terminalLayers[terminal.name] = terminalLayer
        for terminal in terminals:
            setattr(self, terminal.name, self.terminalLayers[terminal.name])

    def makeLayer(self, block, dimension, blocks_, stride=1):
        downsample = None
        if stride != 1 or self.inputDimension != dimension * block.expansion:
            downsample = torch.nn.Sequential(
                torch.nn.Conv2d(self.inputDimension, dimension * block.expansion, kernel_size=1, stride=stride,
                                bias=False),
                torch.nn.BatchNorm2d(dimension * block.expansion, momentum=BNMOMENTUM))
        layers = [block(self.inputDimension, dimension, stride, downsample)]
        self.inputDimension = dimension * block.expansion
        for _ in range(1, blocks_):
            layers.append(block(self.inputDimension, dimension))
        return torch.nn.Sequential(*layers)

    def getDeconvConfig(self, kernel, index):
        if kernel == 4:
            return kernel, 1, 0
        if kernel == 3:
            return kernel, 1, 1
        if kernel == 2:
            return kernel, 0, 0
        raise ValueError("unsupported deconv kernel %d" % kernel)

    def makeDeconvLayer(self, nLayers, dimensions, kernels):
        if nLayers != len(dimensions) or nLayers != len(kernels):
            Logger.err(":: residuals.py :: Inconsistant Number of Layers. ")
            sys.exit()
        numLayers = []
        for i in range(nLayers):
            kernel, padding, outputPadding = self.getDeconvConfig(kernels[i], i)
            dimension = dimensions[i]
            numLayers.append(torch.nn.ConvTranspose2d(
                in_channels=self.inputDimension, out_channels=dimension, kernel_size=kernel, stride=2,
                padding=padding, output_padding=outputPadding, bias=self.deconvolutionWithBias))
            numLayers.append(torch.nn.BatchNorm2d(dimension, momentum=BNMOMENTUM))
            numLayers.append(torch.nn.ReLU(inplace=True))
            self.inputDimension = dimension
        return torch.nn.Sequential(*numLayers)

    # ------------------------------------------------------------------ HIP execution
    def backbone_forward(self, x):
        """(N,1,H,W) fp32 NCHW -> deconv-stack output, NHWC compute dtype (residuals.py:312-325)."""
        if not x.is_cuda:
            raise RuntimeError("scd-resnet_amd executes on MI355X only (got a CPU input); the CPU restatement "
                               "of the reference is oracle/ (test infrastructure)")
        conv, bn = self.preprocess[0], self.preprocess[1]
        if not (isinstance(self.preprocess, torch.nn.Sequential) and len(self.preprocess) == 4
                and conv.in_channels == 1 and conv.stride == (2, 2)):
            raise NotImplementedError("only the default stem (Conv7x7 s2 + BN + ReLU + MaxPool) runs on HIP")
        h = blocks.StemFn.apply(x.float().contiguous(), conv.weight, conv, bn, self.compute_dtype)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                h = blk(h)
        dl = self.deconvolutionLayers
        for i in range(0, len(dl), 3):
            dc, dbn = dl[i], dl[i + 1]
            if dc.bias is not None or dc.output_padding != (0, 0):
                raise NotImplementedError("deconv with bias/output_padding")
            h = blocks.DeconvBNFn.apply(h, dc.weight, dc, dbn)
        return h

    def heads_forward(self, feat, *x, **kwargs):
        names = list(self.terminalLayers.keys())
        mods = [getattr(self, n) for n in names]
        ret = {}
        plain = [n for n, m in zip(names, mods) if _is_plain_head(m)]
        corner = [n for n, m in zip(names, mods) if n not in plain and _is_corner_head(m)]
        if len(plain) + len(corner) == len(names):
            # every consumer of feat is an scdhip Function: one input-gradient buffer instead of autograd's sums
            nplain = (1 if len({getattr(self, n)[0].weight.shape[0] for n in plain}) == 1 else len(plain)) if plain else 0
            ops.share_grad(feat, nplain + len(corner))
        if plain:
            hm = [getattr(self, n) for n in plain]
            if len({m[0].weight.shape[0] for m in hm}) == 1:
                outs = blocks.HeadsFn.apply(feat, hm[0][0].weight, hm)
                ret.update(dict(zip(plain, outs)))
            else:
                for n, m in zip(plain, hm):
                    ret[n] = blocks.HeadsFn.apply(feat, m[0].weight, [m])[0]
        for n, m in zip(names, mods):
            if n in ret:
                continue
            if _is_corner_head(m):
                # CornerNet terminal: CornerPool -> Conv3x3+bias -> ReLU -> Conv1x1 (cornerNetCPool.py:163-199)
                cp = m[0]
                h = blocks.CornerPoolFn.apply(feat, cp.branch1.conv.weight, cp, cp.dirs)
                ret[n] = blocks.HeadsFn.apply(h, m[1].weight, [(m[1], m[2], m[3])])[0]
                continue
            if self.terminals[n].process is None:
                Logger.err("Processor function of the terminal '{}' is not implemented.".format(n))
                sys.exit()
            ret[n] = self.terminals[n].process(feat, m, *x, **kwargs)
        return {n: ret[n] for n in names}

    def forward(self, *x, **kwargs):
        decode = kwargs.get("decode", False)
        # all packed weight operands of this step in one launch (scdhip.ops.PackPlan)
        plan = self.__dict__.get("_scd_packplan")
        if plan is None:
            plan = self.__dict__["_scd_packplan"] = ops.PackPlan()
        ops.pack_begin(plan)
        feat = self.backbone_forward(x[0])
        ret = self.heads_forward(feat, *x, **kwargs)
        return [ret] if not decode else self.decoder(ret)

    def initialize(self, num_layers):
        """residuals.py:336-353 -- including the terminal loop nested in the deconv loop (its RNG draws)."""
        for _, m in self.deconvolutionLayers.named_modules():
            if isinstance(m, torch.nn.ConvTranspose2d):
                torch.nn.init.normal_(m.weight, std=0.001)
                if self.deconvolutionWithBias:
                    torch.nn.init.constant_(m.bias, 0)
            elif isinstance(m, torch.nn.BatchNorm2d):
                torch.nn.init.constant_(m.weight, 1)
                torch.nn.init.constant_(m.bias, 0)
            for head in self.terminalLayers.keys():
                terminal = self.terminalLayers[head]
                for i, mm in enumerate(terminal.modules()):
                    if isinstance(mm, torch.nn.Conv2d):
                        if mm.weight.shape[0] == self.terminals[head].outputDimension:
                            if self.terminals[head].initializer is not None:
                                self.terminals[head].initializer(mm)

    def set_compute_dtype(self, dtype):
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError("compute dtype must be torch.float32, torch.bfloat16 or torch.float16")
        self.compute_dtype = dtype
        return self


ResNetSpec = {18: (BasicBlock, [2, 2, 2, 2]),
              34: (BasicBlock, [3, 4, 6, 3]),
              50: (Bottleneck, [3, 4, 6, 3]),
              101: (Bottleneck, [3, 4, 23, 3]),
              152: (Bottleneck, [3, 8, 36, 3]),
              16: (BasicBlock, [1, 2, 2, 2]),
              14: (BasicBlock, [1, 2, 2, 1]),
              12: (BasicBlock, [1, 1, 2, 1]),
              10: (BasicBlock, [1, 1, 1, 1])}
