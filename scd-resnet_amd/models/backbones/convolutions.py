"""Convolution = conv + BN + ReLU (models/backbones/convolutions.py:25-49 of the reference).

Takes / returns NHWC activations in the compute dtype (it is only used inside the HIP
CornerNet terminals); runs as one scdhip ConvBNFn (MFMA implicit GEMM + training BN).
"""
import torch

from scdhip import blocks


class Convolution(torch.nn.Module):
    def __init__(self, convSize, inputDimension, outputDimension, stride=1, batchNorm=True):
        super(Convolution, self).__init__()
        pad = (convSize - 1) // 2
        self.conv = torch.nn.Conv2d(inputDimension, outputDimension, (convSize, convSize), padding=(pad, pad),
                                    stride=(stride, stride), bias=not batchNorm)
        self.bn = torch.nn.BatchNorm2d(outputDimension) if batchNorm else torch.nn.Sequential()
        self.relu = torch.nn.ReLU(inplace=True)

    def forward(self, x):
        if not isinstance(self.bn, torch.nn.BatchNorm2d):
            raise NotImplementedError("Convolution(batchNorm=False) is not on the HIP path")
        return blocks.ConvBNFn.apply(x, self.conv.weight, self.conv, self.bn, True)
