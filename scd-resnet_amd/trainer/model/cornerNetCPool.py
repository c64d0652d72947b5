"""Model plugin `cornerNetCPool`: CornerNetResidual(10) with corner pooling (models/cornerNetCPool.py
of the reference; it ships no trainer/model plugin for it, this one follows the
centerOffsetRes10 layout).  Pair with the `syntheticCorner` dataset plugin."""
import torch

from models.cornerNetCPool import CornerNetLoss, CornerNetResidual, cornerNetEvaluation
from models.centerNetOffset import expression  # noqa: F401
from models.losses.focal import focalLoss

torch.random.manual_seed(42)

model = CornerNetResidual
loss = CornerNetLoss(focal=focalLoss)
modelParams = {'numLayers': 10}
evaluation = cornerNetEvaluation

