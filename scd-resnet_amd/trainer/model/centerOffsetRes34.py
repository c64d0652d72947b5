"""Model plugin `centerOffsetRes34` (trainer/model/centerOffsetRes34.py of the reference): exports
model, loss, modelParams, evaluation, expression.  Importing it reseeds torch with 42, as the
reference's import chain does (networkFactory.py:34, scdx16p100.py:43), so construction
draws the same initial weights."""
import torch

from models.centerNetOffset import CenterNetLoss, CenterNetResidual, centerNetEvaluation
from models.centerNetOffset import expression  # noqa: F401
from models.losses.focal import focalLoss
from models.losses.regression import L1LossMask

torch.random.manual_seed(42)

model = CenterNetResidual
loss = CenterNetLoss(0.1, 0.1, focal=focalLoss, regression=L1LossMask)
modelParams = {'numLayers': 34,
               'dims': [64, 64, 128, 256, 512, 256, 256, 256]}
evaluation = centerNetEvaluation
