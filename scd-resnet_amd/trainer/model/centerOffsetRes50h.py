"""Model plugin `centerOffsetRes50h` (trainer/model/centerOffsetRes50h.py of the reference): exports
model, loss, modelParams, evaluation, expression.  Importing it reseeds torch with 42, as the
reference's import chain does (networkFactory.py:34, scdx16p100.py:43), so construction
draws the same initial weights."""
import torch

from models.centerNetOffseth import CenterNetLoss, CenterNetResidual, centerNetEvaluation
from models.centerNetOffseth import expression  # noqa: F401
from models.losses.focal import focalLoss
from models.losses.regression import L1LossMask

torch.random.manual_seed(42)

model = CenterNetResidual
loss = CenterNetLoss(0.1, 0.1, focal=focalLoss, regression=L1LossMask)
modelParams = {'numLayers': 50,
               'dims': [32, 32, 64, 128, 256, 128, 128, 128]}
evaluation = centerNetEvaluation
