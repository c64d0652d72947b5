"""CenterNet with 64-channel heads (models/centerNetOffseth.py of the reference: identical to
centerNetOffset.py except the terminal hidden width, :146-148)."""
from models.centerNetOffset import (CenterNetLoss, centerNetEvaluation, decodeCenterNet, expression,  # noqa: F401
                                    make_terminals)
from models.centerNetOffset import CenterNetResidual as _CenterNetResidual

resnetHeatmapTerminal, resnetSizeTerminal, resnetOffsetTerminal = make_terminals(64)


class CenterNetResidual(_CenterNetResidual):
    HEAD_DIM = 64
