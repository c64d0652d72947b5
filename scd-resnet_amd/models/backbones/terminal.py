class BackboneTerminal(object):
    """Head descriptor (models/backbones/terminal.py:2-15 of the reference):
    name, optional initializer(module), makeLayer(predictionDim, currentDim, outputDim),
    process(input, module, *xs, **kwargs)."""

    def __init__(self, name, initializerFunction=None, makeLayerFunction=None, process=None):
        self.name = name
        self.makeLayer = makeLayerFunction
        self.initializer = initializerFunction
        self.process = process
