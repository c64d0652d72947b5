"""Project-wide configuration (configuration.py of the reference).

Same default keys and the same overlay rule: a JSON config replaces only keys that already
exist (configuration.py:150-153); string values may reference other keys as `{key}` format
fields.  Two keys are added: ``computeDtype`` ("bf16" | "fp16" | "fp32"), the MFMA precision of the
HIP path (the reference trains in fp32 without AMP), and ``stepGraph`` (true | false, default false):
replay the training step as a captured HIP graph after two eager steps (single-process runs;
scdhip/graph.py -- measured slower than eager issue on ROCm 7).
"""
import os


class Configuration:
    _DIR_KEYS = ("dirTemp", "dirResult", "dirConfig")

    def __init__(self):
        c = {}
        c["datasetName"] = None
        c["modelName"] = None
        c["trainName"] = None
        c["learningRate"] = 0.00025
        c["learningRateDecay"] = [80000]
        c["learningRateDecayRate"] = [10]
        c["currentIter"] = 0
        c["iterations"] = 117000
        c["validation"] = 200
        c["snapshot"] = 2000
        c["batchSize"] = 32
        c["validationBatchSize"] = 160
        c["naming"] = "{modelName}.{trainName}.{currentIter}.pth"
        c["namingOptimizer"] = "{naming}.{optimizer}.pth"
        c["pretrain"] = None
        c["optimizer"] = "adam"
        c["dirData"] = "trainer.dataset.{datasetName}"
        c["dirModel"] = "trainer.model.{modelName}"
        c["dirTemp"] = "/temp/"
        c["dirPretrain"] = "/pretrain/"
        c["dirConfig"] = "/configs/"
        c["dirResult"] = "/results/"
        c["dirDataset"] = "/datasets/"
        c["dirDatafile"] = "{dirDataset}{datasetName}.d"
        c["dirDataSplitProfile"] = "{dirDataset}{datasetName}.split.json"
        c["useGPU"] = False
        c["computeDtype"] = "bf16"
        c["stepGraph"] = False
        self.config = c

    # -- formatted / plain accessors (configuration.py:46-146)
    def _fmt(self, key):
        return self.config[key].format(**self.config)

    def _dir(self, key):
        d = self.config[key]
        if not os.path.exists(d):
            os.makedirs(d)
        return d

    pretrain = property(lambda s: (s.config["dirPretrain"] + s.config["pretrain"])
                        if s.config["pretrain"] is not None else None)
    datasetName = property(lambda s: s.config["datasetName"])
    modelName = property(lambda s: s.config["modelName"])
    trainName = property(lambda s: s.config["trainName"])
    learningRate = property(lambda s: s.config["learningRate"])
    learningRateDecay = property(lambda s: s.config["learningRateDecay"])
    learningRateDecayRate = property(lambda s: s.config["learningRateDecayRate"])
    totalIterations = property(lambda s: s.config["iterations"])
    snapshotFrequency = property(lambda s: s.config["snapshot"])
    validationFrequency = property(lambda s: s.config["validation"])
    batchSize = property(lambda s: s.config["batchSize"])
    validationBatchSize = property(lambda s: s.config["validationBatchSize"])
    currentIteration = property(lambda s: s.config["currentIter"])
    naming = property(lambda s: s._fmt("naming"))
    optimizer = property(lambda s: s._fmt("optimizer"))
    namingOptimizer = property(lambda s: s.config["namingOptimizer"])
    dirData = property(lambda s: s._fmt("dirData"))
    dirModel = property(lambda s: s._fmt("dirModel"))
    dirTemp = property(lambda s: s._dir("dirTemp"))
    dirResult = property(lambda s: s._dir("dirResult"))
    dirConfig = property(lambda s: s._dir("dirConfig"))
    dirDatafile = property(lambda s: s._fmt("dirDatafile"))
    dirDataSplitProfile = property(lambda s: s._fmt("dirDataSplitProfile"))
    computeDtype = property(lambda s: s.config["computeDtype"])
    stepGraph = property(lambda s: bool(s.config["stepGraph"]))

    def useGPU(self):
        # a bound method, hence always truthy when tested without a call (reference quirk)
        return self.config["useGPU"]

    def updateConfig(self, configObj):
        for key, value in configObj.items():
            if key in self.config:
                self.config[key] = value

    def updateIteration(self, it):
        self.config["currentIter"] = it

    def update(self, configName, value):
        self.config[configName] = value


defaultConfig = Configuration()
