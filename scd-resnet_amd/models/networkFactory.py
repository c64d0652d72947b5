"""NetworkFactory -- plugin loading, optimizer, data-parallel wrap and the training loop
(models/networkFactory.py of the reference).

Same constructor (useGPU), same plugin protocol (trainer.model.<name>: model, modelParams,
loss, evaluation, expression; trainer.dataset.<name>: dataset(zipPath, useGPU, dataSplit)),
same loop (train/validate/snapshot/LR-decay) and file outputs.  Differences, all on the
execution side:
  * the model runs on libscdhip (HIP MFMA kernels) in ``computeDtype`` (bf16 default);
  * DistributedDataParallel -> scdhip.flat.FlatDDP (flat-buffer RCCL all-reduce, average),
    SyncBatchNorm -> global-batch statistics all-reduced inside the BN kernels' finalize
    (enabled by the reference rule: more than one GPU on the machine, networkFactory.py:128);
  * torch.optim.Adam -> scdhip.flat.FlatAdam (same defaults: lr 1e-3 until the first decay);
  * torch.optim.SGD -> scdhip.flat.FlatSGD (momentum 0.9, weight_decay 1e-4, lr = learningRate);
  * batches are moved to this rank's device (the reference datasets pin cuda:0);
  * with ``stepGraph`` (opt-in) a single-process run replays the step as a captured HIP graph after two
    eager steps (scdhip.graph.StepGraph: same kernels, one hipGraphLaunch per step);
  * resume loads after the wrap and uses learningRateDecayRate[index] (fixes the reference's
    `module.` prefix mismatch and [t] index, networkFactory.py:116-124).
The CPU path (no -gpu) is not part of this framework: the CPU restatement is oracle/.
"""
import importlib
import json
import os
import sys

import numpy
import torch
import torch.distributed as dist
import torch.utils.data.distributed as utilsDataDist
from torch.utils.data import DataLoader
from tqdm import tqdm

from configuration import defaultConfig
from logger import Logger, monitorStdOutStream
from scdhip import ops
from scdhip.flat import FlatAdam, FlatDDP, FlatSGD
from scdhip.graph import StepGraph
from scdhip.loss import mean_backward

torch.random.manual_seed(42)

_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp16": torch.float16, "float16": torch.float16,
           "fp32": torch.float32, "float32": torch.float32}


def _to_device(obj, device):
    if torch.is_tensor(obj):
        return obj.to(device, non_blocking=True)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_device(o, device) for o in obj)
    if isinstance(obj, dict):
        return {k: _to_device(v, device) for k, v in obj.items()}
    return obj


class GPUBatchLoader:
    """Training batches from a dataset plugin's gpu_batch(indices, device) -- the batched HIP augmentation and
    target rendering -- visiting indices exactly as DataLoader(batch_size, sampler, drop_last=True) would."""

    def __init__(self, dataset, sampler, batch_size, device):
        from torch.utils.data import BatchSampler, SequentialSampler
        self.dataset, self.device = dataset, device
        self.batches = BatchSampler(sampler if sampler is not None else SequentialSampler(dataset), batch_size,
                                    drop_last=True)

    def __len__(self):
        return len(self.batches)

    def __iter__(self):
        for idx in self.batches:
            yield self.dataset.gpu_batch(list(idx), self.device)


def resumeSchedule(learningRate, decay, rates, current):
    """Learning rate on resuming at iteration `current` (networkFactory.py:140-145 rebuilds it but keeps the
    past milestones, so the loop's `it == learningRateDecay[0]` test never matches again and every later
    decay is skipped; a milestone equal to `current` -- applied right after that snapshot was written -- is
    missed too).  Here every milestone <= current is applied and popped from both lists, in place."""
    while decay and decay[0] <= current:
        learningRate /= rates[0]
        decay.pop(0)
        rates.pop(0)
    return learningRate


class NetworkFactory(object):
    GPUCOUNT = 0

    def __init__(self, useGPU):
        super(NetworkFactory, self).__init__()
        self.useGPU = useGPU
        self.GPUCOUNT = torch.cuda.device_count()
        if not useGPU:
            raise RuntimeError("scd-resnet_amd trains on MI355X only (run train.py with -gpu); the CPU "
                               "restatement of the reference lives in oracle/ and is test infrastructure")

        modelPy = defaultConfig.dirModel
        Logger.info("Loaded Model From: {}".format(modelPy))
        modelLoader = importlib.import_module(modelPy)
        self.model = modelLoader.model(**modelLoader.modelParams)
        if hasattr(self.model, "set_compute_dtype"):
            self.model.set_compute_dtype(_DTYPES[defaultConfig.computeDtype])
        self.loss = modelLoader.loss
        self.evaluation = modelLoader.evaluation
        self.evalExpr = modelLoader.expression

        dataPy = defaultConfig.dirData
        Logger.info("Loaded Dataset File From: {}".format(dataPy))
        dataLoader = importlib.import_module(dataPy)
        split = None
        if os.path.exists(defaultConfig.dirDataSplitProfile):
            with open(defaultConfig.dirDataSplitProfile, "r") as f:
                split = json.loads(f.read())
        self.dataset = dataLoader.dataset(defaultConfig.dirDatafile, useGPU, split)

        self.parameterCount = sum(p.numel() for p in self.model.parameters())
        Logger.log("Parameter Count: {}".format(self.parameterCount))

        if defaultConfig.optimizer == "adam":
            self.optimizer = FlatAdam(filter(lambda p: p.requires_grad, self.model.parameters()))
        elif defaultConfig.optimizer == "sgd":
            # networkFactory.py:84-89
            self.optimizer = FlatSGD(filter(lambda p: p.requires_grad, self.model.parameters()),
                                     lr=defaultConfig.learningRate, momentum=0.9, weight_decay=0.0001)
        else:
            Logger.err(":: networkFactory.py :: Unknown Optimizer '{}', Currently Support 'sgd' or 'adam'".format(
                defaultConfig.optimizer))
            sys.exit()
        self.device = None
        self.stepGraph = None

    @property
    def isGPU(self):
        return self.useGPU

    def _distributed(self):
        return dist.is_available() and dist.is_initialized()

    def beginTraining(self, localRank):
        localRank = max(localRank, 0)
        self.device = torch.device("cuda", localRank)
        distributed = self._distributed()
        Logger.info(":: networkFactory.py :: Begin Training Task on Local Device {}".format(localRank))
        sampler = utilsDataDist.DistributedSampler(self.dataset, drop_last=True, shuffle=False) if distributed else None
        if hasattr(self.dataset, "gpu_batch"):
            # whole batches augmented / target-rendered on the GPU (one launch each) in the DataLoader's order
            trainLoader = GPUBatchLoader(self.dataset, sampler, defaultConfig.batchSize, self.device)
        elif distributed:
            trainLoader = DataLoader(self.dataset, batch_size=defaultConfig.batchSize, sampler=sampler,
                                     drop_last=True, shuffle=False)
        else:
            trainLoader = DataLoader(self.dataset, batch_size=defaultConfig.batchSize, drop_last=True,
                                     shuffle=False)
        Logger.log("Loaded Dataset Loader: {}".format(defaultConfig.datasetName))
        Logger.info("Loaded with Training Samples: {}".format(len(self.dataset)))

        learningRate = defaultConfig.learningRate
        # the step runs on a high-priority stream: scdhip's weight-gradient side stream has the lowest priority, so
        # the input-gradient chain's small kernels are dispatched first when both have work (bench.py: +1.3%)
        torch.cuda.set_stream(torch.cuda.Stream(device=self.device, priority=-10))
        self.cuda()
        if distributed and self.GPUCOUNT > 1 and dist.get_world_size() > 1:
            # SyncBatchNorm semantics (networkFactory.py:128-133): over peer memory when every rank maps its peers, so
            # FlatDDP's buckets overlap the backward; else through RCCL (ops.setup_syncbn logs which and why)
            ops.setup_syncbn(log=Logger.info if dist.get_rank() == 0 else None)
        self.model = FlatDDP(self.model)
        if defaultConfig.stepGraph and not (distributed and dist.get_world_size() > 1):
            self.stepGraph = StepGraph(self._trainStep, optimizer=self.optimizer, warmup=2)
        if defaultConfig.currentIteration > 0:
            learningRate = resumeSchedule(learningRate, defaultConfig.learningRateDecay,
                                          defaultConfig.learningRateDecayRate, defaultConfig.currentIteration)
            self.loadParameters()
            self.setLearningRate(learningRate)

        pretrainedModel = defaultConfig.pretrain
        if pretrainedModel is not None:
            if not os.path.exists(pretrainedModel):
                Logger.err(":: networkFactory.py :: Pretrained Model Does not Exist")
                sys.exit()
            self.loadPretrained(pretrainedModel)

        self.trainMode()
        it = defaultConfig.currentIteration
        learningRateDecay = defaultConfig.learningRateDecay
        learningRateDecayRate = defaultConfig.learningRateDecayRate
        lossSave = []
        evalResult = ["Experiment: {}".format(defaultConfig.trainName) + "\n",
                      "Parameter Count: {}".format(self.parameterCount) + "\n"]

        with monitorStdOutStream() as saveStdOut:
            with tqdm(total=defaultConfig.totalIterations - it, file=saveStdOut, ncols=100) as pbar:
                finished = False
                while not finished:
                    for batchId, data in enumerate(trainLoader):
                        defaultConfig.updateIteration(it)
                        it += 1
                        loss, lossStatsT = self.train(**data)
                        lossv = loss.item()
                        pbar.set_description("Loss:" + format(lossv, "-10.4f"))
                        lossSave += [it, lossv]
                        lossSave += [x.item() for x in lossStatsT]

                        if it % defaultConfig.validationFrequency == 0:
                            trainResults, _ = self.validate(**data)
                            evalTr = "[Tr] {}:     ".format(format(it, "7d")) + self.evalExpr([trainResults])
                            batches = []
                            with torch.no_grad():
                                for item in self.dataset.getValidationSet():
                                    results, _ = self.validate(**item)
                                    batches.append(results)
                            evalr = "[It] {}:     ".format(format(it, "7d")) + self.evalExpr(batches)
                            evalResult += [evalTr + "\n" + evalr + "\n"]
                            Logger.infoGreen(evalTr)
                            Logger.info(evalr)

                        if it % defaultConfig.snapshotFrequency == 0:
                            self.saveParameters()
                            numpyLoss = numpy.array(lossSave)
                            dim = 2 + len(lossStatsT)
                            saveData = numpy.zeros((len(numpyLoss[0::dim]), dim))
                            for i in range(dim):
                                saveData[:, i] = numpyLoss[i::dim]
                            numpy.savetxt(defaultConfig.dirResult + "losses.{}.{}.txt".format(
                                defaultConfig.trainName, it), saveData, delimiter=",", fmt="%.5f")
                            lossSave = []

                        pbar.update()
                        if len(learningRateDecay) >= 1 and it == learningRateDecay[0]:
                            learningRate /= learningRateDecayRate[0]
                            self.setLearningRate(learningRate)
                            learningRateDecayRate.pop(0)
                            learningRateDecay.pop(0)
                        if it >= defaultConfig.totalIterations:
                            finished = True
                            break

        with open(defaultConfig.dirResult + "evals.{}.txt".format(defaultConfig.trainName), "w") as evalText:
            evalText.writelines(evalResult)

    def cuda(self):
        self.model = self.model.cuda(self.device)

    def trainMode(self):
        self.model.train()

    def evalMode(self):
        self.model.eval()

    def _passParams(self, xs, ys, **kwargs):
        prepare = getattr(self.loss, "prepare", None)     # CenterNetLoss: the heads keep what the loss gathers
        if prepare is not None and torch.is_grad_enabled():
            prepare(ys)
        preds = self.model(*xs, **kwargs)
        return self.loss(preds, ys)

    def train(self, xs, ys, **kwargs):
        """networkFactory.py:257-263 (replayed as a HIP graph when stepGraph is on)"""
        xs, ys = _to_device(xs, self.device), _to_device(ys, self.device)
        if self.stepGraph is not None and not kwargs:
            return self.stepGraph(xs, ys)
        return self._trainStep(xs, ys, **kwargs)

    def _trainStep(self, xs, ys, **kwargs):
        self.optimizer.zero_grad()
        loss, lossStats = self._passParams(xs, ys, decode=False)
        loss = mean_backward(loss)          # loss.mean(); loss.backward() (scdhip.loss.mean_backward)
        self.optimizer.step()
        return loss, lossStats

    def validate(self, xs, ys, **kwargs):
        """networkFactory.py:265-271 (BN stays in train mode, as in the reference)."""
        xs, ys = _to_device(xs, self.device), _to_device(ys, self.device)
        with torch.no_grad():
            decodeResult = self.model(*xs, **kwargs, decode=True)
            return self.evaluation(xs, ys, *decodeResult)

    def setLearningRate(self, lr):
        Logger.warn(":: networkFactory.py :: Setting Learning Rate to: {}".format(lr))
        for group in self.optimizer.param_groups:
            group["lr"] = lr

    def _load_into_wrapped(self, params):
        keys = list(params.keys())
        if keys and not keys[0].startswith("module."):
            params = {"module." + k: v for k, v in params.items()}
        self.model.load_state_dict(params)

    def loadPretrained(self, pretrained):
        Logger.warn(":: networkFactory.py :: Loading from Pretrained: {}".format(pretrained))
        with open(pretrained, "rb") as f:
            self._load_into_wrapped(torch.load(f, map_location=self.device, weights_only=True))

    def loadParameters(self):
        cacheFile = defaultConfig.dirTemp + defaultConfig.naming
        Logger.warn(":: networkFactory.py :: Loading Model from Cached: {}".format(cacheFile))
        with open(cacheFile, "rb") as f:
            self._load_into_wrapped(torch.load(f, map_location=self.device, weights_only=True))

    def saveParameters(self):
        cacheFile = defaultConfig.dirTemp + defaultConfig.naming
        Logger.warn(":: networkFactory.py :: Saving Model to {}".format(cacheFile))
        with open(cacheFile, "wb") as f:
            torch.save(self.model.state_dict(), f)
