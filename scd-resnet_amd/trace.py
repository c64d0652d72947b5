"""trace.py -- TorchScript `.pt` of a trained model's decoded inference (trace.py of the reference, same arguments).

python trace.py <output.pt> -a <architecture> -m <state_dict.pth> -s "1 1 512 512" [-gpu] [-wrapped] [-eval]
        [-dtype bf16|fp16|fp32]

The traced graph is one scd::centernet_decode call over the model's parameters and buffers (scdhip/export.py), so
the `.pt` replays the libscdhip path after torch.jit.load in a process that imported scdhip.export (slide.py does).
The model always runs on the GPU (-gpu is accepted for the reference's command lines); -wrapped strips the
DataParallel `module.` prefix the reference adds; -eval traces BatchNorm on running statistics (the reference
traces the model as constructed, i.e. on batch statistics).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from logger import Logger  # noqa: E402


def parseArguments(argv=None):
    parser = argparse.ArgumentParser(description="trace.py - generate a TorchScript version of a model on MI355X")
    parser.add_argument("output", type=str, help="the output .pt file of the traced model")
    parser.add_argument("-a", dest="modelArchitecture", type=str, help="the architecture name of the model")
    parser.add_argument("-m", type=str, dest="model", help="the path to the model file, in .pth format")
    parser.add_argument("-s", type=str, dest="inputShape", help="input tensor shape, space separated, e.g. '1 1 64 64'")
    parser.add_argument("-gpu", dest="useGPU", const=True, default=False, action="store_const")
    parser.add_argument("-wrapped", dest="isWrapped", const=True, default=False, action="store_const")
    parser.add_argument("-eval", dest="evalMode", const=True, default=False, action="store_const")
    parser.add_argument("-dtype", dest="dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    return parser.parse_args(argv)


@torch.no_grad()
def begin(args):
    import importlib
    from scdhip import export
    modelPy = "trainer.model." + args.modelArchitecture
    Logger.info("Loaded Model From: {}".format(modelPy))
    plugin = importlib.import_module(modelPy)
    model = plugin.model(**plugin.modelParams)
    if not os.path.exists(args.model):
        Logger.err(":: trace.py :: Pretrained Model Does not Exist: {}".format(args.model))
        sys.exit(1)
    with open(args.model, "rb") as f:
        params = torch.load(f, map_location="cpu", weights_only=True)
    if args.isWrapped or next(iter(params)).startswith("module."):
        params = {k[len("module."):] if k.startswith("module.") else k: v for k, v in params.items()}
    model.load_state_dict(params)
    dev = torch.device("cuda", torch.cuda.current_device())
    model = model.to(dev)
    shape = [int(s) for s in args.inputShape.split()]
    dummy = torch.rand(*shape, device=dev)
    traced = export.trace(args.modelArchitecture, model, dummy, args.output, mode="eval" if args.evalMode else "train",
                          dtype=args.dtype)
    out = traced(dummy)
    Logger.log("The loaded models accepts Input in {} and Output in {}".format(tuple(dummy.shape), tuple(out.shape)))
    Logger.log("Output saved to {}".format(args.output))


if __name__ == "__main__":
    begin(parseArguments())
