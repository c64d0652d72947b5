"""train.py <config.json> [-gpu] [-debug] [--local_rank N | --local-rank N]  (train.py of the reference).

One process per GPU.  With -gpu the process group is initialised over RCCL ("nccl" backend of
torch.distributed, env:// rendezvous as launched by torch.distributed.run / launch); the
local rank comes from --local_rank, --local-rank or LOCAL_RANK (torch >= 2 launchers).
"""
import argparse
import json
import os
import sys
from pprint import pprint

import torch
import torch.distributed as dist

from configuration import defaultConfig
from logger import Logger
from models.networkFactory import NetworkFactory


def parseArguments(argv=None):
    parser = argparse.ArgumentParser(description="train.py - train neural networks with a given set of configuration.")
    parser.add_argument("configuration", type=str, help="the path to the JSON configuration file")
    parser.add_argument("-gpu", dest="useGPU", const=True, default=False, action="store_const",
                        help="whether the trainer detect and use GPUs")
    parser.add_argument("-debug", dest="debug", const=True, default=False, action="store_const",
                        help="enable debug features")
    parser.add_argument("--local_rank", "--local-rank", default=int(os.environ.get("LOCAL_RANK", -1)), type=int,
                        dest="localRank", help="local process index (torch.distributed launchers)")
    return parser.parse_args(argv)


def begin(args):
    localRank = -1
    if args["useGPU"]:
        if not (torch.cuda.device_count() > 0 and torch.cuda.is_available()):
            Logger.err(":: train.py :: No GPU available; scd-resnet_amd has no CPU path (see oracle/ for the CPU "
                       "restatement)")
            sys.exit(1)
        if not dist.is_nccl_available():
            Logger.err(":: train.py :: The NCCL (RCCL) Backend is Not Set Up on This Machine")
            sys.exit(1)
        localRank = max(args["localRank"], 0)
        torch.cuda.set_device(localRank)
        if "WORLD_SIZE" in os.environ and not dist.is_initialized():
            dist.init_process_group("nccl", device_id=torch.device("cuda", localRank))
    with open(args["config"], "r") as f:
        defaultConfig.updateConfig(json.load(f))
    pprint(defaultConfig.config, indent=4)
    Logger.info(":: train.py :: configuration :::::::::::::::::::::::::::::::::::::::::::::::::")
    trainFactory = NetworkFactory(args["useGPU"])
    trainFactory.beginTraining(localRank)


def main(args):
    Logger.info(":: train.py :: trainer program of neural networks ::::::::::::::::::::::::::::")
    settings = {"config": args.configuration, "useGPU": args.useGPU, "localRank": args.localRank,
                "debug": args.debug}
    defaultConfig.update("useGPU", args.useGPU)
    pprint(settings, indent=4)
    Logger.info(":: train.py :: trainer task begin ::::::::::::::::::::::::::::::::::::::::::::")
    begin(settings)
    if dist.is_initialized():
        dist.destroy_process_group()
    Logger.info(":: train.py :: trainer task completed ::::::::::::::::::::::::::::::::::::::::")


if __name__ == "__main__":
    main(parseArguments())
