"""cProfile of the host side of the Res10 B=32 bf16 training step (what issuing one step costs in Python / ctypes).

python tools/host_profile.py [--steps 20] [--top 40] [--engine-thread]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--engine-thread", action="store_true",
                    help="leave the backward on the autograd engine's device thread (cProfile then sees it as one "
                         "opaque run_backward call)")
    a = ap.parse_args()
    import importlib
    if not a.engine_thread:
        # run the backward's Python Functions on this thread so cProfile attributes their time
        torch.autograd.set_multithreading_enabled(False)

    from scdhip.flat import FlatAdam
    from scdhip.loss import mean_backward
    from trainer.dataset.syntheticSCD import SCD
    plugin = importlib.import_module("trainer.model.centerOffsetRes10")
    dev = torch.device("cuda", 0)
    model = plugin.model(**plugin.modelParams).to(dev).set_compute_dtype(torch.bfloat16).train()
    opt = FlatAdam(filter(lambda p: p.requires_grad, model.parameters()))
    ds = SCD(None, True, seed=1000)
    items = [ds[i] for i in range(32)]
    x = torch.stack([it["xs"][0] for it in items]).to(dev)
    ys = [torch.stack([it["ys"][k] for it in items]).to(dev) for k in range(len(items[0]["ys"]))]
    lossfn = plugin.loss

    def step():
        opt.zero_grad()
        lossfn.prepare(ys)
        loss, _ = lossfn(model(x, decode=False), ys)
        mean_backward(loss)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
    ps.print_stats(a.top)
    print("per step: see tottime / %d" % a.steps)
    print(s.getvalue())


if __name__ == "__main__":
    main()
