"""Is the training step host-bound?  Times, for the bench's Res10 B=32 bf16 step, (a) the host time to issue one
step (no synchronisation inside a step, so this is pure Python/ctypes/launch cost unless the HIP queue is full)
and (b) the wall time per step, and (c) the host issue time with a GPU that is kept busy (queue full).

python tools/host_overhead.py [--steps 20]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import trainer.model.centerOffsetRes10 as plugin
    from scdhip.flat import FlatAdam
    from scdhip.loss import mean_backward
    from trainer.dataset.syntheticSCD import SCD
    dev = torch.device("cuda", 0)
    model = plugin.model(**plugin.modelParams).to(dev).set_compute_dtype(torch.bfloat16).train()
    opt = FlatAdam(filter(lambda p: p.requires_grad, model.parameters()))
    ds = SCD(None, True, seed=1000)
    b = ds.gpu_batch(list(range(32)), dev)
    x, ys = b["xs"][0], b["ys"]

    def step():
        opt.zero_grad()
        loss, _ = plugin.loss(model(x, decode=False), ys)
        loss = mean_backward(loss)
        opt.step()
        return loss

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    issue = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = time.perf_counter()
        step()
        issue.append(time.perf_counter() - s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    issue.sort()
    print("wall %.3f ms/step; host issue per step: median %.3f ms, min %.3f ms, max %.3f ms"
          % (wall * 1e3, issue[len(issue) // 2] * 1e3, issue[0] * 1e3, issue[-1] * 1e3))
    # host issue time of one step right after a sync (GPU idle, queue empty): pure host cost
    iso = []
    for _ in range(5):
        torch.cuda.synchronize()
        s = time.perf_counter()
        step()
        iso.append(time.perf_counter() - s)
    torch.cuda.synchronize()
    iso.sort()
    print("host issue per step from an idle GPU: median %.3f ms" % (iso[len(iso) // 2] * 1e3))


if __name__ == "__main__":
    main()
