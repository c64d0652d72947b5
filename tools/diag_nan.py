"""Which parameter gradients go non-finite in one bf16 step (cornerNetCPool / centerOffsetRes10, B=32 512^2)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "scd-resnet_amd")]
import importlib  # noqa: E402

import torch  # noqa: E402

from oracle import targets as T  # noqa: E402

for name in ("centerOffsetRes10", "cornerNetCPool"):
    plugin = importlib.import_module("trainer.model." + name)
    torch.random.manual_seed(42)
    m = plugin.model(**plugin.modelParams).cuda().train().set_compute_dtype(torch.bfloat16)
    if name.startswith("corner"):
        from trainer.dataset.syntheticCorner import CornerSCD
        ds = CornerSCD(None, True, seed=1000)
    else:
        from trainer.dataset.syntheticSCD import SCD
        ds = SCD(None, True, seed=1000)
    items = [ds[i] for i in range(32)]
    x = torch.stack([it["xs"][0] for it in items]).cuda()
    ys = [torch.stack([it["ys"][k] for it in items]).cuda() for k in range(len(items[0]["ys"]))]
    for step in range(2):
        for p in m.parameters():
            p.grad = None
        loss, _ = plugin.loss(m(x, decode=False), ys)
        loss.mean().backward()
        torch.cuda.synchronize()
        bad = [(k, p.grad.shape) for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        print(name, "step", step, "loss", loss.mean().item(), "non-finite grads:", bad[:20], flush=True)
