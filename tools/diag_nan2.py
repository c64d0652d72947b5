"""cornerNetCPool bf16 B=32: 4 Adam steps from the hash weights (tests/test_bf16_parity_gpu.py config3); report the
first non-finite gradient / parameter per step."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "scd-resnet_amd")]
import torch  # noqa: E402

import trainer.model.cornerNetCPool as plugin  # noqa: E402
from oracle import cornernet as OC  # noqa: E402
from scdhip.flat import FlatAdam  # noqa: E402
from trainer.dataset.syntheticCorner import CornerSCD  # noqa: E402

ds = CornerSCD(None, True, seed=77)
items = [ds[i] for i in range(32)]
x = torch.stack([it["xs"][0] for it in items]).cuda()
ys = [torch.stack([it["ys"][k] for it in items]).cuda() for k in range(len(items[0]["ys"]))]
entries, _ = OC.model_spec(10)
state = OC.hash_weights(entries)
for ns_env in (os.environ.get("SCD_WGRAD_PP2", "1"),):
    m = plugin.model(**plugin.modelParams)
    m.load_state_dict(state)
    m = m.cuda().train().set_compute_dtype(torch.bfloat16)
    opt = FlatAdam(filter(lambda p: p.requires_grad, m.parameters()))
    for step in range(4):
        opt.zero_grad()
        loss, _ = plugin.loss(m(x, decode=False), ys)
        loss.mean().backward()
        torch.cuda.synchronize()
        badg = [k for k, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        big = sorted(((p.grad.abs().max().item(), k) for k, p in m.named_parameters() if p.grad is not None),
                     reverse=True)[:3]
        opt.step()
        badp = [k for k, p in m.named_parameters() if not torch.isfinite(p).all()]
        print("PP2=%s step %d loss %.5f badgrad %s badparam %s maxgrad %s" % (ns_env, step, loss.mean().item(),
              badg[:6], badp[:4], big), flush=True)
