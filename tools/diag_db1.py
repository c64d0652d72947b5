"""Diagnose the heatmap.2.bias gradient of the HIP bf16 step against fp32 / PyTorch bf16 (yardstick test)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "scd-resnet_amd")]
import torch  # noqa: E402

from oracle import centernet as O  # noqa: E402
from oracle import targets as T  # noqa: E402

DEV = "cuda"
x = T.batch_inputs(41, 4, 512)
ys = [y.to(DEV) for y in T.batch_targets(42, 4, 128)]
entries, topo = O.model_spec(10)
state = O.hash_weights(entries)


def torch_run(bf16):
    P, Bf = O.split_state({k: v.clone() for k, v in state.items()})
    P = {k: v.to(DEV).requires_grad_(True) for k, v in P.items()}
    Bf = {k: v.to(DEV) for k, v in Bf.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        out = O.forward(P, Bf, x.to(DEV), topo)
    out = {k: v.float() for k, v in out.items()}
    out["heatmap"].retain_grad()
    loss, _ = O.centernet_loss(out, ys)
    loss.sum().backward()
    return P["heatmap.2.bias"].grad.double(), out["heatmap"].grad.double(), out["heatmap"].detach().double()


for dt in (torch.float32, torch.bfloat16):
    import trainer.model.centerOffsetRes10 as plugin
    m = plugin.model(**plugin.modelParams)
    m.load_state_dict(state)
    m = m.to(DEV).train().set_compute_dtype(dt)
    outs = m(x.to(DEV), decode=False)
    outs[0]["heatmap"].retain_grad()
    loss, _ = plugin.loss(outs, ys)
    loss.mean().backward()
    g = outs[0]["heatmap"].grad
    print(dt, "HIP db1", m.heatmap[2].bias.grad.double().item(), "sum dout(fp64)",
          g.double().sum().item() if g is not None else None)
    if dt == torch.float32:
        hip32 = outs[0]["heatmap"].detach().double()
    else:
        hipbf = outs[0]["heatmap"].detach().double()
g32, d32, h32 = torch_run(False)
gbf, dbf, hbf = torch_run(True)
print("torch fp32 db1", g32.item(), "sum dout", d32.sum().item())
print("torch bf16 db1", gbf.item(), "sum dout", dbf.sum().item())
print("heatmap logits rel err: HIP fp32 %.3e HIP bf16 %.3e torch bf16 %.3e" % (
    ((hip32 - h32).norm() / h32.norm()).item(), ((hipbf - h32).norm() / h32.norm()).item(),
    ((hbf - h32).norm() / h32.norm()).item()))
print("mean logit err: HIP bf16 %.3e torch bf16 %.3e" % ((hipbf - h32).mean().item(), (hbf - h32).mean().item()))
