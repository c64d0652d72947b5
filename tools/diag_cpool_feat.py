"""Diagnostic: the model's tl/br CornerPool modules on the model's own backbone features."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "scd-resnet_amd")]
import torch
from oracle import centernet as O, cornernet as OC, cpool as OP, targets as T
import trainer.model.cornerNetCPool as plugin
from scdhip import ops, blocks

entries, topo = OC.model_spec(10); state = OC.hash_weights(entries)
m = plugin.model(**plugin.modelParams); m.load_state_dict(state)
m = m.cuda().train().set_compute_dtype(torch.float32)
x = T.batch_inputs(41, 2, 128)
with torch.no_grad():
    feat = m.backbone_forward(x.cuda()) if hasattr(m, "backbone_forward") else None
print("feat", None if feat is None else tuple(feat.shape), "zeros frac", (feat == 0).float().mean().item())
P, Bf = O.split_state(state)
torch.manual_seed(0)
for name, dirs in (("tl", (0, 2)), ("br", (1, 3))):
    mod = getattr(m, name)[0]
    xf = feat.detach().clone().requires_grad_(True)
    y = mod(xf)
    dy = torch.randn_like(y)
    for p in mod.parameters():
        p.grad = None
    y.backward(dy)
    Pn = {k: v.detach().clone().requires_grad_(True) for k, v in P.items() if k.startswith(name + ".0.")}
    xc = feat.detach().cpu().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yc = OC.corner_pool(xc, Pn, {k: v.clone() for k, v in Bf.items()}, name + ".0", dirs)
    yc.backward(dy.cpu().permute(0, 3, 1, 2))
    print(name, "fwd", (y.detach().cpu().permute(0, 3, 1, 2) - yc.detach()).abs().max().item(),
          "dx", ((xf.grad.cpu().permute(0, 3, 1, 2) - xc.grad).abs().max() / xc.grad.abs().max()).item())
    for k, v in mod.named_parameters():
        r = Pn[name + ".0." + k].grad
        print("  %-28s %.2e" % (k, ((v.grad.cpu() - r).abs().max() / (r.abs().max() + 1e-30)).item()))
