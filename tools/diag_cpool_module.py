"""Diagnostic: CornerPoolFn (tl/br) standalone vs oracle corner_pool autograd, fp32."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "scd-resnet_amd")]
import torch
from oracle import centernet as O, cornernet as OC
import models.cornerNetCPool as M

torch.manual_seed(0)
for name, cls, dirs in (("tl", M.TopLeftPool, (0, 2)), ("br", M.BottomRightPool, (1, 3))):
    mod = cls(64)
    for p in mod.parameters():
        p.data.normal_(0, 0.1)
    st = {name + ".0." + k: v.clone() for k, v in mod.state_dict().items()}
    P, Bf = O.split_state(st)
    P = {k: v.requires_grad_(True) for k, v in P.items()}
    x = torch.randn(2, 64, 16, 24, requires_grad=True)
    y = OC.corner_pool(x, P, Bf, name + ".0", dirs)
    dy = torch.randn_like(y)
    y.backward(dy)
    mod = mod.cuda().train()
    xg = x.detach().permute(0, 2, 3, 1).contiguous().cuda().requires_grad_(True)
    yg = mod(xg)
    yg.backward(dy.permute(0, 2, 3, 1).contiguous().cuda())
    torch.cuda.synchronize()
    print(name, "fwd maxabs", (yg.detach().cpu().permute(0, 3, 1, 2) - y.detach()).abs().max().item(),
          "ref max", y.abs().max().item())
    print(name, "dx rel", ((xg.grad.cpu().permute(0, 3, 1, 2) - x.grad).abs().max() / x.grad.abs().max()).item())
    for k, v in mod.named_parameters():
        r = P[name + ".0." + k].grad
        print("  %-28s %.2e" % (k, ((v.grad.cpu() - r).abs().max() / (r.abs().max() + 1e-30)).item()))

# run-to-run determinism of the full model backward
import trainer.model.cornerNetCPool as plugin
from oracle import targets as T
entries, topo = OC.model_spec(10); state = OC.hash_weights(entries)
gs = []
for rep in range(2):
    m = plugin.model(**plugin.modelParams); m.load_state_dict(state)
    m = m.cuda().train().set_compute_dtype(torch.float32)
    x = T.batch_inputs(41, 2, 128); ys = T.corner_targets(42, 2, 32)
    loss, _ = plugin.loss(m(x.cuda(), decode=False), [y.cuda() for y in ys])
    loss.sum().backward(); torch.cuda.synchronize()
    gs.append({k: v.grad.cpu().clone() for k, v in m.named_parameters()})
for k in gs[0]:
    d = (gs[0][k] - gs[1][k]).abs().max().item()
    if d > 0:
        print("nondet", k, d)
print("determinism check done")
