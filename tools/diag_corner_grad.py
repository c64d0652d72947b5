"""Diagnostic: per-parameter gradient error of the HIP CornerNet/CenterNet fp32 path vs oracle."""
import sys, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scd-resnet_amd")]
import torch
from oracle import centernet as O, cornernet as OC, targets as T

def run(kind):
    if kind == "corner":
        import trainer.model.cornerNetCPool as plugin
        entries, topo = OC.model_spec(10); state = OC.hash_weights(entries)
        ys = T.corner_targets(42, 2, 32); fwd, lossf = OC.forward, OC.cornernet_loss
    else:
        import trainer.model.centerOffsetRes10 as plugin
        entries, topo = O.model_spec(10); state = O.hash_weights(entries)
        ys = T.batch_targets(42, 2, 32); fwd = O.forward
        lossf = lambda o, y: O.centernet_loss(o, y)[0]
    m = plugin.model(**plugin.modelParams); m.load_state_dict(state)
    m = m.cuda().train().set_compute_dtype(torch.float32)
    P, Bf = O.split_state(state)
    P = {k: v.requires_grad_(True) for k, v in P.items()}
    x = T.batch_inputs(41, 2, 128)
    lossf(fwd(P, Bf, x, topo), ys).sum().backward()
    loss, _ = plugin.loss(m(x.cuda(), decode=False), [y.cuda() for y in ys])
    loss.sum().backward(); torch.cuda.synchronize()
    names = dict(m.named_parameters())
    rows = []
    for k, v in P.items():
        gr, gg = v.grad.double(), names[k].grad.cpu().double()
        rows.append((k, ((gg - gr).abs().max() / (gr.abs().max() + 1e-30)).item(),
                     ((gg - gr).norm() / (gr.norm() + 1e-30)).item()))
    print(kind, "loss", loss.item())
    for r in rows:
        print("%-45s maxrel %.2e  normrel %.2e" % r)

for k in sys.argv[1:]:
    run(k)
