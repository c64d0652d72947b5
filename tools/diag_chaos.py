"""Sensitivity of a residual plugin's fp32 forward to a bf16-sized relative perturbation of its weights
(2^-9 relative Gaussian noise): separates precision amplification by the network from kernel errors."""
import sys
import torch
sys.path.insert(0, "scd-resnet_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
from test_model_gpu import make_model  # noqa: E402
from oracle import targets as T  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "centerOffsetRes50"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 256
x = T.batch_inputs(9, 2, size).cuda()
res = []
for noise in (0.0, 2.0 ** -9):
    m, *_ = make_model(torch.float32, name)
    if noise:
        g = torch.Generator(device="cuda").manual_seed(3)
        with torch.no_grad():
            for p in m.parameters():
                if p.dim() == 4:
                    p.mul_(1 + noise * torch.randn(p.shape, generator=g, device="cuda"))
    outs = {}
    hooks = [mod.register_forward_hook(lambda mod, i, o, n=n: outs.__setitem__(n, o.detach().float().cpu()))
             for n, mod in m.named_modules() if n.count(".") == 1 and n.startswith("layer")]
    with torch.no_grad():
        outs["heads"] = m(x, decode=False)[0]["heatmap"].float().cpu()
    res.append(outs)
for n in res[0]:
    a, b = res[1][n], res[0][n]
    print("%-10s rel %.4f" % (n, ((a - b).abs().max() / b.abs().max()).item()), flush=True)
