"""Per-block bf16-vs-fp32 drift of a residual plugin (default centerOffsetRes50): where does bf16 diverge?"""
import sys
import torch
sys.path.insert(0, "scd-resnet_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
from test_model_gpu import make_model  # noqa: E402
from oracle import targets as T  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "centerOffsetRes50"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 256
x = T.batch_inputs(9, 2, size).cuda()
rec = {}
for dt in (torch.float32, torch.bfloat16):
    m, *_ = make_model(dt, name)
    outs = {}
    hooks = []
    for n, mod in m.named_modules():
        if n.count(".") == 1 and n.startswith("layer") or n in ("preprocess",) or n.startswith("deconv"):
            hooks.append(mod.register_forward_hook(lambda mod, i, o, n=n: outs.__setitem__(n, o.detach().float().cpu())))
    with torch.no_grad():
        m(x, decode=False)
    rec[dt] = outs
    for h in hooks:
        h.remove()
for n in rec[torch.float32]:
    a, b = rec[torch.bfloat16].get(n), rec[torch.float32][n]
    if a is None or a.shape != b.shape:
        print(n, "shape", None if a is None else a.shape, b.shape)
        continue
    print("%-16s %s rel %.4f" % (n, tuple(b.shape), ((a - b).abs().max() / b.abs().max()).item()), flush=True)
