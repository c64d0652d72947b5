import sys, torch
sys.path.insert(0, "scd-resnet_amd"); sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_model_gpu import make_model
from oracle import targets as T
for name in ["centerOffsetRes10", "centerOffsetRes50"]:
    for size in [128, 256, 512]:
        x = T.batch_inputs(9, 2, size).cuda()
        outs = {}
        for dt in (torch.float32, torch.bfloat16):
            m, *_ = make_model(dt, name)
            with torch.no_grad():
                outs[dt] = {k: v.float().cpu() for k, v in m(x, decode=False)[0].items()}
            del m
        errs = {k: ((outs[torch.bfloat16][k] - outs[torch.float32][k]).abs().max() / outs[torch.float32][k].abs().max()).item() for k in ("heatmap", "regr", "offset")}
        print(name, size, {k: round(v, 4) for k, v in errs.items()}, flush=True)
