"""Time the step's ping-pong GEMM shapes on the ping-pong kernel and on the two-workgroups-per-CU kernel
(conv_gemm_duo_kernel; SCD_GEMM_DUO=1, read per call), with the duo's first-round stagger at several lengths
(SCD_DUO_DELAY = percent of the default half tile).  HIP events, 20 launches each, random bf16 operands, B = 32.

python tools/duo_probe.py [--delays 0,50,100,200]
"""
import argparse
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def cases(dev):
    g = torch.Generator(device=dev).manual_seed(3)
    bf = torch.bfloat16
    st = types.SimpleNamespace(mean=torch.randn(256, device=dev, generator=g) * 0.1,
                               invstd=torch.rand(256, device=dev, generator=g) + 0.5,
                               scale=torch.rand(256, device=dev, generator=g) + 0.5,
                               shift=torch.randn(256, device=dev, generator=g) * 0.1)
    stats = ops.new_stats(256, dev)
    c = {}
    dy = torch.randn(32, 128, 128, 128, device=dev, generator=g).to(bf)
    wt = ops.pack_weight(torch.randn(128, 256, 3, 3, device=dev, generator=g) / 30, bf, 1)
    y = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
    dx = torch.empty(32, 128, 128, 256, device=dev, dtype=bf)
    c["heads_dgrad_bnbwd"] = (lambda: ops.conv_dgrad(dy, wt, 256, 128, 128, 3, 3, 1, 1, out=dx, bn_bwd=(st, y, stats)),
                              2.0 * 32 * 128 * 128 * 256 * 9 * 128)
    dy3 = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
    wp3 = ops.pack_weight(torch.randn(256, 256, 4, 4, device=dev, generator=g) / 60, bf, 0)
    y3 = torch.randn(32, 64, 64, 256, device=dev, generator=g).to(bf)
    dx3 = torch.empty(32, 64, 64, 256, device=dev, dtype=bf)
    c["deconv3_dgrad_bnbwd"] = (lambda: ops.deconv_dgrad(dy3, wp3, 256, 4, 2, 1, out=dx3, bn_bwd=(st, y3, stats)),
                                2.0 * 32 * 64 * 64 * 256 * 16 * 256)
    x3 = torch.randn(32, 64, 64, 256, device=dev, generator=g).to(bf)
    wt3 = ops.pack_weight(torch.randn(256, 256, 4, 4, device=dev, generator=g) / 60, bf, 1)
    c["deconv3_fwd_stats"] = (lambda: ops.deconv_fwd(x3, wt3, 256, stats=stats), 2.0 * 32 * 128 * 128 * 256 * 4 * 256)
    x2 = torch.randn(32, 32, 32, 256, device=dev, generator=g).to(bf)
    c["deconv2_fwd_stats"] = (lambda: ops.deconv_fwd(x2, wt3, 256, stats=stats), 2.0 * 32 * 64 * 64 * 256 * 4 * 256)
    dy2 = torch.randn(32, 64, 64, 256, device=dev, generator=g).to(bf)
    y2 = torch.randn(32, 32, 32, 256, device=dev, generator=g).to(bf)
    dx2 = torch.empty(32, 32, 32, 256, device=dev, dtype=bf)
    c["deconv2_dgrad_bnbwd"] = (lambda: ops.deconv_dgrad(dy2, wp3, 256, 4, 2, 1, out=dx2, bn_bwd=(st, y2, stats)),
                                2.0 * 32 * 32 * 32 * 256 * 16 * 256)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--delays", default="0,50,100,200")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, (fn, flop) in cases(dev).items():
        res = {}
        os.environ["SCD_GEMM_DUO"] = "0"
        res["pp"] = timed(fn)
        os.environ["SCD_GEMM_DUO"] = "1"
        for d in a.delays.split(","):
            os.environ["SCD_DUO_DELAY"] = d
            res["duo_d%s" % d] = timed(fn)
        os.environ["SCD_GEMM_DUO"] = "0"
        print(name, json.dumps({k: {"us": round(v, 1), "pflops": round(flop / v / 1e9, 3)} for k, v in res.items()}),
              flush=True)


if __name__ == "__main__":
    main()
