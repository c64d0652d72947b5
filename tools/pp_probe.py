"""Time the backward's big ping-pong GEMMs alone (HIP events, 10 launches each), with and without the BN-backward-sum
epilogue, to split each into main loop and epilogue cost.

python tools/pp_probe.py
  heads dgrad    dy (32,128,128,128) -> dx (32,128,128,256), 3x3 (the heatmap head's dense input gradient)
  deconv3 dgrad  dy (32,128,128,256) -> dx (32,64,64,256), ConvTranspose 4x4 / 2 input gradient
  heads fwd      for scale: feat (32,128,128,256) -> 384 hidden, 3x3, plain epilogue (no tails)
"""
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def bnstate(C, dev):
    g = torch.Generator(device=dev).manual_seed(5)
    return types.SimpleNamespace(mean=torch.randn(C, device=dev, generator=g) * 0.1,
                                 invstd=torch.rand(C, device=dev, generator=g) + 0.5,
                                 scale=torch.rand(C, device=dev, generator=g) + 0.5,
                                 shift=torch.randn(C, device=dev, generator=g) * 0.1)


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    bf = torch.bfloat16
    out = {}
    # heads dgrad
    dy = torch.randn(32, 128, 128, 128, device=dev, generator=g).to(bf)
    w = torch.randn(128, 256, 3, 3, device=dev, generator=g) / 30
    wt = ops.pack_weight(w, bf, 1)
    y = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
    st = bnstate(256, dev)
    stats = ops.new_stats(256, dev)
    dx = torch.empty(32, 128, 128, 256, device=dev, dtype=bf)
    fl = 2.0 * 32 * 128 * 128 * 256 * 9 * 128
    t0 = timed(lambda: ops.conv_dgrad(dy, wt, 256, 128, 128, 3, 3, 1, 1, out=dx))
    t1 = timed(lambda: ops.conv_dgrad(dy, wt, 256, 128, 128, 3, 3, 1, 1, out=dx, bn_bwd=(st, y, stats)))
    out["heads_dgrad"] = {"plain_us": round(t0, 1), "bnbwd_us": round(t1, 1), "gflop": round(fl / 1e9, 1),
                          "plain_pflops": round(fl / t0 / 1e9, 3), "bnbwd_pflops": round(fl / t1 / 1e9, 3)}
    # deconv3 dgrad (ConvTranspose2d(256, 256, 4, 2, 1) input gradient = conv forward of dy)
    dy3 = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
    w3 = torch.randn(256, 256, 4, 4, device=dev, generator=g) / 60
    wp3 = ops.pack_weight(w3, bf, 0)
    y3 = torch.randn(32, 64, 64, 256, device=dev, generator=g).to(bf)
    dx3 = torch.empty(32, 64, 64, 256, device=dev, dtype=bf)
    fl3 = 2.0 * 32 * 64 * 64 * 256 * 16 * 256
    t2 = timed(lambda: ops.deconv_dgrad(dy3, wp3, 256, 4, 2, 1, out=dx3))
    t3 = timed(lambda: ops.deconv_dgrad(dy3, wp3, 256, 4, 2, 1, out=dx3, bn_bwd=(st, y3, stats)))
    out["deconv3_dgrad"] = {"plain_us": round(t2, 1), "bnbwd_us": round(t3, 1), "gflop": round(fl3 / 1e9, 1),
                            "plain_pflops": round(fl3 / t2 / 1e9, 3), "bnbwd_pflops": round(fl3 / t3 / 1e9, 3)}
    # heads forward without tails
    feat = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
    wh = torch.randn(384, 256, 3, 3, device=dev, generator=g) / 48
    wph = ops.pack_weight(wh, bf, 0)
    hid = torch.empty(32, 128, 128, 384, device=dev, dtype=bf)
    flh = 2.0 * 32 * 128 * 128 * 384 * 9 * 256
    t4 = timed(lambda: ops.conv_fwd(feat, wph, 384, 3, 3, 1, 1, out=hid))
    out["heads_fwd_plain"] = {"us": round(t4, 1), "gflop": round(flh / 1e9, 1), "pflops": round(flh / t4 / 1e9, 3)}
    for k, v in out.items():
        print(k, json.dumps(v), flush=True)


if __name__ == "__main__":
    main()
