"""Time the backward input-gradient GEMMs that carry a BN layer's backward sums in their epilogue (Res10 B=32):
the heatmap head's 3x3 dgrad (128 -> 256 channels at 128^2) and deconv3's dgrad (256 -> 256, k4 s2, 128^2 -> 64^2),
plain and with the BN-backward epilogue (scd_conv_gemm_bnbwd).  Kernel choice follows the process env
(SCD_GEMM_PP / SCD_GEMM_RING), so run it once per setting.

python tools/dgrad_bench.py [--reps 20]
"""
import argparse
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402

B = 32


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def bn_args(C, y):
    st = types.SimpleNamespace(mean=torch.randn(C, device="cuda") * 0.1, invstd=torch.rand(C, device="cuda") + 0.5,
                               scale=torch.rand(C, device="cuda") + 0.5, shift=torch.randn(C, device="cuda") * 0.1)
    return (st, y, torch.zeros(4 * 64 * C, dtype=torch.float64, device="cuda"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dt = torch.bfloat16
    tag = "PP=%s RING=%s" % (os.environ.get("SCD_GEMM_PP", "1"), os.environ.get("SCD_GEMM_RING", "auto"))
    # heatmap head dgrad: dhid [B,128,128,128] -> dX [B,128,128,256], W [128,256,3,3]
    w = torch.randn(128, 256, 3, 3, device="cuda") / (256 * 9) ** 0.5
    wt = ops.pack_weight(w, dt, 1)
    gy = torch.randn(B, 128, 128, 128, device="cuda").to(dt)
    yb = torch.randn(B, 128, 128, 256, device="cuda").to(dt)
    out = torch.empty(B, 128, 128, 256, device="cuda", dtype=dt)
    fl = 2.0 * B * 128 * 128 * 256 * 128 * 9
    bnb = bn_args(256, yb)
    for name, fn in (("heads-hm dgrad", lambda: ops.conv_dgrad(gy, wt, 256, 128, 128, 3, 3, 1, 1, out=out)),
                     ("heads-hm dgrad+bnb", lambda: ops.conv_dgrad(gy, wt, 256, 128, 128, 3, 3, 1, 1, out=out,
                                                                   bn_bwd=bnb))):
        ms = timed(fn, a.reps)
        print("%-22s %-18s %8.3f ms %7.1f TF/s" % (name, tag, ms, fl / ms / 1e9))
    # deconv3 dgrad: dy [B,128,128,256] -> dX [B,64,64,256], W_t [256,256,4,4]
    w = torch.randn(256, 256, 4, 4, device="cuda") / (256 * 4) ** 0.5
    wp = ops.pack_weight(w, dt, 0)
    gy = torch.randn(B, 128, 128, 256, device="cuda").to(dt)
    yb = torch.randn(B, 64, 64, 256, device="cuda").to(dt)
    out = torch.empty(B, 64, 64, 256, device="cuda", dtype=dt)
    fl = 2.0 * B * 64 * 64 * 256 * 256 * 16
    bnb = bn_args(256, yb)
    for name, fn in (("deconv3 dgrad", lambda: ops.deconv_dgrad(gy, wp, 256, out=out)),
                     ("deconv3 dgrad+bnb", lambda: ops.deconv_dgrad(gy, wp, 256, out=out, bn_bwd=bnb))):
        ms = timed(fn, a.reps)
        print("%-22s %-18s %8.3f ms %7.1f TF/s" % (name, tag, ms, fl / ms / 1e9))


if __name__ == "__main__":
    main()
