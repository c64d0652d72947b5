"""Time the Res10 B=32 GEMM shapes (fwd / dgrad / wgrad of every conv + deconv + heads) in one process.

python tools/gemm_bench.py [--dtype bf16] [--reps 10]
Prints achieved TFLOP/s per launch shape (HIP events on the launch stream).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402

B = 32
# name, Cin, H, W, Cout, k, stride, pad, kind
SHAPES = [
    ("stem 1x1(im2col)", 64, 256, 256, 64, 1, 1, 0, "conv"),
    ("layer1 3x3", 64, 128, 128, 64, 3, 1, 1, "conv"),
    ("layer2 3x3 s2", 64, 128, 128, 128, 3, 2, 1, "conv"),
    ("layer2 3x3", 128, 64, 64, 128, 3, 1, 1, "conv"),
    ("layer3 3x3", 256, 32, 32, 256, 3, 1, 1, "conv"),
    ("layer4 3x3", 512, 16, 16, 512, 3, 1, 1, "conv"),
    ("deconv1", 512, 16, 16, 256, 4, 2, 1, "deconv"),
    ("deconv2", 256, 32, 32, 256, 4, 2, 1, "deconv"),
    ("deconv3", 256, 64, 64, 256, 4, 2, 1, "deconv"),
    ("heads 3x3 N=384", 256, 128, 128, 384, 3, 1, 1, "conv"),
]


def timed(fn, reps):
    fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="", help="comma-separated substrings of layer names")
    a = ap.parse_args()
    only = [o for o in a.only.split(",") if o]
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = "cuda"
    print("%-20s %-6s %10s %10s %8s" % ("layer", "pass", "GFLOP", "ms", "TF/s"))
    tot_ms = 0.0
    for name, Cin, H, W, Cout, k, s, p, kind in SHAPES:
        if only and not any(o in name for o in only):
            continue
        if kind == "conv":
            w = torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5
            x = torch.randn(B, H, W, Cin, device=dev).to(dt)
            Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
            gy = torch.randn(B, Ho, Wo, Cout, device=dev).to(dt)
            flops = 2.0 * B * Ho * Wo * Cout * Cin * k * k
            wp, wt = ops.pack_weight(w, dt, 0), ops.pack_weight(w, dt, 1)
            dw = torch.zeros_like(w)
            runs = [("fwd", lambda: ops.conv_fwd(x, wp, Cout, k, k, s, p)),
                    ("dgrad", lambda: ops.conv_dgrad(gy, wt, Cin, H, W, k, k, s, p)),
                    ("wgrad", lambda: ops.conv_wgrad(gy, x, k, k, s, p, dw, (Cin * k * k, k * k, 1)))]
        else:
            w = torch.randn(Cin, Cout, k, k, device=dev) / (Cin * 4) ** 0.5
            x = torch.randn(B, H, W, Cin, device=dev).to(dt)
            gy = torch.randn(B, 2 * H, 2 * W, Cout, device=dev).to(dt)
            flops = 2.0 * B * H * W * Cin * Cout * k * k
            wp, wt = ops.pack_weight(w, dt, 0), ops.pack_weight(w, dt, 1)
            dw = torch.zeros_like(w)
            runs = [("fwd", lambda: ops.deconv_fwd(x, wt, Cout)),
                    ("dgrad", lambda: ops.deconv_dgrad(gy, wp, Cin)),
                    ("wgrad", lambda: ops.conv_wgrad(x, gy, k, k, s, p, dw, (Cout * k * k, k * k, 1)))]
        if name.startswith("heads") and dt == torch.bfloat16:
            # the fused head GEMM of the model (bias + ReLU + the three 1x1 tails in the epilogue)
            L = ops.L
            od = [1, 4, 2]
            b0 = torch.randn(Cout, device=dev) * 0.1
            w1 = [torch.randn(o, 128, device=dev) / 128 ** 0.5 for o in od]
            b1 = [torch.randn(o, device=dev) * 0.1 for o in od]
            outs = [torch.empty(B, o, H, W, device=dev) for o in od]
            hid = torch.empty(B, H, W, Cout, device=dev, dtype=dt)
            odarr, w1p, b1p = L.int_array(od), L.ptr_array([t.data_ptr() for t in w1]), \
                L.ptr_array([t.data_ptr() for t in b1])
            op = L.ptr_array([t.data_ptr() for t in outs])
            runs.insert(1, ("fused", lambda: L.call(
                "scd_conv_gemm_heads", ops.dt(x), ops.ptr(x), ops.ptr(wp), ops.ptr(hid), ops.ptr(b0), B, H, W, Cin,
                len(od), odarr, w1p, b1p, op, ops.stream())))
        for pas, fn in runs:
            ms = timed(fn, a.reps)
            tot_ms += ms
            print("%-20s %-6s %10.1f %10.3f %8.1f" % (name, pas, flops / 1e9, ms, flops / ms / 1e9))
    print("total GEMM ms (one of each, B=32): %.3f" % tot_ms)


if __name__ == "__main__":
    main()
