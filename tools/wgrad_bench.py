"""Weight-gradient GEMM and split reduce timed separately, per Res10 B=32 shape and split count.

python tools/wgrad_bench.py [--ns 0,8,16]   (0 = the library's split model)
HIP events on the launch stream; TF/s over the GEMM alone and over GEMM + reduce.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402

L = ops.L
B = 32
# name, g (output gradient) N,Ho,Wo,Cg ; x N,Hi,Wi,Ci ; k, stride, pad
SHAPES = [
    ("layer1 3x3", (B, 128, 128, 64), (B, 128, 128, 64), 3, 1, 1),
    ("layer2 3x3 s2", (B, 64, 64, 128), (B, 128, 128, 64), 3, 2, 1),
    ("layer2 3x3", (B, 64, 64, 128), (B, 64, 64, 128), 3, 1, 1),
    ("layer3 3x3 s2", (B, 32, 32, 256), (B, 64, 64, 128), 3, 2, 1),
    ("layer3 3x3", (B, 32, 32, 256), (B, 32, 32, 256), 3, 1, 1),
    ("layer4 3x3 s2", (B, 16, 16, 512), (B, 32, 32, 256), 3, 2, 1),
    ("layer4 3x3", (B, 16, 16, 512), (B, 16, 16, 512), 3, 1, 1),
    ("deconv1", (B, 16, 16, 512), (B, 32, 32, 256), 4, 2, 1),
    ("deconv2", (B, 32, 32, 256), (B, 64, 64, 256), 4, 2, 1),
    ("deconv3", (B, 64, 64, 256), (B, 128, 128, 256), 4, 2, 1),
    ("heatmap 3x3", (B, 128, 128, 128), (B, 128, 128, 256), 3, 1, 1),
]


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="0")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = "cuda"
    dt = torch.bfloat16
    print("%-16s %5s %9s %9s %9s %8s %8s" % ("layer", "ns", "gemm_us", "red_us", "total_us", "TF_gemm", "TF_all"))
    for name, gs, xs, k, s, p in SHAPES:
        if a.only and a.only not in name:
            continue
        g = torch.randn(*gs, device=dev).to(dt)
        x = torch.randn(*xs, device=dev).to(dt)
        N, Ho, Wo, Cg = gs
        _, Hi, Wi, Ci = xs
        T = k * k
        dh = L.int_array([r - p for r in range(k) for c in range(k)])
        dw = L.int_array([c - p for r in range(k) for c in range(k)])
        M = N * Ho * Wo
        flop = 2.0 * M * Cg * T * Ci
        dst = torch.zeros(Cg, Ci, k, k, device=dev)
        for nsv in [int(v) for v in a.ns.split(",")]:
            ns = nsv or L.lib().scd_conv_wgrad_nsplit2(ops.dt(g), M, Ho, Wo, Cg, T, Ci)
            ws = torch.empty(L.lib().scd_conv_wgrad_workspace(Cg, T, Ci, ns) // 4, dtype=torch.float32, device=dev)
            st = torch.cuda.current_stream().cuda_stream

            def gemm():
                L.call("scd_conv_wgrad", ops.dt(g), ops.ptr(g), ops.ptr(x), ops.ptr(ws), ns, N, Ho, Wo, Cg, Hi, Wi, Ci,
                       s, T, dh, dw, st)

            def red():
                L.call("scd_wgrad_reduce", ops.ptr(ws), ns, Cg, T, Ci, 0, Cg, Ci, Ci * T, T, 1, ops.ptr(dst), 0, 1.0,
                       st)
            gemm()
            red()
            e = [ev() for _ in range(3)]
            tg = tr = 0.0
            for _ in range(a.reps):
                e[0].record()
                gemm()
                e[1].record()
                red()
                e[2].record()
                e[2].synchronize()
                tg += e[0].elapsed_time(e[1])
                tr += e[1].elapsed_time(e[2])
            tg, tr = 1e3 * tg / a.reps, 1e3 * tr / a.reps
            print("%-16s %5d %9.1f %9.1f %9.1f %8.1f %8.1f" % (name, ns, tg, tr, tg + tr, flop / tg / 1e6,
                                                               flop / (tg + tr) / 1e6))


if __name__ == "__main__":
    main()
