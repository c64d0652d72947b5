"""Calibrate the sustained MFMA rate of this box with the vendor GEMM (torch.matmul -> hipBLASLt), for the heads
and ping-pong kernels' shapes: what rate a plain library GEMM of the same M/N/K holds under the same clocks.

python tools/gemm_calib.py [--reps 20]
"""
import argparse
import json

import torch


def rate(m, n, k, reps, dt=torch.bfloat16):
    dev = torch.device("cuda", 0)
    a = torch.randn(m, k, device=dev).to(dt)
    b = torch.randn(k, n, device=dev).to(dt)
    c = torch.empty(m, n, device=dev, dtype=dt)
    for _ in range(3):
        torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b, out=c)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"m": m, "n": n, "k": k, "dtype": str(dt).split(".")[-1], "ms": round(ms, 4),
            "pflops": round(2.0 * m * n * k / ms / 1e12, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    shapes = [(8192, 8192, 8192), (16384, 16384, 16384),
              (524288, 384, 2304),      # Res10 heads conv as a plain GEMM (B=32, 128x128 px, 9*256 -> 384)
              (131072, 256, 2304),      # deconv-size ping-pong shape
              (2304, 384, 524288)]      # heads weight gradient (K = pixels)
    for s in shapes:
        print(json.dumps(rate(*s, a.reps)), flush=True)


if __name__ == "__main__":
    main()
