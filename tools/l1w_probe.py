"""Time the layer1 weight gradient (conv_wgrad_l1_kernel + its split reduce) alone on the Res10 B=32 shape
(dy, x: (32, 128, 128, 64) bf16, 3x3): HIP events, 10 launches.  Run against ablation builds
(SCDHIP_LIB=.../libscdhip_ablate41.so: no DMA after the prologue; 42: fragment reads, no MFMA) to find its bound.

python tools/l1w_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    dy = torch.randn(32, 128, 128, 64, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(32, 128, 128, 64, device=dev, generator=g).to(torch.bfloat16)
    dw = torch.zeros(64, 64, 3, 3, device=dev)

    def run():
        ops._conv_wgrad(dy, x, 3, 3, 1, 1, dw, (64 * 9, 9, 1), accumulate=False)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1000
    fl = 2.0 * 32 * 128 * 128 * 64 * 576
    print(json.dumps({"lib": os.path.basename(os.environ.get("SCDHIP_LIB", "libscdhip.so")), "us_with_reduce": round(us, 1),
                      "pflops": round(fl / us / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
