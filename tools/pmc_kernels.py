"""Launch ONE dominant-kernel shape of a BASELINE config repeatedly, for rocprofv3 --pmc passes (HBM bytes per
launch of exactly that kernel on exactly that shape; bench.py reads the summaries for its `traffic` fields).

python tools/pmc_kernels.py --case {lastconv,cpool_add,heads_res50}[,...] [--reps 5]

  lastconv     cornerNetCPool (configs[3]) CornerPool lastConv: 3x3 256->256 conv + BN sums, B=32 at 128x128, bf16
               (conv_gemm_pp_kernel<256,false>, as _train_bn_conv launches it)
  cpool_add    its corner pool with the addend: (32,128,128,128) bf16 (cpool_fwd_kernel)
  heads_res50  centerOffsetRes50 1024^2 (configs[4]) fused heads GEMM, B=16 at 256x256, fp16, hidden channels of the
               size / offset heads kept at 30 random pixels per image (conv_gemm_heads384_kernel, as HeadsFn)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True, help="comma-separated: lastconv, cpool_add, heads_res50")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for case in a.case.split(","):
        run_case(case, a.reps)


def run_case(case, reps):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    if case == "lastconv":
        x = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(torch.bfloat16)
        w = torch.randn(256, 256, 3, 3, device=dev, generator=g) / 48.0
        wp = ops.pack_weight(w, torch.bfloat16, 0)
        stats = ops.new_stats(256, dev)

        def run():
            ops.conv_fwd(x, wp, 256, 3, 3, 1, 1, stats=stats)
    elif case == "cpool_add":
        x = torch.randn(32, 128, 128, 128, device=dev, generator=g).to(torch.bfloat16)
        add = torch.randn(32, 128, 128, 128, device=dev, generator=g).to(torch.bfloat16)

        def run():
            ops.cpool_fwd(x, 1, addend=add)
    elif case == "heads_res50":
        N, H, W, Cin, Hd = 16, 256, 256, 256, 128
        dt = torch.float16
        feat = torch.randn(N, H, W, Cin, device=dev, generator=g).to(dt)
        w0 = torch.randn(3 * Hd, Cin, 3, 3, device=dev, generator=g) / 48.0
        wp = ops.pack_weight(w0, dt, 0)
        b0 = torch.randn(3 * Hd, device=dev, generator=g)
        od = [1, 4, 2]
        w1 = [torch.randn(o, Hd, 1, 1, device=dev, generator=g) for o in od]
        b1 = [torch.randn(o, device=dev, generator=g) for o in od]
        outs = [torch.empty(N, o, H, W, device=dev) for o in od]
        hid = torch.empty(N, H, W, 3 * Hd, device=dev, dtype=dt)
        inds = torch.randint(0, H * W, (N, 30), device=dev, generator=g)
        keep = ops.heads_keep_map(inds, N, H * W)
        args = (ops.dt(feat), ops.ptr(feat), ops.ptr(wp), ops.ptr(hid), ops.ptr(b0), N, H, W, Cin, 3,
                ops.L.int_array(od), ops.L.ptr_array([t.data_ptr() for t in w1]),
                ops.L.ptr_array([t.data_ptr() for t in b1]), ops.L.ptr_array([t.data_ptr() for t in outs]),
                ops.ptr(keep), Hd)

        def run():
            ops.L.call("scd_conv_gemm_heads_keep", *args, ops.stream())
    else:
        raise SystemExit("unknown case %s" % case)
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    print("ok", case, reps)


if __name__ == "__main__":
    main()
