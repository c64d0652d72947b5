"""Launch ONE dominant-kernel shape of a BASELINE config repeatedly, for rocprofv3 --pmc passes (HBM bytes per
launch of exactly that kernel on exactly that shape; bench.py reads the summaries for its `traffic` fields).

python tools/pmc_kernels.py --case {lastconv,cpool_add,heads_res50,s1x1_fwd,s1x1_bnbwd}[,...] [--reps 5]

  lastconv     cornerNetCPool (configs[3]) CornerPool lastConv: 3x3 256->256 conv + BN sums, B=32 at 128x128, bf16
               (conv_gemm_pp_kernel<256,false>, as _train_bn_conv launches it)
  cpool_add    its corner pool with the addend: (32,128,128,128) bf16 (cpool_fwd_kernel)
  heads_res50  centerOffsetRes50 1024^2 (configs[4]) fused heads GEMM, B=16 at 256x256, fp16, hidden channels of the
               size / offset heads kept at 30 random pixels per image (conv_gemm_heads384_kernel, as HeadsFn)
  s1x1_fwd     its layer1 conv3 / downsample forward: 1x1 64 -> 256 + BN statistics, B=16 at 256x256, fp16
               (conv1x1_stream_kernel<64,256,0,4,2,4>; algorithmic 2 x (64 + 256) B = 640 B per pixel, 671 MB)
  heads_dgrad  centerOffsetRes10 B=32 (configs[1]) heatmap-head input gradient with the deconv3 BN's backward sums:
               dhid (32,128,128,128) -> dfeat (32,128,128,256), 3x3 (conv_gemm_pp_kernel<256>, bnbwd epilogue)
  deconv3_dgrad  its deconv3 input gradient with the deconv2 BN's backward sums: dy (32,128,128,256) -> (32,64,64,256),
               ConvTranspose 4x4 / 2 (conv_gemm_pp_kernel<256>, bnbwd epilogue)
  wgrad_hm     its heatmap-head weight gradient: dhid (32,128,128,128) x feat (32,128,128,256), 3x3
               (conv_wgrad_pp2_kernel<2> + wgrad_reduce_kernel)
  wgrad_d3     its deconv3 weight gradient: x (32,64,64,256) x dy (32,128,128,256), 4x4 / 2 taps
               (conv_wgrad_pp2_kernel<4> + wgrad_reduce_kernel)
  s1x1_bnbwd   its layer1 conv3 input gradient with the bn2 backward sums: 1x1 256 -> 64, B=16 at 256x256, fp16
               (conv1x1_stream_kernel<256,64,2,1,1,4>; 2 x (256 + 64 + 64) B = 768 B per pixel, 805 MB)
"""
import argparse
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True, help="comma-separated: lastconv, cpool_add, heads_res50, s1x1_fwd, s1x1_bnbwd, heads_dgrad, "
                    "deconv3_dgrad, wgrad_hm, wgrad_d3")
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
    elif case in ("heads_dgrad", "deconv3_dgrad"):
        bf = torch.bfloat16
        st = types.SimpleNamespace(mean=torch.randn(256, device=dev, generator=g) * 0.1,
                                   invstd=torch.rand(256, device=dev, generator=g) + 0.5,
                                   scale=torch.rand(256, device=dev, generator=g) + 0.5,
                                   shift=torch.randn(256, device=dev, generator=g) * 0.1)
        stats = ops.new_stats(256, dev)
        if case == "heads_dgrad":
            dy = torch.randn(32, 128, 128, 128, device=dev, generator=g).to(bf)
            wt = ops.pack_weight(torch.randn(128, 256, 3, 3, device=dev, generator=g) / 30, bf, 1)
            y = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
            dx = torch.empty(32, 128, 128, 256, device=dev, dtype=bf)

            def run():
                ops.conv_dgrad(dy, wt, 256, 128, 128, 3, 3, 1, 1, out=dx, bn_bwd=(st, y, stats))
        else:
            dy = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
            wp = ops.pack_weight(torch.randn(256, 256, 4, 4, device=dev, generator=g) / 60, bf, 0)
            y = torch.randn(32, 64, 64, 256, device=dev, generator=g).to(bf)
            dx = torch.empty(32, 64, 64, 256, device=dev, dtype=bf)

            def run():
                ops.deconv_dgrad(dy, wp, 256, 4, 2, 1, out=dx, bn_bwd=(st, y, stats))
    elif case in ("wgrad_hm", "wgrad_d3"):
        bf = torch.bfloat16
        if case == "wgrad_hm":
            gy = torch.randn(32, 128, 128, 128, device=dev, generator=g).to(bf)
            x = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
            dst = torch.zeros(128, 256, 3, 3, device=dev)
            k, s, pd = 3, 1, 1
        else:
            gy = torch.randn(32, 64, 64, 256, device=dev, generator=g).to(bf)
            x = torch.randn(32, 128, 128, 256, device=dev, generator=g).to(bf)
            dst = torch.zeros(256, 256, 4, 4, device=dev)
            k, s, pd = 4, 2, 1
        T = k * k

        def run():
            ops._conv_wgrad(gy, x, k, k, s, pd, dst, (dst.shape[1] * T, T, 1))
    elif case in ("s1x1_fwd", "s1x1_bnbwd"):
        N, H, W = 16, 256, 256
        dt = torch.float16
        K, C = 64, 256                       # conv3: 64 -> 256 (its input gradient: 256 -> 64)
        w = torch.randn(C, K, 1, 1, device=dev, generator=g) / K ** 0.5
        if case == "s1x1_fwd":
            x = torch.randn(N, H, W, K, device=dev, generator=g).to(dt)
            wp = ops.pack_weight(w, dt, 0)
            stats = ops.new_stats(C, dev)

            def run():
                ops.conv_fwd(x, wp, C, 1, 1, 1, 0, stats=stats)
        else:
            dy = torch.randn(N, H, W, C, device=dev, generator=g).to(dt)
            ybn = torch.randn(N, H, W, K, device=dev, generator=g).to(dt)
            wt = ops.pack_weight(w, dt, 1)

            class St:
                pass
            st = St()
            st.mean = torch.randn(K, device=dev, generator=g) * 0.1
            st.invstd = torch.rand(K, device=dev, generator=g) + 0.5
            st.scale = torch.rand(K, device=dev, generator=g) + 0.5
            st.shift = torch.randn(K, device=dev, generator=g) * 0.2
            bst = ops.new_stats(K, dev)

            def run():
                ops.conv_dgrad(dy, wt, K, H, W, 1, 1, 1, 0, bn_bwd=(st, ybn, bst))
    else:
        raise SystemExit("unknown case %s" % case)
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    print("ok", case, reps)


if __name__ == "__main__":
    main()
