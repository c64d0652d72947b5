"""Time the HBM-bound kernels of the Res10 B=32 step at their largest shapes, one process.

python tools/hbm_bench.py [--reps 20]
Prints per launch: microseconds and achieved GB/s over the algorithmic bytes (each tensor read or
written once), HIP events on the launch stream.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import lib as L  # noqa: E402
from scdhip import ops  # noqa: E402


def timed(fn, reps):
    fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="bn,heads,stem,cpool", help="comma list of groups")
    a = ap.parse_args()
    groups = set(a.only.split(","))
    dev = "cuda"
    bf = torch.bfloat16
    st = ops.stream
    rows = []

    def report(name, us, nbytes):
        rows.append((name, us, nbytes))
        print("%-34s %9.1f us %9.1f MB %8.0f GB/s" % (name, us, nbytes / 1e6, nbytes / us / 1e3), flush=True)

    if "cpool" in groups:
        # corner pools at the cornerNetCPool B=32 shape (32,128,128,128) bf16: fwd x(+addend) -> y, bwd x, dy -> dx
        x = torch.randn(32, 128, 128, 128, device=dev).to(bf)
        ad = torch.randn_like(x)
        g = torch.randn_like(x)
        B = x.numel() * 2
        for d in range(4):
            report("cpool_fwd+add dir%d 32x128x128x128" % d, timed(lambda: ops.cpool_fwd(x, d, addend=ad), a.reps),
                   3 * B)
            report("cpool_bwd dir%d 32x128x128x128" % d, timed(lambda: ops.cpool_bwd(x, g, d), a.reps), 3 * B)
        del x, ad, g
    for (N, H, W, C) in ([(32, 128, 128, 256), (32, 128, 128, 64), (32, 64, 64, 128)] if "bn" in groups else []):
        y = torch.randn(N, H, W, C, device=dev).to(bf)
        r = torch.randn(N, H, W, C, device=dev).to(bf)
        d = torch.randn(N, H, W, C, device=dev).to(bf)
        out = torch.empty_like(y)
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.1
        mean = torch.randn(C, device=dev) * 0.1
        invstd = torch.rand(C, device=dev) + 0.5
        n = y.numel()
        B = n * 2
        tag = "%dx%dx%dx%d" % (N, H, W, C)
        report("bn_apply relu " + tag, timed(lambda: L.call(
            "scd_bn_apply", L.DT_BF16, y.data_ptr(), out.data_ptr(), C, n, sc.data_ptr(), sh.data_ptr(), 0, 0, 0, 1,
            st()), a.reps), 2 * B)
        report("bn_apply res+bn relu " + tag, timed(lambda: L.call(
            "scd_bn_apply", L.DT_BF16, y.data_ptr(), out.data_ptr(), C, n, sc.data_ptr(), sh.data_ptr(), r.data_ptr(),
            sc.data_ptr(), sh.data_ptr(), 1, st()), a.reps), 3 * B)
        stats = torch.zeros(L.STAT_REPLICAS * 2 * C, dtype=torch.float64, device=dev)
        report("bn_bwd_reduce relu " + tag, timed(lambda: L.call(
            "scd_bn_bwd_reduce", L.DT_BF16, d.data_ptr(), 0, y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
            mean.data_ptr(), invstd.data_ptr(), C, n, stats.data_ptr(), st()), a.reps), 2 * B)
        report("bn_bwd_reduce mask " + tag, timed(lambda: L.call(
            "scd_bn_bwd_reduce", L.DT_BF16, d.data_ptr(), r.data_ptr(), y.data_ptr(), 0, 0,
            mean.data_ptr(), invstd.data_ptr(), C, n, stats.data_ptr(), st()), a.reps), 3 * B)
        coef = torch.randn(3 * C, device=dev)
        report("bn_bwd_apply relu " + tag, timed(lambda: L.call(
            "scd_bn_bwd_apply", L.DT_BF16, d.data_ptr(), 0, y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
            coef.data_ptr(), C, n, out.data_ptr(), 0, st()), a.reps), 3 * B)
        report("bn_bwd_apply mask+dz " + tag, timed(lambda: L.call(
            "scd_bn_bwd_apply", L.DT_BF16, d.data_ptr(), r.data_ptr(), y.data_ptr(), 0, 0,
            coef.data_ptr(), C, n, out.data_ptr(), r.data_ptr(), st()), a.reps), 5 * B)
        del y, r, d, out

    if "heads" in groups:
        heads_rows(a, report, dev, bf, st)
    if "stem" in groups:
        stem_rows(a, report, dev, bf, st)
    print("total us: %.1f" % sum(r[1] for r in rows))


def heads_rows(a, report, dev, bf, st):
    # heads tail backward: hid (32,128,128,384) bf16, douts NCHW fp32 (1,4,2 channels)
    N, HW, nh, Hd = 32, 128 * 128, 3, 128
    od = [1, 4, 2]
    hid = torch.randn(N * HW, nh * Hd, device=dev).to(bf)
    dhid = torch.empty_like(hid)
    w1 = [torch.randn(o, Hd, device=dev) * 0.05 for o in od]
    dts = [torch.randn(N, o, HW, device=dev) for o in od]
    odarr = L.int_array(od)
    acc = torch.zeros(L.lib().scd_heads_bwd_accsize(nh, Hd, odarr) // 8, dtype=torch.float64, device=dev)
    wp = L.ptr_array([w.data_ptr() for w in w1])
    dp = L.ptr_array([t.data_ptr() for t in dts])
    report("heads_bwd 32x128x128x384", timed(lambda: L.call(
        "scd_heads_bwd", L.DT_BF16, hid.data_ptr(), N, HW, nh, Hd, odarr, wp, dp, dhid.data_ptr(), acc.data_ptr(),
        st()), a.reps), hid.numel() * 4 + N * HW * 7 * 4)
    del hid, dhid


def stem_rows(a, report, dev, bf, st):
    # stem pool backward + BN reduce: y (32,256,256,64), dout (32,128,128,64), argmax u8
    N, H, W, C = 32, 256, 256, 64
    y = torch.randn(N, H, W, C, device=dev).to(bf)
    dz = torch.empty_like(y)
    dout = torch.randn(N, H // 2, W // 2, C, device=dev).to(bf)
    am = torch.randint(0, 9, (N, H // 2, W // 2, C), dtype=torch.uint8, device=dev)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.1
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    stats = torch.zeros(L.STAT_REPLICAS * 2 * C, dtype=torch.float64, device=dev)
    report("stem_pool_bwd_bn 32x256x256x64", timed(lambda: L.call(
        "scd_stem_pool_bwd_bn", L.DT_BF16, dout.data_ptr(), am.data_ptr(), y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
        mean.data_ptr(), invstd.data_ptr(), dz.data_ptr(), stats.data_ptr(), N, H, W, C, H // 2, W // 2, st()),
        a.reps), y.numel() * 4 + dout.numel() * 3)
    pooled = torch.empty_like(dout)
    report("stem_pool_fwd 32x256x256x64", timed(lambda: L.call(
        "scd_stem_pool_fwd", L.DT_BF16, y.data_ptr(), sc.data_ptr(), sh.data_ptr(), pooled.data_ptr(), am.data_ptr(),
        N, H, W, C, H // 2, W // 2, st()), a.reps), y.numel() * 2 + dout.numel() * 3)
    # direct stem conv forward / weight gradient: x (32,1,512,512) fp32 -> y (32,256,256,64) bf16
    xs = torch.randn(32, 1, 512, 512, device=dev)
    w = torch.randn(64, 1, 7, 7, device=dev) / 7.0
    wpk = ops.pack_weight(w, bf, 0, ldp=64)
    st64 = torch.zeros(L.STAT_REPLICAS * 2 * 64, dtype=torch.float64, device=dev)
    ys = ops.stem_conv_fwd(xs, wpk, stats=st64)
    report("stem_conv_fwd 32x512x512 -> 64ch", timed(lambda: ops.stem_conv_fwd(xs, wpk, stats=st64), a.reps),
           xs.numel() * 4 + ys.numel() * 2)
    dw = torch.zeros_like(w)
    report("stem_conv_wgrad (dz, y, coef)", timed(lambda: ops.stem_conv_wgrad(ys, xs, dw, ybn=ys,
                                                                             coef=torch.ones(192, device=dev)),
                                                  a.reps), xs.numel() * 4 + ys.numel() * 4)


if __name__ == "__main__":
    main()
