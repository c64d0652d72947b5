"""Achievable bf16 MFMA peak and the clocks the step's big GEMMs run at (MI355X_MICROARCH.md
"DVFS give-back" item 6).

python tools/clock_probe.py [--gemms]
  1. scdhip.calib.mfma_peak: bare 16x16x32 bf16 MFMA loops on random operands (1 and 2 waves per SIMD) and on zeros,
     each after >= 2.5 s of back-to-back launches: TFLOP/s, in-kernel clock, cycles per MFMA.
  2. --gemms (needs the stamped diagnostic build, SCDHIP_LIB=.../libscdhip_stamp.so: make variant VAR=stamp
     VFLAGS=-DSCD_STAMP=1): the Res10 B=32 heads forward (conv_gemm_heads384_kernel), the heatmap-head input gradient
     with the deconv3 BN's backward sums and the deconv3 input gradient (conv_gemm_pp_kernel), each run back to back
     for 2.5 s on random data, then one stamped launch: median in-kernel clock over workgroups, median main-loop
     cycles, and the HIP-event time per launch.
"""
import argparse
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import torch  # noqa: E402

from scdhip import calib, ops  # noqa: E402
from scdhip import lib as L  # noqa: E402


def sustained(fn, warm_s=2.5, reps=10):
    fn()
    torch.cuda.synchronize()
    t_end = time.time() + warm_s
    while time.time() < t_end:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def gemm_cases(dev):
    g = torch.Generator(device=dev).manual_seed(3)
    bf = torch.bfloat16
    cases = {}
    # heads forward, as HeadsFn launches it (keep map of 30 pixels per image)
    N, H, W, Cin, Hd = 32, 128, 128, 256, 128
    feat = torch.randn(N, H, W, Cin, device=dev, generator=g).to(bf)
    w0 = torch.randn(3 * Hd, Cin, 3, 3, device=dev, generator=g) / 48.0
    wp = ops.pack_weight(w0, bf, 0)
    b0 = torch.randn(3 * Hd, device=dev, generator=g)
    od = [1, 4, 2]
    w1 = [torch.randn(o, Hd, 1, 1, device=dev, generator=g) for o in od]
    b1 = [torch.randn(o, device=dev, generator=g) for o in od]
    outs = [torch.empty(N, o, H, W, device=dev) for o in od]
    hid = torch.empty(N, H, W, 3 * Hd, device=dev, dtype=bf)
    inds = torch.randint(0, H * W, (N, 30), device=dev, generator=g)
    keep = ops.heads_keep_map(inds, N, H * W)
    args = (ops.dt(feat), ops.ptr(feat), ops.ptr(wp), ops.ptr(hid), ops.ptr(b0), N, H, W, Cin, 3,
            L.int_array(od), L.ptr_array([t.data_ptr() for t in w1]), L.ptr_array([t.data_ptr() for t in b1]),
            L.ptr_array([t.data_ptr() for t in outs]), ops.ptr(keep), Hd)
    cases["heads_fwd"] = (lambda: L.call("scd_conv_gemm_heads_keep", *args, ops.stream()),
                          2.0 * N * H * W * 3 * Hd * 9 * Cin, (N * H * W + 191) // 192)
    # heatmap-head input gradient with the deconv3 BN's backward sums (the step's dense heads dgrad)
    dy = torch.randn(N, H, W, Hd, device=dev, generator=g).to(bf)
    wh = torch.randn(Hd, Cin, 3, 3, device=dev, generator=g) / 30
    wt = ops.pack_weight(wh, bf, 1)
    y = torch.randn(N, H, W, Cin, device=dev, generator=g).to(bf)
    st = types.SimpleNamespace(mean=torch.randn(Cin, device=dev, generator=g) * 0.1,
                               invstd=torch.rand(Cin, device=dev, generator=g) + 0.5,
                               scale=torch.rand(Cin, device=dev, generator=g) + 0.5,
                               shift=torch.randn(Cin, device=dev, generator=g) * 0.1)
    stats = ops.new_stats(Cin, dev)
    dx = torch.empty(N, H, W, Cin, device=dev, dtype=bf)
    cases["heads_dgrad_bnbwd"] = (lambda: ops.conv_dgrad(dy, wt, Cin, H, W, 3, 3, 1, 1, out=dx, bn_bwd=(st, y, stats)),
                                  2.0 * N * H * W * Cin * 9 * Hd, (N * H * W // 256))
    # deconv3 input gradient (ConvTranspose2d(256, 256, 4, 2, 1)) with the deconv2 BN's backward sums
    dy3 = torch.randn(N, 128, 128, 256, device=dev, generator=g).to(bf)
    w3 = torch.randn(256, 256, 4, 4, device=dev, generator=g) / 60
    wp3 = ops.pack_weight(w3, bf, 0)
    y3 = torch.randn(N, 64, 64, 256, device=dev, generator=g).to(bf)
    dx3 = torch.empty(N, 64, 64, 256, device=dev, dtype=bf)
    cases["deconv3_dgrad_bnbwd"] = (lambda: ops.deconv_dgrad(dy3, wp3, 256, 4, 2, 1, out=dx3, bn_bwd=(st, y3, stats)),
                                    2.0 * N * 64 * 64 * 256 * 16 * 256, N * 64 * 64 // 256)
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemms", action="store_true")
    a = ap.parse_args()
    lib = L.lib()
    print("library", lib.dll.scd_version().decode(), "stamped", lib.scd_calib_stamped_build(), flush=True)
    for k, z in ((1, False), (2, False), (2, True)):
        print("mfma_peak", json.dumps(calib.mfma_peak(waves_per_simd=k, zeros=z)), flush=True)
    if a.gemms:
        if not lib.scd_calib_stamped_build():
            raise SystemExit("--gemms needs the stamped build (SCDHIP_LIB=.../libscdhip_stamp.so)")
        dev = torch.device("cuda", 0)
        stamps = torch.zeros(16384 * 4, device=dev, dtype=torch.int64)
        for name, (fn, flop, nwg) in gemm_cases(dev).items():
            L.call("scd_calib_set_stamps", None)
            us = sustained(fn)
            stamps.zero_()
            L.call("scd_calib_set_stamps", ops.ptr(stamps))
            fn()
            torch.cuda.synchronize()
            L.call("scd_calib_set_stamps", None)
            ghz, cyc = calib.stamp_clock(stamps.view(-1, 4), nwg)
            print("gemm", name, json.dumps({"us": round(us, 1), "pflops": round(flop / us / 1e9, 3),
                                            "workgroups": nwg, "clock_ghz": round(ghz, 3) if ghz else None,
                                            "main_loop_cycles_median": cyc}), flush=True)


if __name__ == "__main__":
    main()
