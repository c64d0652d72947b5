"""Time the stem kernels at the Res10 B=32 512^2 shape: conv (+BN statistics), BN-apply+ReLU+max-pool, pool backward
(+BN backward sums) and the weight gradient (+BN backward apply) (stem.hip, layers.hip), HIP events.

python tools/stem_bench.py [--reps 20] [--batch 32]
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
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = "cuda"
    B = a.batch
    x = torch.randn(B, 1, 512, 512, device=dev)
    w = torch.randn(64, 1, 7, 7, device=dev) / 7
    bn = torch.nn.BatchNorm2d(64).to(dev)
    wpk = ops.pack_weight(w, torch.bfloat16, 0, ldp=64)
    stats = ops.new_stats(64, dev)
    y = ops.stem_conv_fwd(x, wpk, stats=stats)
    M = y.numel() // 64
    st = ops.bn_finalize(bn, stats, 64, M)
    out, am = ops.stem_pool_fwd(y, st)
    dout = torch.randn(out.shape, device=dev).to(torch.bfloat16)
    dw = torch.zeros_like(w)
    rows = []

    def rep(name, us):
        rows.append((name, us))
        print("%-40s %9.1f us" % (name, us), flush=True)

    # chain with the activation
    rep("stem_conv_fwd (+stats)", timed(lambda: ops.stem_conv_fwd(x, wpk, stats=stats), a.reps))
    rep("stem_pool_fwd", timed(lambda: ops.stem_pool_fwd(y, st), a.reps))
    rep("stem_pool_bwd_bn", timed(lambda: ops.stem_pool_bwd_bn(bn, dout, am, y, st), a.reps))
    dz, coef = ops.stem_pool_bwd_bn(bn, dout, am, y, st)
    rep("stem_conv_wgrad (+BN apply)", timed(lambda: ops.stem_conv_wgrad(dz, x, dw, ybn=y, coef=coef), a.reps))
    print("chain %.1f us" % sum(us for _, us in rows))
    # the one-pass backward the model runs (scd_stem_bwd_fused + reduce + BN finalize + combine)
    rep("stem_backward_fused (one pass)", timed(lambda: ops.stem_backward_fused(bn, dout, am, y, st, x, wpk, dw),
                                                a.reps))

if __name__ == "__main__":
    main()
