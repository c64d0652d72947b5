"""Time the GPU validation metrics for one validation batch: decoded detections (N images x K=100) against
N x 30 objects -> scd_ceval_count + scd_ceval_emit (evaluation) and scd_ceval_summary (expression), HIP events
on the launch stream; the host read of the per-image counts is inside the timed region.
The reference's CPU time for the same shapes is measured in the build container by
`python tests/golden/make_golden_eval.py --time` (it imports the reference, which never reaches the GPU box)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from scdhip import ops  # noqa: E402


def case(N, K=100, L=30, seed=0):
    rs = np.random.RandomState(seed)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    ys2 = np.concatenate([rs.uniform(0, 4, (N, L, 2)), rs.uniform(-6, 6, (N, L, 2)), rs.uniform(1, 3, (N, L, 1)),
                          rs.uniform(1, 7, (N, L, 1))], -1).astype(np.float32)
    inds = rs.randint(0, 128 * 128, (N, L)).astype(np.int64)
    ctx = np.where(rs.rand(N, K) < 0.3, (inds % 128)[:, rs.randint(0, L, K)], rs.randint(0, 128, (N, K)))
    cty = np.where(rs.rand(N, K) < 0.3, (inds // 128)[:, rs.randint(0, L, K)], rs.randint(0, 128, (N, K)))
    regr = np.concatenate([rs.uniform(-6, 6, (N, K, 2)), rs.uniform(0.5, 4, (N, K, 2))], -1).astype(np.float32)
    return [t(rs.rand(N, K).astype(np.float32)), t(cty.astype(np.int64)), t(ctx.astype(np.int64)),
            t(rs.uniform(0, 4, (N, K, 2)).astype(np.float32)), t(regr), t(ys2), t(inds)]


for N in (32, 256):
    args = case(N)
    ops.center_eval(*args)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        s = ops.center_eval(*args)
    torch.cuda.synchronize()
    ev_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        m, ap = ops.center_eval_summary(s, N * 30)
    sm_ms = (time.perf_counter() - t0) / reps * 1e3
    print("N=%d K=100 L=30: evaluation %.3f ms (incl. counts read), expression summary %.3f ms over %d pairs kept"
          % (N, ev_ms, sm_ms, s[0].numel()))

# whole-slide tiling (scd_slide_tiles) for a 3092 x 2056 RGB slide (48 clips of 512^2) and detections
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import slide  # noqa: E402

rs = np.random.RandomState(1)
rgb = torch.from_numpy(rs.randint(0, 256, (2056, 3092, 3)).astype(np.uint8)).cuda()
clips, g = slide.tiles(rgb)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(20):
    ops.slide_tiles(rgb, 512, 384, g["clipH"], g["clipV"], g["padLR"], g["padTB"], True)
e1.record(s)
e1.synchronize()
ms = e0.elapsed_time(e1) / 20
print("slide tiles 3092x2056 -> %d clips: %.3f ms (%.0f GB/s of clip writes)" % (clips.shape[0], ms,
                                                                             clips.numel() * 4 / ms / 1e6))
dec = torch.rand(10, clips.shape[0], 100, device="cuda")
t0 = time.perf_counter()
for _ in range(20):
    ops.slide_detections(dec, 384, g["padLR"], g["padTB"], g["clipV"], 0.3)
print("slide detections (48 x 100, incl. count read): %.3f ms" % ((time.perf_counter() - t0) / 20 * 1e3))
