"""Time CenterNet target rendering for one B=32 batch: the dataset plugin's per-sample CPU renderer (the
reference's algorithm) vs scd_render_center_targets on the GPU (HIP events on the launch stream)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from scdhip import ops  # noqa: E402
from trainer.dataset.syntheticSCD import encode_targets, sample_objects  # noqa: E402

B, K = 32, 30
objs = [sample_objects(np.random.RandomState(500 + i)) for i in range(B)]
t0 = time.perf_counter()
for _ in range(5):
    for o in objs:
        encode_targets(o, 128)
cpu_ms = (time.perf_counter() - t0) / 5 * 1e3
locs = np.zeros((B, K, 8), np.float32)
counts = np.zeros(B, np.int32)
for b, o in enumerate(objs):
    locs[b, :len(o)] = o[:K]
    counts[b] = min(len(o), K)
L = torch.from_numpy(locs).cuda()
C = torch.from_numpy(counts).cuda()
ops.render_center_targets(L, C)
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(50):
    ops.render_center_targets(L, C)
e1.record(s)
e1.synchronize()
gpu_ms = e0.elapsed_time(e1) / 50
print("B=%d targets: CPU per-sample renderer %.2f ms (1 thread), GPU %.4f ms" % (B, cpu_ms, gpu_ms))

# tile augmentation (scd_augment_tiles): B=32 512x512 tiles already in HBM, flips + normalize + jitter + device noise
tiles = torch.randn(B, 1, 512, 512, device="cuda") * 30 + 100
flips = torch.randint(0, 2, (B, 2), dtype=torch.uint8, device="cuda")
jit = 1 + 0.05 * torch.randn(B, device="cuda")
out = torch.empty_like(tiles)
ops.augment_tiles(tiles, flips, jit, None, 0.05, 1, out=out)
e0.record(s)
for k in range(50):
    ops.augment_tiles(tiles, flips, jit, None, 0.05, k, out=out)
e1.record(s)
e1.synchronize()
aug_ms = e0.elapsed_time(e1) / 50
nbytes = B * 512 * 512 * 4 * 3   # stats read + apply read + write
print("B=%d augment 512x512: GPU %.4f ms (%.0f GB/s over %d algorithmic bytes)" % (B, aug_ms, nbytes / aug_ms / 1e6, nbytes))
x = tiles[0].cpu()
t0 = time.perf_counter()
for _ in range(20):
    t = torch.flip(x, [2])
    m = torch.mean(t)
    t = (t - m) / torch.sqrt(torch.mean(torch.square(t - m)))
    t = t * (1 + 0.05 * torch.randn(1))
    t = t + torch.randn(1, 512, 512) * 0.05
cpu_aug_ms = (time.perf_counter() - t0) / 20 * 1e3
print("per-sample reference augmentation ops on the host (torch CPU, %d threads): %.2f ms per tile, %.1f ms per batch"
      % (torch.get_num_threads(), cpu_aug_ms, cpu_aug_ms * B))
