"""Golden fixture for whole-slide tiled inference, from the REAL reference (build container only).

Run:  python tests/golden/make_golden_slide.py      (needs /root/reference; never runs on the GPU box)

Imports the reference's test.py (its module body calls torch.jit.load('xxx.pt') for a checkpoint that does not
exist: torch.jit.load is stubbed for the import only, nothing of the reference is changed) and runs its
analyseImages(model, path) on oracle.slide_case.slide() saved as PNG, with `model` a recorder that keeps every
clip batch the reference feeds it and answers with the seeded (10, b, K) stack of oracle.slide_case.decoded.
Writes tests/golden/slide.npz:
  clip_sub      (T, 64, 64) every clip subsampled [::8, ::8]
  clip_stats    (T, 2) float64 sum / sum of squares of each float32 clip
  win_first     (64, 64) clip 0 rows 0..63, cols 0..63 (left fix-up + top padding)
  win_last      (64, 64) last clip rows 448..511, cols 448..511 (right fix-up + bottom padding)
  decoded       (10, T, K) what the recorder returned
  detections    (n, 3) float64 [x, y, ratio]
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
WORK = "/tmp/slide_golden"

sys.dont_write_bytecode = True
for _n in ["torchvision", "torchvision.transforms", "torchvision.transforms.functional"]:
    sys.modules[_n] = types.ModuleType(_n)
sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
sys.path.insert(0, REF)
sys.path.insert(1, REPO)

import torch  # noqa: E402
import torch.jit  # noqa: E402
from PIL import Image  # noqa: E402

from oracle import slide_case  # noqa: E402


class _Dummy:
    def eval(self):
        return self


_load = torch.jit.load
torch.jit.load = lambda *a, **k: _Dummy()
try:
    import test as ref_test  # noqa: E402  (reference test.py)
finally:
    torch.jit.load = _load


def main():
    os.makedirs(WORK, exist_ok=True)
    img = slide_case.slide()
    path = os.path.join(WORK, "slide.png")
    Image.fromarray(img).save(path)
    clips = []
    T = 48
    dec = torch.from_numpy(slide_case.decoded(T))
    state = {"at": 0}

    def recorder(inp):
        clips.append(inp.clone())
        b = inp.shape[0]
        out = dec[:, state["at"]:state["at"] + b]
        state["at"] += b
        return out

    det = ref_test.analyseImages(recorder, path)
    allc = torch.cat(clips).numpy().astype(np.float32)[:, 0]
    assert allc.shape[0] == T, allc.shape
    out = {
        "clip_sub": allc[:, ::8, ::8].copy(),
        "clip_stats": np.stack([allc.astype(np.float64).sum((1, 2)), (allc.astype(np.float64) ** 2).sum((1, 2))], 1),
        "win_first": allc[0, :64, :64].copy(),
        "win_last": allc[-1, 448:, 448:].copy(),
        "decoded": dec.numpy(),
        "detections": np.array(det, np.float64).reshape(-1, 3),
    }
    np.savez_compressed(os.path.join(HERE, "slide.npz"), **out)
    print("clips", allc.shape, "detections", out["detections"].shape, "batches", [c.shape[0] for c in clips])


if __name__ == "__main__":
    main()
