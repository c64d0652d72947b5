"""Whole-slide tiled inference (test.py:13-135 of the reference) on MI355X.

analyseImages(model, path) keeps the reference's signature and output: a list of [x, y, ratio] detections in
slide pixels.  `model` is the inference Wrapper (trainer/wrappers/centerOffsetResidual.py) around a model plugin,
i.e. anything returning the (10, B, K) decoded stack -- the reference passes the TorchScript trace of the same
wrapper (trace.py:62-66).  Geometry is the reference's: 512-px clips on a 384-px stride with 64-px margins, the
slide resized to whole strides by torch-'reflect' padding plus its opencv column fix-up, batches of 24 clips.
Clip extraction + greyscale + normalisation run as scd_slide_tiles (nothing padded is materialised), the score
threshold and the projection back to slide pixels as scd_slide_detections; the slide goes to the device once.

CLI:  python slide.py <architecture> <state_dict.pt | traced.pt> <image> [<image> ...]   (-eval: BN in eval mode)
"""
import sys
from math import ceil

import numpy as np
import torch

INPUTSIZE = 512
PADDINGSIZE = 64
DOWNSAMPLERATIO = 4
BATCHSIZE = 24
THRESHOLD = 0.3


def geometry(height, width):
    """test.py:41-54: clip counts, padded size and the symmetric padding."""
    step = INPUTSIZE - 2 * PADDINGSIZE
    clipHorizontal = ceil((width - 2 * PADDINGSIZE) / step)
    clipVertical = ceil((height - 2 * PADDINGSIZE) / step)
    resizeW = step * clipHorizontal + 2 * PADDINGSIZE
    resizeH = step * clipVertical + 2 * PADDINGSIZE
    if (resizeW - width) % 2 != 0:
        resizeW += 1
    if (resizeH - height) % 2 != 0:
        resizeH += 1
    return dict(clipH=clipHorizontal, clipV=clipVertical, resizeW=resizeW, resizeH=resizeH,
                padLR=(resizeW - width) // 2, padTB=(resizeH - height) // 2)


@torch.no_grad()
def tiles(rgb, device=None):
    """RGB (H,W,C) uint8 (numpy or tensor) -> ((T,1,512,512) normalised clips on the device, geometry)."""
    from scdhip import ops
    if not torch.is_tensor(rgb):
        rgb = torch.from_numpy(np.ascontiguousarray(rgb))
    dev = device or torch.device("cuda", torch.cuda.current_device())
    rgb = rgb.to(dev)
    H, W = rgb.shape[:2]
    g = geometry(H, W)
    # the reference's fix-up (test.py:79-82) indexes padded columns 0..63 and 3136..3199
    clips = ops.slide_tiles(rgb, INPUTSIZE, INPUTSIZE - 2 * PADDINGSIZE, g["clipH"], g["clipV"], g["padLR"],
                            g["padTB"], fix=g["resizeW"] >= 3200)
    return clips, g


@torch.no_grad()
def analyseArray(model, rgb, batch=BATCHSIZE):
    from scdhip import ops
    clips, g = tiles(rgb)
    decoded = [model(clips[i:i + batch]) for i in range(0, clips.shape[0], batch)]
    dec = torch.cat(decoded, 1)
    xy, ratio = ops.slide_detections(dec, INPUTSIZE - 2 * PADDINGSIZE, g["padLR"], g["padTB"], g["clipV"], THRESHOLD)
    xy, ratio = xy.cpu().tolist(), ratio.cpu().tolist()
    return [[p[0], p[1], r] for p, r in zip(xy, ratio)]


def analyseImages(model, fullPath):
    """test.py:38-135."""
    from PIL import Image
    return analyseArray(model, np.array(Image.open(fullPath)))


def main(argv):
    import importlib
    evalMode = "-eval" in argv
    argv = [a for a in argv if a != "-eval"]
    if len(argv) < 3:
        print(__doc__)
        return 2
    arch, ckpt, images = argv[0], argv[1], argv[2:]
    import zipfile
    if zipfile.is_zipfile(ckpt) and any(n.endswith("constants.pkl") for n in zipfile.ZipFile(ckpt).namelist()):
        # a TorchScript archive (test.py:145 loads the trace.py output): ours replays scd::centernet_decode, a
        # reference trace has its weights moved into the plugin model (scdhip/export.py)
        from scdhip import export
        wrapper = export.load(ckpt, arch=arch, mode="eval" if evalMode else "train")
    else:
        plugin = importlib.import_module("trainer.model." + arch)
        model = plugin.model(**plugin.modelParams)
        model.load_state_dict(torch.load(ckpt, map_location="cpu", weights_only=True))
        model = model.cuda()
        model.train(not evalMode)
        wrapper = importlib.import_module("trainer.wrappers.centerOffsetResidual").Wrapper(model)
    for img in images:
        for d in analyseImages(wrapper, img):
            print("%s\t%d\t%d\t%.6f" % (img, d[0], d[1], d[2]))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
