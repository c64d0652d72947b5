"""Whole-slide tiled inference (scd_slide_tiles, scd_slide_detections, slide.analyseArray,
the inference Wrapper) against the reference's test.py.analyseImages run on the same synthetic slide and the
same decoded outputs (tests/golden/slide.npz, tests/golden/make_golden_slide.py).

Tolerances: clips are float64-normalised integers cast to float32 on both sides; the fp64 sums differ only in
summation order, so values agree to one float32 ulp (atol 1e-6 on |v| < 8).  Detections: pixel coordinates
exact, ratios 1e-12 relative."""
import numpy as np
import pytest
import torch

from oracle import slide_case

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def clips_and_geom():
    import slide
    return slide.tiles(slide_case.slide())


def test_geometry():
    import slide
    g = slide.geometry(slide_case.SLIDE_H, slide_case.SLIDE_W)
    assert (g["clipH"], g["clipV"], g["resizeW"], g["resizeH"], g["padLR"], g["padTB"]) == (8, 6, 3200, 2432, 54, 188)


def test_slide_tiles_vs_reference(clips_and_geom, golden):
    gold = golden("slide")
    clips, _ = clips_and_geom
    c = clips[:, 0].cpu().numpy()
    assert c.shape == (48, 512, 512)
    np.testing.assert_allclose(c[:, ::8, ::8], gold["clip_sub"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(c[0, :64, :64], gold["win_first"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(c[-1, 448:, 448:], gold["win_last"], rtol=0, atol=1e-6)
    c64 = c.astype(np.float64)
    np.testing.assert_allclose(c64.sum((1, 2)), gold["clip_stats"][:, 0], rtol=0, atol=2e-2)
    np.testing.assert_allclose((c64 ** 2).sum((1, 2)), gold["clip_stats"][:, 1], rtol=1e-6)


def test_slide_detections_vs_reference(clips_and_geom, golden):
    from scdhip import ops
    gold = golden("slide")
    _, g = clips_and_geom
    xy, ratio = ops.slide_detections(torch.from_numpy(gold["decoded"]).to(DEV), 384, g["padLR"], g["padTB"],
                                     g["clipV"], 0.3)
    det = gold["detections"]
    assert xy.shape[0] == det.shape[0]
    np.testing.assert_array_equal(xy.cpu().numpy(), det[:, :2].astype(np.int64))
    np.testing.assert_allclose(ratio.cpu().numpy(), det[:, 2], rtol=1e-12)


def test_analyse_array_end_to_end(golden):
    """The whole reference loop (batches of 24, threshold, projection) with a model answering the recorded
    decoded stack; the clips it is fed are checked too."""
    import slide
    gold = golden("slide")
    dec = torch.from_numpy(gold["decoded"]).to(DEV)
    state = {"at": 0, "shapes": []}

    def model(inp):
        state["shapes"].append(tuple(inp.shape))
        b = inp.shape[0]
        out = dec[:, state["at"]:state["at"] + b]
        state["at"] += b
        return out

    det = slide.analyseArray(model, slide_case.slide())
    assert state["shapes"] == [(24, 1, 512, 512), (24, 1, 512, 512)]
    ref = gold["detections"]
    assert len(det) == len(ref)
    got = np.array(det, np.float64)
    np.testing.assert_array_equal(got[:, :2], ref[:, :2])
    np.testing.assert_allclose(got[:, 2], ref[:, 2], rtol=1e-12)


def test_wrapper_stack_from_model():
    """Wrapper over a real (tiny) plugin model: rows = decode outputs in the reference's order."""
    import trainer.model.centerOffsetRes10 as plugin
    from trainer.wrappers.centerOffsetResidual import Wrapper
    torch.manual_seed(0)
    m = plugin.model(**plugin.modelParams).to(DEV).train()
    x = torch.randn(2, 1, 256, 256, device=DEV)
    with torch.no_grad():
        st = Wrapper(m)(x)
        scores, inds, ys, xs, off, regr, _ = m(x, decode=True)
    assert st.shape == (10, 2, 100) and st.dtype == torch.float32
    for r, v in zip(st, [scores, inds, ys, xs, regr[:, :, 0], regr[:, :, 1], regr[:, :, 2], regr[:, :, 3],
                         off[:, :, 0], off[:, :, 1]]):
        torch.testing.assert_close(r, v.float(), rtol=0, atol=0)


def test_slide_small_image_no_fixup():
    """A slide narrower than 3072 px has no column fix-up in range (the reference would index past its width);
    clips are the reflect-padded, per-clip normalised grey image."""
    import slide
    rs = np.random.RandomState(3)
    img = rs.randint(0, 256, (700, 900, 3)).astype(np.uint8)
    clips, g = slide.tiles(img)
    grey = np.round(0.1140 * img[:, :, 0] + 0.5870 * img[:, :, 1] + 0.2989 * img[:, :, 2])
    pad = np.pad(grey, ((g["padTB"], g["padTB"]), (g["padLR"], g["padLR"])), mode="reflect")
    k = 0
    for i in range(g["clipH"]):
        for j in range(g["clipV"]):
            t = pad[j * 384:j * 384 + 512, i * 384:i * 384 + 512]
            t = ((t - t.mean()) / np.sqrt(((t - t.mean()) ** 2).mean())).astype(np.float32)
            np.testing.assert_allclose(clips[k, 0].cpu().numpy(), t, rtol=0, atol=1e-6)
            k += 1
