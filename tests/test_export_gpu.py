"""TorchScript export / import of the inference Wrapper (trace.py:35-66, test.py:145 of the reference;
scdhip/export.py): a `.pt` written by trace replays the libscdhip decode bit for bit after torch.jit.load (the
weights travel inside the archive, BN in train or eval mode as traced), and a `.pt` that holds an ATen trace with
the reference's `model.` / `model.module.` parameter names loads into the plugin model and gives the same output.
(Same kernels, same weights; BN batch statistics come from fp64 atomics, so equal up to summation order: scores
1e-4, decoded indices / coordinates equal at >= 98% of the slots -- near-tied scores may swap.)"""


def _same(got, want):
    assert got.shape == want.shape
    assert torch.allclose(got[0], want[0], rtol=1e-4, atol=1e-6)
    assert (got[1:4] == want[1:4]).float().mean().item() >= 0.98
import pytest
import torch

from oracle import centernet as O
from oracle import targets as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(name="centerOffsetRes10"):
    import importlib
    plugin = importlib.import_module("trainer.model." + name)
    entries, _ = O.model_spec(plugin.modelParams["numLayers"], plugin.modelParams["dims"])
    m = plugin.model(**plugin.modelParams)
    m.load_state_dict(O.hash_weights(entries))
    return m


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_trace_roundtrip_replays_hip_decode(tmp_path, mode):
    from scdhip import export
    from trainer.wrappers.centerOffsetResidual import Wrapper
    x = T.batch_inputs(5, 2, 512).to(DEV)
    m = _model().to(DEV)
    path = str(tmp_path / "res10.pt")
    export.trace("centerOffsetRes10", m, x, path, mode=mode)
    direct = Wrapper(_model().to(DEV).train(mode == "train"))
    with torch.no_grad():
        want = direct(x)
    loaded = export.load(path)
    assert isinstance(loaded, torch.jit.ScriptModule)
    got = loaded(x)
    assert got.shape == (10, 2, 100)
    _same(got, want)


def test_reference_style_aten_trace_loads_into_plugin(tmp_path):
    """An ATen-graph `.pt` whose parameters carry the reference's Wrapper / DataParallel names."""
    from scdhip import export
    from trainer.wrappers.centerOffsetResidual import Wrapper

    class DP(torch.nn.Module):                 # DataParallel's parameter naming (module.<...>)
        def __init__(self, m):
            super().__init__()
            self.module = m

    class RefLike(torch.nn.Module):            # trace.py's Wrapper(model) naming; any ATen forward
        def __init__(self, m):
            super().__init__()
            self.model = DP(m)

        def forward(self, x):
            return x * 2.0

    path = str(tmp_path / "ref.pt")
    torch.jit.trace(RefLike(_model()), torch.rand(1, 1, 8, 8)).save(path)
    dec = export.load(path, arch="centerOffsetRes10", device=torch.device(DEV))
    x = T.batch_inputs(6, 2, 512).to(DEV)
    with torch.no_grad():
        got = dec(x)
        want = Wrapper(_model().to(DEV).train())(x)
    _same(got, want)
