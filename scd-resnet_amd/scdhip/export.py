"""TorchScript export and import of the inference Wrapper (trace.py:35-66 and test.py:145 of the reference).

The reference traces Wrapper(model) with torch.jit.trace into a `.pt` whose graph is ATen convolutions, and
test.py runs it with torch.jit.load.  Here the network runs on libscdhip through ctypes, which a tracer cannot see,
so the whole decoded forward is one dispatcher op, ``scd::centernet_decode(x, tensors, arch, mode, dtype) -> (10,B,K)``
registered below (a CUDA kernel implemented in Python over the plugin model): ``trace`` records that op with the
model's parameters and buffers as module attributes, so the saved `.pt` carries the weights and replays the HIP
path after ``torch.jit.load`` in any process that has imported this module (``load``).  ``load`` also accepts a
`.pt` written by the reference's trace.py (an ATen graph): its parameters are taken by name (the `model.` /
`model.module.` prefixes of Wrapper / DataParallel) into the plugin model, which then runs on libscdhip.
"""
import importlib
import json

import torch

_LIB = torch.library.Library("scd", "DEF")
_LIB.define("centernet_decode(Tensor x, Tensor[] tensors, str arch, str mode, str dtype) -> Tensor")

_MODELS = {}        # (arch, mode, dtype, device) -> (Wrapper, tensor list it was bound to)
_DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def _plugin_model(arch):
    plugin = importlib.import_module("trainer.model." + arch)
    return plugin.model(**plugin.modelParams)


def _wrapper_for(arch, mode, dtype, device):
    wrappers = importlib.import_module("trainer.wrappers.centerOffsetResidual")
    key = (arch, mode, dtype, str(device))
    hit = _MODELS.get(key)
    if hit is None:
        m = _plugin_model(arch).to(device)
        m.set_compute_dtype(_DTYPES[dtype])
        m.train(mode == "train")
        hit = [wrappers.Wrapper(m), None]
        _MODELS[key] = hit
    return hit


def _decode_impl(x, tensors, arch, mode, dtype):
    hit = _wrapper_for(arch, mode, dtype, x.device)
    w = hit[0]
    ptrs = tuple(t.data_ptr() for t in tensors)
    if hit[1] != ptrs:
        # bind the module's parameters and buffers to the op's tensors (views, no copy)
        own = list(w.model.parameters()) + list(w.model.buffers())
        if len(own) != len(tensors):
            raise RuntimeError("scd::centernet_decode: %d tensors for a %s model with %d" % (len(tensors), arch,
                                                                                          len(own)))
        for o, t in zip(own, tensors):
            if o.shape != t.shape:
                raise RuntimeError("scd::centernet_decode: tensor shape %s for %s" % (tuple(t.shape), tuple(o.shape)))
            o.data = t.to(device=x.device, dtype=o.dtype)
        hit[1] = ptrs
    with torch.no_grad():
        return w(x)


_LIB.impl("centernet_decode", _decode_impl, "CUDA")


class Traceable(torch.nn.Module):
    """Wrapper(model) as one scd::centernet_decode call over the model's parameters and buffers."""

    def __init__(self, arch, model, mode="train", dtype="bf16"):
        super().__init__()
        self.model = model
        self.arch, self.mode, self.dtype = arch, mode, dtype

    def forward(self, inp):
        tensors = list(self.model.parameters()) + list(self.model.buffers())
        return torch.ops.scd.centernet_decode(inp, tensors, self.arch, self.mode, self.dtype)


@torch.no_grad()
def trace(arch, model, example, path, mode="train", dtype="bf16"):
    """torch.jit.trace of the decoded forward (trace.py:58-66); writes `path`, returns the traced module.  `mode`:
    "train" keeps BatchNorm on batch statistics, as the reference's trace of an un-eval'ed model does; "eval"
    uses the running statistics."""
    t = Traceable(arch, model, mode, dtype).to(example.device)
    traced = torch.jit.trace(t, example, check_trace=False)
    traced.save(path)
    meta = {"arch": arch, "mode": mode, "dtype": dtype}
    with open(path + ".json", "w") as f:
        json.dump(meta, f)
    return traced


def load(path, arch=None, device=None, mode="train", dtype="bf16"):
    """A traced `.pt` as a callable (10,B,K) decoder on the HIP path: one written by ``trace`` replays as saved; one
    written by the reference's trace.py (ATen graph) has its parameters loaded into `arch`'s plugin model."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    mod = torch.jit.load(path, map_location=device)
    if any(n.kind() == "scd::centernet_decode" for n in mod.inlined_graph.nodes()):
        return mod
    if arch is None:
        raise RuntimeError("%s is an ATen trace (reference trace.py): name its architecture" % path)
    sd = {}
    for k, v in mod.state_dict().items():
        for pre in ("model.module.", "model."):
            if k.startswith(pre):
                sd[k[len(pre):]] = v
                break
    m = _plugin_model(arch)
    m.load_state_dict(sd)
    m = m.to(device).set_compute_dtype(_DTYPES[dtype])
    m.train(mode == "train")
    wrappers = importlib.import_module("trainer.wrappers.centerOffsetResidual")
    return wrappers.Wrapper(m)
