"""Build the reference's corner-pooling C++ ops (models/backbones/cornerPooling/source/*.cpp) from their
own sources into oracle/_ref/ (TEST INFRASTRUCTURE ONLY; build container only).

The sources only need libtorch + pybind11 (both ship with the installed torch), so they compile
as-is with torch.utils.cpp_extension; nothing is copied or stubbed.  Only the CPU forward is
usable here: the reference backward allocates torch::CUDA tensors (topPool.cpp:44-45).
"""
import os
import sys

from torch.utils.cpp_extension import load

REF = "/root/reference/models/backbones/cornerPooling/source"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref")


def build(verbose=False):
    os.makedirs(OUT, exist_ok=True)
    mods = {}
    for name in ("topPool", "bottomPool", "leftPool", "rightPool"):
        bdir = os.path.join(OUT, name)
        os.makedirs(bdir, exist_ok=True)
        mods[name] = load(name=name, sources=[os.path.join(REF, name + ".cpp")], build_directory=bdir,
                          verbose=verbose, extra_cflags=["-O2"])
    return mods


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference sources not present")
    build(verbose=True)
    print("built into", OUT)
