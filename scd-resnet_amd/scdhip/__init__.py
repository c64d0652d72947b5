"""scdhip -- MI355X (gfx950) kernels for the scd-resnet training hot path.

lib     ctypes binding of libscdhip.so (C-ABI: include/scdhip.h)
ops     tensor-level wrappers (NHWC activations, torch-owned memory and streams)
blocks  block-granular autograd Functions (stem, BasicBlock, Bottleneck, deconv, heads, corner pool)
loss    fused focal + masked-L1 loss Functions
flat    flat parameter/gradient buffers, FlatAdam (torch.optim.Adam semantics), FlatDDP (RCCL)
"""
from . import lib  # noqa: F401
