"""CPU oracle for the scd-resnet training hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain PyTorch-fp32-on-CPU restatement of the reference
(yang-z-03/scd-resnet @ 2024-10-22) algorithm for the CenterNet/CornerNet
training step: ResNet backbone, transposed-conv upsampler, heads, focal + L1
loss, NMS/top-K decode, corner pooling, Adam.  Every function cites the
reference file:line it restates.

Rules (see DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this package, and only as the checker /
    the reported CPU baseline.  The product (``scd-resnet_amd/``) never
    imports it and fails loudly when its HIP library is missing.
  * The oracle is pinned against golden vectors produced by running the real
    reference in the build container (``tests/golden/make_golden.py``); the
    CPU test-suite re-checks it against those fixtures on every run.
"""
