"""Code-generation guard for the LDS-DMA GEMM kernels (CPU: hipcc cross-compiles gfx950 here, no GPU needed).

The ring / ping-pong / row-ring / weight-gradient kernels keep two or three DMA stages in flight with counted
`s_waitcnt vmcnt(N)`.  hipcc's wait-count pass silently falls back to a full `vmcnt(0)` drain before the fragment reads
when it cannot prove the DMA'd LDS does not alias what is read -- e.g. when the kernel gains a second `__shared__`
object (round 4: the fused-finalize arrival flag did that and the ring GEMM lost 20-35 % per call with bit-identical
results, so only a timing A/B showed it).  This test compiles conv_gemm.hip to assembly and checks that the MFMA region
of each such kernel has no more full drains than the schedule itself writes.  A second test counts exec-masked branch
regions in the main loops of the stem backward and the BN backward kernels (their round-4 predecessors had 63, 16 and
8; now at most 3).
"""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "scd-resnet_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# kernel-name fragment -> most `s_waitcnt vmcnt(0)` allowed between its first and last MFMA (what the schedules write:
# the NQ = 2 weight-gradient stage hand-off, the layer1 weight gradient's per-stage wait, the row-ring kernel's
# per-tile waits (its loop is the run of tiles: 5 plain, 3 with the BN-backward sums); the heads kernel's range
# includes its epilogue's 1x1 tails).  Keys are regular expressions on the mangled kernel name.
CEILING = {
    r"conv_gemm_ring_kernel": 0,
    r"conv_gemm_pp_kernel": 0,
    r"conv_gemm_l1p_kernelILi\d+ELb[01]ELb0E": 5,
    r"conv_gemm_l1p_kernelILi\d+ELb[01]ELb1E": 3,
    r"conv_wgrad_pp2_kernelILi4": 0,
    r"conv_wgrad_pp2_kernelILi3": 0,
    r"conv_wgrad_pp2_kernelILi2": 1,
    r"conv_wgrad_l1_kernel": 1,
    r"conv_gemm_heads384_kernel": 13,
}


def _kernels(asm):
    out, cur = {}, None
    for line in asm.split("\n"):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and "s_endpgm" in line:
            cur = None
            continue
        if cur:
            out[cur].append(line)
    return out


def _mfma_loop(lines):
    """[start, end) of the loop around the first MFMA (its header label .. the backward branch to it), widened to the
    last MFMA; the MFMA range itself when the first MFMA is in no loop."""
    idx = [i for i, l in enumerate(lines) if "v_mfma" in l]
    if not idx:
        return 0, 0
    lo, hi = idx[0], idx[-1]
    for j in range(idx[0], -1, -1):
        m = re.match(r"^(\.LBB\d+_\d+):", lines[j])
        if not m:
            continue
        back = [k for k in range(idx[0], len(lines)) if re.search(r"s_cbranch\w*\s+" + re.escape(m.group(1)) + r"\b",
                                                                   lines[k])]
        if back:
            lo, hi = j, max(hi, back[-1])
            break
    return lo, hi


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("python3") is None, reason="no hipcc")
def test_lds_dma_main_loops_keep_counted_waits(tmp_path):
    out = tmp_path / "conv_gemm.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                    "-S", os.path.join(CSRC, "conv_gemm.hip"), "-o", str(out)], check=True, capture_output=True,
                   timeout=600)
    kernels = _kernels(out.read_text())
    seen = {k: 0 for k in CEILING}
    for name, lines in kernels.items():
        for frag, ceiling in CEILING.items():
            if not re.search(frag, name):
                continue
            lo, hi = _mfma_loop(lines)
            assert hi > lo, name
            drains = sum("vmcnt(0)" in l for l in lines[lo:hi])
            assert drains <= ceiling, "%s: %d full vmcnt drains in its MFMA loop (at most %d)" % (name, drains,
                                                                                                  ceiling)
            seen[frag] += 1
    assert all(seen.values()), seen


def _loop_span(lines):
    """[start, end) of the longest loop (a label and the last backward branch to it)."""
    labels = {}
    for k, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = k
    best = (0, 0, 0)
    for k, l in enumerate(lines):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)\b", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k and k - labels[m.group(1)] > best[0]:
            best = (k - labels[m.group(1)], labels[m.group(1)], k)
    return best[1], best[2]


# kernel-name regex -> most exec-masked branch regions (`s_and_saveexec`) allowed in its longest loop: the stem
# backward's tile loop and the BN backward elementwise loops were built from per-read / per-element branch regions
# until round 4 (63 per stem tile, 8 per BN vector) -- a runtime condition around an LDS read or a per-element pointer
# test turns into them silently
BRANCH_CEILING = {
    ("stem.hip", r"stem_bwd_fused_kernel"): 4,
    ("bn.hip", r"bn_bwd_apply_kernelIDF16bE"): 4,
    ("bn.hip", r"bn_bwd_reduce_kernelIDF16bE"): 4,
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_inner_loops_have_no_branch_regions(tmp_path):
    asm = {}
    for src in sorted({s for s, _ in BRANCH_CEILING}):
        out = tmp_path / (src + ".s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                        "-I", CSRC, "-I", os.path.join(os.path.dirname(os.path.dirname(CSRC)), "include"),
                        "-S", os.path.join(CSRC, src), "-o", str(out)], check=True, capture_output=True, timeout=600)
        asm[src] = _kernels(out.read_text())
    for (src, frag), ceiling in BRANCH_CEILING.items():
        names = [n for n in asm[src] if re.search(frag, n)]
        assert names, frag
        for name in names:
            lines = asm[src][name]
            lo, hi = _loop_span(lines)
            assert hi > lo, name
            regions = sum("s_and_saveexec" in l for l in lines[lo:hi])
            assert regions <= ceiling, "%s: %d exec-masked branch regions in its main loop (at most %d)" % (
                name, regions, ceiling)
