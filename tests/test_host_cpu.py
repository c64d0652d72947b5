"""CPU tests of the product's host side: C-ABI library surface, plugin/state_dict interchange,
reference initialisation, synthetic data vs the oracle's restatement, config/CLI semantics,
the no-CPU-fallback rule, and the data-parallel wrapper's logic (gloo, world size 2)."""
import os
import re
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import centernet as O
from oracle import targets as T

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "scdhip.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(scd_\w+)\(", src, re.M)))


def test_lib_loads_and_exports_every_header_symbol():
    import scdhip.lib as L
    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib.dll, s)]
    assert not missing, missing
    assert sorted(L.SIGNATURES) == syms, "ctypes signatures out of sync with include/scdhip.h"
    assert lib.dll.scd_version().startswith(b"libscdhip")


def test_gemm_phase_struct_matches_header():
    import ctypes

    import scdhip.lib as L
    m = re.search(r"#define SCD_MAX_TAPS (\d+)", open(HEADER).read())
    assert int(m.group(1)) == L.MAX_TAPS
    assert ctypes.sizeof(L.GemmPhase) == 4 * (5 + 3 * L.MAX_TAPS)


@pytest.mark.parametrize("struct,cname", [("BnFinArgs", "scd_bn_fin_args"), ("BnBwdFinArgs", "scd_bn_bwd_fin_args")])
def test_bn_finalize_n_structs_match_header(tmp_path, struct, cname):
    """The ctypes mirrors of the scd_bn_finalize_n / scd_bn_bwd_finalize_n layer descriptors have the C layout of
    include/scdhip.h: size and every field offset from a C program compiled against the header with gcc."""
    import ctypes

    import scdhip.lib as L
    S = getattr(L, struct)
    names = [f[0] for f in S._fields_]
    src = tmp_path / "s.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "scdhip.h"\nint main(void){printf("%zu",'
                   ' sizeof(' + cname + '));' + "".join('printf(" %%zu", offsetof(%s, %s));' % (cname, n) for n in names)
                   + "return 0;}\n")
    exe = tmp_path / "s"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(S)
    assert vals[1:] == [getattr(S, n).offset for n in names]
    m = re.search(r"#define SCD_BN_FIN_MAX (\d+)", open(HEADER).read())
    assert m and int(m.group(1)) >= 2


def test_workspace_queries():
    import scdhip.lib as L
    assert L.lib().scd_conv_wgrad_workspace(128, 9, 64, 4) == 4 * 128 * 9 * 64 * 4
    assert L.lib().scd_decode_workspace(2, 16384) == 2 * 16384 * 4
    od = L.int_array([1, 4, 2])
    assert L.lib().scd_heads_bwd_accsize(3, 128, od) == L.STAT_REPLICAS * (7 * 128 + 7 + 384) * 8


@pytest.mark.parametrize("name", ["centerOffsetRes10", "centerOffsetRes18", "centerOffsetRes50",
                                  "centerOffsetRes10h"])
def test_plugin_state_dict_matches_reference_layout(name):
    import importlib
    plugin = importlib.import_module("trainer.model." + name)
    for attr in ("model", "loss", "modelParams", "evaluation", "expression"):
        assert hasattr(plugin, attr)
    m = plugin.model(**plugin.modelParams)
    entries, _ = O.model_spec(plugin.modelParams["numLayers"], plugin.modelParams["dims"],
                              head_dim=m.HEAD_DIM)
    sd = m.state_dict()
    assert list(sd.keys()) == [k for k, _ in entries]
    assert all(tuple(sd[k].shape) == tuple(s) for k, s in entries)


def test_reference_initialisation_reproduced(golden):
    """F0: the plugin under the reference's import-order seed draws the reference's weights."""
    import trainer.model.centerOffsetRes10 as plugin
    g = golden("init")
    torch.random.manual_seed(42)
    m = plugin.model(**plugin.modelParams)
    assert sum(p.numel() for p in m.parameters()) == int(g["param_count"])
    for k, v in m.state_dict().items():
        v = v.double()
        np.testing.assert_allclose(v.sum().item(), float(g[k + "|sum"]), rtol=1e-6, atol=1e-6, err_msg=k)
        np.testing.assert_allclose((v * v).sum().item(), float(g[k + "|sumsq"]), rtol=1e-6, atol=1e-9, err_msg=k)
        np.testing.assert_array_equal(v.reshape(-1)[:4].float().numpy(), g[k + "|head"])


def test_synthetic_dataset_matches_oracle_rendering():
    from trainer.dataset.syntheticSCD import SCD, encode_targets, sample_objects
    rs1, rs2 = np.random.RandomState(5), np.random.RandomState(5)
    for _ in range(20):
        locs = sample_objects(rs1)
        ref_locs = T.random_locs(rs2)
        np.testing.assert_array_equal(locs, ref_locs)
        got = encode_targets(locs)
        ref = T.render(ref_locs)
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)
    ds = SCD(None, True)
    item = ds[3]
    assert item["xs"][0].shape == (1, 512, 512) and item["xs"][0].dtype == torch.float32
    heat, mask, regr, inds = item["ys"]
    assert heat.shape == (1, 128, 128) and mask.dtype == torch.bool and regr.shape == (30, 6)
    assert inds.dtype == torch.int64 and int(inds.max()) < 128 * 128
    assert float(heat.max()) == 1.0                      # every centre is an exact positive
    vs = ds.getValidationSet(batch=32)
    assert len(vs) == 2 and vs[0]["ys"][3].shape == (32, 30, 8)


def test_cornernet_plugin_layout_and_dataset():
    """config 4: the cornerNetCPool plugin's state_dict matches the reference module tree (oracle
    spec, checked against the reference in F8) and the corner dataset renders the oracle's rule."""
    import trainer.model.cornerNetCPool as plugin
    from oracle import cornernet as OC
    from trainer.dataset.syntheticCorner import corner_locs
    from trainer.dataset.syntheticSCD import encode_targets, sample_objects
    for attr in ("model", "loss", "modelParams", "evaluation", "expression"):
        assert hasattr(plugin, attr)
    sd = plugin.model(**plugin.modelParams).state_dict()
    entries, _ = OC.model_spec(10)
    assert list(sd.keys()) == [k for k, _ in entries]
    assert all(tuple(sd[k].shape) == tuple(s) for k, s in entries)
    got = []
    rs = np.random.RandomState(32)
    for _ in range(2):
        locs = sample_objects(rs, 32)
        tl, br = corner_locs(locs, 32)
        got.append((encode_targets(tl, 32)[0], encode_targets(br, 32)[0]))
    ref = T.corner_targets(32, 2, 32)
    for b in range(2):
        np.testing.assert_array_equal(got[b][0], ref[3][b].numpy())
        np.testing.assert_array_equal(got[b][1], ref[4][b].numpy())


def test_configuration_overlay_and_format():
    from configuration import Configuration
    c = Configuration()
    c.updateConfig({"modelName": "centerOffsetRes10", "datasetName": "syntheticSCD", "trainName": "t",
                    "notAKey": 1, "batchSize": 4})
    assert "notAKey" not in c.config
    assert c.batchSize == 4
    assert c.dirModel == "trainer.model.centerOffsetRes10"
    assert c.dirData == "trainer.dataset.syntheticSCD"
    assert c.naming == "centerOffsetRes10.t.0.pth"
    assert c.useGPU  # bound method, always truthy (reference quirk, configuration.py:147-148)


def test_train_cli_accepts_both_local_rank_spellings():
    import train
    assert train.parseArguments(["cfg.json", "-gpu", "--local_rank", "3"]).localRank == 3
    a = train.parseArguments(["cfg.json", "--local-rank", "2"])
    assert a.localRank == 2 and a.useGPU is False


def test_no_cpu_fallback():
    import trainer.model.centerOffsetRes10 as plugin
    m = plugin.model(**plugin.modelParams)
    with pytest.raises(RuntimeError, match="MI355X"):
        m(torch.zeros(1, 1, 64, 64), decode=False)
    from models.networkFactory import NetworkFactory
    with pytest.raises(RuntimeError, match="MI355X"):
        NetworkFactory(False)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_flat_ddp_gloo_world2():
    """FlatDDP semantics with 2 gloo ranks on CPU: initial broadcast, averaged gradients equal to
    the full-batch gradient, buffer broadcast, `module.` state_dict prefix."""
    worker = os.path.join(REPO, "tests", "ddp_cpu_worker.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2",
               PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "scd-resnet_amd")]))
    procs = [subprocess.Popen([sys.executable, worker], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(2)]
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=240)
        outs.append(out.decode())
        assert p.returncode == 0, out.decode()
    assert all("OK" in o for o in outs), outs


def test_bench_launches_n_ranks_itself():
    """`python bench.py --gpus 2` without a torch.distributed launcher starts 2 rank processes itself
    (rendezvous over 127.0.0.1); rank 0's line reports n_gpus 2 and the all-reduce saw both ranks."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SCD_BENCH_PROBE"] = "1"
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=240)
    text = out.stdout.decode()
    assert out.returncode == 0, text
    lines = [json.loads(ln) for ln in text.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, text
    assert lines[0]["n_gpus"] == 2 and lines[0]["world_seen"] == 2


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", SCD_BENCH_PROBE="1")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=240)
    assert out.returncode != 0 and b"WORLD_SIZE" in out.stdout


def test_resume_schedule_pops_past_milestones():
    """resuming past a milestone keeps the later decays (the reference skips them)."""
    from models.networkFactory import resumeSchedule
    decay, rates = [100, 200, 300], [10.0, 2.0, 5.0]
    lr = resumeSchedule(1e-2, decay, rates, 150)
    assert lr == 1e-3 and decay == [200, 300] and rates == [2.0, 5.0]
    lr = resumeSchedule(1e-2, [100, 200], [10.0, 2.0], 200)      # milestone == resume point is applied
    assert abs(lr - 5e-4) < 1e-15
    d2, r2 = [100], [10.0]
    assert resumeSchedule(1e-2, d2, r2, 99) == 1e-2 and d2 == [100]
    # the loop's own rule then fires at the next milestone
    it, lr = 150, 1e-3
    while it < 300:
        it += 1
        if decay and it == decay[0]:
            lr /= rates.pop(0)
            decay.pop(0)
    assert abs(lr - 1e-4) < 1e-15


def test_flat_ddp_buckets_keep_a_small_tail():
    """FlatDDP buckets (reverse parameter order, ~25 MB) tile the flat gradient exactly, and the last bucket -- complete
    only when the backward ends, so never overlapped with it -- holds at most tail_mb of parameters (Res10: layer2,
    layer1 and the stem), the rest of what would have been that bucket launching as soon as layer3 is done."""
    import trainer.model.centerOffsetRes10 as plugin
    from scdhip import flat as F

    class Buckets(F.FlatDDP):
        def __init__(self, module, bucket_mb=25.0, tail_mb=2.0):
            torch.nn.Module.__init__(self)
            self.module = module
            self.flat = F.ensure_flat(module.parameters())
            self.bucket_elems = int(bucket_mb * (1 << 20) / 4)
            self.tail_elems = int(tail_mb * (1 << 20) / 4)
            self._build_buckets()

    m = plugin.model(**plugin.modelParams)
    d = Buckets(m)
    spans = sorted(d._buckets)
    assert spans[0][0] == 0 and spans[-1][1] == d.flat.data.numel()
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert sum(len(ms) for ms in d._bucket_params) == len(d.flat.params)
    lo, hi = d._buckets[-1]
    assert (hi - lo) * 4 <= 2 << 20
    names = {id(p): n for n, p in m.named_parameters()}
    assert names[d._bucket_params[-1][-1]].startswith("preprocess")
    assert len(d._buckets) >= 3


def test_mean_backward_matches_mean_then_backward():
    """scdhip.loss.mean_backward (the step's loss.mean(); loss.backward() without ATen launches for a one-element
    loss) gives the same value and gradients as the reference's two calls, for one- and many-element losses."""
    from scdhip.loss import mean_backward
    for shape in ((1,), (3,)):
        w1 = torch.arange(1.0, 7.0, requires_grad=True)
        w2 = w1.detach().clone().requires_grad_(True)
        l1 = (w1.reshape(3, 2).sum(1) ** 2)[:shape[0]]
        l2 = (w2.reshape(3, 2).sum(1) ** 2)[:shape[0]]
        m1 = mean_backward(l1)
        m2 = l2.mean()
        m2.backward()
        assert m1.shape == m2.shape == ()
        assert torch.equal(m1.detach(), m2.detach()) and torch.equal(w1.grad, w2.grad)


def test_sgd_step_dev_checks_hyper():
    """scd_sgd_step_dev reads and writes hyper[0..3]: a shorter or non-fp64 hyper is refused on the host before any
    launch (ADVICE r4 ops.py:1441)."""
    import torch
    from scdhip import ops
    p = torch.zeros(8)
    for hyper in (torch.zeros(2, dtype=torch.float64), torch.zeros(4, dtype=torch.float32)):
        with pytest.raises(RuntimeError, match="hyper"):
            ops.sgd_step_dev(p, p, p, hyper, 0.9, 0.0, 0.0, False)


def test_no_type_macros_in_the_f16_build():
    """VERDICT r5 hygiene: the fp16 build names its 16-bit type through the h16 typedef and mfma_16x16x32_h16, not by
    macro-redefining the compiler type __bf16 or an MFMA builtin (code that needs a real bf16 inside an fp16
    translation unit would silently become fp16)."""
    import re
    src = open(os.path.join(REPO, "scd-resnet_amd", "csrc", "scd_common.h")).read()
    assert not re.search(r"#\s*define\s+__bf16\b", src)
    assert not re.search(r"#\s*define\s+__builtin_amdgcn_mfma", src)
    assert "typedef _Float16 h16;" in src and "typedef __bf16 h16;" in src


def test_profile_kernel_names():
    """tools/prof_summary.short: the names the kernel summaries, PMC summaries and bench.py's traffic lookups key on
    (bench.py reads `conv_gemm_pp_kernel<bf16,256,256>` for the CornerPool lastConv and `heads384` for the heads)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from prof_summary import short
    cases = {
        "void (anonymous namespace)::conv_gemm_pp_kernel<256, false, false>((anonymous namespace)::GemmParams)":
            "conv_gemm_pp_kernel<bf16,256,256>",
        "void conv_gemm_pp_kernel<256, false, true>": "conv_gemm_pp_kernel<bf16,256,256,bnbwd>",
        "void (anonymous namespace)::f16::conv_gemm_pp_kernel<192, true, false>(GemmParams)":
            "conv_gemm_pp_kernel<f16,256,192,heads>",
        "void conv_gemm_pp_kernel<256, true>": "conv_gemm_pp_kernel<bf16,256,256,heads>",
        "void (anonymous namespace)::conv_gemm_ring_kernel<false, true>(GemmParams)":
            "conv_gemm_ring_kernel<bf16,256,128,bnbwd>",
        "void (anonymous namespace)::conv_gemm_l1p_kernel<128, true, true>(GemmParams, int)":
            "conv_gemm_l1p_kernel<bf16,128,dgrad,bnbwd>",
        "_ZN12_GLOBAL__N_125conv_gemm_heads384_kernelENS_10GemmParamsE": "conv_gemm_heads384_kernel",
    }
    for name, want in cases.items():
        assert short(name) == want, (name, short(name))
