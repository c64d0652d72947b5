"""bench.py -- 512x512 images/s training centerOffsetRes10 (bf16) on N MI355X, one process per GPU.

python bench.py --gpus N --steps K --warmup W

N>1: started under torch.distributed.run (WORLD_SIZE set; it must equal N), or by itself -- without
WORLD_SIZE the script launches N rank processes of itself (one per GPU) before touching the GPU.

A step = NetworkFactory.train on one synthetic batch of 32 tiles per GPU (zero_grad, forward,
CenterNetLoss, backward incl. the RCCL gradient all-reduce + SyncBN statistics, Adam) with the
inputs already resident in HBM.  Prints ONE JSON line on rank 0 with the metric, the roofline of
the dominant kernel (HIP events on the launch stream) and the CPU-oracle baseline.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "scd-resnet_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

TRAIN_GFLOP_PER_IMG = 147.476      # SURVEY §6 / BASELINE.md: conv+deconv fwd+dgrad+wgrad per 512^2 Res10 image
PEAK_BF16_TFLOPS = 2500.0          # MI355X dense bf16 (= dense fp16) MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0              # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="compute dtype (BASELINE configs[4] names fp16: Res50 1024^2)")
    ap.add_argument("--model", default="centerOffsetRes10")
    ap.add_argument("--image-size", type=int, default=512,
                    help="tile size; 512 uses the synthetic SCD dataset plugin, other sizes N(0,1) tiles with "
                         "random sparse targets of the same layout (e.g. BASELINE configs[4]: Res50 at 1024)")
    ap.add_argument("--cpu-baseline-steps", type=int, default=12)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--class-rooflines", type=int, default=None,
                    help="extra steps after the timed region with HIP events around every GEMM / weight-gradient / BN "
                         "launch (scdhip.ops.ClassTimer): per-class time and roofline (default: 5 for models other "
                         "than the Res10 headline, 0 for it)")
    ap.add_argument("--no-calib", action="store_true",
                    help="skip the achievable-peak calibration (scdhip.calib.mfma_peak, ~4 s after the timed steps)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as a captured HIP graph (scdhip/graph.py; single process).  Off by default: "
                         "on ROCm 7 the replayed two-stream step measured 7.85 ms against 7.63 ms eager")
    return ap.parse_args()


def cpu_baseline(steps):
    """The CPU oracle (PyTorch fp32 restatement of the reference step) on this host's cores:
    Res10, B=4, 512^2 -- the reference's CPU train.py configuration (BASELINE.json configs[0])."""
    from oracle import centernet as O
    from oracle import targets as T
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    entries, topo = O.model_spec(10)
    st = O.TrainState(O.hash_weights(entries))
    x = T.batch_inputs(5, 4, 512)
    ys = T.batch_targets(6, 4, 128)
    st.step(x, ys, topo)                       # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        st.step(x, ys, topo)
    dt = time.perf_counter() - t0
    return {"value": round(4 * steps / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": "oracle train step (fwd+loss+bwd+Adam), Res10 fp32, batch 4, 512x512, %d timed steps "
                      "after 1 warm-up (%.1f s)" % (steps, dt)}


HEADS_KERNEL = "conv_gemm_heads384_kernel"


def train_gflop_per_img(model, S):
    """Conv + transposed-conv MACs x 2 x 3 (fwd, dgrad, wgrad) per SxS image, from the model's layer shapes
    (residuals.py layout: stem /2, layerK at /4 / 2^(K-1), deconvs x2 each from /32, heads at /4);
    147.48 GFLOP for Res10 at 512."""
    import re
    tot = 0.0
    ndec = 0
    for n, m in model.named_modules():
        if isinstance(m, torch.nn.ConvTranspose2d):
            ndec += 1
            hin = S // 32 * 2 ** (ndec - 1)
            ci, co, kh, kw = m.weight.shape
            tot += 2.0 * ci * co * kh * kw * hin * hin
        elif isinstance(m, torch.nn.Conv2d):
            co, ci, kh, kw = m.weight.shape
            if n.startswith("preprocess"):
                ho = S // 2
            elif n.startswith("layer"):
                k = int(re.match(r"layer(\d+)", n).group(1))
                ho = S // 4 // 2 ** (k - 1)
                if k > 1 and n.endswith(".0.conv1") and kh == 1:     # Bottleneck: stride on conv2, conv1 at input res
                    ho *= 2
            else:
                ho = S // 4
            tot += 2.0 * co * ci * kh * kw * ho * ho
    return 3.0 * tot / 1e9


def sparse_heads_saved_gflop(model, S, ys):
    """Per image: the dense 3x3 dgrad + wgrad FLOPs of the size / offset terminals (centerNetOffset.py:106-110) that
    the sparse-support backward does not execute, minus what it runs instead (2 GEMMs of slots x 128 x 9*Cin per
    head); 0 when the path is switched off (SCD_SPARSE_HEADS=0)."""
    from scdhip import ops
    if not ops.SparseHeads.enabled:
        return 0.0
    K = ys[3].shape[1]
    h = S // 4
    saved = 0.0
    for name in ("regr", "offset"):
        m = getattr(model, name, None)
        if m is None:
            continue
        co, ci, kh, kw = m[0].weight.shape
        saved += 2 * 2.0 * co * ci * kh * kw * (h * h - K)
    return saved / 1e9


def pmc_traffic(kernel, batch, dtype, model="centerOffsetRes10", S=512):
    """HBM bytes per launch of `kernel` (a key of the summary, or a substring of one) from the newest committed
    rocprofv3 PMC summary for this workload (profiles/r<N>_pmc_*.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE and WRITE_SIZE passes: of this same bench command for Res10, of tools/pmc_kernels.py -- the same kernel
    on the same shape -- for the other BASELINE configs).  Only a summary stamped with THIS library's build identity
    (scd_version(): a hash of the sources built) is used; (None, reason) when none matches."""
    import glob
    import re
    from scdhip import lib as L
    mine = L.lib().dll.scd_version().decode()
    # (round-numbered summaries only: r<N>_pmc_*.json, newest round first; any other name is skipped)
    files = [f for f in glob.glob(os.path.join(REPO, "profiles", "r*_pmc_*.json"))
             if re.match(r"r\d+_pmc_", os.path.basename(f))]
    files.sort(key=lambda f: int(re.match(r"r(\d+)_", os.path.basename(f)).group(1)))
    other = None
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if (d.get("batch") != batch or d.get("dtype") != dtype or d.get("model", "centerOffsetRes10") != model
                or d.get("image_size", 512) != S):
            continue
        ks = d.get("kernels", {})
        hit = kernel if kernel in ks else next((k for k in sorted(ks) if kernel in k), None)
        if hit is None:
            continue
        if d.get("scd_version") != mine:
            other = other or "%s was taken with %s, not this build (%s)" % (
                os.path.relpath(f, REPO), d.get("scd_version", "an unstamped library"), mine)
            continue
        return ks[hit]["hbm_bytes"], os.path.relpath(f, REPO)
    return None, other


def heads_gemm_roofline(B, dtype_name, S=512, cin=256, hd=128, ods=(1, 4, 2), kept_px=None, model="centerOffsetRes10"):
    """The dominant kernel: the fused head GEMM (conv3x3 M=B*(S/4)^2, N=3*128, K=9*256, + bias/ReLU
    + the three 1x1 tails in the epilogue), timed live by HIP events on its launch stream around
    every launch inside the timed steps (scdhip.ops.LaunchTimer).  kept_px: the size / offset heads' hidden
    channels are stored at that many pixels only (the loss's gathered pixels; scd_conv_gemm_heads_keep)."""
    from scdhip import ops
    r = ops.LaunchTimer.mean_ms("heads_gemm")
    if r is None:
        return None
    ms, n = r
    M = B * (S // 4) ** 2
    ct = hd * len(ods)
    flops = 2.0 * M * (ct * 9 * cin + hd * sum(ods))
    esz = 4 if dtype_name == "fp32" else 2
    hid_bytes = M * ct * esz if kept_px is None else M * hd * esz + min(M, kept_px) * (ct - hd) * esz
    algo_bytes = M * cin * esz + hid_bytes + M * sum(ods) * 4 + ct * 9 * cin * esz
    achieved = flops / (ms * 1e-3) / 1e12
    peak = PEAK_F32_TFLOPS if dtype_name == "fp32" else PEAK_BF16_TFLOPS      # dense fp16 = dense bf16 MFMA rate
    kernel = "conv_gemm_kernel<f32,128,128,heads>" if dtype_name == "fp32" else HEADS_KERNEL
    if S == 512:
        traffic, src = pmc_traffic(kernel, B, dtype_name)
    else:
        traffic, src = pmc_traffic("heads384", B, dtype_name, model=model, S=S)
    return {"bound": "mfma", "kernel": kernel, "achieved": round(achieved, 1), "peak": peak,
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": None if traffic is None else round(traffic), "traffic_source": src if traffic is not None else None,
            "traffic_note": None if traffic is not None else src,
            "algorithmic_bytes": algo_bytes, "flop_per_launch": flops, "avg_launch_ms": round(ms, 4),
            "launches_timed": n}


def exchange_probe(model, dev, reps=50):
    """Before the warm-up: the measured cost of the two exchange steps on this run's transports (DESIGN §6 cost model):
    one SyncBN statistics all-reduce (2 x 512 fp64 = the widest layer's sums; ops._allreduce_stats path: peer memory
    or RCCL on the SyncBN group), mean over `reps` back-to-back calls, and one all-reduce of the whole flat fp32
    gradient (FlatDDP's buckets, AVG) on WORLD.  Max over ranks."""
    from scdhip import ops
    out = {}
    stats = torch.zeros(2 * 512, dtype=torch.float64, device=dev)
    peer = ops.bn_sync_peer()
    group = ops.bn_sync_group()

    def one():
        if peer is not None:
            peer.all_reduce(stats)
        else:
            dist.all_reduce(stats, group=group)
    for _ in range(5):
        one()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        one()
    torch.cuda.synchronize()
    out["syncbn_call_us"] = (time.perf_counter() - t0) / reps * 1e6
    g = model.flat.grad
    dist.all_reduce(g)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(3):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    out["grad_allreduce_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    out["grad_bytes"] = g.numel() * g.element_size()
    g.zero_()
    t = torch.tensor([out["syncbn_call_us"], out["grad_allreduce_ms"]], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"syncbn_call_us": round(t[0].item(), 1), "grad_allreduce_ms": round(t[1].item(), 3),
            "grad_bytes": out["grad_bytes"], "syncbn_calls_per_step": None}


def launch_ranks(n):
    """`--gpus N` without a torch.distributed launcher: start N child processes of this script, one per
    GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as torch.distributed.run would --
    the reference's own launch model, README.md:91 / train.py:67-72), before this process touches the
    GPU.  Rank 0's JSON line is passed through; a failing rank fails the run and stops the others."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print("bench: rank process %d exited with %d; stopping the others" % (p.pid, code),
                          file=sys.stderr, flush=True)
                    for q in procs:
                        os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for q in procs:
            try:
                os.killpg(q.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
    return rc


def cornernet_rooflines(B, dtype_name, S=512, C=256, Cp=128):
    """cornerNetCPool (BASELINE configs[3]).  Dominant kernel class: the CornerPool lastConv 3x3 C->C GEMM at the
    heads' resolution (conv_gemm_pp_kernel<bf16,256,256>: M = B*(S/4)^2, N = C, K = 9*C), timed live on its
    launch stream; secondary HBM roofline: the corner pool with the addend (cpool_fwd_kernel: reads the branch
    activation and the first pool's output, writes their sum; 3 x B*(S/4)^2*Cp elements)."""
    from scdhip import ops
    H = S // 4
    M = B * H * H
    esz = 2 if dtype_name == "bf16" else 4
    out = {}
    r = ops.LaunchTimer.mean_ms("cpool_lastconv")
    if r is not None:
        ms, n = r
        flops = 2.0 * M * C * 9 * C
        peak = PEAK_BF16_TFLOPS if dtype_name == "bf16" else PEAK_F32_TFLOPS
        achieved = flops / (ms * 1e-3) / 1e12
        traffic, src = pmc_traffic("conv_gemm_pp_kernel<bf16,256,256>", B, dtype_name, model="cornerNetCPool", S=S)
        out["roofline"] = {"bound": "mfma", "kernel": "conv_gemm_pp_kernel<bf16,256,256> (CornerPool lastConv)"
                           if dtype_name == "bf16" else "conv_gemm_kernel<f32,128,128>", "achieved": round(achieved, 1),
                           "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                           "traffic": None if traffic is None else round(traffic),
                           "traffic_source": src if traffic is not None else None,
                           "traffic_note": None if traffic is not None else src,
                           "algorithmic_bytes": 2 * M * C * esz + 9 * C * C * esz, "flop_per_launch": flops,
                           "avg_launch_ms": round(ms, 4), "launches_timed": n}
    r = ops.LaunchTimer.mean_ms("cpool_fwd_add")
    if r is not None:
        ms, n = r
        nbytes = 3 * M * Cp * esz
        gbs = nbytes / (ms * 1e-3) / 1e9
        traffic, src = pmc_traffic("cpool_fwd", B, dtype_name, model="cornerNetCPool", S=S)
        out["pool_roofline"] = {"bound": "hbm", "kernel": "cpool_fwd_kernel (with addend)", "achieved": round(gbs, 1),
                                "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                                "traffic": None if traffic is None else round(traffic),
                                "traffic_source": src if traffic is not None else None,
                                "traffic_note": None if traffic is not None else src,
                                "algorithmic_bytes": nbytes, "avg_launch_ms": round(ms, 4),
                                "launches_timed": n}
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench: --gpus %d but WORLD_SIZE=%d (the launcher must start one rank per GPU)"
                 % (args.gpus, world))
    if os.environ.get("SCD_BENCH_PROBE") == "1":
        # launcher rehearsal without a GPU (tests/test_host_cpu.py): rendezvous over gloo, report the world
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            world_seen = int(t.item())
            dist.destroy_process_group()
        else:
            world_seen = 1
        if rank == 0:
            print(json.dumps({"metric": "probe", "n_gpus": world, "world_seen": world_seen}), flush=True)
        return
    # rehearsal knob for a one-GPU box: SCD_BENCH_SHARE_GPU=1 puts every rank on cuda:0 over gloo (RCCL needs
    # one GPU per rank); the driver's multi-GPU runs use the default, one GPU per rank over RCCL
    share = os.environ.get("SCD_BENCH_SHARE_GPU", "0") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import importlib

    from scdhip import ops
    from scdhip.flat import FlatAdam, FlatDDP
    from scdhip.loss import mean_backward
    from trainer.dataset.syntheticSCD import SCD
    plugin = importlib.import_module("trainer.model." + args.model)
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]

    model = plugin.model(**plugin.modelParams).to(dev).set_compute_dtype(dtype).train()
    opt = FlatAdam(filter(lambda p: p.requires_grad, model.parameters()))
    if world > 1:
        if torch.cuda.device_count() > 1 or share:
            # SyncBN rule of networkFactory.py:128: peer-memory statistics when every rank maps its peers (buckets
            # then overlap the backward), else RCCL (ops.setup_syncbn)
            ops.setup_syncbn(log=(lambda m: print("bench: " + m, file=sys.stderr, flush=True)) if rank == 0 else None)
        model = FlatDDP(model)
    lossfn = plugin.loss

    # synthetic batch (per-rank shard), resident in HBM before timing
    B = args.batch
    S = args.image_size
    if S == 512:
        if args.model.startswith("cornerNet"):
            from trainer.dataset.syntheticCorner import CornerSCD
            ds = CornerSCD(None, True, seed=1000 + 97 * rank)       # ys: heat, mask, regr, tl, br
        else:
            ds = SCD(None, True, seed=1000 + 97 * rank)
        items = [ds[i] for i in range(B)]
        x = torch.stack([it["xs"][0] for it in items]).to(dev)
        ys = [torch.stack([it["ys"][k] for it in items]).to(dev) for k in range(len(items[0]["ys"]))]
    else:
        # same layout as the dataset plugin at another tile size: N(0,1) tiles, sparse heatmaps, 30 slots
        g = torch.Generator().manual_seed(1000 + 97 * rank)
        H = S // 4
        x = torch.randn(B, 1, S, S, generator=g).to(dev)
        heat = (torch.rand(B, 1, H, H, generator=g) > 0.999).float()
        mask = torch.arange(30)[None, :] < torch.randint(5, 21, (B, 1), generator=g)
        regr = torch.rand(B, 30, 6, generator=g) * 4
        inds = torch.randint(0, H * H, (B, 30), generator=g) * mask
        ys = [heat.to(dev), mask.to(dev), regr.to(dev), inds.to(dev)]

    prepare = getattr(lossfn, "prepare", None)       # CenterNetLoss: tells the heads where the loss will gather

    def train_step():
        opt.zero_grad()
        if prepare is not None:
            prepare(ys)
        loss, _ = lossfn(model(x, decode=False), ys)
        loss = mean_backward(loss)              # loss.mean(); loss.backward()
        opt.step()
        return loss

    # the dominant kernels are timed with HIP events on their launch stream; armed before any step so the
    # events are also recorded inside the captured step graphs
    ops.LaunchTimer.arm("heads_gemm")
    if args.model.startswith("cornerNet"):
        ops.LaunchTimer.arm("cpool_lastconv")
        ops.LaunchTimer.arm("cpool_fwd_add")
    graph = None
    if world == 1 and args.graph:
        # single process: the whole step (zero_grad .. Adam) replays as one HIP graph after 2 eager steps; two
        # alternating copies so the in-graph event pairs are read without stalling the queue (scdhip/graph.py)
        from scdhip.graph import StepGraph
        graph = StepGraph(train_step, optimizer=opt, warmup=2, copies=2)
        step = graph
    else:
        step = train_step

    probe = None
    if world > 1:
        probe = exchange_probe(model, dev)

    # with the graph: 2 eager steps, the capture step and the first replay of the second copy are warm-up
    nwarm = max(args.warmup, 4) if graph is not None else args.warmup
    # the step runs on a high-priority stream (SCD_STEP_PRIORITY=0: the default stream): the weight-gradient side
    # stream has the lowest priority, so the critical chain's small kernels are dispatched ahead of its GEMM tiles
    prio = os.environ.get("SCD_STEP_PRIORITY", "1") != "0"
    step_stream = torch.cuda.Stream(device=dev, priority=-10) if prio else torch.cuda.current_stream(dev)
    step_stream.wait_stream(torch.cuda.current_stream(dev))
    torch.cuda.set_stream(step_stream)
    for _ in range(nwarm):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if graph is not None:
        graph.finish()
    ops.LaunchTimer.reset()
    ops.SyncCounter.calls = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if graph is not None:
        graph.finish()
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    final_loss = loss.item()
    ops.SyncCounter.per_step = ops.SyncCounter.calls / args.steps
    local_ms = None
    if world > 1:
        # after the timed region: the same steps with every collective off (FlatDDP.local_only), max over ranks --
        # what the exchange (gradient buckets, SyncBN, buffer broadcast) adds to each rank's step, measured in-run
        with model.local_only():
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            tl = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
        dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        local_ms = 1e3 * tl.item() / args.steps

    ncls = args.class_rooflines if args.class_rooflines is not None else (
        0 if (args.model == "centerOffsetRes10" and S == 512) else 5)
    classes = None
    if ncls > 0 and world == 1:
        # after the timed region: per-class kernel time and algorithmic work over ncls more steps (events around every
        # launch of a class, on its stream; classes on the two streams overlap, so their times do not add up to the step)
        ops.ClassTimer.on = True
        for _ in range(ncls):
            step()
        ops.ClassTimer.on = False
        classes = ops.ClassTimer.collect(ncls)

    if rank == 0:
        imgs = B * world * args.steps
        value = imgs / elapsed
        # the fused CenterNet head GEMM (HeadsFn) is the dominant kernel of the centerOffset* plugins only
        extra = {}
        if args.model.startswith("centerOffset"):
            kept = None
            if prepare is not None and ops.SparseHeads.enabled and ops._KEEP_MAPS:
                # distinct gathered pixels: where the size / offset hidden channels were stored
                Hh = S // 4
                base = torch.arange(B, device=ys[3].device)[:, None] * (Hh * Hh)
                kept = int(torch.unique(ys[3].long() + base).numel())
            roof = heads_gemm_roofline(B, args.dtype, S, kept_px=kept, model=args.model)
            if roof is not None:
                roof["hidden_kept_px"] = kept
        elif args.model.startswith("cornerNet"):
            extra = cornernet_rooflines(B, args.dtype, S)
            roof = extra.pop("roofline", None)
        else:
            roof = None
        core = model.module if hasattr(model, "module") else model
        gflop = TRAIN_GFLOP_PER_IMG if (args.model == "centerOffsetRes10" and S == 512) else \
            train_gflop_per_img(core, S)
        # the size / offset heads' backward runs over the loss's gathered pixels (scdhip.blocks.HeadsFn sparse
        # path): their dense 3x3 dgrad + wgrad FLOPs are not executed, a [slots x Cs] x [Cs x 9 Cin] GEMM pair is
        gsaved = sparse_heads_saved_gflop(core, S, ys) if args.model.startswith("centerOffset") else 0.0
        executed = gflop - gsaved
        peak = world * (PEAK_F32_TFLOPS if dtype == torch.float32 else PEAK_BF16_TFLOPS)
        step_frac = value * executed / 1e3 / peak
        line = {
            "metric": "512x512 images/sec training, centerOffsetRes10, at 1/2/4/8 MI355X" if (
                args.model == "centerOffsetRes10" and S == 512) else "%dx%d images/sec training, %s" % (S, S, args.model),
            "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": nwarm, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": "%s train step (fwd+focal/L1 loss+bwd+Adam, DDP over RCCL), %dx%d synthetic "
                                   "SCD tiles" % (args.model, S, S), "model": args.model, "global_batch": B * world,
                       "step_issue": "hip graph replay" if graph is not None else "eager launches",
                       "per_gpu_batch": B, "seq_len": None, "parallelism": "dp%d" % world,
                       "image_size": S, "train_gflop_per_img": round(gflop, 3),
                       "executed_gflop_per_img": round(executed, 3)},
            "roofline": roof,
            **extra,
            "step_mfma_frac": round(step_frac, 4),
            "step_mfma_frac_dense_equiv": round(value * gflop / 1e3 / peak, 4),
            "final_loss": round(final_loss, 5),
        }
        if classes:
            mfma_peak = PEAK_F32_TFLOPS if dtype == torch.float32 else PEAK_BF16_TFLOPS
            cr = {}
            for name, d in sorted(classes.items(), key=lambda kv: -kv[1]["ms_per_step"]):
                rate = d["work_per_step"] / (d["ms_per_step"] * 1e-3)
                if name == "bn":
                    ach, peak, unit, bound = rate / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"
                else:
                    ach, peak, unit, bound = rate / 1e12, mfma_peak, "TFLOP/s", "mfma"
                cr[name] = {"bound": bound, "kernel_ms_per_step": round(d["ms_per_step"], 3),
                            "share_of_step": round(d["ms_per_step"] / line["ms_per_step"], 4),
                            "launches_per_step": round(d["launches_per_step"], 1),
                            ("gflop_per_step" if bound == "mfma" else "mb_per_step"):
                                round(d["work_per_step"] / (1e9 if bound == "mfma" else 1e6), 1),
                            "achieved": round(ach, 1), "peak": peak, "unit": unit, "frac": round(ach / peak, 4)}
            line["class_rooflines"] = {
                "method": "HIP events around every launch of a class over %d steps after the timed region "
                          "(scdhip.ops.ClassTimer); gemm = forward / input-gradient gather-GEMMs (all kernels), "
                          "wgrad = weight-gradient GEMM + split reduce, bn = BatchNorm apply / backward passes "
                          "(algorithmic bytes); the side-stream weight gradients overlap the rest" % ncls,
                **cr}
        if local_ms is not None:
            # in-run split of the N-rank step: the same per-rank work without any collective (not the driver's
            # cross-run scaling efficiency, which it computes from the per-N values itself)
            # (the exchange's overhead inside one N-rank run; 1 -> N scaling efficiency is the driver's, from its own
            # per-N runs, and is not reported here)
            shared = ops.bn_sync_shares_group(model.group)
            line["exchange"] = {"ddp_ms_per_step": line["ms_per_step"], "local_ms_per_step": round(local_ms, 3),
                                "local_over_ddp": round(local_ms / line["ms_per_step"], 4),
                                "syncbn": ops.bn_sync_mode(), "syncbn_shares_bucket_group": bool(shared),
                                "peer_fallback_reason": ops._BNSync.why,
                                "buckets_overlap_backward": bool(model.overlap_buckets()),
                                "early_bucket_launches": int(model.early_launches)}
            if probe is not None:
                # measured inputs of DESIGN §6's cost model: per-call SyncBN latency x the step's calls, plus the
                # flat-gradient all-reduce when the buckets do not overlap the backward
                probe["syncbn_calls_per_step"] = ops.SyncCounter.per_step
                line["exchange"]["probe"] = probe
        if world == 1 and not args.no_calib and dtype != torch.float32:
            # the bf16 MFMA rate this box sustains (bare 16x16x32 loops on random operands, 2 waves per SIMD, after
            # 2.5 s of back-to-back launches: MI355X_MICROARCH.md "DVFS give-back"), beside the 2.5 PF/s nameplate
            from scdhip import calib
            cal = calib.mfma_peak(waves_per_simd=2)
            pa = cal["tflops"]
            for r in ([line.get("roofline")] + [v for v in extra.values() if isinstance(v, dict)] +
                      [v for v in line.get("class_rooflines", {}).values() if isinstance(v, dict)]):
                if r and r.get("unit") == "TFLOP/s":
                    r["peak_achievable"] = pa
                    r["frac_achievable"] = round(r["achieved"] / pa, 4)
            line["peak_achievable"] = {"tflops": pa, "clock_ghz": cal["clock_ghz"],
                                       "source": "scd_calib_mfma_peak: 16x16x32 bf16 MFMA loops on random operands, "
                                                 "2 waves/SIMD, in-kernel clock from s_memtime / s_memrealtime"}
            line["step_mfma_frac_achievable"] = round(value * executed / 1e3 / (world * pa), 4)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_baseline_steps)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
