"""Tensor-level wrappers over the libscdhip C-ABI (device memory and streams come from torch).

Layouts: activations NHWC (channels innermost) in the compute dtype (fp32 parity mode,
bf16 performance mode); weights, grads, BN parameters fp32 in the reference layout.
Every wrapper enqueues on torch's current HIP stream and never synchronises.
"""
import contextlib
import ctypes
import math
import os

import torch
import torch.distributed as dist

from . import lib as L

_DT = {torch.float32: L.DT_F32, torch.bfloat16: L.DT_BF16, torch.float16: L.DT_F16}
HALF = (torch.bfloat16, torch.float16)      # 16-bit compute dtypes (same kernels, tiles and dispatch rules)


class LossScale:
    """Static loss scale of the fp16 compute mode: fp16 has 5 exponent bits, so the backward runs on gradients
    multiplied by `f16` (HeadsFn.backward scales the head-output gradients) and every parameter-gradient
    reduction multiplies by 1/scale on its way into .grad (scd_wgrad_reduce / scd_heads_bwd_weight_finalize alpha,
    scd_bn_bwd_finalize gscale): parameters see the unscaled gradient, bit-exact power-of-two unscaling.
    bf16 / fp32 run unscaled.  SCD_F16_LOSS_SCALE overrides the default 1024.  The unscaling applies inside the
    backward pass (autograd graph task) whose head gradients were scaled (``scaled_task``), so direct kernel calls
    and other models see unscaled gradients."""
    f16 = float(os.environ.get("SCD_F16_LOSS_SCALE", "1024"))
    scaled_task = None


def loss_scale(dtype):
    return LossScale.f16 if dtype == torch.float16 else 1.0


def begin_loss_scale(dtype):
    """Called where a backward pass enters the fp16 path (HeadsFn.backward): returns the factor to multiply the
    incoming gradients by and marks the running backward pass as scaled."""
    S = loss_scale(dtype)
    if S != 1.0:
        LossScale.scaled_task = _graph_task()
    return S


def grad_alpha(t):
    """1 / loss scale for a parameter gradient computed from activations / gradients like t in the running backward."""
    if t.dtype == torch.float16 and LossScale.scaled_task is not None and _graph_task() == LossScale.scaled_task:
        return 1.0 / LossScale.f16
    return 1.0


def dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise RuntimeError("libscdhip: unsupported dtype %s" % t.dtype)


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def stream():
    """torch's current HIP stream on the current device, as a raw handle (the same value as
    torch.cuda.current_stream().cuda_stream, without building a Stream object: ~10 us less per launch)."""
    return _raw_stream(_cur_device())


def ptr(t):
    return 0 if t is None else t.data_ptr()


def capturing():
    """True while torch's current stream is being captured into a HIP graph (scdhip.graph)."""
    return torch.cuda.is_initialized() and torch.cuda.is_current_stream_capturing()


def _need_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("scd-resnet_amd runs on MI355X only: got a CPU tensor (no CPU fallback; the CPU "
                               "restatement lives in oracle/ and is test infrastructure)")


# ------------------------------------------------------------------ live kernel timing

class _Event:
    """A HIP event of libscdhip (scd_event_*): torch's ROCm build refuses external event records, which a graph
    capture needs, so the timing events come from the library."""
    __slots__ = ("h",)

    def __init__(self):
        h = ctypes.c_void_p()
        L.call("scd_event_create", ctypes.byref(h))
        self.h = h.value

    def record(self):
        L.call("scd_event_record", self.h, stream())

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        L.call("scd_event_elapsed_ms", self.h, end.h, ctypes.byref(ms))
        return ms.value

    def __del__(self):
        try:
            L.lib().scd_event_destroy(self.h)
        except Exception:
            pass


class LaunchTimer:
    """HIP-event pairs recorded around selected launches on the stream they are issued on
    (bench.py's roofline: the dominant kernel timed inside the timed steps).  Disabled unless
    a name is armed, so the product path records nothing.

    Inside a step-graph capture (scdhip.graph) the pair is recorded as external event nodes of the graph
    (hipEventRecordWithFlags(..., hipEventRecordExternal)): every replay re-stamps the same two events, so the
    graph owner harvests them (``harvest``) after that replay has finished and before the graph is replayed
    again."""
    armed = set()
    events = {}           # name -> [(start, end)] eager pairs, not yet read
    times = {}            # name -> [ms] read pairs
    captured = []         # (name, start, end) recorded during the current graph capture

    @classmethod
    def arm(cls, name):
        cls.armed.add(name)
        cls.events[name] = []
        cls.times[name] = []

    @classmethod
    def reset(cls):
        """Drop what was timed so far (the armed names stay armed)."""
        for name in cls.armed:
            cls.events[name] = []
            cls.times[name] = []

    @classmethod
    def record(cls, name):
        if name not in cls.armed:
            return None
        e = _Event()
        e.record()
        return e

    @classmethod
    def close(cls, name, start):
        if start is None:
            return
        end = cls.record(name)
        if capturing():
            cls.captured.append((name, start, end))
        else:
            cls.events[name].append((start, end))

    @classmethod
    def take_captured(cls):
        out, cls.captured = cls.captured, []
        return out

    @classmethod
    def harvest(cls, pairs):
        """Read the graph-recorded pairs of a finished replay into the armed names' times."""
        for name, a, b in pairs:
            if name in cls.armed:
                cls.times[name].append(a.elapsed_ms(b))

    @classmethod
    def mean_ms(cls, name):
        ts = cls.times.get(name, []) + [a.elapsed_ms(b) for a, b in cls.events.get(name, [])]
        if not ts:
            return None
        return sum(ts) / len(ts), len(ts)


class ClassTimer:
    """Per-class kernel time and algorithmic work (bench.py: the class rooflines of BASELINE configs[3] / [4], taken
    over extra steps after the timed region): HIP-event pairs around every launch of a class on the stream it is
    issued on -- "gemm" (forward / input-gradient gather-GEMMs, FLOPs), "wgrad" (weight-gradient GEMM + split reduce,
    FLOPs), "bn" (BatchNorm apply / backward passes, HBM bytes).  Off unless enabled; eager steps only."""
    on = False
    recs = []

    @classmethod
    def begin(cls):
        if not cls.on or capturing():
            return None
        e = _Event()
        e.record()
        return e

    @classmethod
    def end(cls, name, start, work):
        if start is None:
            return
        e = _Event()
        e.record()
        cls.recs.append((name, start, e, float(work)))

    @classmethod
    def collect(cls, steps):
        """{class: {ms_per_step, work_per_step, launches_per_step}} over `steps` steps (synchronises)."""
        torch.cuda.synchronize()
        out = {}
        for name, a, b, work in cls.recs:
            d = out.setdefault(name, {"ms_per_step": 0.0, "work_per_step": 0.0, "launches_per_step": 0.0})
            d["ms_per_step"] += a.elapsed_ms(b) / steps
            d["work_per_step"] += work / steps
            d["launches_per_step"] += 1.0 / steps
        cls.recs = []
        return out


def _gemm_flops(Ci, Co, N, phases):
    arr = phases.arr
    return 2.0 * Co * Ci * sum(N * arr[i].Qh * arr[i].Qw * arr[i].ntaps for i in range(phases.n))


# ------------------------------------------------------------------ SyncBN / process group

class _BNSync:
    group = None          # torch.distributed group for SyncBatchNorm semantics (None = local BN)
    world = 1
    peer = None           # scdhip.peer.PeerAllReduce when the peer-memory path is on
    why = None            # setup_syncbn: why the peer-memory path is not in use (None when it is, or not tried)


def new_bn_group():
    """A process group of every rank, for the SyncBN statistics only (networkFactory.py:128-134 runs SyncBatchNorm
    and DDP as independent collectives).  With the nccl backend (RCCL) each group owns its communicator and its
    stream, so a critical-path SyncBN all-reduce issued from the compute stream never queues behind a gradient
    bucket that FlatDDP issued on WORLD from the weight-gradient side stream.  Collective: every rank calls it,
    once, before FlatDDP is built."""
    return dist.new_group(ranks=list(range(dist.get_world_size())))


def syncbn_group():
    """The process group for the SyncBN statistics at world > 1 (networkFactory.py:128-133).

    Default: WORLD, the group FlatDDP all-reduces its gradient buckets on -- as the reference's SyncBatchNorm and DDP
    share the default group.  With RCCL every collective of the rank then runs on one communicator and its one stream,
    in issue order, so no two communicators' kernels are ever in flight at once (that combination has not
    run at world >= 2 on RCCL).  The price: a bucket queued on that stream waits for the weight-gradient side stream,
    and a critical-path SyncBN all-reduce issued after it would wait too -- so FlatDDP launches no bucket during the
    backward while SyncBN shares its group (FlatDDP.overlap_buckets), and all buckets go at the end of the backward.
    SCD_SYNCBN_OWN_GROUP=1: a communicator of their own (new_bn_group), buckets overlap the backward.
    Collective when it creates a group: every rank calls it, once, before FlatDDP is built."""
    if os.environ.get("SCD_SYNCBN_OWN_GROUP", "0") == "1":
        return new_bn_group()
    return dist.group.WORLD


def bn_sync_shares_group(group):
    """True when SyncBN all-reduces its statistics through torch.distributed on `group` (None = WORLD), i.e. on the
    same communicator and stream as a collective issued on `group` (the peer-memory path uses no collective)."""
    g = _BNSync.group
    if g is None or _BNSync.peer is not None:
        return False
    world = dist.group.WORLD
    return (g or world) is (group or world)


def set_bn_sync(group, peer=None):
    """Enable global-batch BN statistics (SyncBatchNorm, networkFactory.py:128-133) over `group` (syncbn_group():
    WORLD by default).  peer=True (or SCD_SYNCBN_PEER=1) all-reduces them over peer memory (scdhip/peer.py) instead
    of through torch.distributed."""
    if _BNSync.peer is not None:
        _BNSync.peer.close()
        _BNSync.peer = None
    _BNSync.group = group
    _BNSync.world = dist.get_world_size(group) if group is not None else 1
    if peer is None:
        peer = os.environ.get("SCD_SYNCBN_PEER", "0") == "1"
    if group is not None and peer and _BNSync.world > 1:
        from .peer import PeerAllReduce
        _BNSync.peer = PeerAllReduce(group)


def setup_syncbn(log=None):
    """SyncBatchNorm for a data-parallel run at world > 1 (networkFactory.py:128-133), with the transport chosen so
    that FlatDDP's gradient buckets overlap the backward (networkFactory.py:126-136; BASELINE north_star: the
    all-reduce "overlapped with backward"):

    * default: through torch.distributed on ops.syncbn_group() -- WORLD, where RCCL serialises them with the buckets on
      one communicator, so every bucket goes at the end of the backward (FlatDDP.overlap_buckets) -- or a communicator
      of their own with SCD_SYNCBN_OWN_GROUP=1;
    * SCD_SYNCBN_PEER=auto: over peer memory when every rank can map every peer's mailbox -- checked collectively,
      with a probe all-reduce (scdhip.peer.PeerAllReduce.try_create) -- so SyncBN issues no collective at all and
      FlatDDP launches each bucket on WORLD from inside the backward as soon as its gradients are written; else (a
      rank cannot map its peers, no GPU, more than one node's ranks) the default above, with the reason logged.
      SCD_SYNCBN_PEER=1 requires the peer path (raises if it cannot be set up).  Opt-in until it has run on separate
      GPUs over xGMI: every run so far had its ranks share one GPU.

    Collective: every rank calls it once, before FlatDDP is built.  Returns bn_sync_mode(); `log` (a callable) gets
    one line saying which transport runs and, for a fallback, why."""
    want = os.environ.get("SCD_SYNCBN_PEER", "0").lower()
    if _BNSync.peer is not None:
        _BNSync.peer.close()
        _BNSync.peer = None
    _BNSync.why = None
    if want in ("1", "auto", "on") and torch.cuda.is_available() and dist.get_world_size() > 1:
        from .peer import PeerAllReduce
        peer, why = PeerAllReduce.try_create(dist.group.WORLD)
        if peer is None and want == "1":
            raise RuntimeError("SCD_SYNCBN_PEER=1: the peer-memory SyncBN path could not be set up: %s" % why)
        if peer is not None:
            _BNSync.group, _BNSync.world, _BNSync.peer = dist.group.WORLD, dist.get_world_size(), peer
        else:
            _BNSync.why = why
    elif want not in ("1", "auto", "on"):
        _BNSync.why = "opt-in (SCD_SYNCBN_PEER=auto)"
    else:
        _BNSync.why = "no GPU" if not torch.cuda.is_available() else "world 1"
    if _BNSync.peer is None:
        set_bn_sync(syncbn_group(), peer=False)
        _BNSync.why = _BNSync.why or "fallback"
    mode = bn_sync_mode()
    if log is not None:
        log("SyncBN statistics: %s%s; gradient buckets %s" % (
            mode, "" if _BNSync.peer is not None else " (peer memory not used: %s)" % _BNSync.why,
            "all-reduced on WORLD from inside the backward" if mode != "rccl-world" else
            "all-reduced at the end of the backward (SyncBN shares their RCCL communicator)"))
    return mode


def bn_sync_mode():
    """'peer' (peer-memory kernels), 'rccl-world' (torch.distributed on WORLD, beside the gradient buckets),
    'rccl-own' (a communicator of their own) or 'off' (local BN)."""
    if _BNSync.group is None:
        return "off"
    if _BNSync.peer is not None:
        return "peer"
    return "rccl-world" if _BNSync.group is dist.group.WORLD else "rccl-own"


def bn_sync_peer():
    return _BNSync.peer


@contextlib.contextmanager
def bn_sync_suspended():
    """Local BN statistics inside (FlatDDP.local_only); the group and the peer mailboxes are kept."""
    saved = (_BNSync.group, _BNSync.world, _BNSync.peer)
    _BNSync.group, _BNSync.world, _BNSync.peer = None, 1, None
    try:
        yield
    finally:
        _BNSync.group, _BNSync.world, _BNSync.peer = saved


def bn_sync_group():
    return _BNSync.group


def bn_sync_poll():
    """Once per step: raise if a peer-memory SyncBN call has failed (non-blocking, scdhip/peer.py)."""
    if _BNSync.peer is not None:
        _BNSync.peer.poll()


def bn_sync_world():
    return _BNSync.world if _BNSync.group is not None else 1


class SyncCounter:
    """SyncBN all-reduce calls issued (bench.py: calls per step, for the exchange cost model)."""
    calls = 0
    per_step = None


def _allreduce_stats(stats, C):
    """collapse replicas and all-reduce [2][C] fp64 over the BN group; returns nrep."""
    if _BNSync.group is None:
        return L.STAT_REPLICAS
    SyncCounter.calls += 1
    L.call("scd_stats_collapse", ptr(stats), L.STAT_REPLICAS, C, stream())
    if _BNSync.peer is not None:
        _BNSync.peer.all_reduce(stats[:2 * C])
    else:
        dist.all_reduce(stats[:2 * C], group=_BNSync.group)
    return 1


def _allreduce_stats_pair(sa, Ca, sb, Cb):
    """Two BN layers whose sums are ready together (a residual join's pair in backward; a block's bn1 and downsample BN
    in forward): both collapsed side by side into one staging buffer (scd_stats_collapse_to) and all-reduced ONCE --
    one small collective on the critical path instead of two.  Returns (stats_a, stats_b, nrep) for the finalize."""
    if _BNSync.group is None:
        return sa, sb, L.STAT_REPLICAS
    n = 2 * (Ca + Cb)
    if _BNSync.peer is not None and n > _BNSync.peer.cap:
        _allreduce_stats(sa, Ca)
        _allreduce_stats(sb, Cb)
        return sa, sb, 1
    SyncCounter.calls += 1
    stage = torch.empty(n, dtype=torch.float64, device=sa.device)
    L.call("scd_stats_collapse_to", ptr(sa), L.STAT_REPLICAS, Ca, ptr(stage), stream())
    L.call("scd_stats_collapse_to", ptr(sb), L.STAT_REPLICAS, Cb, ptr(stage[2 * Ca:]), stream())
    if _BNSync.peer is not None:
        _BNSync.peer.all_reduce(stage)
    else:
        dist.all_reduce(stage, group=_BNSync.group)
    return stage[:2 * Ca], stage[2 * Ca:], 1


def new_stats(C, device):
    return torch.zeros(L.STAT_REPLICAS * 2 * C, dtype=torch.float64, device=device)


def persistent_zeros(owner, attr, numel, dtype):
    """A zero-initialised device buffer cached on `owner` (a module/parameter).  The kernels that
    consume it (BN finalize, stats collapse, heads finalize, loss finalize) re-zero what they read,
    so it is ready for the next use without a memset launch."""
    buf = getattr(owner, attr, None)
    dev = owner.device if torch.is_tensor(owner) else owner.weight.device
    if buf is None or buf.numel() != numel or buf.device != dev or buf.dtype != dtype:
        buf = torch.zeros(numel, dtype=dtype, device=dev)
        setattr(owner, attr, buf)
    return buf


def bn_stats(bn, which):
    """Persistent fp64 [replicas][2][C] statistics buffer of a BatchNorm module ('fwd' / 'bwd')."""
    return persistent_zeros(bn, "_scd_stats_" + which, L.STAT_REPLICAS * 2 * bn.num_features, torch.float64)


# ------------------------------------------------------------------ weights

class PackPlan:
    """Per-model cache of the packed weight operands of one training step.

    The first step records every (parameter, layout) a block asks for and packs it on demand; from then on
    ``pack_begin`` repacks all of them in ONE ``scd_pack_weights_batched`` launch at the start of the model's
    forward (the parameters change every optimizer step), and ``pack_weight`` / ``pack_concat`` return the
    packed views.  Only nn.Parameter arguments are cached (keyed by the Parameter object); the plan is active
    from the model's forward until the next optimizer step (``pack_end``)."""

    def __init__(self):
        self.entries = {}           # key -> [out tensor, parts, dtype, used]
        self._sig = None
        self._dev = {}              # dtype -> (device descriptor tensor, n, total)
        self.frozen = False         # a captured step graph uses the operands / descriptors: never free them
        self._retired = []

    def lookup(self, key):
        e = self.entries.get(key)
        if e is None:
            return None
        e[3] = True
        return e[0]

    def add(self, key, out, parts, dtype):
        self.entries[key] = [out, parts, dtype, True]

    def refresh(self):
        # drop entries the previous step did not use, then repack the rest (one launch per dtype); a plan that a
        # captured step graph refers to keeps every operand and descriptor table it ever built alive
        if capturing():
            self.frozen = True
        if not self.frozen:
            self.entries = {k: e for k, e in self.entries.items() if e[3]}
        if not self.entries:
            return
        sig = tuple((k, e[0].data_ptr(), tuple(p[0].data_ptr() for p in e[1])) for k, e in self.entries.items())
        if sig != self._sig:
            if capturing():
                raise RuntimeError("PackPlan: the operand set changed inside a step-graph capture (run an eager "
                                   "step first)")
            self._sig = sig
            if self.frozen:
                self._retired.append(self._dev)
            self._dev = {}
            per = {}
            for e in self.entries.values():
                per.setdefault(e[2], []).append(e)
            for dtype, es in per.items():
                descs, start = [], 0
                for out, parts, _, _ in es:
                    for (w, mode, ldp, row_off, a_off, a_tot) in parts:
                        A, B, T = w.shape[0], w.shape[1], w.shape[2] * w.shape[3]
                        d = L.PackDesc(w.data_ptr(), out.data_ptr(), start, A, B, T, mode, ldp, row_off, a_off, a_tot)
                        descs.append(d)
                        if mode == 0:
                            start += (A * ldp + 4095) // 4096 * 4096      # whole workgroup units per descriptor
                        elif mode == 3:
                            start += (4 * B * ldp + 4095) // 4096 * 4096
                        elif mode == 2:
                            start += (A * B * T + 4095) // 4096 * 4096
                        else:
                            # one 4096-element unit per 64 x max(1, 64 // T) transpose tile (scd_pack_desc)
                            bb = max(1, 64 // T)
                            start += ((A + 63) // 64) * ((B + bb - 1) // bb) * 4096
                arr = (L.PackDesc * len(descs))(*descs)
                host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
                self._dev[dtype] = (host.to(es[0][0].device), len(descs), start)
        for dtype, (dev, n, total) in self._dev.items():
            L.call("scd_pack_weights_batched", _DT[dtype], dev.data_ptr(), n, total, stream())
        for e in self.entries.values():
            e[3] = False


_ACTIVE_PLAN = None


def pack_begin(plan):
    """Start of a model forward: repack every recorded operand (one launch) and activate the plan."""
    global _ACTIVE_PLAN
    clear_bn_fusion()
    _ACTIVE_PLAN = None
    plan.refresh()
    _ACTIVE_PLAN = plan


def pack_end():
    """Parameters are about to change (optimizer step): stop serving cached operands."""
    global _ACTIVE_PLAN
    _ACTIVE_PLAN = None


def pack_concat(ws, dtype, mode):
    """Pack the row-concatenation of the conv weights `ws` (same (B,kh,kw)) without materialising the
    concatenation: mode 0 stacks their output rows, mode 1 interleaves their columns per tap."""
    A_tot = sum(w.shape[0] for w in ws)
    B, T = ws[0].shape[1], ws[0].shape[2] * ws[0].shape[3]
    plan = _ACTIVE_PLAN
    key = (tuple(id(w) for w in ws), dtype, mode)
    if plan is not None and all(isinstance(w, torch.nn.Parameter) for w in ws):
        hit = plan.lookup(key)
        if hit is not None:
            return hit
    if mode == 0:
        out = torch.empty(A_tot, T * B, dtype=dtype, device=ws[0].device)
        parts, off = [], 0
        for w in ws:
            parts.append((w, 0, T * B, off, 0, 0))
            pack_weight(w, dtype, 0, out=out, row_off=off, _cache=False)
            off += w.shape[0]
    elif mode == 2:
        # [taps][B][A_tot]: the transposed weight with tap-major rows (scd_heads_sparse_fixup's operand)
        out = torch.empty(T * B, A_tot, dtype=dtype, device=ws[0].device)
        parts, off = [], 0
        for w in ws:
            parts.append((w, 2, A_tot, 0, off, A_tot))
            L.call("scd_pack_weight", _DT[dtype], ptr(w), ptr(out), w.shape[0], B, T, 2, A_tot, off, stream())
            off += w.shape[0]
    else:
        cat = torch.cat(list(ws), 0)
        out = pack_weight(cat, dtype, 1, _cache=False)
        parts, off = [], 0
        for w in ws:
            parts.append((w, 1, T * A_tot, 0, off, A_tot))
            off += w.shape[0]
    if plan is not None and all(isinstance(w, torch.nn.Parameter) for w in ws):
        plan.add(key, out, parts, dtype)
    return out


def pack_weight(w, dtype, mode, ldp=None, out=None, row_off=0, _cache=True):
    """(A,B,kh,kw) fp32 -> GEMM operand. mode 0: [A][taps][B]; mode 1: [B][taps][A].
    During a model step (PackPlan active) a Parameter's operand comes from the step's batched pack."""
    plan = _ACTIVE_PLAN
    if _cache and out is None and row_off == 0 and plan is not None and isinstance(w, torch.nn.Parameter):
        key = (id(w), dtype, mode, ldp)
        hit = plan.lookup(key)
        if hit is not None:
            return hit
        res = pack_weight(w, dtype, mode, ldp, _cache=False)
        T = w.shape[2] * w.shape[3]
        plan.add(key, res, [(w, mode, res.shape[1], 0, 0, w.shape[0])], dtype)
        return res
    A, B = w.shape[0], w.shape[1]
    T = w.shape[2] * w.shape[3]
    if mode == 3:          # stride-2 3x3 input gradient as a 2x2-tap GEMM: (4 B) x (4 A), scd_conv_dgrad_s2
        rows, ldp = 4 * B, ldp or 4 * A
    else:
        rows = A if mode == 0 else B
        ldp = ldp or T * (B if mode == 0 else A)
    if out is None:
        out = torch.empty(rows, ldp, dtype=dtype, device=w.device)
    L.call("scd_pack_weight", _DT[dtype], ptr(w), ptr(out), A, B, T, mode, ldp, row_off, stream())
    return out


# ------------------------------------------------------------------ gather-GEMM convolution

class _Phases:
    """A GEMM's phase descriptors as the ctypes array the C-ABI takes (built once per geometry and reused: the
    launches of a step would otherwise rebuild ~40 of them in Python)."""
    __slots__ = ("arr", "n", "list")

    def __init__(self, phases):
        self.list = phases
        self.n = len(phases)
        self.arr = (L.GemmPhase * max(1, self.n))(*phases)

    def __len__(self):
        return self.n

    def __iter__(self):
        return iter(self.list)


_PHASES = {}


def _fwd_phase(kh, kw, pad, Ho, Wo):
    key = ("f", kh, kw, pad, Ho, Wo)
    ps = _PHASES.get(key)
    if ps is None:
        ph = L.GemmPhase()
        ph.Qh, ph.Qw, ph.rho_h, ph.rho_w = Ho, Wo, 0, 0
        ph.ntaps = kh * kw
        for r in range(kh):
            for s in range(kw):
                t = r * kw + s
                ph.dh[t], ph.dw[t], ph.wt[t] = r - pad, s - pad, t
        ps = _PHASES[key] = _Phases([ph])
    return ps


def _dgrad_phases(kh, kw, stride, pad, Hc, Wc, nonempty=False):
    """Sub-pixel decomposition of the input-gradient of Conv2d(kh,kw,stride,pad) whose input is
    (Hc,Wc): output pixel st*q+rho gathers dy at q + (rho+pad-r)/st for taps r = rho+pad (mod st).
    nonempty: without the phases that have no taps."""
    key = ("d", kh, kw, stride, pad, Hc, Wc, nonempty)
    ps = _PHASES.get(key)
    if ps is not None:
        return ps
    phases = []
    for rh in range(stride):
        for rw in range(stride):
            Qh = -(-(Hc - rh) // stride)
            Qw = -(-(Wc - rw) // stride)
            if Qh <= 0 or Qw <= 0:
                continue
            ph = L.GemmPhase()
            ph.Qh, ph.Qw, ph.rho_h, ph.rho_w = Qh, Qw, rh, rw
            taps = [(r, s) for r in range(kh) if (r - rh - pad) % stride == 0
                    for s in range(kw) if (s - rw - pad) % stride == 0]
            ph.ntaps = len(taps)
            for t, (r, s) in enumerate(taps):
                ph.dh[t] = (rh + pad - r) // stride
                ph.dw[t] = (rw + pad - s) // stride
                ph.wt[t] = r * kw + s
            if ph.ntaps > 0 or not nonempty:
                phases.append(ph)
    ps = _PHASES[key] = _Phases(phases)
    return ps


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def pad_channels(t, C, Cp, rows):
    """Zero-extend the innermost C channels of `t` (viewed as rows x C) to Cp (scd_pad_channels)."""
    out = torch.empty(rows, Cp, dtype=t.dtype, device=t.device)
    L.call("scd_pad_channels", dt(t), ptr(t), rows, C, Cp, ptr(out), stream())
    return out


def _gemm(x, wpack, y, Co, Ho, Wo, in_stride, out_stride, phases, bias=None, stats=None, relu=False,
          accumulate=False, bn_bwd=None):
    N, Hi, Wi, Ci = x.shape
    bk = 64 if x.dtype in HALF else 32
    if Ci % bk:
        # narrow layer (16/32 channels): zero-extend the input per pixel and the operand per tap to the K-stage
        Cp = -(-Ci // bk) * bk
        T = wpack.shape[1] // Ci
        if T * Ci != wpack.shape[1]:
            raise RuntimeError("narrow-layer padding needs an unpadded [rows][taps*Ci] operand")
        x = pad_channels(_c(x), Ci, Cp, N * Hi * Wi).view(N, Hi, Wi, Cp)
        wpack = pad_channels(wpack, Ci, Cp, wpack.shape[0] * T).view(wpack.shape[0], T * Cp)
        Ci = Cp
    arr, nph = phases.arr, phases.n
    t0 = ClassTimer.begin()
    if bn_bwd is not None:
        # bn_bwd = (st, y_pre_bn, stats): the next BN+ReLU layer's backward sums from the GEMM epilogue
        st, ybn, bstats = bn_bwd
        assert bias is None and stats is None and not relu and not accumulate
        L.call("scd_conv_gemm_bnbwd", dt(x), ptr(x), ptr(wpack), ptr(y), N, Hi, Wi, Ci, Ho, Wo, Co, in_stride,
               out_stride, wpack.shape[1], nph, arr, ptr(ybn), ptr(st.mean), ptr(st.invstd), ptr(st.scale),
               ptr(st.shift), ptr(bstats), stream())
    else:
        L.call("scd_conv_gemm", dt(x), ptr(x), ptr(wpack), ptr(y), ptr(bias), ptr(stats), N, Hi, Wi, Ci, Ho, Wo, Co,
               in_stride, out_stride, wpack.shape[1], int(relu), int(accumulate), nph, arr, stream())
    if t0 is not None:
        ClassTimer.end("gemm", t0, _gemm_flops(Ci, Co, N, phases))
    return y


def conv_fwd(x, wpack, Co, kh, kw, stride, pad, bias=None, stats=None, relu=False, out=None):
    """Conv2d forward (NHWC); wpack = pack_weight(w, mode=0)."""
    _need_gpu(x)
    N, H, W, _ = x.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Co, dtype=x.dtype, device=x.device)
    return _gemm(x, wpack, out, Co, Ho, Wo, stride, 1, _fwd_phase(kh, kw, pad, Ho, Wo), bias, stats, relu)


def conv_dgrad(dy, wpack_t, Cin, Hc, Wc, kh, kw, stride, pad, out=None, accumulate=False, stats=None, bn_bwd=None):
    """Input-gradient of Conv2d (NHWC) as a phase-decomposed gather-GEMM; wpack_t = pack_weight(w, mode=1).
    Also ConvTranspose2d forward (with the transposed conv's geometry).  bn_bwd: see _gemm."""
    N = dy.shape[0]
    if out is None:
        out = torch.empty(N, Hc, Wc, Cin, dtype=dy.dtype, device=dy.device)
    # accumulating: sub-pixel phases without taps (a 1x1 stride-2 conv reaches one pixel in four) would only add zeros
    phases = _dgrad_phases(kh, kw, stride, pad, Hc, Wc, nonempty=accumulate)
    if not phases.n:
        return out
    return _gemm(dy, wpack_t, out, Cin, Hc, Wc, 1, stride, phases, stats=stats, accumulate=accumulate, bn_bwd=bn_bwd)


class DgradS2:
    enabled = os.environ.get("SCD_DGRAD_S2", "1") != "0"


def conv_dgrad_w(dy, w, Hc, Wc, stride, pad, out=None, accumulate=False):
    """Input gradient of Conv2d(w) from the fp32 weight: a 3x3 / stride 2 / pad 1 conv whose input is exactly twice
    dy's size runs as one 2x2-tap GEMM with the sub-pixel phases as output channels (scd_conv_dgrad_s2: no
    one-tap phases of nearly empty tiles) where the ping-pong kernel takes it; everything else as conv_dgrad."""
    N, Hq, Wq, Cg = dy.shape
    Cin, kh, kw = w.shape[1], w.shape[2], w.shape[3]
    if (DgradS2.enabled and dy.dtype in HALF and kh == 3 and kw == 3 and stride == 2 and pad == 1 and Hc == 2 * Hq
            and Wc == 2 * Wq):
        if out is None:
            out = torch.empty(N, Hc, Wc, Cin, dtype=dy.dtype, device=dy.device)
        rc = L.lib().scd_conv_dgrad_s2(dt(dy), ptr(dy), ptr(pack_weight(w, dy.dtype, 3)), ptr(out), N, Hq, Wq, Cg, Cin,
                                       int(accumulate), stream())
        if rc == 0:
            return out
        if rc != 9001:
            L.check(rc, "scd_conv_dgrad_s2")
    return conv_dgrad(dy, pack_weight(w, dy.dtype, 1), Cin, Hc, Wc, kh, kw, stride, pad, out=out,
                      accumulate=accumulate)


def deconv_fwd(x, wpack_t, Cout, k=4, stride=2, pad=1, stats=None):
    """ConvTranspose2d(k, stride, pad, output_padding=0) forward; wpack_t = pack_weight(W_t, mode=1)."""
    _need_gpu(x)
    N, H, W, _ = x.shape
    Ho = (H - 1) * stride - 2 * pad + k
    Wo = (W - 1) * stride - 2 * pad + k
    return conv_dgrad(x, wpack_t, Cout, Ho, Wo, k, k, stride, pad, stats=stats)


def deconv_dgrad(dy, wpack, Cin, k=4, stride=2, pad=1, out=None, accumulate=False, bn_bwd=None):
    """ConvTranspose2d input-gradient = Conv2d forward of dy; wpack = pack_weight(W_t, mode=0)."""
    N, H, W, _ = dy.shape
    Ho = (H + 2 * pad - k) // stride + 1
    Wo = (W + 2 * pad - k) // stride + 1
    if out is None:
        out = torch.empty(N, Ho, Wo, Cin, dtype=dy.dtype, device=dy.device)
    return _gemm(dy, wpack, out, Cin, Ho, Wo, stride, 1, _fwd_phase(k, k, pad, Ho, Wo), accumulate=accumulate,
                 bn_bwd=bn_bwd)


# ------------------------------------------------------------------ BN-backward sums from the producing GEMM
#
# A BN+ReLU layer (DeconvBNFn) registers its output with (bn, BNState, pre-BN y); the module that consumes it
# (HeadsFn, the next DeconvBNFn) looks it up in ITS forward, and in its backward computes the input gradient
# with scd_conv_gemm_bnbwd, which adds that BN layer's backward sums in the GEMM epilogue into a dedicated
# buffer ("bwdf").  The BN layer's backward then takes those sums instead of running scd_bn_bwd_reduce -- only
# if the gradient it receives is exactly the tensor the GEMM wrote; otherwise it zeroes the buffer and reduces
# as usual.  Keys carry data pointer, shape and version, so a stale or copied tensor never matches.

_BN_PRODUCER = {}
_BN_FUSED = {}


class BNFusion:
    enabled = os.environ.get("SCD_BN_FUSE", "1") != "0"


def _tkey(t):
    return (t.data_ptr(), tuple(t.shape), t._version)


def set_bn_producer(out, bn, st, y):
    # (called from autograd Function.forward, where grad mode is off: training mode is the condition)
    if BNFusion.enabled and bn.training:
        _BN_PRODUCER[_tkey(out)] = (bn, st, y)


def bn_producer(t):
    """(bn, st, y) of the BN+ReLU layer that produced t in this forward, or None."""
    return _BN_PRODUCER.pop(_tkey(t), None)


def fused_bn_bwd_args(prod):
    """bn_bwd argument for a GEMM computing the gradient of prod's output (prod from bn_producer)."""
    bn, st, y = prod
    return (st, y, bn_stats(bn, "bwdf"))


# ------------------------------------------------------------------ one input gradient for several consumers
#
# A feature map read by several scdhip Functions (the CornerNet feature: the heatmap head and the TL / BR corner
# pools, cornerNetCPool.py:163-199) would get one input gradient from each, which autograd then sums with
# elementwise adds (2 x 805 MB of HBM traffic per step at B=32).  share_grad registers the consumers in forward;
# in backward the first one to run allocates the gradient buffer, the others accumulate their input-gradient GEMMs
# into it (accumulate epilogue); every consumer but the LAST returns None (autograd adds nothing for None) and the
# last returns the finished sum, so autograd never holds a partial buffer that a later consumer still adds into (an
# extra non-scdhip consumer of the feature -- another loss term, a hook -- is summed with the complete gradient,
# ADVICE r2 ops.py:630).  A consumer registered in forward whose backward never runs would leave the sum unreturned:
# the end-of-backward check raises instead of dropping it.  A slot never matches a later step: the next
# registration clears it, and keys carry data pointer, shape and version.

class SharedGrad:
    enabled = os.environ.get("SCD_SHARED_GRAD", "1") != "0"


_SHARED_GRAD = {}


def share_grad(t, n):
    """t feeds n scdhip Functions in this (grad-enabled) forward."""
    if SharedGrad.enabled and n > 1 and torch.is_grad_enabled() and t.requires_grad:
        _SHARED_GRAD.clear()
        _SHARED_GRAD[_tkey(t)] = [n, None]


def shared_grad_slot(t):
    """In a consumer's backward: [remaining consumers, buffer or None] when t's gradient is shared, else None."""
    return _SHARED_GRAD.get(_tkey(t)) if _SHARED_GRAD else None


def _shared_grad_check(key, slot):
    if slot[0] > 0 and _SHARED_GRAD.get(key) is slot:
        _SHARED_GRAD.pop(key, None)
        raise RuntimeError("scdhip: %d consumer(s) of a shared feature gradient never ran backward; the partial sum "
                           "was not handed to autograd (ops.share_grad)" % slot[0])


def shared_grad_out(t, slot, grad):
    """Record that this consumer has written its part; grad: the buffer it allocated (first consumer) or None.
    Returns what the consumer's backward hands autograd for t: the complete sum from the last consumer, else None."""
    key = _tkey(t)
    if slot[1] is None:
        slot[1] = grad
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _shared_grad_check(key, slot))
    slot[0] -= 1
    if slot[0] <= 0:
        _SHARED_GRAD.pop(key, None)
        return slot[1]
    return None


def mark_bn_bwd_fused(bn, grad):
    _BN_FUSED[id(bn)] = _tkey(grad)


def take_bn_bwd_fused(bn, dout):
    """The epilogue-accumulated backward sums of bn if they belong to dout, else None (buffer re-zeroed)."""
    k = _BN_FUSED.pop(id(bn), None)
    if k is None:
        return None
    buf = bn_stats(bn, "bwdf")
    if k != _tkey(dout):
        buf.zero_()
        return None
    return buf


def clear_bn_fusion():
    _BN_PRODUCER.clear()


# ------------------------------------------------------------------ sparse head-output gradients
#
# CenterNetLoss trains the regression / offset heads through L1LossMask on gather(head, inds) only
# (centerNetOffset.py:199-214): the gradient it hands back for those outputs is zero outside the gathered pixels.
# CenterNetLossFn.backward certifies that here (the gradient buffer, its version, the index tensor); HeadsFn.backward
# then runs those heads' backward over the certified pixels (scd_heads_sparse_bwd / _fixup) instead of dense GEMMs.
# The entry holds the buffer, so its storage cannot be reused while registered; a gradient that autograd summed,
# copied or that was modified in place (other storage / version) does not match and takes the dense path.

class SparseHeads:
    enabled = os.environ.get("SCD_SPARSE_HEADS", "1") != "0"


_SPARSE_GRAD = {}


def certify_sparse_grad(buf, inds):
    """`buf` (and its views) is zero outside the pixels inds[b][k] of each image (inds: (N, K) int64)."""
    if SparseHeads.enabled:
        _SPARSE_GRAD[buf.untyped_storage().data_ptr()] = (buf, buf._version, inds)


def clear_sparse_grads():
    _SPARSE_GRAD.clear()


def sparse_grad_inds(g):
    """The certified index tensor of gradient `g`, or None."""
    if g is None or not _SPARSE_GRAD:
        return None
    e = _SPARSE_GRAD.get(g.untyped_storage().data_ptr())
    if e is None:
        return None
    buf, ver, inds = e
    if buf._version != ver or g._version != ver:
        return None
    return inds


_HEADS_HINT = [None]
_KEEP_MAPS = {}


def hint_sparse_support(inds):
    """The gather indices (N, K) of the loss that will consume the next heads forward (CenterNetLoss.prepare,
    called by the training step before the model): that forward then stores the size / offset heads' hidden
    activations at those pixels only -- their sparse backward reads nothing else, and HeadsFn recomputes the whole
    tensor if the backward turns out dense.  One-shot: taken by the next HeadsFn.forward."""
    if SparseHeads.enabled and inds is not None:
        conv = inds.to(torch.int64).contiguous()
        _HEADS_HINT[0] = (inds, inds._version, conv)


def take_sparse_hint():
    h = _HEADS_HINT[0]
    _HEADS_HINT[0] = None
    _LAST_HINT[0] = h
    return h[2] if h is not None else None


def hinted_inds(inds):
    """inds as int64 contiguous: the very tensor the hint converted when `inds` is the hinted one (so HeadsFn can
    tell by identity that the loss gathers where its forward kept the hidden activations)."""
    h = _HEADS_HINT[0] if _HEADS_HINT[0] is not None else _LAST_HINT[0]
    if h is not None and h[0] is inds and h[1] == inds._version:
        return h[2]
    return inds.to(torch.int64).contiguous()


_LAST_HINT = [None]


def heads_keep_map(inds, N, HW):
    """Persistent uint8 map (N*HW) of inds' pixels for scd_conv_gemm_heads_keep (scd_heads_keep_map clears the
    previous call's pixels itself)."""
    K = inds.shape[1]
    key = (str(inds.device), N * HW, K)
    e = _KEEP_MAPS.get(key)
    if e is None:
        e = (torch.zeros(N * HW, dtype=torch.uint8, device=inds.device),
             torch.full((N * K,), -1, dtype=torch.int64, device=inds.device))
        _KEEP_MAPS[key] = e
    keep, prev = e
    L.call("scd_heads_keep_map", ptr(inds), N, K, HW, ptr(prev), prev.numel(), ptr(keep), stream())
    return keep


_SPARSE_MAPS = {}


def sparse_maps(dev, npix):
    """Persistent pixel maps of the sparse heads backward (slot map -1, owner map INT_MAX; the kernels restore
    them after every use)."""
    key = (str(dev), npix)
    m = _SPARSE_MAPS.get(key)
    if m is None:
        m = (torch.full((npix,), -1, dtype=torch.int32, device=dev),
             torch.full((npix,), 0x7fffffff, dtype=torch.int32, device=dev))
        _SPARSE_MAPS[key] = m
    return m


# ------------------------------------------------------------------ weight gradients on a side stream
#
# Inside a backward pass the weight-gradient GEMMs (+ their split reductions) only feed the optimizer (and
# the DDP buckets), while the input-gradient chain (dgrad GEMM -> BN backward -> next dgrad ...) is the
# critical path.  They go to one side HIP stream per device, ordered after everything the compute stream
# has queued so far, so they fill the gaps the chain leaves (small BN / finalize launches, GEMM tails).
# Their operands are recorded on the side stream (the caching allocator keeps them alive until it is
# done); an end-of-backward callback makes the compute stream wait for the side stream, before Adam,
# zero_grad or anything else can touch the gradients.  SCD_WGRAD_STREAM=0 keeps everything on one stream.

class _Side:
    enabled = os.environ.get("SCD_WGRAD_STREAM", "1") != "0"
    batch = None          # inside side_batch(): device indices whose side stream is already ordered
    priority = 10         # mapped to the lowest valid stream priority
    streams = {}          # device index -> side stream
    joined_task = {}      # device index -> graph task whose end-of-backward join is queued


def _graph_task():
    try:
        return torch._C._current_graph_task_id()
    except Exception:
        return -1


def side_stream(dev):
    """The device's side stream, ordered after the current stream, if called inside a backward pass."""
    task = _graph_task()
    if not _Side.enabled or task == -1:
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _Side.streams.get(idx)
    if s is None:
        # the lowest priority the device offers: when both queues have work ready, the CP dispatches the critical
        # input-gradient chain's workgroups first (a training step run on a high-priority stream benefits; on the
        # default stream both are equal)
        s = _new_side_stream(idx)
        _Side.streams[idx] = s
    if _Side.batch is None or idx not in _Side.batch:
        s.wait_stream(torch.cuda.current_stream(idx))
        if _Side.batch is not None:
            _Side.batch.add(idx)
    if _Side.joined_task.get(idx) != task:
        _Side.joined_task[idx] = task
        torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
    return s


def _new_side_stream(idx):
    return torch.cuda.Stream(device=idx, priority=_Side.priority)


@contextlib.contextmanager
def side_batch():
    """Weight gradients submitted to the side stream back to back, with no compute-stream work between them: the side
    stream is ordered after the compute stream once.  Each ordering is an event marker in the compute stream's queue,
    a ~6 us bubble there (profiles/r6_ab.txt)."""
    outer = _Side.batch
    _Side.batch = set() if outer is None else outer
    try:
        yield
    finally:
        _Side.batch = outer


def join_side_streams():
    """Make every device's compute stream wait for its side stream (end of backward)."""
    for idx, s in _Side.streams.items():
        torch.cuda.current_stream(idx).wait_stream(s)
    _Side.joined_task.clear()


def side_stream_for_comm(dev):
    """For a collective launched during backward: the side stream (if any), first ordered after the compute
    stream, so that a collective issued from it sees every gradient written on either stream so far."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _Side.streams.get(idx)
    if s is None or _graph_task() == -1:
        return None
    s.wait_stream(torch.cuda.current_stream(idx))
    return s


def conv_wgrad(g, x, kh, kw, stride, pad, dst, ld, cvalid=None, accumulate=True, rows=None, red_taps=1):
    _conv_wgrad_side(g, x, kh, kw, stride, pad, dst, ld, cvalid, accumulate, rows, red_taps)


def _conv_wgrad_side(g, x, kh, kw, stride, pad, dst, ld, cvalid=None, accumulate=True, rows=None, red_taps=1):
    side = side_stream(g.device) if g.is_cuda else None
    if side is None:
        return _conv_wgrad(g, x, kh, kw, stride, pad, dst, ld, cvalid, accumulate, rows, red_taps)
    with torch.cuda.stream(side):
        _conv_wgrad(g, x, kh, kw, stride, pad, dst, ld, cvalid, accumulate, rows, red_taps)
    g.record_stream(side)
    x.record_stream(side)


def _conv_wgrad(g, x, kh, kw, stride, pad, dst, ld, cvalid=None, accumulate=True, rows=None, red_taps=1):
    """Weight gradient of the gather-GEMM: dst[(r-r0)*ld_n + ci*ld_c + t*ld_t] (+)= sum_pix g[pix,r] x[gather,ci].

    g: (N,Ho,Wo,Cg) NHWC output-gradient; x: (N,Hi,Wi,Ci) NHWC input; taps gather
    x at (stride*oh + r - pad, stride*ow + s - pad).  `rows` = list of (r0, r1, dst, ld) slices.
    """
    N, Ho, Wo, Cg = g.shape
    _, Hi, Wi, Ci = x.shape
    T = kh * kw
    d = dt(g)
    key = (d, N, Ho, Wo, Cg, Ci, kh, kw, pad)
    plan = _WGRAD_PLANS.get(key)
    if plan is None:
        dh = L.int_array([r - pad for r in range(kh) for s in range(kw)])
        dw = L.int_array([s - pad for r in range(kh) for s in range(kw)])
        ns = L.lib().scd_conv_wgrad_nsplit2(d, N * Ho * Wo, Ho, Wo, Cg, T, Ci)
        plan = _WGRAD_PLANS[key] = (dh, dw, ns, L.lib().scd_conv_wgrad_workspace(Cg, T, Ci, ns) // 4)
    dh, dw, ns, wsn = plan
    ws = torch.empty(wsn, dtype=torch.float32, device=g.device)
    t0 = ClassTimer.begin()
    L.call("scd_conv_wgrad", d, ptr(g), ptr(x), ptr(ws), ns, N, Ho, Wo, Cg, Hi, Wi, Ci, stride, T, dh, dw, stream())
    if rows is None:
        rows = [(0, Cg, dst, ld)]
    # red_taps: read the T*Ci workspace columns as red_taps taps of T*Ci/red_taps channels (a 1x1 GEMM over
    # im2col rows, whose columns are the taps of a wider convolution)
    Tr, Cr = T * red_taps, Ci // red_taps
    cv = Cr if cvalid is None else cvalid
    for i in range(0, len(rows), 4):      # up to four row slices per reduce launch
        part = rows[i:i + 4]
        rkey = tuple((r[0], r[1], ptr(r[2]), tuple(r[3])) for r in part)
        arrs = _WGRAD_ROWS.get(rkey)
        if arrs is None:
            if len(_WGRAD_ROWS) > 4096:
                _WGRAD_ROWS.clear()
            arrs = _WGRAD_ROWS[rkey] = (
                L.int_array([r[0] for r in part]), L.int_array([r[1] for r in part]),
                L.long_array([r[3][0] for r in part]), L.long_array([r[3][1] for r in part]),
                L.long_array([r[3][2] for r in part]), L.ptr_array([ptr(r[2]) for r in part]))
        L.call("scd_wgrad_reduce_rows", ptr(ws), ns, Cg, Tr, Cr, len(part), *arrs, cv, int(accumulate), grad_alpha(g),
               stream())
    if t0 is not None:
        ClassTimer.end("wgrad", t0, 2.0 * N * Ho * Wo * Cg * T * Ci)


# geometry -> (dh, dw, split count, workspace floats); (row slices) -> the reduce's argument arrays (keyed by the
# destination pointers, which are views of the persistent flat gradient buffer)
_WGRAD_PLANS = {}
_WGRAD_ROWS = {}


# ------------------------------------------------------------------ BatchNorm (training)

class BNState:
    """Per-call BN quantities kept for backward."""
    __slots__ = ("mean", "invstd", "scale", "shift", "count")


def bn_finalize(bn, stats, C, count, training=True):
    """Finalize statistics of a torch.nn.BatchNorm2d-shaped module `bn` (weight/bias/running_*)."""
    st = _bn_state(C, bn.weight.device)
    if training:
        return _bn_finalize_launch(bn, st, stats, _allreduce_stats(stats, C), C, count)
    else:
        L.call("scd_bn_finalize", 0, 0, C, 1.0, ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
               ptr(bn.running_var), 0, 0.0, float(bn.eps), ptr(st.mean), ptr(st.invstd), ptr(st.scale),
               ptr(st.shift), stream())
    st.count = count
    return st


def _bn_finalize_launch(bn, st, stats, nrep, C, count):
    count = count * bn_sync_world()
    L.call("scd_bn_finalize", ptr(stats), nrep, C, float(count), ptr(bn.weight), ptr(bn.bias),
           ptr(bn.running_mean), ptr(bn.running_var), ptr(bn.num_batches_tracked), float(bn.momentum),
           float(bn.eps), ptr(st.mean), ptr(st.invstd), ptr(st.scale), ptr(st.shift), stream())
    st.count = count
    return st


def _bn_state(C, dev):
    # one allocation for the four per-channel vectors (one caching-allocator call per BN layer instead of four)
    st = BNState()
    st.mean, st.invstd, st.scale, st.shift = torch.empty(4, C, device=dev).unbind(0)
    return st


def bn_finalize_pair(bn_a, stats_a, Ca, count_a, bn_b, stats_b, Cb, count_b):
    """Training-mode bn_finalize of two layers whose statistics are complete together (a block's bn1 and its
    downsample BN): with SyncBN one all-reduce for both (_allreduce_stats_pair), and both finalizes in one launch
    (scd_bn_finalize_n)."""
    sa, sb, nrep = _allreduce_stats_pair(stats_a, Ca, stats_b, Cb)
    sts, args = [], (L.BnFinArgs * 2)()
    for i, (bn, stats, C, count) in enumerate(((bn_a, sa, Ca, count_a), (bn_b, sb, Cb, count_b))):
        st = _bn_state(C, bn.weight.device)
        st.count = count * bn_sync_world()
        args[i] = L.BnFinArgs(ptr(stats), nrep, C, float(st.count), ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
                              ptr(bn.running_var), ptr(bn.num_batches_tracked), float(bn.momentum), float(bn.eps),
                              ptr(st.mean), ptr(st.invstd), ptr(st.scale), ptr(st.shift))
        sts.append(st)
    L.call("scd_bn_finalize_n", args, 2, stream())
    return sts[0], sts[1]


def bn_apply(y, st, relu, res=None, rst=None, out=None):
    C = y.shape[-1]
    if out is None:
        out = torch.empty_like(y)
    t0 = ClassTimer.begin()
    L.call("scd_bn_apply", dt(y), ptr(y), ptr(out), C, y.numel(), ptr(st.scale), ptr(st.shift), ptr(res),
           ptr(rst.scale) if rst is not None else 0, ptr(rst.shift) if rst is not None else 0, int(relu), stream())
    if t0 is not None:
        ClassTimer.end("bn", t0, y.numel() * y.element_size() * (3 if res is not None else 2))
    return out


def bn_backward(bn, st, dout, y, mask=None, dz_out=None, relu=False, stats=None):
    """Training BN backward: dgamma/dbeta accumulated into bn.weight.grad / bn.bias.grad, returns dy.
    relu=True: the layer is BN+ReLU and its ReLU mask is recomputed from y (no activation read);
    mask: the stored activation whose > 0 pattern is the ReLU mask (residual joins);
    stats: the backward sums already accumulated by the producing GEMM (take_bn_bwd_fused)."""
    C = y.shape[-1]
    rsc, rsh = (ptr(st.scale), ptr(st.shift)) if (relu and mask is None) else (0, 0)
    E = y.numel() * y.element_size()
    if stats is None:
        stats = bn_stats(bn, "bwd")
        t0 = ClassTimer.begin()
        L.call("scd_bn_bwd_reduce", dt(y), ptr(dout), ptr(mask), ptr(y), rsc, rsh, ptr(st.mean), ptr(st.invstd),
               C, y.numel(), ptr(stats), stream())
        if t0 is not None:
            ClassTimer.end("bn", t0, E * (3 if mask is not None else 2))
    coef = bn_backward_coef(bn, st, stats, C, grad_alpha(y))
    dy = torch.empty_like(y)
    t0 = ClassTimer.begin()
    L.call("scd_bn_bwd_apply", dt(y), ptr(dout), ptr(mask), ptr(y), rsc, rsh, ptr(coef), C, y.numel(), ptr(dy),
           ptr(dz_out), stream())
    if t0 is not None:
        ClassTimer.end("bn", t0, E * (3 + (mask is not None) + (dz_out is not None)))
    return dy


class BNPair:
    enabled = os.environ.get("SCD_BN_PAIR", "1") != "0"


def bn_backward_pair(bn_a, st_a, y_a, bn_b, st_b, y_b, dout, mask):
    """Two BN layers behind one residual join, out = relu(bn_a(y_a) + bn_b(y_b)) (BasicBlock / Bottleneck with a
    downsample, CornerPool merge + shortcut): their backward from the same dout and ReLU mask (the stored `out`),
    dout / mask read once per pass (scd_bn_bwd_reduce2 / scd_bn_bwd_apply2).  Returns (dy_a, dy_b), equal to two
    bn_backward calls."""
    if not BNPair.enabled:
        return (bn_backward(bn_a, st_a, dout, y_a, mask=mask), bn_backward(bn_b, st_b, dout, y_b, mask=mask))
    C = y_a.shape[-1]
    sa, sb = bn_stats(bn_a, "bwd"), bn_stats(bn_b, "bwd")
    alpha = grad_alpha(y_a)
    E = y_a.numel() * y_a.element_size()
    t0 = ClassTimer.begin()
    L.call("scd_bn_bwd_reduce2", dt(y_a), ptr(dout), ptr(mask), ptr(y_a), ptr(y_b), ptr(st_a.mean),
           ptr(st_a.invstd), ptr(st_b.mean), ptr(st_b.invstd), C, y_a.numel(), ptr(sa), ptr(sb), stream())
    if t0 is not None:
        ClassTimer.end("bn", t0, 4 * E)
    sa, sb, nrep = _allreduce_stats_pair(sa, C, sb, C)
    # both backward finalizes in one launch (scd_bn_bwd_finalize_n)
    ca, cb = torch.empty(2, 3 * C, device=sa.device).unbind(0)
    args = (L.BnBwdFinArgs * 2)()
    for i, (bn, st, stats, coef) in enumerate(((bn_a, st_a, sa, ca), (bn_b, st_b, sb, cb))):
        args[i] = L.BnBwdFinArgs(ptr(stats), nrep, C, float(st.count), ptr(bn.weight), ptr(st.mean), ptr(st.invstd),
                                 ptr(grad_of(bn.weight)), ptr(grad_of(bn.bias)), alpha / bn_sync_world(), ptr(coef))
    L.call("scd_bn_bwd_finalize_n", args, 2, stream())
    dya, dyb = torch.empty_like(y_a), torch.empty_like(y_b)
    t0 = ClassTimer.begin()
    L.call("scd_bn_bwd_apply2", dt(y_a), ptr(dout), ptr(mask), ptr(y_a), ptr(y_b), ptr(ca), ptr(cb), C, y_a.numel(),
           ptr(dya), ptr(dyb), stream())
    if t0 is not None:
        ClassTimer.end("bn", t0, 6 * E)
    return dya, dyb


def bn_backward_coef(bn, st, stats, C, alpha=1.0):
    """SyncBN all-reduce of the backward sums, dgamma/dbeta accumulation (times alpha: 1 / the fp16 loss scale)
    and the apply coefficients."""
    return _bn_bwd_finalize_launch(bn, st, stats, _allreduce_stats(stats, C), C, alpha)


def _bn_bwd_finalize_launch(bn, st, stats, nrep, C, alpha):
    coef = torch.empty(3 * C, device=stats.device)
    L.call("scd_bn_bwd_finalize", ptr(stats), nrep, C, float(st.count), ptr(bn.weight), ptr(st.mean),
           ptr(st.invstd), ptr(grad_of(bn.weight)), ptr(grad_of(bn.bias)), alpha / bn_sync_world(), ptr(coef),
           stream())
    return coef


def grad_of(p):
    """The parameter's .grad buffer (created zero if absent); kernels accumulate into it."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


# ------------------------------------------------------------------ misc layers

def im2col_stem(x, dtype, kh=7, kw=7, stride=2, pad=3, Kpad=64):
    _need_gpu(x)
    N, _, H, W = x.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    cols = torch.empty(N, Ho, Wo, Kpad, dtype=dtype, device=x.device)
    L.call("scd_im2col_stem", _DT[dtype], ptr(x.contiguous()), ptr(cols), N, H, W, Ho, Wo, kh, kw, stride, pad, Kpad,
           stream())
    return cols


def stem_direct_ok(x, dtype):
    """The direct stem kernels (bf16; Conv2d(1,64,7,s2,p3) with an output width that is a multiple of 128)."""
    N, _, H, W = x.shape
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    return dtype in HALF and Wo % 128 == 0 and Ho % 2 == 0


def stem_conv_fwd(x, wpk, stats=None):
    """Conv2d(1,64,7,s2,p3) of NCHW fp32 x -> (N,Ho,Wo,64) bf16 NHWC (+BN sums); wpk = pack_weight(w, bf16, 0, ldp=64)."""
    _need_gpu(x)
    N, _, H, W = x.shape
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    y = torch.empty(N, Ho, Wo, 64, dtype=wpk.dtype, device=x.device)
    L.call("scd_stem_conv_fwd", dt(wpk), ptr(x), ptr(wpk), ptr(y), ptr(stats), N, H, W, Ho, Wo, stream())
    return y


def stem_out_count(x):
    """Pixels of the stem conv output per channel (the BN count)."""
    H, W = x.shape[2], x.shape[3]
    return x.shape[0] * ((H + 6 - 7) // 2 + 1) * ((W + 6 - 7) // 2 + 1)


def stem_conv_wgrad(dy, x, dst, accumulate=True, ybn=None, coef=None):
    """dst (64,1,7,7) fp32 (+)= weight gradient of the stem conv from dy (N,Ho,Wo,64) bf16 and the input x.
    With coef (scd_bn_bwd_finalize coefficients) dy is the masked dz and the BN backward apply runs fused."""
    N, _, H, W = x.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    M = N * Ho * Wo
    ns = L.lib().scd_stem_conv_wgrad_nsplit(M)
    ws = torch.empty(ns * 64 * 64, dtype=torch.float32, device=dy.device)
    L.call("scd_stem_conv_wgrad", dt(dy), ptr(dy), ptr(ybn), ptr(coef), ptr(x), ptr(ws), ns, N, H, W, Ho, Wo,
           stream())
    L.call("scd_wgrad_reduce", ptr(ws), ns, 64, 1, 64, 0, 64, 49, 49, 1, 0, ptr(dst), int(accumulate), grad_alpha(dy),
           stream())


def stem_pool_fwd(y, st):
    N, H, W, C = y.shape
    Ho, Wo = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    out = torch.empty(N, Ho, Wo, C, dtype=y.dtype, device=y.device)
    am = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device=y.device)
    L.call("scd_stem_pool_fwd", dt(y), ptr(y), ptr(st.scale), ptr(st.shift), ptr(out), ptr(am), N, H, W, C, Ho, Wo,
           stream())
    return out, am


def stem_pool_bwd_bn(bn, dout, am, y, st):
    """MaxPool/ReLU backward of the stem fused with its BN backward reduction; returns (dz, coef):
    dgamma/dbeta are accumulated, coef = the apply coefficients for dy = a*dz + b*y + c."""
    N, H, W, C = y.shape
    dz = torch.empty_like(y)
    stats = bn_stats(bn, "bwd")
    L.call("scd_stem_pool_bwd_bn", dt(y), ptr(dout), ptr(am), ptr(y), ptr(st.scale), ptr(st.shift), ptr(st.mean),
           ptr(st.invstd), ptr(dz), ptr(stats), N, H, W, C, dout.shape[1], dout.shape[2], stream())
    return dz, bn_backward_coef(bn, st, stats, C, grad_alpha(y))


def stem_backward_fused(bn, dout, am, y, st, x, wpk, dst):
    """The stem's MaxPool / ReLU / BN / conv weight-gradient backward in one pass (scd_stem_bwd_fused): the BN
    backward sums (dgamma / dbeta accumulated, SyncBN all-reduce as bn_backward_coef) and dst (64,1,7,7) += the weight
    gradient a*T1 + b*W G + c*s; the full-resolution dz is never materialised."""
    N, C = y.shape[0], y.shape[3]
    H, W = x.shape[2], x.shape[3]
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    ns = L.lib().scd_stem_bwd_nsplit()
    ws = torch.empty(ns * 2 * 64 * 64, dtype=torch.float32, device=y.device)
    tg = torch.empty(2 * 64 * 64, dtype=torch.float32, device=y.device)
    stats = bn_stats(bn, "bwd")
    L.call("scd_stem_bwd_fused", dt(y), ptr(dout), ptr(am), ptr(y),
           ptr(st.scale), ptr(st.shift), ptr(st.mean), ptr(st.invstd), ptr(x), ptr(stats), ptr(ws), ns, ptr(tg), N, H,
           W, Ho, Wo, stream())
    alpha = grad_alpha(y)
    coef = bn_backward_coef(bn, st, stats, C, alpha)
    L.call("scd_stem_bwd_combine", dt(y), ptr(tg), ptr(wpk), ptr(coef), ptr(dst), 1, float(alpha), stream())


def stem_pool_bwd(dout, am, y, st):
    N, H, W, C = y.shape
    dz = torch.empty_like(y)
    L.call("scd_stem_pool_bwd", dt(y), ptr(dout), ptr(am), ptr(y), ptr(st.scale), ptr(st.shift), ptr(dz), N, H, W,
           C, dout.shape[1], dout.shape[2], stream())
    return dz


def cpool_fwd(x, direction, addend=None):
    """directional corner pool (NHWC); y = pool(x) + addend when given."""
    N, H, W, C = x.shape
    y = torch.empty_like(x)
    L.call("scd_cpool_fwd", dt(x), direction, ptr(x), ptr(addend), ptr(y), N, H, W, C, stream())
    return y


def cpool_bwd(x, dy, direction):
    N, H, W, C = x.shape
    dx = torch.empty_like(x)
    L.call("scd_cpool_bwd", dt(x), direction, ptr(x), ptr(dy), ptr(dx), N, H, W, C, stream())
    return dx


def adam_step(p, g, m, v, lr, beta1, beta2, eps, step, gscale=1.0):
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    L.call("scd_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr), float(beta1), float(beta2),
           float(eps), float(bc1), float(bc2), float(gscale), stream())


def optimizer_skip_word():
    """The device word the optimizer kernels test before updating: the peer-memory SyncBN error word when
    that path is on -- a failed call NaN-poisons its statistics, so that step's gradients must not reach the weights
    -- else None (no test)."""
    return _BNSync.peer.err if _BNSync.peer is not None else None


def adam_step_dev(p, g, m, v, hyper, beta1, beta2, eps, gscale=1.0, skip=None):
    """Adam with the step state on the device (hyper = {lr, step} fp64, step advanced on the stream); skip: a device
    int64 word, non-zero = leave everything unchanged."""
    L.call("scd_adam_step_dev", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(hyper), float(beta1), float(beta2),
           float(eps), float(gscale), ptr(skip) if skip is not None else None, stream())


def sgd_step_dev(p, g, buf, hyper, momentum, dampening, weight_decay, nesterov, gscale=1.0, skip=None):
    """torch.optim.SGD step over the flat buffer (networkFactory.py:84-89); hyper = {lr, step, initialised, snapshot}
    fp64 on the device (scd_sgd_step_dev reads and writes all four)."""
    if hyper.dtype != torch.float64 or hyper.numel() < 4 or not hyper.is_contiguous():
        raise RuntimeError("sgd_step_dev: hyper must be a contiguous fp64 tensor of at least 4 elements "
                           "{lr, step, initialised, snapshot}")
    _need_gpu(p)
    L.call("scd_sgd_step_dev", ptr(p), ptr(g), ptr(buf) if buf is not None else None, p.numel(), ptr(hyper),
           float(momentum), float(dampening), float(weight_decay), int(bool(nesterov)), float(gscale),
           ptr(skip) if skip is not None else None, stream())


def decode_topk(heat, offset, regr, K=100):
    """decodeCenterNet core: sigmoid -> 3x3 NMS -> top-K -> gather (centerNetOffset.py:219-251)."""
    _need_gpu(heat)
    N, _, H, W = heat.shape
    K = min(K, H * W)
    dev = heat.device
    scores = torch.empty(N, K, device=dev)
    inds = torch.empty(N, K, dtype=torch.int64, device=dev)
    ys = torch.empty_like(inds)
    xs = torch.empty_like(inds)
    od_off = offset.shape[1] if offset is not None else 0
    od_regr = regr.shape[1] if regr is not None else 0
    off_out = torch.empty(N, K, max(od_off, 1), device=dev)[:, :, :od_off]
    regr_out = torch.empty(N, K, max(od_regr, 1), device=dev)[:, :, :od_regr]
    ws = torch.empty(L.lib().scd_decode_workspace(N, H * W) // 4, device=dev)
    L.call("scd_decode_topk", ptr(heat.contiguous()), N, H, W, K,
           ptr(offset.contiguous()) if offset is not None else 0, od_off,
           ptr(regr.contiguous()) if regr is not None else 0, od_regr, ptr(scores), ptr(inds), ptr(ys), ptr(xs),
           ptr(off_out), ptr(regr_out), ptr(ws), stream())
    return scores, inds, ys, xs, (off_out if offset is not None else None), (regr_out if regr is not None else None)


def render_center_targets(locs, counts, size=128, threshold=0.5):
    """CenterNet targets on the GPU (scd_render_center_targets): locs (B,K,8) fp32 object rows, counts (B,)
    objects per tile -> [heat (B,1,size,size) f32, mask (B,K) bool, regr (B,K,6) f32, inds (B,K) i64], the
    dataset contract of scdx16p100.py:376-379 batched."""
    _need_gpu(locs)
    locs = locs.float().contiguous()
    counts = counts.to(device=locs.device, dtype=torch.int32).contiguous()
    B, K, _ = locs.shape
    dev = locs.device
    heat = torch.empty(B, 1, size, size, device=dev)
    mask = torch.empty(B, K, dtype=torch.bool, device=dev)
    regr = torch.empty(B, K, 6, device=dev)
    inds = torch.empty(B, K, dtype=torch.int64, device=dev)
    L.call("scd_render_center_targets", ptr(locs), ptr(counts), B, K, size, float(threshold), ptr(heat),
           ptr(mask), ptr(regr), ptr(inds), stream())
    return [heat, mask, regr, inds]



CEVAL_STREAMS = ("iou", "score", "ortho", "ioucenter", "iouoffsetwo", "iouoffset", "aemaj", "aemin", "aerad")
_CEVAL_STREAM_MASK = (0, 0, 1, 2, 3, 4, 1, 1, 1)


def center_eval(scores, cty, ctx, offset, regr, gt_regr, gt_loc, heatmap_size=128, threshold=0.3):
    """centerNetEvaluation's pair metrics on the GPU (scd_ceval_count + scd_ceval_emit): the nine masked_select
    streams of models/centerNetOffset.py:253-354 / evaluations/detection.py:11-180, in CEVAL_STREAMS order.
    gt_loc: heat indices (N,L) int64 or locs rows (N,L,>=2) float [x, y, ...] (the reference's ys[3] dim test,
    centerNetOffset.py:287-292).  One host read of the (N,5) per-image counts sizes the outputs."""
    _need_gpu(scores, cty, ctx, offset, regr, gt_regr, gt_loc)
    N, K = scores.shape
    L_ = gt_regr.shape[1]
    dev = scores.device
    scores = scores.float().contiguous()
    cty = cty.long().contiguous()
    ctx = ctx.long().contiguous()
    offset = offset.float().contiguous()
    regr = regr.float().contiguous()
    gt_regr = gt_regr.float().contiguous()
    if offset.shape != (N, K, 2) or regr.shape != (N, K, 4) or gt_regr.shape != (N, L_, 6):
        raise RuntimeError("center_eval: offset (N,K,2), regr (N,K,4), gt_regr (N,L,6) expected")
    if gt_loc.dim() == 2:
        loc_mode, loc_w, gt_loc = 0, 0, gt_loc.long().contiguous()
    else:
        loc_mode, loc_w, gt_loc = 1, gt_loc.shape[2], gt_loc.float().contiguous()
    if gt_loc.shape[:2] != (N, L_):
        raise RuntimeError("center_eval: ys[3] must be (N,L) or (N,L,w)")
    counts = torch.empty(N, 5, dtype=torch.int32, device=dev)
    args = (ptr(scores), ptr(cty), ptr(ctx), ptr(offset), ptr(regr), ptr(gt_regr), ptr(gt_loc), loc_mode, loc_w,
            N, K, L_, int(heatmap_size), float(threshold))
    L.call("scd_ceval_count", *args, ptr(counts), stream())
    totals = counts.sum(0).cpu().tolist()
    outs = [torch.empty(max(1, totals[m]), device=dev) for m in _CEVAL_STREAM_MASK]
    L.call("scd_ceval_emit", *args, ptr(counts), L.ptr_array([o.data_ptr() for o in outs]), stream())
    return [o[:totals[m]] for o, m in zip(outs, _CEVAL_STREAM_MASK)]


def center_eval_summary(streams, objnum, thresholds=(0.3, 0.5, 0.7, 0.9)):
    """expression()'s reductions (trainer/model/centerOffsetRes10.py:81-88; detection.py:183-230) on the GPU:
    returns (means[9] in CEVAL_STREAMS order, APs[len(thresholds)]) as Python floats."""
    _need_gpu(*streams)
    if len(streams) != 9:
        raise RuntimeError("center_eval_summary: nine streams expected")
    dev = streams[0].device
    streams = [s.float().contiguous() for s in streams]
    lens = (ctypes.c_long * 9)(*[s.numel() for s in streams])
    thr = torch.tensor(list(thresholds), dtype=torch.float32).to(dev)
    out = torch.zeros(9 + len(thresholds), dtype=torch.float64, device=dev)
    ws = torch.empty(max(8, L.lib().scd_ceval_summary_workspace(streams[0].numel())), dtype=torch.uint8, device=dev)
    L.call("scd_ceval_summary", L.ptr_array([s.data_ptr() for s in streams]), lens, int(objnum), ptr(thr),
           len(thresholds), ptr(out), ptr(ws), stream())
    vals = out.cpu().tolist()
    return vals[:9], vals[9:]


def augment_tiles(tiles, flips=None, jitter=None, noise=None, noise_sv=0.0, seed=0, out=None):
    """SCD.argumentation's sample half on the GPU (scd_augment_tiles; scdx16p100.py:416-441,
    argumentations.py:38-64): per tile optional x / y flip, normalize, * jitter factor, + noise * noise_sv.
    tiles (B,1,H,W) or (B,H,W) fp32; flips (B,2) bool/u8; jitter (B,) factors (1 + 0.05 g); noise (B,H,W)
    N(0,1) draws or None (device counter-based generator keyed by `seed`).  Returns a new tensor."""
    _need_gpu(tiles, flips, jitter, noise)
    shape = tiles.shape
    t = tiles.float().contiguous()
    B, H, W = shape[0], shape[-2], shape[-1]
    if t.numel() != B * H * W:
        raise RuntimeError("augment_tiles: one channel per tile expected")
    if out is None:
        out = torch.empty_like(t)
    f = flips.to(torch.uint8).contiguous() if flips is not None else None
    j = jitter.float().contiguous() if jitter is not None else None
    n = noise.float().contiguous() if noise is not None else None
    ws = torch.empty(L.lib().scd_augment_workspace(B), dtype=torch.uint8, device=t.device)
    L.call("scd_augment_tiles", ptr(t), ptr(out), B, H, W, ptr(f), ptr(j), ptr(n), float(noise_sv),
           int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(ws), stream())
    return out.view(shape)


def slide_tiles(rgb, tile, stride, clip_h, clip_v, pad_lr, pad_tb, fix):
    """test.py:19-87 on the GPU (scd_slide_tiles): RGB slide (H,W,C) uint8 -> (clip_h*clip_v, 1, tile, tile)
    normalised float32 clips, x-major."""
    _need_gpu(rgb)
    rgb = rgb.contiguous()
    if rgb.dtype != torch.uint8 or rgb.dim() != 3:
        raise RuntimeError("slide_tiles: (H, W, C) uint8 slide expected")
    H, W, C = rgb.shape
    T = clip_h * clip_v
    out = torch.empty(T, 1, tile, tile, device=rgb.device)
    ws = torch.empty(L.lib().scd_slide_workspace(T), dtype=torch.uint8, device=rgb.device)
    L.call("scd_slide_tiles", ptr(rgb), H, W, C, tile, stride, clip_h, clip_v, pad_lr, pad_tb, int(bool(fix)),
           ptr(out), ptr(ws), stream())
    return out


def slide_detections(decoded, stride, pad_lr, pad_tb, clip_v, threshold=0.3):
    """test.py:104-135 on the GPU (scd_slide_detections): decoded (10, T, K) Wrapper stack -> (xy (n,2) int32,
    ratio (n,) float64) in the reference's order; one host read of the count."""
    _need_gpu(decoded)
    d = decoded.float().contiguous()
    _, T, K = d.shape
    xy = torch.empty(T * K, 2, dtype=torch.int32, device=d.device)
    ratio = torch.empty(T * K, dtype=torch.float64, device=d.device)
    count = torch.empty(1, dtype=torch.int32, device=d.device)
    L.call("scd_slide_detections", ptr(d), T, K, stride, pad_lr, pad_tb, clip_v, float(threshold), ptr(xy),
           ptr(ratio), ptr(count), stream())
    n = int(count.item())
    return xy[:n], ratio[:n]
