"""Flat parameter / gradient buffers, the Adam step and data-parallel gradient averaging.

* ``FlatParams``: all trainable fp32 parameters of a model live in one contiguous device
  buffer and every ``param.grad`` is a view of one flat gradient buffer, so the optimizer
  is a single kernel launch and the DDP all-reduce is one (or a few bucketed) RCCL calls.
* ``FlatAdam``: torch.optim.Adam semantics (defaults lr=1e-3, betas (0.9,0.999), eps 1e-8,
  as the reference builds it without an lr, networkFactory.py:79-82) on scd_adam_step_dev;
  ``FlatSGD``: torch.optim.SGD (momentum 0.9, weight_decay 1e-4 in the reference, networkFactory.py:84-89) on
  scd_sgd_step_dev; ``param_groups`` keeps the reference's setLearningRate (networkFactory.py:273-276) working.
* ``FlatDDP``: replaces DistributedDataParallel (networkFactory.py:126-136): gradients are
  averaged across ranks with torch.distributed (RCCL over xGMI on MI355X, gloo in CPU tests)
  in ~25 MB buckets of the flat gradient, each launched asynchronously as soon as the backward
  pass has written all of its parameters' gradients (so RCCL runs on its own stream while the
  remaining backward kernels run), the rest from an autograd end-of-backward callback that then
  joins every bucket; BN buffers are broadcast from rank 0 before each forward (DDP
  broadcast_buffers=True, coalesced per dtype); state_dict keys keep the ``module.`` prefix.
"""
import contextlib
import weakref

import torch
import torch.distributed as dist

_REGISTRY = {}      # id(param) -> FlatParams
_LISTENERS = weakref.WeakSet()      # FlatDDP instances (world > 1) told when a Function wrote its gradients


def grads_ready(*modules):
    """Called by the scdhip autograd Functions (blocks.py) at the end of their backward: every parameter of
    `modules` has its gradient written (or its weight-gradient GEMM queued on the side stream), so a FlatDDP
    bucket holding them may be all-reduced now."""
    for d in list(_LISTENERS):
        d._written(modules)


class FlatParams:
    def __init__(self, params):
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        dev = params[0].device
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise ValueError("flat buffers need fp32 parameters on one device")
        self.params = params
        self.numel = sum(p.numel() for p in params)
        self.data = torch.empty(self.numel, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.offsets = []
        o = 0
        for p in params:
            n = p.numel()
            self.data[o:o + n].copy_(p.detach().reshape(-1))
            if p.grad is not None:
                self.grad[o:o + n].copy_(p.grad.reshape(-1))
            p.data = self.data[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
            self.offsets.append((o, n))
            o += n
        self.grad_scale = 1.0
        for p in params:
            _REGISTRY[id(p)] = self

    def rebind_grads(self):
        """Re-attach .grad views if something set them to None (e.g. Module.zero_grad())."""
        gbase = self.grad.data_ptr()
        for p, (o, n) in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != gbase + 4 * o:
                if g is not None:
                    self.grad[o:o + n].copy_(g.reshape(-1))
                else:
                    self.grad[o:o + n].zero_()
                p.grad = self.grad[o:o + n].view_as(p)

    def valid(self):
        base = self.data.data_ptr()
        return all(p.data_ptr() == base + 4 * o for p, (o, _) in zip(self.params, self.offsets))


def ensure_flat(params):
    params = [p for p in params if p.requires_grad]
    holders = {id(_REGISTRY.get(id(p))) for p in params}
    if len(holders) == 1 and id(params[0]) in _REGISTRY:
        fp = _REGISTRY[id(params[0])]
        if fp.valid() and len(fp.params) == len(params):
            return fp
    return FlatParams(params)


class _FlatOptimizer(torch.optim.Optimizer):
    """One launch per step over the flat fp32 buffer (FlatParams); {lr, step} live in device memory (``_hyper``,
    fp64) so a captured step graph replays with the current learning rate.  ``param_groups`` keeps the
    reference's setLearningRate working (networkFactory.py:273-276)."""

    def __init__(self, params, defaults):
        super(_FlatOptimizer, self).__init__(params, defaults)
        self._flat = None
        self._step = 0          # host mirror of the device step counter (state_dict)
        self._hyper = None      # device {lr, step} fp64
        self._dev_lr = None     # the lr last written to _hyper

    def _all_params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _new_state(self, fp):
        raise NotImplementedError

    def _hyper_init(self):
        """The device step state: {lr, step} (FlatSGD adds its buffer's initialised flag)."""
        return [self.param_groups[0]["lr"], float(self._step)]

    def flat(self):
        if self._flat is None or not self._flat.valid():
            self._flat = ensure_flat(self._all_params())
            self._new_state(self._flat)
            self._hyper = torch.tensor(self._hyper_init(), dtype=torch.float64, device=self._flat.data.device)
            self._dev_lr = self.param_groups[0]["lr"]
        return self._flat

    def sync_lr(self):
        """Write the param group's lr to the device state if setLearningRate changed it (a captured step graph
        calls this before each replay; the eager step does it itself)."""
        lr = self.param_groups[0]["lr"]
        # never recorded into a step graph: a captured fill would write this lr back on every replay, after the
        # replay-time sync (ADVICE r2 graph.py:66)
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return
        if self._hyper is not None and lr != self._dev_lr:
            self._hyper[0].fill_(lr)
            self._dev_lr = lr

    def zero_grad(self, set_to_none=False):
        fp = self.flat() if self._all_params()[0].is_cuda else None
        if fp is None:
            return super(_FlatOptimizer, self).zero_grad(set_to_none=set_to_none)
        fp.rebind_grads()
        fp.grad.zero_()

    def _begin_step(self):
        from . import ops
        ops.pack_end()          # the packed operands of this step go stale now
        fp = self.flat()
        fp.rebind_grads()
        self.sync_lr()
        self._step += 1
        return fp, self.param_groups[0]

    def _load_common(self, sd):
        self._step = sd["step"]
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
        if self._hyper is not None:
            self._hyper[:2].copy_(torch.tensor([self.param_groups[0]["lr"], float(self._step)], dtype=torch.float64))
            self._dev_lr = self.param_groups[0]["lr"]

    def _groups_sd(self):
        return [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]


class FlatAdam(_FlatOptimizer):
    """torch.optim.Adam (networkFactory.py:79-82: built without an lr, so lr 1e-3, betas (0.9, 0.999), eps 1e-8)
    on scd_adam_step_dev."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay != 0.0:
            raise NotImplementedError("weight decay is not used by the reference Adam")
        super(FlatAdam, self).__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._m = self._v = None

    def _new_state(self, fp):
        self._m = torch.zeros_like(fp.data)
        self._v = torch.zeros_like(fp.data)

    @torch.no_grad()
    def step(self, closure=None):
        from . import ops
        fp, g = self._begin_step()
        ops.adam_step_dev(fp.data, fp.grad, self._m, self._v, self._hyper, g["betas"][0], g["betas"][1], g["eps"],
                          gscale=fp.grad_scale, skip=ops.optimizer_skip_word())
        return None

    def state_dict(self):
        return {"step": self._step, "param_groups": self._groups_sd(),
                "exp_avg": None if self._m is None else self._m.cpu(),
                "exp_avg_sq": None if self._v is None else self._v.cpu()}

    def load_state_dict(self, sd):
        self._load_common(sd)
        if sd.get("exp_avg") is not None:
            self.flat()
            self._m.copy_(sd["exp_avg"])
            self._v.copy_(sd["exp_avg_sq"])


class FlatSGD(_FlatOptimizer):
    """torch.optim.SGD (networkFactory.py:84-89: lr = learningRate, momentum 0.9, weight_decay 1e-4) on
    scd_sgd_step_dev; dampening / nesterov as torch's."""

    def __init__(self, params, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super(FlatSGD, self).__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                                   weight_decay=weight_decay, nesterov=nesterov))
        self._buf = None

    def _new_state(self, fp):
        # a new buffer starts uninitialised: its first update copies d, as torch does for a parameter without a
        # momentum_buffer (hyper[2], the flag the kernel reads; _hyper_init), whatever the global step
        self._buf = torch.zeros_like(fp.data) if self.param_groups[0]["momentum"] != 0 else None

    def _hyper_init(self):
        return [self.param_groups[0]["lr"], float(self._step), 0.0, 0.0]

    @torch.no_grad()
    def step(self, closure=None):
        from . import ops
        fp, g = self._begin_step()
        ops.sgd_step_dev(fp.data, fp.grad, self._buf, self._hyper, g["momentum"], g["dampening"], g["weight_decay"],
                         g["nesterov"], gscale=fp.grad_scale, skip=ops.optimizer_skip_word())
        return None

    def state_dict(self):
        # torch emits a momentum_buffer only once a step has created it: the flat buffer exists from flat() on, so the
        # device flag hyper[2] (set by the first step or a loaded buffer) says whether it is one yet
        init = self._buf is not None and self._hyper is not None and float(self._hyper[2].item()) != 0.0
        return {"step": self._step, "param_groups": self._groups_sd(),
                "momentum_buffer": self._buf.cpu() if init else None}

    def load_state_dict(self, sd):
        buf = sd.get("momentum_buffer")
        if buf is not None and self.param_groups[0]["momentum"] == 0:
            raise ValueError("FlatSGD.load_state_dict: the state has a momentum_buffer but this optimizer has "
                             "momentum 0 (no buffer to load it into)")
        self._load_common(sd)
        self.flat()
        if buf is not None:
            self._buf.copy_(buf)
        elif self._buf is not None:
            self._buf.zero_()
        self._hyper[2].fill_(1.0 if buf is not None else 0.0)


class _EndOfBackward(torch.autograd.Function):
    """Identity on the model outputs whose backward queues the gradient all-reduce at the
    end of the backward pass (the hook torch's DDP reducer also uses)."""

    @staticmethod
    def forward(ctx, ddp, *xs):
        ctx.ddp = ddp
        return xs if len(xs) > 1 else xs[0]

    @staticmethod
    def backward(ctx, *gs):
        ddp = ctx.ddp
        if not ddp._queued:
            ddp._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(ddp._allreduce_grads)
        return (None,) + gs


class FlatDDP(torch.nn.Module):
    """DistributedDataParallel replacement: one process per GPU, grads averaged over the
    world (bucketed RCCL all-reduce of the flat gradient buffer, overlapped with backward).

    Gradient readiness: the model's blocks write parameter gradients straight into the flat buffer
    (no AccumulateGrad hooks fire) and say so at the end of their backward (``grads_ready``, which marks
    the parameters of the modules they name -- blocks, deconv+BN, heads, stem).  For other modules the
    leaf Conv2d/BatchNorm2d modules that hold the parameters
    never run their own forward (the block, deconv and head containers hand the weights to autograd
    Functions), so readiness is observed at whichever module's forward does run -- every module that
    holds parameters, directly or below it, gets a forward pre-hook that hooks its first grad-requiring
    input; the gradient w.r.t. a module's input is complete only after that module's backward has run,
    so the hook marks all of the module's (recursive) parameters ready.  Buckets are contiguous flat ranges of the parameters in
    reverse registration order (the order backward produces them, as torch DDP buckets them); a bucket
    whose parameters are all ready is all-reduced asynchronously (RCCL queues it behind the kernels
    already on the compute stream).  Parameters whose module input needs no gradient (the stem) are
    covered by the end-of-backward callback, which launches what is left in order and joins all
    buckets before the optimizer can run.  Parameters whose gradients torch's own AccumulateGrad
    writes (plain torch modules) may be accumulated after their module's input gradient exists:
    the first backward only learns which they are (post-accumulate hooks) and launches every bucket
    at the end; from then on those parameters are marked by their post-accumulate hook instead."""

    def __init__(self, module, process_group=None, broadcast_buffers=True, bucket_mb=25.0, tail_mb=2.0,
                 force_collectives=False):
        super(FlatDDP, self).__init__()
        self.module = module
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # force_collectives: run the whole exchange (hooks, bucket all-reduces from the side stream, waits, buffer
        # broadcasts) even in a world of one -- the RCCL path's test on a one-GPU box (tests/test_ddp_gpu.py)
        self._comm = dist.is_initialized() and (self.world > 1 or force_collectives)
        self.broadcast_buffers = broadcast_buffers
        self.flat = ensure_flat(module.parameters())
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) / 4))
        # the last bucket is only complete when the backward ends (stem), so it is never overlapped: keep it to the
        # parameters of the last few layers (<= tail_mb) and launch the rest of what would have been that bucket as
        # soon as its own parameters are ready
        self.tail_elems = max(1, int(tail_mb * (1 << 20) / 4))
        self._queued = False
        self._use_avg = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        self._engine = set()                  # ids of parameters written by torch's AccumulateGrad
        self._learned = False                 # one backward seen: early launches allowed
        self.early_launches = 0               # buckets launched from inside backward, last backward
        self._build_buckets()
        self._hooks = []
        if self._comm:
            for m in module.modules():
                if any(p.requires_grad for p in m.parameters()):
                    self._hooks.append(m.register_forward_pre_hook(self._pre_hook))
            for p in self.flat.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._acc_hook))
            _LISTENERS.add(self)
            # identical initial replicas (DDP broadcasts parameters from rank 0 at wrap time)
            dist.broadcast(self.flat.data, 0, group=process_group)
            self._sync_buffers()

    # ---- buckets
    def _build_buckets(self):
        fp = self.flat
        self._bucket_of = {}
        self._buckets = []                    # [lo, hi) flat ranges, in launch (reverse-parameter) order
        self._bucket_params = []
        lo = hi = None
        members = []
        for p, (o, n) in reversed(list(zip(fp.params, fp.offsets))):
            if hi is None:
                lo, hi = o, o + n
            elif o + n == lo and hi - o <= self.bucket_elems:
                lo = o
            else:
                self._buckets.append((lo, hi))
                self._bucket_params.append(members)
                lo, hi, members = o, o + n, []
            members.append(id(p))
        self._buckets.append((lo, hi))
        self._bucket_params.append(members)
        self._split_tail()
        for b, ms in enumerate(self._bucket_params):
            for pid in ms:
                self._bucket_of[pid] = b
        self._reset_step()

    def _split_tail(self):
        """Split the last bucket (launch order) so that its final part holds at most tail_elems of parameters."""
        lo, hi = self._buckets[-1]
        members = self._bucket_params[-1]
        K = len(members)
        if hi - lo <= self.tail_elems or K < 2:
            return
        span = {id(p): (o, o + n) for p, (o, n) in zip(self.flat.params, self.flat.offsets)}
        # members are in launch order (reverse parameter order): member K-1 sits at lo; the tail is the suffix
        # members[k:], occupying [lo, end of members[k])
        if span[members[K - 1]][1] - lo > self.tail_elems:
            return
        k = K - 1
        while k > 1 and span[members[k - 1]][1] - lo <= self.tail_elems:
            k -= 1
        split = span[members[k]][1]
        self._buckets[-1] = (split, hi)
        self._buckets.append((lo, split))
        self._bucket_params[-1] = members[:k]
        self._bucket_params.append(members[k:])

    def _reset_step(self):
        self._early = 0
        self._ready = set()
        self._pending = [len(ms) for ms in self._bucket_params]
        self._works = [None] * len(self._buckets)
        self._next = 0                        # buckets are launched in order: RCCL needs one order on all ranks

    def overlap_buckets(self):
        """Buckets may be all-reduced from inside the backward unless SyncBN all-reduces its statistics on the same
        group (ops.syncbn_group's default): on one RCCL communicator a bucket waits for the side stream's weight
        gradients, and every critical-path SyncBN collective issued after it would wait with it -- then all buckets
        go at the end of the backward, after the last SyncBN collective."""
        from . import ops
        return not ops.bn_sync_shares_group(self.group)

    def _launch_ready(self, final=False):
        if not final and not self.overlap_buckets():
            return
        while self._next < len(self._buckets) and (final or self._pending[self._next] == 0):
            b = self._next
            lo, hi = self._buckets[b]
            bucket = self.flat.grad[lo:hi]
            # weight gradients may be written on scdhip's side stream (ops.conv_wgrad): issue the collective
            # from that stream, ordered after both
            side = None
            if bucket.is_cuda:
                from . import ops
                side = ops.side_stream_for_comm(bucket.device)
            with torch.cuda.stream(side) if side is not None else _nullctx():
                if self._use_avg:
                    self._works[b] = dist.all_reduce(bucket, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
                else:
                    self._works[b] = dist.all_reduce(bucket, group=self.group, async_op=True)
            self._next += 1
            if not final:
                self._early += 1

    def _mark(self, pid):
        b = self._bucket_of.get(pid)
        if b is None or pid in self._ready:
            return
        self._ready.add(pid)
        self._pending[b] -= 1

    def _mark_ready(self, module):
        if not self._learned:
            return
        for p in module.parameters():
            if id(p) not in self._engine:
                self._mark(id(p))
        self._launch_ready()

    def _written(self, modules):
        if not self._comm:
            return
        for m in modules:
            for p in m.parameters():
                if id(p) not in self._engine:
                    self._mark(id(p))
        self._launch_ready()

    def _acc_hook(self, p):
        if not self._comm:
            return
        self._engine.add(id(p))
        if self._learned:
            self._mark(id(p))
            self._launch_ready()

    def _pre_hook(self, module, args):
        if not (self._comm and self.training and torch.is_grad_enabled()):
            return None
        for a in args:
            if torch.is_tensor(a) and a.requires_grad:
                a.register_hook(lambda g, m=module: self._mark_ready(m))
                break
        return None

    def _sync_buffers(self):
        bufs = list(self.module.buffers())
        if not bufs:
            return
        pg = self.group if self.group is not None else dist.distributed_c10d._get_default_group()
        coalesced = getattr(dist, "_broadcast_coalesced", None)
        if coalesced is not None:
            coalesced(pg, bufs, 256 << 20, 0)         # one broadcast per dtype (as torch DDP does)
        else:
            for b in bufs:
                dist.broadcast(b, 0, group=self.group)

    def _allreduce_grads(self):
        self._queued = False
        if not self._comm:
            return
        if self.flat.grad.is_cuda:
            # every gradient written on scdhip's side stream is ordered before the remaining buckets
            from . import ops
            ops.join_side_streams()
        self._launch_ready(final=True)
        self.early_launches = self._early
        for b, w in enumerate(self._works):
            w.wait()                                # NCCL: the compute stream waits; gloo: blocks
            if not self._use_avg:
                lo, hi = self._buckets[b]
                self.flat.grad[lo:hi].div_(self.world)
        self._learned = True
        self._reset_step()
        if self.flat.grad.is_cuda:
            from . import ops
            ops.bn_sync_poll()                      # peer-memory SyncBN: raise on a failed call (non-blocking)

    @contextlib.contextmanager
    def local_only(self):
        """Steps inside run this rank's shard with no collective at all (no gradient buckets, no buffer broadcast, no
        SyncBN): bench.py times them beside the data-parallel steps to separate the exchange's cost from the
        per-GPU work.  The replicas diverge meanwhile; broadcast the parameters again before training on."""
        from . import ops
        was = self._comm
        self._comm = False
        try:
            with ops.bn_sync_suspended():
                yield
        finally:
            self._comm = was
            self._reset_step()

    def forward(self, *args, **kwargs):
        if self._comm and self.broadcast_buffers and self.training:
            self._sync_buffers()
        if self._comm:
            self._reset_step()
        out = self.module(*args, **kwargs)
        if not torch.is_grad_enabled() or not self._comm:
            return out
        # route every differentiable output tensor through the end-of-backward hook
        flat, spec = _flatten(out)
        idx = [i for i, t in enumerate(flat) if torch.is_tensor(t) and t.requires_grad]
        if not idx:
            return out
        hooked = _EndOfBackward.apply(self, *[flat[i] for i in idx])
        if len(idx) == 1:
            hooked = (hooked,)
        for i, t in zip(idx, hooked):
            flat[i] = t
        return _unflatten(flat, spec)


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def _flatten(obj):
    if isinstance(obj, (list, tuple)):
        items, specs = [], []
        for o in obj:
            f, s = _flatten(o)
            items.extend(f)
            specs.append((len(f), s))
        return items, (type(obj), specs)
    if isinstance(obj, dict):
        items, specs = [], []
        for k, o in obj.items():
            f, s = _flatten(o)
            items.extend(f)
            specs.append((k, len(f), s))
        return items, (dict, specs)
    return [obj], None


def _unflatten(items, spec):
    if spec is None:
        return items[0]
    kind, specs = spec
    out, o = [], 0
    if kind is dict:
        d = {}
        for k, n, s in specs:
            d[k] = _unflatten(items[o:o + n], s)
            o += n
        return d
    for n, s in specs:
        out.append(_unflatten(items[o:o + n], s))
        o += n
    return kind(out)
