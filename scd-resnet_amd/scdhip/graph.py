"""The training step as a replayed HIP graph (networkFactory.py:257-263: zero_grad, forward, CenterNetLoss,
backward, Adam).

One eager step issues ~200 kernel launches from Python through ctypes (~4 ms of host time per Res10 B=32 step,
tools/host_overhead.py); the GPU only stays ahead because the kernels are longer.  ``StepGraph`` runs the first
``warmup`` calls eagerly (they create every persistent buffer: packed-operand plan, BN statistics, flat gradients,
the side stream), then captures the next call's step with ``torch.cuda.graph`` (HIP stream capture: the
weight-gradient side stream joins the capture through its event waits, the caching allocator serves the step's
activations from the graph's private pool) and replays it -- one ``hipGraphLaunch`` per step from then on.

What keeps a replayed step identical to an eager one:
  * every kernel takes device pointers only; per-step host scalars live in device memory (FlatAdam's {lr, step},
    ``scd_adam_step_dev``; the BN / loss / heads accumulators are re-zeroed by the kernels that consume them);
  * the step's inputs are the captured tensors: a call with new batch tensors copies them in first (bench.py
    captures its resident batch and passes nothing);
  * ``optimizer.sync_lr()`` before each replay carries setLearningRate changes, and the host step mirror is
    advanced per replay.
Multi-rank runs stay eager (a captured RCCL collective is not exercised on a one-GPU box).

``copies=2`` captures the step twice (independent private pools) and alternates the two graphs, so the HIP
events bench.py records around the dominant kernel inside each graph (``ops.LaunchTimer``) are read for replay
i while replay i+1 is already queued -- the timed region never waits for the host.
"""
import torch

from . import ops


def _tensors(obj):
    if torch.is_tensor(obj):
        return [obj]
    if isinstance(obj, (list, tuple)):
        return [t for o in obj for t in _tensors(o)]
    if isinstance(obj, dict):
        return [t for o in obj.values() for t in _tensors(o)]
    return []


class StepGraph:
    def __init__(self, fn, optimizer=None, warmup=2, copies=1):
        self.fn = fn
        self.optimizer = optimizer
        self.warmup = max(1, int(warmup))
        self.copies = max(1, int(copies))
        self.calls = 0
        self.graphs = []
        self.outputs = []
        self.pairs = []            # per graph: LaunchTimer pairs captured in it
        self.pending = []          # per graph: its last replay's pairs are not read yet
        self.static_args = None
        self._next = 0
        self._side = None

    # ---- eager phase
    def _eager(self, args):
        if self._side is None:
            self._side = torch.cuda.Stream()
        cur = torch.cuda.current_stream()
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            out = self.fn(*args)
        cur.wait_stream(self._side)
        return out

    # ---- capture
    def _capture(self, args):
        if args:
            self.static_args = tuple(_clone(a) for a in args)
        else:
            self.static_args = ()
        if self.optimizer is not None:
            self.optimizer.sync_lr()        # the lr is device state the captured Adam reads; set it outside capture
        torch.cuda.synchronize()
        host_step = getattr(self.optimizer, "_step", None)
        for _ in range(self.copies):
            g = torch.cuda.CUDAGraph()
            ops.LaunchTimer.take_captured()
            with torch.cuda.graph(g):
                out = self.fn(*self.static_args)
            self.graphs.append(g)
            self.outputs.append(out)
            self.pairs.append(ops.LaunchTimer.take_captured())
            self.pending.append(False)
            if host_step is not None:
                self.optimizer._step = host_step      # capture records the step, it does not run it
        torch.cuda.synchronize()

    def _copy_in(self, args):
        for dst, src in zip(_tensors(self.static_args), _tensors(args)):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)

    def __call__(self, *args):
        self.calls += 1
        if self.calls <= self.warmup:
            return self._eager(args)
        if not self.graphs:
            self._capture(args)
        elif args:
            self._copy_in(args)
        i = self._next
        self._next = (self._next + 1) % len(self.graphs)
        if self.pending[i]:
            ops.LaunchTimer.harvest(self.pairs[i])
            self.pending[i] = False
        if self.optimizer is not None:
            self.optimizer.sync_lr()
        self.graphs[i].replay()
        if self.optimizer is not None and hasattr(self.optimizer, "_step"):
            self.optimizer._step += 1
        self.pending[i] = bool(self.pairs[i])
        return self.outputs[i]

    def finish(self):
        """Read every outstanding graph-recorded timing (waits for the replays that recorded them)."""
        for i, p in enumerate(self.pending):
            if p:
                ops.LaunchTimer.harvest(self.pairs[i])
                self.pending[i] = False


def _clone(obj):
    if torch.is_tensor(obj):
        return obj.clone()
    if isinstance(obj, (list, tuple)):
        return type(obj)(_clone(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _clone(v) for k, v in obj.items()}
    return obj
