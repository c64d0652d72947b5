"""SyncBN statistics all-reduce over peer memory (peer.hip; networkFactory.py:128-133 SyncBatchNorm).

Every BN layer of a multi-GPU step all-reduces 2C fp64 sums twice (forward statistics, backward sums), each a small
message on the critical path.  PeerAllReduce maps every rank's fine-grained mailbox into every process (hipIpc
handles exchanged once through torch.distributed) and reduces with one kernel per call: write into every mailbox,
flag, wait, sum in rank order.  Opt-in (SCD_SYNCBN_PEER=auto: used when every rank can map every peer's mailbox,
``try_create``: checked collectively at set-up, with a probe all-reduce, else RCCL; SCD_SYNCBN_PEER=1: required),
because it takes the SyncBN statistics off the RCCL communicator, so FlatDDP can all-reduce its gradient buckets on
WORLD from inside the backward.  RCCL stays the default until this path has run on separate GPUs over xGMI (every
run so far had its ranks share one GPU).  Single node, <= MAX_RANKS ranks, eager steps (the epoch is a host
counter).

Late ranks: a rank whose host is seconds behind (a checkpoint write, validation, first-step allocation, a GC pause) is
waited for on the device, up to SCD_PEER_TIMEOUT_S (120 s).  Only a peer that never arrives is an error: the kernel then
records the failing epoch in a sticky device word, fills that call's data with NaN and posts a poison flag into every
peer's mailbox, so the peers fail at that call too instead of waiting out their own timeout (and poison theirs); every
later call re-posts the poison and returns NaN at once, so no replica silently continues on statistics reduced over a
subset of the ranks.  ``poll()`` -- called once per step by FlatDDP at the end of backward -- raises on the first step
whose copy of the error word is non-zero, and ``check()`` raises synchronously.
"""
import ctypes
import os

import torch
import torch.distributed as dist

from . import lib as L


def _gather(obj, group):
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


class PeerAllReduce:
    MAX_RANKS = 8          # one node: every peer's mailbox mapped into every process

    @classmethod
    def try_create(cls, group=None, cap=4096, timeout_s=None, probe_timeout_s=10.0):
        """Collective and failure-tolerant: every rank returns a working PeerAllReduce, or every rank returns None, with
        the reason (the first failing rank's).  The mailbox allocation, the IPC mapping of every peer's mailbox and one
        probe all-reduce (rank-ordered sum checked against its closed form, within probe_timeout_s) must succeed on
        every rank; the ranks agree on that through the group (all_gather_object) after each phase, so no rank is left
        waiting in a collective another rank has abandoned."""
        R = dist.get_world_size(group)
        if R > cls.MAX_RANKS:
            # every rank sees the same world size: all of them return here, none is left in a collective
            return None, "world %d > %d ranks (peer memory is single-node)" % (R, cls.MAX_RANKS)
        self = cls.__new__(cls)
        self._setup(group, cap, timeout_s)
        err = None
        try:
            self._alloc()
        except RuntimeError as e:
            err = "rank %d: mailbox allocation / IPC handle failed (%s)" % (self.rank, e)
        got = _gather((None, err) if err else (bytes(self._handle), None), group)
        if any(h is None for h, _ in got):
            self.close()
            return None, next(e for _, e in got if e)
        handles = [h for h, _ in got]
        try:
            self._map(handles)
        except RuntimeError as e:
            err = "rank %d: mapping a peer's mailbox failed (%s)" % (self.rank, e)
        errs = _gather(err, group)
        if any(errs):
            self.close()
            return None, next(e for e in errs if e)
        dist.barrier(group=group)           # every mailbox mapped before the first flag is written
        dev = torch.device("cuda", torch.cuda.current_device())
        v = torch.arange(16, dtype=torch.float64, device=dev) * (self.rank + 1) + 0.5
        self.epoch += 1
        L.call("scd_peer_allreduce_f64", v.data_ptr(), v.numel(), self.rank, self.R, self.boxes, self.cap, self.epoch,
               self.err.data_ptr(), max(1, int(probe_timeout_s * 1000)), torch.cuda.current_stream().cuda_stream)
        want = torch.arange(16, dtype=torch.float64) * (self.R * (self.R + 1) // 2) + 0.5 * self.R
        ok = int(self.err.item()) == 0 and torch.equal(v.cpu(), want)
        errs = _gather(None if ok else "rank %d: the probe all-reduce over peer memory failed (%s)" % (
            self.rank, "timed out" if int(self.err.item()) else "wrong sum"), group)
        if any(errs):
            self.close()
            return None, next(e for e in errs if e)
        return self, None

    def __init__(self, group=None, cap=4096, timeout_s=None):
        self._setup(group, cap, timeout_s)
        self._alloc()
        handles = _gather(bytes(self._handle), group)
        self._map(handles)
        dist.barrier(group=group)           # every mailbox mapped before the first flag is written

    def _setup(self, group, cap, timeout_s):
        self.group = group
        if timeout_s is None:
            timeout_s = float(os.environ.get("SCD_PEER_TIMEOUT_S", "120"))
        self.timeout_ms = max(1, min(int(timeout_s * 1000), 0xFFFFFFFF))
        self.R = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.R > self.MAX_RANKS:
            raise RuntimeError("PeerAllReduce: at most %d ranks (one node)" % self.MAX_RANKS)
        self.cap = cap
        self.own = None
        self.mapped = []
        dev = torch.device("cuda", torch.cuda.current_device())
        self.err = torch.zeros(1, dtype=torch.int64, device=dev)     # sticky: epoch of the first failed call
        self._err_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self._err_event = None
        self.epoch = 0

    def _alloc(self):
        lib = L.lib()
        nbytes = lib.scd_peer_mailbox_bytes(self.R, self.cap)
        own = ctypes.c_void_p()
        L.call("scd_peer_alloc", nbytes, ctypes.byref(own))
        self.own = own.value
        h = (ctypes.c_char * 64)()
        L.call("scd_peer_ipc_handle", self.own, h)
        self._handle = h

    def _map(self, handles):
        boxes = []
        for r, hb in enumerate(handles):
            if r == self.rank:
                boxes.append(self.own)
                continue
            p = ctypes.c_void_p()
            L.call("scd_peer_ipc_open", ctypes.create_string_buffer(hb, 64), ctypes.byref(p))
            self.mapped.append(p.value)
            boxes.append(p.value)
        self.boxes = (ctypes.c_void_p * self.R)(*boxes)
    def all_reduce(self, t):
        """In-place sum of the contiguous fp64 CUDA tensor t over the group (enqueued on the current stream)."""
        if t.dtype != torch.float64 or not t.is_contiguous() or t.numel() > self.cap:
            raise RuntimeError("PeerAllReduce: contiguous fp64, at most %d elements" % self.cap)
        self.epoch += 1
        L.call("scd_peer_allreduce_f64", t.data_ptr(), t.numel(), self.rank, self.R, self.boxes, self.cap,
               self.epoch, self.err.data_ptr(), self.timeout_ms, torch.cuda.current_stream().cuda_stream)

    def _raise(self, epoch):
        raise RuntimeError("PeerAllReduce: rank %d waited %.1f s for a peer's flag of call %d; SyncBN statistics "
                           "from that call on are not reduced" % (self.rank, self.timeout_ms / 1e3, epoch))

    def poll(self):
        """Non-blocking: raise if the error word copied at the previous poll is set, then enqueue the next copy on
        the current stream (read at the next poll, once its event has completed).  Called once per step."""
        ev = self._err_event
        if ev is not None and ev.query():
            if int(self._err_host[0]):
                self._raise(int(self._err_host[0]))
            ev = None
        if ev is None:
            self._err_host.copy_(self.err, non_blocking=True)
            self._err_event = torch.cuda.Event()
            self._err_event.record()

    def check(self):
        """Raise if any call so far timed out waiting for a peer (synchronises)."""
        e = int(self.err.item())
        if e:
            self._raise(e)

    def close(self):
        torch.cuda.synchronize()
        for p in self.mapped:
            L.lib().scd_peer_ipc_close(p)
        self.mapped = []
        if self.own:
            L.lib().scd_peer_free(self.own)
            self.own = None
