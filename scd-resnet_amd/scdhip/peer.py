"""SyncBN statistics all-reduce over peer memory (peer.hip; networkFactory.py:128-133 SyncBatchNorm).

Every BN layer of a multi-GPU step all-reduces 2C fp64 sums twice (forward statistics, backward sums), each a small
message on the critical path.  PeerAllReduce maps every rank's fine-grained mailbox into every process (hipIpc
handles exchanged once through torch.distributed) and reduces with one kernel per call: write into every mailbox,
flag, wait, sum in rank order.  Opt-in (ops.set_bn_sync(group, peer=True) or SCD_SYNCBN_PEER=1); RCCL stays the
default until an 8-GPU run has compared them.  Single node, <= 8 ranks, eager steps (the epoch is a host counter).

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


class PeerAllReduce:
    def __init__(self, group=None, cap=4096, timeout_s=None):
        self.group = group
        if timeout_s is None:
            timeout_s = float(os.environ.get("SCD_PEER_TIMEOUT_S", "120"))
        self.timeout_ms = max(1, min(int(timeout_s * 1000), 0xFFFFFFFF))
        self.R = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.R > 8:
            raise RuntimeError("PeerAllReduce: at most 8 ranks (one node)")
        self.cap = cap
        lib = L.lib()
        nbytes = lib.scd_peer_mailbox_bytes(self.R, cap)
        own = ctypes.c_void_p()
        L.call("scd_peer_alloc", nbytes, ctypes.byref(own))
        self.own = own.value
        h = (ctypes.c_char * 64)()
        L.call("scd_peer_ipc_handle", self.own, h)
        handles = [None] * self.R
        dist.all_gather_object(handles, bytes(h), group=group)
        self.mapped = []
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
        dev = torch.device("cuda", torch.cuda.current_device())
        self.err = torch.zeros(1, dtype=torch.int64, device=dev)     # sticky: epoch of the first failed call
        self._err_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self._err_event = None
        self.epoch = 0
        dist.barrier(group=group)           # every mailbox mapped before the first flag is written

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
