"""SyncBN statistics all-reduce over peer memory (peer.hip; networkFactory.py:128-133 SyncBatchNorm).

Every BN layer of a multi-GPU step all-reduces 2C fp64 sums twice (forward statistics, backward sums), each a small
message on the critical path.  PeerAllReduce maps every rank's fine-grained mailbox into every process (hipIpc
handles exchanged once through torch.distributed) and reduces with one kernel per call: write into every mailbox,
flag, wait, sum in rank order.  Opt-in (ops.set_bn_sync(group, peer=True) or SCD_SYNCBN_PEER=1); RCCL stays the
default until an 8-GPU run has compared them.  Single node, <= 8 ranks, eager steps (the epoch is a host counter).
"""
import ctypes

import torch
import torch.distributed as dist

from . import lib as L


class PeerAllReduce:
    def __init__(self, group=None, cap=4096):
        self.group = group
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
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.epoch = 0
        dist.barrier(group=group)           # every mailbox mapped before the first flag is written

    def all_reduce(self, t):
        """In-place sum of the contiguous fp64 CUDA tensor t over the group (enqueued on the current stream)."""
        if t.dtype != torch.float64 or not t.is_contiguous() or t.numel() > self.cap:
            raise RuntimeError("PeerAllReduce: contiguous fp64, at most %d elements" % self.cap)
        self.epoch += 1
        L.call("scd_peer_allreduce_f64", t.data_ptr(), t.numel(), self.rank, self.R, self.boxes, self.cap,
               self.epoch, self.err.data_ptr(), torch.cuda.current_stream().cuda_stream)

    def check(self):
        """Raise if any call so far timed out waiting for a peer (synchronises)."""
        if int(self.err.item()):
            raise RuntimeError("PeerAllReduce: a peer's flag did not arrive (rank %d)" % self.rank)

    def close(self):
        torch.cuda.synchronize()
        for p in self.mapped:
            L.lib().scd_peer_ipc_close(p)
        self.mapped = []
        if self.own:
            L.lib().scd_peer_free(self.own)
            self.own = None
