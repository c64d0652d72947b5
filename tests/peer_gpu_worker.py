"""One rank of the peer-memory SyncBN latency/late-rank test (scdhip/peer.py), 2 ranks sharing cuda:0 over gloo.
Phase 1: rank 1 reaches its call 2 s late on the host -- rank 0's kernel waits on the device and both get the sum.
Phase 2 (a second mailbox with a 0.3 s timeout): rank 1 is 2 s late again -- rank 0 times out, its error is sticky
(the next call is a no-op that returns at once), poll() raises on the step after and check() raises; rank 1 still
gets the correct sum (rank 0's data and flag were posted before it waited) and then times out on rank 0's missing
second flag."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from scdhip import ops
    from scdhip.peer import PeerAllReduce
    dev = torch.device("cuda", 0)
    ar = torch.arange(1024, dtype=torch.float64, device=dev)
    want = (ar * 1 + 0.1) + (ar * 2 + 0.1)          # the rank-ordered sum: the kernel's exact bits on every rank

    # phase 1: a late rank is not an error
    peer = PeerAllReduce(ops.new_bn_group())
    v = torch.arange(1024, dtype=torch.float64, device=dev) * (rank + 1) + 0.1
    if rank == 1:
        time.sleep(2.0)
    peer.all_reduce(v)
    torch.cuda.synchronize()
    peer.check()
    assert torch.equal(v, want), "phase 1 sum"
    peer.poll()
    torch.cuda.synchronize()
    peer.poll()
    dist.barrier()
    peer.close()

    # phase 2: a peer that does not come within the timeout
    peer = PeerAllReduce(ops.new_bn_group(), timeout_s=0.3)
    v = torch.arange(1024, dtype=torch.float64, device=dev) * (rank + 1) + 0.1
    if rank == 1:
        time.sleep(2.0)
    t0 = time.perf_counter()
    peer.all_reduce(v)
    torch.cuda.synchronize()
    if rank == 0:
        assert int(peer.err.item()) == 1, peer.err          # epoch 1 failed
        v2 = torch.ones(8, dtype=torch.float64, device=dev)
        t1 = time.perf_counter()
        peer.all_reduce(v2)                                 # sticky: no-op, no wait
        torch.cuda.synchronize()
        assert time.perf_counter() - t1 < 0.25 and torch.equal(v2, torch.ones_like(v2))
        peer.poll()                                         # enqueues the copy of the error word
        torch.cuda.synchronize()
        try:
            peer.poll()
            raise AssertionError("poll() did not raise")
        except RuntimeError as e:
            assert "call 1" in str(e), e
    else:
        assert torch.equal(v, want), "phase 2 sum on the late rank"
        assert int(peer.err.item()) == 0
        v2 = torch.ones(8, dtype=torch.float64, device=dev)
        peer.all_reduce(v2)                                 # rank 0 never posts call 2: times out
        torch.cuda.synchronize()
        assert int(peer.err.item()) == 2, peer.err
    try:
        peer.check()
        raise AssertionError("check() did not raise")
    except RuntimeError:
        pass
    print("rank %d phase 2 took %.2f s" % (rank, time.perf_counter() - t0))
    dist.barrier()
    peer.close()
    dist.destroy_process_group()
    print("OK rank", rank)


if __name__ == "__main__":
    sys.exit(main())
