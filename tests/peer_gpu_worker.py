"""One rank of the peer-memory SyncBN latency/late-rank test (scdhip/peer.py), 2 ranks sharing cuda:0 over gloo.
Phase 1: rank 1 reaches its call 2 s late on the host -- rank 0's kernel waits on the device and both get the sum.
Phase 2 (a second mailbox with a 0.3 s timeout): rank 1 is 2 s late again -- rank 0 times out, its data become NaN,
its error is sticky (the next call returns at once with NaN data), poll() raises on the step after and check() raises;
rank 0 poisoned its flag in rank 1's mailbox, so rank 1 fails at once when it arrives (no second timeout), with NaN
data and the same failing call (ADVICE r3 peer.hip:36)."""
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
    took = time.perf_counter() - t0
    assert int(peer.err.item()) == 1, peer.err              # call 1 failed on both ranks
    assert torch.isnan(v).all(), "a failed call leaves NaN, not a partial sum"
    if rank == 1:
        assert took < 0.25, took                            # the poison ended the wait: no timeout of its own
    v2 = torch.ones(8, dtype=torch.float64, device=dev)
    t1 = time.perf_counter()
    peer.all_reduce(v2)                                     # sticky: no wait, NaN data
    torch.cuda.synchronize()
    assert time.perf_counter() - t1 < 0.25 and torch.isnan(v2).all()
    peer.poll()                                             # enqueues the copy of the error word
    torch.cuda.synchronize()
    try:
        peer.poll()
        raise AssertionError("poll() did not raise")
    except RuntimeError as e:
        assert "call 1" in str(e), e
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
