"""One rank of the CPU (gloo) FlatDDP test -- launched by tests/test_host_cpu.py with RANK/WORLD_SIZE."""
import os

import torch
import torch.distributed as dist

from scdhip.flat import FlatDDP


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = torch.nn.Linear(8, 4)
        self.bn = torch.nn.BatchNorm1d(4)

    def forward(self, x):
        return {"y": self.bn(self.fc(x)), "aux": [self.fc.weight.sum()]}


class _LinearInto(torch.autograd.Function):
    """Like the model's block Functions: the weight gradient is written straight into weight.grad (the flat
    buffer view) and no gradient is returned for the weight, so no AccumulateGrad hook fires."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.b = b
        return x @ w.detach().t() + b.detach()

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        ctx.b.grad.add_(g.sum(0))
        w.grad.add_(g.t() @ x)
        return g @ w.detach(), None, None


class Block(torch.nn.Module):
    """A container whose forward runs while its leaf Linear's forward never does (the residual blocks)."""

    def __init__(self, n):
        super().__init__()
        self.fc = torch.nn.Linear(n, n)

    def forward(self, x):
        return torch.relu(_LinearInto.apply(x, self.fc.weight, self.fc.bias))


class Deep(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = torch.nn.Linear(8, 8)
        self.body = torch.nn.Sequential(Block(8), Block(8), Block(8))

    def forward(self, x):
        return self.body(self.stem(x))


def check_early_buckets(rank, world, expect_early=True):
    """Buckets are all-reduced from inside backward once the hook kinds are learned, also when the
    parameter-holding leaves never run forward (the hooks must sit on modules that run); with
    expect_early=False (SyncBN sharing FlatDDP's group) none is, and all still average correctly at the end."""
    torch.manual_seed(5 + rank)
    m = Deep()
    ddp = FlatDDP(m, bucket_mb=1e-5)
    ref = Deep()
    ref.load_state_dict({k[len("module."):]: v.clone() for k, v in ddp.state_dict().items()})
    g = torch.Generator().manual_seed(11)
    xfull = torch.randn(8, 8, generator=g)
    grads = []
    for r in range(world):
        ref.zero_grad(set_to_none=False)
        for p in ref.parameters():
            p.grad = torch.zeros_like(p)
        ref(xfull[4 * r:4 * r + 4]).square().mean().backward()
        grads.append({k: p.grad.clone() for k, p in ref.named_parameters()})
    for it in range(3):
        ddp.flat.grad.zero_()
        ddp(xfull[4 * rank:4 * rank + 4]).square().mean().backward()
        for k, p in m.named_parameters():
            exp = sum(gr[k] for gr in grads) / world
            assert torch.allclose(p.grad, exp, atol=1e-6), (it, k)
        if it > 0 and expect_early:
            # 6 body buckets (3 blocks x weight/bias) become ready inside backward; the stem's only at the end
            assert ddp.early_launches >= 6, ddp.early_launches
        if not expect_early:
            assert ddp.early_launches == 0 and not ddp.overlap_buckets(), ddp.early_launches


def check(rank, world, bucket_mb):
    torch.manual_seed(100 + rank)                      # different init per rank: the wrap must broadcast
    m = Toy()
    ddp = FlatDDP(m, bucket_mb=bucket_mb)
    if bucket_mb < 1:
        assert len(ddp._buckets) == 4
    ref = Toy()
    ref.load_state_dict({k[len("module."):]: v.clone() for k, v in ddp.state_dict().items()})
    assert all(k.startswith("module.") for k in ddp.state_dict())
    g = torch.Generator().manual_seed(7)
    xfull = torch.randn(8, 8, generator=g)
    x = xfull[4 * rank:4 * rank + 4]
    out = ddp(x)
    loss = out["y"].square().mean() + 0 * out["aux"][0]
    loss.backward()
    # reference: average of the per-shard gradients, each shard with its own BN batch statistics
    grads = []
    for r in range(world):
        ref.zero_grad()
        o = ref(xfull[4 * r:4 * r + 4])
        (o["y"].square().mean()).backward()
        grads.append({k: p.grad.clone() for k, p in ref.named_parameters()})
    expected = {}
    for k, p in m.named_parameters():
        exp = sum(gr[k] for gr in grads) / world
        expected[k] = exp
        assert torch.allclose(p.grad, exp, atol=1e-6), (k, p.grad, exp)
    # flat buffer views
    assert ddp.flat.grad.numel() == sum(p.numel() for p in m.parameters())
    assert m.fc.weight.grad.data_ptr() == ddp.flat.grad.data_ptr()
    # replicas identical after the initial broadcast
    w = m.fc.weight.detach().clone()
    dist.all_reduce(w)
    assert torch.allclose(w / world, m.fc.weight.detach())
    # later steps launch buckets during backward (after the first backward learned the hook kinds)
    for _ in range(2):
        ddp.flat.grad.zero_()
        out = ddp(x)
        (out["y"].square().mean() + 0 * out["aux"][0]).backward()
        for k, p in m.named_parameters():
            assert torch.allclose(p.grad, expected[k], atol=1e-6), (k, p.grad, expected[k])


def check_bn_group(rank, world):
    """SyncBN group policy (ops.syncbn_group; ADVICE r3 networkFactory.py:164).  Default: WORLD, shared with FlatDDP's
    buckets (one RCCL communicator and stream), so FlatDDP launches no bucket inside the backward and every bucket
    still averages correctly from the end-of-backward callback.  SCD_SYNCBN_OWN_GROUP=1: a group of its own, distinct
    from WORLD, and the buckets overlap the backward again (networkFactory.py:128-134)."""
    from scdhip import ops
    os.environ.pop("SCD_SYNCBN_OWN_GROUP", None)
    g = ops.syncbn_group()
    assert g is dist.group.WORLD
    ops.set_bn_sync(g)
    try:
        assert ops.bn_sync_shares_group(None)
        check_early_buckets(rank, world, expect_early=False)
    finally:
        ops.set_bn_sync(None)
    os.environ["SCD_SYNCBN_OWN_GROUP"] = "1"
    try:
        g = ops.syncbn_group()
        ops.set_bn_sync(g)
        assert ops.bn_sync_group() is g
        assert g is not dist.group.WORLD and g != dist.distributed_c10d._get_default_group()
        assert dist.get_world_size(g) == world and dist.get_rank(g) == rank
        ddp = FlatDDP(Toy())
        assert ddp.group is None or ddp.group is dist.group.WORLD
        assert not ops.bn_sync_shares_group(ddp.group) and ddp.overlap_buckets()
        assert ops.bn_sync_world() == world
        t = torch.full((4,), float(rank + 1), dtype=torch.float64)
        dist.all_reduce(t, group=g)
        assert torch.all(t == world * (world + 1) / 2)
        check_early_buckets(rank, world, expect_early=True)
    finally:
        os.environ.pop("SCD_SYNCBN_OWN_GROUP", None)
        ops.set_bn_sync(None)
    # setup_syncbn (networkFactory / bench): by default SyncBN runs on WORLD over torch.distributed (the peer-memory
    # path is opt-in) and the buckets wait for the end of the backward; with SCD_SYNCBN_PEER=auto and no GPU the peer
    # path is not tried either (every rank agrees, the reason is logged)
    if not torch.cuda.is_available():
        logs = []
        try:
            assert ops.setup_syncbn(log=logs.append) == "rccl-world"
            assert ops.bn_sync_mode() == "rccl-world" and "opt-in" in ops._BNSync.why, ops._BNSync.why
            assert len(logs) == 1 and "opt-in" in logs[0] and "end of the backward" in logs[0], logs
            os.environ["SCD_SYNCBN_PEER"] = "auto"
            assert ops.setup_syncbn(log=logs.append) == "rccl-world"
            assert ops._BNSync.why == "no GPU" and "no GPU" in logs[-1], (ops._BNSync.why, logs)
            os.environ["SCD_SYNCBN_OWN_GROUP"] = "1"
            assert ops.setup_syncbn() == "rccl-own"
        finally:
            os.environ.pop("SCD_SYNCBN_OWN_GROUP", None)
            os.environ.pop("SCD_SYNCBN_PEER", None)
            ops.set_bn_sync(None)
        assert ops.bn_sync_mode() == "off"
        # more ranks than one node's peer memory serves: try_create declines on every rank before any GPU call or
        # collective (it raised), so setup_syncbn falls back instead of crashing
        from scdhip.peer import PeerAllReduce
        saved = PeerAllReduce.MAX_RANKS
        PeerAllReduce.MAX_RANKS = world - 1
        try:
            peer, why = PeerAllReduce.try_create(dist.group.WORLD)
            assert peer is None and "world %d > %d" % (world, world - 1) in why, why
        finally:
            PeerAllReduce.MAX_RANKS = saved


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    for bucket_mb in (25.0, 1e-5):                     # one bucket / one bucket per parameter
        check(rank, world, bucket_mb)
    check_early_buckets(rank, world)
    check_bn_group(rank, world)
    dist.barrier()
    dist.destroy_process_group()
    print("OK rank", rank)


if __name__ == "__main__":
    main()
