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


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    for bucket_mb in (25.0, 1e-5):                     # one bucket / one bucket per parameter
        check(rank, world, bucket_mb)
    dist.barrier()
    dist.destroy_process_group()
    print("OK rank", rank)


if __name__ == "__main__":
    main()
