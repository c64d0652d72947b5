"""One rank of the bf16 data-parallel test: the performance-mode training step (bf16 compute, SyncBN on the
transport ops.setup_syncbn picks, FlatDDP gradient average, FlatAdam) at world size 2 on cuda:0 over gloo.

bf16 against the fp32 reference vectors is chaotic for a whole hash-initialised network (test_bf16_parity_gpu.py), so
this checks what data parallelism itself must guarantee, exactly: after each of 3 steps every rank holds bit-identical
averaged gradients, parameters, Adam moments and BN running statistics (the all-reduced sums and the AVG buckets give
every rank the same bits, so the replicas never drift) and every value is finite."""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _same_on_all_ranks(t, what):
    """Every rank's copy of `t` (flattened) is bit-identical to rank 0's."""
    t = t.detach().reshape(-1).contiguous()
    raw = t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int64)
    got = [torch.empty_like(raw).cpu() for _ in range(dist.get_world_size())]
    dist.all_gather(got, raw.cpu())
    for r, g in enumerate(got):
        assert torch.equal(g, got[0]), (what, r, int((g != got[0]).sum()))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import trainer.model.centerOffsetRes10 as plugin
    from oracle import centernet as O
    from oracle import targets as T
    from scdhip import ops
    from scdhip.flat import FlatAdam, FlatDDP

    entries, _ = O.model_spec(10)
    m = plugin.model(**plugin.modelParams)
    m.load_state_dict(O.hash_weights(entries))
    m = m.cuda().train().set_compute_dtype(torch.bfloat16)
    logs = []
    mode = ops.setup_syncbn(log=logs.append)
    print("rank %d: %s" % (rank, logs[0]), flush=True)
    ddp = FlatDDP(m)
    opt = FlatAdam(m.parameters())
    B = 4                                              # images per rank, 256 x 256
    x = T.batch_inputs(61, B * world, 256)[B * rank:B * (rank + 1)].cuda()
    ys = [y[B * rank:B * (rank + 1)].cuda() for y in T.batch_targets(62, B * world, 64)]
    losses = []
    for step in range(3):
        opt.zero_grad()
        loss, _ = plugin.loss(ddp(x, decode=False), ys)
        loss.mean().backward()
        torch.cuda.synchronize()
        assert torch.isfinite(loss).all(), step
        flat = ddp.flat
        assert torch.isfinite(flat.grad).all(), step
        _same_on_all_ranks(flat.grad, "averaged gradient, step %d" % step)
        loss_sum = torch.tensor([loss.mean().item()], dtype=torch.float64)
        dist.all_reduce(loss_sum)
        losses.append(loss_sum.item() / world)
        opt.step()
        torch.cuda.synchronize()
        _same_on_all_ranks(flat.data, "parameters after step %d" % step)
        _same_on_all_ranks(opt._m, "Adam first moment after step %d" % step)
        _same_on_all_ranks(opt._v, "Adam second moment after step %d" % step)
    for k, b in m.named_buffers():
        if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
            _same_on_all_ranks(b, k)
    print("rank %d: syncbn %s, bf16, losses %s" % (rank, mode, ["%.4f" % v for v in losses]), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    print("OK rank", rank)


if __name__ == "__main__":
    sys.exit(main())
