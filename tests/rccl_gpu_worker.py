"""The RCCL code path at world size 1 (one GPU box): init_process_group("nccl") with device_id, and FlatDDP steps with
every collective forced on -- buckets all-reduced with ReduceOp.AVG from the weight-gradient side stream, async
work.wait(), the buffer broadcast -- compared with the same step without any of it, for both SyncBN group policies
(ops.syncbn_group): WORLD shared with the buckets (the default: every bucket at the end of the backward) and a group of
its own (SCD_SYNCBN_OWN_GROUP=1: buckets from inside the backward).  Launched by tests/test_ddp_gpu.py with
MASTER_ADDR / MASTER_PORT set."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    import trainer.model.centerOffsetRes10 as plugin
    from oracle import centernet as O
    from oracle import targets as T
    from scdhip import ops
    from scdhip.flat import FlatDDP

    entries, _ = O.model_spec(10)
    state = O.hash_weights(entries)
    x = T.batch_inputs(8, 2, 128).to(dev)
    ys = [y.to(dev) for y in T.batch_targets(9, 2, 32)]

    def make():
        m = plugin.model(**plugin.modelParams)
        m.load_state_dict(state)
        return m.to(dev).train().set_compute_dtype(torch.float32)

    def step(net, core):
        for p in core.parameters():
            if p.grad is not None:
                p.grad.zero_()
        loss, _ = plugin.loss(net(x, decode=False), ys)
        loss.mean().backward()
        torch.cuda.synchronize()
        return loss.item(), {k: p.grad.detach().double().cpu() for k, p in core.named_parameters()}

    # plain: no process group in the step
    ref_m = make()
    ref_loss, ref_g = step(ref_m, ref_m)

    worst = 0.0
    for policy in ("world", "own"):
        if policy == "own":
            os.environ["SCD_SYNCBN_OWN_GROUP"] = "1"
        bn_group = ops.syncbn_group()
        os.environ.pop("SCD_SYNCBN_OWN_GROUP", None)
        ops.set_bn_sync(bn_group)
        assert ops.bn_sync_group() is bn_group and (bn_group is dist.group.WORLD) == (policy == "world")
        m = make()
        ddp = FlatDDP(m, force_collectives=True)
        assert ddp._use_avg and ddp._comm and ddp.overlap_buckets() == (policy == "own")
        for it in range(2):          # the second backward launches the head bucket from inside backward (own group)
            loss, g = step(ddp, m)
            assert abs(loss - ref_loss) <= 1e-6 * abs(ref_loss), (policy, it, loss, ref_loss)
            for k, r in ref_g.items():
                e = (g[k] - r).norm().item() / max(r.norm().item(), 1e-30)
                worst = max(worst, e)
                # the collectives themselves are exact at world 1 (AVG of one rank); what differs is the SyncBN
                # statistics' replica collapse (sequential fp64) against the local finalize's fp64 wave tree --
                # rounding only
                assert e <= 1e-6, (policy, it, k, e)
            if it == 0 and policy == "world":
                # BN running statistics after one forward each (SyncBN count = local count at world 1)
                rs = ref_m.state_dict()
                for k, v in m.state_dict().items():
                    np.testing.assert_allclose(v.double().cpu().numpy(), rs[k].double().cpu().numpy(), rtol=1e-6,
                                               atol=1e-7, err_msg=k)
        if policy == "own":
            assert ddp.early_launches >= 1, ddp.early_launches
        else:
            assert ddp.early_launches == 0, ddp.early_launches
        ops.set_bn_sync(None)
    dist.destroy_process_group()
    print("OK rccl world1: loss %.6f, worst normwise gradient difference %.2e, %d early bucket launches, %d buckets"
          % (loss, worst, ddp.early_launches, len(ddp._buckets)))


if __name__ == "__main__":
    sys.exit(main())
