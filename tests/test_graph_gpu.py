"""The training step replayed as a captured HIP graph (scdhip/graph.py) against the same steps issued eagerly.

Both runs start from the same hash-initialised Res10 (fp32 parity mode, B=2, 256^2) and take the same five
batches; the graph run captures its third step.  Losses and parameters after every step must agree with the
eager run to the run-to-run noise of the fp64-atomic BN statistics (1e-5 relative); a learning-rate change after
capture must reach the replayed Adam (lr 0 freezes the parameters exactly); graph-recorded HIP events time the
head GEMM inside the replays."""
import numpy as np
import pytest
import torch

from oracle import centernet as O
from oracle import targets as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(dtype=torch.float32):
    import trainer.model.centerOffsetRes10 as plugin
    entries, _ = O.model_spec(10)
    m = plugin.model(**plugin.modelParams)
    m.load_state_dict(O.hash_weights(entries))
    return m.to(DEV).train().set_compute_dtype(dtype), plugin


def _batches(n, B=2, S=256):
    return [(T.batch_inputs(100 + i, B, S).to(DEV), [y.to(DEV) for y in T.batch_targets(200 + i, B, S // 4)])
            for i in range(n)]


def _run(graph, batches, dtype=torch.float32):
    from scdhip.flat import FlatAdam
    from scdhip.graph import StepGraph
    m, plugin = _model(dtype)
    opt = FlatAdam(filter(lambda p: p.requires_grad, m.parameters()))

    def step(x, ys):
        opt.zero_grad()
        loss, _ = plugin.loss(m(x, decode=False), ys)
        loss = loss.mean()
        loss.backward()
        opt.step()
        return loss

    runner = StepGraph(step, optimizer=opt, warmup=2) if graph else step
    losses, params = [], []
    for x, ys in batches:
        losses.append(runner(x, ys).item())
        params.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu())
    return losses, params, m, opt, runner


def test_step_graph_matches_eager():
    batches = _batches(5)
    le, pe, _, _, _ = _run(False, batches)
    lg, pg, m, opt, runner = _run(True, batches)
    assert len(runner.graphs) == 1 and runner.calls == 5
    np.testing.assert_allclose(lg, le, rtol=1e-5)
    for i, (a, b) in enumerate(zip(pg, pe)):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-6, err_msg="params after step %d" % i)
    assert opt.state_dict()["step"] == 5
    np.testing.assert_allclose(opt._hyper.cpu().numpy(), [1e-3, 5.0])
    # the replay keeps training: learning rate 0 freezes the parameters exactly (Adam update = lr * ...)
    opt.param_groups[0]["lr"] = 0.0
    before = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    x, ys = batches[0]
    runner(x, ys)
    torch.cuda.synchronize()
    after = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(before, after)
    opt.param_groups[0]["lr"] = 1e-3
    runner(x, ys)
    torch.cuda.synchronize()
    assert not torch.equal(before, torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    assert opt.state_dict()["step"] == 7


def test_step_graph_new_batches_are_copied_in():
    """A call with different batch tensors runs on those values (copied into the captured inputs)."""
    batches = _batches(4)
    le, _, _, _, _ = _run(False, batches[:3] + [batches[1]])
    lg, _, _, _, _ = _run(True, batches[:3] + [batches[1]])
    np.testing.assert_allclose(lg, le, rtol=1e-5)


def test_graph_recorded_events_time_the_head_gemm():
    from scdhip import ops
    from scdhip.flat import FlatAdam
    from scdhip.graph import StepGraph
    m, plugin = _model(torch.bfloat16)
    opt = FlatAdam(filter(lambda p: p.requires_grad, m.parameters()))
    x, ys = _batches(1, B=4, S=512)[0]

    def step():
        opt.zero_grad()
        loss, _ = plugin.loss(m(x, decode=False), ys)
        loss.mean().backward()
        opt.step()

    ops.LaunchTimer.arm("heads_gemm")
    try:
        g = StepGraph(step, optimizer=opt, warmup=2, copies=2)
        for _ in range(4):
            g()
        torch.cuda.synchronize()
        g.finish()
        ops.LaunchTimer.reset()
        for _ in range(6):
            g()
        g.finish()
        ms, n = ops.LaunchTimer.mean_ms("heads_gemm")
    finally:
        ops.LaunchTimer.armed.discard("heads_gemm")
    assert n == 6
    assert 0.005 < ms < 5.0
