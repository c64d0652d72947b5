"""Data-parallel parity on the GPU (F7: SyncBN + DDP gradient averaging, world size 2)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(worker, world, **extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "scd-resnet_amd")]), **extra)
    worker = os.path.join(REPO, "tests", worker)
    procs = [subprocess.Popen([sys.executable, worker], env=dict(env, RANK=str(r), LOCAL_RANK="0"),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode()[-3000:])
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
    return outs


# the opt-in peer-memory transport at 4 and 8 ranks: 4-8 processes time-slicing ONE GPU while their peer kernels
# spin-wait can stall the card's queue scheduling (one 150-s timeout in round 6, otherwise 10-12 s per case), a
# property of the one-GPU rehearsal, not of the path; they run with SCD_TEST_PEER=1 (profiles/README.md records the runs)
_PEER_WIDE = pytest.mark.skipif(os.environ.get("SCD_TEST_PEER") != "1",
                                reason="peer transport at 4-8 ranks sharing one GPU: SCD_TEST_PEER=1")


@pytest.mark.parametrize("world,sync", [(2, "default"), (2, "peer"), (2, "own"), (4, "default"),
                                        pytest.param(4, "peer", marks=_PEER_WIDE), (8, "default"),
                                        pytest.param(8, "peer", marks=_PEER_WIDE)])
def test_syncbn_ddp_matches_reference(world, sync):
    """F7 (W=2), F7b (W=4) and F7c (W=8: the driver's scaling world size; tests/golden/make_golden_ddp4.py) against
    the reference's golden vectors, with each SyncBN transport: the default set-up (ops.setup_syncbn: torch.distributed
    on WORLD beside the gradient buckets, all at the end of the backward), the opt-in peer-memory statistics
    (SCD_SYNCBN_PEER=auto, scdhip/peer.py: the gradient buckets are all-reduced from inside the backward -- asserted)
    and a group of their own (SCD_SYNCBN_OWN_GROUP=1)."""
    env = {"default": dict(EXPECT_SYNCBN="rccl-world"),
           "peer": dict(SCD_SYNCBN_PEER="auto", EXPECT_SYNCBN="peer"),
           "own": dict(SCD_SYNCBN_OWN_GROUP="1", EXPECT_SYNCBN="rccl-own")}[sync]
    outs = _run("ddp_gpu_worker.py", world, **env)
    for o in outs:
        assert "OK rank" in o, o
    print([line for o in outs for line in o.splitlines() if "per call" in line or "worst" in line or "buckets" in line])


def test_rccl_world1_flatddp_syncbn():
    """The nccl (RCCL) backend executed: SyncBN on its own communicator, FlatDDP's AVG buckets from the side stream,
    async waits -- one step equal to the step without collectives (tests/rccl_gpu_worker.py)."""
    outs = _run("rccl_gpu_worker.py", 1)
    assert "OK rccl world1" in outs[0], outs[0]
    print([line for line in outs[0].splitlines() if "OK rccl" in line])


def test_peer_syncbn_late_rank_and_sticky_error():
    """A rank 2 s late on the host is waited for (no error); a peer missing past the timeout gives a sticky error that
    poll()/check() raise (tests/peer_gpu_worker.py; ADVICE r2 peer.hip:47)."""
    outs = _run("peer_gpu_worker.py", 2)
    for o in outs:
        assert "OK rank" in o, o


def test_bf16_ddp_replicas_stay_identical():
    """bf16 performance mode at world size 2 (nothing checked bf16 at world > 1): three training steps
    with SyncBN + FlatDDP + FlatAdam; every rank ends each step with bit-identical averaged gradients, parameters,
    Adam moments and BN running statistics, all finite (tests/ddp_bf16_gpu_worker.py)."""
    outs = _run("ddp_bf16_gpu_worker.py", 2, EXPECT_SYNCBN="rccl-world")
    for o in outs:
        assert "OK rank" in o, o
    print([line for o in outs for line in o.splitlines() if "losses" in line])
