"""Data-parallel parity on the GPU (F7: SyncBN + DDP gradient averaging, world size 2)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("peer", [False, True])
def test_syncbn_ddp_world2_matches_reference(peer):
    """F7 with the SyncBN statistics through torch.distributed, and (peer) through the peer-memory one-shot
    all-reduce (scdhip/peer.py: IPC-mapped mailboxes, flag-synchronised kernel) -- same golden vectors."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
               PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "scd-resnet_amd")]),
               SCD_SYNCBN_PEER="1" if peer else "0")
    worker = os.path.join(REPO, "tests", "ddp_gpu_worker.py")
    procs = [subprocess.Popen([sys.executable, worker], env=dict(env, RANK=str(r), LOCAL_RANK="0"),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
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
        assert "OK rank" in o, o
    if peer:
        print([line for o in outs for line in o.splitlines() if "per call" in line])
