"""RCCL on the box (VERDICT r05 missing #3: the nccl backend had never run): the one-GPU box cannot hold two RCCL
ranks (RCCL refuses a duplicate GPU, profiles/r05/rccl_same_device_probe.txt), so this runs the nccl process group
at world size 1 -- RCCL communicator setup and its collective kernels on device tensors, the calls DQN and bench.py
issue (all_reduce sync / async with work.wait(), MAX all-reduce, broadcast), then DQN.learn() inside the group
(rccl_world1_worker.py).  The multi-rank exchange itself is covered over gloo (test_parallel_gpu.py)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_nccl_backend_world1_collectives_and_learn():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_world1_worker.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert "RCCL_OK nccl 1" in out
