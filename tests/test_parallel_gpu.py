"""Multi-rank DQN training on the GPU: two ranks (gloo, both on GPU 0 -- the one-GPU box
rehearsal of the RCCL path the driver's multi-GPU bench takes), each with its own graphs, episodes, replay
and seed.  After a short learn() the parameters must be bitwise identical on every rank (one flat gradient
all-reduce per optimiser step, the mean folded into Adam), must have moved from the broadcast initial
weights, and every rank must have taken the same number of gradient steps.  The worker also checks the
exchange of the first three gradient steps: reduced buffer == rank-order sum of the local gradients, scale
1/world, and Adam's first moment moved by (1 - beta1)(mean gradient - m) (see dist_train_worker.py)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(worker, world=2):
    port = str(_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, worker)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        assert p.returncode == 0, out[-3000:]
    return outs


def test_two_ranks_train_to_identical_parameters():
    world = 2
    outs = _run_ranks("dist_train_worker.py", world)
    ex = next(l for l in outs[0].splitlines() if l.startswith("EXCHANGE_OK")).split()
    assert int(ex[1]) == 3 and float(ex[2]) < 1e-5
    line = next(l for l in outs[0].splitlines() if l.startswith("DIST_OK"))
    parts = line.split(maxsplit=5)
    steps, diff, init_same, moved = int(parts[1]), float(parts[2]), float(parts[3]), float(parts[4])
    assert steps > 0
    assert init_same == 0.0      # rank 0's initial weights broadcast to every rank
    assert diff == 0.0           # identical updates on every rank
    assert moved > 0.0
    assert "True" in parts[5] and parts[5].count(str(steps)) >= world


def test_two_ranks_evaluate_once_per_crossing():
    """learn() with evaluations at two ranks, every vector step crossing a test point (B x world > test_frequency,
    configs[3]'s regime at 8 GPUs): exactly one evaluation per crossing for the job, dealt round-robin to the ranks,
    the same test scores recorded on every rank, the `_best` checkpoint reproducing the best score, and no host
    synchronisation in learn()'s steady state (torch sync-debug mode "error", no eco_check_errors call;
    dist_eval_worker.py)."""
    outs = _run_ranks("dist_eval_worker.py", 2)
    line = next(l for l in outs[0].splitlines() if l.startswith("EVAL_OK"))
    assert int(line.split()[1]) > 4
