"""Multi-GPU plumbing for the sharded episode engine (one process per GPU).

Episodes shard across ranks with no data-path collective: rank r owns its own graph
pool, replay ring and RNG stream (seed + r).  Training has one exchange step, the
gradient all-reduce of the flat 58,425-float buffer (233.7 KB) per optimiser step over
RCCL (torch.distributed backend "nccl" on ROCm); the average is folded into the Adam
kernel (grad_scale = 1/world), so parameters stay bit-identical on every rank.
"""
import torch
import torch.distributed as dist


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def rank_seed(seed, rank):
    """Per-rank stream key (Philox-style key = (seed, rank))."""
    return int(seed) * 1000003 + int(rank)


def allreduce_gradients(grad, group=None):
    """Sum the flat gradient over ranks in place; returns the scale the optimiser applies
    (1/world) so that the update uses the mean gradient."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    world = dist.get_world_size(group)
    if world == 1:
        return 1.0
    dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


def allreduce_gradients_async(grad, group=None):
    """Start the sum all-reduce of the flat gradient (RCCL on its own stream) and return (work, scale): the
    caller issues independent work (the next minibatch's replay sample) and calls work.wait() -- which makes
    the current stream wait for the collective -- before the optimiser reads grad.  work is None without a
    process group (or at world size 1)."""
    if not (dist.is_available() and dist.is_initialized()):
        return None, 1.0
    world = dist.get_world_size(group)
    if world == 1:
        return None, 1.0
    return dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group, async_op=True), 1.0 / world


def broadcast_parameters(flat, src=0, group=None):
    """Make every rank start from rank src's parameters (DQN init)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)


def max_over_ranks(seconds, device=None):
    """bench.py timing: the job time is the slowest rank's."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def best_cut_over_ranks(best_cut, best_spins, device=None):
    """C5 best-cut search: MAX all-reduce of the per-rank best cut, then the winning rank
    broadcasts its spin vector."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return best_cut, best_spins
    rank, world = dist.get_rank(), dist.get_world_size()
    v = torch.tensor([float(best_cut), float(-rank)], dtype=torch.float64, device=device)
    allv = [torch.zeros_like(v) for _ in range(world)]
    dist.all_gather(allv, v)
    winner = max(range(world), key=lambda r: (allv[r][0].item(), allv[r][1].item()))
    spins = best_spins.clone()
    dist.broadcast(spins, src=winner)
    return allv[winner][0].item(), spins
