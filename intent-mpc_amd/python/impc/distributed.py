"""Multi-GPU plumbing for the batched solve: one process per GPU, independent QPs per rank.

The path shards by planning instance: every rank owns whole instances (all of an
instance's intent hypotheses stay on one device), so the solve itself needs no collective.  The
only exchange is the gather of the per-QP result records (instance, hypothesis, objective,
status, iterations) that the hypothesis selection consumes, plus the max-over-ranks timing of
bench.py.  torch.distributed is the transport (RCCL over xGMI with backend "nccl" on MI355X,
gloo in the CPU tests).
"""
import os

import numpy as np

RECORD_FIELDS = ("rank", "inst", "hyp", "obj", "status", "iter")


def env():
    """(rank, local_rank, world) from the torchrun environment (1 process = 1 GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def rank_seed(base, rank):
    """Seed of a rank's synthetic instances: disjoint streams, identical for a given rank
    whatever the world size (weak scaling: per-rank work is fixed)."""
    return base + 7919 * rank


def init(backend, local_rank):
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
    return dist


def _device(dist):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def max_over_ranks(dist, value):
    """Max of a float over all ranks (the timed region ends when the slowest rank ends)."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_records(rank, inst, hyp, info):
    """[B, 6] float64 records of one rank's QPs (RECORD_FIELDS order)."""
    rec = np.zeros((len(inst), len(RECORD_FIELDS)))
    rec[:, 0] = rank
    rec[:, 1] = inst
    rec[:, 2] = hyp
    rec[:, 3] = info["obj_val"]
    rec[:, 4] = info["status_val"]
    rec[:, 5] = info["iter"]
    return rec


def gather_records(dist, rec):
    """All-gather of every rank's records (equal counts per rank: weak scaling)."""
    if dist is None:
        return rec
    import torch
    local = torch.as_tensor(np.ascontiguousarray(rec), dtype=torch.float64).to(_device(dist))
    out = [torch.empty_like(local) for _ in range(dist.get_world_size())]
    dist.all_gather(out, local)
    return torch.cat(out).cpu().numpy()

