"""Multi-GPU plumbing for the batched solve: one process per GPU, independent QPs per rank.

The path shards by planning instance: every rank owns whole instances (all of an
instance's intent hypotheses stay on one device), so the solve itself needs no collective.  The
only exchange is the gather of the per-QP result records (instance, hypothesis, objective,
status, iterations) that the hypothesis selection consumes, plus the max-over-ranks timing of
bench.py.

Transports: the device records move over RCCL/xGMI through the solver library's own
communicator (impc.Comm, include/impc_comm.h: one ncclAllGather of the packed impc_info
records), on the solver's HIP runtime -- a solver process never initialises the launching
framework's GPU runtime (PyTorch-ROCm bundles its own HIP runtime; two runtimes in one process
do not share the device).  torch.distributed runs on gloo (CPU) for the rendezvous, the RCCL
unique id, barriers and host-side reductions; the CPU tests run the same shard / gather code on
gloo alone.
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


def init(backend="gloo", local_rank=0):
    """torch.distributed process group for the host-side exchange (gloo: CPU only)."""
    import torch.distributed as dist
    if backend != "gloo":
        raise ValueError("solver processes use gloo for host traffic and impc.Comm (RCCL) for device records")
    dist.init_process_group("gloo")
    return dist


def make_comm(dist, ctx):
    """impc.Comm over all ranks: rank 0's RCCL unique id broadcast over the gloo group."""
    import impc
    import torch
    world = 1 if dist is None else dist.get_world_size()
    rank = 0 if dist is None else dist.get_rank()
    uid = torch.zeros(impc.COMM_ID_BYTES, dtype=torch.uint8)
    if rank == 0:
        uid[:] = torch.frombuffer(bytearray(impc.comm_unique_id()), dtype=torch.uint8)
    if dist is not None:
        dist.broadcast(uid, 0)
    return impc.Comm(ctx, uid.numpy().tobytes(), rank, world)


def _device(dist):
    import torch
    return torch.device("cpu")


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


def shard_plan(weights, world):
    """Contiguous ranges of planning instances per rank, balanced by weight (config 4
    shards by the summed constraint count, Sigma m, not by QP count).  Returns bounds [world + 1]:
    rank r owns instances [bounds[r], bounds[r + 1]).  Each cut is placed at the prefix-sum
    position closest to r * total / world, so no rank's load differs from the ideal share by more
    than one instance's weight."""
    w = np.asarray(weights, dtype=np.float64)
    c = np.concatenate([[0.0], np.cumsum(w)])
    total = c[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        j = int(np.searchsorted(c, target))
        j = min(max(j, 1), len(w))
        if j > 1 and abs(c[j - 1] - target) <= abs(c[j] - target):
            j -= 1
        bounds.append(max(j, bounds[-1]))
    bounds.append(len(w))
    return np.array(bounds, dtype=np.int64)


def equal_instance_bounds(instances, world):
    """Config 3 strong scaling: the fixed batch's planning instances in `world` contiguous ranges
    of equal size (+-1); every instance carries the same 8 hypothesis QPs, so equal instance counts
    are equal QP counts and equal constraint sums.  Returns bounds [world + 1]."""
    return np.linspace(0, int(instances), int(world) + 1).astype(np.int64)


def unpad(flat, counts):
    """Rank-ordered records from an all-gather of zero-padded blocks: flat [world * max, ...]
    (rank r's block at rows [r * max, (r + 1) * max)), rank r's first counts[r] rows kept."""
    world = len(counts)
    flat = np.asarray(flat)
    mx = flat.shape[0] // world
    return np.concatenate([flat[r * mx: r * mx + int(counts[r])] for r in range(world)])


def gather_costs(dist, local, counts):
    """Host-side all-gather of per-QP cost records when ranks hold different QP counts (Sigma
    m-balanced shards): every rank pads its [counts[rank], F] array to the largest shard, one
    gloo all_gather, padding dropped (unpad).  The device path does the same packing and padding
    in impc_comm_gather_info (one ncclAllGather).  Returns [sum(counts), F] in rank order."""
    local = np.asarray(local)
    if dist is None:
        return local
    import torch
    world = dist.get_world_size()
    mx = int(max(counts))
    buf = np.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype)
    buf[: local.shape[0]] = local
    t = torch.as_tensor(buf)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return unpad(np.concatenate([o.numpy() for o in out]), counts)


REPLAN_FIELDS = ("rank", "inst", "branch", "best_cand", "valid", "plan_sum", "plan_x0", "plan_y0", "plan_z0")


def replan_records(rank, inst, branch, best_cand, valid, plan_x):
    """[I_local, 9] float64 per-instance records of one rank's replan (REPLAN_FIELDS order): the
    makePlanWithPred branch, the selected candidate, validTraj, and the committed plan (its sum and
    its first state's position) -- what the multi-GPU replan returns to every rank (the hypothesis
    selection is local to an instance, so this is the only exchange)."""
    px = np.asarray(plan_x, np.float64)
    rec = np.zeros((len(inst), len(REPLAN_FIELDS)))
    rec[:, 0] = rank
    rec[:, 1] = inst
    rec[:, 2] = branch
    rec[:, 3] = best_cand
    rec[:, 4] = valid
    rec[:, 5] = px.sum(axis=1)
    rec[:, 6:9] = px[:, 0:3]
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

