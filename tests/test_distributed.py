"""World-size-2 rehearsal (gloo, CPU) of the multi-GPU path in bench.py: per-rank instance
shards, max-over-ranks timing, all-gather of the per-QP result records.  The solves here use the
oracle (test infrastructure); on MI355X the same helpers run over RCCL with the HIP solver."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from impc import distributed as D

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(WORLD))
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [here, os.path.dirname(here)]
        from helpers import oracle
        import impc
        from impc import scenarios
        r, lr, w = D.env()
        dist = D.init("gloo", lr)
        buckets = scenarios.intent_config(instances=2, seed=D.rank_seed(3000, r))
        s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
        recs = []
        for K, bk in sorted(buckets.items()):
            _, _, info = oracle(bk, s)
            recs.append(D.make_records(r, bk["inst"], bk["hyp"], info))
        rec = np.concatenate(recs)
        allrec = D.gather_records(dist, rec)
        tmax = D.max_over_ranks(dist, 1.0 + r)
        dist.barrier()
        dist.destroy_process_group()
        q.put((r, rec, allrec, tmax))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None, None))


def test_two_rank_gather_and_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        r, rec, allrec, tmax = q.get(timeout=240)
        assert allrec is not None, rec
        out[r] = (rec, allrec, tmax)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rec0, all0, t0 = out[0]
    rec1, all1, t1 = out[1]
    assert t0 == t1 == 2.0
    np.testing.assert_array_equal(all0, all1)
    np.testing.assert_array_equal(all0, np.concatenate([rec0, rec1]))
    assert set(all0[:, 0]) == {0.0, 1.0}
    # every instance keeps its 8 hypotheses on one rank
    for r in range(WORLD):
        rows = all0[all0[:, 0] == r]
        for i in np.unique(rows[:, 1]):
            assert sorted(rows[rows[:, 1] == i, 2]) == list(range(8))
    # rank shards are different instances (disjoint seeds)
    assert not np.array_equal(rec0[:, 3], rec1[:, 3])


def test_rank_seed_weak_scaling_invariant():
    assert D.rank_seed(3000, 0) == 3000
    assert len({D.rank_seed(3000, r) for r in range(8)}) == 8
