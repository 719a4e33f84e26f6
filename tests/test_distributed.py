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


def test_shard_plan_balances_sigma_m():
    """Config 4's instance sharding: contiguous ranges, every rank within one
    instance's weight of the ideal Sigma m share, ranges cover every instance once."""
    from impc import scenarios
    K, w = scenarios.config4_plan(total_qps=262144)
    assert K.min() == 0 and K.max() == 20 and w.size == 32768
    for world in (1, 2, 4, 8):
        b = D.shard_plan(w, world)
        assert b[0] == 0 and b[-1] == w.size and (np.diff(b) > 0).all()
        share = np.array([w[b[r]:b[r + 1]].sum() for r in range(world)])
        assert abs(share - w.sum() / world).max() <= w.max()
    # a skewed weight vector still splits within one instance of the ideal cut
    w2 = np.concatenate([np.full(10, 100.0), np.ones(1000)])
    b2 = D.shard_plan(w2, 2)
    s2 = [w2[:b2[1]].sum(), w2[b2[1]:].sum()]
    assert abs(s2[0] - s2[1]) <= 2 * 100.0


def _config4_worker(rank, port, q):
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
        # bench.py --workload config4's rank path at a small job size, the oracle solving on CPU
        Kinst, wt = scenarios.config4_plan(total_qps=96, kmax=6)
        bounds = D.shard_plan(wt, w)
        lo, hi = int(bounds[r]), int(bounds[r + 1])
        bks = scenarios.config4_rank(lo, hi, Kinst)
        counts = [8 * int(bounds[k + 1] - bounds[k]) for k in range(w)]
        s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
        recs = []
        for bk in bks:
            _, _, info = oracle(bk, s)
            rec = np.zeros((bk["values"]["q"].shape[0], 8))
            rec[:, 0] = r
            rec[:, 1] = bk["inst"]
            rec[:, 2] = bk["hyp"]
            rec[:, 3] = info["obj_val"]
            rec[:, 4] = info["status_val"]
            rec[:, 5] = info["iter"]
            rec[:, 6] = bk["K"]
            recs.append(rec)
        allrec = D.gather_costs(dist, np.concatenate(recs), counts)
        dist.barrier()
        dist.destroy_process_group()
        q.put((r, np.concatenate(recs), allrec, (Kinst, bounds, counts)))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_two_rank_config4_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        r, rec, allrec, plan = q.get(timeout=300)
        assert allrec is not None, rec
        out[r] = (rec, allrec, plan)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Kinst, bounds, counts = out[0][2]
    all0, all1 = out[0][1], out[1][1]
    np.testing.assert_array_equal(all0, all1)                        # every rank holds every cost
    np.testing.assert_array_equal(all0, np.concatenate([out[0][0], out[1][0]]))
    assert all0.shape[0] == sum(counts) == 96                      # the whole job, no padding left
    # every instance: 8 hypotheses on the rank that owns its range, with its planned K
    for i in range(Kinst.size):
        rows = all0[all0[:, 1] == i]
        owner = int(np.searchsorted(bounds, i, side="right") - 1)
        assert sorted(rows[:, 2]) == list(range(8)) and (rows[:, 0] == owner).all()
        k = Kinst[i]
        assert set(rows[:, 6]) <= ({0} if k == 0 else {k, k + 1})
    assert (all0[:, 4] != 0).all()                                   # every QP solved (a status set)


def _config3_strong_worker(rank, port, q):
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
        # bench.py --workload config3 --scaling strong's rank path at a small batch: one fixed
        # scenario (same seed on every rank) split by instance, per-rank solve, padded cost gather
        I = 5
        full = scenarios.intent_config(instances=I, seed=3000)
        bounds = D.equal_instance_bounds(I, w)
        mine = scenarios.slice_instances(full, int(bounds[r]), int(bounds[r + 1]))
        counts = [8 * int(bounds[k + 1] - bounds[k]) for k in range(w)]
        s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
        recs = []
        for K, bk in sorted(mine.items()):
            _, _, info = oracle(bk, s)
            rec = D.make_records(r, bk["inst_global"], bk["hyp"], info)
            recs.append(np.concatenate([rec, np.full((rec.shape[0], 1), K)], axis=1))
            # the slice's own instance indices address its sliced per-instance arrays
            assert (bk["instances"]["xref"][bk["inst"]] == full[K]["instances"]["xref"][bk["inst_global"]]).all()
        allrec = D.gather_costs(dist, np.concatenate(recs), counts)
        dist.barrier()
        dist.destroy_process_group()
        q.put((r, np.concatenate(recs), allrec, counts))
    except Exception:  # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_two_rank_config3_strong_split_matches_whole_batch():
    """Strong scaling of config 3: two ranks split one fixed batch by instance; the gathered
    records are exactly those of solving the whole batch in one process (same QPs, same costs),
    each instance's 8 hypotheses on one rank."""
    import impc
    from helpers import oracle
    from impc import scenarios
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config3_strong_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        r, rec, allrec, counts = q.get(timeout=300)
        assert allrec is not None, rec
        out[r] = (rec, allrec, counts)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    all0, all1 = out[0][1], out[1][1]
    np.testing.assert_array_equal(all0, all1)
    assert all0.shape[0] == sum(out[0][2]) == 5 * 8
    assert out[0][2] == [16, 24]
    s = impc.default_settings(verbose=0, adaptive_rho_interval=25)
    whole = {}
    for K, bk in sorted(scenarios.intent_config(instances=5, seed=3000).items()):
        _, _, info = oracle(bk, s)
        for i, h, o, it in zip(bk["inst"], bk["hyp"], info["obj_val"], info["iter"]):
            whole[(int(i), int(h))] = (o, it, K)
    for row in all0:
        o, it, K = whole[(int(row[1]), int(row[2]))]
        assert row[3] == o and row[5] == it and row[6] == K
        assert row[0] == (0 if row[1] < 2 else 1)


def _closed_loop_oracle(bks, steps, s):
    """bench.py --workload config5's closed receding window (RecedingLoop) restated on the CPU for
    a rank's buckets: oracle persistent workspaces; per step each QP's x0 = state 1 of its own last
    solution and its linearisation point = that solution's states (when it has one,
    impc_batch_follow_plan_device), the reference and the predicted obstacles one step on, A / q /
    l / u from the host builder, update A + update_lin_cost + update_bounds + solve.  Returns per
    step the (inst, hyp, obj, status, iter) rows of every QP."""
    import impc
    from oracle import osqp_oracle as ora
    out = [[] for _ in range(steps)]
    so = ora.settings_from(s)
    for bk in bks:
        N, K = bk["N"], bk["K"]
        d, inst = bk["instances"], bk["inst"]
        xref, prev = d["xref"][inst], d["prev"][inst]
        p, _ = impc.mpc_params(horizon=N)
        T = steps + 1
        step = xref[:, -1, :] - xref[:, -2, :]
        path = np.concatenate([xref, xref[:, -1:, :] + step[:, None, :] * np.arange(1, T + 1)[None, :, None]], axis=1)
        dpx = np.concatenate([bk["dyn_pos"], np.repeat(bk["dyn_pos"][:, :, -1:], T, axis=2)], axis=2)
        dsx = np.concatenate([bk["dyn_size"], np.repeat(bk["dyn_size"][:, :, -1:], T, axis=2)], axis=2)
        L = bk["dyn_pos"].shape[2]
        v = bk["values"]
        pos, vel, lin = d["pos"][inst].copy(), d["vel"][inst].copy(), prev.copy()
        ws, sol = [], []
        for i in range(inst.size):
            w = ora.Workspace(bk["pattern"], v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], so)
            w.warm_start(bk["x_ws"][i], np.zeros(int(bk["pattern"]["m"])))
            sol.append(w.solve())
            ws.append(w)
        for t in range(1, steps + 1):
            for i, (x, _, info) in enumerate(sol):
                if int(info["status_val"]) in (1, 2, -2, -6):
                    pos[i], vel[i], lin[i] = x[8:11], x[11:14], x[: 8 * N].reshape(N, 8)
            vals = impc.mpc_values(p, pos, vel, path[:, t:t + N], lin, dyn_pos=dpx[:, :, t:t + L],
                                   dyn_size=dsx[:, :, t:t + L])
            for i, w in enumerate(ws):
                w.update_matrices(None, vals["Ax"][i])
                w.update_lin_cost(vals["q"][i])
                w.update_bounds(vals["l"][i], vals["u"][i])
                sol[i] = w.solve()
                out[t - 1].append((bk.get("inst_global", bk["inst"])[i], bk["hyp"][i], sol[i][2]["obj_val"], sol[i][2]["status_val"],
                                   sol[i][2]["iter"]))
        for w in ws:
            w.close()
    return [np.array(r, dtype=np.float64).reshape(-1, 5) for r in out]


def _config5_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(WORLD))
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [here, os.path.dirname(here)]
        import impc
        from impc import scenarios
        r, lr, w = D.env()
        dist = D.init("gloo", lr)
        # bench.py --workload config5's rank path at a small job: one fixed N = 40 scenario split by
        # instance, per-rank persistent workspaces through the closed receding loop, and every
        # step's cost records gathered (padded to the largest shard)
        I, steps = 3, 2
        full = scenarios.intent_config(N=40, K=10, instances=I, hyps=8, seed=5000)
        bounds = D.equal_instance_bounds(I, w)
        mine = scenarios.slice_instances(full, int(bounds[r]), int(bounds[r + 1]))
        counts = [8 * int(bounds[k + 1] - bounds[k]) for k in range(w)]
        s = impc.default_settings(verbose=0)
        per_step = _closed_loop_oracle([bk for _, bk in sorted(mine.items())], steps, s)
        gathered = []
        for rec in per_step:
            full_rec = np.zeros((rec.shape[0], 8))
            full_rec[:, 0] = r
            full_rec[:, 1:6] = rec
            gathered.append(D.gather_costs(dist, full_rec, counts))
        dist.barrier()
        dist.destroy_process_group()
        q.put((r, per_step, gathered, counts))
    except Exception:  # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_two_rank_config5_closed_loop_split_matches_whole_batch():
    """configs[4]'s multi-GPU path rehearsed on two gloo ranks: the N = 40 instances split by
    instance, each rank's persistent workspaces stepping the closed receding window (x0 from its
    own solutions, reference and obstacles moving on), every step's cost records gathered to every
    rank -- equal, step by step, to the whole batch stepped in one process."""
    import impc
    from impc import scenarios
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config5_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        r, per_step, gathered, counts = q.get(timeout=600)
        assert gathered is not None, per_step
        out[r] = (per_step, gathered, counts)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][2] == [8, 16]
    whole = _closed_loop_oracle([bk for _, bk in sorted(scenarios.intent_config(N=40, K=10, instances=3, hyps=8,
                                                                                   seed=5000).items())],
                                2, impc.default_settings(verbose=0))
    for t in range(2):
        g0, g1 = out[0][1][t], out[1][1][t]
        np.testing.assert_array_equal(g0, g1)                       # every rank holds every record
        assert g0.shape[0] == 24
        ref = {(int(a[0]), int(a[1])): a[2:] for a in whole[t]}
        for row in g0:
            np.testing.assert_array_equal(row[3:6], ref[(int(row[1]), int(row[2]))])
            assert row[0] == (0 if row[1] < 1 else 1)


def _replan_chain(idx, steps=2, seed=6060):
    """Chained makePlanWithPred replans of the instances `idx` of one fixed mixed-branch scenario on
    the restatement (oracle/replan_ref.py): per replan the per-instance records (REPLAN_FIELDS
    without the rank), x0 moving to each plan's next state and the predictions one step on."""
    import impc
    from impc import scenarios
    from oracle import replan_ref as ref
    I, K, N = 6, 3, 20
    inst = next(iter(scenarios.intent_config(N=N, K=K, instances=I, hyps=6, seed=seed).values()))["instances"]
    _, pd = impc.mpc_params(horizon=N)
    s = impc.default_settings(verbose=0)
    pred_size = np.broadcast_to(inst["size"], inst["pred"].shape).copy()
    cur_size = np.broadcast_to(inst["size"], (I, K, 3)).copy()
    ar = np.arange(I)
    first = ar % 3 == 0
    has_pred = [ar % 4 != 1, ar % 5 != 2]
    cur_count = np.where(ar % 2 == 0, K, 0)
    n = 13 * N - 5
    recs = [[] for _ in range(steps)]
    for i in idx:
        st = dict(first_time=int(first[i]), plan_x=np.concatenate([inst["prev"][i].reshape(-1), np.zeros(n - 8 * N)]))
        pos, vel, pred = inst["pos"][i].copy(), inst["vel"][i].copy(), inst["pred"][i].copy()
        for t in range(steps):
            o = ref.make_plan_with_pred(pd, pd, s, st, pos, vel, inst["xref"][i], pred[:, 0, 0, :], pred, pred_size[i],
                                        inst["prob_all"][i], bool(has_pred[t][i]), cur_size[i], int(cur_count[i]))
            px = st["plan_x"]
            recs[t].append([i, o["branch"], o["best"], int(o["valid"]), px.sum(), px[0], px[1], px[2]])
            if o["valid"]:
                pos, vel = px[8:11].copy(), px[11:14].copy()
            pred = np.concatenate([pred[:, :, 1:], pred[:, :, -1:]], axis=2)
    return [np.array(r, np.float64).reshape(-1, 8) for r in recs]


def _replan_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(WORLD))
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [here, os.path.dirname(here)]
        r, lr, w = D.env()
        dist = D.init("gloo", lr)
        # tools/live_loop.py --gpus N's rank path: the planning instances split in contiguous ranges,
        # every rank replans its own (no exchange inside a replan: the selection is per instance),
        # and each replan's per-instance records reach every rank
        bounds = D.equal_instance_bounds(6, w)
        mine = list(range(int(bounds[r]), int(bounds[r + 1])))
        counts = [int(bounds[k + 1] - bounds[k]) for k in range(w)]
        per_step = _replan_chain(mine)
        gathered = []
        for rec in per_step:
            full = D.replan_records(r, rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3], np.zeros((rec.shape[0], 3)))
            full[:, 5:9] = rec[:, 4:8]
            gathered.append(D.gather_costs(dist, full, counts))
        dist.barrier()
        dist.destroy_process_group()
        q.put((r, per_step, gathered, counts))
    except Exception:  # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_two_rank_replan_split_matches_whole_batch():
    """The batched makePlanWithPred split over two gloo ranks by planning instance (the multi-GPU
    replan / live loop): first plans, fan-outs and current-obstacle solves on both ranks over two
    chained replans; every rank ends each replan with every instance's record, equal to the whole
    batch replanned in one process."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replan_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        r, per_step, gathered, counts = q.get(timeout=600)
        assert gathered is not None, per_step
        out[r] = (per_step, gathered, counts)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][2] == [3, 3]
    whole = _replan_chain(range(6))
    branches = set()
    for t in range(2):
        g0, g1 = out[0][1][t], out[1][1][t]
        np.testing.assert_array_equal(g0, g1)
        np.testing.assert_array_equal(g0[:, 1:], whole[t])
        np.testing.assert_array_equal(g0[:, 0], [0, 0, 0, 1, 1, 1])
        branches.update(int(b) for b in g0[:, 2])
    assert branches == {0, 1, 2}
