#!/usr/bin/env python3
"""The live replan loop's rate: I planning instances flying the reference's benchmark path
(ref_trajectory_dynus_benchmark.txt) at the live horizon N = 30 with up to K dynamic obstacles each,
R chained replans as mpcNavigation::mpcCB runs them -- per replan getXRef on the device
(impc_reference_traj_device), ONE impc_replan_run (makePlanWithPred for every instance) and the
vehicle following its plan for 0.1 s (impc_replan_advance_device).  Every replan's predictions are
resident on the device before the timed loop (the predictor's output, scenarios.live_loop); each
replan is timed from its first call to the end of its device work.  Prints one JSON line.

--mixed-k: every instance sees its own number of obstacles each replan (K_i in 0..K, seeded: a
synthetic stand-in for the detector keeping the obstacles in range and view, fakeDetector.cpp:493 ->
updatePredObstacles predPos.size(), mpcPlanner.cpp:343-373; K_i = 0 replans without predictions).

--statics S: every instance also carries S static obstacles (obclustering_->getStaticObstacles(),
mpcPlanner.cpp:594; impc_replan_config.num_static) -- boxes of 0.6-1.2 m beside its own reference
path, 0.8-1.6 m off it, at random yaw (seeded; the live planner has clustering off, :191-193, so this
is the dormant path at scale).

--gpus N: one process per GPU (started here with torch.distributed.run before anything touches a
GPU, or under the caller's torchrun); the instances are split in contiguous ranges, every rank
replans its own (the selection is per instance: no exchange inside a replan), a barrier and the
max over ranks bound each replan's time, and the last replan's per-instance records
(impc.distributed.replan_records) reach every rank.  The rate is all ranks' instances over that
time.  The same loop at small I is checked replan by replan against the restatements in
tests/test_live_loop.py; the rank split in tests/test_distributed.py."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "intent-mpc_amd", "python")]


def relaunch(n, argv):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=8192)
    ap.add_argument("--obstacles", type=int, default=4)
    ap.add_argument("--replans", type=int, default=30)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--mixed-k", action="store_true", help="per-instance obstacle counts K_i in 0..K per replan")
    ap.add_argument("--statics", type=int, default=0, help="static obstacles per instance (num_static)")
    ap.add_argument("--gpus", type=int, default=1)
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(relaunch(a.gpus, sys.argv[1:]))
    import impc  # noqa: E402  (after a possible relaunch: nothing touched the GPU before it)
    from impc import distributed as D  # noqa: E402
    from impc import scenarios  # noqa: E402
    from impc.replan import DeviceReplan  # noqa: E402
    rank, local_rank, world = D.env()
    if world != a.gpus:
        sys.exit(f"live_loop.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    dist = D.init("gloo", local_rank) if world > 1 else None
    Iall, K, R, N = a.instances, a.obstacles, a.replans, a.horizon
    t0 = time.time()
    sc = scenarios.live_loop(Iall, K, R, N=N, seed=4100)
    bounds = D.equal_instance_bounds(Iall, world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    I = hi - lo
    num_pred = None
    if a.mixed_k:
        num_pred = np.random.default_rng(4101).integers(0, K + 1, (R, Iall)).astype(np.int32)[:, lo:hi]
    static = None
    if a.statics:
        rs = np.random.default_rng(4102)
        S = a.statics
        cen = np.empty((I, S, 3))
        for i in range(I):
            path = np.asarray(sc["paths"][lo + i], np.float64).reshape(-1, 3)
            at = path[np.linspace(1, min(len(path) - 1, 6), S).astype(int)]
            off = rs.uniform(0.8, 1.6, (S, 2)) * rs.choice([-1.0, 1.0], (S, 2))
            cen[i] = at + np.concatenate([off, np.zeros((S, 1))], axis=1)
        static = (cen, rs.uniform(0.6, 1.2, (I, S, 3)), rs.uniform(-np.pi, np.pi, (I, S)))
    gen_s = time.time() - t0
    p, pd, L = sc["params"], sc["pd"], sc["L"]
    # IMPC_RANK_DEVICE: every rank on that device (a rehearsal of the rank path on a one-GPU box)
    ctx = impc.Context(int(os.environ.get("IMPC_RANK_DEVICE", local_rank)))
    rp = DeviceReplan(ctx, p, pd, I, K, L, impc.default_settings(verbose=0), num_static=a.statics)
    paths = impc.ReferencePaths(ctx, list(sc["paths"][lo:hi]), pd["ts"], N)
    Dv = impc.DeviceArray
    c = np.ascontiguousarray
    pos_d, vel_d, xref_d = Dv(ctx, c(sc["pos0"][lo:hi])), Dv(ctx, c(sc["vel0"][lo:hi])), Dv(ctx, (I, N, 8))
    psize_d, prob_d = Dv(ctx, c(sc["pred_size"][lo:hi])), Dv(ctx, c(sc["prob"][lo:hi]))
    pred_d, cur_d = Dv(ctx, c(sc["pred_pos"][:, lo:hi])), Dv(ctx, c(sc["dyn_cur"][:, lo:hi]))
    np_d = Dv(ctx, c(num_pred)) if num_pred is not None else None
    st_d = [Dv(ctx, c(x)) for x in static] if static is not None else []
    st_ptr = dict(zip(("st_centroid", "st_size", "st_yaw"), (d.ptr for d in st_d)))
    step_pred, step_cur = pred_d.nbytes // R, cur_d.nbytes // R
    walls, stats = [], []
    for r in range(R):
        ctx.synchronize()
        if dist is not None:
            dist.barrier()
        t = time.perf_counter()
        paths.xref_device(pos_d.ptr, xref_d.ptr)
        rp.run_device(pos_d.ptr, vel_d.ptr, xref_d.ptr, cur_d.ptr + r * step_cur, pred_d.ptr + r * step_pred,
                      psize_d.ptr, prob_d.ptr, num_pred=None if np_d is None else np_d.ptr + r * 4 * I, **st_ptr)
        rp.advance_device(pd["ts"], pos_d.ptr, vel_d.ptr)
        ctx.synchronize()
        if dist is not None:
            dist.barrier()
        walls.append(D.max_over_ranks(dist, time.perf_counter() - t))
        st = rp.stats()
        stats.append((st["fanout"], st["single_first"], st["single_current"]))
    last = rp.results(values=False)
    its = np.concatenate([s["info"]["iter"] for s in last["shapes"].values()])
    sts = np.concatenate([s["info"]["status_val"] for s in last["shapes"].values()])
    plan_x, _, _, valid = rp.plans()
    rec = D.replan_records(rank, np.arange(lo, hi), last["branch"], last["best_cand"], valid, plan_x)
    allrec = D.gather_costs(dist, rec, [int(bounds[k + 1] - bounds[k]) for k in range(world)])
    st_all = D.gather_costs(dist, np.array([stats[-1]], np.float64), [1] * world)
    w = np.array(walls)
    fan = w[1:]  # replans 1..R-1: every instance past its first plan
    n_qps = int(its.size)
    if rank == 0:
        print(json.dumps({
            "workload": f"live loop: {Iall} instances on ref_trajectory_dynus_benchmark.txt, N={N}, "
                        f"{'K_i in 0..' + str(K) + ' per instance and replan' if a.mixed_k else 'K=' + str(K)} dynamic "
                        f"obstacles{', ' + str(a.statics) + ' static obstacles' if a.statics else ''}, {R} chained "
                        f"replans (getXRef + makePlanWithPred + follow plan 0.1 s per replan)",
            "instances": Iall, "replans": R, "n_gpus": world, "first_replan_s": float(w[0]),
            "fanout_replan_s": fan.tolist(), "fanout_replan_s_median": float(np.median(fan)),
            "replans_per_s": float(Iall / np.median(fan)), "branches_last": st_all.astype(int).sum(axis=0).tolist(),
            "last_replan_rank0": {"qps": n_qps, "mean_iter": float(its.mean()), "p50_iter": float(np.median(its)),
                                  "max_iter": int(its.max()),
                                  "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(sts, return_counts=True))},
                                  "shapes": {str(k): int(s["x"].shape[0]) for k, s in last["shapes"].items()}},
            "qp_solves_per_s_rank0": float(n_qps / np.median(fan)),
            "valid_plans": int(allrec[:, 4].sum()), "records_gathered": int(allrec.shape[0]),
            "ref_start_idx_mean": float(paths.last_idx().mean()), "gen_s": gen_s,
            "build_id": impc.lib.impc_build_id().decode()}), flush=True)
    for d in (pos_d, vel_d, xref_d, psize_d, prob_d, pred_d, cur_d) + ((np_d,) if np_d is not None else ()) + tuple(st_d):
        d.free()
    paths.close()
    rp.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
