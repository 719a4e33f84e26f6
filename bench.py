#!/usr/bin/env python3
"""Benchmark of the batched MPC QP solve (BASELINE.json metric) on MI355X.

One step = one pass of the hot path over one batch: for every QP of the workload, the device
runs osqp_setup's numeric part (Ruiz scaling, rho vector, factorisation of P + sigma I + A'RA),
the warm start, osqp_solve (ADMM to OSQP 0.6.2's termination) and the unscaling of x, y --
i.e. everything mpcPlanner::solveTraj asks OsqpEigen for (mpcPlanner.cpp:475-526).  Inputs
(P, q, A, l, u and the warm start) are resident in HBM before the timed region.

Workload (BASELINE.json configs[2], the metric's batch=65536): per GPU 8192 planning instances x
8 intent hypotheses, N=20, 8 predicted dynamic obstacles (hypotheses LEFT+FORWARD / RIGHT+FORWARD
carry a 9th), synthetic data from impc.scenarios.intent_config, bucketed by obstacle count.

Multi-GPU: one process per GPU (torchrun), each rank solves its own 65536 QPs (independent
instances, weak scaling, no data-path collective); an all_gather of the per-QP cost/status
records returns the hypothesis costs to every rank, outside the timed region.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "intent-mpc_amd", "python"))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP64_TFLOPS = 78.6    # MI355X FP64 vector peak (spec)


def throughput(world, qps_per_rank, steps, elapsed_s):
    """Whole-job QP solves per second: every rank solves qps_per_rank QPs per step, `steps` steps
    in `elapsed_s` (max over ranks)."""
    return world * qps_per_rank * steps / elapsed_s


def algorithmic_bytes(n, m, K, N):
    """B_solve = 8(n + 2m + 4K W) + 8(n + m) + 16 per QP."""
    W = N - 1
    return 8 * (n + 2 * m + 4 * K * W) + 8 * (n + m) + 16


def algorithmic_flops(n, m, nnzA, N, iters):
    """F_iter ~ 754 N + 4 nnzA + 4m + 6n + 10m per ADMM iteration."""
    return iters * (754 * N + 4 * nnzA + 4 * m + 6 * n + 10 * m) + 3700 * N


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instances", type=int, default=8192, help="planning instances per GPU (x8 hypotheses)")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="QPs solved by the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--full-values", action="store_true",
                    help="ship every QP's full CSC values (default: shared P / dynamics / box values, "
                         "per-QP obstacle rows, impc_batch_set_values_shared)")
    args = ap.parse_args()

    import impc
    from impc import distributed as D
    from impc import scenarios

    rank, local_rank, world = D.env()
    dist = D.init("nccl", local_rank) if world > 1 else None


    t_gen = time.time()
    buckets = scenarios.intent_config(N=20, K=8, instances=args.instances, hyps=8, seed=D.rank_seed(3000, rank))
    t_gen = time.time() - t_gen
    settings = impc.default_settings(verbose=0)

    ctx = impc.Context(local_rank if world > 1 else 0)
    batches, nvar = [], {}
    for K, bk in sorted(buckets.items()):
        pat, vals = bk["pattern"], bk["values"]
        B = vals["q"].shape[0]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
        b.set_settings(settings)
        split = None if args.full_values else impc.shared_split(vals["Px"], vals["Ax"])
        if split is None:
            b.set_values(vals["Px"], vals["q"], vals["Ax"], vals["l"], vals["u"])
        else:
            Px0, Ax0, var, Axv = split
            b.set_values_shared(Px0, Ax0, var, Axv, vals["q"], vals["l"], vals["u"])
            nvar[K] = int(var.size)
        b.warm_start(bk["x_ws"], np.zeros((B, pat["m"])))
        b.set_profiling(True)
        batches.append((K, bk, b))
    total_qps = sum(b.B for _, _, b in batches)

    grouped = all(b.stats()["kernel"] == impc.KERNEL_STRUCTURED for _, _, b in batches) and len(batches) > 1

    def step():
        if grouped:  # one persistent launch over all pattern buckets (impc_batch_solve_group)
            impc.solve_group([b for _, _, b in batches])
            return
        for _, _, b in batches:
            b.setup()
            b.solve()

    def sync():
        ctx.synchronize()  # hipStreamSynchronize + hipDeviceSynchronize

    for _ in range(args.warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    # timed region: barrier + device sync on both sides
    t0 = time.perf_counter()
    kt = {K: [0.0, 0.0, 0.0] for K, _, _ in batches}
    for _ in range(args.steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # per-kernel durations of the last step (HIP events on the solver stream)
    for K, _, b in batches:
        kt[K] = list(b.timings())
    # per-QP device solve latency of the last step (structured kernel; work-queue pick-up to results)
    try:
        lat = np.concatenate([b.qp_latency() for _, _, b in batches])
        qp_lat = {"p50": float(np.percentile(lat, 50)), "p90": float(np.percentile(lat, 90)),
                  "p99": float(np.percentile(lat, 99)), "max": float(lat.max()), "unit": "ms",
                  "what": "per-QP device solve latency (dequeue to results written), last timed step"}
    except impc.ImpcError:
        qp_lat = None
    elapsed = D.max_over_ranks(dist, elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps

    # results + parity-relevant statistics (outside the timed region)
    iters_all, status_all, rho_all, recs = [], [], [], []
    for K, bk, b in batches:
        x, y, info = b.get()
        iters_all.append(info["iter"])
        status_all.append(info["status_val"])
        rho_all.append(info["rho_updates"])
        recs.append(D.make_records(rank, bk["inst"], bk["hyp"], info))
    iters_all = np.concatenate(iters_all)
    status_all = np.concatenate(status_all)

    # device-side candidate scoring + selection of every instance's replan (SURVEY.md 8f row 1,
    # mpcPlanner.cpp:771-887), on the solutions still in HBM; timed on its own
    sel = select_candidates(impc, scenarios, ctx, buckets, batches, pd_params=settings_params(buckets))
    if not args.no_allgather:
        D.gather_records(dist, np.concatenate(recs))  # hypothesis costs to every rank

    value = throughput(world, total_qps, args.steps, elapsed)

    # roofline of the dominant kernel, SURVEY.md 8(d) algorithmic bytes
    kernel_name = ("k_mpc_wave_group" if grouped else "k_mpc_wave") \
        if all(b.stats()["kernel"] == impc.KERNEL_STRUCTURED for _, _, b in batches) else "k_solve"
    solve_ms = sum(kt[K][1] for K in kt)
    setup_ms = sum(kt[K][0] for K in kt)
    alg_bytes = 0.0
    alg_flops = 0.0
    for K, bk, b in batches:
        pat = bk["pattern"]
        alg_bytes += b.B * algorithmic_bytes(pat["n"], pat["m"], K, 20)
    mean_iter = float(iters_all.mean())
    for K, bk, b in batches:
        pat = bk["pattern"]
        alg_flops += b.B * algorithmic_flops(pat["n"], pat["m"], int(pat["Ap"][-1]), 20, mean_iter)
    achieved = alg_bytes / (solve_ms * 1e-3) / 1e9 if solve_ms > 0 else None
    values_mode = "shared" if nvar and len(nvar) == len(batches) else "full"
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_k_solve.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("qps_per_launch") == total_qps and pm.get("kernel") == kernel_name and \
                    pm.get("values", "full") == values_mode:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline(buckets, settings, args.cpu_sample, args.cpu_threads)

    line = {
        "metric": "QP-solves/s + p50 solve latency, N=20 horizon, batch=65536, 1/2/4/8 MI355X",
        "value": value,
        "unit": "QP-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "p50_latency_ms": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded intent-hypothesis scenarios, SURVEY.md 8d)",
        "config": {
            "workload": "configs[2]: 8192 instances x 8 intent hypotheses per GPU, N=20, 8(+1) dynamic obstacles",
            "global_batch": world * total_qps,
            "batch_per_gpu": total_qps,
            "buckets": {str(K): int(b.B) for K, _, b in batches},
            "horizon": 20,
            "settings": "OSQP 0.6.2 defaults, adaptive_rho_interval auto->25, warm-started from previous plan",
            "parallelism": f"independent QPs, {world} rank(s)",
            "values": values_mode + (f" (P and dynamics/box A entries once per bucket, per-QP A entries {nvar})"
                                     if values_mode == "shared" else " (every QP's full CSC values)"),
        },
        "qp_latency_ms": qp_lat,
        "iters": {"mean": mean_iter, "p50": float(np.median(iters_all)), "max": int(iters_all.max()),
                  "rho_updates_mean": float(np.concatenate(rho_all).mean())},
        "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(status_all, return_counts=True))},
        "kernel_ms": {"setup": setup_ms, "solve": solve_ms,
                      "outputs": sum(kt[K][2] for K in kt)},
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": (achieved / PEAK_HBM_GBS) if achieved else None,
            "traffic": traffic,
            "kernel": kernel_name,
            "algorithmic_bytes_per_launch": alg_bytes,
        },
        "fp64": {"achieved_tflops": alg_flops / ((solve_ms + setup_ms) * 1e-3) / 1e12 if solve_ms else None,
                 "peak_tflops": PEAK_FP64_TFLOPS},
        "cpu_baseline": cpu,
        "selection": sel,
        "gen_seconds": t_gen,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    for _, _, b in batches:
        b.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def settings_params(buckets):
    return next(iter(buckets.values()))["params"]


def select_candidates(impc, scenarios, ctx, buckets, batches, pd_params):
    """impc_select_best over all instances (6 candidates each, all solved QPs count as solveTraj
    successes, as OSQP's exitflag is 0 for every status); returns timing and the pick histogram."""
    ptrs = {K: b.device_results()[0] for K, _, b in batches}
    d = scenarios.selection_arrays(buckets, ptrs)
    I, C, N = d["I"], d["C"], d["N"]
    params = dict(horizon=N, num_candidates=C, max_dynamic=d["kmax"], pred_len=d["L"], num_static=0, prev_len=N,
                  dynamic_safety_dist=pd_params["dynamic_safety_dist"],
                  static_safety_dist=pd_params["static_safety_dist"])
    args = (ctx, params, d["x_ptrs"], np.ones((I, C), np.int8), np.zeros(I, np.int8), d["prev"],
            np.full(I, N, np.int32), d["xref"], np.zeros((I, 0, 3)), np.zeros((I, 0, 3)), d["dyn_count"],
            d["dyn_pos"], d["dyn_size"], d["prob"])
    impc.select_best(*args)  # warm-up (module load)
    t = time.perf_counter()
    out = impc.select_best(*args)
    t = time.perf_counter() - t
    picks = np.bincount(out["best_cand"][out["best_cand"] >= 0], minlength=C)
    return {"instances": int(I), "candidates": int(C), "ms_incl_transfers": 1000.0 * t,
            "picked_histogram": [int(v) for v in picks]}


def cpu_baseline(buckets, settings, sample, threads):
    """The oracle (C restatement of OSQP 0.6.2, reference per-call pattern) on host cores,
    over a bounded sample of the same workload (first QPs of each bucket, bucket-proportional)."""
    from oracle import osqp_oracle as ora
    total = sum(bk["values"]["q"].shape[0] for bk in buckets.values())
    s = ora.settings_from(settings)
    t_all, n_all = 0.0, 0
    for K, bk in sorted(buckets.items()):
        B = bk["values"]["q"].shape[0]
        k = max(1, int(round(sample * B / total)))
        v = bk["values"]
        t = time.perf_counter()
        ora.solve_batch(bk["pattern"], v["Px"][:k], v["q"][:k], v["Ax"][:k], v["l"][:k], v["u"][:k], s,
                        x_ws=bk["x_ws"][:k], threads=threads)
        t_all += time.perf_counter() - t
        n_all += k
    return {"value": n_all / t_all, "unit": "QP-solves/s", "cores": threads, "kind": "port",
            "sample": f"{n_all} QPs of the same workload (first of each bucket), one setup+warm-start+solve per QP"}


if __name__ == "__main__":
    main()
