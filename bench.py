#!/usr/bin/env python3
"""Benchmark of the batched MPC QP solve (BASELINE.json metric) on MI355X.

One step = one pass of the hot path over one batch: for every QP of the workload, the device
runs osqp_setup's numeric part (Ruiz scaling, rho vector, factorisation of P + sigma I + A'RA),
the warm start, osqp_solve (ADMM to OSQP 0.6.2's termination) and the unscaling of x, y --
i.e. everything mpcPlanner::solveTraj asks OsqpEigen for (mpcPlanner.cpp:475-526).  Inputs
(P, q, A, l, u and the warm start) are resident in HBM before the timed region.

Workloads (--workload):
  config3 (default; BASELINE.json configs[2], the metric's batch=65536): 8192 planning instances
      x 8 intent hypotheses, N=20, 8 predicted dynamic obstacles (hypotheses LEFT+FORWARD /
      RIGHT+FORWARD carry a 9th), bucketed by obstacle count.  Strong scaling (default): the fixed
      65,536-QP batch is split across the ranks by planning instance (equal ranges: every instance
      has the same 8 QPs), and each timed step ends with one RCCL all_gather of every QP's cost
      record (N > 1).  --scaling weak: every rank solves its own 65,536 QPs and the records are
      gathered after the timed region.
  config4 (BASELINE.json configs[3]): 262,144 QPs in total (32,768 instances x 8 hypotheses,
      K ~ U{0..20} obstacles), instances sharded across the ranks in contiguous ranges balanced by
      Sigma m (impc.distributed.shard_plan).  Strong scaling: the job is fixed, each rank runs one
      grouped launch over its ~42 pattern buckets per step, and each step ends with one RCCL
      all_gather of every QP's cost record (the 64-byte impc_info, read straight from HBM).
  config5 (BASELINE.json configs[4]): 65,536 N=40 QPs (8192 instances x 8 hypotheses, 10(+1)
      dynamic obstacles), split by instance across the ranks, as a CLOSED receding window on
      persistent workspaces: setup + first solve before the timed region, then every timed step,
      all on the device: each QP's next x0 = getPos / getVel(dt) of its own last solution and its
      next linearisation point = that solution's states (impc_batch_follow_plan_device,
      mpc_node.cpp:216-224, mpcPlanner.cpp:1042-1051), the reference one step further along the
      path and the predicted obstacles one step on (impc_copy_rows_device windows), the next A
      (obstacle rows), q, l, u built by impc_mpc_build_values_device, osqp_update_A +
      osqp_update_lin_cost + osqp_update_bounds (impc_batch_update_*_device) and the solve
      continuing from the kept rho and scaled iterates (the warm-started receding window; the
      device refactors on every resume); one RCCL all_gather of the cost records (N > 1).
  live: the reference's live planner horizon N = 30 (autonomous_flight planner_param.yaml:25) on
      config 3's workload -- 8192 instances x 8 intent hypotheses, 8(+1) dynamic obstacles, full
      setup + warm start + solve per QP every step (the long shape's compile-time W = 29 instance);
      split by instance like config 3.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` without a torchrun environment
starts `torch.distributed.run` with N processes itself (before touching the GPU) and exits with
its code; under torchrun, WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "intent-mpc_amd", "python"))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP64_TFLOPS = 78.6    # MI355X FP64 vector peak (spec; 256 CU x 2.4 GHz x 128 flop/clk)
METRIC = "QP-solves/s + p50 solve latency, N=20 horizon, batch=65536, 1/2/4/8 MI355X"


def throughput(world, qps_per_rank, steps, elapsed_s):
    """Whole-job QP solves per second: every rank solves qps_per_rank QPs per step, `steps` steps
    in `elapsed_s` (max over ranks)."""
    return world * qps_per_rank * steps / elapsed_s


def algorithmic_bytes(n, m, K, N):
    """B_solve = 8(n + 2m + 4K W) + 8(n + m) + 16 per QP."""
    W = N - 1
    return 8 * (n + 2 * m + 4 * K * W) + 8 * (n + m) + 16


def flops_per_iter(n, m, nnzA, N):
    """F_iter ~ 754 N + 4 nnzA + 4m + 6n + 10m per ADMM iteration."""
    return 754 * N + 4 * nnzA + 4 * m + 6 * n + 10 * m


def algorithmic_flops(n, m, nnzA, N, iters):
    """F_solve = iters x F_iter + ~3.7k N (factorisation); iters may be an array
    (one QP each) or a scalar."""
    it = np.asarray(iters, dtype=np.float64)
    return float(it.sum() * flops_per_iter(n, m, nnzA, N) + it.size * 3700 * N)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(args_n, argv):
    """--gpus N outside torchrun: start N ranks with torch.distributed.run as a child process
    (nothing has touched the GPU yet) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args_n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def cpu_quota():
    """CPUs the process may use per the cgroup v2 quota (cpu.max "quota period"), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def make_batch(impc, ctx, bk, settings, full_values, profile, queue_weight=None):
    pat, vals = bk["pattern"], bk["values"]
    B = vals["q"].shape[0]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
    b.set_settings(settings)
    split = None if full_values else impc.shared_split(vals["Px"], vals["Ax"])
    nvar = None
    if split is None:
        b.set_values(vals["Px"], vals["q"], vals["Ax"], vals["l"], vals["u"])
    else:
        Px0, Ax0, var, Axv = split
        b.set_values_shared(Px0, Ax0, var, Axv, vals["q"], vals["l"], vals["u"])
        nvar = int(var.size)
    if bk.get("x_ws") is not None:  # solveTraj: x = previous plan, y = 0 (mpcPlanner.cpp:480-497)
        b.warm_start(bk["x_ws"], None)
    if queue_weight is not None:
        b.set_queue_order(impc.QUEUE_LONGEST_FIRST, queue_weight)
    b.set_profiling(profile)
    return b, nvar


def end_to_end(impc, ctx, batches, args, grouped):
    """PCIe-inclusive steps (SURVEY.md 8d latency definition, end to end): the QP inputs from host
    arrays (impc_batch_set_values_shared / set_values + the warm start), the solve, and x, y and the
    info records back into host arrays (impc_batch_get), host wall clock per step.  Outside the
    headline value, which is measured with the inputs resident in HBM."""
    # which A entries vary per QP is pattern-level knowledge of the caller (the device builder's
    # templates), not per-step work: split once, ship the per-QP arrays every step
    splits = [None if args.full_values else impc.shared_split(bk["values"]["Px"], bk["values"]["Ax"])
              for bk, _ in batches]
    times = []
    for _ in range(args.e2e_steps):
        ctx.synchronize()
        t = time.perf_counter()
        for (bk, b), split in zip(batches, splits):
            vals = bk["values"]
            if split is None:
                b.set_values(vals["Px"], vals["q"], vals["Ax"], vals["l"], vals["u"])
            else:
                Px0, Ax0, var, Axv = split
                b.set_values_shared(Px0, Ax0, var, Axv, vals["q"], vals["l"], vals["u"])
            if bk.get("x_ws") is not None:
                b.warm_start(bk["x_ws"], None)
        if grouped:
            impc.solve_group([b for _, b in batches])
        else:
            for _, b in batches:
                b.setup()
                b.solve()
        for _, b in batches:
            b.get()
        times.append(time.perf_counter() - t)
    qps = sum(b.B for _, b in batches)
    ms = 1000.0 * float(np.mean(times))
    return {"qps_per_s": qps / (ms * 1e-3), "ms_per_step": ms, "steps": len(times), "qps": qps,
            "what": "host wall clock per step, rank-local: host arrays -> impc_batch_set_values_shared + "
                    "impc_batch_warm_start (H2D, pageable) -> solve -> impc_batch_get (x, y, info D2H)"}


def end_to_end_pipelined(impc, ctx, bks, settings, args, queue_weight):
    """PCIe-inclusive throughput of a stream of batches (end to end) with the
    transfers overlapped: two sets of the workload's batches; while one set solves (the context's
    stream), the copy stream downloads the other set's previous results and uploads its next inputs
    (impc_batch_set_values_async / get_async from pinned host arrays, impc_host_alloc).  Host wall
    clock over `steps` steps, from the first upload to the last download: every QP's inputs cross
    PCIe in and its x, y and info come back inside the measured time."""
    steps = max(2, args.e2e_steps)
    C = impc.Stream(ctx)
    sets, host = [], []
    try:
        for _ in range(2):
            bs, hs = [], []
            for bk in bks:
                b, _ = make_batch(impc, ctx, bk, settings, False, False, queue_weight)
                v = bk["values"]
                Px0, Ax0, var, Axv = impc.shared_split(v["Px"], v["Ax"])
                h = {k: impc.HostArray(ctx, a.shape) for k, a in (("Axv", Axv), ("q", v["q"]), ("l", v["l"]),
                                                                  ("u", v["u"]), ("x_ws", bk["x_ws"]))}
                for k, a in (("Axv", Axv), ("q", v["q"]), ("l", v["l"]), ("u", v["u"]), ("x_ws", bk["x_ws"])):
                    h[k].a[...] = a  # the producer's data, already in pinned memory when the step starts
                h["x"] = impc.HostArray(ctx, (b.B, b.n))
                h["y"] = impc.HostArray(ctx, (b.B, b.m))
                h["info"] = impc.HostArray(ctx, (b.B,), impc.INFO_DTYPE)
                bs.append(b)
                hs.append(h)
            sets.append(bs)
            host.append(hs)

        def upload(s):
            for b, h in zip(sets[s], host[s]):
                b.set_values_async(h["Axv"], h["q"], h["l"], h["u"], h["x_ws"], stream=C)

        def download(s):
            for b, h in zip(sets[s], host[s]):
                b.get_async(h["x"], h["y"], h["info"], stream=C)

        for rep in range(2):  # rep 0: warm-up (module load, scratch growth)
            ctx.synchronize()
            t0 = time.perf_counter()
            upload(0)
            impc.ctx_stream_wait(ctx, C)
            for t in range(steps):
                s = t % 2
                impc.solve_group(sets[s])                  # context stream
                if t + 1 < steps:
                    upload(1 - s)                          # after set 1-s's previous solve (C waited for it)
                    impc.ctx_stream_wait(ctx, C)           # the next solve waits for that upload
                C.wait(None)                               # after this solve
                download(s)
            C.synchronize()
            ctx.synchronize()
            el = time.perf_counter() - t0
        ok = all(np.array_equal(host[(steps - 1) % 2][k]["info"].a["iter"], b.get()[2]["iter"])
                 for k, b in enumerate(sets[(steps - 1) % 2]))
        qps = sum(b.B for b in sets[0])
    finally:
        for bs in sets:
            for b in bs:
                b.close()
        for hs in host:
            for h in hs:
                for a in h.values():
                    a.free()
        C.close()
    ms = 1000.0 * el / steps
    return {"qps_per_s": qps / (ms * 1e-3), "ms_per_step": ms, "steps": steps, "qps": qps, "results_match": bool(ok),
            "what": "host wall clock per step of a pipelined stream of batches: per-QP inputs (pinned host arrays) "
                    "-> impc_batch_set_values_async on a copy stream, solve on the context stream, x, y, info -> "
                    "pinned host arrays (impc_batch_get_async); the next batch set's upload and the previous one's "
                    "download overlap each solve; first upload and last download inside the measured time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("config3", "config4", "config5", "live"), default="config3")
    ap.add_argument("--instances", type=int, default=8192,
                    help="config3 / config5: planning instances of the job (x8 hypotheses)")
    ap.add_argument("--total-qps", type=int, default=262144, help="config4: QPs of the whole job")
    ap.add_argument("--cpu-sample", type=int, default=8192, help="QPs solved by the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="CPU baseline threads (the GPU box's CPU share per GPU is 16)")
    ap.add_argument("--cpu-all-cores", type=int, default=1,
                    help="also time the CPU baseline with one thread per CPU of the process's affinity set")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="config3: split the fixed 65,536-QP batch across ranks (strong) or 65,536 per rank (weak)")
    ap.add_argument("--queue", choices=("longest", "fifo"), default="longest",
                    help="work-queue order of the persistent launches (impc_batch_set_queue_order)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="single-GPU study: run only rank 0's shard of a W-way strong split (not a headline line)")
    ap.add_argument("--e2e-steps", type=int, default=4,
                    help="end-to-end steps after the timed region: host arrays in -> solve -> results on the host")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--receding", type=int, default=1,
                    help="config5: 0 = every step a full setup + warm start + solve of the same QPs (no receding "
                         "window; a kernel-study workload, not the configs[4] line)")
    ap.add_argument("--receding-replay", type=int, default=1,
                    help="config5: the untimed replay after the timed steps (per-step stats, CPU baseline, parity); "
                         "0 for profiler passes that must see only the timed launches")
    ap.add_argument("--full-values", action="store_true",
                    help="ship every QP's full CSC values (default: shared P / dynamics / box values, "
                         "per-QP obstacle rows, impc_batch_set_values_shared)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus, sys.argv[1:]))
    from impc import distributed as D
    rank, local_rank, world = D.env()
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.shard_of and world != 1:
        sys.exit("bench.py: --shard-of is a single-GPU study of one rank's shard")

    import impc
    from impc import scenarios
    # host traffic (rendezvous, barriers, max over ranks) on gloo; the device records move over
    # RCCL through the solver library's communicator (impc_comm.h) -- this process never starts
    # PyTorch's own HIP runtime
    dist = D.init("gloo", local_rank) if world > 1 else None

    settings = impc.default_settings(verbose=0)
    strong = args.workload != "config3" or args.scaling == "strong"
    t_gen = time.time()
    if args.workload in ("config3", "config5", "live"):
        N_, K_, seed_ = {"config3": (20, 8, 3000), "config5": (40, 10, 5000), "live": (30, 8, 3030)}[args.workload]
        buckets = scenarios.intent_config(N=N_, K=K_, instances=args.instances, hyps=8,
                                          seed=seed_ if strong else D.rank_seed(seed_, rank))
        if strong:  # equal instance ranges (every instance carries the same 8 hypotheses)
            bounds = D.equal_instance_bounds(args.instances, args.shard_of or world)
            buckets = scenarios.slice_instances(buckets, int(bounds[rank]), int(bounds[rank + 1]))
        bks = [bk for _, bk in sorted(buckets.items())]
    else:
        Kinst, w = scenarios.config4_plan(total_qps=args.total_qps)
        bounds = D.shard_plan(w, args.shard_of or world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        bks = scenarios.config4_rank(lo, hi, Kinst)
        share = [float(w[bounds[r]:bounds[r + 1]].sum()) for r in range(args.shard_of or world)]
    t_gen = time.time() - t_gen

    # IMPC_RANK_DEVICE: every rank on that device (a rehearsal of the rank path on a one-GPU box;
    # never set by the driver)
    ctx = impc.Context(int(os.environ.get("IMPC_RANK_DEVICE", local_rank)))
    batches, nvar = [], []
    qw = scenarios.queue_weight(bks[0]["params"], bks[0]["N"]) if args.queue == "longest" else None
    for bk in bks:
        b, nv = make_batch(impc, ctx, bk, settings, args.full_values, profile=True, queue_weight=qw)
        batches.append((bk, b))
        if nv is not None:
            nvar.append(nv)
    total_qps = sum(b.B for _, b in batches)
    structured = all(b.stats()["kernel"] == impc.KERNEL_STRUCTURED for _, b in batches)
    grouped = structured and len(batches) > 1
    # every rank's QP count (config 4's shards differ) and the RCCL communicator of the cost gather
    counts = [total_qps] * world
    if dist is not None:
        import torch
        t = torch.zeros(world, dtype=torch.int64)
        t[rank] = total_qps
        dist.all_reduce(t)
        counts = [int(c) for c in t]
    # (a rehearsal with every rank on one device, IMPC_RANK_DEVICE, has no RCCL communicator: RCCL
    # refuses two ranks on one GPU, "invalid usage"; the step then skips the cost all-gather)
    rehearsal = "IMPC_RANK_DEVICE" in os.environ and world > 1
    comm = D.make_comm(dist, ctx) if ((world > 1 or args.workload == "config4") and not rehearsal) else None
    receding = None
    if args.workload == "config5" and args.receding:  # persistent workspaces: setup + first solve, untimed
        receding = RecedingLoop(impc, ctx, batches, args.warmup + args.steps)
        receding.start()
    max_qps = max(counts)
    recv = impc.DeviceArray(ctx, (world * max_qps,), impc.INFO_DTYPE) if comm is not None else None
    # strong scaling: the cost records of the step's QPs reach every rank inside the step
    gather_in_step = (args.workload == "config4" or (strong and world > 1)) and not args.no_allgather and comm is not None

    def launch():
        if receding is not None:  # the closed loop's next step, built on the device
            receding.advance()
        if grouped:  # one persistent launch over all pattern buckets (impc_batch_solve_group)
            impc.solve_group([b for _, b in batches])
        else:
            for _, b in batches:
                b.setup()
                b.solve()

    def step():
        ctx.timer_mark()
        launch()
        ctx.timer_mark()
        if gather_in_step:  # every QP's cost record to every rank, one ncclAllGather
            comm.gather_info([b for _, b in batches], max_qps, recv.ptr)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    ctx.timer_read()  # drop the warm-up marks
    if dist is not None:
        dist.barrier()
    # timed region: barrier + device sync on both sides
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [float(v) for v in ctx.timer_read()]  # HIP events around each launch, on its stream
    elapsed = D.max_over_ranks(dist, elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps
    launch_ms = float(np.mean(kernel_ms))

    # per-QP device solve latency of the last step (structured kernel; work-queue pick-up to results)
    try:
        lat = np.concatenate([b.qp_latency() for _, b in batches])
        qp_lat = {"p50": float(np.percentile(lat, 50)), "p90": float(np.percentile(lat, 90)),
                  "p99": float(np.percentile(lat, 99)), "max": float(lat.max()), "unit": "ms",
                  "what": "per-QP device solve latency (dequeue to results written), last timed step"}
    except impc.ImpcError:
        qp_lat = None

    # results + parity-relevant statistics (outside the timed region)
    iters_all, status_all, rho_all, recs, results = [], [], [], [], []
    alg_bytes = alg_flops = 0.0
    for bk, b in batches:
        x, y, info = b.get()
        results.append((x, y, info))
        pat = bk["pattern"]
        iters_all.append(info["iter"])
        status_all.append(info["status_val"])
        rho_all.append(info["rho_updates"])
        recs.append(D.make_records(rank, bk.get("inst_global", bk["inst"]), bk["hyp"], info))
        alg_bytes += b.B * algorithmic_bytes(pat["n"], pat["m"], bk["K"], bk["N"])
        alg_flops += algorithmic_flops(pat["n"], pat["m"], int(pat["Ap"][-1]), bk["N"], info["iter"])
    iters_all = np.concatenate(iters_all)
    status_all = np.concatenate(status_all)

    sel = None
    if args.workload == "config3":
        # device-side candidate scoring + selection of every instance's replan (SURVEY.md 8f row 1,
        # mpcPlanner.cpp:771-887), on the solutions still in HBM; timed on its own
        sel = select_candidates(impc, scenarios, ctx, buckets, dict((bk["K"], b) for bk, b in batches),
                                pd_params=bks[0]["params"])
        if comm is not None and not args.no_allgather and not gather_in_step:  # costs to every rank
            comm.gather_info([b for _, b in batches], max_qps, recv.ptr)
    gathered = None
    if recv is not None and not args.no_allgather:
        allinfo = D.unpad(recv.get(), counts)
        mine = np.concatenate([r[:, 4] for r in recs])
        off = sum(counts[:rank])
        gathered = {"records": int(allinfo.size), "ranks": world,
                    "own_block_matches": bool(np.array_equal(allinfo["status_val"][off:off + total_qps], mine))}

    global_batch = int(sum(counts))
    value = global_batch * args.steps / elapsed  # every rank's QPs, each timed step, max-over-ranks time

    # roofline of the dominant kernel: FP64 compute/latency bound, so the headline
    # fraction is the algorithmic FP64 rate over the vector peak; the HBM fraction and the
    # PMC-measured traffic ride along
    kernel_name = ("k_mpc_wave_group" if grouped else "k_mpc_wave") if structured else "k_solve"
    tflops = alg_flops / (launch_ms * 1e-3) / 1e12
    gbs = alg_bytes / (launch_ms * 1e-3) / 1e9
    values_mode = "shared" if len(nvar) == len(batches) else "full"
    nvar_desc = {str(bk["K"]): nv for (bk, _), nv in zip(batches, nvar)} if values_mode == "shared" else None
    build_id = impc.lib.impc_build_id().decode()
    # the PMC summary is keyed on the workload as timed: config 5's full-setup study is another workload
    pmc_workload = "config5_fullsetup" if (args.workload == "config5" and not args.receding) else args.workload
    traffic, traffic_src = measured_traffic(build_id, total_qps, kernel_name, values_mode, pmc_workload)

    e2e = e2e_serial = None
    if args.e2e_steps > 0 and receding is None:
        e2e_serial = end_to_end(impc, ctx, batches, args, grouped)
        if grouped and not args.full_values and all(bk.get("x_ws") is not None for bk in bks):
            e2e = end_to_end_pipelined(impc, ctx, bks, settings, args, qw)
            e2e["frac_of_resident"] = e2e["qps_per_s"] / (total_qps * args.steps / elapsed) if world == 1 else None

    cpu = parity = None
    per_step = None
    if receding is not None and args.receding_replay:
        # untimed replay of the same closed loop (the device is deterministic: its last step must
        # equal the timed run's bit for bit), recording every step's iterations / statuses and the
        # CPU sample's per-step q, l, u for the oracle
        k_sample = min(args.cpu_sample, 1024) if (rank == 0 and world == 1) else 0
        rec = receding.replay(k_sample, persist=bool(k_sample))
        per_step = rec["per_step"]
        per_step_det = all(np.array_equal(r[0], x) and np.array_equal(r[2]["iter"], inf["iter"])
                           for r, (x, _, inf) in zip(rec["last"], results))
        per_step = {"steps": per_step, "replay_bitwise_equal": bool(per_step_det)}
        if k_sample:
            cpu, ref = cpu_baseline_receding(bks, settings, rec, args.cpu_threads)
            # parity: the first closed-loop step (setup + solve, then osqp_update_A / _lin_cost /
            # _bounds + solve on both sides from identical inputs), and every later step from the same
            # starting point -- the oracle re-synchronised to the device's persisted state (chain)
            got = [[e["got"][t] for e in rec["buckets"]] for t in range(len(rec["per_step"]))]
            parity = parity_vs_oracle(got[0], [r[0] for r in ref])
            parity["what"] = ("the first closed-loop step's x, y, status, iterations for the CPU sample's QPs vs the "
                              "oracle's persistent workspaces after the same setup + update sequence (osqp_update_A, "
                              "_lin_cost, _bounds; parity unpinned against the real libosqp, DESIGN.md 3); chain: "
                              "every step with the oracle re-synchronised to the device's state")
            parity["chain"] = receding_chain_parity(rec, settings, args.cpu_threads, ref)
            parity["pass"] = bool(parity["pass"] and parity["chain"]["pass"])
        args.cpu_all_cores = 0
    elif rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu, ref = cpu_baseline(bks, settings, args.cpu_sample, args.cpu_threads)
        parity = parity_vs_oracle(results, ref)
        if args.cpu_all_cores:
            cores = len(os.sched_getaffinity(0))
            allc, _ = cpu_baseline(bks, settings, min(total_qps, args.cpu_sample * max(1, cores // args.cpu_threads)),
                                   cores)
            cpu["all_cores"] = {k: allc[k] for k in ("value", "unit", "cores", "sample")}
            cpu["all_cores"]["cgroup_cpu_quota"] = cpu_quota()
            cpu["all_cores"]["what"] = ("one oracle thread per CPU of os.sched_getaffinity(0); the box's cgroup "
                                        "quota (cgroup_cpu_quota CPUs) bounds what they get")

    if args.workload == "config3":
        config = {
            "workload": ("configs[2]: 65536 QPs = 8192 instances x 8 intent hypotheses, split by instance over the "
                         "ranks, N=20, 8(+1) dynamic obstacles, per-step RCCL all-gather of the cost records (N>1)")
            if strong else "configs[2]: 8192 instances x 8 intent hypotheses per GPU, N=20, 8(+1) dynamic obstacles",
            "global_batch": global_batch, "batch_per_gpu": total_qps, "shard_qps": counts,
            "buckets": {str(bk["K"]): int(b.B) for bk, b in batches},
        }
    elif args.workload == "live":
        config = {
            "workload": ("live planner horizon: 65536 N=30 QPs = 8192 instances x 8 intent hypotheses, 8(+1) dynamic "
                         "obstacles (planner_param.yaml:25), split by instance over the ranks, full setup + warm start "
                         "+ solve per QP, per-step RCCL all-gather of the cost records (N>1)"),
            "global_batch": global_batch, "batch_per_gpu": total_qps, "shard_qps": counts,
            "buckets": {str(bk["K"]): int(b.B) for bk, b in batches},
        }
    elif args.workload == "config5":
        config = {
            "workload": ("configs[4]: 65536 N=40 QPs = 8192 instances x 8 intent hypotheses, 10(+1) dynamic obstacles, "
                         "split by instance over the ranks, closed receding window on persistent workspaces (per step, "
                         "on the device: x0 = getPos/getVel(dt) of each QP's last solution, reference and predicted "
                         "obstacles one step on, obstacle rows re-linearised at the last plan, A / q / l / u built, "
                         "osqp_update_A + update q + update l, u + solve from the kept rho / iterates with the data "
                         "scaled afresh), per-step RCCL all-gather of the cost records (N>1)")
            if args.receding else
            ("configs[4] QPs (65536 N=40, 10(+1) dynamic obstacles), kernel study: full setup + warm start + solve "
             "of the same QPs every step (--receding 0, not the configs[4] line)"),
            "global_batch": global_batch, "batch_per_gpu": total_qps, "shard_qps": counts,
            "buckets": {str(bk["K"]): int(b.B) for bk, b in batches},
        }
    else:
        config = {
            "workload": "configs[3]: 262144 mixed-K QPs (K ~ U{0..20}) sharded by Sigma m, per-step RCCL "
                        "all-gather of the cost records",
            "global_batch": global_batch, "batch_per_gpu": total_qps, "shard_qps": counts,
            "shard_sigma_m": share, "pattern_buckets": len(batches), "allgather": gathered,
        }
    config.update({
        "horizon": bks[0]["N"],
        "settings": "OSQP 0.6.2 defaults, adaptive_rho_interval auto->25, warm-started from previous plan",
        "parallelism": f"independent QPs, {world} rank(s)",
        "queue": ("longest-first (device-estimated key: warm-start violation + q_weight*||q||_inf, "
                  "impc_batch_set_queue_order)") if args.queue == "longest" else "fifo",
        "values": values_mode + (f" (P and dynamics/box A entries once per bucket, per-QP A entries {nvar_desc})"
                                 if values_mode == "shared" else " (every QP's full CSC values)"),
    })
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "QP-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "p50_latency_ms": qp_lat["p50"] if qp_lat else None,
        "step_latency_ms": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded intent-hypothesis scenarios, SURVEY.md 8d)",
        "config": config,
        "shard_study": (f"rank 0's shard of a {args.shard_of}-way strong split, alone on one GPU"
                        if args.shard_of else None),
        "qp_latency_ms": qp_lat,
        "iters": {"mean": float(iters_all.mean()), "p50": float(np.median(iters_all)), "max": int(iters_all.max()),
                  "rho_updates_mean": float(np.concatenate(rho_all).mean())},
        "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(status_all, return_counts=True))},
        "kernel_ms": {"mean": launch_ms, "per_step": kernel_ms,
                      "what": "HIP events around each timed step's launch, on its stream (rank 0)"},
        "roofline": {
            "bound": "fp64",
            "achieved": tflops,
            "peak": PEAK_FP64_TFLOPS,
            "unit": "TFLOP/s",
            "frac": tflops / PEAK_FP64_TFLOPS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kernel_name,
            "build_id": build_id,
            "algorithmic_flops_per_launch": alg_flops,
            "what": "SURVEY.md 8d F_iter x each QP's iterations + 3.7k N per QP, over the mean event-timed launch",
            "hbm": {"achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                    "algorithmic_bytes_per_launch": alg_bytes, "traffic_bytes_per_launch": traffic},
        },
        "cpu_baseline": cpu,
        "parity": parity,
        "e2e": e2e,
        "e2e_serial": e2e_serial,
        "selection": sel,
        "cost_allgather": gathered,
        "receding_steps": per_step,
        "gen_seconds": t_gen,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if receding is not None:
        receding.close()
    if recv is not None:
        recv.free()
    if comm is not None:
        comm.close()
    for _, b in batches:
        b.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def select_candidates(impc, scenarios, ctx, buckets, batch_by_k, pd_params):
    """impc_select_best over all instances (6 candidates each, all solved QPs count as solveTraj
    successes, as OSQP's exitflag is 0 for every status); returns timing and the pick histogram."""
    ptrs = {K: b.device_results()[0] for K, b in batch_by_k.items()}
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


class RecedingLoop:
    """Config 5's closed receding window on the device (module docstring).  Per bucket: each QP's
    reference path extended past the horizon (the last segment continued, as getReferenceTraj pads),
    its predicted obstacles extended by their last entry (the builder's .back() rule), x0 / v0 and
    the linearisation point (initially the scenario's previous plan) as device rows updated from
    each solve (impc_batch_follow_plan_device)."""

    def __init__(self, impc, ctx, batches, steps):
        self.impc, self.ctx, self.batches, self.steps, self.t = impc, ctx, batches, steps, 0
        self.buckets = []
        for bk, b in batches:
            N, K = bk["N"], bk["K"]
            d, inst = bk["instances"], bk["inst"]
            xref, prev = d["xref"][inst], d["prev"][inst]
            nb = inst.size
            p, pd = impc.mpc_params(horizon=N)
            L = bk["dyn_pos"].shape[2]
            T = steps + 1
            step = xref[:, -1, :] - xref[:, -2, :]
            ext = xref[:, -1:, :] + step[:, None, :] * np.arange(1, T + 1)[None, :, None]
            path = np.ascontiguousarray(np.concatenate([xref, ext], axis=1))            # [nb][N + T][8]
            dpx = np.concatenate([bk["dyn_pos"], np.repeat(bk["dyn_pos"][:, :, -1:], T, axis=2)], axis=2)
            dsx = np.concatenate([bk["dyn_size"], np.repeat(bk["dyn_size"][:, :, -1:], T, axis=2)], axis=2)
            n, m, nnzP, nnzA = impc.mpc_dims(p, 0, K)
            D = impc.DeviceArray
            e = dict(N=N, K=K, L=L, T=T, nb=nb, ts=pd["ts"], b=b, bk=bk,
                     bld=impc.MpcBuilder(ctx, p, 0, K, L),
                     path=D(ctx, path), dpx=D(ctx, np.ascontiguousarray(dpx)), dsx=D(ctx, np.ascontiguousarray(dsx)),
                     lin=D(ctx, np.ascontiguousarray(prev, np.float64)), lin0=np.ascontiguousarray(prev, np.float64),
                     pos0=np.ascontiguousarray(d["pos"][inst], np.float64),
                     vel0=np.ascontiguousarray(d["vel"][inst], np.float64),
                     pos=D(ctx, (nb, 3)), vel=D(ctx, (nb, 3)), xr=D(ctx, (nb, N, 8)), dp=D(ctx, (nb, K, L, 3)),
                     ds=D(ctx, (nb, K, L, 3)), Px=D(ctx, (nb, nnzP)), Ax=D(ctx, (nb, nnzA)), q=D(ctx, (nb, n)),
                     l=D(ctx, (nb, m)), u=D(ctx, (nb, m)))
            self.buckets.append(e)

    def _solve(self):
        bs = [b for _, b in self.batches]
        self.impc.solve_group(bs) if len(bs) > 1 else bs[0].solve()

    def start(self):
        """Setup + first solve of every QP from the scenario's values and warm start (untimed)."""
        for e in self.buckets:
            bk, b = e["bk"], e["b"]
            v = bk["values"]
            b.set_persistent(True)
            split = self.impc.shared_split(v["Px"], v["Ax"])
            if split is None:
                b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
            else:
                b.set_values_shared(*split, v["q"], v["l"], v["u"])
            b.warm_start(bk["x_ws"], None)
            e["pos"].set(e["pos0"])
            e["vel"].set(e["vel0"])
            e["lin"].set(e["lin0"])
        self._solve()
        self.ctx.synchronize()
        self.t = 0

    def build(self):
        """The next step's x0 (from the last solve), windows and q, l, u -- all enqueued on the device."""
        impc, ctx = self.impc, self.ctx
        self.t += 1
        t = self.t
        for e in self.buckets:
            N, K, L, T, nb = e["N"], e["K"], e["L"], e["T"], e["nb"]
            e["b"].follow_plan_device(N, e["ts"], e["ts"], e["pos"].ptr, e["vel"].ptr, e["lin"].ptr)
            impc.copy_rows_device(ctx, e["xr"].ptr, 64 * N, e["path"].ptr + 64 * t, 64 * (N + T), 64 * N, nb)
            for src, dst in (("dpx", "dp"), ("dsx", "ds")):
                impc.copy_rows_device(ctx, e[dst].ptr, 24 * L, e[src].ptr + 24 * t, 24 * (L + T), 24 * L, nb * K)
            e["bld"].build(nb, e["pos"].ptr, e["vel"].ptr, e["xr"].ptr, e["lin"].ptr, None, None, None, e["dp"].ptr,
                           e["ds"].ptr, e["Px"].ptr, e["q"].ptr, e["Ax"].ptr, e["l"].ptr, e["u"].ptr)

    def advance(self):
        """One timed closed-loop step: next values on the device, persistent updates -- the new A
        (osqp_update_A), q, l, u (the solve follows in the caller's launch)."""
        self.build()
        for e in self.buckets:
            e["b"].update_matrices_device(None, e["Ax"].ptr)
            e["b"].update_lin_cost_device(e["q"].ptr)
            e["b"].update_bounds_device(e["l"].ptr, e["u"].ptr)

    def replay(self, k_sample, persist=False):
        """The same loop again from the setup, untimed: per step the iterations / statuses of every
        QP and the first k_sample QPs' q, l, u (bucket-proportional) for the oracle; the last step's
        results per bucket.  persist: also the sample's persistent workspaces (rho and the scaled
        iterates, impc_batch_get_persistent) after the first solve and after every step's solve --
        the state the oracle is re-synchronised to before the next step."""
        total = sum(e["nb"] for e in self.buckets)
        for e in self.buckets:
            e["k"] = min(e["nb"], max(1, int(round(k_sample * e["nb"] / total)))) if k_sample else 0
            e["ups"], e["got"], e["pst"] = [], [], []
        self.start()
        if persist:
            for e in self.buckets:
                if e["k"]:
                    e["pst"].append(tuple(a[: e["k"]] for a in e["b"].get_persistent()))
        per_step = []
        for _ in range(self.steps):
            self.advance()
            for e in self.buckets:
                if e["k"]:
                    e["ups"].append(tuple(rows_to_host(self.impc, self.ctx, e[a], e["k"]) for a in ("Ax", "q", "l", "u")))
            self._solve()
            its, sts = [], []
            for e in self.buckets:
                x, y, info = e["b"].get()
                its.append(info["iter"])
                sts.append(info["status_val"])
                if e["k"]:  # the sample's results of this step (the oracle's per-step comparison)
                    e["got"].append((x[: e["k"]], y[: e["k"]], info[: e["k"]]))
                    if persist:
                        e["pst"].append(tuple(a[: e["k"]] for a in e["b"].get_persistent()))
            it, st = np.concatenate(its), np.concatenate(sts)
            per_step.append({"step": self.t, "mean_iter": float(it.mean()), "p50_iter": float(np.median(it)),
                             "max_iter": int(it.max()),
                             "status_counts": {str(int(k)): int(v) for k, v in zip(*np.unique(st, return_counts=True))}})
        last = [e["b"].get() for e in self.buckets]
        return {"per_step": per_step, "last": last, "buckets": self.buckets}

    def close(self):
        for e in self.buckets:
            e["bld"].close()
            for k in ("path", "dpx", "dsx", "lin", "pos", "vel", "xr", "dp", "ds", "Px", "Ax", "q", "l", "u"):
                e[k].free()


def rows_to_host(impc, ctx, darr, k):
    """The first k rows of a QP-major device array."""
    row = darr.nbytes // darr.shape[0]
    out = np.empty((k,) + tuple(darr.shape[1:]), darr.dtype)
    impc._check(impc.lib.impc_copy_to_host(ctx.h, impc._P(out.ctypes.data), impc._P(darr.ptr), row * k),
                "impc_copy_to_host")
    return out


def oracle_chains(rec, settings, threads, resync=False, q1_perturb=0.0, seed=0):
    """Config 5's closed loop on the oracle's persistent workspaces (osqp_setup, warm start, solve
    once, then per closed-loop step osqp_update_A + osqp_update_lin_cost + osqp_update_bounds +
    osqp_solve with that step's device-built A, q, l, u) for the sample of every bucket, on `threads`
    host threads (one QP's chain per task; the oracle's C calls release the GIL).
    resync: before each step the workspace takes the device's persisted rho and scaled iterates
    after the previous solve (impc_batch_get_persistent -> ora_set_state), so each step starts
    where the device's did; the oracle's own state at that point is kept for the drift report.
    q1_perturb: the first closed-loop step's q times (1 + q1_perturb * U(-1, 1)) (seeded) -- the
    oracle against itself under a perturbation of the size the two implementations differ by.
    Returns (seconds of the update + solve steps, per bucket [(k, x, y, info) per step],
    per bucket [per step: (oracle rho, x, z, y) before the resync] or None)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import osqp_oracle as ora
    s = ora.settings_from(settings)
    out, states, t_all = [], [], 0.0
    for e in rec["buckets"]:
        bk, k, ups, pst = e["bk"], e["k"], e["ups"], e.get("pst")
        v = bk["values"]
        if resync and (not pst or len(pst) < len(ups)):
            raise ValueError("resync needs the device's persistent states (replay(..., persist=True))")
        rng = np.random.default_rng(seed)
        dq = 1.0 + q1_perturb * rng.uniform(-1.0, 1.0, size=ups[0][1].shape) if q1_perturb else None

        def setup(i):
            w = ora.Workspace(bk["pattern"], v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], s)
            w.warm_start(bk["x_ws"][i], np.zeros(int(bk["pattern"]["m"])))
            w.solve()
            return w

        with ThreadPoolExecutor(max_workers=threads) as ex:
            ws = list(ex.map(setup, range(k)))

        def chain(i):
            res, own = [], []
            for t, (Ax, q, l, u) in enumerate(ups):
                if resync:
                    own.append(ws[i].get_state())
                    rho, x, z, y = (a[i] for a in pst[t])
                    ws[i].set_state(rho, x, z, y)
                ws[i].update_matrices(None, Ax[i])
                ws[i].update_lin_cost(q[i] * dq[i] if (dq is not None and t == 0) else q[i])
                ws[i].update_bounds(l[i], u[i])
                res.append(ws[i].solve())
            return res, own

        t = time.perf_counter()
        with ThreadPoolExecutor(max_workers=threads) as ex:
            res = list(ex.map(chain, range(k)))
        t_all += time.perf_counter() - t
        for w in ws:
            w.close()
        out.append([(k, np.array([r[0][t][0] for r in res]), np.array([r[0][t][1] for r in res]),
                     np.array([r[0][t][2] for r in res], dtype=res[0][0][t][2].dtype)) for t in range(len(ups))])
        states.append([[r[1][t] for r in res] for t in range(len(ups))] if resync else None)
    return t_all, out, states


def cpu_baseline_receding(bks, settings, rec, threads):
    """Config 5's CPU path: the oracle's persistent workspaces over a bounded sample, the first QPs
    of each bucket (oracle_chains without resync); the timed part is the update + solve steps.
    Returns (line object, [(k, x, y, info) per step] per bucket, for the parity check)."""
    t_all, ref, _ = oracle_chains(rec, settings, threads)
    steps = len(rec["buckets"][0]["ups"])
    n_sample = sum(e["k"] for e in rec["buckets"])
    return {"value": n_sample * steps / t_all, "unit": "QP-solves/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_info(),
            "sample": f"{n_sample} QPs of the workload (first of each bucket) x {steps} closed-loop "
                      f"steps, oracle persistent workspaces (update A, q, l/u, solve) with the device-built values "
                      f"of each step, {threads} threads ({t_all:.1f} s)"}, ref


def state_diff(dev, own):
    """Worst relative differences over a sample between the device's persisted state and the
    oracle's own at the same point: (scaled iterates x, z, y; rho)."""
    rho, x, z, y = dev
    worst = worst_rho = 0.0
    for i, (orho, ox, oz, oy) in enumerate(own):
        worst_rho = max(worst_rho, abs(rho[i] - orho) / orho)
        for a, b in ((x[i], ox), (z[i], oz), (y[i], oy)):
            if b.size:
                worst = max(worst, float(np.abs(a - b).max()) / max(float(np.abs(b).max()), 1e-12))
    return worst, worst_rho


def receding_chain_parity(rec, settings, threads, ref_free):
    """Config 5's chain pinned step by step: (1) the oracle re-synchronised to the
    device's persisted state before every step -- each step's status, iterations and x compared from
    the same starting point; (2) the free-running chains' drift, device vs oracle (ref_free) next to
    the oracle against itself with a 1e-13 relative perturbation of the first step's q."""
    steps = len(rec["buckets"][0]["ups"])
    got = [[e["got"][t] for e in rec["buckets"]] for t in range(steps)]
    _, ref_sync, own = oracle_chains(rec, settings, threads, resync=True)
    _, ref_pert, _ = oracle_chains(rec, settings, threads, q1_perturb=1e-13, seed=13)
    table = []
    for t in range(steps):
        ps = parity_vs_oracle(got[t], [r[t] for r in ref_sync])
        fr = parity_vs_oracle(got[t], [r[t] for r in ref_free])
        # oracle vs oracle: the perturbed chain's results in the "device" slot
        oo = parity_vs_oracle([(x, y, i) for (_, x, y, i) in (r[t] for r in ref_pert)], [r[t] for r in ref_free])
        sd = [state_diff(e["pst"][t], own[bi][t]) for bi, e in enumerate(rec["buckets"])]
        table.append({"step": t + 1, "resync": {k: ps[k] for k in ("qps", "status_equal", "iter_equal", "max_rel_x",
                                                                      "max_rel_y", "pass")},
                      "state_before_step": {"max_rel_xzy": max(a for a, _ in sd), "max_rel_rho": max(b for _, b in sd)},
                      "free": {k: fr[k] for k in ("status_equal", "iter_equal", "max_rel_x")},
                      "oracle_vs_oracle_1e-13": {k: oo[k] for k in ("status_equal", "iter_equal", "max_rel_x")}})
    return {"steps": table, "pass": bool(all(r["resync"]["pass"] for r in table)),
            "what": "resync: the oracle loads the device's persisted rho + scaled iterates before each closed-loop "
                    "step (ora_set_state), then the same osqp_update_A / _lin_cost / _bounds + solve -- identical "
                    "status and iterations, x and y within 1e-5 at every step; state_before_step: device vs the "
                    "oracle's own free-running state at that point; free: the two free-running chains; "
                    "oracle_vs_oracle_1e-13: the oracle chain against itself with the first step's q perturbed by "
                    "1e-13 relative (same per-step values)"}


def measured_traffic(build_id, qps, kernel, values_mode, workload):
    """HBM bytes per launch from the committed PMC summary (tools/pmc_summary.py), only when it was
    measured on this very library (its build_id equals impc_build_id()) and this workload; else
    (None, reason)."""
    name = "pmc_k_solve.json" if workload == "config3" else f"pmc_{workload}.json"
    path = os.path.join(ROOT, "profiles", name)
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None, f"no PMC summary (profiles/{name})"
    if pm.get("build_id") != build_id:
        return None, f"PMC summary is of build {pm.get('build_id')}, not the loaded library {build_id}"
    if pm.get("qps_per_launch") != qps or pm.get("kernel") != kernel or pm.get("values", "full") != values_mode or \
            pm.get("workload", "config3") != workload:
        return None, "PMC summary is of another workload / kernel / value mode"
    return pm.get("hbm_bytes_per_launch"), f"profiles/{name} (build {build_id}, {pm.get('source', '')})"


def parity_vs_oracle(results, ref):
    """The benched launch's results for the QPs the CPU baseline solved (the first k of each
    bucket) against the oracle's: identical status and iteration count, x and y within 1e-5
    relative (BASELINE.json north_star; inf-norm per QP, over QPs with a solution)."""
    n = st_eq = it_eq = 0
    worst_x = worst_y = 0.0
    for (x, y, info), (k, xo, yo, io) in zip(results, ref):
        x, y, info = x[:k], y[:k], info[:k]
        n += k
        st_eq += int((info["status_val"] == io["status_val"]).sum())
        it_eq += int((info["iter"] == io["iter"]).sum())
        ok = np.isin(io["status_val"], (1, 2, -2, -6))
        if ok.any():
            rx = np.abs(x - xo).max(axis=1) / np.maximum(np.abs(xo).max(axis=1), 1e-12)
            ry = np.abs(y - yo).max(axis=1) / np.maximum(np.abs(yo).max(axis=1), 1e-12)
            worst_x = max(worst_x, float(rx[ok].max()))
            worst_y = max(worst_y, float(ry[ok].max()))
    return {"qps": n, "status_equal": st_eq, "iter_equal": it_eq, "max_rel_x": worst_x, "max_rel_y": worst_y,
            "tolerance": 1e-5, "pass": bool(st_eq == n and it_eq == n and worst_x <= 1e-5 and worst_y <= 1e-5),
            "what": "the timed launch's x, y, status, iterations for the CPU baseline's QPs vs the oracle "
                    "(C restatement of OSQP 0.6.2; parity unpinned against the real libosqp, DESIGN.md 3)"}


def cpu_baseline(bks, settings, sample, threads):
    """The oracle (C restatement of OSQP 0.6.2, reference per-call pattern: setup + warm start +
    solve per QP) on `threads` host threads of the GPU box, over a bounded sample of the same
    workload (the first QPs of each bucket, bucket-proportional).  Returns (line object,
    [(k, x, y, info) per bucket])."""
    from oracle import osqp_oracle as ora
    total = sum(bk["values"]["q"].shape[0] for bk in bks)
    s = ora.settings_from(settings)
    t_all, n_all = 0.0, 0
    ref = []
    for bk in bks:
        B = bk["values"]["q"].shape[0]
        k = min(B, max(1, int(round(sample * B / total))))
        v = bk["values"]
        t = time.perf_counter()
        xo, yo, io = ora.solve_batch(bk["pattern"], v["Px"][:k], v["q"][:k], v["Ax"][:k], v["l"][:k], v["u"][:k], s,
                                     x_ws=None if bk.get("x_ws") is None else bk["x_ws"][:k], threads=threads)
        t_all += time.perf_counter() - t
        n_all += k
        ref.append((k, xo, yo, io))
    # per-QP latency on one thread, the reference's own measures: solveProblem only
    # (mpcPlanner.cpp:512-520) and setup + warm start + solve
    lat_s, lat_all = [], []
    bk = max(bks, key=lambda x: x["values"]["q"].shape[0])
    v = bk["values"]
    for i in range(min(128, v["q"].shape[0])):
        t = time.perf_counter()
        w = ora.Workspace(bk["pattern"], v["Px"][i], v["q"][i], v["Ax"][i], v["l"][i], v["u"][i], s)
        if bk.get("x_ws") is not None:
            w.warm_start(bk["x_ws"][i], np.zeros(int(bk["pattern"]["m"])))
        t1 = time.perf_counter()
        w.solve()
        t2 = time.perf_counter()
        w.close()
        lat_s.append(t2 - t1)
        lat_all.append(t2 - t)
    single = {"solve_p50_ms": 1e3 * float(np.median(lat_s)), "setup_solve_p50_ms": 1e3 * float(np.median(lat_all)),
              "sample": f"first {len(lat_s)} QPs of the K={bk['K']} bucket, one thread"}
    return {"value": n_all / t_all, "unit": "QP-solves/s", "cores": threads, "kind": "port", "single_qp": single,
            "host_cpus": os.cpu_count(), "cpu_model": cpu_info(),
            "sample": f"{n_all} QPs of the same workload (first of each bucket), one setup+warm-start+solve "
                      f"per QP, {threads} threads ({t_all:.1f} s wall)"}, ref


if __name__ == "__main__":
    main()
