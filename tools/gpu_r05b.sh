#!/bin/bash
# Round 5: the long shape's compile-time W = 29 instance (N = 30, the live planner horizon):
# parity (N = 30 intent buckets, horizons, long-horizon chunks), then the live and config-5 bench
# lines on the same build.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05b
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "live_horizon or horizons or long_horizon" \
    --timeout 300 --timeout-method thread > gpurun_out/r05b/pytest_n30.log 2>&1 || { tail -40 gpurun_out/r05b/pytest_n30.log; exit 1; }
tail -3 gpurun_out/r05b/pytest_n30.log
timeout -k 10 600 python -u bench.py --workload live --steps 5 --warmup 1 --e2e-steps 0 --cpu-all-cores 0 \
    > gpurun_out/r05b/bench_live.json 2> gpurun_out/r05b/bench_live.err || { tail -20 gpurun_out/r05b/bench_live.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05b/bench_live.json')); print('live', d['value'], d['ms_per_step'], d['roofline']['frac'], d['iters'], d['parity']['pass'])"
timeout -k 10 600 python -u bench.py --workload config5 --steps 3 --warmup 1 --e2e-steps 0 --cpu-all-cores 0 \
    > gpurun_out/r05b/bench_c5.json 2> gpurun_out/r05b/bench_c5.err || { tail -20 gpurun_out/r05b/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05b/bench_c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms']['per_step'])"
