#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05f
timeout -k 10 400 python -u tools/diag_live.py > gpurun_out/r05f/diag.log 2>&1; tail -12 gpurun_out/r05f/diag.log
timeout -k 10 600 python -u bench.py --workload config5 --steps 10 --warmup 1 --e2e-steps 0 --cpu-all-cores 0 \
    > gpurun_out/r05f/bench_c5.json 2> gpurun_out/r05f/bench_c5.err || { tail -20 gpurun_out/r05f/bench_c5.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05f/bench_c5.json'))
print('c5', round(d['value']), d['ms_per_step'], d['roofline']['frac'], [round(v) for v in d['kernel_ms']['per_step']])
for s in d['receding_steps']['steps']: print(s['step'], s['mean_iter'], s['status_counts'])
print(d['receding_steps']['replay_bitwise_equal'], d['parity'], d['cpu_baseline']['value'])
PY
bash tools/gpu_r05c.sh
