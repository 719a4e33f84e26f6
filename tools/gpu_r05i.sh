#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05i
timeout -k 10 300 python -u -m pytest tests/test_shim.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r05i/shim.log 2>&1; tail -3 gpurun_out/r05i/shim.log
timeout -k 10 900 python -u bench.py --workload config5 --steps 10 --warmup 10 --e2e-steps 0 --cpu-all-cores 0 \
    > gpurun_out/r05i/bench_c5.json 2> gpurun_out/r05i/bench_c5.err || { tail -20 gpurun_out/r05i/bench_c5.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05i/bench_c5.json'))
print('c5', round(d['value']), d['ms_per_step'], d['roofline']['frac'], [round(v) for v in d['kernel_ms']['per_step']])
for s in d['receding_steps']['steps']: print(s['step'], round(s['mean_iter'],1), s['status_counts'])
p=d['parity']; print(d['receding_steps']['replay_bitwise_equal'], {k:p[k] for k in ('qps','status_equal','iter_equal','max_rel_x','max_rel_y','pass')}, d['cpu_baseline']['value'])
print([ (c['iter_equal'], c['status_equal']) for c in p['chain']])
PY
