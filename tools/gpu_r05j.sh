#!/bin/bash
# Round 5: persistent matrix-update tests (q after the matrices), the closed-loop config-5 line,
# then the long-horizon (W = 39) phase costs: each IMPC_DUP variant runs one phase twice per ADMM
# iteration; config 5's QPs with a full setup per step (--receding 0: identical iterations in every
# variant), alternating with the product library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05j
timeout -k 10 400 python -u -m pytest tests/test_persistent.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05j/persist.log 2>&1; tail -3 gpurun_out/r05j/persist.log
timeout -k 10 900 python -u bench.py --workload config5 --steps 10 --warmup 10 --e2e-steps 0 --cpu-all-cores 0 \
    > gpurun_out/r05j/bench_c5.json 2> gpurun_out/r05j/bench_c5.err || { tail -20 gpurun_out/r05j/bench_c5.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05j/bench_c5.json'))
print('c5', round(d['value']), d['ms_per_step'], d['roofline']['frac'], [round(v) for v in d['kernel_ms']['per_step']])
p=d['parity']; print(d['receding_steps']['replay_bitwise_equal'], {k:p[k] for k in ('qps','status_equal','iter_equal','max_rel_x','max_rel_y','pass')}, d['cpu_baseline']['value'])
print([ (c['iter_equal'], c['status_equal']) for c in p['chain']])
PY
BARGS="--workload config5 --receding 0 --e2e-steps 0" STEPS=2 bash tools/exp.sh base dupfwd dupbwd dups3 dups5 duprhs dups1 dupprod dupchk dupfac base
