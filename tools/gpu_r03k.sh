#!/bin/bash
# Round 3, final kernel (branch-free phases, v_max projections, counted inner loop): queue-order tests over every kernel class, per-config rates, the rank-0
# shard studies of config 3 / config 4 and the config-4 whole job.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_queue_order.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_queue.log 2>&1 || { tail -40 $O/pytest_queue.log; exit 1; }
tail -n 1 $O/pytest_queue.log
timeout -k 10 600 python3 -u tools/bench_configs.py --steps 3 > $O/configs_s3.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cut -c1-200 $O/configs_s3.jsonl
B="timeout -k 10 400 python3 -u bench.py --cpu-sample 0 --e2e-steps 0"
$B --shard-of 8 --steps 5 > $O/shard8_c3.json 2> $O/b1.err || { tail -20 $O/b1.err; exit 1; }
$B --workload config4 > $O/c4.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
$B --workload config4 --shard-of 8 --steps 5 > $O/shard8_c4.json 2> $O/b3.err || { tail -20 $O/b3.err; exit 1; }
for f in shard8_c3 c4 shard8_c4; do
  python3 -c "import json; d=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', round(d['value']), round(d['ms_per_step'],2), d['iters']['mean'])"
done
timeout -k 10 300 python3 -u tools/latency_ab.py > $O/lat_base.jsonl 2> $O/lat.err || { tail -20 $O/lat.err; exit 1; }
cut -c1-200 $O/lat_base.jsonl
