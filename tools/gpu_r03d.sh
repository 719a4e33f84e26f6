#!/bin/bash
# Round-3: GPU suite on the queue-order / zero-dual warm-start library, then bench lines:
# default (config 3 strong, longest-first queue), FIFO A/B, rank-0 shard studies of the 8-way
# splits of config 3 and config 4 (longest-first vs FIFO).  Stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
B="timeout -k 10 400 python3 -u bench.py"
$B > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-400 $O/bench_default.json
$B --queue fifo --cpu-sample 0 --e2e-steps 0 > $O/bench_fifo.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
$B --shard-of 8 --steps 5 --cpu-sample 0 --e2e-steps 0 > $O/shard8_c3_longest.json 2> $O/b3.err || { tail -20 $O/b3.err; exit 1; }
$B --shard-of 8 --steps 5 --queue fifo --cpu-sample 0 --e2e-steps 0 > $O/shard8_c3_fifo.json 2> $O/b4.err || { tail -20 $O/b4.err; exit 1; }
$B --workload config4 --cpu-sample 0 --e2e-steps 0 > $O/c4_longest.json 2> $O/b5.err || { tail -20 $O/b5.err; exit 1; }
$B --workload config4 --shard-of 8 --steps 5 --cpu-sample 0 --e2e-steps 0 > $O/shard8_c4_longest.json 2> $O/b6.err || { tail -20 $O/b6.err; exit 1; }
$B --workload config4 --shard-of 8 --steps 5 --queue fifo --cpu-sample 0 --e2e-steps 0 > $O/shard8_c4_fifo.json 2> $O/b7.err || { tail -20 $O/b7.err; exit 1; }
for f in bench_fifo shard8_c3_longest shard8_c3_fifo c4_longest shard8_c4_longest shard8_c4_fifo; do
  python3 -c "import json,sys; d=json.load(open('$O/$f.json')); print('$f', round(d['value']), round(d['ms_per_step'],2), d['iters']['max'])"
done
