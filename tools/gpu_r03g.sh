#!/bin/bash
# Round-3: twisted elimination kernel -- parity tests of the structured path, then the bench
# (default, and the FIFO / shard lines) against the round's earlier numbers.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_queue_order.py tests/test_persistent.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_core.log 2>&1 || { tail -40 $O/pytest_core.log; exit 1; }
tail -n 1 $O/pytest_core.log
B="timeout -k 10 400 python3 -u bench.py"
$B --cpu-sample 0 --e2e-steps 0 > $O/bench.json 2> $O/b1.err || { tail -20 $O/b1.err; exit 1; }
$B --shard-of 8 --steps 5 --cpu-sample 0 --e2e-steps 0 > $O/shard8.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
for f in bench shard8; do
  python3 -c "import json; d=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', round(d['value']), round(d['kernel_ms']['mean'],2), d['iters']['mean'], d['roofline']['frac'])"
done
