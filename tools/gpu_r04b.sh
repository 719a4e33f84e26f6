#!/bin/bash
# Round 4: GPU suite + default bench line, then an A/B of a kernel variant (lib/libimpc_qp_$V.so,
# IMPC_LIB_VARIANT) against the product library on the bench workload: parity tests of the
# variant, then alternating bench runs (no CPU baseline / e2e).  Every step has its own limit.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; export TMPDIR=/tmp
O="$R/gpurun_out/${TAG:-r04b}"; mkdir -p "$O"
V="${V:-s1f}"
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -n 2 $O/pytest_gpu.log
  timeout -k 10 500 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
  cut -c1-600 $O/bench_default.json
fi
IMPC_LIB_VARIANT=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tail_seed3000.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$V.log 2>&1 || { tail -40 $O/pytest_$V.log; exit 1; }
tail -n 1 $O/pytest_$V.log
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --cpu-sample 0 --e2e-steps 0 > $O/ab_base_$r.json 2>> $O/ab.err || exit 1
  IMPC_LIB_VARIANT=$V timeout -k 10 300 python3 -u bench.py --steps 5 --cpu-sample 0 --e2e-steps 0 > $O/ab_${V}_$r.json 2>> $O/ab.err || exit 1
  python3 -c "import json,sys; [print(f, json.load(open(f))['kernel_ms']['mean'], json.load(open(f))['iters']['mean']) for f in sys.argv[1:]]" $O/ab_base_$r.json $O/ab_${V}_$r.json
done
