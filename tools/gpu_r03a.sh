#!/bin/bash
# Round-3 first check: full GPU suite (incl. the strict replan time-limit tests), smoke, default
# bench.  Stops at the first failure; every GPU step has its own time limit.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -n 3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-600 $O/bench_default.json
