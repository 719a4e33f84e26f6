#!/bin/bash
# Round 4, first GPU call: the GPU suite on the pruned kernel + the default bench line (parity and
# build id in the line).  Each step has its own time limit; the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; export TMPDIR=/tmp
O="$R/gpurun_out/${TAG:-r04a}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -n 3 $O/pytest_gpu.log
timeout -k 10 500 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-400 $O/bench_default.json
