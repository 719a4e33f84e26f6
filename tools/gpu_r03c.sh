#!/bin/bash
# Round-3: the round-2 tree's own GPU suite (with a diagnostic print in its budget test) to
# reproduce the round-2 time-limit failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R/_r02tree" || exit 1
O=$R/gpurun_out/r03c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/pytest_r02_suite.log 2>&1
echo "rc=$?"
grep -E "TLIMDIAG|passed|failed" $O/pytest_r02_suite.log | tail -5
