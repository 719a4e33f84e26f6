#!/bin/bash
# Round-3: time-limit diagnosis (round-2 library vs current), then the new oracle-checked shim tests.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/tlim_diag.py _r02tree r02 > $O/tlim_r02.jsonl 2> $O/tlim_r02.err || { tail -20 $O/tlim_r02.err; exit 1; }
cat $O/tlim_r02.jsonl
timeout -k 10 120 python -u tools/tlim_diag.py . r03 > $O/tlim_r03.jsonl 2> $O/tlim_r03.err || { tail -20 $O/tlim_r03.err; exit 1; }
cat $O/tlim_r03.jsonl
timeout -k 10 300 python -u -m pytest tests/test_shim.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_shim.log 2>&1 || { tail -40 $O/pytest_shim.log; exit 1; }
tail -n 5 $O/pytest_shim.log
