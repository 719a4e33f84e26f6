#!/bin/bash
# Round 5: the live-loop test after the persistent-workspace tests (the order that failed), with
# the failure dump.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05s
timeout -k 10 600 python -u -m pytest tests/test_persistent.py tests/test_live_loop.py -m gpu -x -q --timeout 500 --timeout-method thread \
    > gpurun_out/r05s/pytest_live.log 2>&1; echo rc=$?
tail -5 gpurun_out/r05s/pytest_live.log
ls gpurun_out/*.npz 2>/dev/null
exit 0
