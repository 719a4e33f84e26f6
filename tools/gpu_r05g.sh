#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05g
timeout -k 10 400 python -u -m pytest tests/test_live_loop.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/alone.log 2>&1; tail -5 gpurun_out/r05g/alone.log
timeout -k 10 400 python -u -m pytest tests/test_persistent.py tests/test_live_loop.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/after.log 2>&1; tail -5 gpurun_out/r05g/after.log
grep -n "replan [0-9]*:" gpurun_out/r05g/*.log | head
