#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05y
timeout -k 10 600 python -u -m pytest tests/test_closed_loop.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/r05y/pytest_cl.log 2>&1; rc=$?
tail -30 gpurun_out/r05y/pytest_cl.log; exit $rc
