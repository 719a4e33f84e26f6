#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05h
timeout -k 10 500 python -u tools/repeat_live.py 6 > gpurun_out/r05h/repeat.log 2>&1; tail -8 gpurun_out/r05h/repeat.log
