#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05e
timeout -k 10 300 python -u tools/diag_live.py > gpurun_out/r05e/diag.log 2>&1; tail -30 gpurun_out/r05e/diag.log
bash tools/gpu_r05b.sh || exit 1
bash tools/gpu_r05c.sh
