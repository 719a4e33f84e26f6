#!/bin/bash
# Round 4 chunk fix-up: the long-horizon GPU parity tests on the product library, then A/B of the
# chunk re-run kernel (variant "rerun", the parent commit) against the product ("base") on the
# config-5 and config-3 bench workloads.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exp/c5 gpurun_out/exp/c3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp/pytest_fix.log 2>&1 || { tail -30 gpurun_out/exp/pytest_fix.log; exit 1; }
tail -2 gpurun_out/exp/pytest_fix.log
BARGS="--workload config5 --e2e-steps 0" STEPS=2 bash tools/exp.sh rerun base rerun base || exit 1
for v in rerun base; do cp gpurun_out/exp/$v.log gpurun_out/exp/c5/$v.log; done
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh rerun base || exit 1
for v in rerun base; do cp gpurun_out/exp/$v.log gpurun_out/exp/c3/$v.log; done
