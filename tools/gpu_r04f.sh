#!/bin/bash
# Round 4 chunked long-horizon recursions: the GPU suite on the product library, then A/B of the
# previous kernel (variant "orig", built from the parent commit's sources) against the product
# ("base") on the config-5 and config-3 bench workloads.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exp/c5 gpurun_out/exp/c3
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/exp/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/exp/pytest_gpu.log
fi
BARGS="--workload config5 --e2e-steps 0" STEPS=2 bash tools/exp.sh ${C5VARS:-orig base orig base} || exit 1
for v in ${C5VARS:-orig base}; do cp gpurun_out/exp/$v.log gpurun_out/exp/c5/$v.log; done
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh ${C3VARS:-orig base orig base} || exit 1
for v in ${C3VARS:-orig base}; do cp gpurun_out/exp/$v.log gpurun_out/exp/c3/$v.log; done
