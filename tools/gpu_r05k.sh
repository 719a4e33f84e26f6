#!/bin/bash
# Round 5: five-chunk long-horizon sweeps (IMPC_CHUNK5 variant) -- parity on the GPU, then A/B
# against the product on config 5 (full setup per step, W = 39) and the live N = 30 workload (W = 29).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05k
IMPC_LIB_VARIANT=chunk5 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "long_horizon or live_horizon" > gpurun_out/r05k/parity_chunk5.log 2>&1 || { tail -30 gpurun_out/r05k/parity_chunk5.log; exit 1; }
tail -2 gpurun_out/r05k/parity_chunk5.log
BARGS="--workload config5 --receding 0 --e2e-steps 0" STEPS=2 bash tools/exp.sh base chunk5 base chunk5 || exit 1
mkdir -p gpurun_out/r05k/c5 && mv gpurun_out/exp/*.log gpurun_out/r05k/c5/
BARGS="--workload live --e2e-steps 0" STEPS=3 bash tools/exp.sh base chunk5 base chunk5 || exit 1
mkdir -p gpurun_out/r05k/live && mv gpurun_out/exp/*.log gpurun_out/r05k/live/
