#!/bin/bash
# Round 5: the factorisation's 13-term products unrolled by 4 / 2 (6 scratch loads in the default
# horizon's ADMM loop) against the full unroll (12): config 3, then config 5's closed loop.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05u; mkdir -p $O
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh base f2u4 f2u2 base f2u4 f2u2 || exit 1
mkdir -p $O/c3 && mv gpurun_out/exp/*.log $O/c3/
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh base f2u4 base f2u4 || exit 1
mkdir -p $O/c5 && mv gpurun_out/exp/*.log $O/c5/
