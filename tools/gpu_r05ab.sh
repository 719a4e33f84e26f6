#!/bin/bash
# Round 5: the long shape's factorisation products unrolled by 4 (u3) against full unroll.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ab; mkdir -p $O
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh base u3 base u3 || exit 1
mkdir -p $O/c5 && mv gpurun_out/exp/*.log $O/c5/
BARGS="--workload live --e2e-steps 0" STEPS=3 bash tools/exp.sh base u3 || exit 1
mkdir -p $O/live && mv gpurun_out/exp/*.log $O/live/
