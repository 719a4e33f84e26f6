#!/bin/bash
# Round 5: LLVM scheduler strategies on the current kernel (config 3, alternating), then config 5.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
bash tools/exp.sh base minreg mclause base minreg mclause 2>&1 | tee gpurun_out/exp/sched_c3.txt || exit 1
mkdir -p gpurun_out/exp/c5
BARGS="--workload config5 --steps 5 --receding-replay 0" STEPS=5 bash tools/exp.sh base minreg mclause 2>&1 | tee gpurun_out/exp/sched_c5.txt
