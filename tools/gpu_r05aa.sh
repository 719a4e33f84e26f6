#!/bin/bash
# Round 5: the factorisation assembly's codes 8 / 12 per batch (fewer global round trips for the
# obstacle-heavy entries) against 4.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05aa; mkdir -p $O
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh base f2b8 f2b12 base f2b8 f2b12 || exit 1
mkdir -p $O/c3 && mv gpurun_out/exp/*.log $O/c3/
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh base f2b8 f2b12 || exit 1
mkdir -p $O/c5 && mv gpurun_out/exp/*.log $O/c5/
