#!/bin/bash
# Round 5: config 3 with the factorisation's round-4 loops (nof2: 4 scratch loads in the ADMM loop)
# against the product (FACT2: 12), alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh base nof2 base nof2 base nof2 || exit 1
mkdir -p gpurun_out/r05t && mv gpurun_out/exp/*.log gpurun_out/r05t/
