#!/bin/bash
# Round 5 item 3: the default horizon's (W = 19) stage recursions in chunks (variant c19,
# -DIMPC_CHUNK19=1: chunks of 6 / 6 / 6 / 1 on the four wavefronts) against the product's
# single-wavefront sweeps, config-3 bench workload, alternating runs; then the SQ counters of both.
cd "$GRAFT_REPO_ROOT" || exit 1
BARGS="--e2e-steps 0 --cpu-all-cores 0" STEPS=3 bash tools/exp.sh c19 base c19 base || exit 1
mkdir -p gpurun_out/r05c && cp gpurun_out/exp/c19.log gpurun_out/exp/base.log gpurun_out/r05c/
PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  BARGS="--e2e-steps 0 --cpu-all-cores 0" STEPS=1 bash tools/exp.sh c19 base || exit 1
cp -r gpurun_out/exp/pmc_c19.log gpurun_out/exp/pmc_base.log gpurun_out/r05c/ 2>/dev/null
