#!/bin/bash
# Round 5: the Ruiz passes with the |A| write moved into the previous pass (one barrier less per
# pass): parity with the variant, then config 3 and config 5 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05v; mkdir -p $O
IMPC_LIB_VARIANT=rz timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_persistent.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/parity_rz.log 2>&1 || { tail -30 $O/parity_rz.log; exit 1; }
tail -1 $O/parity_rz.log
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh base rz base rz || exit 1
mkdir -p $O/c3 && mv gpurun_out/exp/*.log $O/c3/
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh base rz || exit 1
mkdir -p $O/c5 && mv gpurun_out/exp/*.log $O/c5/
