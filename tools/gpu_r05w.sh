#!/bin/bash
# Round 5: IMPC_FACT3 (E_k in registers, B_k double-buffered, one barrier less per stage) on top of
# the Ruiz-pass merge (rz): parity with the variant, then config 3 / config 5 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05w; mkdir -p $O
IMPC_LIB_VARIANT=f3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_persistent.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/parity_f3.log 2>&1 || { tail -30 $O/parity_f3.log; exit 1; }
tail -1 $O/parity_f3.log
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh rz f3 rz f3 base || exit 1
mkdir -p $O/c3 && mv gpurun_out/exp/*.log $O/c3/
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh rz f3 || exit 1
mkdir -p $O/c5 && mv gpurun_out/exp/*.log $O/c5/
