#!/bin/bash
# Round 5: Ruiz reductions double-buffered (rzdb) and 3 x 3 Gauss-Jordan pivots on top (gj3):
# parity with gj3 (full GPU suite), then config 3 / config 5 A/B against the product.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05x; mkdir -p $O
IMPC_LIB_VARIANT=gj3 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gj3.log 2>&1 || { tail -30 $O/pytest_gj3.log; exit 1; }
tail -1 $O/pytest_gj3.log
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh base rzdb gj3 base rzdb gj3 || exit 1
mkdir -p $O/c3 && mv gpurun_out/exp/*.log $O/c3/
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh base rzdb gj3 || exit 1
mkdir -p $O/c5 && mv gpurun_out/exp/*.log $O/c5/
