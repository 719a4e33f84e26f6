#!/bin/bash
# A/B of kernel variants + the structured-kernel parity tests of the product library.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_persistent.py > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
bash tools/exp.sh "$@"
