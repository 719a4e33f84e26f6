#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?" | tee -a gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench.log 2>&1
echo "bench rc=$?" | tee -a gpurun_out/bench.log
tail -c 3000 gpurun_out/bench.log
