#!/bin/bash
# Round-2 GPU check: new parity tests, bench (config3 default + config4), per-config rates.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== new tests"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_configs_gpu.py tests/test_device_builder.py tests/test_shim.py > gpurun_out/pytest_new.log 2>&1 || { tail -40 gpurun_out/pytest_new.log; exit 1; }
tail -5 gpurun_out/pytest_new.log
echo "== bench config3"
timeout -k 10 600 python bench.py > gpurun_out/bench3.log 2>&1 || { tail -30 gpurun_out/bench3.log; exit 1; }
tail -c 3000 gpurun_out/bench3.log
echo "== bench config4"
timeout -k 10 900 python bench.py --workload config4 --steps 2 --cpu-sample 0 > gpurun_out/bench4.log 2>&1 || { tail -30 gpurun_out/bench4.log; exit 1; }
tail -c 2000 gpurun_out/bench4.log
echo "== configs"
timeout -k 10 900 python tools/bench_configs.py --steps 3 > gpurun_out/configs.log 2>&1 || { tail -30 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log
