#!/bin/bash
# Structured-kernel parity (grouped launches incl. config 4 / 5), bench config3 + config4, per-config rates.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_persistent.py tests/test_replan_pipeline.py > gpurun_out/pytest_b.log 2>&1 || { tail -40 gpurun_out/pytest_b.log; exit 1; }
tail -2 gpurun_out/pytest_b.log
timeout -k 10 600 python bench.py --cpu-sample 0 > gpurun_out/bench3.log 2>&1 || { tail -30 gpurun_out/bench3.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench3.log').read().strip().splitlines()[-1]);print('config3',round(d['value']),d['kernel_ms']['mean'],d['iters']['mean'])"
timeout -k 10 900 python bench.py --workload config4 --steps 2 --cpu-sample 0 > gpurun_out/bench4.log 2>&1 || { tail -30 gpurun_out/bench4.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench4.log').read().strip().splitlines()[-1]);print('config4',round(d['value']),d['kernel_ms']['mean'],d['iters']['mean'],d['cost_allgather'])"
timeout -k 10 900 python tools/bench_configs.py --steps 3 > gpurun_out/configs.log 2>&1 || { tail -30 gpurun_out/configs.log; exit 1; }
cut -c1-220 gpurun_out/configs.log
