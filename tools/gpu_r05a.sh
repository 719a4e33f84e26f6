#!/bin/bash
# Round 5 first GPU pass: the replan C-ABI (impc_replan_run) tests -- Python mirror, C++ program,
# budget, pipeline -- plus the pool / set_active fixes, then the full-call replan rate.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest tests/test_replan_native.py tests/test_replan_branches.py \
    tests/test_replan_pipeline.py tests/test_replan_budget.py tests/test_shim.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r05a/pytest_replan.log 2>&1 || { tail -40 gpurun_out/r05a/pytest_replan.log; exit 1; }
tail -3 gpurun_out/r05a/pytest_replan.log
timeout -k 10 300 python -u tools/replan_bench.py --reps 5 > gpurun_out/r05a/replan_bench.json 2> gpurun_out/r05a/replan_bench.err || { tail -20 gpurun_out/r05a/replan_bench.err; exit 1; }
cat gpurun_out/r05a/replan_bench.json
