#!/bin/bash
# Round 5: live replan loop on the reference's benchmark path (test + rate), then r05b (N = 30
# parity, live + closed-loop config-5 bench lines), then r05c (chunked default-horizon A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_persistent.py tests/test_live_loop.py -m gpu -x -v --timeout 500 --timeout-method thread \
    > gpurun_out/r05d/pytest_live.log 2>&1 || { tail -40 gpurun_out/r05d/pytest_live.log; exit 1; }
tail -2 gpurun_out/r05d/pytest_live.log
timeout -k 10 600 python -u tools/live_loop.py > gpurun_out/r05d/live_loop.json 2> gpurun_out/r05d/live_loop.err || { tail -20 gpurun_out/r05d/live_loop.err; exit 1; }
cat gpurun_out/r05d/live_loop.json
bash tools/gpu_r05b.sh || exit 1
bash tools/gpu_r05c.sh
