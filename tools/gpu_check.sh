#!/bin/bash
# GPU-box check run: parity tests, smoke, bench, kernel-trace profile.  Every GPU step has its own
# time limit and the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -c 2500 gpurun_out/bench.log
if [ -n "${PROFILE:-}" ]; then
  step rocprof
  cd /tmp || exit 1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  find "$R/gpurun_out/prof" -name "*kernel_stats.csv" -exec cat {} \;
fi
if [ -n "${PMC:-}" ]; then
  step pmc
  cd /tmp || exit 1
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o pmc -- python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-sample 0 > "$R/gpurun_out/pmc_fetch.log" 2>&1 || { tail -30 "$R/gpurun_out/pmc_fetch.log"; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o pmc -- python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-sample 0 > "$R/gpurun_out/pmc_write.log" 2>&1 || { tail -30 "$R/gpurun_out/pmc_write.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_fetch" "$R/gpurun_out/pmc_write" k_mpc_wave_group 65536 shared > "$R/gpurun_out/pmc_k_solve.json" && cat "$R/gpurun_out/pmc_k_solve.json"
fi
if [ -n "${CONFIGS:-}" ]; then
  step configs
  cd "$R" || exit 1
  timeout -k 10 600 python3 tools/bench_configs.py --steps 3 > gpurun_out/configs.log 2>&1 || { tail -30 gpurun_out/configs.log; exit 1; }
  cat gpurun_out/configs.log
fi
