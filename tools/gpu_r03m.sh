#!/bin/bash
# Round 3 closing evidence on the final kernel (3c26add): GPU suite, default bench line,
# rocprofv3 kernel-trace stats of the same command, HBM PMC passes (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; export TMPDIR=/tmp
O="$R/gpurun_out/r03m"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
cd /tmp || exit 1
B="$R/bench.py"; ARGS0="--cpu-sample 0 --e2e-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench -- python3 "$B" $ARGS0 > "$O/bench_traced.log" 2>&1 || { tail -20 "$O/bench_traced.log"; exit 1; }
find "$O/trace" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_bench.csv" \;
head -6 "$O/kernel_stats_bench.csv"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- python3 "$B" --steps 1 --warmup 0 $ARGS0 > "$O/pmc_fetch.log" 2>&1 || { tail -20 "$O/pmc_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- python3 "$B" --steps 1 --warmup 0 $ARGS0 > "$O/pmc_write.log" 2>&1 || { tail -20 "$O/pmc_write.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$O/pmc_fetch" "$O/pmc_write" k_mpc_wave_group 65536 shared > "$O/pmc_k_solve.json" && cat "$O/pmc_k_solve.json"
