#!/bin/bash
# Round 4 evidence for profiles/r04 on the library in this tree (its impc_build_id is recorded in
# every summary): rocprofv3 kernel-trace stats of the default bench command, the two HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs), the SQ stall mix (two passes), the drop-in path's
# per-call cost (shim_test bench, 1000 calls), the config-4 / config-5 bench lines, per-config
# rates and the whole-replan rate.  Every step has its own time limit; the script stops at the
# first failure.  SKIP_SUITE unset: the GPU suite and the default bench line run first.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; export TMPDIR=/tmp
O="$R/gpurun_out/${TAG:-r04c}"; mkdir -p "$O"
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -n 1 $O/pytest_gpu.log
  timeout -k 10 500 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
  cut -c1-300 $O/bench_default.json
fi
python3 -c "import sys; sys.path.insert(0, 'intent-mpc_amd/python'); import impc; print(impc.lib.impc_build_id().decode())" > $O/build_id.txt
cat $O/build_id.txt
cd /tmp || exit 1
B="$R/bench.py"; ARGS0="--cpu-sample 0 --e2e-steps 0"
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench -- python3 "$B" $ARGS0 > "$O/bench_traced.log" 2>&1 || { tail -20 "$O/bench_traced.log"; exit 1; }
find "$O/trace" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_bench_default.csv" \;
head -6 "$O/kernel_stats_bench_default.csv"
grep '^{' "$O/bench_traced.log" > "$O/bench_default_traced.json" || true
echo "== pmc fetch"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- python3 "$B" --steps 1 --warmup 0 $ARGS0 > "$O/pmc_fetch.log" 2>&1 || { tail -20 "$O/pmc_fetch.log"; exit 1; }
echo "== pmc write"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- python3 "$B" --steps 1 --warmup 0 $ARGS0 > "$O/pmc_write.log" 2>&1 || { tail -20 "$O/pmc_write.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$O/pmc_fetch" "$O/pmc_write" k_mpc_wave_group 65536 shared > "$O/pmc_k_solve.json" && cat "$O/pmc_k_solve.json"
echo "== sq counters"
ARGS="--steps 1 --warmup 0 $ARGS0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d "$O/sq1" -o sq -- python3 "$B" $ARGS > "$O/sq1.log" 2>&1 || { tail -20 "$O/sq1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$O/sq2" -o sq -- python3 "$B" $ARGS > "$O/sq2.log" 2>&1 || { tail -20 "$O/sq2.log"; exit 1; }
python3 - "$O" <<'PY' > "$O/sq_counters.txt"
import csv, glob, sys, collections
tot = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_mpc_wave" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
print("# bench.py --steps 1 --warmup 0 (65,536 QPs, one grouped launch), k_mpc_wave_group, summed over dispatches")
print("# build " + open(sys.argv[1] + "/build_id.txt").read().strip())
for k in sorted(tot): print(f"{k:24s} {tot[k]:.4g}")
if tot.get("SQ_WAVE_CYCLES"):
    print(f"WAIT_ANY / WAVE_CYCLES   {tot['SQ_WAIT_ANY'] / tot['SQ_WAVE_CYCLES']:.3f}")
    print(f"ACTIVE_INST_VALU / WAVE_CYCLES {tot['SQ_ACTIVE_INST_VALU'] / tot['SQ_WAVE_CYCLES']:.3f}")
PY
cat "$O/sq_counters.txt"
cd "$R" || exit 1
echo "== shim per-call cost"
timeout -k 10 300 python -u -m pytest tests/test_shim.py -m gpu -k per_call -x -s -q --timeout 240 --timeout-method thread > $O/shim_bench.log 2>&1 || { tail -20 $O/shim_bench.log; exit 1; }
grep "host_wall_ms" $O/shim_bench.log | tail -1
echo "== config5 / config4 bench lines"
timeout -k 10 500 python3 -u bench.py --workload config5 > $O/bench_config5.json 2> $O/bench_config5.err || { tail -20 $O/bench_config5.err; exit 1; }
cut -c1-300 $O/bench_config5.json
timeout -k 10 500 python3 -u bench.py --workload config4 --cpu-sample 0 --e2e-steps 0 > $O/bench_config4.json 2> $O/bench_config4.err || { tail -20 $O/bench_config4.err; exit 1; }
cut -c1-300 $O/bench_config4.json
echo "== per-config rates, replan"
timeout -k 10 500 python3 -u tools/bench_configs.py --steps 3 > $O/configs_s3.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs_s3.jsonl | cut -c1-200
timeout -k 10 300 python3 -u tools/replan_bench.py > $O/replan_device.json 2> $O/replan.err || { tail -20 $O/replan.err; exit 1; }
cat $O/replan_device.json
echo "== small-batch latency"
timeout -k 10 300 python3 -u tools/latency_ab.py > $O/latency.jsonl 2> $O/latency.err || { tail -20 $O/latency.err; exit 1; }
cut -c1-160 $O/latency.jsonl
