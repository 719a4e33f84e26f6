#!/bin/bash
# Round-3 evidence for profiles/r03: GPU suite, the time-limit diagnosis on this tree, the section
# profile, rocprofv3 kernel-trace stats of the default bench command (the roofline's launch time),
# the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) and the SQ stall mix (two passes).
# Every step has its own time limit; the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; export TMPDIR=/tmp
O="$R/gpurun_out/${TAG:-r03f}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 120 python -u tools/tlim_diag.py . r03 > $O/tlim_r03.jsonl 2> $O/tlim.err || { tail -20 $O/tlim.err; exit 1; }
head -1 $O/tlim_r03.jsonl | cut -c1-200
if [ -f intent-mpc_amd/lib/libimpc_qp_prof.so ]; then
  IMPC_LIB_VARIANT=prof timeout -k 10 300 python -u tools/section_profile.py > $O/section_profile.txt 2> $O/sec.err || { tail -20 $O/sec.err; exit 1; }
fi
timeout -k 10 400 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
cd /tmp || exit 1
B="$R/bench.py"
ARGS0="--cpu-sample 0 --e2e-steps 0"
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench -- python3 "$B" $ARGS0 > "$O/bench_traced.log" 2>&1 || { tail -20 "$O/bench_traced.log"; exit 1; }
find "$O/trace" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_bench.csv" \;
head -6 "$O/kernel_stats_bench.csv"
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
for k in sorted(tot): print(f"{k:24s} {tot[k]:.4g}")
if tot.get("SQ_WAVE_CYCLES"):
    print(f"WAIT_ANY / WAVE_CYCLES   {tot['SQ_WAIT_ANY'] / tot['SQ_WAVE_CYCLES']:.3f}")
    print(f"ACTIVE_INST_VALU / WAVE_CYCLES {tot['SQ_ACTIVE_INST_VALU'] / tot['SQ_WAVE_CYCLES']:.3f}")
PY
cat "$O/sq_counters.txt"
