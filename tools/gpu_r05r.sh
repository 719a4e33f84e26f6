#!/bin/bash
# Round 5 evidence run (five chunks + factorisation latency form): PMC traffic of config 3 and of config 5's closed
# loop (summaries also written into this box's profiles/ so the bench lines below quote them), SQ
# counters of config 5, the GPU suite, smoke, the bench lines (default, config 5, live) and the
# rocprofv3 kernel traces of the default and config-5 benches.  Stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O="$R/gpurun_out/r05r"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp || exit 1
A3="--steps 1 --warmup 0 --cpu-sample 0 --e2e-steps 0"
A5="--workload config5 --steps 1 --warmup 10 --receding-replay 0 --cpu-sample 0 --e2e-steps 0"
pmc() {  # name counter args...
  local n=$1 c=$2; shift 2
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$O/$n" -o pmc -- python3 "$R/bench.py" "$@" > "$O/$n.log" 2>&1 || { tail -20 "$O/$n.log"; return 1; }
}
pmc pmc3_fetch FETCH_SIZE $A3 && pmc pmc3_write WRITE_SIZE $A3 || exit 1
python3 "$R/tools/pmc_summary.py" "$O/pmc3_fetch" "$O/pmc3_write" k_mpc_wave_group 65536 shared config3 > "$O/pmc_k_solve.json" || exit 1
cp "$O/pmc_k_solve.json" "$R/profiles/pmc_k_solve.json"
pmc pmc5_fetch FETCH_SIZE $A5 && pmc pmc5_write WRITE_SIZE $A5 || exit 1
python3 "$R/tools/pmc_summary.py" "$O/pmc5_fetch" "$O/pmc5_write" k_mpc_wave_group 65536 shared config5 last > "$O/pmc_config5.json" || exit 1
cp "$O/pmc_config5.json" "$R/profiles/pmc_config5.json"
pmc sq5_1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" $A5 || exit 1
pmc sq5_2 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" $A5 || exit 1
python3 - "$O" > "$O/sq_counters_config5.txt" <<'PY'
import csv, glob, sys
o = sys.argv[1]
print("rocprofv3 --pmc, two passes, bench.py --workload config5 --steps 1 --warmup 10 --receding-replay 0:")
print("k_mpc_wave_group, the last dispatch (closed-loop step 11), summed over the GPU's counter instances")
for p in ("sq5_1", "sq5_2"):
    vals = {}
    for f in glob.glob(f"{o}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mpc_wave_group" in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"]); vals.setdefault(d, {}); n = r["Counter_Name"]
                vals[d][n] = vals[d].get(n, 0.0) + float(r["Counter_Value"])
    last = vals[max(vals)]
    for k in sorted(last): print(f"{k:24s} {last[k]:.6g}")
PY
cat "$O/sq_counters_config5.txt"
cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -20 "$O/bench_default.err"; exit 1; }
timeout -k 10 900 python bench.py --workload config5 --steps 10 --warmup 10 > "$O/bench_config5.json" 2> "$O/bench_config5.err" || { tail -20 "$O/bench_config5.err"; exit 1; }
timeout -k 10 600 python bench.py --workload live --steps 3 --warmup 1 > "$O/bench_live.json" 2> "$O/bench_live.err" || { tail -20 "$O/bench_live.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
for n in ("bench_default", "bench_config5", "bench_live"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    r = d["roofline"]
    print(n, round(d["value"]), round(d["ms_per_step"], 2), r["frac"], r["traffic"], d["cpu_baseline"] and round(d["cpu_baseline"]["value"]),
          d["parity"] and d["parity"]["pass"])
PY
cd /tmp || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_default" -o kt -- python3 "$R/bench.py" --cpu-sample 0 --e2e-steps 0 > "$O/kt_default.log" 2>&1 || { tail -20 "$O/kt_default.log"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_config5" -o kt -- python3 "$R/bench.py" --workload config5 --steps 10 --warmup 10 --receding-replay 0 --cpu-sample 0 --e2e-steps 0 > "$O/kt_config5.log" 2>&1 || { tail -20 "$O/kt_config5.log"; exit 1; }
find "$O/kt_default" "$O/kt_config5" -name "*kernel_stats.csv" -exec head -4 {} \;
cd "$R" || exit 1
timeout -k 10 600 python bench.py --workload config5 --receding 0 --steps 2 --warmup 1 --e2e-steps 0 --cpu-sample 0 > "$O/bench_config5_fullsetup.json" 2> "$O/bench_config5_fullsetup.err" || { tail -20 "$O/bench_config5_fullsetup.err"; exit 1; }
for a in "40 10" "30 8" "20 8"; do
  timeout -k 10 300 python -u tools/setup_cost.py $a 1024 >> "$O/setup_cost.jsonl" 2> "$O/sc.err" || { tail -20 "$O/sc.err"; exit 1; }
done
timeout -k 10 600 python -u tools/live_loop.py > "$O/live_loop.json" 2> "$O/live_loop.err" || { tail -20 "$O/live_loop.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
d = json.load(open(f"{o}/bench_config5_fullsetup.json")); print("fullsetup", round(d["value"]), d["ms_per_step"], d["roofline"]["frac"])
for ln in open(f"{o}/setup_cost.jsonl"): d = json.loads(ln); print(d["workload"][:28], d["fit"])
d = json.load(open(f"{o}/live_loop.json")); print("live loop", d["replans_per_s"], d["fanout_replan_s_median"])
PY
