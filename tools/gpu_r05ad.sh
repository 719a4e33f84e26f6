#!/bin/bash
# Round 5: SQ counters of the default line's launch (config 3) on the final build, two passes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r05ad"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp || exit 1
A="--steps 1 --warmup 0 --cpu-sample 0 --e2e-steps 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d "$O/sq1" -o pmc -- python3 "$R/bench.py" $A > "$O/sq1.log" 2>&1 || { tail -20 "$O/sq1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$O/sq2" -o pmc -- python3 "$R/bench.py" $A > "$O/sq2.log" 2>&1 || { tail -20 "$O/sq2.log"; exit 1; }
python3 - "$O" > "$O/sq_counters_config3.txt" <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
bid = None
for ln in open(f"{o}/sq1.log"):
    if ln.startswith("{") and '"roofline"' in ln:
        bid = json.loads(ln)["roofline"]["build_id"]
print(f"rocprofv3 --pmc, two passes, bench.py --steps 1 --warmup 0 (config 3, 65,536 QPs), build {bid}")
print("k_mpc_wave_group (one launch), summed over the GPU's counter instances")
tot = {}
for p in ("sq1", "sq2"):
    for f in glob.glob(f"{o}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mpc_wave_group" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot): print(f"{k:24s} {tot[k]:.6g}")
print(f"WAIT_ANY/WAVE_CYCLES {tot['SQ_WAIT_ANY']/tot['SQ_WAVE_CYCLES']:.3f}  ACTIVE_INST_VALU/WAVE_CYCLES {tot['SQ_ACTIVE_INST_VALU']/tot['SQ_WAVE_CYCLES']:.3f}")
PY
cat "$O/sq_counters_config3.txt"
