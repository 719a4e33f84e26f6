#!/bin/bash
# Two rocprofv3 --pmc passes of SQ counters over a reduced bench run (structured kernel stall mix).
R="$GRAFT_REPO_ROOT"; cd /tmp || exit 1; export TMPDIR=/tmp
ARGS="--instances 2048 --steps 1 --warmup 0 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d "$R/gpurun_out/sq1" -o sq -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/sq1.log" 2>&1 || { tail -20 "$R/gpurun_out/sq1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$R/gpurun_out/sq2" -o sq -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/sq2.log" 2>&1 || { tail -20 "$R/gpurun_out/sq2.log"; exit 1; }
python3 - "$R/gpurun_out" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_mpc_wave" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot): print(f"{k:24s} {tot[k]:.4g}")
PY
