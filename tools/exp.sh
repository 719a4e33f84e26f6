#!/bin/bash
# Kernel-variant A/B on the GPU box: bench value per variant (lib/libimpc_qp_<v>.so; "base" = the
# product library), optional PMC pass (PMC="SQ_... SQ_...") of each.  Stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
mkdir -p gpurun_out/exp; export TMPDIR=/tmp
# a variant "env:NAME=VALUE" runs the product library with that environment variable set
prev=
for v in "$@"; do
  unset IMPC_LIB_VARIANT
  [ -n "$prev" ] && unset "$prev"; prev=
  case "$v" in
    base) ;;
    env:*) kv=${v#env:}; export "$kv"; prev=${kv%%=*}; v=${kv//=/_} ;;
    *) export IMPC_LIB_VARIANT=$v ;;
  esac
  timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --cpu-sample 0 ${BARGS:-} > gpurun_out/exp/$v.log 2>&1 || { tail -20 gpurun_out/exp/$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), d['kernel_ms'], d['iters']['mean'])" gpurun_out/exp/$v.log $v
  if [ -n "${PMC:-}" ]; then
    ( cd /tmp && timeout -k 10 120 rocprofv3 --pmc $PMC --output-format csv -d "$R/gpurun_out/exp/pmc_$v" -o p -- python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-sample 0 ${BARGS:-} > "$R/gpurun_out/exp/pmc_$v.log" 2>&1 ) || { tail -20 gpurun_out/exp/pmc_$v.log; exit 1; }
    python3 - "$R/gpurun_out/exp/pmc_$v" <<'PY'
import csv,glob,sys,collections
t=collections.defaultdict(float)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_mpc_wave" in r["Kernel_Name"]: t[r["Counter_Name"]]+=float(r["Counter_Value"])
print({k:f"{v:.4g}" for k,v in t.items()})
PY
  fi
done
