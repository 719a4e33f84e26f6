#!/bin/bash
# Round-3 occupancy experiment: D/E off chip (offscl), and 3 teams per CU at <= 168 VGPRs (w3),
# against the product library; bench workload, identical iteration counts expected.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03e; mkdir -p $O; export TMPDIR=/tmp
for v in base offscl w3; do
  if [ $v = base ]; then unset IMPC_LIB_VARIANT; else export IMPC_LIB_VARIANT=$v; fi
  timeout -k 10 300 python3 -u bench.py --steps 2 --cpu-sample 0 --e2e-steps 0 > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$v.json') if l.startswith('{')][-1]); print('$v', round(d['value']), round(d['kernel_ms']['mean'],2), d['iters']['mean'])"
done
