#!/bin/bash
# Round 3: A/B of the check-hoisted loop (variant chk) against the product, and small-batch
# latency of the one-ended (product) vs twisted (variant tw) elimination.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r03i; mkdir -p $O; export TMPDIR=/tmp
BARGS="--e2e-steps 0" bash tools/exp.sh base chk base chk || exit 1
for v in base tw; do
  if [ $v = base ]; then unset IMPC_LIB_VARIANT; else export IMPC_LIB_VARIANT=$v; fi
  timeout -k 10 300 python3 -u tools/latency_ab.py > $O/lat_$v.jsonl 2> $O/lat_$v.err || { tail -20 $O/lat_$v.err; exit 1; }
  cut -c1-220 $O/lat_$v.jsonl
done
