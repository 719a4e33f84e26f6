#!/bin/bash
# Round 5: setup cost against iteration cost (per-QP device latency fit) at N = 40, 30 and 20.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05n; mkdir -p $O
for a in "40 10" "30 8" "20 8"; do
  timeout -k 10 300 python -u tools/setup_cost.py $a 1024 >> $O/setup_cost.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
cat $O/setup_cost.jsonl
