#!/bin/bash
# Round 5: setup cost split -- Ruiz passes on / off (settings.scaling 10 / 0) at N = 40 and 20.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05p; mkdir -p $O
for a in "40 10 1024 10" "40 10 1024 0" "20 8 1024 10" "20 8 1024 0"; do
  timeout -k 10 300 python -u tools/setup_cost.py $a > $O/sc.tmp 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['workload'][:50], d['fit'], d['persistent_max_iter_1'], d['build_id'])" $O/sc.tmp
  cat $O/sc.tmp >> $O/setup_cost.jsonl
done
