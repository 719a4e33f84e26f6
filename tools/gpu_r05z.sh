#!/bin/bash
# Round 5: setup cost against the horizon on the default shape (N = 5..20, K = 8): the slope is the
# per-stage factorisation cost; the scaling=0 runs isolate the Ruiz passes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05z; mkdir -p $O
for a in "5 8 1024 10" "10 8 1024 10" "15 8 1024 10" "20 8 1024 10" "20 8 1024 0" "10 8 1024 0"; do
  timeout -k 10 300 python -u tools/setup_cost.py $a >> $O/setup_cost_N.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
for ln in open("gpurun_out/r05z/setup_cost_N.jsonl"):
    d = json.loads(ln); print(d["workload"][:60], round(d["fit"]["setup_ms"] * 1e3, 1), "us", round(d["fit"]["per_iter_us"], 3), d["persistent_max_iter_1"]["first_solve_ms"])
PY
