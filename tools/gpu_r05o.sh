#!/bin/bash
# Round 5: factorisation latency variant (IMPC_FACT2) -- parity, setup cost, A/B on config 5
# (closed loop and full setup) and config 3.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05o; mkdir -p $O
IMPC_LIB_VARIANT=fact2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/parity_fact2.log 2>&1 || { tail -30 $O/parity_fact2.log; exit 1; }
tail -1 $O/parity_fact2.log
for v in base fact2; do
  if [ $v = base ]; then unset IMPC_LIB_VARIANT; else export IMPC_LIB_VARIANT=$v; fi
  for a in "40 10" "20 8"; do
    timeout -k 10 300 python -u tools/setup_cost.py $a 1024 > $O/sc_$v.tmp 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['workload'][:24], d['fit'], d['persistent_max_iter_1'])" $O/sc_$v.tmp $v
    cat $O/sc_$v.tmp >> $O/setup_cost_$v.jsonl
  done
done
unset IMPC_LIB_VARIANT
BARGS="--workload config5 --steps 5 --warmup 5 --receding-replay 0 --e2e-steps 0" STEPS=5 bash tools/exp.sh base fact2 base fact2 || exit 1
mkdir -p $O/c5loop && mv gpurun_out/exp/*.log $O/c5loop/
BARGS="--e2e-steps 0" STEPS=3 bash tools/exp.sh base fact2 base fact2 || exit 1
mkdir -p $O/c3 && mv gpurun_out/exp/*.log $O/c3/
