#!/bin/bash
# Round 6 GPU runs, one phase per call: bash tools/gpu_r06.sh <phase> [args].  Every GPU step runs
# under its own time limit; the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
mkdir -p gpurun_out/r06; export TMPDIR=/tmp
O=gpurun_out/r06
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
case "$1" in
  tests)  # tests/<files...> given after the phase, then (after "--") an A/B of library variants
    shift; T=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do T+=("$1"); shift; done; [ "${1:-}" = "--" ] && shift
    timeout -k 10 1000 $PYT "${T[@]}" > $O/pytest_sel.log 2>&1 || { tail -80 $O/pytest_sel.log; exit 1; }
    tail -3 $O/pytest_sel.log
    [ $# -gt 0 ] && bash tools/exp.sh "$@"
    ;;
  lds)  # LDS bank conflicts per phase: each phase-duplication variant (lib/libimpc_qp_dup<id>.so,
        # IMPC_DUP = section id) against the product, bench value + one PMC pass each
    shift
    PMC="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS" BARGS="--e2e-steps 0" \
      bash tools/exp.sh "$@" 2>&1 | tee $O/lds_phases.txt
    ;;
  gpu)  # the whole -m gpu suite
    timeout -k 10 1000 $PYT -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
    tail -3 $O/pytest_gpu.log
    ;;
  c5)  # config 5's closed loop with the step-by-step chain parity
    timeout -k 10 900 python -u bench.py --workload config5 --steps 10 --warmup 10 > $O/bench_config5.json.log 2>&1 \
      || { tail -30 $O/bench_config5.json.log; exit 1; }
    tail -1 $O/bench_config5.json.log > $O/bench_config5.json
    ;;
  meas)  # replan / live-loop measurements of the final build and the NON_CVX trace
    timeout -k 10 600 python -u tools/trace_noncvx.py > $O/noncvx_trace.json 2> $O/noncvx_trace.err || { tail -30 $O/noncvx_trace.err; exit 1; }
    for I in 8192 16 1; do
      R=5; [ $I -lt 100 ] && R=30
      timeout -k 10 300 python -u tools/replan_bench.py --instances $I --reps $R > $O/replan_full_call_I$I.json 2> $O/replan_I$I.err || { tail -30 $O/replan_I$I.err; exit 1; }
      ( cd ab_r05 && timeout -k 10 300 python -u tools/replan_bench.py --instances $I --reps $R ) > $O/replan_full_call_I${I}_r05.json 2> $O/replan_I${I}_r05.err || { tail -30 $O/replan_I${I}_r05.err; exit 1; }
    done
    timeout -k 10 600 python -u tools/live_loop.py > $O/live_loop.json 2> $O/live_loop.err || { tail -30 $O/live_loop.err; exit 1; }
    timeout -k 10 600 python -u tools/live_loop.py --mixed-k --obstacles 8 > $O/live_loop_mixed_k.json 2> $O/live_loop_mixed.err || { tail -30 $O/live_loop_mixed.err; exit 1; }
    tail -n 1 $O/*.json
    ;;
  *) echo "unknown phase $1"; exit 2 ;;
esac
