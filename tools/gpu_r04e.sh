#!/bin/bash
# Round 4: GPU suite on the product library, then for each variant in $VARS (lib/libimpc_qp_<v>.so)
# its parity tests and an alternating A/B against the product on the bench workload.  Each step has
# its own time limit; a failing suite stops the script.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1; export TMPDIR=/tmp
O="$R/gpurun_out/${TAG:-r04e}"; mkdir -p "$O" gpurun_out/exp
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -n 1 $O/pytest_gpu.log
fi
for v in ${VARS:-}; do
  IMPC_LIB_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tail_seed3000.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
  echo "$v parity: $(tail -n 1 $O/pytest_$v.log)"
done
[ -n "${VARS:-}" ] && STEPS=5 bash tools/exp.sh base ${VARS} base ${VARS}
exit 0
