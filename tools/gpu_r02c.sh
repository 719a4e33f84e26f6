#!/bin/bash
# Round-2 refresh after the kernel scheduling work: full GPU test suite, per-config rates, the
# reference-speed iteration sweep, then the profile set (tools/profile_r02.sh).  Stops at the
# first failure; every GPU step has its own time limit.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
O=gpurun_out/r02c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
timeout -k 10 600 python -u tools/bench_configs.py --steps 3 > $O/configs_s3.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs_s3.jsonl | cut -c1-200
timeout -k 10 300 python -u tools/xref_sweep.py > $O/xref_sweep.jsonl 2> $O/xref.err || { tail -20 $O/xref.err; exit 1; }
cat $O/xref_sweep.jsonl
bash tools/profile_r02.sh
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
