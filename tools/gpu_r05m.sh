#!/bin/bash
# Round 5: section profile (profiling build) of the long shape at N = 40 and N = 30 (full setup +
# warm-started solve), and of the default horizon for comparison.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05m; mkdir -p $O
export IMPC_SECTION_PROF=1
timeout -k 10 300 python -u tools/section_profile.py 1024 40 10 > $O/sec_n40.txt 2>&1 || { tail -20 $O/sec_n40.txt; exit 1; }
cat $O/sec_n40.txt
timeout -k 10 300 python -u tools/section_profile.py 1024 30 8 > $O/sec_n30.txt 2>&1 || { tail -20 $O/sec_n30.txt; exit 1; }
cat $O/sec_n30.txt
timeout -k 10 300 python -u tools/section_profile.py 2048 > $O/sec_n20.txt 2>&1 || { tail -20 $O/sec_n20.txt; exit 1; }
cat $O/sec_n20.txt
unset IMPC_SECTION_PROF
timeout -k 10 600 python -u tools/live_loop.py > $O/live_loop.json 2> $O/live_loop.err || { tail -20 $O/live_loop.err; exit 1; }
cat $O/live_loop.json
