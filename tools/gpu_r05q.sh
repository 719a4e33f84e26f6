#!/bin/bash
# Round 5: the setup's sections alone (profiling build, max_iter = 1) at N = 40 and N = 20.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05q; mkdir -p $O
export IMPC_SECTION_PROF=1
timeout -k 10 300 python -u tools/section_profile.py 512 40 10 1 > $O/sec_n40_mi1.txt 2>&1 || { tail -20 $O/sec_n40_mi1.txt; exit 1; }
cat $O/sec_n40_mi1.txt
timeout -k 10 300 python -u tools/section_profile.py 512 20 8 1 > $O/sec_n20_mi1.txt 2>&1 || { tail -20 $O/sec_n20_mi1.txt; exit 1; }
cat $O/sec_n20_mi1.txt
