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
      if [ -d ab_r05 ]; then  # the round-5 build beside, when staged (before / after of the host syncs)
        ( cd ab_r05 && timeout -k 10 300 python -u tools/replan_bench.py --instances $I --reps $R ) > $O/replan_full_call_I${I}_r05.json 2> $O/replan_I${I}_r05.err || { tail -30 $O/replan_I${I}_r05.err; exit 1; }
      fi
    done
    timeout -k 10 600 python -u tools/live_loop.py > $O/live_loop.json 2> $O/live_loop.err || { tail -30 $O/live_loop.err; exit 1; }
    timeout -k 10 600 python -u tools/live_loop.py --mixed-k --obstacles 8 > $O/live_loop_mixed_k.json 2> $O/live_loop_mixed.err || { tail -30 $O/live_loop_mixed.err; exit 1; }
    tail -n 1 $O/*.json
    ;;
  prof)  # PMC HBM traffic (config 3, config 5's closed loop, live) and SQ counters (config 3, config 5, live)
          # of the final build; the summaries land in this box's profiles/ and come back via gpurun_out
    cd /tmp || exit 1
    A3="--steps 1 --warmup 0 --cpu-sample 0 --e2e-steps 0"
    A5="--workload config5 --steps 1 --warmup 10 --receding-replay 0 --cpu-sample 0 --e2e-steps 0"
    Al="--workload live --steps 1 --warmup 0 --cpu-sample 0 --e2e-steps 0"
    P="$R/$O/prof"; mkdir -p "$P"
    pmc() {  # name counters args...
      local n=$1 c=$2; shift 2
      timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$P/$n" -o pmc -- python3 "$R/bench.py" "$@" > "$P/$n.log" 2>&1 || { tail -20 "$P/$n.log"; return 1; }
    }
    SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
    SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
    if [ "${2:-}" = sqlive ]; then  # only the live workload's SQ passes
      pmc sql_1 "$SQ1" $Al && pmc sql_2 "$SQ2" $Al || exit 1
      python3 - "$P" <<'PY'
import csv, glob, sys
o = sys.argv[1]
tot = {}
for p in ("1", "2"):
    for f in glob.glob(f"{o}/sql_{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mpc_wave_group" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot): print(f"{k:24s} {tot[k]:.6g}")
print(f"WAIT_ANY/WAVE_CYCLES {tot['SQ_WAIT_ANY']/tot['SQ_WAVE_CYCLES']:.3f}  ACTIVE_INST_VALU/WAVE_CYCLES {tot['SQ_ACTIVE_INST_VALU']/tot['SQ_WAVE_CYCLES']:.3f}  LDS_BANK_CONFLICT/ACTIVE_INST_LDS {tot['SQ_LDS_BANK_CONFLICT']/tot['SQ_ACTIVE_INST_LDS']:.3f}")
PY
      exit 0
    fi
    pmc pmc3_fetch FETCH_SIZE $A3 && pmc pmc3_write WRITE_SIZE $A3 || exit 1
    python3 "$R/tools/pmc_summary.py" "$P/pmc3_fetch" "$P/pmc3_write" k_mpc_wave_group 65536 shared config3 > "$P/pmc_k_solve.json" || exit 1
    pmc pmc5_fetch FETCH_SIZE $A5 && pmc pmc5_write WRITE_SIZE $A5 || exit 1
    python3 "$R/tools/pmc_summary.py" "$P/pmc5_fetch" "$P/pmc5_write" k_mpc_wave_group 65536 shared config5 last > "$P/pmc_config5.json" || exit 1
    pmc pmcl_fetch FETCH_SIZE $Al && pmc pmcl_write WRITE_SIZE $Al || exit 1
    python3 "$R/tools/pmc_summary.py" "$P/pmcl_fetch" "$P/pmcl_write" k_mpc_wave_group 65536 shared live > "$P/pmc_live.json" || exit 1
    for w in 3 5 l; do
      eval A=\$A$w
      pmc sq${w}_1 "$SQ1" $A && pmc sq${w}_2 "$SQ2" $A || exit 1
    done
    python3 - "$P" <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
for w, name, what in (("3", "config3", "bench.py --steps 1 --warmup 0 (config 3, 65,536 QPs, N = 20), its one launch"),
                      ("5", "config5", "bench.py --workload config5 --steps 1 --warmup 10 --receding-replay 0, the last dispatch (closed-loop step 11)"),
                      ("l", "live", "bench.py --workload live --steps 1 --warmup 0 (65,536 N = 30 QPs), its one launch")):
    bid = None
    for ln in open(f"{o}/sq{w}_1.log"):
        if ln.startswith("{") and '"roofline"' in ln:
            bid = json.loads(ln)["roofline"]["build_id"]
    out = [f"rocprofv3 --pmc, two passes, {what}; build {bid}",
           "k_mpc_wave_group, summed over the GPU's counter instances"]
    tot = {}
    for p in ("1", "2"):
        vals = {}
        for f in glob.glob(f"{o}/sq{w}_{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_mpc_wave_group" in r["Kernel_Name"]:
                    d = int(r["Dispatch_Id"]); vals.setdefault(d, {})
                    vals[d][r["Counter_Name"]] = vals[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        tot.update(vals[max(vals)])
    out += [f"{k:24s} {tot[k]:.6g}" for k in sorted(tot)]
    out.append(f"WAIT_ANY/WAVE_CYCLES {tot['SQ_WAIT_ANY']/tot['SQ_WAVE_CYCLES']:.3f}  ACTIVE_INST_VALU/WAVE_CYCLES "
               f"{tot['SQ_ACTIVE_INST_VALU']/tot['SQ_WAVE_CYCLES']:.3f}  LDS_BANK_CONFLICT/ACTIVE_INST_LDS "
               f"{tot['SQ_LDS_BANK_CONFLICT']/tot['SQ_ACTIVE_INST_LDS']:.3f}")
    open(f"{o}/sq_counters_{name}.txt", "w").write("\n".join(out) + "\n")
    print("\n".join(out))
PY
    cat "$P"/pmc_*.json
    ;;
  final)  # the GPU suite, smoke, the bench lines (default, config 5, live) and the kernel traces, on the
          # final build with its PMC summaries committed under profiles/
    P="$O/final"; mkdir -p "$P"
    timeout -k 10 1000 $PYT -m gpu tests > "$P/pytest_gpu.log" 2>&1 || { tail -60 "$P/pytest_gpu.log"; exit 1; }
    tail -2 "$P/pytest_gpu.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$P/smoke.log" 2>&1 || { tail -30 "$P/smoke.log"; exit 1; }
    echo smoke ok
    timeout -k 10 600 python bench.py > "$P/bench_default.json" 2> "$P/bench_default.err" || { tail -20 "$P/bench_default.err"; exit 1; }
    timeout -k 10 900 python bench.py --workload config5 --steps 10 --warmup 10 > "$P/bench_config5.json" 2> "$P/bench_config5.err" || { tail -20 "$P/bench_config5.err"; exit 1; }
    timeout -k 10 600 python bench.py --workload live --steps 3 --warmup 1 > "$P/bench_live.json" 2> "$P/bench_live.err" || { tail -20 "$P/bench_live.err"; exit 1; }
    python3 - "$P" <<'PY'
import json, sys
for n in ("bench_default", "bench_config5", "bench_live"):
    d = json.load(open(f"{sys.argv[1]}/{n}.json"))
    r = d["roofline"]
    print(n, round(d["value"]), round(d["ms_per_step"], 2), r["frac"], r["traffic"], r["build_id"],
          d["cpu_baseline"] and round(d["cpu_baseline"]["value"]), d["parity"] and d["parity"]["pass"])
PY
    cd /tmp || exit 1
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/kt_default" -o kt -- python3 "$R/bench.py" --cpu-sample 0 --e2e-steps 0 > "$R/$P/kt_default.log" 2>&1 || { tail -20 "$R/$P/kt_default.log"; exit 1; }
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/kt_config5" -o kt -- python3 "$R/bench.py" --workload config5 --steps 10 --warmup 10 --receding-replay 0 --cpu-sample 0 --e2e-steps 0 > "$R/$P/kt_config5.log" 2>&1 || { tail -20 "$R/$P/kt_config5.log"; exit 1; }
    find "$R/$P/kt_default" "$R/$P/kt_config5" -name "*kernel_stats.csv" -exec head -4 {} \;
    ;;
  *) echo "unknown phase $1"; exit 2 ;;
esac
