#!/usr/bin/env python3
"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --steps 1 --warmup 0`
into the per-step HBM traffic of the solver kernel (MI355X_MICROARCH.md, HBM section: FETCH_SIZE
counts half the bytes of wide coalesced reads on gfx950 -> x2; WRITE_SIZE exact; both in KB).

usage: pmc_summary.py FETCH_DIR WRITE_DIR KERNEL QPS_PER_STEP [VALUES_MODE [WORKLOAD [LAUNCH]]] > pmc_k_solve.json
(LAUNCH: "all" (default: the sum over every launch of KERNEL -- one launch in a --steps 1 --warmup 0
run of config 3) or "last": the last dispatch only -- config 5's timed step, after its untimed
setup solve, in a run with --receding-replay 0)
(VALUES_MODE: bench.py's input mode, shared | full; bench only quotes a summary of its own mode,
workload and library build.  The build id is the one the profiled runs themselves reported: each
pass's bench JSON line (FETCH_DIR.log / WRITE_DIR.log, the runs' stdout) carries roofline.build_id
of the library it loaded; both passes must agree.  Nothing here loads the library.)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def collect(d, counter, kernel, launch="all"):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", ""):
                key = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(vals))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    out = [vals[k] for k in sorted(vals)]
    return out[-1:] if launch == "last" else out


def main():
    fdir, wdir, kernel, qps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else "full"
    workload = sys.argv[6] if len(sys.argv) > 6 else "config3"
    launch = sys.argv[7] if len(sys.argv) > 7 else "all"
    ids, versions = [], []
    for d in (fdir, wdir):
        line = None
        with open(os.path.normpath(d) + ".log") as f:
            for ln in f:
                if ln.startswith("{") and '"roofline"' in ln:
                    line = json.loads(ln)
        if line is None:
            sys.exit(f"no bench line in {os.path.normpath(d)}.log: the pass's build id is unknown")
        ids.append(line["roofline"]["build_id"])
    if ids[0] != ids[1]:
        sys.exit(f"the two passes ran different builds: {ids}")
    build_id = ids[0]
    fetch = collect(fdir, "FETCH_SIZE", kernel, launch)
    write = collect(wdir, "WRITE_SIZE", kernel, launch)
    if not fetch or not write:
        sys.exit(f"no {kernel} rows (fetch {len(fetch)}, write {len(write)})")
    fetch_b = 2.0 * 1024.0 * sum(fetch)   # KB -> bytes, gfx950 half-count correction
    write_b = 1024.0 * sum(write)
    print(json.dumps({
        "kernel": kernel, "qps_per_launch": qps, "values": mode, "workload": workload, "build_id": build_id,
        "build_id_source": "roofline.build_id of the profiled runs' own bench lines", "launches": len(fetch),
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({os.path.basename(os.path.normpath(fdir))}, "
                  f"{os.path.basename(os.path.normpath(wdir))})",
        "fetch_size_kb_raw": sum(fetch), "write_size_kb_raw": sum(write),
        "hbm_bytes_per_launch": fetch_b + write_b, "fetch_bytes": fetch_b, "write_bytes": write_b,
        "launch": launch,
        "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), WRITE_SIZE x1; summed over the step's launches",
    }, indent=1))


if __name__ == "__main__":
    main()
