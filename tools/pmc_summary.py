#!/usr/bin/env python3
"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --steps 1 --warmup 0`
into the per-step HBM traffic of the solver kernel (MI355X_MICROARCH.md, HBM section: FETCH_SIZE
counts half the bytes of wide coalesced reads on gfx950 -> x2; WRITE_SIZE exact; both in KB).

usage: pmc_summary.py FETCH_DIR WRITE_DIR KERNEL QPS_PER_STEP [VALUES_MODE [WORKLOAD]] > pmc_k_solve.json
(VALUES_MODE: bench.py's input mode, shared | full; bench only quotes a summary of its own mode,
workload and library build: the summary records impc_build_id() of the library in this tree, which
is the one the profiled runs loaded)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def collect(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", ""):
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, kernel, qps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else "full"
    workload = sys.argv[6] if len(sys.argv) > 6 else "config3"
    sys.path.insert(0, os.path.join(ROOT, "intent-mpc_amd", "python"))
    import impc  # loads the library only (no device call): its build identity
    build_id = impc.lib.impc_build_id().decode()
    fetch = collect(fdir, "FETCH_SIZE", kernel)
    write = collect(wdir, "WRITE_SIZE", kernel)
    if not fetch or not write:
        sys.exit(f"no {kernel} rows (fetch {len(fetch)}, write {len(write)})")
    fetch_b = 2.0 * 1024.0 * sum(fetch)   # KB -> bytes, gfx950 half-count correction
    write_b = 1024.0 * sum(write)
    print(json.dumps({
        "kernel": kernel, "qps_per_launch": qps, "values": mode, "workload": workload, "build_id": build_id,
        "version": impc.lib.impc_version().decode(), "launches": len(fetch),
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({os.path.basename(os.path.normpath(fdir))}, "
                  f"{os.path.basename(os.path.normpath(wdir))})",
        "fetch_size_kb_raw": sum(fetch), "write_size_kb_raw": sum(write),
        "hbm_bytes_per_launch": fetch_b + write_b, "fetch_bytes": fetch_b, "write_bytes": write_b,
        "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), WRITE_SIZE x1; summed over the step's launches",
    }, indent=1))


if __name__ == "__main__":
    main()
