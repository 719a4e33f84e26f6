"""Generates tests/golden/tail_seed3000.npz: the tail of the bench workload (bench.py's default,
BASELINE.json configs[2]: scenarios.intent_config(N=20, K=8, instances=8192, hyps=8, seed=3000)) as
the oracle (oracle/osqp_oracle.c, OSQP 0.6.2 restatement; parity unpinned against the real
libosqp) solves it: per pattern bucket (K = 8, 9), the index, status and iteration count of every
QP that did not end SOLVED or ran to the 4000-iteration cap.

usage: python tests/golden/make_tail_seed3000.py   (about 70 s on 8 threads)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "intent-mpc_amd", "python"))
sys.path.insert(0, ROOT)

import impc  # noqa: E402
from impc import scenarios  # noqa: E402
from oracle import osqp_oracle as ora  # noqa: E402


def main():
    buckets = scenarios.intent_config(N=20, K=8, instances=8192, hyps=8, seed=3000)
    s = ora.settings_from(impc.default_settings(verbose=0))
    out = {}
    for K, bk in sorted(buckets.items()):
        v = bk["values"]
        _, _, io = ora.solve_batch(bk["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"], s, x_ws=bk["x_ws"],
                                   threads=min(8, os.cpu_count() or 1))
        st, it = io["status_val"], io["iter"]
        tail = np.nonzero((st != 1) | (it == 4000))[0]
        out[f"K{K}_index"] = tail.astype(np.int64)
        out[f"K{K}_status"] = st[tail].astype(np.int64)
        out[f"K{K}_iter"] = it[tail].astype(np.int64)
        out[f"K{K}_count"] = np.int64(st.size)
        print(K, st.size, len(tail), dict(zip(*[a.tolist() for a in np.unique(st, return_counts=True)])))
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "tail_seed3000.npz"), **out)


if __name__ == "__main__":
    main()
