"""Run tests/test_live_loop.py's live loop several times in one process (determinism check of the
chained device replans; tools only)."""
import os
import sys

R0 = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R0, "tests"), os.path.join(R0, "intent-mpc_amd/python"), R0]
import impc  # noqa: E402
import test_live_loop as T  # noqa: E402

ctx = impc.Context(0)
fails = 0
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    try:
        T.test_live_loop_thirty_replans_on_the_benchmark_path(ctx)
        print("run", k, "ok", flush=True)
    except AssertionError as e:
        fails += 1
        print("run", k, "FAILED", str(e)[:600], flush=True)
print("fails", fails)
sys.exit(1 if fails else 0)
