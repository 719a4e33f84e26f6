"""Longest-first work queue (impc_batch_set_queue_order, csrc/queue.hpp): the device-estimated
difficulty order changes which workgroup solves a QP and when, never its arithmetic -- results
must be bitwise those of the FIFO queue, for grouped and single launches, shared and full values."""
import numpy as np
import pytest

import impc
from impc import scenarios

pytestmark = pytest.mark.gpu


def _batches(ctx, buckets, shared, order, qw):
    out = []
    for K, bk in sorted(buckets.items()):
        pat, v = bk["pattern"], bk["values"]
        B = v["q"].shape[0]
        b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], B)
        b.set_settings(impc.default_settings(verbose=0))
        if shared:
            b.set_values_shared(*impc.shared_split(v["Px"], v["Ax"]), v["q"], v["l"], v["u"])
        else:
            b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
        b.warm_start(bk["x_ws"], None)
        if order:
            b.set_queue_order(impc.QUEUE_LONGEST_FIRST, qw)
        out.append(b)
    return out


@pytest.mark.parametrize("shared", [True, False], ids=["shared", "full"])
@pytest.mark.parametrize("grouped", [True, False], ids=["grouped", "single"])
def test_longest_first_is_bitwise_fifo(ctx, shared, grouped):
    buckets = scenarios.intent_config(instances=160, seed=3131)   # 1,280 QPs: > 512 in flight
    pd = next(iter(buckets.values()))["params"]
    qw = scenarios.queue_weight(pd, 20)
    res = {}
    for order in (False, True):
        bs = _batches(ctx, buckets, shared, order, qw)
        try:
            if grouped:
                impc.solve_group(bs)
            else:
                for b in bs:
                    b.solve()
            res[order] = [b.get() for b in bs]
        finally:
            for b in bs:
                b.close()
    for (x0, y0, i0), (x1, y1, i1) in zip(res[False], res[True]):
        np.testing.assert_array_equal(x0, x1)
        np.testing.assert_array_equal(y0, y1)
        np.testing.assert_array_equal(i0, i1)


def test_queue_order_arguments(ctx):
    bk = scenarios.intent_config(instances=2, seed=3132)[8]
    pat = bk["pattern"]
    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], 4)
    try:
        with pytest.raises(impc.ImpcError):
            b.set_queue_order(2, 0.0)
        with pytest.raises(impc.ImpcError):
            b.set_queue_order(impc.QUEUE_LONGEST_FIRST, -1.0)
        b.set_queue_order(impc.QUEUE_FIFO)
    finally:
        b.close()


def test_longest_first_mixed_classes_and_long_horizon(ctx):
    """Every kernel class of a config-4 launch (general-row slot counts 2..4, two-tier products,
    22 buckets K = 0..21 in one grouped launch) and the long-horizon shape (N = 40, three variables
    per lane): longest-first results bitwise equal to FIFO."""
    K = np.repeat(np.arange(21), 3)
    groups = [scenarios.config4_rank(0, K.size, K, seed=4500),
              list(scenarios.intent_config(N=40, K=10, instances=40, hyps=8, seed=5200).values())]
    pd = impc.mpc_params(horizon=20)[1]
    for bks in groups:
        qw = scenarios.queue_weight(pd, bks[0]["N"])
        res = {}
        for order in (False, True):
            bs = []
            try:
                for bk in bks:
                    pat, v = bk["pattern"], bk["values"]
                    b = impc.Batch(ctx, pat["n"], pat["m"], pat["Pp"], pat["Pi"], pat["Ap"], pat["Ai"], v["q"].shape[0])
                    bs.append(b)
                    b.set_settings(impc.default_settings(verbose=0))
                    b.set_values(v["Px"], v["q"], v["Ax"], v["l"], v["u"])
                    if bk.get("x_ws") is not None:
                        b.warm_start(bk["x_ws"], None)
                    if order:
                        b.set_queue_order(impc.QUEUE_LONGEST_FIRST, qw)
                impc.solve_group(bs)
                res[order] = [b.get() for b in bs]
            finally:
                for b in bs:
                    b.close()
        for (x0, y0, i0), (x1, y1, i1) in zip(res[False], res[True]):
            np.testing.assert_array_equal(x0, x1)
            np.testing.assert_array_equal(y0, y1)
            np.testing.assert_array_equal(i0, i1)
