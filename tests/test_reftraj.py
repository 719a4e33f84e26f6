"""getReferenceTraj / getXRef (mpcPlanner.cpp:968-981, 1199-1231) on the device
(impc_reference_traj_device) against the restatement oracle/reftraj_ref.py: bit-exact references
and identical lastRefStartIdx_ over a sequence of replans, ragged and empty paths, the 30-point
search window ((int)(3.0 / ts)), padding with the last point, and the per-candidate repeat layout."""
import numpy as np
import pytest

import impc
from oracle.reftraj_ref import ReferencePath


def test_oracle_window_quirk_and_padding():
    # a straight path, 1 m spacing; the drone sits at x = 40.2: the window from index 0 holds 30
    # points (0..29), so the nearest point found is 29 although 40 is closer
    path = [(float(k), 0.0, 1.0) for k in range(60)]
    r = ReferencePath(path, 0.1, 20)
    ref = r.reference_traj((40.2, 0.0, 1.0))
    assert r.last == 29 and ref[0] == path[29]
    ref = r.reference_traj((40.2, 0.0, 1.0))              # next replan: window 29..58
    assert r.last == 40 and ref[:3] == path[40:43]
    assert ReferencePath(path, 0.3, 5).reference_traj((40.2, 0.0, 1.0)) and int(3.0 / 0.3) == 10
    ref = r.reference_traj((59.0, 0.0, 1.0))              # near the end: padded with the last point
    assert r.last == 59 and ref == [path[59]] * 20
    assert ReferencePath([], 0.1, 5).reference_traj((1.0, 2.0, 3.0)) == [(1.0, 2.0, 3.0)] * 5
    x = ReferencePath(path, 0.1, 3).xref((0.0, 0.0, 1.0))
    assert x[1] == [1.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0]


def _paths(rng, ni):
    paths = []
    for i in range(ni):
        L = 0 if i % 7 == 3 else int(rng.integers(1, 90))
        step = rng.uniform(0.05, 2.5)
        p0 = rng.uniform(-5, 5, 3)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        paths.append(p0 + step * np.arange(L)[:, None] * d + rng.normal(0, 0.02, (L, 3)))
    return paths


@pytest.mark.gpu
def test_device_reference_matches_oracle_over_replans(ctx):
    rng = np.random.default_rng(77)
    ni, N = 61, 20
    paths = _paths(rng, ni)
    dev = impc.ReferencePaths(ctx, paths, 0.1, N)
    refs = [ReferencePath(p, 0.1, N) for p in paths]
    pos = np.array([p[0] if len(p) else rng.uniform(-5, 5, 3) for p in paths])
    try:
        for step in range(12):
            # the drone moves along its path (sometimes past it, sometimes jittered)
            for i, p in enumerate(paths):
                if len(p):
                    pos[i] = p[min(len(p) - 1, 3 * step + i % 5)] + rng.normal(0, 0.3, 3)
            rep = 1 + step % 3
            got = dev.xref(pos, repeat=rep)
            exp = np.array([r.xref(pos[i]) for i, r in enumerate(refs)])
            for k in range(rep):
                assert np.array_equal(got[:, k], exp), step
            assert np.array_equal(dev.last_idx(), [r.last for r in refs])
    finally:
        dev.close()
