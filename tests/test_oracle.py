"""The oracle (oracle/osqp_oracle.c, CPU restatement of OSQP 0.6.2) against known answers.

The reference ships no tests for this path and its vendored libosqp.so may not
be executed here, so the oracle's anchors are: OSQP's published demo problem (x* = (0.3, 0.7),
objective 1.88), closed-form QPs (unconstrained, equality-constrained, active bound), and the
status semantics of osqp/constants.h:18-30 and :96 (primal / dual infeasible, max-iter,
NaN-constant x).  "Parity unpinned" otherwise -- see DESIGN.md.
"""
import numpy as np
import pytest

from oracle import osqp_oracle as ora

NAN_X = 2143289344.0  # OSQP_NAN, constants.h:96


def dense_pattern(P, A):
    """Upper-triangular CSC of P and CSC of A from dense matrices (explicit zeros dropped)."""
    P, A = np.asarray(P, float), np.asarray(A, float)
    n, m = P.shape[0], A.shape[0]
    Pp, Pi, Px, Ap, Ai, Ax = [0], [], [], [0], [], []
    for c in range(n):
        for r in range(c + 1):
            if P[r, c] != 0:
                Pi.append(r)
                Px.append(P[r, c])
        Pp.append(len(Pi))
        for r in range(m):
            if A[r, c] != 0:
                Ai.append(r)
                Ax.append(A[r, c])
        Ap.append(len(Ai))
    pat = dict(n=n, m=m, Pp=np.array(Pp), Pi=np.array(Pi, dtype=np.int64), Ap=np.array(Ap),
               Ai=np.array(Ai, dtype=np.int64))
    return pat, np.array(Px)[None], np.array(Ax)[None]


def solve(P, q, A, l, u, **kw):
    pat, Px, Ax = dense_pattern(P, A)
    s = ora.default_settings(**dict(dict(verbose=0, adaptive_rho_interval=25), **kw))
    x, y, info = ora.solve_batch(pat, Px, np.asarray(q, float)[None], Ax, np.asarray(l, float)[None],
                                 np.asarray(u, float)[None], s)
    return x[0], y[0], info[0]


def test_default_settings_match_osqp_062():
    s = ora.default_settings()
    # osqp_set_default_settings / constants.h:59-119
    assert (s.rho, s.sigma, s.scaling, s.adaptive_rho, s.adaptive_rho_interval) == (0.1, 1e-6, 10, 1, 0)
    assert (s.adaptive_rho_tolerance, s.adaptive_rho_fraction, s.max_iter) == (5.0, 0.4, 4000)
    assert (s.eps_abs, s.eps_rel, s.eps_prim_inf, s.eps_dual_inf, s.alpha) == (1e-3, 1e-3, 1e-4, 1e-4, 1.6)
    assert (s.polish, s.scaled_termination, s.check_termination, s.warm_start) == (0, 0, 25, 1)


def test_osqp_demo_problem():
    """OSQP's published demo QP: x* = (0.3, 0.7), objective 1.88."""
    x, y, info = solve([[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]], [1, 0, 0], [1, 0.7, 0.7])
    assert info["status_val"] == 1
    assert np.allclose(x, [0.3, 0.7], atol=2e-3)
    assert abs(info["obj_val"] - 1.88) < 5e-3
    assert np.allclose(y, [-2.9, 0.0, 0.2], atol=2e-2)
    # KKT stationarity P x + q + A' y = 0 to the tolerance
    P = np.array([[4, 1], [1, 2]])
    A = np.array([[1, 1], [1, 0], [0, 1]])
    assert np.abs(P @ x + np.array([1, 1]) + A.T @ y).max() < 1e-2


def test_tight_tolerance_converges_to_optimum():
    x, y, info = solve([[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]], [1, 0, 0], [1, 0.7, 0.7],
                       eps_abs=1e-9, eps_rel=1e-9, max_iter=100000)
    assert info["status_val"] == 1
    assert np.allclose(x, [0.3, 0.7], atol=1e-7)


def test_equality_constrained_closed_form():
    rng = np.random.default_rng(1)
    n, me = 6, 2
    M = rng.standard_normal((n, n))
    P = M @ M.T + n * np.eye(n)
    q = rng.standard_normal(n)
    E = rng.standard_normal((me, n))
    b = rng.standard_normal(me)
    K = np.block([[P, E.T], [E, np.zeros((me, me))]])
    xs = np.linalg.solve(K, np.concatenate([-q, b]))[:n]
    x, _, info = solve(P, q, E, b, b, eps_abs=1e-10, eps_rel=1e-10, max_iter=100000)
    assert info["status_val"] == 1
    assert np.abs(x - xs).max() < 1e-6


def test_active_box_bound():
    # min (x - 2)^2 s.t. x <= 1  ->  x* = 1, y* = 2 (multiplier of the upper bound)
    x, y, info = solve([[2.0]], [-4.0], [[1.0]], [-np.inf], [1.0], eps_abs=1e-9, eps_rel=1e-9, max_iter=100000)
    assert info["status_val"] == 1
    assert abs(x[0] - 1.0) < 1e-6 and abs(y[0] - 2.0) < 1e-5


def test_primal_infeasible():
    x, y, info = solve([[1.0]], [0.0], [[1.0], [1.0]], [1.0, -np.inf], [np.inf, 0.0])
    assert info["status_val"] == -3
    assert np.all(x == NAN_X)
    assert info["obj_val"] == 1e30  # OSQP_INFTY (constants.h) objective on primal infeasibility


def test_dual_infeasible():
    x, y, info = solve([[0.0, 0.0], [0.0, 1.0]], [-1.0, 0.0], [[0.0, 1.0]], [-1.0], [1.0])
    assert info["status_val"] == -4
    assert np.all(x == NAN_X)
    assert info["obj_val"] == -1e30


def test_max_iter_status():
    x, y, info = solve([[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]], [1, 0, 0], [1, 0.7, 0.7],
                       eps_abs=1e-14, eps_rel=1e-14, max_iter=30)
    assert info["iter"] == 30
    assert info["status_val"] in (-2, 2)  # max-iter, or solved-inaccurate by the x10 check


def test_warm_start_from_solution_is_fast():
    P, q, A, l, u = [[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]], [1, 0, 0], [1, 0.7, 0.7]
    x, y, info = solve(P, q, A, l, u)
    pat, Px, Ax = dense_pattern(P, A)
    s = ora.default_settings(verbose=0, adaptive_rho_interval=25)
    x2, y2, info2 = ora.solve_batch(pat, Px, np.array([q], float), Ax, np.array([l], float), np.array([u], float),
                                    s, x_ws=x[None], y_ws=y[None])
    assert info2[0]["status_val"] == 1 and info2[0]["iter"] <= info["iter"]


def test_batch_threads_bitwise_deterministic():
    from impc import scenarios
    cfg = scenarios.static_config(batch=16, identical=False, seed=77)
    v, s = cfg["values"], ora.default_settings(verbose=0, adaptive_rho_interval=25)
    r1 = ora.solve_batch(cfg["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"], s, threads=1)
    r8 = ora.solve_batch(cfg["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"], s, threads=8)
    assert np.array_equal(r1[0], r8[0]) and np.array_equal(r1[2], r8[2])


def test_infinite_bounds_equal_1e30():
    """OSQP clamps bounds to +-OSQP_INFTY (1e30) in setup; +-inf and +-1e30 give identical results."""
    P, q, A = [[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]]
    a = solve(P, q, A, [1, -np.inf, 0], [1, 0.7, np.inf])
    b = solve(P, q, A, [1, -1e30, 0], [1, 0.7, 1e30])
    assert np.array_equal(a[0], b[0]) and a[2]["iter"] == b[2]["iter"]


@pytest.mark.parametrize("rho_interval", [25, 50])
def test_adaptive_rho_fires_and_is_counted(rho_interval):
    """A tight-tolerance solve runs long enough for adapt_rho to fire; it is counted in info and
    the solution is still the optimum."""
    x, y, info = solve([[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]], [1, 0, 0], [1, 0.7, 0.7],
                       eps_abs=1e-9, eps_rel=1e-9, max_iter=100000, adaptive_rho_interval=rho_interval)
    assert info["status_val"] == 1 and info["rho_updates"] >= 1
    assert info["iter"] % rho_interval == 0 or info["iter"] % 25 == 0
    assert np.allclose(x, [0.3, 0.7], atol=1e-7) and np.allclose(y, [-2.9, 0.0, 0.2], atol=1e-6)


def test_no_adaptive_rho():
    x, y, info = solve([[4, 1], [1, 2]], [1, 1], [[1, 1], [1, 0], [0, 1]], [1, 0, 0], [1, 0.7, 0.7],
                       eps_abs=1e-9, eps_rel=1e-9, max_iter=100000, adaptive_rho=0)
    assert info["status_val"] == 1 and info["rho_updates"] == 0
    assert np.allclose(x, [0.3, 0.7], atol=1e-7)


def test_setup_state_matches_libosqp_probe_facts():
    """The only reference-side facts about osqp_setup's internals (the survey's
    probe read them from the vendored libosqp.so's OSQPWorkspace on an N=20, K=10 mpcPlanner QP):
    constr_type 1 / rho_vec 100 on the dynamics (equality) rows, -1 / 1e-6 on the box rows bounded
    by +-inf on both sides (x position and the two dummy states), 0 / 0.1 on the finite box, slack
    and obstacle rows; cost scale c of order 1e-3; D and E in roughly [0.1, 10]."""
    import impc
    from impc import scenarios
    cfg = scenarios.static_config(N=20, K=10, batch=1, seed=2000)
    pat, v = cfg["pattern"], cfg["values"]
    N, n, m = 20, pat["n"], pat["m"]
    w = ora.Workspace(pat, v["Px"][0], v["q"][0], v["Ax"][0], v["l"][0], v["u"][0],
                      ora.settings_from(impc.default_settings(verbose=0)))
    st = w.setup_state()
    w.close()
    ct, rho = st["constr_type"], st["rho_vec"]
    dyn = slice(0, 8 * N)
    assert (ct[dyn] == 1).all() and np.allclose(rho[dyn], 100.0)
    box = np.arange(8 * N, 8 * N + n)
    state_box = box[: 8 * N].reshape(N, 8)
    loose = state_box[:, [0, 6, 7]].ravel()                    # x position, the two dummy states
    assert (ct[loose] == -1).all() and np.allclose(rho[loose], 1e-6)
    finite = np.concatenate([state_box[:, 1:6].ravel(), box[8 * N:], np.arange(8 * N + n, m)])
    assert (ct[finite] == 0).all() and np.allclose(rho[finite], 0.1)
    assert 1e-4 < st["c"] < 1e-2
    for vec in (st["D"], st["E"]):
        assert 0.05 < vec.min() and vec.max() < 20.0


def test_reachable_reference_needs_fewer_iterations():
    """the synthetic reference (0.5-2.5 m per 0.1 s step, mostly beyond
    vmax = 5 m/s) explains the iteration counts above the survey's libosqp probe (125 at K = 0):
    with a reachable reference the same first-call QPs converge in far fewer iterations."""
    import impc
    from impc import scenarios
    s = impc.default_settings(verbose=0)
    it = {}
    for step in (0.3, 2.5):
        cfg = scenarios.first_call_config(batch=16, seed=11, step_range=(step, step))
        v = cfg["values"]
        _, _, info = ora.solve_batch(cfg["pattern"], v["Px"], v["q"], v["Ax"], v["l"], v["u"],
                                     ora.settings_from(s), threads=4)
        it[step] = float(info["iter"].mean())
    assert it[0.3] <= 200 and it[2.5] >= 1.5 * it[0.3], it


def test_set_state_reproduces_the_workspace_it_was_taken_from():
    """ora_set_state (the closed-loop tests' re-synchronisation): a second workspace of the same QP
    loaded with the first's rho and scaled iterates continues bitwise like the first through an
    osqp_update_A + _lin_cost + _bounds + solve step; an unchanged rho leaves the factor alone."""
    import impc
    from impc import scenarios
    cfg = scenarios.static_config(N=20, K=4, batch=1, identical=False, seed=531)
    pat, v = cfg["pattern"], cfg["values"]
    s = ora.settings_from(impc.default_settings(verbose=0, adaptive_rho_interval=25))
    a = ora.Workspace(pat, v["Px"][0], v["q"][0], v["Ax"][0], v["l"][0], v["u"][0], s)
    b = ora.Workspace(pat, v["Px"][0], v["q"][0], v["Ax"][0], v["l"][0], v["u"][0], s)
    a.solve()
    rho, x, z, y = a.get_state()
    b.set_state(rho, x, z, y)
    rb, xb, zb, yb = b.get_state()
    assert rb == rho and np.array_equal(xb, x) and np.array_equal(zb, z) and np.array_equal(yb, y)
    rng = np.random.default_rng(3)
    A2 = v["Ax"][0] * (1 + 0.01 * rng.standard_normal(v["Ax"][0].shape))
    q2 = v["q"][0] * 1.05
    out = []
    for w in (a, b):
        w.update_matrices(None, A2)
        w.update_lin_cost(q2)
        w.update_bounds(v["l"][0], v["u"][0])
        out.append(w.solve())
    (xa, ya, ia), (xb2, yb2, ib) = out
    assert ia["iter"] == ib["iter"] and ia["status_val"] == ib["status_val"]
    np.testing.assert_array_equal(xa, xb2)
    np.testing.assert_array_equal(ya, yb2)
    a.close()
    b.close()
