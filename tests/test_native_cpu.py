"""The device algorithms, compiled for the host (test-only builds under tests/native/), against
the oracle -- the GPU-less half of the parity story.

* admm_core.hpp (generic one-QP-per-lane kernel body) through tests/native/core_harness.cpp
* mpc_wave.hpp (structured one-QP-per-128-lane-team kernel body) through tests/native/wave_emu.cpp,
  which runs the 128 lanes as threads meeting at a barrier wherever the GPU team synchronises.

Both must reproduce the oracle's iteration count and status exactly and its primal/dual to
PRIMAL_RTOL (they use different but exact-arithmetic-equivalent linear algebra).
"""
import numpy as np
import pytest

import impc
from impc import scenarios

from helpers import EMU64_PATH, compare, emulate, harness, oracle, take

S25 = dict(verbose=0, adaptive_rho_interval=25)


def configs():
    b3 = scenarios.intent_config(instances=3, seed=303)
    return {
        "config1": scenarios.first_call_config(batch=4, seed=101),
        "config2": scenarios.static_config(batch=4, identical=False, seed=202),
        "config3_K8": b3[8],
        "config3_K9": b3[9],
        "config5_N40": scenarios.static_config(N=40, K=10, batch=2, identical=False, seed=505),
    }


CFG = configs()


@pytest.mark.parametrize("name", list(CFG))
def test_generic_core_matches_oracle(name):
    s = impc.default_settings(**S25)
    compare(harness(CFG[name], s), oracle(CFG[name], s))


@pytest.mark.parametrize("rho", [0.1, 1e-3])
def test_generic_core_infeasible_and_rho_paths(rho):
    """Primal-infeasible instances (a box row contradicting the pinned initial state) and a small initial rho that forces
    adaptive rho updates (in-kernel refactorisation) follow the oracle too."""
    cfg = scenarios.static_config(batch=4, identical=False, seed=909)
    v = cfg["values"]
    l = v["l"].copy()
    N = cfg["N"]
    l[1, 8 * N + 1] = 4.9  # y of x0 boxed to [4.9, 5] while the dynamics rows pin x0 -> infeasible
    cfg = dict(cfg, values=dict(v, l=l))
    s = impc.default_settings(rho=rho, **S25)
    res, ref = harness(cfg, s), oracle(cfg, s)
    compare(res, ref)
    assert ref[2]["status_val"][1] in (-3, 3)
    if rho < 0.1:
        assert ref[2]["rho_updates"].max() >= 1


def test_structured_emulation_matches_oracle():
    """One intent-hypothesis QP (config 3 shape, warm-started) through the 128-lane emulation."""
    cfg = take(CFG["config3_K9"], 1)
    s = impc.default_settings(**S25)
    compare(emulate(cfg, s), oracle(cfg, s))


def test_structured_emulation_odd_stage_count():
    """N=19 (W-1 odd) takes the other parity of the backward sweep (mpc_wave.hpp bwd_sweep)."""
    cfg = scenarios.static_config(N=19, K=4, batch=1, identical=False, seed=1919)
    s = impc.default_settings(**S25)
    compare(emulate(cfg, s), oracle(cfg, s))


@pytest.mark.parametrize("N", [3, 6])
def test_structured_emulation_short_horizons(N):
    cfg = scenarios.static_config(N=N, K=2, batch=1, identical=False, seed=1300 + N)
    s = impc.default_settings(**S25)
    compare(emulate(cfg, s), oracle(cfg, s))


def test_structured_emulation_long_horizon():
    """N=40 (n=515): the three-slot team shape of the structured kernel, whose W = 39 instance runs
    the stage recursions in four chunks (mpc_wave.hpp fwd_chunked / bwd_chunked), including
    refactorisations by adaptive rho (the chunk operators rebuilt)."""
    cfg = take(scenarios.intent_config(N=40, K=10, instances=1, seed=4040)[10], 1)
    s = impc.default_settings(**S25)
    compare(emulate(cfg, s), oracle(cfg, s))
    cfg = scenarios.static_config(N=40, K=11, batch=1, identical=False, seed=606)
    s = impc.default_settings(rho=1e-3, **S25)
    ref = oracle(cfg, s)
    assert ref[2]["rho_updates"].max() >= 1
    compare(emulate(cfg, s), ref)


def test_structured_emulation_live_horizon():
    """N=30 (n=385, the reference's live planner horizon, planner_param.yaml:25): the three-slot
    shape's W = 29 instance, chunked recursions of 6 / 6 / 6 / 6 / 5 steps (five chunks on four
    wavefronts, IMPC_CHUNK5, the product form), with adaptive-rho refactorisations."""
    cfg = take(scenarios.intent_config(N=30, K=8, instances=1, seed=3030)[8], 1)
    s = impc.default_settings(**S25)
    compare(emulate(cfg, s), oracle(cfg, s))
    cfg = scenarios.static_config(N=30, K=9, batch=1, identical=False, seed=3031)
    s = impc.default_settings(rho=1e-3, **S25)
    ref = oracle(cfg, s)
    assert ref[2]["rho_updates"].max() >= 1
    compare(emulate(cfg, s), ref)


@pytest.mark.parametrize("rho", [0.1, 1e-3])
def test_structured_emulation_default_horizon_batch(rho):
    """The default-horizon (W = 19) instance of the structured kernel -- fully unrolled stage
    recursions with register-captured results (mpc_wave.hpp fwd_sweep / bwd_sweep) -- over several
    QPs of both intent buckets, and with a small initial rho whose adaptive updates refactorise
    in-kernel (F_k and the Ahat_k^{-1} rows rebuilt)."""
    s = impc.default_settings(rho=rho, **S25)
    for name in ("config3_K8", "config2"):
        cfg = take(CFG[name], 2)
        res, ref = emulate(cfg, s), oracle(cfg, s)
        compare(res, ref)
        if rho < 0.1:
            assert ref[2]["rho_updates"].max() >= 1


@pytest.mark.parametrize("name", ["config3_K8", "config3_K9", "config2"])
def test_structured_emulation_wavefront_team(name):
    """The one-QP-per-wavefront team shape (64 lanes, four variable slots and up to six
    general-row slots per lane, D / E and the check deltas off LDS) against the oracle: the same
    kernel body at NL = 64 (mpc_wave.hpp, Gauss-Jordan with several elements per lane)."""
    s = impc.default_settings(**S25)
    cfg = take(CFG[name], 2)
    compare(emulate(cfg, s, EMU64_PATH), oracle(cfg, s))


@pytest.mark.parametrize("N", [3, 19])
def test_structured_emulation_wavefront_team_horizons(N):
    cfg = scenarios.static_config(N=N, K=4, batch=1, identical=False, seed=1900 + N)
    s = impc.default_settings(**S25)
    compare(emulate(cfg, s, EMU64_PATH), oracle(cfg, s))


def test_structured_emulation_failed_rho_update_ends_unsolved():
    """The structured kernel body's osqp_solve exit on a failed adaptive-rho refactorisation (P
    indefinite; P + sigma I + A'RA positive definite at the first rho only): status UNSOLVED at the
    iteration of the update, as the oracle (the GPU twin: tests/test_persistent.py::
    test_failed_rho_update_ends_the_solve_unsolved, same QPs)."""
    cfg = scenarios.static_config(N=20, K=4, batch=4, identical=False, seed=520)
    keep = [0, 1, 3]
    v = {k: a[keep] for k, a in cfg["values"].items()}
    v["Px"] = np.full_like(v["Px"], -1e3)
    c = dict(cfg, values=v)
    s = impc.default_settings(**S25)
    _, _, info = emulate(c, s)
    _, _, io = oracle(c, s)
    assert (io["status_val"] == impc.UNSOLVED).any()
    np.testing.assert_array_equal(info["status_val"], io["status_val"])
    np.testing.assert_array_equal(info["iter"], io["iter"])
    np.testing.assert_array_equal(info["rho_updates"], io["rho_updates"])


@pytest.mark.parametrize("which", ["long", "wave64"])
def test_structured_emulation_scaling_vectors_in_lds(which, monkeypatch):
    """The wavefront and long shapes keep D, E in LDS after the products region when the CU has
    the room (WaveTables::scal_lds, decided at batch setup): the same results as the oracle (and,
    checked when built, bitwise the same as with them in the HBM scratch)."""
    monkeypatch.setenv("EMU_SCAL_LDS", "1")
    s = impc.default_settings(**S25)
    if which == "long":
        cfg = CFG["config5_N40"]
        compare(emulate(take(cfg, 1), s), oracle(take(cfg, 1), s))
    else:
        cfg = take(CFG["config3_K8"], 1)
        compare(emulate(cfg, s, EMU64_PATH), oracle(cfg, s))
