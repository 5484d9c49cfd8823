"""CPU, no GPU: the Q1 oracles against a THIRD-PARTY QP solver (VERDICT r4 "what's missing" 1).

tests/golden/highs_qp_{c3,c4}.npz hold 48 trust-region subproblems of Distributed_opt/dist_scvx_3d.py:51-111 (no
SOC): 24 of the C3 family (every one with an active sphere row) and 24 C4-shard agents on the lattice (2-52 active
collision rows with the shared slack S_t).  Their optimum comes from SciPy's HiGHS active-set QP solver, polished
to the exact active-set solution and certified by the KKT conditions (tests/golden/make_highs_qp_goldens.py) -- an
answer shared with neither oracle/qp_dense.py's interior-point method nor the kernel's CPU twin.

Checked: the dense reference-form oracle and the twin (at the bench's tol 1e-8) reach the certified optimal value
to 1e-8 relative; inputs within the strong-convexity bound of that value gap (U_BOUND: the objective has
curvature 2 in every input, so sum ||u_t - u*_t||^2 is bounded by the objective error, tests/highs_fixtures.py)."""
import numpy as np
import pytest

from highs_fixtures import FAMILIES, K, U_BOUND, dense_prob, load, rel, u_dist
from oracle import qp_cpu, qp_dense as qd


@pytest.mark.parametrize("name", FAMILIES)
def test_fixture_is_certified_and_active(name):
    f = load(name)
    assert f["obj"].shape[0] == 24
    assert (f["n_active"].sum(1) >= 1).all()
    # the stored optimum satisfies the reference-form constraints (a solver-free feasibility check)
    for a in range(f["obj"].shape[0]):
        p = dense_prob(f, a)
        v = qd.constraint_violation(p, f["X"][a], f["U"][a], f["S"][a] if f["jm"] else None)
        assert max(v.values()) < 1e-9, (a, v)
    # HiGHS's own (unpolished) value sits within its tolerance of the certified optimum, never below it
    assert (rel(f["obj_highs"], f["obj"]) < 1e-7).all()
    assert (f["obj_highs"] >= f["obj"] - 1e-9 * np.maximum(1, np.abs(f["obj"]))).all()


@pytest.mark.parametrize("name", FAMILIES)
def test_twin_matches_highs(name):
    f = load(name)
    tpl = qp_cpu.make_template(6, 3, K, box=f["box_list"], obs=f["obs_list"], w_obs=1e6, j_max=f["jm"], w_coll=1e4,
                               tol=1e-8, max_iter=80)
    out = qp_cpu.solve_batched(tpl, f["disc"], f["sigma"], f["Xref"], f["Uref"], f["x_init"], f["x_final"], f["tr"],
                               f["rows"] if f["jm"] else None, f["cnt"] if f["jm"] else None)
    assert (out["status"] == 0).all(), out["status"]
    r = rel(out["obj"], f["obj"])
    print(name, "twin max rel obj diff", r.max())
    assert (r <= 1e-8).all(), r
    assert (u_dist(out["U"], f) <= U_BOUND * np.maximum(1.0, np.abs(f["obj"]))).all(), u_dist(out["U"], f)


@pytest.mark.parametrize("name", FAMILIES)
def test_dense_oracle_matches_highs(name):
    f = load(name)
    worst = 0.0
    for a in range(f["obj"].shape[0]):
        with np.errstate(all="ignore"):
            Xd, Ud, od, info = qd.solve_agent(dense_prob(f, a), sparse=True, tol=1e-10)
        # the oracle's reduced-accuracy exit is taken on a few penalty-dominated C4 instances; the value is what
        # the test pins
        assert info["status"] in ("optimal", "optimal_inaccurate"), (a, info["status"])
        r = float(rel(od, f["obj"][a]))
        worst = max(worst, r)
        assert r <= 1e-8, (a, od, f["obj"][a])
        assert ((Ud - f["U"][a])[:K - 1] ** 2).sum() <= U_BOUND * max(1.0, abs(f["obj"][a])), a
    print(name, "dense oracle max rel obj diff", worst)
