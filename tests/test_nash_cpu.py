"""Host logic of the Nash best-response drop-ins (no GPU): GameUnicycleModel / GameSIModel records
(game_model.py:54-126, game_si_model.py:69-136), AgentBestResponse.setup's parameter flow and the
kernel template it derives (agent_best_response.py:46-98)."""
import numpy as np
import pytest

from tests.test_nash_gpu import GAME, OBS_G, SI_GAME, SI_OBS, _cfg, _mam


def test_game_model_surface_and_records():
    from SCvx.global_parameters import K
    from SCvx.models.game_model import GameCost, GameUnicycleModel, SlabConstraint
    from SCvx.optimization.variables import Parameter
    m = GameUnicycleModel(r_init=np.array([0.0, -1.0, 0.0]), r_final=np.array([2.0, 3.0, 0.0]), obstacles=OBS_G,
                          control_weight=5.0, path_weight=0.0, v_max=2.0)
    assert (m.control_weight, m.control_rate_weight, m.curvature_weight, m.collision_radius) == (5.0, 5.0, 100.0, 0.5)
    assert m.v_max == 2.0 and m.z_params == [] and m.extra_constraints == []
    with pytest.raises(IndexError):            # z_params exist only after get_cost_function (game_model.py:111)
        m.update_slabs(np.zeros((2, K)), [np.ones((2, K))])
    P = [Parameter((2, K)), Parameter((2, K))]
    rng = np.random.default_rng(0)
    for p in P:
        p.value = rng.standard_normal((2, K))
    Xp = Parameter((3, K))
    Xp.value = rng.standard_normal((3, K))
    cost = m.get_cost_function(None, None, P, Xp, [p.value for p in P])
    assert isinstance(cost, GameCost) and len(m.extra_constraints) == 2 * K
    assert all(isinstance(c, SlabConstraint) for c in m.extra_constraints)
    assert all(not z.value.any() for row in m.z_params for z in row)          # zero until the first update
    p_i = rng.standard_normal((2, K))
    m.update_slabs(p_i, [p.value for p in P])
    d = p_i[:, 3] - P[1].value[:, 3]
    np.testing.assert_allclose(m.z_params[1][3].value, d / np.linalg.norm(d))
    X, U = rng.standard_normal((3, K)), rng.standard_normal((2, K))
    want = 5 * (U ** 2).sum() + 5 * (np.diff(U, axis=1) ** 2).sum() + 100 * (np.diff(X[2]) ** 2).sum()
    assert abs(cost.value(X, U) - want) < 1e-9 * want
    c = m.extra_constraints[K + 3]
    assert c.j == 1 and c.k == 3
    assert abs(c.violation(X) - max(0.0, 0.5 - m.z_params[1][3].value @ (X[:2, 3] - P[1].value[:, 3]))) < 1e-15


def test_best_response_setup_builds_the_game_template():
    from SCvx.global_parameters import K, TRUST_RADIUS0
    from SCvx.optimization.agent_best_response import AgentBestResponse, slab_arrays
    from SCvx.utils.initial_guess import initial_guess
    mam = _mam()
    X0, U0 = zip(*(initial_guess(np.array(a), np.array(b), OBS_G, 0.05, K) for a, b in GAME))
    br = AgentBestResponse(1, mam)
    assert sorted(br.Y_params) == [0, 2] and br.X_prev_param.shape == (3, K)
    with pytest.raises(RuntimeError):
        br.solve()
    mats = tuple(np.zeros_like(a) for a in (br.foh.A_bar, br.foh.B_bar, br.foh.C_bar, br.foh.S_bar, br.foh.z_bar))
    refs = {0: X0[0], 2: X0[2]}
    br.setup(X0[1], U0[1], 1.0, mats, refs, X0[1], refs)
    spec = br.spec()
    t = spec.to_c()
    assert (t.game, t.sigma_fixed, t.theta_idx, t.n_slab) == (1, 1, 2, 2)
    assert (t.w_u2, t.w_du, t.w_dth, t.w_in, t.r_slab) == (5.0, 5.0, 100.0, 0.0, 0.5)
    assert br.scp.par["tr_radius"].value == TRUST_RADIUS0 and br.scp.par["sigma_ref"].value == 1.0
    z, P = slab_arrays(br.slab_constraints(), 2, 2)
    np.testing.assert_array_equal(P[1], X0[2][:2].T)
    d = X0[1][:2, 7] - X0[0][:2, 7]
    np.testing.assert_allclose(z[0, 7], d / np.linalg.norm(d))
    mam.models[1].path_weight = 1.0
    br.setup(X0[1], U0[1], 1.0, mats, refs, X0[1], refs)
    with pytest.raises(NotImplementedError):
        br.spec()


def test_game_si_model_records():
    from SCvx.global_parameters import K
    from SCvx.models.game_si_model import GameSIModel
    from SCvx.optimization.variables import Parameter
    m = GameSIModel(r_init=np.array([-4.0, 0, 0]), r_final=np.array([4.0, 0, 0]), obstacles=[],
                    control_weight=5.0, curvature_weight=100.0)
    assert m.agent_coll_rad == 1.0 and m.collision_weight == 80.0 and m.curvature_weight == 100.0
    P = [Parameter((3, K))]
    P[0].value = np.ones((3, K))
    Xp = Parameter((3, K))
    Xp.value = np.zeros((3, K))
    cost = m.get_cost_function(None, None, P, Xp, [P[0].value])
    assert cost.curvature_weight == 0.0 and len(m.extra_constraints) == K and len(m.coll_slacks) == 1
    np.testing.assert_allclose(m.z_params[0][0].value, -np.ones(3) / np.sqrt(3))
    m.update_intersample_constraints(None, None, np.zeros((3, K)), np.zeros((3, K)), None, 1.0)
    assert m.extra_constraints == [] and m.inter_slacks == []   # replaced (no obstacles -> no rows)


def test_config_modules_hold_the_reference_scenarios():
    """SCvx/config data against the reference's default_game.py / SI_default_game.py values."""
    g, sg = _cfg()
    assert [(tuple(p["r_init"]), tuple(p["r_final"])) for p in g.AGENT_PARAMS] == GAME and g.OBSTACLES == OBS_G
    assert [(tuple(p["r_init"]), tuple(p["r_final"])) for p in sg.AGENT_PARAMS] == SI_GAME and sg.OBSTACLES == SI_OBS
    assert sg.AGT_COLL_RAD == 1.0 and g.COLL_RAD == 0.5
