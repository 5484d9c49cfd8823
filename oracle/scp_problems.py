"""ORACLE / TEST INFRASTRUCTURE ONLY: SCProblem / AgentSolver instances.

Builds the reference's subproblem data for the unicycle (SCvx/models/unicycle_model.py:12-122) and
3-D single integrator (SCvx/models/single_integrator_model.py:12-141) at a given reference
trajectory, discretized by the C FOH restatement (oracle/foh_ref.c, pinned to the reference's
FirstOrderHold by tests/golden).  Node index first: X (K,n) is the reference's X.T."""
import numpy as np

from . import foh_oracle

UNI_OBS = [([5.0, 4.0], 3.0), ([-5.0, -4.0], 3.0), ([0.0, 0.0], 2.0)]       # unicycle_model.py:48
SI_OBS = [([-5.0, -4.0, -5.0], 2.0), ([0.0, 0.0, 4.0], 2.0)]                 # single_integrator_model.py:49
WEIGHT_NU, WEIGHT_SLACK, WEIGHT_SIGMA, TRUST_RADIUS0 = 1e4, 1e6, 100.0, 100.0  # global_parameters.py:4-18


def straight(x0, x1, K):
    a = np.linspace(0.0, 1.0, K)[:, None]
    return (1 - a) * np.asarray(x0, float)[None] + a * np.asarray(x1, float)[None]


def model_constraints(model, x_init, x_final, robot_radius=0.5, bounds=(-10.0, 10.0), v_max=1.0,
                      w_max=np.pi / 6, obstacles=None, margin=0.0):
    """The constraint data of model.get_constraints as plain arrays."""
    lb, ub = bounds
    if model == "unicycle":
        obs = UNI_OBS if obstacles is None else obstacles
        return dict(model=model, pos_dim=2, x_init=np.asarray(x_init, float), x_final=np.asarray(x_final, float),
                    u_bounds=[(0, 0.0, v_max), (1, -w_max, w_max)], u_soc=None,
                    x_bounds=[(i, lb + robot_radius, ub - robot_radius) for i in range(2)],
                    obs=[(np.asarray(c, float), r + robot_radius) for c, r in obs])
    obs = SI_OBS if obstacles is None else obstacles
    return dict(model=model, pos_dim=3, x_init=np.asarray(x_init, float), x_final=np.asarray(x_final, float),
                u_bounds=[], u_soc=v_max, x_bounds=[(i, lb + robot_radius, ub - robot_radius) for i in range(3)],
                obs=[(np.asarray(c, float), r + robot_radius + margin) for c, r in obs])


def scp_instance(model="unicycle", K=30, Xref=None, Uref=None, sigma_ref=1.0, tr=TRUST_RADIUS0, nsub=16,
                 x_init=None, x_final=None, **kw):
    """One SCProblem instance (sc_problem.py:15-83) at (Xref, Uref, sigma_ref)."""
    n, m = (3, 2) if model == "unicycle" else (3, 3)
    if x_init is None:
        x_init = [-8.0, -8.0, 0.0] if model == "unicycle" else [-8.0, -8.0, -8.0]
    if x_final is None:
        x_final = [8.0, 8.0, 0.0] if model == "unicycle" else [8.0, 8.0, 8.0]
    if Xref is None:
        Xref = straight(x_init, x_final, K)
    if Uref is None:
        Uref = np.zeros((K, m))
    Ab, Bb, Cb, Sb, zb = foh_oracle.foh(model, Xref.T.copy(), Uref.T.copy(), sigma_ref, nsub=nsub)
    p = model_constraints(model, x_init, x_final, **kw)
    p.update(A=Ab.T.reshape(K - 1, n, n).transpose(0, 2, 1), B=Bb.T.reshape(K - 1, m, n).transpose(0, 2, 1),
             C=Cb.T.reshape(K - 1, m, n).transpose(0, 2, 1), S=Sb.T.copy(), z=zb.T.copy(),
             Xref=np.asarray(Xref, float), Uref=np.asarray(Uref, float), sigma_ref=float(sigma_ref), tr=float(tr),
             w_nu=WEIGHT_NU, w_slack=WEIGHT_SLACK, w_sigma=WEIGHT_SIGMA,
             disc=np.hstack([Ab.T, Bb.T, Cb.T, Sb.T, zb.T]))
    return p


def add_admm(p, nbr_refs, Y=None, Lam=None, rho=1.0, d_min=1.0):
    """AgentSolver terms (agent_solver.py:78-95): neighbour reference positions (K,pd) per j."""
    pd = p["pos_dim"]
    K = p["Xref"].shape[0]
    p = dict(p)
    p["nbrs"] = [dict(Pref=np.asarray(r, float)[:, :pd], Y=(np.asarray(r, float)[:, :pd] if Y is None else Y[j]),
                      Lam=np.zeros((K, pd)) if Lam is None else Lam[j]) for j, r in enumerate(nbr_refs)]
    p["rho"], p["d_min"] = float(rho), float(d_min)
    return p
