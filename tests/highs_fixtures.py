"""Loader of tests/golden/highs_qp_{c3,c4}.npz (written by tests/golden/make_highs_qp_goldens.py): Q1 trust-region
subproblems (Distributed_opt/dist_scvx_3d.py:51-111, no SOC) whose optimum was found by SciPy's HiGHS QP solver
and certified by the convex-QP KKT conditions on its active set.  Every instance has >= 1 active obstacle or
collision row at the optimum."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FAMILIES = ("c3", "c4")
K, W_OBS, W_COLL = 50, 1e6, 1e4
# sum_t ||u_t - u*_t||^2 <= U_BOUND * max(1, |obj*|): the objective's curvature is 2 in every input (t < T-1), so a
# feasible point within 1e-8 relative of the optimal value has its inputs within sum ||du||^2 <= 1e-8 max(1, |obj|);
# the factor 4 covers the stopping rule's primal residual (1e-8 relative) priced by the multipliers
U_BOUND = 4e-8


def load(name):
    f = dict(np.load(os.path.join(HERE, "golden", f"highs_qp_{name}.npz")))
    f["box_list"] = [(int(b[0]), float(b[1]), float(b[2])) for b in f["box"]]
    f["obs_list"] = [(f["obs_c"][i], float(f["obs_r"][i])) for i in range(len(f["obs_r"]))]
    f["jm"] = int(f["j_max"])
    return f


def dense_prob(f, a):
    """oracle/qp_dense.py reference-form dict of instance a."""
    from oracle import problems as pb
    A, B, C, S, z = pb.unpack_disc(f["disc"][a], 6, 3)
    coll = None
    if f["jm"]:
        coll = []
        for t in range(K - 1):
            r = f["rows"][a, t, :f["cnt"][a, t]]
            c = r[:, 3] - r[:, :3] @ f["Xref"][a, t, :3]
            coll.append(np.hstack([r[:, :3], c[:, None]]))
    return dict(A=A, B=B, C=C, c=S * f["sigma"][a] + z, Xref=f["Xref"][a], Uref=f["Uref"][a],
                x_final=f["x_final"][a], tr=float(f["tr"][a]), box=f["box_list"], obs=f["obs_list"], w_obs=W_OBS,
                coll=coll, w_coll=W_COLL, umax=None, fix_last_input=True)


def rel(a, b):
    return np.abs(a - b) / np.maximum(1.0, np.abs(b))


def u_dist(U, f):
    """Per-instance sum_t ||U_t - U*_t||^2 over the priced inputs t < T-1."""
    return ((U - f["U"])[:, :K - 1] ** 2).sum(axis=(1, 2))
