"""Loader of tests/golden/c4_stiff_subset.npz (tests/golden/make_c4_stiff_subset.py): twelve late-step C4
trust-region subproblems (Distributed_opt/dist_scvx_3d.py:51-111 with collision rows) whose active L1 trust-region
facets carry barrier weights ~1e12.  kind 0: the CPU twin ends optimal with its stiff-facet stage system and
optimal_inaccurate without it; kind 1: optimal_inaccurate with it too (the state-side limit);
kind 2: solved to full accuracy by the GPU loop.  `cert` / `obj_cert`: SciPy HiGHS's active-set optimum, certified by
the convex-QP KKT conditions, where it certifies (7 of 12)."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
K, W_COLL, J_MAX, BOX = 50, 1e4, 8, [(0, -50.0, 50.0), (1, -50.0, 50.0)]
INPUTS = ("disc", "sigma", "X", "U", "x_init", "x_final", "tr", "rows", "count")


def load():
    return dict(np.load(os.path.join(HERE, "golden", "c4_stiff_subset.npz")))
