"""Writes tests/golden/c4_stiff_subset.npz: twelve late-step C4 trust-region subproblems for the CPU test of the
stiff-facet stage system (tests/test_stiff_facets_cpu.py).

Source: the step-17 dump of the GPU C4 loop (`DUMP_ALL=1 python tools/c4_drift.py ...` on an MI355X, written to
gpurun_out/c4_late_step17.npz: every status-1 subproblem of that step and 64 status-0 ones; round 5).  The CPU
twin (oracle/scvx_cpu.cpp) re-solves all of them cold twice, with its stiff-facet stage system on and off
(SCVX_TWIN_STIFF=1 / 0, one process each), and the subset keeps
  * 8 subproblems that end optimal with the stage system and optimal_inaccurate without it,
  * 2 that stay optimal_inaccurate with it (the state-side limit),
  * 2 that the GPU loop solved to full accuracy;
and, per subproblem, SciPy HiGHS's active-set optimum certified by the convex-QP KKT conditions on its active set
(tests/golden/make_highs_qp_goldens.py: assemble / solve_highs / certify; `cert` 0 where it does not certify).
usage: python tests/golden/make_c4_stiff_subset.py <dump.npz>   (runs the twin in two child processes)"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
KEYS = ("disc", "sigma", "X", "U", "x_init", "x_final", "tr", "rows", "count")
CHILD = """
import sys, numpy as np
sys.path[:0] = [{repo!r}, {pkg!r}]
from oracle import qp_cpu
d = np.load({dump!r})
tpl = qp_cpu.make_template(6, 3, 50, box=[(0, -50., 50.), (1, -50., 50.)], j_max=8, w_coll=1e4, tol=1e-8, max_iter=60)
o = qp_cpu.solve_batched(tpl, *[d[k] for k in {keys!r}], nthreads=8)
np.save({out!r}, o["status"])
"""


def twin_status(dump, stiff):
    out = f"/tmp/c4_stiff_status_{stiff}.npy"
    code = CHILD.format(repo=REPO, pkg=os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"),
                        dump=dump, keys=KEYS, out=out)
    subprocess.run([sys.executable, "-c", code], check=True, env=dict(os.environ, SCVX_TWIN_STIFF=str(stiff)))
    return np.load(out)


def main(dump):
    d = np.load(dump)
    on, off = twin_status(dump, 1), twin_status(dump, 0)
    repaired = np.nonzero((on == 0) & (off == 1))[0]
    still = np.nonzero(on == 1)[0]
    gpu0 = np.nonzero(d["status"] == 0)[0]
    pick = np.concatenate([repaired[:: max(1, len(repaired) // 8)][:8], still[:2], gpu0[:2]])
    out = {k: d[k][pick] for k in KEYS}
    sys.path.insert(0, HERE)
    import make_highs_qp_goldens as mh
    cert, obj_cert = np.zeros(len(pick), np.int32), np.full(len(pick), np.nan)
    for i, a in enumerate(pick):
        P = mh.assemble(d["disc"][a], float(d["sigma"][a]), d["X"][a], d["U"][a], d["x_init"][a], d["x_final"][a],
                        float(d["tr"][a]), [(0, -50.0, 50.0), (1, -50.0, 50.0)], [], d["rows"][a], d["count"][a])
        _, zh, _ = mh.solve_highs(P)
        if len(zh) == P["nv"] and np.all(np.isfinite(zh)):
            ok, z, _ = mh.certify(P, zh)
            if ok:
                cert[i], obj_cert[i] = 1, mh.unpack(P, z, d["U"][a])[3]
    out.update(cert=cert, obj_cert=obj_cert)
    out.update(agents=d["agents"][pick], gpu_status=d["status"][pick], twin_status_stiff=on[pick],
               twin_status_plain=off[pick], kind=np.array([0] * 8 + [1] * 2 + [2] * 2))
    np.savez_compressed(os.path.join(HERE, "c4_stiff_subset.npz"), **out)
    print("picked", pick.tolist(), "twin with / without the stage system:", on[pick].tolist(), off[pick].tolist(),
          "HiGHS certified:", cert.tolist())


if __name__ == "__main__":
    main(sys.argv[1])
