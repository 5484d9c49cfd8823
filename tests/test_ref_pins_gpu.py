"""Reference-held solver results (the only numbers the reference publishes for its solver path),
reproduced through the drop-in SCvx surface (tests/ref_pins.py, one subprocess per scenario so the
doc-era constants are set before any SCvx module binds them).

ADMM (SCvx/docs/documentation_mutli_agent_game.md:465, made by SCvx/examples/compare_admm_vs_nash.py:69-78):
  min-sep 0.5000 and path length 9.5391 are reproduced (tolerances 1e-3 absolute and 1 % relative);
  the control effort is not (63.6 here against 91.06): the document predates the code it sits next to --
  its SCvx chapter states a squared virtual-control objective (documentation_SCvx.md:254-268, 356) where
  SCProblem (sc_problem.py:77-83) has the induced 1-norm -- so the effort of a 20-round, not yet converged
  ADMM run (primal residual 5.8e-3 at round 20) is not comparable.  Recorded, not asserted.
Unicycle sigma 24.1419 (documentation_SCvx.md:383): not reproducible from the code's objective for the
  same reason; no test.
NASH (documentation_mutli_agent_game.md:466, compare_admm_vs_nash.py:81-98): 6 iterations, min-sep 0.5665,
  effort 2.9906, length 9.6735 are NOT reproduced (20 iterations, 0.541, 0.0796, 31.5 here): besides the
  doc-era objective, every best response is non-unique in X (sigma fixed, virtual control priced by the
  induced norm max_k ||nu_k||_1, so every column below the max is free -- tests/test_nash_gpu.py), and the
  iteration follows whichever optimizer the solver returns.  U is unique per solve: the oracle's own IBR
  restatement (oracle/nash_ref.py, a different optimizer choice, length 32.4) ends at effort 0.07960
  against 0.07963 here.  Asserted: the run completes, the boundary conditions hold and the agents keep
  the slab radius 0.5 apart at every node."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(name):
    out = subprocess.run([sys.executable, os.path.join(HERE, "ref_pins.py"), name], capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_admm_default_scenario_matches_documented_min_sep_and_length(cuda):
    r = _run("admm")
    assert r["rounds"] == 20
    assert abs(r["min_sep"] - 0.5000) < 1e-3, r["min_sep"]          # the d_min = 0.5 collision rows bind
    assert abs(r["length"] - 9.5391) < 0.01 * 9.5391, r["length"]
    assert r["primal"][-1] < 0.01 * r["primal"][0]                   # consensus converging
    print("ADMM effort", r["effort"], "(documented 91.0586, not comparable: see module docstring)")


def test_nash_default_game_runs_and_keeps_the_slab_radius(cuda):
    r = _run("nash")
    assert r["iters"] <= 20 and r["hist"][-1] < r["hist"][0]
    assert r["min_sep_xy"] >= 0.5 - 1e-6, r["min_sep_xy"]
    assert 0.0 < r["effort"] < 1.0
    print("NASH", {k: r[k] for k in ("iters", "min_sep", "effort", "length", "seconds")},
          "(documented 6 / 0.5665 / 2.9906 / 9.6735 / 7.57 s: not reproducible, see module docstring)")
