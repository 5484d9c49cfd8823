"""CPU, no GPU: the trust-radius bookkeeping of the Jacobi driver (scvx_hip.scvx.JacobiSCvx.step) for
failed subproblems -- "halve" (default) and "grow" (x2 up to tr_max) -- and the cost rule of
Distributed_opt/dist_scvx_3d.py:248-252 (per-agent form), with stub kernels through the backend hook."""
import pytest
import torch

from scvx_hip import QPSpec
from scvx_hip.scvx import JacobiSCvx


class _StubQP:
    def __init__(self, status):
        self.status = status

    def solve(self, disc, sigma, Xref, Uref, x_init, x_final, tr, rows=None, count=None, n=None, warm=None):
        N = Xref.shape[0]
        return {"X": Xref + 1.0, "U": Uref * 0.5, "slack_coll": torch.zeros(N, Xref.shape[1], dtype=torch.float64),
                "obj": torch.zeros(N, dtype=torch.float64), "status": self.status.clone(),
                "iters": torch.ones(N, dtype=torch.int32)}


class _StubBackend:
    def __init__(self, status):
        self.status = status

    def foh(self, model, X, U, sigma, nsub, out):
        return torch.zeros(X.shape[0], X.shape[1] - 1, 90, dtype=torch.float64)

    def qp_solver(self, spec, N, device):
        return _StubQP(self.status)


@pytest.mark.parametrize("on_fail", ["halve", "grow"])
def test_failed_agent_trust_radius(on_fail):
    N, K = 3, 5
    status = torch.tensor([0, 1, 2], dtype=torch.int32)
    X = torch.zeros(N, K, 6, dtype=torch.float64)
    U = torch.ones(N, K, 3, dtype=torch.float64)
    drv = JacobiSCvx(QPSpec(model="di", K=K), torch.zeros(N, 6), torch.zeros(N, 6), torch.ones(N), 0.25,
                     backend=_StubBackend(status), on_fail=on_fail, tr_max=0.5)
    Xn, Un, _ = drv.step(X, U)
    # failed agent 2 keeps its iterate; the others take the step
    assert torch.equal(Xn[2], X[2]) and torch.equal(Un[2], U[2])
    assert torch.equal(Xn[0], X[0] + 1.0)
    # first step: no cost increase (prev cost = inf); failure: x1/2 or x2 (clamped to tr_max)
    assert drv.tr.tolist() == [0.25, 0.25, 0.125 if on_fail == "halve" else 0.5]
    Xn, Un, _ = drv.step(Xn, Un)
    # agents 0, 1: cost fell (U halved) -> unchanged; agent 2 failed again
    assert drv.tr.tolist() == [0.25, 0.25, 0.0625 if on_fail == "halve" else 0.5]


def test_on_fail_rejects_unknown_rule():
    with pytest.raises(ValueError):
        JacobiSCvx(QPSpec(model="di", K=5), torch.zeros(1, 6), torch.zeros(1, 6), torch.ones(1), 0.25,
                   backend=_StubBackend(torch.zeros(1, dtype=torch.int32)), on_fail="keep")
