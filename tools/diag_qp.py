"""Diagnostics (not a test): solve the C4 shard / C5 subproblems on the GPU, print status and iteration
histograms, and the IPM trace of one failing agent next to the dense oracle's answer.
usage: python tools/diag_qp.py c4|c5 [agent]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, REPO)


def main(cfg="c4", agent=None, cap=None):
    cap = int(cap or os.environ.get("CAP", 60))
    tol = float(os.environ.get("TOL", 1e-8))
    import torch
    import scvx_hip
    from scvx_hip import workloads
    from oracle import problems as pb, qp_dense as qd
    dev = torch.device("cuda:0")
    T = lambda x, dt=torch.float64: torch.tensor(np.ascontiguousarray(x), device=dev, dtype=dt)  # noqa: E731
    if cfg == "c4":
        sc = workloads.synthetic_lattice(side=16, K=50, seed=2, sigma=30.0)
        model, n_loc, R, box, obs = "di", 512, 2.3, [(0, -50.0, 50.0), (1, -50.0, 50.0)], []
    else:
        sc = workloads.synthetic_quad(64, K=50, seed=3, obstacles=8)
        model, n_loc, R, box, obs = "quad", 64, 0.5, workloads.QUAD_BOX, sc["obs"]
    n, m = scvx_hip.MODEL_DIMS[model]
    sl = slice(0, n_loc)
    X_all = T(sc["X"])
    X, U, sig = T(sc["X"][sl]), T(sc["U"][sl]), T(sc["sigma"][sl])
    disc = scvx_hip.foh_batched(model, X, U, sig)
    rows, cnt = scvx_hip.collision_rows(X_all, 0, n_loc, R, j_max=8)
    spec = scvx_hip.QPSpec(model=model, K=50, box=box, obs=obs, w_obs=1e6, j_max=8, w_coll=1e4, tol=tol,
                           max_iter=cap)
    solver = scvx_hip.QPSolver(spec, n_loc, device=dev)
    tr = np.full(n_loc, 0.25)
    out = solver.solve(disc, sig, X, U, T(sc["x_init"][sl]), T(sc["x_final"][sl]), T(tr), rows, cnt)
    st, it = out["status"].cpu().numpy(), out["iters"].cpu().numpy()
    print("status", np.bincount(st, minlength=3), "iters hist", dict(zip(*np.unique(it, return_counts=True))))
    codes = torch.zeros(n_loc, dtype=torch.float64, device=dev)
    scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(codes.data_ptr()), -1, 0)
    out = solver.solve(disc, sig, X, U, T(sc["x_init"][sl]), T(sc["x_final"][sl]), T(tr), rows, cnt)
    torch.cuda.synchronize()
    scvx_hip.lib().scvx_qp_set_trace(None, 0, 0)
    cd = codes.cpu().numpy().astype(int)
    for s_ in (1, 2):
        print(f"status {s_} agents / exit codes / iters:", [(int(i), int(cd[i]), int(it[i])) for i in np.nonzero(st == s_)[0][:24]])
    a = int(agent) if agent is not None else int(np.nonzero(st == 2)[0][0]) if (st == 2).any() else \
        int(np.nonzero(st == 1)[0][0]) if (st == 1).any() else 0
    buf = torch.zeros(8 * cap + 32, dtype=torch.float64, device=dev)
    scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(buf.data_ptr()), a, cap)
    out = solver.solve(disc, sig, X, U, T(sc["x_init"][sl]), T(sc["x_final"][sl]), T(tr), rows, cnt)
    torch.cuda.synchronize()
    scvx_hip.lib().scvx_qp_set_trace(None, 0, 0)
    bb = buf.cpu().numpy()
    print(f"agent {a}: status {out['status'][a].item()} iters {out['iters'][a].item()} fail_code {bb[8 * cap + 3]} "
          f"obj {out['obj'][a].item():.9e}")
    b = bb[:8 * cap].reshape(cap, 8)
    for i in range(min(int(out["iters"][a].item()) + 1, cap)):
        print("  it %2d pres %.2e dres %.2e gap %.2e pobj %.9e aa %.3f al %.3f sg %.2e mu %.2e" % ((i,) + tuple(b[i])))
    dn = disc.cpu().numpy()
    A, B, C, S, z = pb.unpack_disc(dn[a], n, m)
    rr, cc = rows.cpu().numpy()[a], cnt.cpu().numpy()[a]
    coll = []
    for t in range(49):
        r = rr[t, :cc[t]]
        coll.append(np.hstack([r[:, :3], (r[:, 3] - r[:, :3] @ sc["X"][a, t, :3])[:, None]]))
    prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a], x_final=sc["x_final"][a],
                tr=0.25, box=box, obs=obs, w_obs=1e6, coll=coll, w_coll=1e4, fix_last_input=True)
    with np.errstate(all="ignore"):
        Xd, Ud, objd, info = qd.solve_agent(prob, tol=1e-10, maxit=150)
    print("dense oracle:", info["status"], info["iters"], f"obj {objd:.9e}", "rows/node", cc[:49].min(), cc[:49].max())


def run(cfg="c5", iters=7):
    """The bench's coupled driver for `iters` SCvx iterations: per iteration, status / exit-code histograms,
    the trust radius and the full-row check; then the dense oracle on the first failing subproblem."""
    import torch
    import bench
    import scvx_hip
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    from oracle import problems as pb, qp_dense as qd
    dev = torch.device("cuda:0")
    sc, w, cfgd = bench.make_coupled(cfg, 1, 0, dev)
    model = cfgd["model"]
    n, m = scvx_hip.MODEL_DIMS[model]
    wf = float(os.environ.get("WF", 0))
    spec = scvx_hip.QPSpec(model=model, K=bench.K, box=cfgd["box"], obs=cfgd["obs"], w_obs=1e6,
                           j_max=cfgd["j_max"], w_coll=1e4, max_iter=60, has_final=wf <= 0, w_final=wf)
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0,
                     coupling=CouplingSpec(R=cfgd["R"], check=os.environ.get("CHECK", "1") == "1",
                                           j_max_hi=int(os.environ.get("JHI", 32))),
                     tr_rule="global", on_fail=os.environ.get("ONFAIL", "halve"),
                     tr_max=float(os.environ.get("TRMAX", bench.TR0)))
    X, U = w["X"].clone(), w["U"].clone()
    codes = torch.zeros(X.shape[0], dtype=torch.float64, device=dev)
    for it in range(int(iters)):
        Xp, Up, trp = X.clone(), U.clone(), drv.tr.clone()
        scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(codes.data_ptr()), -1, 0)
        Xn, Un, o = drv.step(X, U)
        torch.cuda.synchronize()
        scvx_hip.lib().scvx_qp_set_trace(None, 0, 0)
        st = o["status"].cpu().numpy()
        cd = codes.cpu().numpy().astype(int)
        print(f"iter {it}: tr {trp.min().item():.4g}..{trp.max().item():.4g} status {np.bincount(st, minlength=3)} exit codes "
              f"{dict(zip(*np.unique(cd[st == 2], return_counts=True)))} iters mean {o['iters'].float().mean().item():.1f} "
              f"check {drv.last_check} terminal err max {(Xn[:, -1] - w['x_final']).abs().max().item():.3e} "
              f"cost {(Un[:, :-1] ** 2).sum().item():.6e}", flush=True)
        bad = np.nonzero(st == 2)[0]
        if it == int(iters) - 1 and bad.size:
            a = int(bad[0])
            dn = drv.disc[a].cpu().numpy()
            A, B, C, S, z = pb.unpack_disc(dn, n, m)
            rr, cc = drv.rows[a].cpu().numpy(), drv.count[a].cpu().numpy()
            Xr = Xp[a].cpu().numpy()
            coll = []
            for t in range(bench.K - 1):
                r = rr[t, :cc[t]]
                coll.append(np.hstack([r[:, :3], (r[:, 3] - r[:, :3] @ Xr[t, :3])[:, None]]))
            prob = dict(A=A, B=B, C=C, c=S * w["sigma"][a].item() + z, Xref=Xr, Uref=Up[a].cpu().numpy(),
                        x_final=w["x_final"][a].cpu().numpy(), tr=trp[a].item(), box=cfgd["box"], obs=cfgd["obs"],
                        w_obs=1e6, coll=coll, w_coll=1e4, fix_last_input=True)
            with np.errstate(all="ignore"):
                Xd, Ud, objd, info = qd.solve_agent(prob, tol=1e-9, maxit=150)
            print(f"agent {a} exit {cd[a]}: dense oracle {info['status']} iters {info['iters']} obj {objd:.6e} "
                  f"cert {info['cert']}")
        X.copy_(Xn)
        U.copy_(Un)


def jac(iters=3):
    """The C5 n64 test's coupled loop: per step, status histogram; for agents that exit at 0 IPM
    iterations, a re-solve of the step's subproblems with per-agent exit codes."""
    import torch
    import scvx_hip
    from scvx_hip import workloads
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    dev = torch.device("cuda:0")
    T = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev, dtype=torch.float64)  # noqa: E731
    N, K = 64, 50
    sc = workloads.synthetic_quad(N, K=K, seed=3, obstacles=8)
    box = workloads.QUAD_BOX
    spec = scvx_hip.QPSpec(model="quad", K=K, box=box, obs=sc["obs"], w_obs=1e6, j_max=8, w_coll=1e4, tol=1e-8,
                           max_iter=60)
    drv = JacobiSCvx(spec, T(sc["x_init"]), T(sc["x_final"]), T(sc["sigma"]), 0.25, coupling=CouplingSpec(R=0.5),
                     tr_rule="global")
    X, U = T(sc["X"]), T(sc["U"])
    for k in range(int(iters)):
        Xp, Up, trp = X.clone(), U.clone(), drv.tr.clone()
        X, U, o = drv.step(X, U)
        st, it = o["status"].cpu().numpy(), o["iters"].cpu().numpy()
        print(f"step {k}: tr {trp[0].item():.4g} status {np.bincount(st, minlength=3)} zero-it {np.nonzero(it == 0)[0]}")
        if (it == 0).any():
            codes = torch.zeros(N, dtype=torch.float64, device=dev)
            scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(codes.data_ptr()), -1, 0)
            o2 = drv.solver.solve(drv.disc, drv.sigma, Xp, Up, drv.x_init, drv.x_final, trp, drv.rows, drv.count)
            torch.cuda.synchronize()
            scvx_hip.lib().scvx_qp_set_trace(None, 0, 0)
            z = np.nonzero(o2["iters"].cpu().numpy() == 0)[0]
            print("   re-solve zero-it agents", z, "codes", codes.cpu().numpy()[z], "U min thrust",
                  [float(Up[a, :, 0].min()) for a in z])
            for a in z:
                d = drv.disc[a].cpu().numpy()
                xa = Xp[a].cpu().numpy()
                print(f"   agent {a}: disc finite {np.isfinite(d).all()} max|disc| {np.abs(d).max():.3e} "
                      f"max|angles| {np.abs(xa[:, 6:9]).max():.3f} max|rates| {np.abs(xa[:, 9:12]).max():.3f} "
                      f"max|v| {np.abs(xa[:, 3:6]).max():.3f} U range {Up[a].min().item():.3f} {Up[a].max().item():.3f}")
                np.savez(f"gpurun_out/c5_zero_{k}_{a}.npz", disc=d, X=xa, U=Up[a].cpu().numpy(), tr=trp[a].item(),
                         rows=drv.rows[a].cpu().numpy(), count=drv.count[a].cpu().numpy(),
                         x_init=drv.x_init[a].cpu().numpy(), x_final=drv.x_final[a].cpu().numpy(),
                         sigma=drv.sigma[a].item())


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        run(*sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "jac":
        jac(*sys.argv[2:])
    else:
        main(*sys.argv[1:])
