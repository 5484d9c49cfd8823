import sys, os, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, time
import scvx_hip
from oracle import problems as pb
d = torch.device("cuda")
T_ = lambda x, dt=torch.float64: torch.tensor(np.ascontiguousarray(x), device=d, dtype=dt)
for N in (1, 64, 1024):
    K = 50
    sc = pb.synthetic_di(N, K=K, seed=1, obstacles=8)
    X, U, sig = T_(sc["X"]), T_(sc["U"]), T_(sc["sigma"])
    disc = scvx_hip.foh_batched("di", X, U, sig)
    spec = scvx_hip.QPSpec(model="di", K=K, box=[(0,-12,12),(1,-12,12)], obs=sc["obs"], u_max=1.0, max_iter=60)
    s = scvx_hip.QPSolver(spec, N)
    cap = 100
    buf = torch.zeros(8 * cap + 64 * 40 + 32, dtype=torch.float64, device=d)
    scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(buf.data_ptr()), 0, cap)
    args = (disc, sig, X, U, T_(sc["x_init"]), T_(sc["x_final"]), T_(np.full(N, 0.25)))
    out = s.solve(*args); torch.cuda.synchronize()
    t0 = time.time(); out = s.solve(*args); torch.cuda.synchronize(); el = time.time() - t0
    b = buf.cpu().numpy()[8 * cap + 64 * 40 + 16:][:15]
    st = b[3:15]
    print("factor phase cycles (stage 25):", np.diff(st[st > 0]).astype(int).tolist())
    it = out["iters"][0].item()
    print(f"N={N} wall {el*1e3:.2f} ms iters(agent0) {it}  cycles: factor {b[0]:.3e} solve {b[1]:.3e} total {b[2]:.3e}  -> per-iter factor {b[0]/it:.0f} solve(x2) {b[1]/it:.0f} other {(b[2]-b[0]-b[1])/it:.0f}")
