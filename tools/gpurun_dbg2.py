import sys, os, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import scvx_hip
from oracle import problems as pb
d = torch.device("cuda")
T_ = lambda x, dt=torch.float64: torch.tensor(np.ascontiguousarray(x), device=d, dtype=dt)
sc = pb.dist3_scenario(); T = sc["T"]
A = np.repeat(sc["Ad"][None], T - 1, 0); B = np.repeat(sc["Bd"][None], T - 1, 0)
disc = np.stack([pb.pack_disc(A, B)] * 3)
Xref = np.stack([x[:, 0:6] for x in sc["X_traj"]]); Uref = np.stack([x[:, 6:9] for x in sc["X_traj"]])
xdes = np.stack([x[0:6] for x in sc["x_des"]])
rows = np.zeros((3, T, 2, 4)); cnt = np.zeros((3, T), np.int32)
dr = [pb.collision_rows(sc["X_traj"], i, sc["R"]) for i in range(3)]
for i in range(3):
    for t in range(T - 1): rows[i, t] = dr[i][t]; cnt[i, t] = 2
spec = scvx_hip.QPSpec(model="di", K=T, box=[(0, -1, 22), (1, -1, 20)], j_max=2, w_coll=1e4, tol=1e-10, max_iter=2)
s = scvx_hip.QPSolver(spec, 3)
cap = 100
buf = torch.zeros(8 * cap + 64 * 40 + 16, dtype=torch.float64, device=d)
scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(buf.data_ptr()), 1, cap)
out = s.solve(T_(disc), T_(np.zeros(3)), T_(Xref), T_(Uref), T_(Xref[:, 0]), T_(xdes), T_(np.full(3, sc["tr"])), T_(rows), T_(cnt, torch.int32))
torch.cuda.synchronize()
b = buf.cpu().numpy()
gd = b[8 * cap: 8 * cap + 64 * 40].reshape(64, 40)[:T]
gyi = b[8 * cap + 64 * 40: 8 * cap + 64 * 40 + 6]
cd = np.fromfile(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dbg/cpu_dz1.bin"), dtype=np.float64)
cyi = cd[T * 40: T * 40 + 6]
cd = cd[:T * 40].reshape(T, 40)
np.set_printoptions(linewidth=200, precision=4)
print("max diff dz", np.abs(gd[:, :9] - cd[:, :9]).max(), "aux", np.abs(gd[:, 9:10] - cd[:, 9:10]).max(), "dyi", np.abs(gyi - cyi).max())
for t in [0, 1, 2, 10, 25, 48, 49, 50]:
    print(t, "gpu", gd[t, :10]); print(t, "cpu", cd[t, :10])
print("gyi", gyi, "cyi", cyi)
