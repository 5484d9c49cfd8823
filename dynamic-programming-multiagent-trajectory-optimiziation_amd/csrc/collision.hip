// Batched pairwise collision linearization (the inter-agent coupling of the Jacobi SCvx step).
//
// Replaces the per-agent, per-node, per-neighbour Python loop of
// Distributed_opt/dist_scvx_3d.py:93-107:
//     S = 2R - ||p_i - p_j||,   S_grad = (p_i - p_j)/||p_i - p_j||,   S - S_grad' d_t <= S_t
// evaluated at the previous iterate for every node t < T-1.  Rows are emitted in the absolute form
// consumed by scvx_qp_solve_batched:  b - g' p_t <= S_t  with g = S_grad and b = S + g' pbar_i.
// (No epsilon in the normal: coincident agents give NaN exactly as the reference's 0/0.)
//
// Exact mode (cull_radius <= 0 and j_max >= N_total-1) reproduces the reference's full neighbour
// set.  With culling only neighbours closer than cull_radius are kept, and at most j_max of them
// per node (the closest ones, i.e. the rows with the largest violation S); the QP is then exact
// whenever the culled rows stay inactive, which the host layer verifies after the solve.
//
// Mapping: one 64-lane workgroup per local agent, lane = node t; every lane streams all N_total
// positions of its node (X_all rows are read with consecutive lanes on consecutive nodes) and
// keeps its current top-j_max list in the output rows (the list's worst entry tracked in
// registers).  X_all is the all-gathered [N_total][K][n_x] state (RCCL all_gather over xGMI).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "scvx_hip.h"

namespace scvx {

__global__ __launch_bounds__(64) void collision_rows_kernel(int K, int pd, int nx, int N_total,
                                                            const double* __restrict__ X_all, int i0, double R,
                                                            double cull, int j_max, double* __restrict__ rows,
                                                            int32_t* __restrict__ count) {
    const int t = threadIdx.x;
    const long long a = blockIdx.x;  // local agent
    const long long gi = i0 + a;     // global agent index
    if (t >= K) return;
    int32_t* cnt = count + a * K + t;
    if (t >= K - 1) { *cnt = 0; return; }
    double pi[3] = {0, 0, 0};
    for (int d = 0; d < pd; ++d) pi[d] = X_all[(gi * K + t) * nx + d];
    double* out = rows + (a * K + t) * (long long)j_max * (pd + 1);
    int n = 0;
    int worst = 0;
    double worst_c = 1e300;  // smallest S among kept rows (the one to evict)
    const double cull2 = cull > 0 ? cull * cull : -1.0;
    for (long long j = 0; j < N_total; ++j) {
        if (j == gi) continue;
        double diff[3] = {0, 0, 0}, d2 = 0.0;
        for (int d = 0; d < pd; ++d) {
            diff[d] = pi[d] - X_all[(j * K + t) * nx + d];
            d2 += diff[d] * diff[d];
        }
        if (cull2 > 0 && !(d2 < cull2)) continue;
        const double nr = sqrt(d2);
        const double c = 2.0 * R - nr;
        int slot;
        if (n < j_max) {
            slot = n++;
        } else {
            if (!(c > worst_c)) continue;
            slot = worst;
        }
        double* row = out + slot * (pd + 1);
        double b = c;
        for (int d = 0; d < pd; ++d) {
            const double g = diff[d] / nr;
            row[d] = g;
            b += g * pi[d];
        }
        row[pd] = b;
        // S of the stored row: c = b - g'pbar_i
        if (n == j_max) {  // recompute the eviction candidate
            worst_c = 1e300;
            for (int k = 0; k < j_max; ++k) {
                const double* rk = out + k * (pd + 1);
                double ck = rk[pd];
                for (int d = 0; d < pd; ++d) ck -= rk[d] * pi[d];
                if (ck < worst_c) { worst_c = ck; worst = k; }
            }
        }
    }
    *cnt = n;
}

}  // namespace scvx

extern "C" int scvx_collision_rows_batched(int K, int pos_dim, int n_x, int N_total, const double* X_all, int i0,
                                           int N_local, double R, double cull_radius, int j_max, double* rows,
                                           int32_t* count, void* stream) {
    if (K < 2 || K > 64 || pos_dim < 1 || pos_dim > 3 || pos_dim > n_x || N_total < 0 || N_local < 0 || i0 < 0 ||
        i0 + N_local > N_total || j_max < 1 || !X_all || !rows || !count)
        return scvx::set_error(SCVX_EINVAL, "collision: bad args");
    if (N_local == 0) return SCVX_OK;
    hipLaunchKernelGGL(scvx::collision_rows_kernel, dim3(N_local), dim3(64), 0, (hipStream_t)stream, K, pos_dim,
                       n_x, N_total, X_all, i0, R, cull_radius, j_max, rows, count);
    return scvx::check_launch("collision_rows_kernel");
}
