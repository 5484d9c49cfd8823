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
// per node (the closest ones, i.e. the rows with the largest violation S).  The culled QP is a
// relaxation of the reference's (it drops rows), so its solution is the reference's solution
// whenever it also satisfies every dropped row: collision_check_kernel below evaluates ALL
// N_total-1 rows of every node at the solution, and the host (scvx_hip/scvx.py JacobiSCvx)
// re-solves the agents with a violated row at a larger j_max, flagging any that still violate.
//
// Mapping: one workgroup per (node t, block of 64 local agents), lane = local agent.  All lanes scan
// the same neighbour sequence j = 0..N_total-1, so node t's positions of a tile of TJ neighbours are
// staged in LDS once per workgroup (cooperative loads) and read back as LDS broadcasts; the X_all
// traffic is then ~N_total*pos_dim*8 bytes per workgroup instead of per agent.  Each lane keeps its
// top-j_max list (S values and neighbour indices) in registers and writes its rows once at the end.
// The kept SET is that of a reference-order sequential scan (up to how exact distance ties are
// broken); the row ORDER is the insertion order of the pre-filtered scan below (the tau bound skips
// neighbours a sequential scan would have inserted and later evicted), so it is not the sequential
// scan's slot order -- the QP's solution depends on the order only through rounding.  X_all is the
// all-gathered [N_total][K][n_x] state (RCCL all_gather over xGMI).
//
// Indexed form (scvx_collision_rows_indexed): local agent a is global agent idx[a] instead of i0 + a
// -- the rows of an arbitrary subset, e.g. the agents the full-row check found violating.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "scvx_hip.h"

namespace scvx {

constexpr int COLL_TJ = 512;  // neighbours staged per LDS tile
constexpr int COLL_CH = 8;    // neighbours per branch-free chunk of the scans

// |p_i - p_j|^2 summed in coordinate order (d0^2 + d1^2) + d2^2, the rounding of the sequential
// scan the selection and the check were pinned with.  Positions past pos_dim are 0 in both operands
// (tile and lane registers), so the unused terms add exact zeros.
__device__ __forceinline__ double coll_d2(const double* pi, const double* pj, int) {
    const double d0 = pi[0] - pj[0], d1 = pi[1] - pj[1], d2 = pi[2] - pj[2];
    return fma(d2, d2, fma(d1, d1, d0 * d0));
}

// Stage node t's positions of neighbours [j0, j0 + nt) in LDS as [jj][3] (zeros past pos_dim), and
// pad the tile to a whole chunk with far-away positions (|d|^2 = inf: never kept, never checked), so
// the chunk loops need no bounds tests.
__device__ __forceinline__ void coll_stage(double* tile, const double* __restrict__ X_all, int j0, int nt, int K,
                                           int t, int nx, int pd, int lane) {
    const int ntp = (nt + COLL_CH - 1) / COLL_CH * COLL_CH;
    for (int e = lane; e < ntp * 3; e += 64) {
        const int jj = e / 3, d = e - jj * 3;
        tile[e] = jj >= nt ? 1e200 : (d < pd ? X_all[((long long)(j0 + jj) * K + t) * nx + d] : 0.0);
    }
}

template <int JM>
__global__ __launch_bounds__(64) void collision_rows_kernel(int K, int pd, int nx, int N_total, int N_local,
                                                            const double* __restrict__ X_all, int i0,
                                                            const int32_t* __restrict__ idx, double R,
                                                            double cull, int j_max, double* __restrict__ rows,
                                                            int32_t* __restrict__ count) {
    __shared__ double tile[COLL_TJ * 3];
    const int lane = threadIdx.x;
    const int t = blockIdx.y;
    const long long a = (long long)blockIdx.x * 64 + lane;  // local agent
    const bool live = a < N_local;
    const long long gi = idx ? (live ? (long long)idx[a] : -1) : i0 + a;  // global agent index
    if (t >= K - 1) {             // no rows at the last node
        if (live) count[a * K + t] = 0;
        return;
    }
    double pi[3] = {0, 0, 0};
    if (live)
        for (int d = 0; d < pd; ++d) pi[d] = X_all[(gi * K + t) * nx + d];
    // selection on squared distances: S = 2R - |d| is decreasing in |d|^2, so "largest S kept,
    // evict the smallest" is "smallest |d|^2 kept, evict the largest" (no sqrt in the scan)
    double kd[JM];
    int kj[JM];
#pragma unroll
    for (int k = 0; k < JM; ++k) { kd[k] = 0.0; kj[k] = -1; }
    int n = 0, worst = 0;
    double worst_d2 = -1.0;  // largest |d|^2 among kept rows (the one to evict)
    const double cull2 = cull > 0 ? cull * cull : -1.0;
    // A first bound tau on the j_max-th smallest |d|^2: the j_max-th smallest over this wave's other
    // agents (their positions are the lanes' pi).  Every kept row has |d|^2 <= tau, so the scan below
    // considers only those: the kept set is unchanged (rows are stored in insertion order), and the
    // insertion code runs for a few dozen neighbours instead of whenever one lane's list changes.
    __shared__ double blk[64 * 3];
#pragma unroll
    for (int d = 0; d < 3; ++d) blk[lane * 3 + d] = pi[d];
    __syncthreads();
    double tau = 1e300;
    if (live) {
        double sv[JM];  // ascending
#pragma unroll
        for (int k = 0; k < JM; ++k) sv[k] = 1e300;
        const long long b0 = (long long)blockIdx.x * 64;
        for (int l = 0; l < 64; ++l) {
            if (l == lane || b0 + l >= N_local) continue;
            const double d2 = coll_d2(pi, blk + l * 3, pd);
            if (cull2 > 0 && !(d2 < cull2)) continue;
#pragma unroll
            for (int k = JM - 1; k > 0; --k) sv[k] = d2 < sv[k - 1] ? sv[k - 1] : fmin(sv[k], d2);
            sv[0] = fmin(sv[0], d2);
        }
#pragma unroll
        for (int k = 0; k < JM; ++k) tau = (k == j_max - 1) ? sv[k] : tau;
    }
    for (int j0 = 0; j0 < N_total; j0 += COLL_TJ) {
        const int nt = min(COLL_TJ, N_total - j0);
        __syncthreads();
        coll_stage(tile, X_all, j0, nt, K, t, nx, pd, lane);
        __syncthreads();
        if (!live) continue;
        for (int jb = 0; jb < nt; jb += COLL_CH) {
            // squared distances of a chunk of neighbours, branch-free (independent LDS broadcasts and
            // FMAs); the sequential insertion below runs only if some lane of the wave may keep one
            double d2v[COLL_CH], m = 1e300;
#pragma unroll
            for (int c = 0; c < COLL_CH; ++c) {
                d2v[c] = coll_d2(pi, tile + (jb + c) * 3, pd);
                m = fmin(m, d2v[c]);
            }
            // some element of the chunk may enter the list iff its smallest |d|^2 may
            const bool need = m <= tau && (n < j_max || m < worst_d2);
            if (!__builtin_amdgcn_ballot_w64(need)) continue;
#pragma unroll
            for (int c = 0; c < COLL_CH; ++c) {
                const long long j = j0 + jb + c;
                const double d2 = d2v[c];
                if (jb + c >= nt || j == gi || !(d2 <= tau) || (cull2 > 0 && !(d2 < cull2))) continue;
                int slot;
                if (n < j_max) {
                    slot = n++;
                } else {
                    if (!(d2 < worst_d2)) continue;
                    slot = worst;
                }
#pragma unroll
                for (int k = 0; k < JM; ++k)
                    if (k == slot) { kd[k] = d2; kj[k] = (int)j; }
                if (n == j_max) {  // recompute the eviction candidate (first maximum, as a sequential scan)
                    worst_d2 = -1.0;
#pragma unroll
                    for (int k = 0; k < JM; ++k)
                        if (k < j_max && kd[k] > worst_d2) { worst_d2 = kd[k]; worst = k; }
                }
            }
        }
    }
    if (!live) return;
    double* out = rows + (a * K + t) * (long long)j_max * (pd + 1);
#pragma unroll
    for (int k = 0; k < JM; ++k) {
        if (k >= n) break;
        const long long j = kj[k];
        double diff[3] = {0, 0, 0}, d2 = 0.0;
        for (int d = 0; d < pd; ++d) {
            diff[d] = pi[d] - X_all[(j * K + t) * nx + d];
            d2 += diff[d] * diff[d];
        }
        const double nr = sqrt(d2);
        double b = 2.0 * R - nr;
        for (int d = 0; d < pd; ++d) {
            const double g = diff[d] / nr;
            out[k * (pd + 1) + d] = g;
            b += g * pi[d];
        }
        out[k * (pd + 1) + pd] = b;
    }
    count[a * K + t] = n;
}

// A-posteriori check of the full reference row set at a solution (dist_scvx_3d.py:93-107):
//     (2R - ||pbar_i - pbar_j||) - g_ij' (p_t - pbar_i) <= S_t     for every j != i, t < K-1
// with pbar the linearisation point (X_all, the previous iterate of every agent), p_t the solved
// position of local agent i and S_t its solved shared slack.  Same mapping as collision_rows_kernel
// (workgroup = (node t, 64 local agents), neighbour positions staged in LDS).  Per (agent, node):
// the number of rows violated by more than tol and the largest violation.
// Bound skip: by Cauchy-Schwarz |g'dp| <= |dp|, so a row's value is at most 2R + |dp| - S - ||pbar_i -
// pbar_j||.  A neighbour whose squared distance is at least (2R + |dp| - S - m)^2, m = min(largest value
// so far, tol), can neither be counted nor raise the maximum, and its sqrt / division are skipped
// (both outputs stay exact; coincident agents still give NaN).
__global__ __launch_bounds__(64) void collision_check_kernel(int K, int pd, int nx, int N_total, int N_local,
                                                             const double* __restrict__ X_all, int i0, double R,
                                                             const double* __restrict__ X_new,
                                                             const double* __restrict__ slack, double tol,
                                                             int32_t* __restrict__ viol, double* __restrict__ vmax) {
    __shared__ double tile[COLL_TJ * 3];
    const int lane = threadIdx.x;
    const int t = blockIdx.y;
    const long long a = (long long)blockIdx.x * 64 + lane;
    const bool live = a < N_local;
    const long long gi = i0 + a;
    if (t >= K - 1) {
        if (live) { viol[a * K + t] = 0; vmax[a * K + t] = 0.0; }
        return;
    }
    double pi[3] = {0, 0, 0}, dp[3] = {0, 0, 0}, S = 0.0;
    if (live) {
        for (int d = 0; d < pd; ++d) {
            pi[d] = X_all[(gi * K + t) * nx + d];
            dp[d] = X_new[(a * K + t) * nx + d] - pi[d];
        }
        S = slack[a * K + t];
    }
    int nv = 0;
    double worst = -1e300;
    const double rr = 2.0 * R;
    const double ndp = sqrt(dp[0] * dp[0] + dp[1] * dp[1] + dp[2] * dp[2]);
    double skip2 = 1e300;  // skip the exact row when d2 >= skip2 (none before the first row)
    // the rows of this wave's other agents first (their positions are the lanes' pi, usually the
    // nearest ones): the bound then skips most of the scan below, which leaves those agents out
    __shared__ double blk[64 * 3];
#pragma unroll
    for (int d = 0; d < 3; ++d) blk[lane * 3 + d] = pi[d];
    __syncthreads();
    const long long b0 = (long long)blockIdx.x * 64;
    const long long blo = i0 + b0, bhi = i0 + min(b0 + 64, (long long)N_local);  // global [blo, bhi)
    auto row = [&](const double* pj) __attribute__((always_inline)) {
        double gd = 0.0;
        for (int d = 0; d < pd; ++d) gd += (pi[d] - pj[d]) * dp[d];
        const double d2 = coll_d2(pi, pj, pd);
        if (!(d2 < skip2)) return;
        const double nr = sqrt(d2);
        const double v = (rr - nr) - gd / nr - S;  // NaN for coincident agents, as the reference's 0/0
        worst = (v > worst || v != v) ? v : worst;
        nv += (v > tol || v != v) ? 1 : 0;
        // fmin ignores a NaN maximum: the count threshold tol still bounds the skip
        const double cb = (rr + ndp - S - fmin(worst, tol)) * (1.0 + 1e-12) + 1e-12;
        skip2 = cb > 0.0 ? cb * cb : 1e-300;  // cb <= 0: every row but a coincident one (d2 = 0) skips
    };
    if (live) {
        for (int l = 0; l < 64; ++l)
            if (l != lane && b0 + l < N_local) row(blk + l * 3);
    }
    for (int j0 = 0; j0 < N_total; j0 += COLL_TJ) {
        const int nt = min(COLL_TJ, N_total - j0);
        __syncthreads();
        coll_stage(tile, X_all, j0, nt, K, t, nx, pd, lane);
        __syncthreads();
        if (!live) continue;
        for (int jb = 0; jb < nt; jb += COLL_CH) {
            double d2v[COLL_CH], m = 1e300;
#pragma unroll
            for (int c = 0; c < COLL_CH; ++c) {
                d2v[c] = coll_d2(pi, tile + (jb + c) * 3, pd);
                m = fmin(m, d2v[c]);
            }
            const bool need = m < skip2;  // (block-mates, done above, are skipped below)
            if (!__builtin_amdgcn_ballot_w64(need)) continue;
#pragma unroll
            for (int c = 0; c < COLL_CH; ++c) {
                const int jj = jb + c;
                const long long j = j0 + jj;
                if (jj >= nt || (j >= blo && j < bhi) || !(d2v[c] < skip2)) continue;
                row(tile + jj * 3);
            }
        }
    }
    if (!live) return;
    viol[a * K + t] = nv;
    vmax[a * K + t] = worst;
}

}  // namespace scvx

extern "C" int scvx_collision_check_batched(int K, int pos_dim, int n_x, int N_total, const double* X_all, int i0,
                                            int N_local, double R, const double* X_new, const double* slack,
                                            double tol, int32_t* viol, double* vmax, void* stream) {
    if (K < 2 || K > 64 || pos_dim < 1 || pos_dim > 3 || pos_dim > n_x || N_total < 0 || N_local < 0 || i0 < 0 ||
        i0 + N_local > N_total || !X_all || !X_new || !slack || !viol || !vmax)
        return scvx::set_error(SCVX_EINVAL, "collision_check: bad args");
    if (N_local == 0) return SCVX_OK;
    const dim3 grid((unsigned)((N_local + 63) / 64), (unsigned)K);
    hipLaunchKernelGGL(scvx::collision_check_kernel, grid, dim3(64), 0, (hipStream_t)stream, K, pos_dim, n_x, N_total,
                       N_local, X_all, i0, R, X_new, slack, tol, viol, vmax);
    return scvx::check_launch("collision_check_kernel");
}

namespace {
int collision_rows_launch(int K, int pos_dim, int n_x, int N_total, const double* X_all, int i0, const int32_t* idx,
                          int N_local, double R, double cull_radius, int j_max, double* rows, int32_t* count,
                          void* stream) {
    if (N_local == 0) return SCVX_OK;
    const dim3 grid((unsigned)((N_local + 63) / 64), (unsigned)K);
    hipStream_t st = (hipStream_t)stream;
    if (j_max <= 8)
        hipLaunchKernelGGL(scvx::collision_rows_kernel<8>, grid, dim3(64), 0, st, K, pos_dim, n_x, N_total, N_local,
                           X_all, i0, idx, R, cull_radius, j_max, rows, count);
    else if (j_max <= 16)
        hipLaunchKernelGGL(scvx::collision_rows_kernel<16>, grid, dim3(64), 0, st, K, pos_dim, n_x, N_total, N_local,
                           X_all, i0, idx, R, cull_radius, j_max, rows, count);
    else
        hipLaunchKernelGGL(scvx::collision_rows_kernel<32>, grid, dim3(64), 0, st, K, pos_dim, n_x, N_total, N_local,
                           X_all, i0, idx, R, cull_radius, j_max, rows, count);
    return scvx::check_launch("collision_rows_kernel");
}
}  // namespace

extern "C" int scvx_collision_rows_batched(int K, int pos_dim, int n_x, int N_total, const double* X_all, int i0,
                                           int N_local, double R, double cull_radius, int j_max, double* rows,
                                           int32_t* count, void* stream) {
    if (K < 2 || K > 64 || pos_dim < 1 || pos_dim > 3 || pos_dim > n_x || N_total < 0 || N_local < 0 || i0 < 0 ||
        i0 + N_local > N_total || j_max < 1 || j_max > 32 || !X_all || !rows || !count)
        return scvx::set_error(SCVX_EINVAL, "collision: bad args");
    return collision_rows_launch(K, pos_dim, n_x, N_total, X_all, i0, nullptr, N_local, R, cull_radius, j_max, rows,
                                 count, stream);
}

extern "C" int scvx_collision_rows_indexed(int K, int pos_dim, int n_x, int N_total, const double* X_all,
                                           const int32_t* idx, int N_sel, double R, double cull_radius, int j_max,
                                           double* rows, int32_t* count, void* stream) {
    if (K < 2 || K > 64 || pos_dim < 1 || pos_dim > 3 || pos_dim > n_x || N_total < 0 || N_sel < 0 || j_max < 1 ||
        j_max > 32 || !X_all || !rows || !count || (N_sel > 0 && !idx))
        return scvx::set_error(SCVX_EINVAL, "collision: bad args");
    return collision_rows_launch(K, pos_dim, n_x, N_total, X_all, 0, idx, N_sel, R, cull_radius, j_max, rows, count,
                                 stream);
}
