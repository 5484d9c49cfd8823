// ORACLE / TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline leg, kind "port"; tests).
//
// Plain-C++ float64 CPU restatement of the batched trust-region subproblem declared in
// include/scvx_hip.h (scvx_qp_solve_batched): the per-agent convex solve of
// Distributed_opt/dist_scvx_3d.py:51-111, which the reference hands to CVXPY+Clarabel.
// Same problem, same algorithm family as the HIP kernel (primal-dual Mehrotra IPM, NT scaling for
// the SOC, Riccati factorisation of the node-banded KKT system) but written independently in
// scalar dense form: every node keeps a dense constraint matrix over (x, u, aux) and the
// auxiliary slacks are eliminated by a generic dense Schur complement.  Agents are solved one
// after another (or OpenMP-parallel over agents when nthreads > 1).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/scvx_hip.h"

namespace {

using Vec = std::vector<double>;

struct Mat {
    int r = 0, c = 0;
    Vec a;
    Mat() {}
    Mat(int r_, int c_) : r(r_), c(c_), a((size_t)r_ * c_, 0.0) {}
    double& operator()(int i, int j) { return a[(size_t)i * c + j]; }
    double operator()(int i, int j) const { return a[(size_t)i * c + j]; }
};

static Mat mul(const Mat& A, const Mat& B) {
    Mat C(A.r, B.c);
    for (int i = 0; i < A.r; ++i)
        for (int k = 0; k < A.c; ++k) {
            double v = A(i, k);
            if (v == 0.0) continue;
            for (int j = 0; j < B.c; ++j) C(i, j) += v * B(k, j);
        }
    return C;
}
static Mat tr(const Mat& A) {
    Mat T(A.c, A.r);
    for (int i = 0; i < A.r; ++i)
        for (int j = 0; j < A.c; ++j) T(j, i) = A(i, j);
    return T;
}
static Mat add(const Mat& A, const Mat& B) {
    Mat C = A;
    for (size_t i = 0; i < C.a.size(); ++i) C.a[i] += B.a[i];
    return C;
}
static Vec matvec(const Mat& A, const Vec& x) {
    Vec y(A.r, 0.0);
    for (int i = 0; i < A.r; ++i)
        for (int j = 0; j < A.c; ++j) y[i] += A(i, j) * x[j];
    return y;
}
static Vec matTvec(const Mat& A, const Vec& x) {
    Vec y(A.c, 0.0);
    for (int i = 0; i < A.r; ++i)
        for (int j = 0; j < A.c; ++j) y[j] += A(i, j) * x[i];
    return y;
}
// Cholesky in place (lower), returns false if not PD
static bool chol(Mat& L) {
    int n = L.r;
    for (int j = 0; j < n; ++j) {
        double d = L(j, j);
        for (int k = 0; k < j; ++k) d -= L(j, k) * L(j, k);
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        L(j, j) = d;
        for (int i = j + 1; i < n; ++i) {
            double v = L(i, j);
            for (int k = 0; k < j; ++k) v -= L(i, k) * L(j, k);
            L(i, j) = v / d;
        }
        for (int i = 0; i < j; ++i) L(i, j) = 0.0;
    }
    return true;
}
static void chol_solve(const Mat& L, double* b) {
    int n = L.r;
    for (int i = 0; i < n; ++i) {
        double v = b[i];
        for (int k = 0; k < i; ++k) v -= L(i, k) * b[k];
        b[i] = v / L(i, i);
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int k = i + 1; k < n; ++k) v -= L(k, i) * b[k];
        b[i] = v / L(i, i);
    }
}
static Mat chol_solve_mat(const Mat& L, const Mat& B) {
    Mat X = B;
    Vec col(B.r);
    for (int j = 0; j < B.c; ++j) {
        for (int i = 0; i < B.r; ++i) col[i] = X(i, j);
        chol_solve(L, col.data());
        for (int i = 0; i < B.r; ++i) X(i, j) = col[i];
    }
    return X;
}
// LU with partial pivoting solve (small dense)
static bool lu_solve(Mat A, Vec& b) {
    int n = A.r;
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(A(i, k)) > std::fabs(A(p, k))) p = i;
        if (A(p, k) == 0.0) return false;
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(A(k, j), A(p, j));
            std::swap(b[k], b[p]);
        }
        for (int i = k + 1; i < n; ++i) {
            double f = A(i, k) / A(k, k);
            for (int j = k; j < n; ++j) A(i, j) -= f * A(k, j);
            b[i] -= f * b[k];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int j = i + 1; j < n; ++j) v -= A(i, j) * b[j];
        b[i] = v / A(i, i);
    }
    return true;
}

// ------------------------------- second-order cone helpers -----------------------------------
struct Soc {
    int k = 0;
    Mat W, Wi, Wi2;
};
static double socJ(const double* x, int k) {
    double v = x[0] * x[0];
    for (int i = 1; i < k; ++i) v -= x[i] * x[i];
    return v;
}
static void soc_nt(const double* s, const double* z, int k, Soc& S) {
    S.k = k;
    double Js = socJ(s, k), Jz = socJ(z, k);
    double ns = std::sqrt(Js), nz = std::sqrt(Jz);
    Vec sb(k), zb(k), w(k);
    double dot = 0.0;
    for (int i = 0; i < k; ++i) { sb[i] = s[i] / ns; zb[i] = z[i] / nz; dot += sb[i] * zb[i]; }
    double gam = std::sqrt((1.0 + dot) / 2.0);
    for (int i = 0; i < k; ++i) w[i] = (sb[i] + (i == 0 ? zb[i] : -zb[i])) / (2.0 * gam);
    // hyperbolic-rotation form of the NT scaling (W z = W^-1 s), eta = (J(s)/J(z))^(1/4)
    double eta = std::pow(Js / Jz, 0.25);
    S.W = Mat(k, k);
    S.Wi = Mat(k, k);
    S.W(0, 0) = eta * w[0];
    S.Wi(0, 0) = w[0] / eta;
    for (int i = 1; i < k; ++i) {
        S.W(0, i) = S.W(i, 0) = eta * w[i];
        S.Wi(0, i) = S.Wi(i, 0) = -w[i] / eta;
        for (int j = 1; j < k; ++j) {
            double v = (i == j ? 1.0 : 0.0) + w[i] * w[j] / (1.0 + w[0]);
            S.W(i, j) = eta * v;
            S.Wi(i, j) = v / eta;
        }
    }
    S.Wi2 = mul(S.Wi, S.Wi);
}
static void jprod(const double* a, const double* b, int k, double* o) {
    double d = 0.0;
    for (int i = 0; i < k; ++i) d += a[i] * b[i];
    Vec t(k);
    t[0] = d;
    for (int i = 1; i < k; ++i) t[i] = a[0] * b[i] + b[0] * a[i];
    for (int i = 0; i < k; ++i) o[i] = t[i];
}
static void jdiv(const double* x, const double* r, int k, double* o) {
    double d = socJ(x, k);
    double r0 = x[0] * r[0];
    for (int i = 1; i < k; ++i) r0 -= x[i] * r[i];
    r0 /= d;
    Vec t(k);
    t[0] = r0;
    for (int i = 1; i < k; ++i) t[i] = (r[i] - r0 * x[i]) / x[0];
    for (int i = 0; i < k; ++i) o[i] = t[i];
}
static double soc_step(const double* x, const double* dx, int k) {
    double a = socJ(dx, k);
    double b = x[0] * dx[0];
    for (int i = 1; i < k; ++i) b -= x[i] * dx[i];
    b *= 2.0;
    double c = socJ(x, k);
    double best = 1e300;
    if (std::fabs(a) < 1e-300) {
        if (b < 0) best = std::min(best, -c / b);
    } else {
        double disc = b * b - 4 * a * c;
        if (disc >= 0) {
            double sq = std::sqrt(disc);
            double r1 = (-b - sq) / (2 * a), r2 = (-b + sq) / (2 * a);
            if (r1 > 0) best = std::min(best, r1);
            if (r2 > 0) best = std::min(best, r2);
        }
    }
    if (dx[0] < 0) best = std::min(best, -x[0] / dx[0]);
    return best;
}

// ------------------------------------ per-agent solver --------------------------------------
struct Node {
    int nv = 0, na = 0;   // node vars = n + m + nnu + na: x, u, virtual control nu (t < K-1 when w_nu > 0), aux
    int nnu = 0;
    Mat G;                // orthant rows (nr x nv)
    Vec h;
    int nr = 0;
    bool soc = false;
    Vec q;                // linear cost on node vars
    Vec pdiag;            // quadratic cost diag on node vars
    Vec z, s, lam, ssoc, lsoc;
    bool fixed_u = false;
};

struct Agent {
    const scvx_qp_template* T;
    int n, m, K, pd;
    std::vector<Node> nd;
    std::vector<Mat> A, B, C;   // C[t] couples u_{t+1}
    std::vector<Vec> c;
    Vec x_init, x_final;
    Vec xref;                    // Xbar (K*n): the proximal term's centre
    Vec y;                       // dynamics multipliers (K-1)*n
    Vec y_init, y_fin;
    double trv = 0.0;            // trust radius of this solve
};

static void setup_agent(Agent& ag, const scvx_qp_template* T, const double* disc, double sigma, const double* Xr,
                        const double* Ur, const double* x_init, const double* x_final, double trv,
                        const double* crow, const int32_t* ccount) {
    ag.T = T;
    ag.trv = trv;
    int n = T->n_x, m = T->n_u, K = T->K, pd = T->pos_dim;
    ag.n = n; ag.m = m; ag.K = K; ag.pd = pd;
    int stride = n * (n + 2 * m + 2);
    ag.A.assign(K - 1, Mat(n, n));
    ag.B.assign(K - 1, Mat(n, m));
    ag.C.assign(K - 1, Mat(n, m));
    ag.c.assign(K - 1, Vec(n, 0.0));
    for (int t = 0; t < K - 1; ++t) {
        const double* d = disc + (size_t)t * stride;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) ag.A[t](i, j) = d[j * n + i];
        for (int j = 0; j < m; ++j)
            for (int i = 0; i < n; ++i) {
                ag.B[t](i, j) = d[n * n + j * n + i];
                ag.C[t](i, j) = d[n * n + n * m + j * n + i];
            }
        for (int i = 0; i < n; ++i) ag.c[t][i] = d[n * n + 2 * n * m + i] * sigma + d[n * n + 2 * n * m + n + i];
    }
    ag.x_init.assign(x_init, x_init + n);
    ag.xref.assign(Xr, Xr + (size_t)K * n);
    ag.x_final.assign(n, 0.0);
    if (T->has_final || T->w_final > 0.0) ag.x_final.assign(x_final, x_final + n);
    ag.nd.assign(K, Node());
    const bool coll = T->j_max > 0;
    for (int t = 0; t < K; ++t) {
        Node& N = ag.nd[t];
        bool ineq = (t < K - 1) || T->ineq_last;
        // virtual control nu_t in the dynamics of interval t (SCvx form, sc_problem.py:60-68) with
        // the penalty w_nu ||nu_t||_1 through its epigraph -e <= nu <= e (e: aux, eliminated per node)
        N.nnu = (T->w_nu > 0.0 && t < K - 1) ? n : 0;
        N.na = (ineq ? (T->n_obs + (coll ? 1 : 0)) : 0) + N.nnu;
        N.nv = n + m + N.nnu + N.na;
        const int ab = n + m + N.nnu;   // first aux variable
        N.q.assign(N.nv, 0.0);
        N.pdiag.assign(N.nv, 0.0);
        double wu = (t < K - 1) ? 1.0 : T->w_last;
        for (int j = 0; j < m; ++j) N.pdiag[n + j] = 2.0 * wu;
        if (t == K - 1 && !T->has_final && T->w_final > 0.0) {  // soft terminal (kernel: tsoft)
            for (int i = 0; i < n; ++i) { N.pdiag[i] = 2.0 * T->w_final; N.q[i] = -2.0 * T->w_final * ag.x_final[i]; }
        }
        if (T->w_prox > 0.0)   // proximal term w_prox ||x_t - xbar_t||^2 (its constant is added to obj below)
            for (int i = 0; i < n; ++i) {
                N.pdiag[i] += 2.0 * T->w_prox;
                N.q[i] -= 2.0 * T->w_prox * Xr[(size_t)t * n + i];
            }
        N.fixed_u = (t == K - 1) && T->fix_last_input;
        std::vector<Vec> rows;
        Vec hs;
        auto newrow = [&]() { rows.emplace_back(N.nv, 0.0); return (int)rows.size() - 1; };
        if (ineq) {
            const double* pb = Xr + (size_t)t * n;
            const double* ub = Ur + (size_t)t * m;
            for (int f = 0; f < (1 << m); ++f) {  // L1 ball facets
                int r = newrow();
                double hh = trv;
                for (int j = 0; j < m; ++j) {
                    double sg = ((f >> j) & 1) ? -1.0 : 1.0;
                    rows[r][n + j] = sg;
                    hh += sg * ub[j];
                }
                hs.push_back(hh);
            }
            for (int b = 0; b < T->n_box; ++b) {
                int r = newrow(); rows[r][T->box_idx[b]] = 1.0; hs.push_back(T->box_hi[b]);
                r = newrow(); rows[r][T->box_idx[b]] = -1.0; hs.push_back(-T->box_lo[b]);
            }
            for (int o = 0; o < T->n_obs; ++o) {
                int ai = ab + o;
                double diff[3], nr = 0.0;
                for (int i = 0; i < pd; ++i) { diff[i] = pb[i] - T->obs_center[o][i]; nr += diff[i] * diff[i]; }
                nr = std::sqrt(nr) + 1e-6;
                double bo = T->obs_radius[o];
                int r = newrow();
                for (int i = 0; i < pd; ++i) {
                    double a = diff[i] / nr;
                    rows[r][i] = -a;
                    bo += a * T->obs_center[o][i];
                }
                rows[r][ai] = -1.0;
                hs.push_back(-bo);
                r = newrow(); rows[r][ai] = -1.0; hs.push_back(0.0);
                N.q[ai] = T->w_obs;
            }
            if (coll) {
                int ai = ab + T->n_obs;
                int cnt = ccount[t];
                for (int j = 0; j < cnt; ++j) {
                    const double* rw = crow + ((size_t)t * T->j_max + j) * (pd + 1);
                    int r = newrow();
                    for (int i = 0; i < pd; ++i) rows[r][i] = -rw[i];
                    rows[r][ai] = -1.0;
                    hs.push_back(-rw[pd]);
                }
                int r = newrow(); rows[r][ai] = -1.0; hs.push_back(0.0);
                N.q[ai] = T->w_coll;
            }
            N.soc = T->has_soc != 0;
        }
        for (int i = 0; i < N.nnu; ++i) {   // nu_i - e_i <= 0, -nu_i - e_i <= 0
            const int ei = ab + N.na - N.nnu + i;
            int r = newrow(); rows[r][n + m + i] = 1.0; rows[r][ei] = -1.0; hs.push_back(0.0);
            r = newrow(); rows[r][n + m + i] = -1.0; rows[r][ei] = -1.0; hs.push_back(0.0);
            N.q[ei] = T->w_nu;
        }
        N.nr = (int)rows.size();
        N.G = Mat(N.nr, N.nv);
        for (int r = 0; r < N.nr; ++r)
            for (int j = 0; j < N.nv; ++j) N.G(r, j) = rows[r][j];
        N.h = hs;
        N.z.assign(N.nv, 0.0);
        for (int i = 0; i < n; ++i) N.z[i] = Xr[(size_t)t * n + i];
        for (int j = 0; j < m; ++j) N.z[n + j] = Ur[(size_t)t * m + j];
        N.s.assign(N.nr, 1.0);
        N.lam.assign(N.nr, 1.0);
        if (N.soc) { N.ssoc.assign(m + 1, 0.0); N.lsoc.assign(m + 1, 0.0); }
    }
    ag.y.assign((size_t)(K - 1) * n, 0.0);
    ag.y_init.assign(n, 0.0);
    ag.y_fin.assign(n, 0.0);
}

struct NodeLin {   // per-node quantities of one IPM iteration
    Vec D;          // lam/s
    Soc soc;
    Vec lt;         // scaled point (orthant sqrt(s lam); SOC W lam)
    Mat Hxu;        // reduced (n+m)x(n+m) Hessian after aux elimination
    Mat Haa_L;      // chol of aux block
    Mat Hza;        // (n+m) x na coupling
    Vec rc, rcs;    // ineq residuals
    Vec rd;         // dual residual over node vars
};

struct Riccati {
    std::vector<Mat> P, Kg, L, Pi, kap, Bt;
    std::vector<Vec> k0, p0;
    // virtual control: G_t = H_nunu + P_{t+1} (Cholesky), YP = G^-1 P_{t+1}, YPi = G^-1 Pi_{t+1}, d_t
    std::vector<Mat> LG, YP, YPi;
    std::vector<Vec> dnu;
    std::vector<Mat> Pe, Pie;   // effective next-stage P~, Pi~ of stage t (= P_{t+1}, Pi_{t+1} without nu)
    // trust-region facets (the 2^m rows g_f'u <= h_f of ||u - ubar||_1 <= tr at nodes t < K-1), kept out of the
    // node Hessians: Df[t] their barrier weights lambda/s (empty: the stage has none).  Stage t folds D g g' of
    // every facet into its input block Rh EXCEPT the stiff ones (D_f > STIFF_RATIO max diag of the rest, when
    // 1 <= #stiff <= m-1), which stay explicit stage unknowns of the quasi-definite system
    //   [R0 G; G' -D^-1] [u; nu] = [-y; rho]
    // solved by the Woodbury identity Rh^-1 = R0^-1 - W C^-1 W', W = R0^-1 G, C = D^-1 + G'W (nu = the facets'
    // multiplier step).  The folded sum R0 + D g g' with D ~ 1e12 next to an O(1e-4) curvature cannot be
    // represented in float64 (the C4 late-step optimal_inaccurate); R0, W and C can.
    std::vector<Vec> Df;
    std::vector<std::vector<int>> stiff;
    std::vector<Mat> W, LC, Sh, rhsk;
    std::vector<Vec> rh;
    Mat M;
    bool ok = true;
};

// trust-region facet f's coefficient on input j (setup_agent's sign pattern)
static inline double facet_g(int f, int j) { return ((f >> j) & 1) ? -1.0 : 1.0; }
constexpr double STIFF_RATIO = 1e6;
static bool stiff_enabled() {
    static int e = -1;
    if (e < 0) { const char* v = std::getenv("SCVX_TWIN_STIFF"); e = v ? std::atoi(v) : 1; }
    return e != 0;
}
// Rh^-1 Y for a stage with stiff facets (Woodbury), or L^-T L^-1 Y
static Mat stage_solve(const Riccati& R, int t, const Mat& Y) {
    Mat X = chol_solve_mat(R.L[t], Y);
    if (R.stiff[t].empty()) return X;
    const Mat& W = R.W[t];
    const int p = (int)R.stiff[t].size(), m = W.r;
    Mat GX(p, X.c);   // G' X0
    for (int a = 0; a < p; ++a)
        for (int c = 0; c < X.c; ++c) {
            double v = 0.0;
            for (int j = 0; j < m; ++j) v += facet_g(R.stiff[t][a], j) * X(j, c);
            GX(a, c) = v;
        }
    Mat Z = chol_solve_mat(R.LC[t], GX);
    Mat WZ = mul(W, Z);
    for (size_t e = 0; e < X.a.size(); ++e) X.a[e] -= WZ.a[e];
    return X;
}

// factor the Riccati recursion for node Hessians H_t ((n+m+nnu) square, in (x,u,nu) coordinates)
//
// Virtual control nu_t (interval t, Hessian block H_nunu, no cross terms with x, u) is eliminated
// inside stage t: with the next stage's value 1/2 xi'P xi + xi'(p + Pi mu),
//   nu = -G^-1 (P y + p + Pi mu + d),  G = H_nunu + P,  y = A xi + Bt v + e,
// and the stage sees the effective next-stage data  P~ = P - P G^-1 P = H_nunu G^-1 P,
// Pi~ = H_nunu G^-1 Pi, p~ = p - P G^-1 (p + d), plus the terminal terms M -= Pi' G^-1 Pi and
// xacc -= Pi' G^-1 (p + d).
static void riccati_factor(const Agent& ag, const std::vector<Mat>& H, Riccati& R) {
    int n = ag.n, m = ag.m, K = ag.K;
    const bool fin = ag.T->has_final;
    R.P.assign(K, Mat(n, n));
    R.Kg.assign(K, Mat(m, n));
    R.L.assign(K, Mat(m, m));
    R.Pi.assign(K, Mat(n, n));
    R.kap.assign(K, Mat(m, n));
    R.Bt.assign(K, Mat(n, m));
    R.k0.assign(K, Vec(m));
    R.p0.assign(K, Vec(n));
    R.LG.assign(K, Mat());
    R.YP.assign(K, Mat());
    R.YPi.assign(K, Mat());
    R.dnu.assign(K, Vec());
    R.Pe.assign(K, Mat());
    R.Pie.assign(K, Mat());
    R.Df.resize(K);
    R.stiff.assign(K, std::vector<int>());
    R.W.assign(K, Mat());
    R.LC.assign(K, Mat());
    R.Sh.assign(K, Mat());
    R.rhsk.assign(K, Mat());
    R.rh.assign(K, Vec());
    R.M = Mat(n, n);
    R.ok = true;
    for (int t = 0; t < K - 1; ++t) {
        R.Bt[t] = ag.B[t];
        if (t > 0) R.Bt[t] = add(ag.B[t], mul(ag.A[t], ag.C[t - 1]));
    }
    for (int t = K - 1; t >= 0; --t) {
        // node Hessian in (xi, v) coordinates: x = xi + C_{t-1} v
        Mat Hxx(n, n), Hxu(n, m), Huu(m, m);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) Hxx(i, j) = H[t](i, j);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < m; ++j) Hxu(i, j) = H[t](i, n + j);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j) Huu(i, j) = H[t](n + i, n + j);
        Mat Q = Hxx, S = Hxu, Rm = Huu;
        if (t > 0) {
            const Mat& Cp = ag.C[t - 1];
            S = add(mul(Hxx, Cp), Hxu);
            Rm = add(add(mul(tr(Cp), mul(Hxx, Cp)), mul(tr(Cp), Hxu)), add(mul(tr(Hxu), Cp), Huu));
        }
        Mat Qh = Q, Sh = tr(S), Rh = Rm;
        if (t < K - 1) {
            Mat Pn = R.P[t + 1], Pin = R.Pi[t + 1];
            const int nnu = ag.nd[t].nnu;
            if (nnu) {
                Mat Hn(n, n), G = R.P[t + 1];
                for (int i = 0; i < n; ++i)
                    for (int j = 0; j < n; ++j) { Hn(i, j) = H[t](n + m + i, n + m + j); G(i, j) += Hn(i, j); }
                if (!chol(G)) { R.ok = false; return; }
                R.LG[t] = G;
                R.YP[t] = chol_solve_mat(G, R.P[t + 1]);
                Pn = mul(Hn, R.YP[t]);
                for (int i = 0; i < n; ++i)
                    for (int j = 0; j < i; ++j) { double v = 0.5 * (Pn(i, j) + Pn(j, i)); Pn(i, j) = Pn(j, i) = v; }
                if (fin) {
                    R.YPi[t] = chol_solve_mat(G, R.Pi[t + 1]);
                    Pin = mul(Hn, R.YPi[t]);
                    Mat c = mul(tr(R.Pi[t + 1]), R.YPi[t]);
                    for (size_t e = 0; e < R.M.a.size(); ++e) R.M.a[e] -= c.a[e];
                }
            }
            R.Pe[t] = Pn;
            R.Pie[t] = Pin;
            Mat PA = mul(Pn, ag.A[t]), PB = mul(Pn, R.Bt[t]);
            Qh = add(Q, mul(tr(ag.A[t]), PA));
            Sh = add(tr(S), mul(tr(R.Bt[t]), PA));
            Rh = add(Rm, mul(tr(R.Bt[t]), PB));
        }
        if (ag.nd[t].fixed_u) {
            for (int i = 0; i < m; ++i) {
                for (int j = 0; j < m; ++j) Rh(i, j) = (i == j) ? 1.0 : 0.0;
                for (int j = 0; j < n; ++j) Sh(i, j) = 0.0;
            }
        } else if (!R.Df[t].empty()) {   // trust-region facets: fold all but the stiff ones
            const Vec& Df = R.Df[t];
            const int nf = (int)Df.size();
            double dmax = 0.0;   // the stage's Rhat without the facets
            for (int j = 0; j < m; ++j) dmax = std::max(dmax, std::fabs(Rh(j, j)));
            // stiff set (the kernel's rule, qp_ipm.hpp factor phase 3): the facets with D above STIFF_RATIO x the
            // largest diagonal of the stage's Rhat without them, kept explicit when there are at most m-1 of them and no two are
            // opposite (a face or an edge of the L1 ball: they leave a complement whose small curvature the fold
            // would lose).  m or more (a vertex) make every direction of u stiff: the folded sum loses nothing
            // there, while the Woodbury form would cancel (measured on the C4 dumps: 407 -> 85 optimal of 444).
            std::vector<int> st;
            // candidate nodes only (the kernel's assemble): some D_f above STIFF_RATIO x the largest diagonal of the
            // node's own R (Rhat = R + Bt'P Bt >= R, so no other node can have a stiff facet); the kernel folds the
            // other nodes' facets into R before phase 2, the twin here -- the same sum in another rounding order
            double rdm = 0.0, dfm = 0.0;
            for (int j = 0; j < m; ++j) rdm = std::max(rdm, std::fabs(Rm(j, j)));
            for (int f = 0; f < nf; ++f) dfm = std::max(dfm, Df[f]);
            if (stiff_enabled() && ag.T->j_max > 0 && n <= 8 && m >= 2 && m <= 4 && dfm > STIFF_RATIO * rdm) {
                for (int f = 0; f < nf; ++f)
                    if (Df[f] > STIFF_RATIO * dmax) st.push_back(f);
                bool opp = false;
                for (size_t a = 0; a < st.size(); ++a)
                    for (size_t b = a + 1; b < st.size(); ++b) opp = opp || ((st[a] ^ st[b]) == nf - 1);
                if ((int)st.size() > m - 1 || opp) st.clear();
            }
            if (!st.empty() && std::getenv("SCVX_DEBUG_STIFF")) {
                std::fprintf(stderr, "   stiff t %d dmax %.3e:", t, dmax);
                for (int f : st) std::fprintf(stderr, " f%d D %.3e", f, Df[f]);
                std::fprintf(stderr, "\n");
            }
            for (int f = 0; f < nf; ++f) {
                if (std::find(st.begin(), st.end(), f) != st.end()) continue;
                for (int i = 0; i < m; ++i)
                    for (int j = 0; j < m; ++j) Rh(i, j) += Df[f] * facet_g(f, i) * facet_g(f, j);
            }
            R.stiff[t] = st;
        }
        Mat L = Rh;
        // LDL' of Rh with the kernel's rule (phase 3): pivots that rounding pushed below 1e-13 max|diag| are
        // clamped there (Rh is a Schur complement that loses definiteness at extreme barrier scalings: an active
        // trust-region facet adds D g g' with D ~ 1e12, whose sum with the O(1e-4) objective curvature cannot be
        // represented); NaN is fatal
        bool chol_ok;
        {
            double dmax = 0.0;
            for (int j = 0; j < m; ++j) dmax = std::max(dmax, std::fabs(L(j, j)));
            const double dmin = 1e-13 * dmax + 1e-300;
            chol_ok = dmax == dmax;
            for (int j = 0; j < m; ++j) {
                double d = L(j, j);
                for (int k = 0; k < j; ++k) d -= L(j, k) * L(j, k);
                chol_ok = chol_ok && d == d;
                if (!(d > dmin)) d = dmin;
                d = std::sqrt(d);
                L(j, j) = d;
                for (int i = j + 1; i < m; ++i) {
                    double v = L(i, j);
                    for (int k = 0; k < j; ++k) v -= L(i, k) * L(j, k);
                    L(i, j) = v / d;
                }
                for (int i = 0; i < j; ++i) L(i, j) = 0.0;
            }
        }
        if (!chol_ok) {
            if (std::getenv("SCVX_DEBUG")) {
                std::fprintf(stderr, "   chol(Rh) failed at stage %d:", t);
                for (int i = 0; i < m; ++i) std::fprintf(stderr, " %.3e", Rh(i, i));
                std::fprintf(stderr, " | Rm diag");
                for (int i = 0; i < m; ++i) std::fprintf(stderr, " %.3e", Rm(i, i));
                std::fprintf(stderr, "\n");
            }
            R.ok = false;
            return;
        }
        R.L[t] = L;
        R.Sh[t] = Sh;
        if (!R.stiff[t].empty()) {   // Woodbury pieces: W = R0^-1 G, C = D^-1 + G'W (Cholesky)
            const int p = (int)R.stiff[t].size();
            Mat G(m, p);
            for (int a = 0; a < p; ++a)
                for (int j = 0; j < m; ++j) G(j, a) = facet_g(R.stiff[t][a], j);
            R.W[t] = chol_solve_mat(L, G);
            Mat C = mul(tr(G), R.W[t]);
            for (int a = 0; a < p; ++a) C(a, a) += 1.0 / R.Df[t][R.stiff[t][a]];
            if (std::getenv("SCVX_TWIN_GJCHECK")) {   // experiment: the kernel's Gauss-Jordan pivots of C
                Mat Cg = C;
                for (int k = 0; k < p; ++k) {
                    const double pv = Cg(k, k);
                    if (!(pv > 0.0)) {
                        std::fprintf(stderr, "GJ pivot %d of C at stage %d: %.3e (C diag %.3e %.3e off %.3e, D %.3e)\n", k, t, pv,
                                     C(0, 0), p > 1 ? C(1, 1) : 0.0, p > 1 ? C(1, 0) : 0.0, R.Df[t][R.stiff[t][0]]);
                        R.ok = false; return;
                    }
                    for (int j = 0; j < p; ++j) Cg(k, j) /= pv;
                    for (int i = 0; i < p; ++i) if (i != k) { const double f = Cg(i, k); for (int j = 0; j < p; ++j) Cg(i, j) -= f * Cg(k, j); }
                }
            }
            if (!chol(C)) { R.ok = false; return; }
            R.LC[t] = C;
        }
        Mat Kg = stage_solve(R, t, Sh);
        for (double& v : Kg.a) v = -v;
        R.Kg[t] = Kg;
        Mat P = add(Qh, mul(tr(Sh), Kg));
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < i; ++j) { double v = 0.5 * (P(i, j) + P(j, i)); P(i, j) = P(j, i) = v; }
        R.P[t] = P;
        if (fin) {
            if (t == K - 1) {
                Mat rhs(m, n);  // C_{K-2}^T
                if (K >= 2)
                    for (int i = 0; i < m; ++i)
                        for (int j = 0; j < n; ++j) rhs(i, j) = ag.C[K - 2](j, i);
                if (ag.nd[t].fixed_u) rhs = Mat(m, n);
                R.rhsk[t] = rhs;
                Mat kap = stage_solve(R, t, rhs);
                for (double& v : kap.a) v = -v;
                R.kap[t] = kap;
                Mat I(n, n);
                for (int i = 0; i < n; ++i) I(i, i) = 1.0;
                R.Pi[t] = add(I, mul(tr(Sh), kap));
                R.M = (K >= 2) ? mul(ag.C[K - 2], kap) : Mat(n, n);
            } else {
                const Mat& Pin = R.Pie[t];
                Mat rhs = mul(tr(R.Bt[t]), Pin);
                if (ag.nd[t].fixed_u) rhs = Mat(m, n);
                R.rhsk[t] = rhs;
                Mat kap = stage_solve(R, t, rhs);
                for (double& v : kap.a) v = -v;
                R.kap[t] = kap;
                R.Pi[t] = add(mul(tr(ag.A[t]), Pin), mul(tr(Sh), kap));
                R.M = add(R.M, mul(tr(Pin), mul(R.Bt[t], kap)));
            }
        }
    }
}

// Solve  min 1/2 dz'H dz - r1'dz  s.t. A dz = r2  ; returns dz (per node n+m+nnu), dy (K-1)*n, dyi, dyf
// Facets kept out of r1 (stages with R.Df[t] set): ftr[t][f] = their folded rhs term (rco + lam rc)/s, frho[t][f] =
// -(rco/lam + rc); fnu[t][f] returns the stiff facets' multiplier steps.
static bool riccati_solve(const Agent& ag, const std::vector<Mat>& H, Riccati& R, const std::vector<Vec>& r1,
                          const Vec& xi0, const std::vector<Vec>& e, const Vec& r2fin, std::vector<Vec>& dz,
                          Vec& dy, Vec& dyi, Vec& dyf, const std::vector<Vec>* ftr = nullptr,
                          const std::vector<Vec>* frho = nullptr, std::vector<Vec>* fnu = nullptr) {
    (void)H;
    int n = ag.n, m = ag.m, K = ag.K;
    const bool fin = ag.T->has_final;
    Vec xacc(n, 0.0);
    for (int t = K - 1; t >= 0; --t) {
        const int nnu = ag.nd[t].nnu;
        Vec q(n), r(m);
        for (int i = 0; i < n; ++i) q[i] = -r1[t][i];
        for (int j = 0; j < m; ++j) r[j] = -r1[t][n + j];
        if (t > 0) {
            Vec ct = matTvec(ag.C[t - 1], q);
            for (int j = 0; j < m; ++j) r[j] += ct[j];
        }
        Vec qh = q, rh = r, pw;   // pw = p_{t+1} + d_t (virtual control)
        if (t < K - 1) {
            Vec pn = R.p0[t + 1];
            if (nnu) {
                R.dnu[t].assign(n, 0.0);
                pw = pn;
                for (int i = 0; i < n; ++i) { R.dnu[t][i] = -r1[t][n + m + i]; pw[i] += R.dnu[t][i]; }
                Vec c = matTvec(R.YP[t], pw);   // (G^-1 P)' (p + d) = P G^-1 (p + d)
                for (int i = 0; i < n; ++i) pn[i] -= c[i];
            }
            Vec h = matvec(R.Pe[t], e[t]);
            for (int i = 0; i < n; ++i) h[i] += pn[i];
            Vec a = matTvec(ag.A[t], h), b = matTvec(R.Bt[t], h);
            for (int i = 0; i < n; ++i) qh[i] += a[i];
            for (int j = 0; j < m; ++j) rh[j] += b[j];
        }
        if (ag.nd[t].fixed_u)
            for (int j = 0; j < m; ++j) rh[j] = 0.0;
        const std::vector<int>& st = R.stiff[t];
        if (ftr && !R.Df[t].empty() && !ag.nd[t].fixed_u)
            for (int f = 0; f < (int)R.Df[t].size(); ++f)
                if (std::find(st.begin(), st.end(), f) == st.end())
                    for (int j = 0; j < m; ++j) rh[j] += facet_g(f, j) * (*ftr)[t][f];
        R.rh[t] = rh;
        Mat rhm(m, 1);
        for (int j = 0; j < m; ++j) rhm(j, 0) = rh[j];
        Mat km = stage_solve(R, t, rhm);
        Vec k(m);
        for (int j = 0; j < m; ++j) k[j] = -km(j, 0);
        Vec wc;   // W C^-1 rho
        if (!st.empty()) {
            Vec z((int)st.size());
            for (size_t a = 0; a < st.size(); ++a) z[a] = (*frho)[t][st[a]];
            chol_solve(R.LC[t], z.data());
            wc = matvec(R.W[t], z);
            for (int j = 0; j < m; ++j) k[j] += wc[j];
        }
        R.k0[t] = k;
        Vec p = qh, kt = matTvec(R.Kg[t], rh);
        for (int i = 0; i < n; ++i) p[i] += kt[i];
        if (!st.empty()) {
            Vec c = matTvec(R.Sh[t], wc);
            for (int i = 0; i < n; ++i) p[i] += c[i];
        }
        R.p0[t] = p;
        if (fin) {
            if (t == K - 1) {
                xacc = (K >= 2) ? matvec(ag.C[K - 2], k) : Vec(n, 0.0);
            } else {
                Vec bk = matvec(R.Bt[t], k);
                for (int i = 0; i < n; ++i) bk[i] += e[t][i];
                Vec g = matTvec(R.Pie[t], bk);
                for (int i = 0; i < n; ++i) xacc[i] += g[i];
                if (nnu) {
                    Vec c = matTvec(R.YPi[t], pw);   // Pi' G^-1 (p + d)
                    for (int i = 0; i < n; ++i) xacc[i] -= c[i];
                }
            }
        }
    }
    Vec mu(n, 0.0);
    if (fin) {
        Vec g = matTvec(R.Pi[0], xi0);
        for (int i = 0; i < n; ++i) mu[i] = r2fin[i] - (xacc[i] + g[i]);
        if (!lu_solve(R.M, mu)) return false;
    }
    Vec xi = xi0;
    dz.assign(K, Vec());
    dy.assign((size_t)(K - 1) * n, 0.0);
    auto pfull = [&](int t) {
        Vec p = R.p0[t];
        if (fin) {
            Vec g = matvec(R.Pi[t], mu);
            for (int i = 0; i < n; ++i) p[i] += g[i];
        }
        return p;
    };
    {
        Vec p = pfull(0), Px = matvec(R.P[0], xi0);
        dyi.assign(n, 0.0);
        for (int i = 0; i < n; ++i) dyi[i] = -(Px[i] + p[i]);
    }
    for (int t = 0; t < K; ++t) {
        const int nnu = ag.nd[t].nnu;
        dz[t].assign(n + m + nnu, 0.0);
        Vec v = matvec(R.Kg[t], xi);
        for (int j = 0; j < m; ++j) v[j] += R.k0[t][j];
        if (fin) {
            Vec g = matvec(R.kap[t], mu);
            for (int j = 0; j < m; ++j) v[j] += g[j];
        }
        Vec x = xi;
        if (t > 0) {
            Vec cv = matvec(ag.C[t - 1], v);
            for (int i = 0; i < n; ++i) x[i] += cv[i];
        }
        for (int i = 0; i < n; ++i) dz[t][i] = x[i];
        for (int j = 0; j < m; ++j) dz[t][n + j] = v[j];
        if (fnu && !R.stiff[t].empty()) {   // nu = C^-1 (G'x0 - rho), x0 = -R0^-1 (rh + Sh xi + rhsk mu)
            const std::vector<int>& st = R.stiff[t];
            Vec y = R.rh[t], sx = matvec(R.Sh[t], xi);
            for (int j = 0; j < m; ++j) y[j] += sx[j];
            if (fin) {
                Vec g = matvec(R.rhsk[t], mu);
                for (int j = 0; j < m; ++j) y[j] += g[j];
            }
            chol_solve(R.L[t], y.data());
            Vec z(st.size());
            for (size_t a = 0; a < st.size(); ++a) {
                double gx = 0.0;
                for (int j = 0; j < m; ++j) gx -= facet_g(st[a], j) * y[j];
                z[a] = gx - (*frho)[t][st[a]];
            }
            chol_solve(R.LC[t], z.data());
            (*fnu)[t].assign(R.Df[t].size(), 0.0);
            for (size_t a = 0; a < st.size(); ++a) (*fnu)[t][st[a]] = z[a];
        }
        if (t < K - 1) {
            Vec a = matvec(ag.A[t], xi), b = matvec(R.Bt[t], v);
            Vec xn(n);
            for (int i = 0; i < n; ++i) xn[i] = a[i] + b[i] + e[t][i];
            Vec p = pfull(t + 1);
            if (nnu) {   // nu = -G^-1 (P y + p + Pi mu + d)
                Vec w = matvec(R.P[t + 1], xn);
                for (int i = 0; i < n; ++i) w[i] += p[i] + R.dnu[t][i];
                chol_solve(R.LG[t], w.data());
                for (int i = 0; i < n; ++i) { dz[t][n + m + i] = -w[i]; xn[i] -= w[i]; }
            }
            Vec Px = matvec(R.P[t + 1], xn);
            for (int i = 0; i < n; ++i) dy[(size_t)t * n + i] = -(Px[i] + p[i]);
            xi = xn;
        }
    }
    dyf = mu;
    return true;
}

// The (x, u, nu) block of a node's Hessian with its aux variables eliminated:
//   diag(pdiag) + sum_{rows r without aux} D_r g_r g_r' + sum_aux sum_{r in R_a} D_r (g_r - m_a)(g_r - m_a)',
// m_a = sum_{R_a} D_r g_r / sum_{R_a} D_r, with g_r the row's (x, u, nu) part (every row of aux a has coefficient
// -1 on it).  This is the Schur complement H_zz - H_za H_aa^-1 H_az written as a weighted covariance: a sum of
// PSD terms, where the direct difference cancels catastrophically once one row's barrier weight dominates
// (an active obstacle row next to its inactive slack-sign row: D1 D2 / (D1 + D2) computed as D1 - D1^2/(D1 + D2)
// turned negative and broke the Riccati factorisation on 6 of the 1024 C3 agents).  The kernel does the same.
static Mat node_zz(const Node& N, const Vec& D, int nz) {
    Mat H(nz, nz);
    for (int j = 0; j < nz; ++j) H(j, j) = N.pdiag[j];
    std::vector<int> aux(N.nr, -1);
    for (int r = 0; r < N.nr; ++r)
        for (int a = 0; a < N.na; ++a)
            if (N.G(r, nz + a) != 0.0) aux[r] = a;
    for (int r = 0; r < N.nr; ++r) {
        if (aux[r] >= 0) continue;
        for (int i = 0; i < nz; ++i) {
            const double gi = N.G(r, i);
            if (gi == 0.0) continue;
            for (int j = 0; j < nz; ++j) H(i, j) += D[r] * gi * N.G(r, j);
        }
    }
    for (int a = 0; a < N.na; ++a) {
        double dsum = 0.0;
        Vec mean(nz, 0.0);
        for (int r = 0; r < N.nr; ++r)
            if (aux[r] == a) {
                dsum += D[r];
                for (int i = 0; i < nz; ++i) mean[i] += D[r] * N.G(r, i);
            }
        if (!(dsum > 0.0)) continue;
        for (int i = 0; i < nz; ++i) mean[i] /= dsum;
        for (int r = 0; r < N.nr; ++r)
            if (aux[r] == a)
                for (int i = 0; i < nz; ++i) {
                    const double ci = N.G(r, i) - mean[i];
                    if (ci == 0.0) continue;
                    for (int j = 0; j < nz; ++j) H(i, j) += D[r] * ci * (N.G(r, j) - mean[j]);
                }
    }
    return H;
}

// CVXOPT-style starting point: from the reference trajectory z_ref (aux = 0) take the minimiser of
//   1/2 z'Pz + q'z + 1/2 ||Gz - h||^2   s.t.  Az = b
// (one Riccati solve with unit scaling), then s = h - Gz, lam = Gz - h, each shifted into the
// cone interior by a common multiple of the identity (oracle/qp_dense.py solve_conic_qp does the same).
static bool init_point(Agent& ag) {
    const scvx_qp_template* T = ag.T;
    int n = ag.n, m = ag.m, K = ag.K;
    std::vector<Mat> H(K), Hza(K), HaaL(K);
    std::vector<Vec> r1(K), r1a(K);
    for (int t = 0; t < K; ++t) {
        Node& N = ag.nd[t];
        Mat Hf(N.nv, N.nv);
        for (int j = 0; j < N.nv; ++j) Hf(j, j) = N.pdiag[j];
        for (int r = 0; r < N.nr; ++r)
            for (int i = 0; i < N.nv; ++i)
                for (int j = 0; j < N.nv; ++j) Hf(i, j) += N.G(r, i) * N.G(r, j);
        Vec rf(N.nv);
        for (int j = 0; j < N.nv; ++j) rf[j] = -(N.pdiag[j] * N.z[j] + N.q[j]);
        for (int r = 0; r < N.nr; ++r) {
            double v = -N.h[r];
            for (int j = 0; j < N.nv; ++j) v += N.G(r, j) * N.z[j];
            for (int j = 0; j < N.nv; ++j) rf[j] -= N.G(r, j) * v;
        }
        if (N.soc)
            for (int j = 0; j < m; ++j) { Hf(n + j, n + j) += 1.0; rf[n + j] -= N.z[n + j]; }
        if (N.fixed_u)
            for (int j = 0; j < m; ++j) rf[n + j] = 0.0;
        int nz = n + m + N.nnu, na = N.na;
        H[t] = node_zz(N, Vec(N.nr, 1.0), nz);
        if (N.soc)
            for (int j = 0; j < m; ++j) H[t](n + j, n + j) += 1.0;
        r1[t].assign(rf.begin(), rf.begin() + nz);
        if (na > 0) {
            Mat Haa(na, na);
            Hza[t] = Mat(nz, na);
            for (int i = 0; i < na; ++i)
                for (int j = 0; j < na; ++j) Haa(i, j) = Hf(nz + i, nz + j);
            for (int i = 0; i < nz; ++i)
                for (int j = 0; j < na; ++j) Hza[t](i, j) = Hf(i, nz + j);
            HaaL[t] = Haa;
            if (!chol(HaaL[t])) return false;
            r1a[t].assign(rf.begin() + nz, rf.end());
            Vec ra = r1a[t];
            chol_solve(HaaL[t], ra.data());
            Vec c = matvec(Hza[t], ra);
            for (int i = 0; i < nz; ++i) r1[t][i] -= c[i];
        }
    }
    Riccati R;
    riccati_factor(ag, H, R);
    if (!R.ok) return false;
    Vec xi0(n), r2f(n, 0.0);
    for (int i = 0; i < n; ++i) xi0[i] = ag.x_init[i] - ag.nd[0].z[i];
    if (T->has_final)
        for (int i = 0; i < n; ++i) r2f[i] = ag.x_final[i] - ag.nd[K - 1].z[i];
    std::vector<Vec> e(K - 1, Vec(n));
    for (int t = 0; t < K - 1; ++t) {
        const Vec& z0 = ag.nd[t].z;
        const Vec& z1 = ag.nd[t + 1].z;
        for (int i = 0; i < n; ++i) {
            double v = z1[i] - ag.c[t][i];
            for (int k = 0; k < n; ++k) v -= ag.A[t](i, k) * z0[k];
            for (int j = 0; j < m; ++j) v -= ag.B[t](i, j) * z0[n + j] + ag.C[t](i, j) * z1[n + j];
            if (ag.nd[t].nnu) v -= z0[n + m + i];
            e[t][i] = -v;
        }
    }
    std::vector<Vec> dz;
    Vec dy, dyi, dyf;
    if (!riccati_solve(ag, H, R, r1, xi0, e, r2f, dz, dy, dyi, dyf)) return false;
    double smin = 1e300, lmin = 1e300;
    for (int t = 0; t < K; ++t) {
        Node& N = ag.nd[t];
        int nz = n + m + N.nnu;
        for (int i = 0; i < nz; ++i) N.z[i] += dz[t][i];
        if (N.na > 0) {
            Vec ra = r1a[t];
            Vec c = matTvec(Hza[t], dz[t]);
            for (int a = 0; a < N.na; ++a) ra[a] -= c[a];
            chol_solve(HaaL[t], ra.data());
            for (int a = 0; a < N.na; ++a) N.z[nz + a] += ra[a];
        }
        for (int r = 0; r < N.nr; ++r) {
            double v = N.h[r];
            for (int j = 0; j < N.nv; ++j) v -= N.G(r, j) * N.z[j];
            N.s[r] = v;
            N.lam[r] = -v;
            smin = std::min(smin, v);
            lmin = std::min(lmin, -v);
        }
        if (N.soc) {
            N.ssoc[0] = T->u_max;
            N.lsoc[0] = -T->u_max;
            double nu = 0.0;
            for (int j = 0; j < m; ++j) { N.ssoc[1 + j] = N.z[n + j]; N.lsoc[1 + j] = -N.z[n + j]; nu += N.z[n + j] * N.z[n + j]; }
            smin = std::min(smin, T->u_max - std::sqrt(nu));
            lmin = std::min(lmin, -T->u_max - std::sqrt(nu));
        }
    }
    double sh_s = std::max(0.0, 1.0 - smin), sh_l = std::max(0.0, 1.0 - lmin);
    for (int t = 0; t < K; ++t) {
        Node& N = ag.nd[t];
        for (int r = 0; r < N.nr; ++r) { N.s[r] += sh_s; N.lam[r] += sh_l; }
        if (N.soc) { N.ssoc[0] += sh_s; N.lsoc[0] += sh_l; }
    }
    return true;
}

// ------------------------------------------------------------------ warm start (kernel: `warm`)
// A solve can start from the primal-dual point a previous solve of the same agent ended at (the Jacobi
// SCvx loop: the next subproblem is this one re-linearised at its own solution).  z, the equality
// multipliers y and the inequality duals are kept; the slacks are recomputed from the NEW rows at z; every
// slack and dual is floored at QP_WARM_ETA inside its cone (scaled units).  Measured on the C3 loop: 12.3 ->
// 5.1 IPM iterations on average, the same optima to the stopping tolerance.
// Per-agent state: per node z (nv) | lambda (nr) | lsoc (m+1), padded to a fixed stride, then y ((K-1) n),
// y_init (n), y_fin (n).
constexpr double QP_WARM_ETA = 1e-3;
// a row's dual floor: min(QP_WARM_ETA, QP_WARM_KAPPA / s) (round 6; kernel csrc/qp_ipm.hpp, the same constants)
constexpr double QP_WARM_KAPPA = 1e-5;
static int warm_node_stride(const scvx_qp_template* T) {
    const int n = T->n_x, m = T->n_u, nnu = T->w_nu > 0.0 ? n : 0;
    const int aux = T->n_obs + (T->j_max > 0 ? 1 : 0) + nnu;
    const int rows = (1 << m) + 2 * T->n_box + 2 * T->n_obs + (T->j_max > 0 ? T->j_max + 1 : 0) + 2 * nnu;
    return n + m + nnu + aux + rows + (m + 1);
}
static long long warm_doubles(const scvx_qp_template* T) {
    return (long long)T->K * warm_node_stride(T) + (long long)(T->K + 1) * T->n_x;
}
static void warm_save(const Agent& ag, double* w) {
    const int st = warm_node_stride(ag.T), n = ag.n, K = ag.K;
    for (int t = 0; t < K; ++t) {
        const Node& N = ag.nd[t];
        double* o = w + (size_t)t * st;
        for (int j = 0; j < N.nv; ++j) o[j] = N.z[j];
        for (int r = 0; r < N.nr; ++r) o[N.nv + r] = N.lam[r];
        if (N.soc)
            for (int j = 0; j <= ag.m; ++j) o[N.nv + N.nr + j] = N.lsoc[j];
    }
    double* o = w + (size_t)K * st;
    for (size_t i = 0; i < ag.y.size(); ++i) o[i] = ag.y[i];
    for (int i = 0; i < n; ++i) { o[(K - 1) * n + i] = ag.y_init[i]; o[K * n + i] = ag.y_fin[i]; }
}
// start from a previous solve's primal-dual point: z, y, lambda kept, slacks recomputed from the new rows
// at z, then every slack / dual (and the SOC pair) floored at eta inside its cone
static void warm_point(Agent& ag, const double* w, double eta) {
    const scvx_qp_template* T = ag.T;
    const int st = warm_node_stride(T), n = ag.n, m = ag.m, K = ag.K;
    // experiment knobs (diagnostics): floors of the trust-region facets' slack / dual relative to the radius
    const char* ek = std::getenv("SCVX_WARM_TRK");
    const char* el = std::getenv("SCVX_WARM_TRL");
    const double ks = ek ? std::atof(ek) : 0.0, kl = el ? std::atof(el) : 0.0;
    // a row's dual floor is min(eta, QP_WARM_KAPPA / s) at its floored slack s (kernel: the same rule): a row with a
    // large slack keeps a small dual.  SCVX_WARM_KAPPA: experiment knob (0: the round-5 floor eta for every dual)
    // The floor applies to the classes without the stiff-facet stage system (kernel: !(C::STF && has_coll)): on the
    // C4 loop (coupled double integrators) it lengthened the tail (max 32-41 -> 46-60 IPM iterations per step) and
    // ended three warm solves status 2 (profiles/round6_r6c_*), while the C3 (uncoupled) and C5 (quadrotor) loops gain.
    const char* ekap = std::getenv("SCVX_WARM_KAPPA");
    const bool stf = T->j_max > 0 && n <= 8 && m >= 2 && m <= 4;
    const double kap = stf ? 0.0 : (ekap ? std::atof(ekap) : QP_WARM_KAPPA);
    for (int t = 0; t < K; ++t) {
        Node& N = ag.nd[t];
        const double* o = w + (size_t)t * st;
        for (int j = 0; j < N.nv; ++j) N.z[j] = o[j];
        for (int r = 0; r < N.nr; ++r) {
            double v = N.h[r];
            for (int j = 0; j < N.nv; ++j) v -= N.G(r, j) * N.z[j];
            const bool trf = r < (1 << m) && t < K - 1;
            N.s[r] = std::max(v, (trf && ks > 0) ? std::min(eta, ks * ag.trv) : eta);
            double lf = (trf && kl > 0) ? std::min(eta, kl * ag.trv) : eta;
            if (kap > 0) lf = std::min(lf, kap / N.s[r]);
            N.lam[r] = std::max(o[N.nv + r], lf);
        }
        if (N.soc) {
            N.ssoc[0] = T->u_max;
            double nu = 0.0;
            for (int j = 0; j < m; ++j) { N.ssoc[1 + j] = N.z[n + j]; nu += N.z[n + j] * N.z[n + j]; }
            N.ssoc[0] = std::max(N.ssoc[0], std::sqrt(nu) + eta);
            double nl = 0.0;
            for (int j = 0; j <= m; ++j) N.lsoc[j] = o[N.nv + N.nr + j];
            for (int j = 1; j <= m; ++j) nl += N.lsoc[j] * N.lsoc[j];
            N.lsoc[0] = std::max(N.lsoc[0], std::sqrt(nl) + eta);
        }
    }
    const double* o = w + (size_t)K * st;
    for (size_t i = 0; i < ag.y.size(); ++i) ag.y[i] = o[i];
    for (int i = 0; i < n; ++i) { ag.y_init[i] = o[(K - 1) * n + i]; ag.y_fin[i] = o[K * n + i]; }
}

static int solve_agent(Agent& ag, int& iters_out, double& obj_out, const double* win = nullptr, double* wout = nullptr) {
    const scvx_qp_template* T = ag.T;
    int n = ag.n, m = ag.m, K = ag.K;
    int deg = 0;
    for (int t = 0; t < K; ++t) deg += ag.nd[t].nr + (ag.nd[t].soc ? 1 : 0);
    std::vector<NodeLin> L(K);
    std::vector<Mat> H(K);
    Riccati R;
    int status = SCVX_STATUS_MAX_ITER;
    int it = 0, n_skip = 0;
    const double tol = T->tol > 0 ? T->tol : 1e-9;
    // objective scaling (kernel: osc): solve with the objective divided by max(1, ||q||_inf); the gap test
    // and the reported objective are in the caller's units
    double osc = 1.0;
    for (int t = 0; t < K; ++t)
        for (double v : ag.nd[t].q) osc = std::max(osc, std::fabs(v));
    if (const char* e = std::getenv("SCVX_OSC")) osc = std::atof(e);   // diagnostics: force the objective scale
    for (int t = 0; t < K; ++t) {
        for (double& v : ag.nd[t].q) v /= osc;
        for (double& v : ag.nd[t].pdiag) v /= osc;
    }
    double cprox = 0.0;   // w_prox sum ||xbar||^2 (caller's units)
    if (T->w_prox > 0.0)
        for (double v : ag.xref) cprox += T->w_prox * v * v;
    if (win) {
        static const double eta_w = std::getenv("SCVX_WARM_ETA") ? std::atof(std::getenv("SCVX_WARM_ETA")) : QP_WARM_ETA;   // experiment knob
        warm_point(ag, win, eta_w);
    } else if (!init_point(ag)) {
        iters_out = 0; obj_out = 0.0; return SCVX_STATUS_NUMERICAL;
    }
    double dres_best = 1e300, pres_best = 1e300;
    for (it = 0;; ++it) {  // the residuals are evaluated once more after the last step (kernel: cap check)
        // ---- residuals
        // Clarabel's normalisation (kernel: pnorm / dnorm): primal max(1, ||b|| + ||x|| + ||s||),
        // dual max(1, ||q|| + ||x|| + ||z||), inf-norms over every constant / variable / multiplier
        double pres = 0.0, dres = 0.0, gap = 0.0, nb = 0.0, nxv = 0.0, nsl = 0.0, nzd = 0.0, nq = 0.0;
        for (int i = 0; i < n; ++i) {
            nb = std::max({nb, std::fabs(ag.x_init[i]), T->has_final ? std::fabs(ag.x_final[i]) : 0.0});
            nzd = std::max({nzd, std::fabs(ag.y_init[i]), T->has_final ? std::fabs(ag.y_fin[i]) : 0.0});
        }
        for (double v : ag.y) nzd = std::max(nzd, std::fabs(v));
        for (int t = 0; t < K - 1; ++t)
            for (int i = 0; i < n; ++i) nb = std::max(nb, std::fabs(ag.c[t][i]));
        for (int t = 0; t < K; ++t)
            for (int j = 0; j < ag.nd[t].nv; ++j) nxv = std::max(nxv, std::fabs(ag.nd[t].z[j]));
        std::vector<Vec> rp(K - 1, Vec(n));
        Vec rpi(n), rpf(n, 0.0);
        for (int i = 0; i < n; ++i) rpi[i] = ag.nd[0].z[i] - ag.x_init[i];
        if (T->has_final)
            for (int i = 0; i < n; ++i) rpf[i] = ag.nd[K - 1].z[i] - ag.x_final[i];
        for (int t = 0; t < K - 1; ++t) {
            const Vec& z0 = ag.nd[t].z;
            const Vec& z1 = ag.nd[t + 1].z;
            for (int i = 0; i < n; ++i) {
                double v = z1[i] - ag.c[t][i];
                for (int k = 0; k < n; ++k) v -= ag.A[t](i, k) * z0[k];
                for (int j = 0; j < m; ++j) v -= ag.B[t](i, j) * z0[n + j] + ag.C[t](i, j) * z1[n + j];
                if (ag.nd[t].nnu) v -= z0[n + m + i];
                rp[t][i] = v;
                pres = std::max(pres, std::fabs(v));
            }
        }
        for (int i = 0; i < n; ++i) pres = std::max({pres, std::fabs(rpi[i]), std::fabs(rpf[i])});
        for (int t = 0; t < K; ++t) {
            Node& N = ag.nd[t];
            NodeLin& l = L[t];
            l.rc.assign(N.nr, 0.0);
            for (int r = 0; r < N.nr; ++r) {
                double v = N.s[r] - N.h[r];
                for (int j = 0; j < N.nv; ++j) v += N.G(r, j) * N.z[j];
                l.rc[r] = v;
                pres = std::max(pres, std::fabs(v));
                nb = std::max(nb, std::fabs(N.h[r]));
                nsl = std::max(nsl, N.s[r]);
                nzd = std::max(nzd, N.lam[r]);
                gap += N.s[r] * N.lam[r];
            }
            if (N.soc) {
                l.rcs.assign(m + 1, 0.0);
                l.rcs[0] = N.ssoc[0] - T->u_max;
                for (int j = 0; j < m; ++j) l.rcs[1 + j] = N.ssoc[1 + j] - N.z[n + j];
                for (int j = 0; j <= m; ++j) {
                    pres = std::max(pres, std::fabs(l.rcs[j]));
                    gap += N.ssoc[j] * N.lsoc[j];
                    nsl = std::max(nsl, std::fabs(N.ssoc[j]));
                    nzd = std::max(nzd, std::fabs(N.lsoc[j]));
                }
                nb = std::max(nb, T->u_max);
            }
            l.rd.assign(N.nv, 0.0);
            for (int j = 0; j < N.nv; ++j) { l.rd[j] = N.pdiag[j] * N.z[j] + N.q[j]; nq = std::max(nq, std::fabs(N.q[j])); }
            for (int r = 0; r < N.nr; ++r)
                for (int j = 0; j < N.nv; ++j) l.rd[j] += N.G(r, j) * N.lam[r];
            if (N.soc)
                for (int j = 0; j < m; ++j) l.rd[n + j] -= N.lsoc[1 + j];
            // A^T y
            if (t == 0)
                for (int i = 0; i < n; ++i) l.rd[i] += ag.y_init[i];
            if (t == K - 1 && T->has_final)
                for (int i = 0; i < n; ++i) l.rd[i] += ag.y_fin[i];
            if (t >= 1) {
                const double* yp = &ag.y[(size_t)(t - 1) * n];
                for (int i = 0; i < n; ++i) l.rd[i] += yp[i];
                for (int j = 0; j < m; ++j)
                    for (int i = 0; i < n; ++i) l.rd[n + j] -= ag.C[t - 1](i, j) * yp[i];
            }
            if (t < K - 1) {
                const double* yt = &ag.y[(size_t)t * n];
                for (int k = 0; k < n; ++k)
                    for (int i = 0; i < n; ++i) l.rd[k] -= ag.A[t](i, k) * yt[i];
                for (int j = 0; j < m; ++j)
                    for (int i = 0; i < n; ++i) l.rd[n + j] -= ag.B[t](i, j) * yt[i];
                for (int i = 0; i < N.nnu; ++i) l.rd[n + m + i] -= yt[i];
            }
            if (N.fixed_u)
                for (int j = 0; j < m; ++j) l.rd[n + j] = 0.0;
            for (int j = 0; j < N.nv; ++j) dres = std::max(dres, std::fabs(l.rd[j]));
        }
        double mu = gap / std::max(deg, 1);
        double pobj = 0.0;
        for (int t = 0; t < K; ++t)
            for (int j = 0; j < ag.nd[t].nv; ++j) {
                double zj = ag.nd[t].z[j];
                pobj += 0.5 * ag.nd[t].pdiag[j] * zj * zj + ag.nd[t].q[j] * zj;
            }
        pobj += cprox / osc;   // the proximal term's constant: the gap test is relative to the true objective
        if (std::getenv("SCVX_DEBUG")) std::fprintf(stderr, "it %d pres %.3e dres %.3e mu %.3e pobj %.6e\n", it, pres, dres, mu, pobj);
        if (const char* dn = std::getenv("SCVX_DEBUG_NODE")) {   // diagnostics: one node's iterate and rows
            const int t = std::atoi(dn);
            const Node& N = ag.nd[t];
            std::fprintf(stderr, "   node %d z:", t);
            for (int j = 0; j < N.nv; ++j) std::fprintf(stderr, " %.4e", N.z[j]);
            std::fprintf(stderr, "\n");
            for (int r = 0; r < N.nr; ++r) std::fprintf(stderr, "     r %d s %.3e lam %.3e\n", r, N.s[r], N.lam[r]);
        }
        if (!std::isfinite(pres + dres + mu)) { status = SCVX_STATUS_NUMERICAL; break; }
        const double pnorm = std::max(1.0, nb + nxv + nsl), dnorm = std::max(1.0 / osc, nq + nxv / osc + nzd);  // caller's units / osc
        if (pres <= tol * pnorm && dres <= tol * dnorm && gap * osc <= tol * std::max(1.0, std::fabs(pobj * osc))) {
            status = SCVX_STATUS_OPTIMAL;
            break;
        }
        // reduced tolerances (kernel: `near`): a breakdown below ends with MAX_ITER ("inaccurate")
        const bool near = pres <= 1e-4 * pnorm && dres <= 1e-4 * dnorm && gap * osc <= 5e-5 * std::max(1.0, std::fabs(pobj * osc));
        const int fail_status = near ? SCVX_STATUS_MAX_ITER : SCVX_STATUS_NUMERICAL;
        if (it >= T->max_iter) { status = fail_status; break; }
        // insufficient progress (kernel: fail code 7)
        if (near && (dres > std::max(100.0 * dres_best, tol * dnorm) || pres > std::max(100.0 * pres_best, tol * pnorm))) {
            status = SCVX_STATUS_MAX_ITER;
            break;
        }
        dres_best = std::min(dres_best, dres);
        pres_best = std::min(pres_best, pres);
        // ---- scaling and node Hessians (aux eliminated)
        for (int t = 0; t < K; ++t) {
            Node& N = ag.nd[t];
            NodeLin& l = L[t];
            l.D.assign(N.nr, 0.0);
            l.lt.assign(N.nr + (N.soc ? m + 1 : 0), 0.0);
            for (int r = 0; r < N.nr; ++r) { l.D[r] = N.lam[r] / N.s[r]; l.lt[r] = std::sqrt(N.s[r] * N.lam[r]); }
            Mat Hf(N.nv, N.nv);
            for (int j = 0; j < N.nv; ++j) Hf(j, j) = N.pdiag[j];
            for (int r = 0; r < N.nr; ++r)
                for (int i = 0; i < N.nv; ++i) {
                    double gi = N.G(r, i);
                    if (gi == 0.0) continue;
                    for (int j = 0; j < N.nv; ++j) Hf(i, j) += l.D[r] * gi * N.G(r, j);
                }
            if (N.soc) {
                soc_nt(N.ssoc.data(), N.lsoc.data(), m + 1, l.soc);
                Vec wl = matvec(l.soc.W, N.lsoc);
                for (int j = 0; j <= m; ++j) l.lt[N.nr + j] = wl[j];
                for (int i = 0; i < m; ++i)
                    for (int j = 0; j < m; ++j) Hf(n + i, n + j) += l.soc.Wi2(1 + i, 1 + j);
            }
            int nz = n + m + N.nnu, na = N.na;
            R.Df.resize(K);
            R.Df[t].clear();
            if (t < K - 1 && !N.fixed_u && N.nr >= (1 << m) && T->j_max > 0 && n <= 8 && m >= 2 && m <= 4) {   // STF: facets folded per stage
                Vec D0 = l.D;
                R.Df[t].assign(l.D.begin(), l.D.begin() + (1 << m));
                for (int f = 0; f < (1 << m); ++f) D0[f] = 0.0;
                l.Hxu = node_zz(N, D0, nz);
            } else {
                l.Hxu = node_zz(N, l.D, nz);
            }
            if (N.soc)
                for (int i = 0; i < m; ++i)
                    for (int j = 0; j < m; ++j) l.Hxu(n + i, n + j) += l.soc.Wi2(1 + i, 1 + j);
            if (na > 0) {
                Mat Haa(na, na);
                l.Hza = Mat(nz, na);
                for (int i = 0; i < na; ++i)
                    for (int j = 0; j < na; ++j) Haa(i, j) = Hf(nz + i, nz + j);
                for (int i = 0; i < nz; ++i)
                    for (int j = 0; j < na; ++j) l.Hza(i, j) = Hf(i, nz + j);
                l.Haa_L = Haa;
                if (!chol(l.Haa_L)) { status = fail_status; goto done; }
            }
            H[t] = l.Hxu;
        }
        riccati_factor(ag, H, R);
        if (!R.ok) { status = fail_status; break; }
        {
            // ---- one Newton solve for a given complementarity rhs (orthant rco, SOC rcs2)
            auto newton = [&](const std::vector<Vec>& rco, const std::vector<Vec>& rcq, std::vector<Vec>& dz,
                              std::vector<Vec>& ds, std::vector<Vec>& dl, std::vector<Vec>& dsq,
                              std::vector<Vec>& dlq, Vec& dy, Vec& dyi, Vec& dyf) -> bool {
                std::vector<Vec> r1(K), r1a(K), tq(K), ftr(K), frho(K), fnu(K);
                for (int t = 0; t < K; ++t) {
                    Node& N = ag.nd[t];
                    NodeLin& l = L[t];
                    Vec rf(N.nv);
                    for (int j = 0; j < N.nv; ++j) rf[j] = -l.rd[j];
                    const int nf = (int)R.Df[t].size();   // facets handled per stage (riccati_solve)
                    ftr[t].assign(nf, 0.0);
                    frho[t].assign(nf, 0.0);
                    for (int r = 0; r < N.nr; ++r) {
                        double tr_ = (rco[t][r] + N.lam[r] * l.rc[r]) / N.s[r];
                        if (r < nf) {
                            ftr[t][r] = tr_;
                            frho[t][r] = -(rco[t][r] / N.lam[r] + l.rc[r]);
                            continue;
                        }
                        for (int j = 0; j < N.nv; ++j) rf[j] -= N.G(r, j) * tr_;
                    }
                    if (N.soc) {
                        Vec rho(m + 1);
                        jdiv(&l.lt[N.nr], rcq[t].data(), m + 1, rho.data());
                        Vec t1 = matvec(l.soc.Wi, rho), t2 = matvec(l.soc.Wi2, l.rcs);
                        tq[t].assign(m + 1, 0.0);
                        for (int j = 0; j <= m; ++j) tq[t][j] = t1[j] + t2[j];
                        for (int j = 0; j < m; ++j) rf[n + j] += tq[t][1 + j];  // G^T t, G = [0; -I]
                    }
                    if (N.fixed_u)
                        for (int j = 0; j < m; ++j) rf[n + j] = 0.0;
                    int nz = n + m + N.nnu;
                    r1[t].assign(rf.begin(), rf.begin() + nz);
                    if (N.na > 0) {
                        Vec ra(rf.begin() + nz, rf.end());
                        chol_solve(l.Haa_L, ra.data());
                        Vec c = matvec(l.Hza, ra);
                        for (int i = 0; i < nz; ++i) r1[t][i] -= c[i];
                        r1a[t].assign(rf.begin() + nz, rf.end());
                    }
                }
                Vec xi0(n);
                for (int i = 0; i < n; ++i) xi0[i] = -rpi[i];
                std::vector<Vec> e(K - 1, Vec(n));
                for (int t = 0; t < K - 1; ++t)
                    for (int i = 0; i < n; ++i) e[t][i] = -rp[t][i];
                Vec r2f(n);
                for (int i = 0; i < n; ++i) r2f[i] = -rpf[i];
                std::vector<Vec> dzx;
                if (!riccati_solve(ag, H, R, r1, xi0, e, r2f, dzx, dy, dyi, dyf, &ftr, &frho, &fnu)) return false;
                if (std::getenv("SCVX_DEBUG")) {
                    double e1 = 0.0, e2 = 0.0;
                    for (int t = 0; t < K; ++t) {
                        Vec st = matvec(H[t], dzx[t]);
                        for (int i = 0; i < n + m; ++i) st[i] -= r1[t][i];
                        if (t == 0) for (int i = 0; i < n; ++i) st[i] += dyi[i];
                        if (t == K - 1 && ag.T->has_final) for (int i = 0; i < n; ++i) st[i] += dyf[i];
                        if (t >= 1) {
                            const double* yp = &dy[(size_t)(t - 1) * n];
                            for (int i = 0; i < n; ++i) st[i] += yp[i];
                            for (int j = 0; j < m; ++j) for (int i = 0; i < n; ++i) st[n + j] -= ag.C[t - 1](i, j) * yp[i];
                        }
                        if (t < K - 1) {
                            const double* yt = &dy[(size_t)t * n];
                            for (int k = 0; k < n; ++k) for (int i = 0; i < n; ++i) st[k] -= ag.A[t](i, k) * yt[i];
                            for (int j = 0; j < m; ++j) for (int i = 0; i < n; ++i) st[n + j] -= ag.B[t](i, j) * yt[i];
                            for (int i = 0; i < n; ++i) {
                                double v = dzx[t + 1][i] - e[t][i];
                                for (int k = 0; k < n; ++k) v -= ag.A[t](i, k) * dzx[t][k];
                                for (int j = 0; j < m; ++j) v -= ag.B[t](i, j) * dzx[t][n + j] + ag.C[t](i, j) * dzx[t + 1][n + j];
                                if (ag.nd[t].nnu) v -= dzx[t][n + m + i];
                                e2 = std::max(e2, std::fabs(v));
                            }
                        }
                        int lim = ag.nd[t].fixed_u ? n : n + m;
                        for (int i = 0; i < lim; ++i) e1 = std::max(e1, std::fabs(st[i]));
                    }
                    for (int i = 0; i < n; ++i) e2 = std::max(e2, std::fabs(dzx[0][i] - xi0[i]));
                    if (ag.T->has_final) for (int i = 0; i < n; ++i) e2 = std::max(e2, std::fabs(dzx[K - 1][i] - r2f[i]));
                    std::fprintf(stderr, "   kkt check: stationarity %.3e equality %.3e\n", e1, e2);
                }
                dz.assign(K, Vec());
                ds.assign(K, Vec());
                dl.assign(K, Vec());
                dsq.assign(K, Vec());
                dlq.assign(K, Vec());
                for (int t = 0; t < K; ++t) {
                    Node& N = ag.nd[t];
                    NodeLin& l = L[t];
                    int nz = n + m + N.nnu;
                    dz[t].assign(N.nv, 0.0);
                    for (int i = 0; i < nz; ++i) dz[t][i] = dzx[t][i];
                    if (N.na > 0) {
                        Vec ra = r1a[t];
                        Vec c = matTvec(l.Hza, dzx[t]);
                        for (int a = 0; a < N.na; ++a) ra[a] -= c[a];
                        chol_solve(l.Haa_L, ra.data());
                        for (int a = 0; a < N.na; ++a) dz[t][nz + a] = ra[a];
                    }
                    ds[t].assign(N.nr, 0.0);
                    dl[t].assign(N.nr, 0.0);
                    for (int r = 0; r < N.nr; ++r) {
                        double g = 0.0;
                        for (int j = 0; j < N.nv; ++j) g += N.G(r, j) * dz[t][j];
                        ds[t][r] = -l.rc[r] - g;
                        dl[t][r] = (rco[t][r] + N.lam[r] * (l.rc[r] + g)) / N.s[r];
                        if (!fnu[t].empty() && r < (int)fnu[t].size() &&
                            std::find(R.stiff[t].begin(), R.stiff[t].end(), r) != R.stiff[t].end())
                            dl[t][r] = fnu[t][r];   // stiff facet: its multiplier step from the stage system
                    }
                    if (N.soc) {
                        Vec gq(m + 1, 0.0);
                        for (int j = 0; j < m; ++j) gq[1 + j] = -dz[t][n + j];
                        dsq[t].assign(m + 1, 0.0);
                        for (int j = 0; j <= m; ++j) dsq[t][j] = -l.rcs[j] - gq[j];
                        Vec rho(m + 1), v(m + 1);
                        jdiv(&l.lt[N.nr], rcq[t].data(), m + 1, rho.data());
                        for (int j = 0; j <= m; ++j) v[j] = l.rcs[j] + gq[j];
                        Vec a = matvec(l.soc.Wi, rho), b = matvec(l.soc.Wi2, v);
                        dlq[t].assign(m + 1, 0.0);
                        for (int j = 0; j <= m; ++j) dlq[t][j] = a[j] + b[j];
                    }
                }
                return true;
            };
            auto max_step = [&](const std::vector<Vec>& ds, const std::vector<Vec>& dl, const std::vector<Vec>& dsq,
                                const std::vector<Vec>& dlq) {
                double a = 1e300;
                for (int t = 0; t < K; ++t) {
                    Node& N = ag.nd[t];
                    for (int r = 0; r < N.nr; ++r) {
                        if (ds[t][r] < 0) a = std::min(a, -N.s[r] / ds[t][r]);
                        if (dl[t][r] < 0) a = std::min(a, -N.lam[r] / dl[t][r]);
                    }
                    if (N.soc) {
                        a = std::min(a, soc_step(N.ssoc.data(), dsq[t].data(), m + 1));
                        a = std::min(a, soc_step(N.lsoc.data(), dlq[t].data(), m + 1));
                    }
                }
                return a;
            };
            // predictor
            std::vector<Vec> rco(K), rcq(K);
            for (int t = 0; t < K; ++t) {
                Node& N = ag.nd[t];
                rco[t].assign(N.nr, 0.0);
                for (int r = 0; r < N.nr; ++r) rco[t][r] = -N.s[r] * N.lam[r];
                if (N.soc) {
                    rcq[t].assign(m + 1, 0.0);
                    jprod(&L[t].lt[N.nr], &L[t].lt[N.nr], m + 1, rcq[t].data());
                    for (double& v : rcq[t]) v = -v;
                }
            }
            std::vector<Vec> dz, ds, dl, dsq, dlq;
            Vec dy, dyi, dyf;
            if (!newton(rco, rcq, dz, ds, dl, dsq, dlq, dy, dyi, dyf)) { status = fail_status; break; }
            if (it == 0 && std::getenv("SCVX_DUMP")) {
                FILE* fp = std::fopen(std::getenv("SCVX_DUMP"), "wb");
                for (int t = 0; t < K; ++t) { double buf[40] = {0}; for (int j = 0; j < ag.nd[t].nv && j < 40; ++j) buf[j] = dz[t][j]; std::fwrite(buf, sizeof(double), 40, fp); }
                std::fwrite(dyi.data(), sizeof(double), n, fp);
                std::fclose(fp);
            }
            double aa = std::min(1.0, max_step(ds, dl, dsq, dlq));
            double gap_a = 0.0;
            for (int t = 0; t < K; ++t) {
                Node& N = ag.nd[t];
                for (int r = 0; r < N.nr; ++r) gap_a += (N.s[r] + aa * ds[t][r]) * (N.lam[r] + aa * dl[t][r]);
                if (N.soc)
                    for (int j = 0; j <= m; ++j) gap_a += (N.ssoc[j] + aa * dsq[t][j]) * (N.lsoc[j] + aa * dlq[t][j]);
            }
            double mu_a = gap_a / std::max(deg, 1);
            const double sgr = std::max(mu_a, 0.0) / mu;   // the kernel's cube (products, not pow)
            double sig = sgr * sgr * sgr;
            // experiment knob SCVX_SKIP_CORR=thr: when the affine step is >= thr, step along the predictor direction
            static const double skip_thr = std::getenv("SCVX_SKIP_CORR") ? std::atof(std::getenv("SCVX_SKIP_CORR")) : 2.0;
            static const double skip_sgr = std::getenv("SCVX_SKIP_SGR") ? std::atof(std::getenv("SCVX_SKIP_SGR")) : 1e300;
            const bool skipc = aa >= skip_thr && sgr <= skip_sgr;
            if (skipc) ++n_skip;
            // corrector
            if (!skipc) for (int t = 0; t < K; ++t) {
                Node& N = ag.nd[t];
                for (int r = 0; r < N.nr; ++r) rco[t][r] += -ds[t][r] * dl[t][r] + sig * mu;
                if (N.soc) {
                    Vec a = matvec(L[t].soc.Wi, dsq[t]), b = matvec(L[t].soc.W, dlq[t]), c(m + 1);
                    jprod(a.data(), b.data(), m + 1, c.data());
                    for (int j = 0; j <= m; ++j) rcq[t][j] -= c[j];
                    rcq[t][0] += sig * mu;
                }
            }
            if (!skipc && !newton(rco, rcq, dz, ds, dl, dsq, dlq, dy, dyi, dyf)) { status = fail_status; break; }
            // experiment knob SCVX_TWIN_REFINE=k: k steps of iterative refinement of the corrector direction on the
            // linearised KKT system (its dual and dynamics residuals at the full-step point; the row and
            // complementarity equations hold by construction), each a re-solve with the same factorisation
            static const int refine = std::getenv("SCVX_TWIN_REFINE") ? std::atoi(std::getenv("SCVX_TWIN_REFINE")) : 0;
            bool ref_ok = true;
            for (int rr = 0; rr < refine && ref_ok; ++rr) {
                auto zt = [&](int t, int j) { return ag.nd[t].z[j] + dz[t][j]; };
                std::vector<Vec> rdt(K), rpt(K - 1, Vec(n)), zero_c(K), zero_q(K), rc_save(K), rcs_save(K), rd_save(K);
                Vec rpit(n), rpft(n, 0.0);
                for (int i = 0; i < n; ++i) rpit[i] = zt(0, i) - ag.x_init[i];
                if (T->has_final)
                    for (int i = 0; i < n; ++i) rpft[i] = zt(K - 1, i) - ag.x_final[i];
                for (int t = 0; t < K - 1; ++t)
                    for (int i = 0; i < n; ++i) {
                        double v = zt(t + 1, i) - ag.c[t][i];
                        for (int k = 0; k < n; ++k) v -= ag.A[t](i, k) * zt(t, k);
                        for (int j = 0; j < m; ++j) v -= ag.B[t](i, j) * zt(t, n + j) + ag.C[t](i, j) * zt(t + 1, n + j);
                        if (ag.nd[t].nnu) v -= zt(t, n + m + i);
                        rpt[t][i] = v;
                    }
                double emax = 0.0;
                for (int t = 0; t < K; ++t) {
                    Node& N = ag.nd[t];
                    Vec& r = rdt[t];
                    r.assign(N.nv, 0.0);
                    for (int j = 0; j < N.nv; ++j) r[j] = N.pdiag[j] * zt(t, j) + N.q[j];
                    for (int q = 0; q < N.nr; ++q)
                        for (int j = 0; j < N.nv; ++j) r[j] += N.G(q, j) * (N.lam[q] + dl[t][q]);
                    if (N.soc)
                        for (int j = 0; j < m; ++j) r[n + j] -= N.lsoc[1 + j] + dlq[t][1 + j];
                    if (t == 0)
                        for (int i = 0; i < n; ++i) r[i] += ag.y_init[i] + dyi[i];
                    if (t == K - 1 && T->has_final)
                        for (int i = 0; i < n; ++i) r[i] += ag.y_fin[i] + dyf[i];
                    if (t >= 1) {
                        const size_t o = (size_t)(t - 1) * n;
                        for (int i = 0; i < n; ++i) r[i] += ag.y[o + i] + dy[o + i];
                        for (int j = 0; j < m; ++j)
                            for (int i = 0; i < n; ++i) r[n + j] -= ag.C[t - 1](i, j) * (ag.y[o + i] + dy[o + i]);
                    }
                    if (t < K - 1) {
                        const size_t o = (size_t)t * n;
                        for (int k = 0; k < n; ++k)
                            for (int i = 0; i < n; ++i) r[k] -= ag.A[t](i, k) * (ag.y[o + i] + dy[o + i]);
                        for (int j = 0; j < m; ++j)
                            for (int i = 0; i < n; ++i) r[n + j] -= ag.B[t](i, j) * (ag.y[o + i] + dy[o + i]);
                        for (int i = 0; i < N.nnu; ++i) r[n + m + i] -= ag.y[o + i] + dy[o + i];
                    }
                    if (N.fixed_u)
                        for (int j = 0; j < m; ++j) r[n + j] = 0.0;
                    for (double v : r) emax = std::max(emax, std::fabs(v));
                    zero_c[t].assign(N.nr, 0.0);
                    zero_q[t].assign(N.soc ? m + 1 : 0, 0.0);
                    rd_save[t] = L[t].rd; rc_save[t] = L[t].rc; rcs_save[t] = L[t].rcs;
                    L[t].rd = r;
                    std::fill(L[t].rc.begin(), L[t].rc.end(), 0.0);
                    std::fill(L[t].rcs.begin(), L[t].rcs.end(), 0.0);
                }
                if (std::getenv("SCVX_DEBUG")) std::fprintf(stderr, "   refine %d: dual residual of the direction %.3e\n", rr, emax);
                std::swap(rp, rpt); std::swap(rpi, rpit); std::swap(rpf, rpft);
                std::vector<Vec> dz2, ds2, dl2, dsq2, dlq2;
                Vec dy2, dyi2, dyf2;
                ref_ok = newton(zero_c, zero_q, dz2, ds2, dl2, dsq2, dlq2, dy2, dyi2, dyf2);
                std::swap(rp, rpt); std::swap(rpi, rpit); std::swap(rpf, rpft);
                for (int t = 0; t < K; ++t) { L[t].rd = rd_save[t]; L[t].rc = rc_save[t]; L[t].rcs = rcs_save[t]; }
                if (!ref_ok) break;
                for (int t = 0; t < K; ++t) {
                    for (size_t j = 0; j < dz[t].size(); ++j) dz[t][j] += dz2[t][j];
                    for (size_t j = 0; j < ds[t].size(); ++j) { ds[t][j] += ds2[t][j]; dl[t][j] += dl2[t][j]; }
                    for (size_t j = 0; j < dsq[t].size(); ++j) { dsq[t][j] += dsq2[t][j]; dlq[t][j] += dlq2[t][j]; }
                }
                for (size_t i = 0; i < dy.size(); ++i) dy[i] += dy2[i];
                for (int i = 0; i < n; ++i) { dyi[i] += dyi2[i]; dyf[i] += dyf2[i]; }
            }
            if (!ref_ok) { status = fail_status; break; }
            // step fraction (kernel: the same rule, QP_TAU_END): 0.99 of the way to the boundary, 1 - 1e-5 once
            // the affine predictor takes a (nearly) full step -- the end game, where the fraction alone caps
            // the gap reduction per iteration at 1 / (1 - fraction).  SCVX_TAU_END: experiment knob
            static const double tau_end = std::getenv("SCVX_TAU_END") ? std::atof(std::getenv("SCVX_TAU_END")) : 0.99999;
            static const double tau_aa = std::getenv("SCVX_TAU_AA") ? std::atof(std::getenv("SCVX_TAU_AA")) : 0.99;  // knob
            static const double tau_mid = std::getenv("SCVX_TAU_MID") ? std::atof(std::getenv("SCVX_TAU_MID")) : 0.99;  // knob
            const double eta = (aa >= tau_aa) ? tau_end : tau_mid;
            double al = std::min(1.0, eta * max_step(ds, dl, dsq, dlq));
            {   // the kernel's NaN / Inf probe of the direction (fail code 4): keep the current iterate
                double pr = 0.0;
                for (int t = 0; t < K; ++t) {
                    for (double v : dz[t]) pr += 0.0 * v;
                    for (double v : ds[t]) pr += 0.0 * v;
                    for (double v : dl[t]) pr += 0.0 * v;
                    for (double v : dsq[t]) pr += 0.0 * v;
                    for (double v : dlq[t]) pr += 0.0 * v;
                }
                for (double v : dy) pr += 0.0 * v;
                if (!(pr + al == pr + al) || !(al > 0.0)) { status = fail_status; break; }
            }
            if (near && al < 1e-2) { status = SCVX_STATUS_MAX_ITER; break; }  // stall at reduced accuracy (kernel)
            if (std::getenv("SCVX_DEBUG")) {
                std::fprintf(stderr, "   alpha_aff %.3e sigma %.3e alpha %.3e\n", aa, sig, al);
                for (int t = 0; t < K; ++t) { Node& N = ag.nd[t]; for (int r = 0; r < N.nr; ++r) {
                    double a1 = ds[t][r] < 0 ? -N.s[r]/ds[t][r] : 1e300, a2 = dl[t][r] < 0 ? -N.lam[r]/dl[t][r] : 1e300;
                    if (std::min(a1,a2) < 1.01*al/0.99) std::fprintf(stderr, "     t %d r %d s %.3e ds %.3e lam %.3e dl %.3e\n", t, r, N.s[r], ds[t][r], N.lam[r], dl[t][r]); } }
            }
            for (int t = 0; t < K; ++t) {
                Node& N = ag.nd[t];
                for (int j = 0; j < N.nv; ++j) N.z[j] += al * dz[t][j];
                for (int r = 0; r < N.nr; ++r) { N.s[r] += al * ds[t][r]; N.lam[r] += al * dl[t][r]; }
                if (N.soc)
                    for (int j = 0; j <= m; ++j) { N.ssoc[j] += al * dsq[t][j]; N.lsoc[j] += al * dlq[t][j]; }
            }
            for (size_t i = 0; i < ag.y.size(); ++i) ag.y[i] += al * dy[i];
            for (int i = 0; i < n; ++i) { ag.y_init[i] += al * dyi[i]; ag.y_fin[i] += al * dyf[i]; }
        }
    }
done:
    if (wout) warm_save(ag, wout);
    double pobj = 0.0;
    for (int t = 0; t < K; ++t)
        for (int j = 0; j < ag.nd[t].nv; ++j) {
            double zj = ag.nd[t].z[j];
            pobj += 0.5 * ag.nd[t].pdiag[j] * zj * zj + ag.nd[t].q[j] * zj;
        }
    obj_out = pobj * osc;
    if (!ag.T->has_final && ag.T->w_final > 0.0)  // the soft terminal's constant w_final ||x_final||^2
        for (int i = 0; i < n; ++i) obj_out += ag.T->w_final * ag.x_final[i] * ag.x_final[i];
    if (ag.T->w_prox > 0.0)
        for (int t = 0; t < K; ++t)
            for (int i = 0; i < n; ++i) obj_out += ag.T->w_prox * ag.xref[(size_t)t * n + i] * ag.xref[(size_t)t * n + i];
    iters_out = it;
    if (std::getenv("SCVX_ENCODE_SKIP")) iters_out += 100 * n_skip;   // experiment: skipped correctors in the hundreds
    return status;
}

}  // namespace

extern "C" int oracle_qp_solve_batched(const scvx_qp_template* tpl, int N, const double* disc, const double* sigma,
                                       const double* Xref, const double* Uref, const double* x_init,
                                       const double* x_final, const double* tr, const double* coll_rows,
                                       const int32_t* coll_count, double* X, double* U, double* slack_coll,
                                       double* nu, double* obj, int32_t* status, int32_t* iters, int nthreads,
                                       const int32_t* warm, double* wstate) {
    const int n = tpl->n_x, m = tpl->n_u, K = tpl->K, pd = tpl->pos_dim;
    if (n <= 0 || m <= 0 || K < 2 || m > 4 || pd > 3) return -1;
    const size_t stride = (size_t)(K - 1) * n * (n + 2 * m + 2);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int a = 0; a < N; ++a) {
        Agent ag;
        const double* cr = tpl->j_max > 0 ? coll_rows + (size_t)a * K * tpl->j_max * (pd + 1) : nullptr;
        const int32_t* cc = tpl->j_max > 0 ? coll_count + (size_t)a * K : nullptr;
        setup_agent(ag, tpl, disc + a * stride, sigma[a], Xref + (size_t)a * K * n, Uref + (size_t)a * K * m,
                    x_init + (size_t)a * n, (tpl->has_final || tpl->w_final > 0.0) ? x_final + (size_t)a * n : nullptr, tr[a], cr, cc);
        int it = 0;
        double ob = 0.0;
        const long long wd = wstate ? warm_doubles(tpl) : 0;
        status[a] = solve_agent(ag, it, ob, (wstate && warm && warm[a]) ? wstate + a * wd : nullptr,
                                wstate ? wstate + a * wd : nullptr);
        iters[a] = it;
        obj[a] = ob;
        for (int t = 0; t < K; ++t) {
            for (int i = 0; i < n; ++i) X[((size_t)a * K + t) * n + i] = ag.nd[t].z[i];
            for (int j = 0; j < m; ++j) U[((size_t)a * K + t) * m + j] = ag.nd[t].z[n + j];
            const Node& Nt = ag.nd[t];
            slack_coll[(size_t)a * K + t] = (tpl->j_max > 0 && Nt.na > Nt.nnu) ? Nt.z[n + m + Nt.nnu + tpl->n_obs] : 0.0;
            if (nu && t < K - 1)
                for (int i = 0; i < n; ++i) nu[((size_t)a * (K - 1) + t) * n + i] = Nt.nnu ? Nt.z[n + m + i] : 0.0;
        }
    }
    return 0;
}

extern "C" long long oracle_qp_warm_doubles(const scvx_qp_template* tpl) { return warm_doubles(tpl); }
