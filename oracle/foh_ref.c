/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile into oracle/build/liboracle.so;
 * loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * path (the HIP library) never links or calls this file.
 *
 * Plain-C float64 restatement of the reference FOH discretizer
 * SCvx/discretization/first_order_hold.py:
 *   - normalized time, dt = 1/(K-1)                                   (:50)
 *   - u(t) = u0 + (t/dt)(u1-u0), alpha=(dt-t)/dt, beta=t/dt           (:91-98)
 *   - A_s = sigma*A(x,u), B_s = sigma*B(x,u), f unscaled, dx = sigma f (:101-113)
 *   - outputs A_k=Phi, B_k=Phi*Btil, C_k=Phi*Ctil, S_k=Phi*Stil, z_k=Phi*ztil, F-order  (:75-85)
 * The reference integrates [x, Phi, Phi^-1 ...] with LSODA and inverts Phi every RHS call
 * (:108).  Here the equivalent forward-sensitivity form is used (no inverse):
 *   Phi' = A_s Phi, P_B' = A_s P_B + B_s alpha, P_C' = A_s P_C + B_s beta,
 *   P_S' = A_s P_S + f, P_z' = A_s P_z - A_s x - B_s u
 * (d/dt(Phi*Btil) = A_s Phi Btil + B_s alpha, etc.), integrated by classical RK4 with
 * `nsub` fixed substeps per interval.  For the double integrator RK4 is exact.
 * Nonlinear roll-outs follow integrate_nonlinear_piecewise/_full/_dx (:127-162):
 * physical time [0, dt*sigma], u interpolated by t/(dt*sigma), dx = f(x,u).
 *
 * Models: 0 = 3-D double integrator (Distributed_opt/dist_scvx_3d.py:10-21),
 *         1 = unicycle (SCvx/models/unicycle_model.py:54-63),
 *         2 = single integrator (SCvx/models/single_integrator_model.py:54-57),
 *         3 = 12-state quadrotor (build-defined, params = mass,g,Jx,Jy,Jz).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NMAX 12
#define MMAX 4

static void model_eval(int model, const double *prm, const double *x, const double *u,
                       double *f, double *A, double *B, int n, int m) {
    /* A, B row-major dense n x n, n x m */
    memset(A, 0, sizeof(double) * n * n);
    memset(B, 0, sizeof(double) * n * m);
    if (model == 0) {
        for (int i = 0; i < 3; ++i) {
            f[i] = x[3 + i];
            f[3 + i] = u[i];
            A[i * n + 3 + i] = 1.0;
            B[(3 + i) * m + i] = 1.0;
        }
    } else if (model == 1) {
        double c = cos(x[2]), s = sin(x[2]);
        f[0] = u[0] * c; f[1] = u[0] * s; f[2] = u[1];
        A[0 * n + 2] = -u[0] * s;
        A[1 * n + 2] = u[0] * c;
        B[0 * m + 0] = c; B[1 * m + 0] = s; B[2 * m + 1] = 1.0;
    } else if (model == 2) {
        for (int i = 0; i < 3; ++i) { f[i] = u[i]; B[i * m + i] = 1.0; }
    } else {
        double mass = prm[0], g = prm[1], Jx = prm[2], Jy = prm[3], Jz = prm[4];
        double ph = x[6], th = x[7], ps = x[8], p = x[9], q = x[10], r = x[11];
        double cf = cos(ph), sf = sin(ph), ct = cos(th), st = sin(th), cp = cos(ps), sp = sin(ps);
        double a = u[0] / mass, tt = st / ct;
        double e0 = cf * st * cp + sf * sp, e1 = cf * st * sp - sf * cp, e2 = cf * ct;
        for (int i = 0; i < 3; ++i) f[i] = x[3 + i];
        f[3] = a * e0; f[4] = a * e1; f[5] = a * e2 - g;
        f[6] = p + (q * sf + r * cf) * tt;
        f[7] = q * cf - r * sf;
        f[8] = (q * sf + r * cf) / ct;
        f[9] = (u[1] + (Jy - Jz) * q * r) / Jx;
        f[10] = (u[2] + (Jz - Jx) * p * r) / Jy;
        f[11] = (u[3] + (Jx - Jy) * p * q) / Jz;
        A[0 * n + 3] = A[1 * n + 4] = A[2 * n + 5] = 1.0;
        A[3 * n + 6] = a * (-sf * st * cp + cf * sp);
        A[3 * n + 7] = a * (cf * ct * cp);
        A[3 * n + 8] = a * (-cf * st * sp + sf * cp);
        A[4 * n + 6] = a * (-sf * st * sp - cf * cp);
        A[4 * n + 7] = a * (cf * ct * sp);
        A[4 * n + 8] = a * (cf * st * cp + sf * sp);
        A[5 * n + 6] = a * (-sf * ct);
        A[5 * n + 7] = a * (-cf * st);
        A[6 * n + 6] = (q * cf - r * sf) * tt;
        A[6 * n + 7] = (q * sf + r * cf) / (ct * ct);
        A[6 * n + 9] = 1.0;
        A[6 * n + 10] = sf * tt;
        A[6 * n + 11] = cf * tt;
        A[7 * n + 6] = -q * sf - r * cf;
        A[7 * n + 10] = cf;
        A[7 * n + 11] = -sf;
        A[8 * n + 6] = (q * cf - r * sf) / ct;
        A[8 * n + 7] = (q * sf + r * cf) * st / (ct * ct);
        A[8 * n + 10] = sf / ct;
        A[8 * n + 11] = cf / ct;
        A[9 * n + 10] = (Jy - Jz) * r / Jx;
        A[9 * n + 11] = (Jy - Jz) * q / Jx;
        A[10 * n + 9] = (Jz - Jx) * r / Jy;
        A[10 * n + 11] = (Jz - Jx) * p / Jy;
        A[11 * n + 9] = (Jx - Jy) * q / Jz;
        A[11 * n + 10] = (Jx - Jy) * p / Jz;
        B[3 * m + 0] = e0 / mass; B[4 * m + 0] = e1 / mass; B[5 * m + 0] = e2 / mass;
        B[9 * m + 1] = 1.0 / Jx; B[10 * m + 2] = 1.0 / Jy; B[11 * m + 3] = 1.0 / Jz;
    }
}

/* augmented state layout: x(n) | Phi(n*n col-major) | PB(n*m) | PC(n*m) | PS(n) | Pz(n) */
static void foh_rhs(int model, const double *prm, int n, int m, double dt, double sigma,
                    const double *u0, const double *u1, double t, const double *V, double *dV) {
    double u[MMAX], f[NMAX], A[NMAX * NMAX], B[NMAX * MMAX];
    double alpha = (dt - t) / dt, beta = t / dt;
    for (int j = 0; j < m; ++j) u[j] = u0[j] + (t / dt) * (u1[j] - u0[j]);
    const double *x = V;
    model_eval(model, prm, x, u, f, A, B, n, m);
    int ncol = n + 2 * m + 2;
    const double *P = V + n;
    double *dP = dV + n;
    for (int i = 0; i < n; ++i) dV[i] = sigma * f[i];
    for (int c = 0; c < ncol; ++c) {
        const double *col = P + c * n;
        double *dcol = dP + c * n;
        for (int i = 0; i < n; ++i) {
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc += sigma * A[i * n + k] * col[k];
            if (c >= n && c < n + m) acc += sigma * B[i * m + (c - n)] * alpha;
            else if (c >= n + m && c < n + 2 * m) acc += sigma * B[i * m + (c - n - m)] * beta;
            else if (c == n + 2 * m) acc += f[i];
            else if (c == n + 2 * m + 1) {
                double z = 0.0;
                for (int k = 0; k < n; ++k) z -= sigma * A[i * n + k] * x[k];
                for (int k = 0; k < m; ++k) z -= sigma * B[i * m + k] * u[k];
                acc += z;
            }
            dcol[i] = acc;
        }
    }
}

/* X: [K][n], U: [K][m]; out: [K-1][n*n + 2*n*m + 2*n] (A|B|C|S|z, each column-major) */
int oracle_foh(int model, const double *prm, int n, int m, int K, const double *X,
               const double *U, double sigma, int nsub, double *out) {
    if (n > NMAX || m > MMAX || K < 2 || nsub < 1) return -1;
    int L = n + n * n + 2 * n * m + 2 * n;
    int stride = L - n;
    double dt = 1.0 / (K - 1), h = dt / nsub;
    double *V = malloc(sizeof(double) * L * 6);
    double *k1 = V + L, *k2 = V + 2 * L, *k3 = V + 3 * L, *k4 = V + 4 * L, *tmp = V + 5 * L;
    for (int k = 0; k < K - 1; ++k) {
        memset(V, 0, sizeof(double) * L);
        for (int i = 0; i < n; ++i) V[i] = X[k * n + i];
        for (int i = 0; i < n; ++i) V[n + i * n + i] = 1.0;
        const double *u0 = U + k * m, *u1 = U + (k + 1) * m;
        for (int s = 0; s < nsub; ++s) {
            double t = s * h;
            foh_rhs(model, prm, n, m, dt, sigma, u0, u1, t, V, k1);
            for (int i = 0; i < L; ++i) tmp[i] = V[i] + 0.5 * h * k1[i];
            foh_rhs(model, prm, n, m, dt, sigma, u0, u1, t + 0.5 * h, tmp, k2);
            for (int i = 0; i < L; ++i) tmp[i] = V[i] + 0.5 * h * k2[i];
            foh_rhs(model, prm, n, m, dt, sigma, u0, u1, t + 0.5 * h, tmp, k3);
            for (int i = 0; i < L; ++i) tmp[i] = V[i] + h * k3[i];
            foh_rhs(model, prm, n, m, dt, sigma, u0, u1, t + h, tmp, k4);
            for (int i = 0; i < L; ++i) V[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
        }
        memcpy(out + (size_t)k * stride, V + n, sizeof(double) * stride);
    }
    free(V);
    return 0;
}

static void nl_rhs(int model, const double *prm, int n, int m, double T, const double *u0,
                   const double *u1, double t, const double *x, double *dx) {
    double u[MMAX], A[NMAX * NMAX], B[NMAX * MMAX];
    for (int j = 0; j < m; ++j) u[j] = u0[j] + (t / T) * (u1[j] - u0[j]);
    model_eval(model, prm, x, u, dx, A, B, n, m);
}

/* piecewise=1: each interval restarts from X[:,k] (integrate_nonlinear_piecewise);
 * piecewise=0: chained from X[:,0] (integrate_nonlinear_full).  Xout: [K][n]. */
int oracle_integrate_nonlinear(int model, const double *prm, int n, int m, int K, const double *X,
                               const double *U, double sigma, int nsub, int piecewise, double *Xout) {
    if (n > NMAX || m > MMAX || K < 2 || nsub < 1) return -1;
    double T = sigma / (K - 1), h = T / nsub;
    double x[NMAX], k1[NMAX], k2[NMAX], k3[NMAX], k4[NMAX], tmp[NMAX];
    for (int i = 0; i < n; ++i) Xout[i] = X[i];
    for (int k = 0; k < K - 1; ++k) {
        const double *src = piecewise ? X + k * n : Xout + k * n;
        for (int i = 0; i < n; ++i) x[i] = src[i];
        const double *u0 = U + k * m, *u1 = U + (k + 1) * m;
        for (int s = 0; s < nsub; ++s) {
            double t = s * h;
            nl_rhs(model, prm, n, m, T, u0, u1, t, x, k1);
            for (int i = 0; i < n; ++i) tmp[i] = x[i] + 0.5 * h * k1[i];
            nl_rhs(model, prm, n, m, T, u0, u1, t + 0.5 * h, tmp, k2);
            for (int i = 0; i < n; ++i) tmp[i] = x[i] + 0.5 * h * k2[i];
            nl_rhs(model, prm, n, m, T, u0, u1, t + 0.5 * h, tmp, k3);
            for (int i = 0; i < n; ++i) tmp[i] = x[i] + h * k3[i];
            nl_rhs(model, prm, n, m, T, u0, u1, t + h, tmp, k4);
            for (int i = 0; i < n; ++i) x[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
        }
        for (int i = 0; i < n; ++i) Xout[(k + 1) * n + i] = x[i];
    }
    return 0;
}
