// Device-side dynamics for the batched SCvx path (gfx950, float64).
//
// Each model provides, in the reference contract's terms (SCvx/models/base_model.py:16-24):
//   f(x,u)            -> dx/dt                 (n)
//   Av(x,u,v)         -> (df/dx) v            (n)   sparse, never materialises A
//   Bw(x,u,w)         -> (df/du) w            (n)
// Models:
//   DoubleIntegrator3D  x=[p;v], u=a          Distributed_opt/dist_scvx_3d.py:10-21
//   Unicycle            x=[x,y,th], u=[v,w]   SCvx/models/unicycle_model.py:54-63
//   SingleIntegrator3D  f=u                   SCvx/models/single_integrator_model.py:54-57
//   Quadrotor12         build-defined 6-DoF rigid body
#pragma once
#include <hip/hip_runtime.h>

#include "foh_body.hpp"  // ModelParams

namespace scvx {

struct DoubleIntegrator3D {
    static constexpr int N = 6, M = 3, ID = 0;
    __device__ __forceinline__ static void f(const double* x, const double* u, double* o, const ModelParams&) {
        o[0] = x[3]; o[1] = x[4]; o[2] = x[5]; o[3] = u[0]; o[4] = u[1]; o[5] = u[2];
    }
    __device__ __forceinline__ static void Av(const double*, const double*, const double* v, double* o,
                                              const ModelParams&) {
        o[0] = v[3]; o[1] = v[4]; o[2] = v[5]; o[3] = 0.0; o[4] = 0.0; o[5] = 0.0;
    }
    __device__ __forceinline__ static void Bw(const double*, const double*, const double* w, double* o,
                                              const ModelParams&) {
        o[0] = 0.0; o[1] = 0.0; o[2] = 0.0; o[3] = w[0]; o[4] = w[1]; o[5] = w[2];
    }
};

struct Unicycle {
    static constexpr int N = 3, M = 2, ID = 1;
    __device__ __forceinline__ static void f(const double* x, const double* u, double* o, const ModelParams&) {
        double s, c;
        sincos(x[2], &s, &c);
        o[0] = u[0] * c; o[1] = u[0] * s; o[2] = u[1];
    }
    __device__ __forceinline__ static void Av(const double* x, const double* u, const double* v, double* o,
                                              const ModelParams&) {
        double s, c;
        sincos(x[2], &s, &c);
        o[0] = -u[0] * s * v[2]; o[1] = u[0] * c * v[2]; o[2] = 0.0;
    }
    __device__ __forceinline__ static void Bw(const double* x, const double*, const double* w, double* o,
                                              const ModelParams&) {
        double s, c;
        sincos(x[2], &s, &c);
        o[0] = c * w[0]; o[1] = s * w[0]; o[2] = w[1];
    }
};

struct SingleIntegrator3D {
    static constexpr int N = 3, M = 3, ID = 2;
    __device__ __forceinline__ static void f(const double*, const double* u, double* o, const ModelParams&) {
        o[0] = u[0]; o[1] = u[1]; o[2] = u[2];
    }
    __device__ __forceinline__ static void Av(const double*, const double*, const double*, double* o,
                                              const ModelParams&) {
        o[0] = 0.0; o[1] = 0.0; o[2] = 0.0;
    }
    __device__ __forceinline__ static void Bw(const double*, const double*, const double* w, double* o,
                                              const ModelParams&) {
        o[0] = w[0]; o[1] = w[1]; o[2] = w[2];
    }
};

struct Quadrotor12 {
    static constexpr int N = 12, M = 4, ID = 3;
    __device__ __forceinline__ static void f(const double* x, const double* u, double* o, const ModelParams& P) {
        const double mass = P.p[0], g = P.p[1], Jx = P.p[2], Jy = P.p[3], Jz = P.p[4];
        double sf, cf, st, ct, sp, cp;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
        sincos(x[8], &sp, &cp);
        const double p = x[9], q = x[10], r = x[11], a = u[0] / mass;
        o[0] = x[3]; o[1] = x[4]; o[2] = x[5];
        o[3] = a * (cf * st * cp + sf * sp);
        o[4] = a * (cf * st * sp - sf * cp);
        o[5] = a * (cf * ct) - g;
        const double w = q * sf + r * cf;
        o[6] = p + w * st / ct;
        o[7] = q * cf - r * sf;
        o[8] = w / ct;
        o[9] = (u[1] + (Jy - Jz) * q * r) / Jx;
        o[10] = (u[2] + (Jz - Jx) * p * r) / Jy;
        o[11] = (u[3] + (Jx - Jy) * p * q) / Jz;
    }
    __device__ __forceinline__ static void Av(const double* x, const double* u, const double* v, double* o,
                                              const ModelParams& P) {
        const double mass = P.p[0], Jx = P.p[2], Jy = P.p[3], Jz = P.p[4];
        double sf, cf, st, ct, sp, cp;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
        sincos(x[8], &sp, &cp);
        const double p = x[9], q = x[10], r = x[11], a = u[0] / mass;
        const double tt = st / ct, ic = 1.0 / ct;
        o[0] = v[3]; o[1] = v[4]; o[2] = v[5];
        o[3] = a * ((-sf * st * cp + cf * sp) * v[6] + (cf * ct * cp) * v[7] + (-cf * st * sp + sf * cp) * v[8]);
        o[4] = a * ((-sf * st * sp - cf * cp) * v[6] + (cf * ct * sp) * v[7] + (cf * st * cp + sf * sp) * v[8]);
        o[5] = a * ((-sf * ct) * v[6] + (-cf * st) * v[7]);
        const double w = q * sf + r * cf, wd = q * cf - r * sf;
        o[6] = wd * tt * v[6] + w * ic * ic * v[7] + v[9] + sf * tt * v[10] + cf * tt * v[11];
        o[7] = -w * v[6] + cf * v[10] - sf * v[11];
        o[8] = wd * ic * v[6] + w * st * ic * ic * v[7] + sf * ic * v[10] + cf * ic * v[11];
        o[9] = (Jy - Jz) / Jx * (r * v[10] + q * v[11]);
        o[10] = (Jz - Jx) / Jy * (r * v[9] + p * v[11]);
        o[11] = (Jx - Jy) / Jz * (q * v[9] + p * v[10]);
    }
    __device__ __forceinline__ static void Bw(const double* x, const double*, const double* w, double* o,
                                              const ModelParams& P) {
        const double mass = P.p[0], Jx = P.p[2], Jy = P.p[3], Jz = P.p[4];
        double sf, cf, st, ct, sp, cp;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
        sincos(x[8], &sp, &cp);
        const double t = w[0] / mass;
        o[0] = 0.0; o[1] = 0.0; o[2] = 0.0;
        o[3] = t * (cf * st * cp + sf * sp);
        o[4] = t * (cf * st * sp - sf * cp);
        o[5] = t * (cf * ct);
        o[6] = 0.0; o[7] = 0.0; o[8] = 0.0;
        o[9] = w[1] / Jx; o[10] = w[2] / Jy; o[11] = w[3] / Jz;
    }
    // f, (df/dx) v and (df/du) w at one (x, u) with one set of sines / cosines and reciprocals (the FOH's right-hand
    // side evaluates all three at every RK4 stage: three separate calls cost nine FP64 sincos, each a range reduction
    // and two polynomials).  The same expressions as f / Av / Bw above, term for term.
    __device__ __forceinline__ static void fab(const double* x, const double* u, const double* v, const double* wv,
                                               double* fo, double* ao, double* bo, const ModelParams& P) {
        const double mass = P.p[0], g = P.p[1], Jx = P.p[2], Jy = P.p[3], Jz = P.p[4];
        double sf, cf, st, ct, sp, cp;
        sincos(x[6], &sf, &cf);
        sincos(x[7], &st, &ct);
        sincos(x[8], &sp, &cp);
        const double p = x[9], q = x[10], r = x[11], a = u[0] / mass;
        const double r1 = cf * st * cp + sf * sp, r2 = cf * st * sp - sf * cp, r3 = cf * ct;
        const double w = q * sf + r * cf, wd = q * cf - r * sf;
        fo[0] = x[3]; fo[1] = x[4]; fo[2] = x[5];
        fo[3] = a * r1;
        fo[4] = a * r2;
        fo[5] = a * r3 - g;
        fo[6] = p + w * st / ct;
        fo[7] = q * cf - r * sf;
        fo[8] = w / ct;
        fo[9] = (u[1] + (Jy - Jz) * q * r) / Jx;
        fo[10] = (u[2] + (Jz - Jx) * p * r) / Jy;
        fo[11] = (u[3] + (Jx - Jy) * p * q) / Jz;
        const double tt = st / ct, ic = 1.0 / ct;
        ao[0] = v[3]; ao[1] = v[4]; ao[2] = v[5];
        ao[3] = a * ((-sf * st * cp + cf * sp) * v[6] + (cf * ct * cp) * v[7] + (-cf * st * sp + sf * cp) * v[8]);
        ao[4] = a * ((-sf * st * sp - cf * cp) * v[6] + (cf * ct * sp) * v[7] + (cf * st * cp + sf * sp) * v[8]);
        ao[5] = a * ((-sf * ct) * v[6] + (-cf * st) * v[7]);
        ao[6] = wd * tt * v[6] + w * ic * ic * v[7] + v[9] + sf * tt * v[10] + cf * tt * v[11];
        ao[7] = -w * v[6] + cf * v[10] - sf * v[11];
        ao[8] = wd * ic * v[6] + w * st * ic * ic * v[7] + sf * ic * v[10] + cf * ic * v[11];
        ao[9] = (Jy - Jz) / Jx * (r * v[10] + q * v[11]);
        ao[10] = (Jz - Jx) / Jy * (r * v[9] + p * v[11]);
        ao[11] = (Jx - Jy) / Jz * (q * v[9] + p * v[10]);
        const double t = wv[0] / mass;
        bo[0] = 0.0; bo[1] = 0.0; bo[2] = 0.0;
        bo[3] = t * r1;
        bo[4] = t * r2;
        bo[5] = t * r3;
        bo[6] = 0.0; bo[7] = 0.0; bo[8] = 0.0;
        bo[9] = wv[1] / Jx; bo[10] = wv[2] / Jy; bo[11] = wv[3] / Jz;
    }
};

// host-side: parameter block of a model id (quadrotor defaults: mass 1, g 9.81, J = diag(.02,.02,.04))
inline ModelParams model_params(int model_id, const double* params) {
    ModelParams P{};
    if (model_id == Quadrotor12::ID) {
        const double dflt[5] = {1.0, 9.81, 0.02, 0.02, 0.04};
        for (int i = 0; i < 5; ++i) P.p[i] = params ? params[i] : dflt[i];
    }
    return P;
}

}  // namespace scvx
