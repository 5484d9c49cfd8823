// Runtime-compiled user models for the batched FOH and nonlinear roll-outs (hipRTC, gfx950).
//
// The reference's FirstOrderHold(model, K) accepts any BaseModel and integrates its numpy f/A/B
// (SCvx/discretization/first_order_hold.py:13-50, 89-125).  The built-in models of csrc/models.hpp
// are compiled into the library; a user model arrives as C expressions (include/scvx_hip.h), is
// wrapped into a model struct with the csrc/models.hpp contract and compiled by hipRTC together with
// csrc/foh_body.hpp -- the integrator the built-in models use, embedded here as text at build time --
// into two extern "C" kernels.  The Jacobians are applied as sparse matrix-vector products: entries
// given as structural zeros generate no code.
//
// Compile at create (host only, no GPU needed); load the code object per device at the first
// launch (hipModuleLoadData).  Launch through hipModuleLaunchKernel on the caller's stream.
#include <hip/hip_runtime.h>
#ifndef SCVX_OFFLOAD_ARCH
#define SCVX_OFFLOAD_ARCH "gfx950"
#endif
#include <hip/hiprtc.h>

#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "common.hpp"
#include "foh_body.hpp"  // ModelParams (the launch argument)
#include "intersample_body.hpp"  // ISArgs, intersample_check
#include "scvx_hip.h"

namespace {

// csrc/foh_body.hpp, csrc/intersample_body.hpp and include/scvx_hip.h as string literals (build/*.inc, generated
// by the Makefile)
const char* const kFohBody =
#include "foh_body.inc"
    ;
const char* const kIsBody =
#include "intersample_body.inc"
    ;
const char* const kScvxHdrF =
#include "scvx_hip_h.inc"
    ;

bool is_zero(const char* e) {
    if (!e) return true;
    std::string s;
    for (const char* c = e; *c; ++c)
        if (*c != ' ' && *c != '\t' && *c != '\n' && *c != '(' && *c != ')') s += *c;
    return s.empty() || s == "0" || s == "0.0" || s == "0." || s == "-0" || s == "-0.0" || s == "+0";
}

// o = M v for a row-major (rows x cols) expression matrix, zero entries skipped
std::string matvec(const char* const* M, int rows, int cols, const char* vec) {
    std::string s;
    for (int i = 0; i < rows; ++i) {
        std::string row;
        for (int j = 0; j < cols; ++j) {
            const char* e = M ? M[i * cols + j] : nullptr;
            if (is_zero(e)) continue;
            if (!row.empty()) row += " + ";
            row += "(" + std::string(e) + ") * " + vec + "[" + std::to_string(j) + "]";
        }
        s += "        o_[" + std::to_string(i) + "] = " + (row.empty() ? std::string("0.0") : row) + ";\n";
    }
    return s;
}

std::string generate(int n, int m, const char* const* f, const char* const* A, const char* const* B,
                     const char* prelude) {
    std::string pre = "        const double* p = P_.p; (void)p;\n";
    if (prelude) {  // one statement line per prelude line, indented
        std::string line;
        for (const char* c = prelude;; ++c) {
            if (*c == '\n' || *c == 0) {
                if (!line.empty()) pre += "        " + line + "\n";
                line.clear();
                if (*c == 0) break;
            } else {
                line += *c;
            }
        }
    }
    std::string s;
    s += "#include \"foh_body.hpp\"\n";
    s += "namespace {\nstruct UserModel {\n";
    s += "    static constexpr int N = " + std::to_string(n) + ", M = " + std::to_string(m) + ";\n";
    s += "    __device__ __forceinline__ static void f(const double* x, const double* u, double* o_,\n"
         "                                             const scvx::ModelParams& P_) {\n";
    s += pre;
    for (int i = 0; i < n; ++i)
        s += "        o_[" + std::to_string(i) + "] = " + (is_zero(f[i]) ? std::string("0.0") : "(" + std::string(f[i]) + ")") + ";\n";
    s += "    }\n";
    s += "    __device__ __forceinline__ static void Av(const double* x, const double* u, const double* v_,\n"
         "                                              double* o_, const scvx::ModelParams& P_) {\n";
    s += pre + matvec(A, n, n, "v_") + "    }\n";
    s += "    __device__ __forceinline__ static void Bw(const double* x, const double* u, const double* w_,\n"
         "                                              double* o_, const scvx::ModelParams& P_) {\n";
    s += pre + matvec(B, n, m, "w_") + "    }\n";
    s += "};\n}  // namespace\n\n";
    s += "extern \"C\" __global__ __launch_bounds__(256) void scvx_rtc_foh(const double* X, const double* U,\n"
         "        const double* sigma, double* out, int K, int N, int nsub, scvx::ModelParams P) {\n"
         "    __shared__ double stage[256 * UserModel::N];\n"
         "    scvx::foh_body<UserModel>(X, U, sigma, out, K, N, nsub, P, stage);\n}\n";
    s += "extern \"C\" __global__ __launch_bounds__(256) void scvx_rtc_nonlinear(const double* X, const double* U,\n"
         "        const double* sigma, double* Xout, int K, int N, int nsub, int piecewise, scvx::ModelParams P) {\n"
         "    scvx::nonlinear_body<UserModel>(X, U, sigma, Xout, K, N, nsub, piecewise, P);\n}\n";
    if (n <= SCVX_IS_MAX_STATE) {   // the inter-sample scan (csrc/intersample_body.hpp) on this model's f
        s += "#include \"intersample_body.hpp\"\n";
        s += "extern \"C\" __global__ __launch_bounds__(256) void scvx_rtc_intersample(scvx::ISArgs a) {\n"
             "    scvx::intersample_body<UserModel>(a);\n}\n";
    }
    return s;
}

struct Loaded {
    hipModule_t mod = nullptr;
    hipFunction_t foh = nullptr, nl = nullptr, is = nullptr;
};

}  // namespace

struct scvx_rtc_model {
    int n = 0, m = 0;
    std::string src, log;
    std::vector<char> code;
    std::mutex mu;
    std::map<int, Loaded> loaded;  // device -> module
};

namespace {

int load(const scvx_rtc_model* cm, Loaded* out) {
    auto* md = const_cast<scvx_rtc_model*>(cm);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return scvx::set_error(SCVX_ELAUNCH, "rtc: no HIP device");
    std::lock_guard<std::mutex> g(md->mu);
    auto it = md->loaded.find(dev);
    if (it != md->loaded.end()) { *out = it->second; return SCVX_OK; }
    Loaded L;
    hipError_t e = hipModuleLoadData(&L.mod, md->code.data());
    if (e != hipSuccess) {
        std::string msg = std::string("rtc: hipModuleLoadData: ") + hipGetErrorString(e);
        return scvx::set_error(SCVX_ELAUNCH, msg.c_str());
    }
    if (hipModuleGetFunction(&L.foh, L.mod, "scvx_rtc_foh") != hipSuccess ||
        hipModuleGetFunction(&L.nl, L.mod, "scvx_rtc_nonlinear") != hipSuccess) {
        (void)hipModuleUnload(L.mod);
        return scvx::set_error(SCVX_ELAUNCH, "rtc: kernels missing from the code object");
    }
    if (md->n <= SCVX_IS_MAX_STATE && hipModuleGetFunction(&L.is, L.mod, "scvx_rtc_intersample") != hipSuccess) {
        (void)hipModuleUnload(L.mod);
        return scvx::set_error(SCVX_ELAUNCH, "rtc: intersample kernel missing from the code object");
    }
    md->loaded[dev] = L;
    *out = L;
    return SCVX_OK;
}

int params_of(const double* params, int n_params, scvx::ModelParams* P) {
    if (n_params < 0 || n_params > SCVX_MAX_MODEL_PARAMS || (n_params > 0 && !params))
        return scvx::set_error(SCVX_EINVAL, "rtc: bad params");
    std::memset(P, 0, sizeof(*P));
    for (int i = 0; i < n_params; ++i) P->p[i] = params[i];
    return SCVX_OK;
}

}  // namespace

extern "C" int scvx_rtc_model_create(int n_x, int n_u, const char* const* f_exprs, const char* const* A_exprs,
                                     const char* const* B_exprs, const char* prelude, scvx_rtc_model** out) {
    if (!out) return scvx::set_error(SCVX_EINVAL, "rtc: out is NULL");
    *out = nullptr;
    if (n_x < 1 || n_x > SCVX_RTC_MAX_NX || n_u < 1 || n_u > SCVX_RTC_MAX_NU || !f_exprs)
        return scvx::set_error(SCVX_EINVAL, "rtc: need 1 <= n_x <= 16, 1 <= n_u <= 8 and f_exprs");
    auto* md = new (std::nothrow) scvx_rtc_model;
    if (!md) return scvx::set_error(SCVX_EINVAL, "rtc: out of host memory");
    md->n = n_x;
    md->m = n_u;
    md->src = generate(n_x, n_u, f_exprs, A_exprs, B_exprs, prelude);
    hiprtcProgram prog;
    const char* hdr_src[3] = {kFohBody, kIsBody, kScvxHdrF};
    const char* hdr_name[3] = {"foh_body.hpp", "intersample_body.hpp", "scvx_hip.h"};
    if (hiprtcCreateProgram(&prog, md->src.c_str(), "scvx_user_model.hip", 3, hdr_src, hdr_name) !=
        HIPRTC_SUCCESS) {
        delete md;
        return scvx::set_error(SCVX_EINVAL, "rtc: hiprtcCreateProgram failed");
    }
    // the library's own target (the Makefile's ARCH): a user model's code object loads where the library runs
    const char* opts[] = {"--offload-arch=" SCVX_OFFLOAD_ARCH, "-O3", "-std=c++17"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    size_t ls = 0;
    if (hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
        md->log.resize(ls);
        hiprtcGetProgramLog(prog, &md->log[0]);
        md->log.resize(std::strlen(md->log.c_str()));
    }
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        std::string msg = std::string("rtc: compile failed: ") + hiprtcGetErrorString(rc) + "\n" + md->log;
        *out = md;  // kept so that the caller can read the log and the source; destroy it
        return scvx::set_error(SCVX_EINVAL, msg.c_str());
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    md->code.resize(cs);
    hiprtcGetCode(prog, md->code.data());
    hiprtcDestroyProgram(&prog);
    if (cs == 0) {
        *out = md;
        return scvx::set_error(SCVX_EINVAL, "rtc: empty code object");
    }
    *out = md;
    return SCVX_OK;
}

extern "C" const char* scvx_rtc_model_source(const scvx_rtc_model* model) { return model ? model->src.c_str() : ""; }
extern "C" const char* scvx_rtc_model_log(const scvx_rtc_model* model) { return model ? model->log.c_str() : ""; }

extern "C" int scvx_rtc_model_destroy(scvx_rtc_model* model) {
    if (!model) return SCVX_OK;
    for (auto& kv : model->loaded) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(kv.first);
        (void)hipModuleUnload(kv.second.mod);
        (void)hipSetDevice(cur);
    }
    delete model;
    return SCVX_OK;
}

extern "C" int scvx_rtc_foh_batched(const scvx_rtc_model* model, const double* params, int n_params, int K, int N,
                                    const double* X, const double* U, const double* sigma, int nsub, double* out,
                                    void* stream) {
    if (!model || model->code.empty() || K < 2 || N < 0 || nsub < 1 || !X || !U || !sigma || !out)
        return scvx::set_error(SCVX_EINVAL, "rtc foh: bad args");
    scvx::ModelParams P;
    if (int rc = params_of(params, n_params, &P)) return rc;
    if (N == 0) return SCVX_OK;
    Loaded L;
    if (int rc = load(model, &L)) return rc;
    const long long total = (long long)N * (K - 1) * (model->n + 2 * model->m + 2);
    const unsigned grid = (unsigned)((total + 255) / 256);
    void* args[] = {(void*)&X, (void*)&U, (void*)&sigma, (void*)&out, (void*)&K, (void*)&N, (void*)&nsub, (void*)&P};
    hipError_t e = hipModuleLaunchKernel(L.foh, grid, 1, 1, 256, 1, 1, 0, (hipStream_t)stream, args, nullptr);
    if (e != hipSuccess) {
        std::string msg = std::string("rtc foh launch: ") + hipGetErrorString(e);
        return scvx::set_error(SCVX_ELAUNCH, msg.c_str());
    }
    return SCVX_OK;
}

extern "C" int scvx_rtc_integrate_nonlinear_batched(const scvx_rtc_model* model, const double* params, int n_params,
                                                    int K, int N, const double* X, const double* U,
                                                    const double* sigma, int nsub, int piecewise, double* Xout,
                                                    void* stream) {
    if (!model || model->code.empty() || K < 2 || N < 0 || nsub < 1 || !X || !U || !sigma || !Xout)
        return scvx::set_error(SCVX_EINVAL, "rtc nl: bad args");
    scvx::ModelParams P;
    if (int rc = params_of(params, n_params, &P)) return rc;
    if (N == 0) return SCVX_OK;
    Loaded L;
    if (int rc = load(model, &L)) return rc;
    const long long total = piecewise ? (long long)N * (K - 1) : (long long)N;
    const int block = piecewise ? 256 : 64;
    const unsigned grid = (unsigned)((total + block - 1) / block);
    void* args[] = {(void*)&X, (void*)&U, (void*)&sigma, (void*)&Xout, (void*)&K, (void*)&N, (void*)&nsub,
                    (void*)&piecewise, (void*)&P};
    hipError_t e = hipModuleLaunchKernel(L.nl, grid, 1, 1, block, 1, 1, 0, (hipStream_t)stream, args, nullptr);
    if (e != hipSuccess) {
        std::string msg = std::string("rtc nl launch: ") + hipGetErrorString(e);
        return scvx::set_error(SCVX_ELAUNCH, msg.c_str());
    }
    return SCVX_OK;
}

extern "C" int scvx_rtc_intersample_batched(const scvx_rtc_model* model, const double* params, int n_params,
                                            const scvx_intersample_template* tpl, int K, int N, const double* X,
                                            const double* U, const double* sigma, int32_t* n_crit, double* t_crit,
                                            double* h0, double* grad_x, double* grad_u, void* stream) {
    if (!model || model->code.empty() || !tpl) return scvx::set_error(SCVX_EINVAL, "rtc intersample: bad args");
    if (const char* bad = scvx::intersample_check(*tpl, K, N, model->n)) return scvx::set_error(SCVX_EINVAL, bad);
    scvx::ModelParams P;
    if (int rc = params_of(params, n_params, &P)) return rc;
    if (N == 0 || tpl->n_obs == 0) return SCVX_OK;
    if (!X || !U || !sigma || !n_crit || !t_crit || !h0 || !grad_x || !grad_u)
        return scvx::set_error(SCVX_EINVAL, "rtc intersample: null buffer");
    Loaded L;
    if (int rc = load(model, &L)) return rc;
    scvx::ISArgs a{};
    a.T = *tpl;
    a.K = K; a.N = N;
    a.X = X; a.U = U; a.sigma = sigma;
    a.n_crit = n_crit; a.t_crit = t_crit; a.h0 = h0; a.grad_x = grad_x; a.grad_u = grad_u;
    a.P = P;
    const long long nwork = (long long)N * (K - 1) * tpl->n_obs;
    const unsigned grid = (unsigned)((nwork + 255) / 256);
    void* args[] = {(void*)&a};
    hipError_t e = hipModuleLaunchKernel(L.is, grid, 1, 1, 256, 1, 1, 0, (hipStream_t)stream, args, nullptr);
    if (e != hipSuccess) {
        std::string msg = std::string("rtc intersample launch: ") + hipGetErrorString(e);
        return scvx::set_error(SCVX_ELAUNCH, msg.c_str());
    }
    return SCVX_OK;
}
