// Runtime-compiled subproblem kernels for user models (hipRTC, the library's own ARCH).
//
// The FOH of any model is runtime-compiled from its expressions (csrc/foh_rtc.hip).  The convex subproblems
// that consume it -- the trust-region QP of Distributed_opt/dist_scvx_3d.py:51-111 (csrc/qp_ipm.hpp) and the
// SCProblem LP/SOCP of SCvx/optimization/sc_problem.py:15-83 (csrc/scp_kernel.hpp) -- do not depend on the
// model's dynamics, only on its dimensions (n_x, n_u) and the template's row counts.  A template with
// model_id = SCVX_MODEL_RUNTIME is therefore served by the same kernel source, instantiated by hipRTC for
// exactly its (n_x, n_u, rows) at the first solve: the headers are embedded in the library as text at build
// time (the Makefile's build/*.inc), so built-in and user classes run one kernel.  Code objects are cached
// per instantiation (and per device once loaded); a compile costs ~10 s once per process.
#include <hip/hip_runtime.h>
#ifndef SCVX_OFFLOAD_ARCH
#define SCVX_OFFLOAD_ARCH "gfx950"
#endif
#include <hip/hiprtc.h>

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "scvx_hip.h"
#include "subproblem_rtc.hpp"

namespace {

const char* const kQpIpm =
#include "qp_ipm.inc"
    ;
const char* const kScpKernel =
#include "scp_kernel.inc"
    ;
const char* const kWaveOps =
#include "wave_ops.inc"
    ;
const char* const kScvxHdr =
#include "scvx_hip_h.inc"
    ;

struct Instance {
    std::vector<char> code;
    std::string lowered, log;
    std::map<int, std::pair<hipModule_t, hipFunction_t>> loaded;  // device -> module, kernel
};

std::mutex g_mu;
std::map<std::string, std::unique_ptr<Instance>> g_cache;

// compile `src` (with the embedded headers) and keep the lowered name of `expr`; cached by key
int compile(const std::string& key, const std::string& src, const std::string& expr, Instance** out) {
    auto it = g_cache.find(key);
    if (it != g_cache.end()) { *out = it->second.get(); return SCVX_OK; }
    hiprtcProgram prog;
    const char* hsrc[4] = {kQpIpm, kScpKernel, kWaveOps, kScvxHdr};
    const char* hname[4] = {"qp_ipm.hpp", "scp_kernel.hpp", "wave_ops.hpp", "scvx_hip.h"};
    if (hiprtcCreateProgram(&prog, src.c_str(), "scvx_subproblem_rtc.hip", 4, hsrc, hname) != HIPRTC_SUCCESS)
        return scvx::set_error(SCVX_EINVAL, "subproblem rtc: hiprtcCreateProgram failed");
    hiprtcAddNameExpression(prog, expr.c_str());
    const char* opts[] = {"--offload-arch=" SCVX_OFFLOAD_ARCH, "-O3", "-std=c++17"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    auto inst = std::make_unique<Instance>();
    size_t ls = 0;
    if (hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
        inst->log.resize(ls);
        hiprtcGetProgramLog(prog, &inst->log[0]);
        inst->log.resize(std::strlen(inst->log.c_str()));
    }
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        std::string msg = "subproblem rtc: compile of " + expr + " failed: " + hiprtcGetErrorString(rc) + "\n" +
                          inst->log.substr(0, 2000);
        return scvx::set_error(SCVX_EINVAL, msg.c_str());
    }
    const char* lowered = nullptr;
    if (hiprtcGetLoweredName(prog, expr.c_str(), &lowered) != HIPRTC_SUCCESS || !lowered) {
        hiprtcDestroyProgram(&prog);
        return scvx::set_error(SCVX_EINVAL, "subproblem rtc: kernel name not found");
    }
    inst->lowered = lowered;
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    inst->code.resize(cs);
    hiprtcGetCode(prog, inst->code.data());
    hiprtcDestroyProgram(&prog);
    if (cs == 0) return scvx::set_error(SCVX_EINVAL, "subproblem rtc: empty code object");
    *out = inst.get();
    g_cache[key] = std::move(inst);
    return SCVX_OK;
}

int function_of(Instance* in, hipFunction_t* f) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return scvx::set_error(SCVX_ELAUNCH, "subproblem rtc: no HIP device");
    auto it = in->loaded.find(dev);
    if (it != in->loaded.end()) { *f = it->second.second; return SCVX_OK; }
    hipModule_t mod = nullptr;
    hipError_t e = hipModuleLoadData(&mod, in->code.data());
    if (e != hipSuccess) {
        std::string msg = std::string("subproblem rtc: hipModuleLoadData: ") + hipGetErrorString(e);
        return scvx::set_error(SCVX_ELAUNCH, msg.c_str());
    }
    hipFunction_t fn = nullptr;
    if (hipModuleGetFunction(&fn, mod, in->lowered.c_str()) != hipSuccess) {
        (void)hipModuleUnload(mod);
        return scvx::set_error(SCVX_ELAUNCH, "subproblem rtc: kernel missing from the code object");
    }
    in->loaded[dev] = {mod, fn};
    *f = fn;
    return SCVX_OK;
}

// the instantiation of a QP class <nx, nu, nb, no, nc, vc> / an SCP class <nx, nu, ne, nw>
struct Inst {
    std::string key, expr;
    const char* header;
};
Inst qp_inst(int nx, int nu, int nb, int no, int nc, int vc) {
    const std::string cls = std::to_string(nx) + ", " + std::to_string(nu) + ", " + std::to_string(nb) + ", " +
                            std::to_string(no) + ", " + std::to_string(nc) + ", " + std::to_string(vc);
    return {"qp<" + cls + ">", "scvx::qp_ipm_kernel<scvx::QPCfg<" + cls + ">>", "qp_ipm.hpp"};
}
Inst scp_inst(int nx, int nu, int ne, int nw) {
    const std::string cls = std::to_string(nx) + ", " + std::to_string(nu) + ", " + std::to_string(ne) + ", " +
                            std::to_string(nw);
    return {"scp<" + cls + ">", "scvx::scp_ipm_kernel<" + cls + ">", "scp_kernel.hpp"};
}

int compile_inst(const Inst& i, Instance** out) {
    return compile(i.key, std::string("#include \"") + i.header + "\"\n", i.expr, out);
}

int launch(const Inst& i, void** args, unsigned grid, unsigned block, size_t lds, hipStream_t st) {
    if (lds > 65536) return scvx::set_error(SCVX_EUNSUPPORTED, "subproblem rtc: class needs more than 64 KiB of LDS");
    hipFunction_t f = nullptr;
    {
        std::lock_guard<std::mutex> g(g_mu);
        Instance* in = nullptr;
        if (int rc = compile_inst(i, &in)) return rc;
        if (int rc = function_of(in, &f)) return rc;
    }
    hipError_t e = hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, (unsigned)lds, st, args, nullptr);
    if (e != hipSuccess) {
        std::string msg = std::string("subproblem rtc launch: ") + hipGetErrorString(e);
        return scvx::set_error(SCVX_ELAUNCH, msg.c_str());
    }
    return SCVX_OK;
}

}  // namespace

namespace scvx {

int rtc_qp_launch(const QPArgs& a, int nb, int no, int nc, int vc, hipStream_t st) {
    const int nx = a.T.n_x, nu = a.T.n_u;
    const size_t lds = sizeof(double) * (size_t)qp_lds_doubles(nx, nu, nb, no, nc, vc, a.T.K);
    QPArgs copy = a;
    void* args[] = {&copy};
    return launch(qp_inst(nx, nu, nb, no, nc, vc), args, (unsigned)a.N, WAVE, lds, st);
}

int rtc_scp_launch(const SCPArgs& a, int ne, int nw, hipStream_t st) {
    SCPArgs copy = a;
    double* ws = a.ws;
    const double* disc = a.disc;
    void* args[] = {&copy, &ws, &disc};   // scp_ipm_kernel(SCPArgs a, double* ws_all, const double* disc_all)
    return launch(scp_inst(a.T.n_x, a.T.n_u, ne, nw), args, (unsigned)a.N, WAVE * nw, 0, st);
}

}  // namespace scvx

extern "C" int scvx_rtc_subproblem_compile(int kind, const int* cls, int ncls, size_t* code_bytes) {
    if (!cls || (kind == 0 && ncls != 6) || (kind == 1 && ncls != 4) || kind < 0 || kind > 1)
        return scvx::set_error(SCVX_EINVAL, "scvx_rtc_subproblem_compile: kind 0 takes 6 class ints, kind 1 takes 4");
    for (int i = 0; i < ncls; ++i)
        if (cls[i] < 0 || cls[i] > 64) return scvx::set_error(SCVX_EINVAL, "scvx_rtc_subproblem_compile: class out of range");
    // the solve entry points' own limits (subproblem_rtc.hpp), checked before a ~10 s compile
    const char* bad = kind == 0 ? scvx::rtc_qp_class_error(cls[0], cls[1], cls[2], cls[3], cls[4], cls[5], 2)
                                : scvx::rtc_scp_class_error(cls[0], cls[1], cls[2]);
    if (bad) return scvx::set_error(SCVX_EUNSUPPORTED, bad);
    const Inst i = kind == 0 ? qp_inst(cls[0], cls[1], cls[2], cls[3], cls[4], cls[5])
                             : scp_inst(cls[0], cls[1], cls[2], cls[3]);
    std::lock_guard<std::mutex> g(g_mu);
    Instance* in = nullptr;
    if (int rc = compile_inst(i, &in)) return rc;
    if (code_bytes) *code_bytes = in->code.size();
    return SCVX_OK;
}
