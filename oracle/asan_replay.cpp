// ORACLE / TEST INFRASTRUCTURE ONLY: the sanitizer leg of SURVEY §5 for the CPU restatements.
//
// Built by `make -C oracle asan` with -fsanitize=address,undefined (no recovery) together with
// scvx_cpu.cpp and foh_ref.c into one executable (no Python process, so the ASan runtime comes first
// without any preload).  tools/asan_twin.py writes cases, runs this binary on them and compares its
// outputs with the regular liboracle.so run through ctypes.
//
// Case file (native endianness): int32 N, nthreads, model, nsub, n_params; double params[n_params];
// the scvx_qp_template bytes; then double X[N][K][n], U[N][K][m], sigma[N], x_init[N][n], x_final[N][n],
// tr[N]; when j_max > 0: double rows[N][K][j_max][pos_dim+1], int32 count[N][K].
// Per case: FOH of every agent (oracle_foh, the discretisation the QP consumes), a cold solve, then a
// warm-started re-solve of the same subproblems from the cold solve's final state (oracle/scvx_cpu.cpp
// warm_point).  Output: for both solves double X, U, obj and int32 status, iters, in that order.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/scvx_hip.h"

extern "C" int oracle_foh(int model, const double* prm, int n, int m, int K, const double* X, const double* U,
                          double sigma, int nsub, double* out);
extern "C" int oracle_qp_solve_batched(const scvx_qp_template* tpl, int N, const double* disc, const double* sigma,
                                       const double* Xref, const double* Uref, const double* x_init,
                                       const double* x_final, const double* tr, const double* coll_rows,
                                       const int32_t* coll_count, double* X, double* U, double* slack_coll,
                                       double* nu, double* obj, int32_t* status, int32_t* iters, int nthreads,
                                       const int32_t* warm, double* wstate);
extern "C" long long oracle_qp_warm_doubles(const scvx_qp_template* tpl);

namespace {
template <class T>
bool rd(FILE* f, T* p, size_t n) { return std::fread(p, sizeof(T), n, f) == n; }
template <class T>
void wr(FILE* f, const std::vector<T>& v) { std::fwrite(v.data(), sizeof(T), v.size(), f); }
}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s case.bin out.bin\n", argv[0]);
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    int32_t hdr[5];
    if (!rd(f, hdr, 5)) return 4;
    const int N = hdr[0], nthreads = hdr[1], model = hdr[2], nsub = hdr[3], npar = hdr[4];
    std::vector<double> prm(npar > 0 ? npar : 1, 0.0);
    if (npar > 0 && !rd(f, prm.data(), npar)) return 4;
    scvx_qp_template T;
    if (!rd(f, &T, 1)) return 4;
    const int n = T.n_x, m = T.n_u, K = T.K, J = T.j_max, pd = T.pos_dim;
    std::vector<double> X((size_t)N * K * n), U((size_t)N * K * m), sig(N), xi((size_t)N * n), xf((size_t)N * n),
        tr(N), rows(J > 0 ? (size_t)N * K * J * (pd + 1) : 1, 0.0);
    std::vector<int32_t> cnt(J > 0 ? (size_t)N * K : 1, 0);
    if (!rd(f, X.data(), X.size()) || !rd(f, U.data(), U.size()) || !rd(f, sig.data(), sig.size()) ||
        !rd(f, xi.data(), xi.size()) || !rd(f, xf.data(), xf.size()) || !rd(f, tr.data(), tr.size()))
        return 4;
    if (J > 0 && (!rd(f, rows.data(), rows.size()) || !rd(f, cnt.data(), cnt.size()))) return 4;
    std::fclose(f);
    const size_t ds = (size_t)(K - 1) * n * (n + 2 * m + 2);
    std::vector<double> disc((size_t)N * ds);
    for (int a = 0; a < N; ++a)
        if (oracle_foh(model, prm.data(), n, m, K, X.data() + (size_t)a * K * n, U.data() + (size_t)a * K * m, sig[a],
                       nsub, disc.data() + (size_t)a * ds) != 0)
            return 5;
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 3;
    const long long wd = oracle_qp_warm_doubles(&T);
    std::vector<double> ws((size_t)N * (size_t)(wd > 0 ? wd : 1), 0.0);
    std::vector<int32_t> warm(N, 0);
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<double> Xo((size_t)N * K * n), Uo((size_t)N * K * m), S((size_t)N * K), nu((size_t)N * (K - 1) * n),
            obj(N);
        std::vector<int32_t> st(N), it(N);
        const int rc = oracle_qp_solve_batched(&T, N, disc.data(), sig.data(), X.data(), U.data(), xi.data(), xf.data(),
                                               tr.data(), J > 0 ? rows.data() : nullptr, J > 0 ? cnt.data() : nullptr,
                                               Xo.data(), Uo.data(), S.data(), nu.data(), obj.data(), st.data(),
                                               it.data(), nthreads, pass ? warm.data() : nullptr, ws.data());
        if (rc != 0) return 6;
        wr(o, Xo); wr(o, Uo); wr(o, obj); wr(o, st); wr(o, it);
        for (int a = 0; a < N; ++a) warm[a] = st[a] == 0 ? 1 : 0;
    }
    std::fclose(o);
    return 0;
}
