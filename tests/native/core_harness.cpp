// core_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Runs the exact per-QP device algorithm of intent-mpc_amd/csrc/admm_core.hpp on the host CPU
// (one QP after another, same batch-interleaved layout) so that the algorithm can be checked
// against the oracle in the GPU-less container.  It is never linked into libimpc_qp.so and no
// product entry point can reach it; the product path runs admm_core only inside HIP kernels.
#include <cstring>
#include <vector>

#include "../../intent-mpc_amd/csrc/admm_core.hpp"
#include "../../intent-mpc_amd/csrc/symbolic.hpp"

extern "C" int harness_solve_batch(int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                                   const int64_t *Ai, int64_t B, const double *Px, const double *q, const double *Ax,
                                   const double *l, const double *u, const impc_settings *s, const double *xws,
                                   const double *yws, double *xo, double *yo, impc_info *info, int64_t *nnzL_out) {
    impc::Symbolic sym;
    if (!sym.build(n, m, Pp, Pi, Ap, Ai).empty()) return 1;
    if (nnzL_out) *nnzL_out = sym.nnzL;
    impc::DevSym d{};
    d.n = sym.n;
    d.m = sym.m;
    d.nnzP = sym.nnzP;
    d.nnzA = sym.nnzA;
    d.nnzM = (int32_t)sym.nnzM;
    d.nnzL = (int32_t)sym.nnzL;
    d.nPt = (int32_t)sym.Pt_dest.size();
    d.nAt = (int32_t)sym.At_dest.size();
    d.Pp = sym.Pp.data();
    d.Pi = sym.Pi.data();
    d.Ap = sym.Ap.data();
    d.Ai = sym.Ai.data();
    d.Arp = sym.Arp.data();
    d.Arpos = sym.Arpos.data();
    d.Arcol = sym.Arcol.data();
    d.Arcolf = sym.Arcolf.data();
    d.perm = sym.perm.data();
    d.iperm = sym.iperm.data();
    d.Mp = sym.Mp.data();
    d.Mi = sym.Mi.data();
    d.Mdiag = sym.Mdiag.data();
    d.Pt_dest = sym.Pt_dest.data();
    d.Pt_src = sym.Pt_src.data();
    d.At_dest = sym.At_dest.data();
    d.At_a = sym.At_a.data();
    d.At_b = sym.At_b.data();
    d.At_r = sym.At_r.data();
    d.Lp = sym.Lp.data();
    d.Li = sym.Li.data();
    d.Lrp = sym.Lrp.data();
    d.Lrc = sym.Lrc.data();
    d.Lrpos = sym.Lrpos.data();
    d.upd_ptr = sym.upd_ptr.data();
    d.upd_c = sym.upd_c.data();
    d.upd_js = sym.upd_js.data();
    d.upd_je = sym.upd_je.data();
    d.upd_w = sym.upd_w.data();

    impc::DevSettings st{};
    st.rho = s->rho;
    st.sigma = s->sigma;
    st.adaptive_rho_tolerance = s->adaptive_rho_tolerance;
    st.eps_abs = s->eps_abs;
    st.eps_rel = s->eps_rel;
    st.eps_prim_inf = s->eps_prim_inf;
    st.eps_dual_inf = s->eps_dual_inf;
    st.alpha = s->alpha;
    st.time_limit = 0;
    st.scaling = (int32_t)s->scaling;
    st.adaptive_rho = (int32_t)s->adaptive_rho;
    st.rho_interval = s->adaptive_rho_interval ? (int32_t)s->adaptive_rho_interval
                                               : (int32_t)(s->check_termination ? s->check_termination : 25);
    st.max_iter = (int32_t)s->max_iter;
    st.scaled_termination = (int32_t)s->scaled_termination;
    st.check_termination = (int32_t)s->check_termination;
    st.warm_start = (int32_t)s->warm_start;

    const int64_t S = B;
    const int64_t nP = sym.nnzP, nA = sym.nnzA, nM = sym.nnzM, nL = sym.nnzL;
    std::vector<std::vector<double>> store;
    auto alloc = [&](int64_t len) {
        store.emplace_back((size_t)(std::max<int64_t>(len, 1) * S), 0.0);
        return store.back().data();
    };
    store.reserve(64);
    impc::DevWork w{};
    w.S = S;
    double *Px_ = alloc(nP), *q_ = alloc(n), *Ax_ = alloc(nA), *l_ = alloc(m), *u_ = alloc(m);
    double *xws_ = alloc(n), *yws_ = alloc(m);
    auto inter = [&](const double *src, double *dst, int64_t len) {
        for (int64_t b = 0; b < B; b++)
            for (int64_t e = 0; e < len; e++) dst[e * S + b] = src[b * len + e];
    };
    inter(Px, Px_, nP);
    inter(q, q_, n);
    inter(Ax, Ax_, nA);
    inter(l, l_, m);
    inter(u, u_, m);
    if (xws) inter(xws, xws_, n);
    if (yws) inter(yws, yws_, m);
    w.Px = Px_;
    w.q = q_;
    w.Ax = Ax_;
    w.l = l_;
    w.u = u_;
    w.xws = xws_;
    w.yws = yws_;
    w.Ps = alloc(nP);
    w.qs = alloc(n);
    w.As = alloc(nA);
    w.ls = alloc(m);
    w.us = alloc(m);
    w.D = alloc(n);
    w.Dinv = alloc(n);
    w.E = alloc(m);
    w.Einv = alloc(m);
    w.rho = alloc(m);
    w.rhoinv = alloc(m);
    w.ctype = alloc(m);
    w.scal = alloc(impc::SC_NSCAL);
    w.x = alloc(n);
    w.z = alloc(m);
    w.y = alloc(m);
    w.v = alloc(m);
    w.w = alloc(n);
    w.dx = alloc(n);
    w.dy = alloc(m);
    w.Mval = alloc(nM);
    w.Lx = alloc(nL);
    w.Dinvf = alloc(n);
    w.yf = alloc(n);
    w.tn1 = alloc(n);
    w.tm1 = alloc(m);
    w.xo = alloc(n);
    w.yo = alloc(m);
    w.info = info;
    for (int64_t b = 0; b < B; b++) {
        impc::qp_setup(d, w, st, (int)b, xws ? 1 : 0);
        impc::qp_solve(d, w, st, (int)b, b, 0);
    }
    for (int64_t b = 0; b < B; b++) {
        for (int64_t e = 0; e < n; e++) xo[b * n + e] = w.xo[e * S + b];
        for (int64_t e = 0; e < m; e++) yo[b * m + e] = w.yo[e * S + b];
    }
    return 0;
}
