// wave_emu.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Executes the one-QP-per-team kernel body (intent-mpc_amd/csrc/mpc_wave.hpp) on the CPU by
// running its NL lanes as NL threads that meet at a barrier wherever the GPU wave synchronises
// (LDS exchange, readlane broadcast, wave reductions).  This lets the structured solver be
// checked against the oracle in the GPU-less container.  Never linked into libimpc_qp.so.
#include <algorithm>
#include <barrier>
#include <utility>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <limits>
#include <vector>

#include "../../intent-mpc_amd/csrc/mpc_structure.hpp"
#include "../../intent-mpc_amd/csrc/mpc_wave.hpp"

namespace {

// the team shape (impc_qp.hip IMPC_TEAM): 256 lanes (the product: one variable per lane, or three
// for the long horizon), or 64 (EMU_NL=64: one QP per wavefront, four variables per lane)
#ifndef EMU_NL
#define EMU_NL 256
#endif
constexpr int NL = EMU_NL;
static_assert(NL == 256 || NL == 64, "emulated team shapes");

struct EmuShared {
    std::barrier<> bar{NL};
    std::barrier<> wbar[NL / 64];
    double scratch[2][NL];
    double wscratch[2][NL];  // wave-level exchanges (bcast / shfl / 8-lane sums), per-wave regions
    EmuShared() : EmuShared(std::make_index_sequence<NL / 64>{}) {}
    template <size_t... I>
    EmuShared(std::index_sequence<I...>) : wbar{((void)I, std::barrier<>{64})...} {}
};

struct EmuWave {
    int l;
    EmuShared *sh;
    int par = 0, wpar = 0;
    int lane() const { return l; }
    void sync() { sh->bar.arrive_and_wait(); }
    void lsync() { sh->bar.arrive_and_wait(); }
    void wsync() { sh->wbar[l >> 6].arrive_and_wait(); }
    double *next_buf() {
        double *b = sh->scratch[par];
        par ^= 1;
        return b;
    }
    double *next_wbuf() {
        double *b = sh->wscratch[wpar];
        wpar ^= 1;
        return b;
    }
    // wave-level operations synchronise only the caller's wavefront (as on the GPU)
    double bcast(double v, int src) {  // lane src of the caller's 64-lane wavefront
        double *b = next_wbuf();
        b[l] = v;
        wsync();
        return b[(l & ~63) + src];
    }
    double shfl(double v, int src) { return bcast(v, src); }
    static double uniform(double v) { return v; }  // every lane already holds the same value
    double sum_contig8(double v) {  // the GPU's DPP order: ((v0+v1)+(v2+v3)) + ((v4+v5)+(v6+v7))
        double *b = next_wbuf();
        b[l] = v;
        wsync();
        const double *g = b + (l & ~7);
        return ((g[0] + g[1]) + (g[2] + g[3])) + ((g[4] + g[5]) + (g[6] + g[7]));
    }
    double sum_stride8(double v) {  // same shape over lanes j, j+8, .., j+56 of the wavefront
        double *b = next_wbuf();
        b[l] = v;
        wsync();
        const double *g = b + (l & ~63) + (l & 7);
        return ((g[0] + g[8]) + (g[16] + g[24])) + ((g[32] + g[40]) + (g[48] + g[56]));
    }
    double max(double v) {
        double *b = next_buf();
        b[l] = v;
        sync();
        double r = b[0];
        for (int i = 1; i < NL; i++) r = b[i] > r ? b[i] : r;
        return r;
    }
    template <int K>
    void max_n(double (&v)[K]) {
        for (int k = 0; k < K; k++) v[k] = max(v[k]);
    }
    template <int KM, int KS>
    void max_sum_n(double (&mx)[KM], double (&sm)[KS]) {  // the GPU's: bitwise max() / sum() each
        for (int k = 0; k < KM; k++) mx[k] = max(mx[k]);
        for (int k = 0; k < KS; k++) sm[k] = sum(sm[k]);
    }
    double sum(double v) {  // per-wavefront xor butterfly (lane 0's value), waves added in order
        double *b = next_buf();
        b[l] = v;
        sync();
        double r = 0.0;
        for (int w = 0; w < NL / 64; w++) {
            double s[64];
            for (int i = 0; i < 64; i++) s[i] = b[64 * w + i];
            for (int mask = 32; mask >= 1; mask >>= 1) {
                double t[64];
                for (int i = 0; i < 64; i++) t[i] = s[i] + s[i ^ mask];
                for (int i = 0; i < 64; i++) s[i] = t[i];
            }
            r = w == 0 ? s[0] : r + s[0];
        }
        return r;
    }
};

template <int VS, int GS, int WF, bool TIER>
void run_w(const impc::WaveTables &T, const impc::WaveIO &io, const impc::DevSettings &st) {
    using LD = impc::WaveLds<NL, VS, GS>;
    // LDS starts as NaN, not zero: the GPU's LDS is uninitialised, so a read of a slot the kernel
    // has not written must show up here
    std::vector<double> lds((size_t)LD::size(T), std::numeric_limits<double>::quiet_NaN());
    EmuShared sh;
    std::vector<std::thread> th;
    for (int l = 0; l < NL; l++)
        th.emplace_back([&, l] {
            EmuWave wv{l, &sh};
            impc::WaveQP<EmuWave, NL, VS, GS, WF, TIER>::load_tables(wv, T, lds.data());
            for (int64_t b = 0; b < io.B; b++) {
                impc::WaveQP<EmuWave, NL, VS, GS, WF, TIER> qp(wv, T, io, st, lds.data());
                qp.solve(b);
            }
        });
    for (auto &t : th) t.join();
}

// the product's dispatch: a compile-time horizon instance when W matches one (impc_qp.hip
// launch_group: WSPEC, or the long shape's WSPEC2)
template <int VS, int GS>
void run(const impc::WaveTables &T, const impc::WaveIO &io, const impc::DevSettings &st) {
    constexpr int WS = impc::WaveLds<NL, VS, GS>::WSPEC, WS2 = impc::WaveLds<NL, VS, GS>::WSPEC2;
    const bool tier = T.T1r < impc::WaveLds<NL, VS, GS>::cg4(T.CG);
    if (T.W == WS)
        tier ? run_w<VS, GS, WS, true>(T, io, st) : run_w<VS, GS, WS, false>(T, io, st);
    else if (WS2 && T.W == WS2)
        tier ? run_w<VS, GS, WS2, true>(T, io, st) : run_w<VS, GS, WS2, false>(T, io, st);
    else
        tier ? run_w<VS, GS, 0, true>(T, io, st) : run_w<VS, GS, 0, false>(T, io, st);
}

// the product's shapes for the team size (impc_qp.hip kWaveVS / kWaveVSLong / kGsMax)
template <int N>
int dispatch(const impc::MpcStructure &ms, const impc::WaveTables &T, const impc::WaveIO &io,
             const impc::DevSettings &st) {
    if constexpr (N == 64) {  // one QP per wavefront: four variable slots, up to six general-row slots
        if (ms.n > 4 * N || ms.mg > 6 * N) return 2;
        const int gs = std::max(2, (ms.mg + N - 1) / N);
        if (gs == 2) run<4, 2>(T, io, st);
        else if (gs == 3) run<4, 3>(T, io, st);
        else if (gs == 4) run<4, 4>(T, io, st);
        else if (gs == 5) run<4, 5>(T, io, st);
        else run<4, 6>(T, io, st);
    } else {
        if (ms.n > 3 * N || ms.mg > 4 * N) return 2;
        const int gs = ms.mg <= 2 * N ? 2 : ms.mg <= 3 * N ? 3 : 4;
        if (ms.n <= N) {
            if (gs == 2) run<1, 2>(T, io, st);
            else if (gs == 3) run<1, 3>(T, io, st);
            else run<1, 4>(T, io, st);
        } else {
            if (gs == 2) run<3, 2>(T, io, st);
            else if (gs == 3) run<3, 3>(T, io, st);
            else run<3, 4>(T, io, st);
        }
    }
    return 0;
}

}  // namespace

extern "C" int emu_wave_solve_batch(int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                                    const int64_t *Ai, int64_t B, const double *Px, const double *q, const double *Ax,
                                    const double *l, const double *u, const impc_settings *s, const double *xws,
                                    const double *yws, double *xo, double *yo, impc_info *info) {
    impc::MpcStructure ms;
    if (!ms.analyse(n, m, Pp, Pi, Ap, Ai).empty()) return 1;
    impc::WaveTables T{ms.n, ms.m, ms.mg, ms.N, ms.W, ms.CG, ms.nnzP, ms.nnzA,
                       ms.var_orig.data(), ms.var_pdiag.data(), ms.var_boxrow.data(), ms.var_boxpos.data(),
                       ms.gen_row.data(), ms.gen_col.data(), ms.gen_pos.data(), ms.colg.data(),
                       ms.term_ptr.data(), ms.term.data(), ms.HS, ms.col_hid.data(), impc::kProdTier1};
    // the emulation takes the two-tier products layout whenever the pattern has heavy columns (the
    // product uses it where one tier would cost occupancy), so both gathers are covered on the CPU
    if (ms.HS == 0) T.T1r = impc::WaveLds<NL, 1, 2>::cg4(ms.CG);
    // EMU_SCAL_LDS=1: the scaling vectors of a shape without them in its fixed layout in LDS
    // (WaveTables::scal_lds, what the product picks where the CU has the room)
    const char *sl = std::getenv("EMU_SCAL_LDS");
    T.scal_lds = sl && sl[0] == '1' ? 1 : 0;
    // per-QP scratch of the scaling vectors (shapes without them in LDS)
    std::vector<double> zx((size_t)B * n, 0.0), zy((size_t)B * m, 0.0), scal((size_t)B * (2 * n + ms.mg), 0.0);
    impc::WaveIO io{B, Px, q, Ax, l, u, xws ? xws : zx.data(), yws ? yws : zy.data(), xws ? 1 : 0,
                    xo, yo, scal.data(), info};
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
    if (ms.CG > impc::WaveLds<NL, 1, 2>::CGM) return 2;
    return dispatch<NL>(ms, T, io, st);
}
