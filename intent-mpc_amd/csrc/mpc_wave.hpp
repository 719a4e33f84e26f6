// mpc_wave.hpp -- the structured kernel's body: one mpcPlanner QP per team of NL = 256 lanes
// (4 wavefronts, one workgroup), all per-QP state on chip, 2 teams per CU.
//
// Why: the ADMM of OSQP 0.6.2 (reference osqp.h:78, osqp_solve) runs hundreds to thousands of
// iterations per QP; each needs one solve with M = P + sigma I + A' R A plus two SpMVs.  Streaming
// that state from HBM per iteration (the generic one-QP-per-lane kernel) is latency/bandwidth
// bound.  Here a team keeps its QP's factor rows, A values, iterates and bounds in VGPRs and the
// stage-coupling blocks, exchange vectors and the general rows' products in LDS (~50-66 KB per QP
// at N = 20), and the teams of the grid pull QPs from a work queue so QPs that need 4000
// iterations do not stall the ones that need 200.
//
// Shapes (template VS = variables per lane): VS = 1 (n <= 256, the reference's default horizon
// N = 20) at 2 waves per SIMD; VS = 3 (n <= 768, N <= 59) at 1 wave per SIMD.  GS = 2..4
// general-row slots per lane.  WF = the shape's default stage count (19 / 39) as a compile-time
// constant, or 0 for any horizon.  TIER = the two-tier products layout (WaveLds) for obstacle-heavy
// patterns whose one-tier products would cost the CU its second team.
//
// Data layout (stage order v' = 13k + r, see mpc_structure.hpp):
//   var slot s of lane L  <-> v' = NL s + L   (VS slots):  x, q, P_jj, the variable's box row
//       (A value, z, y, l, u, type), row v'%13 of Ainv_k (13) and an 8-wide coupling row
//   general-row slot s    <-> g = NL s + L    (GS slots): 4 A values + columns, z, y, l, u, type
//   LDS (WaveLds): F_k (the 8x8 stage-coupling blocks), exchange vectors r / t / e / x~, team
//       reduction scratch, the int16 entry -> product-slot table, D / E and the check deltas
//       (VS = 1), the products buffer (column-slot layout)
//
// Linear solve (block LDL^T of the stage-tridiagonal M, with Ahat_k the Schur complements):
//   G_k = Bbar_k Ahat_k^{-1} (8 x 13), F_k = G_k[:, :8]
//   forward : a_0 = r_0[:8],  a_{k+1} = r_{k+1}[:8] - G_k[:, 8:] r_k[8:] - F_k a_k   (8-dim recursion)
//   middle  : e_k = Ahat_k^{-1} (a_k, r_k[8:])                                     (parallel)
//   backward: x_{N-1} = e_{N-1},  x_k = e_k - G_k^T x_{k+1}[:8]                      (8-dim recursion)
// The 8-dim recursions are the only serial part (2 x (N-1) steps of an 8x8 mat-vec); one
// wavefront of the team (rw) runs each on its 8x8 lane grid with DPP / permlane reductions while
// the others wait at the barrier -- the parallel phases (rhs gather, S1, S3, S5, update,
// products) use all 256 lanes.
//
// The kernel body is written against a team policy `WV`: lane() in [0, NL), sync() (team barrier
// with LDS visibility), bcast(v, j) (v of lane j of the CALLER's wavefront), max()/sum() over the
// team, so the same code runs on the GPU (policy GpuTeam in impc_qp.hip) and, for tests only, in an
// NL-thread CPU emulation (tests/native/wave_emu.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/impc_qp.h"
#include "admm_core.hpp"
#include "mpc_structure.hpp"

namespace impc {

#define IMPC_WF __host__ __device__ __forceinline__

// Phase-cost experiments (tools/exp.sh only): IMPC_DUP=<section id> runs that idempotent phase of
// the ADMM iteration twice; the bench's time difference is the phase's marginal cost.
// The serial recursions' wavefront at a raised issue priority (s_setprio) while it runs them: the
// co-resident team's waves share its SIMD, and the recursion is the team's critical path (round 6:
// config 3 213.9 / 214.1 -> 210.8 / 210.5 ms per launch at priority 2, 211.1 / 211.2 at 3; identical
// iterations; 0 = off)
#ifndef IMPC_PRIO
#define IMPC_PRIO 2
#endif
#if IMPC_PRIO && defined(__HIP_DEVICE_COMPILE__)
#define IMPC_PRIO_UP() __builtin_amdgcn_s_setprio(IMPC_PRIO)
#define IMPC_PRIO_DOWN() __builtin_amdgcn_s_setprio(0)
#else
#define IMPC_PRIO_UP() ((void)0)
#define IMPC_PRIO_DOWN() ((void)0)
#endif
#ifndef IMPC_DUP
#define IMPC_DUP -1
#endif
#ifndef IMPC_CHDUP
#define IMPC_CHDUP 0
#endif
// A/B switch (tools/exp.sh variants only): IMPC_CHUNK19=1 runs the default horizon's (W = 19)
// stage recursions in chunks too (the long shape's form, chunks of 6 / 6 / 6 / 1 steps), their
// operators in an LDS region past the products (the one-slot shape's F region has no tail)
#ifndef IMPC_CHUNK19
#define IMPC_CHUNK19 0
#endif
// The long shape's sweeps in five chunks on the four wavefronts (CL = 2 ceil(W/10): W = 39 -> 8, 8,
// 8, 8, 7; the product since round 5).  IMPC_CHUNK5=0 (A/B variants only): the round-4 four-chunk
// form (W = 39 -> 10, 10, 10, 9), measured 1251.6 vs 1209.6 ms per config-5 launch
#ifndef IMPC_CHUNK5
#define IMPC_CHUNK5 1
#endif
// The factorisation's latency form (round 5; IMPC_FACT2=0: the round-4 loops, A/B variants only):
// assembly codes loaded four at a time with the next stage's ranges prefetched, the Gauss-Jordan
// steps' operands read at once, the 13-term products unrolled.  The long shape's setup runs one
// team per CU, so these latencies are exposed: setup 0.440 -> 0.358 ms per N = 40 QP, config 5's
// closed loop 626 -> 608 ms per step (profiles/r05/exp_phase/README.md)
#ifndef IMPC_FACT2
#define IMPC_FACT2 1
#endif
// A/B knobs of that form (variants only): the 13-term products' unroll count (0 = full) and the
// assembly's codes per batch
#ifndef IMPC_F2U
#define IMPC_F2U 0
#endif
// The long shape's factorisation (IMPC_FACT3, on for VS = 3 only): the Schur complement E_k kept
// in the register of the lane that assembles M_k+1's matching entry (the destinations are assigned
// so that lane 8i + j computes E[i][j] and assembles M[i][j]), B_k double-buffered by stage parity,
// and the barrier between E_k and the next stage's assembly dropped.  Config 5's closed loop
// 610.9 -> 604.0 ms; on the default horizon it measured 214.3 -> 215.2 ms, so that shape keeps the
// barrier (profiles/r05/exp_phase/README.md)
#ifndef IMPC_FACT3
#define IMPC_FACT3 1
#endif
#define IMPC_PRAGMA_(x) _Pragma(#x)
#define IMPC_PRAGMA(x) IMPC_PRAGMA_(x)
#ifndef IMPC_F2B
#define IMPC_F2B 4
#endif
#define IMPC_REP(X) for (int rep_ = 0; rep_ < (IMPC_DUP == (X) ? 2 : 1); rep_++)
// Branch counters of the CPU emulation's instrumented builds (tools only; nothing in the product)
#ifndef IMPC_COUNT
#define IMPC_COUNT(X) ((void)0)
#endif

// Variants measured slower and removed in round 4 (their numbers stay in profiles/r0*/exp/README.md,
// their code in git history): the twisted two-ended elimination, pair-blocked and chunked stage
// recursions, folded recursion subtractions, wave priorities, LDS-only barriers, register-held pair
// captures, split dot-product chains, opaque phase bases, delta-less update instances, per-step
// history / store captures, (c, S)-carried sweeps, off-chip scaling vectors, Cholesky / 1x1-pivot
// stage inverses.  What is left is the measured-best form of each phase.

// Scheduling hint for the parallel phases' LDS reads: under the kernel's register pressure the
// machine scheduler otherwise issues them one ds_read2 at a time, each followed by its own
// lgkmcnt wait (S3 = 7 serialised LDS round trips); this asks for the phase's reads first, then
// its arithmetic, so the round trips overlap.
#if defined(__HIP_DEVICE_COMPILE__)
#define IMPC_LOADS_FIRST(NR, NV)                            \
    do {                                                    \
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0); \
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0); \
    } while (0)
#else
#define IMPC_LOADS_FIRST(NR, NV) ((void)0)
#endif

struct WaveTables {
    int32_t n, m, mg, N, W, CG, nnzP, nnzA;
    const int32_t *var_orig, *var_pdiag, *var_boxrow, *var_boxpos;
    const int32_t *gen_row, *gen_col, *gen_pos, *colg, *term_ptr, *term;
    int32_t HS;               // heavy columns (second products tier), MpcStructure::HS; 0: one tier
    const int32_t *col_hid;   // [n] heavy-column index or -1 (stage order)
    int32_t T1r;              // first-tier rows: cg4(CG) (one tier) or kProdTier1 (two tiers)
    // the scaling vectors D, E of a shape without them in its fixed LDS layout (WaveLds::ONCHIP
    // false): 1 = in LDS after the products region when the CU's LDS has the room (the batch
    // setup decides), 0 = in the per-QP HBM scratch (WaveIO::scal).  (In the struct's padding.)
    int32_t scal_lds;
};

struct WaveIO {
    int64_t B;
    const double *Px, *q, *Ax, *l, *u, *xws, *yws;  // QP-major inputs
    int32_t has_ws;    // 0: none, 1: x and y, 2: x with y = 0 (yws not read)
    double *xo, *yo;   // QP-major outputs (unscaled)
    double *scal;      // per-QP scratch [B][n + n + mg]: D, E(box), E(general)
    impc_info *info;
    unsigned long long *sec = nullptr;  // section-profiling build only: cycle sums [kSecCount]
    unsigned long long *qpt = nullptr;  // profiling: per-QP (start, end) device clock [B][2]
    // shared-structure values (impc_batch_set_values_shared): Px / Ax above are one copy each,
    // A entry p is Ax_var[b][vmap[p]] when vmap[p] >= 0
    int32_t shared = 0;
    int64_t nvar = 0;
    const int32_t *vmap = nullptr;
    const double *Ax_var = nullptr;
    // persistent workspace (impc_batch_set_persistent, OSQP's workspace between solves): per QP
    // [kPersistHdr + 3 n + 2 mg]: cost-scaling factors of the Ruiz passes, rho, then the scaled
    // iterates x, z (box), y (box), z (general), y (general).  resume = 2 (osqp_update_P / _A: new
    // matrix values): Ruiz scaling afresh on the new data, the stored rho and scaled iterates kept, as
    // OSQP 0.6.2 unscales, rescales and refactors but keeps work->x, z, y.  resume = 1: scale with the stored
    // factors (the same D, E, c and scaled P, A as the first setup), start from the stored rho and
    // iterates, and -- when q_updated -- scale q as osqp_update_lin_cost does ((D q) c).
    double *persist = nullptr;
    int32_t resume = 0, q_updated = 0;
    // per-QP time limits [B] (impc_batch_set_time_limits: each solveTraj call sets its own), or
    // nullptr for the settings' time_limit
    const double *tlim = nullptr;
    // resume = 2 with q updated after the matrix update: the q the workspace held when P / A
    // changed [B][n].  OSQP's scale_data after osqp_update_P / _A normalises the cost with that q;
    // the new q (io.q) is then scaled as osqp_update_lin_cost does, (D q) c
    const double *q_scale = nullptr;
};

constexpr int kPersistHdr = 24;      // ct[0 .. kPersistMaxScaling), rho at kPersistHdr - 1
constexpr int kPersistMaxScaling = 20;
IMPC_HD int64_t persist_stride(int n, int mg) { return kPersistHdr + 3 * (int64_t)n + 2 * (int64_t)mg; }

// Section profiling (profiling build of the library only, -DIMPC_SECTION_PROF): lane 0 of each
// team accumulates s_memtime deltas per section; IMPC_SEC(X) closes section X.
enum {
    kSecSetup, kSecFactor, kSecWarm, kSecRhs, kSecS1, kSecFwd, kSecS3, kSecBwd, kSecS5, kSecUpdate, kSecProducts,
    kSecChecks, kSecOutput, kSecFAsm, kSecFDense, kSecIters = 15, kSecCount = 16
};
// The clock is the 100 MHz s_memrealtime counter (the one the time-limit path reads; a
// SHADER_CYCLES s_getreg reads 0 on gfx950, and s_memtime perturbed the LDS wait counts of this
// kernel's instrumented build).  Units: 10 ns ticks.
#if defined(IMPC_SECTION_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define IMPC_SEC_CLOCK() ((uint64_t)__builtin_amdgcn_s_memrealtime())
#define IMPC_SEC(X)                             \
    do {                                        \
        uint64_t t_ = IMPC_SEC_CLOCK();         \
        sec_acc[X] += t_ - sec_t0;              \
        sec_t0 = t_;                            \
    } while (0)
#define IMPC_SEC_START() (sec_t0 = IMPC_SEC_CLOCK())
#else
#define IMPC_SEC(X) ((void)0)
#define IMPC_SEC_START() ((void)0)
#endif

// team reduction scratch (WaveLds RED_OFF): values x wavefronts of one team reduction
constexpr int kRedLen = 128;

// LDS doubles per wave for (VS, GS)
template <int NL, int VS, int GS>
struct WaveLds {
    static constexpr int NMAX = NL * VS;
    static constexpr int WMAX = (NMAX + 5) / 13 - 1;       // max control stages
    // stage count whose recursions are fully unrolled (the reference's default horizon N = 20
    // for the one-variable-per-lane shape, N = 40 for the long-horizon shape)
    static constexpr int WSPEC = NMAX <= 256 ? 19 : 39;
    // a second compile-time horizon of the long shape: the reference's live planner, N = 30
    // (autonomous_flight planner_param.yaml:25, mpc_interactive mpc_param.yaml:1); 0 = none
    static constexpr int WSPEC2 = NMAX <= 256 ? 0 : 29;
    // exchange vector length: zero tail past NMAX, and room for the factorisation scratch
    // (the sweeps' two-steps-ahead prefetches read at most 13 (W + 4) + 8 past the start), and
    // room for the factorisation's dense stage scratch (FA .. DIAGX below)
    static constexpr int NP = (NMAX + 48 > (779 + NMAX + 3) / 4) ? NMAX + 48 : (779 + NMAX + 3) / 4;
    static constexpr int F_OFF = 0;                         // [WMAX][64]
    static constexpr int R_OFF = F_OFF + WMAX * 64;         // rbuf
    static constexpr int T_OFF = R_OFF + NP;                // tbuf
    static constexpr int E_OFF = T_OFF + NP;                // ebuf
    static constexpr int X_OFF = E_OFF + NP;                // xbuf
    static constexpr int RED_OFF = X_OFF + NP;              // team reduction scratch [kRedLen]
    static constexpr int JUNK_OFF = RED_OFF + kRedLen;      // per-lane discard slots [NL]
    static constexpr int GSLOT_OFF = JUNK_OFF + NL;         // int16 [4 NL GS]: general entry -> product slot
    // One-variable-per-lane shape: the Ruiz scaling vectors D, E and the ADMM deltas of the
    // termination checks live here (the long-horizon shape keeps them in HBM / registers: its LDS
    // is full).  Layout of each: [var slots NMAX][box rows NMAX][general slots NL GS].
    static constexpr bool ONCHIP = VS == 1;
    static constexpr int VEC_N = 2 * NMAX + NL * GS;
    static constexpr int SCL_OFF = GSLOT_OFF + NL * GS;           // D, E (scaling)
    static constexpr int DLT_OFF = SCL_OFF + (ONCHIP ? VEC_N : 0);  // dx, dy (check iterations)
    static constexpr int P_OFF = DLT_OFF + (ONCHIP ? VEC_N : 0);  // products, column-slot layout (size below)
    static constexpr int CGM = 24;                          // max general entries per column
    // products region: entry t < T1r of column v at t * stride(n) + v (stride = n rounded up to
    // 64, plus a pad), so a column's gather is independent, conflict-free reads.  When that one
    // tier (T1r = CG4 rows of all n columns) would cost occupancy, a second tier holds the rest:
    // T1r = 4 and entry t >= 4 of a heavy column (index h = col_hid) at
    // 4 stride(n) + (t - 4)(HS + 1) + h -- only the positions and slack of a stage carry one
    // product per obstacle row, so the second tier is (CG4 - 4) rows of the HS heavy columns
    // instead of CG4 rows of all n (K = 21: 21 KB instead of 49 KB).  It doubles as the
    // factorisation's (4g + e) scratch and general-row rho.  Sized from the pattern at run time,
    // followed by 8 discard slots (index p_size).
    static constexpr int T1 = kProdTier1;
    static IMPC_WF int cg4(int CG) { return (CG + 3) & ~3; }
    // +PAD: the obstacle rows of one stage write their products to the same column in different
    // entry slots; a stride that is not a multiple of 16 doubles puts those ds_write_b64 (bank =
    // dword mod 32, 16-lane groups) on distinct banks.  Reads stay lane-contiguous.
    static constexpr IMPC_WF int stride(int n) { return ((n + 63) & ~63) + 1; }
    // the factorisation uses it as (4g + e) scratch followed by the general rows' rho (RHOG_P)
    static IMPC_WF int hsp(int HS) { return HS + 1; }  // second-tier row length
    static IMPC_WF int p_size(int CG, int n, int HS, int mg, int T1r) {
        const int c = T1r * stride(n) + (cg4(CG) > T1r ? (cg4(CG) - T1r) * hsp(HS) : 0), f = 5 * mg;
        return c > f ? c : f;
    }
    static IMPC_WF int p_size(const WaveTables &T) { return p_size(T.CG, T.n, T.HS, T.mg, T.T1r); }
    // the chunk operators' region of the one-slot shape (IMPC_CHUNK19), after the products
    static constexpr int CHX = (VS == 1 && IMPC_CHUNK19) ? 448 : 0;
    static IMPC_WF int ch_off(const WaveTables &T) { return P_OFF + p_size(T) + 8; }
    // D, E in LDS for a shape without them in the fixed layout (WaveTables::scal_lds)
    static IMPC_WF int scl2_off(const WaveTables &T) { return P_OFF + p_size(T) + 8 + CHX; }
    static IMPC_WF int size(const WaveTables &T) {
        return scl2_off(T) + (!ONCHIP && T.scal_lds ? 2 * T.n + T.mg : 0);
    }
    // factorisation aliases (inside R..X region and the products buffer)
    static constexpr int FA = R_OFF, FL = FA + 169, FI = FL + 169, FB = FI + 169, FG = FB + 104, FE = FG + 104,
                         DIAGX = FE + 64;
    // general rows' rho during the factorisation: products region + 4 mg
    static_assert(DIAGX + NMAX <= RED_OFF, "factorisation scratch does not fit");
    // the coupling block of odd stages (IMPC_FACT3: B_k double-buffered by stage parity)
    static constexpr int FB2 = DIAGX + NMAX;
    static_assert(VS != 3 || FB2 + 104 <= RED_OFF, "factorisation scratch does not fit");
};

// the status register's mark of a failed refactorisation inside the iteration loop (never a
// reported status: the exit path writes UNSOLVED)
constexpr int64_t kRefailMark = -1000;

struct WaveRho {
    double rho, r_eq, r_ineq, r_loose, i_eq, i_ineq, i_loose;
    IMPC_WF void set(double r) {
        rho = r;
        r_ineq = r;
        r_eq = kRhoEqOverIneq * r;
        r_loose = kRhoMin;
        i_ineq = 1. / r_ineq;
        i_eq = 1. / r_eq;
        i_loose = 1. / r_loose;
    }
    // Value selection by arithmetic (t in {-1, 0, 1}): a ternary between fields would become a
    // select of member addresses and keep the whole per-QP object out of registers.
    IMPC_WF double of(int t) const {
        double e = t > 0 ? 1.0 : 0.0, i = t == 0 ? 1.0 : 0.0, l = t < 0 ? 1.0 : 0.0;
        return (e * r_eq + i * r_ineq) + l * r_loose;
    }
    IMPC_WF double inv(int t) const {
        double e = t > 0 ? 1.0 : 0.0, i = t == 0 ? 1.0 : 0.0, l = t < 0 ? 1.0 : 0.0;
        return (e * i_eq + i * i_ineq) + l * i_loose;
    }
};

IMPC_WF int row_type(double l, double u) {  // set_rho_vec (auxil.h:34)
    if ((l < -kInf * kMinScaling) && (u > kInf * kMinScaling)) return -1;
    if (u - l < kRhoTol) return 1;
    return 0;
}

// WF: the stage count W fixed at compile time (LD::WSPEC, the default horizon: every stage loop
// and LDS offset becomes a constant and no runtime-W code path shares the kernel's registers), or 0
// for any W read from the tables.
// TIER: the batch uses the two-tier products layout (WaveLds, T1r = kProdTier1); a one-tier
// batch (T1r = CG4) runs the TIER = false instance, whose gathers are the plain CG4-row loops.
template <class WV, int NL, int VS, int GS, int WF = 0, bool TIER = false>
struct WaveQP {
    using LD = WaveLds<NL, VS, GS>;
    static_assert(WF == 0 || WF == LD::WSPEC || WF == LD::WSPEC2, "WF is 0 or one of the shape's compiled horizons");
    IMPC_WF int Wst() const { return WF ? WF : T.W; }
    WV &wv;
    const WaveTables &T;
    const WaveIO &io;
    const DevSettings &st;
    double *lds;
    int L;
    // ---- variable slots
    double x[VS], q[VS], pd[VS], ab[VS], zb[VS], yb[VS], lb[VS], ub[VS], dxv_[VS], dyb_[VS];
    double ainv[VS][13], cp[VS][8];
    int bt[VS], vs_[VS], vr_[VS], hid_[VS];
    bool vok[VS];
    // ---- general-row slots
    double a[GS][4], z[GS], y[GS], lg[GS], ug[GS], dyg_[GS];
    int gc[GS][4], gt[GS];
    bool gok[GS];
    WaveRho R;
    double c = 1.0, cinv = 1.0;
    int rw = 0;  // the wavefront that runs the stage recursions for this QP
    // settings / pattern scalars the ADMM iteration reads, held in registers (a grouped launch's
    // tables and settings live in global memory: read in the loop, each is a scalar-memory round
    // trip after every barrier)
    double sig_, alp_;
    int c4_, sd_;
#if defined(IMPC_SECTION_PROF) && defined(__HIP_DEVICE_COMPILE__)
    uint64_t sec_t0 = 0, sec_acc[kSecCount] = {};
#endif

    IMPC_WF WaveQP(WV &w, const WaveTables &t, const WaveIO &i, const DevSettings &s, double *l)
        : wv(w), T(t), io(i), st(s), lds(l), L(w.lane()), sig_(s.sigma), alp_(s.alpha), c4_(LD::cg4(t.CG)),
          sd_(LD::stride(t.n)) {}

    // the lane index, opaque to the optimiser: per-lane LDS addresses derived from it are formed
    // where they are used instead of being hoisted out of the ADMM loop (dozens of loop-invariant
    // address registers otherwise spill and come back as scratch loads inside the recursions)
    IMPC_WF int lane_o() const {
        int l = L;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(l));
#endif
        return l;
    }

    // a per-lane value the optimiser must treat as freshly computed (see lane_o)
    IMPC_WF static void opaque(int &v) {
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(v));
#else
        (void)v;
#endif
    }

    // team-uniform: R stays in scalar registers, and each row's rho / 1/rho is selected from it
    // by the row type where used instead of occupying 4 VGPRs per row slot
    IMPC_WF void set_rho(double r) { R.set(wv.uniform(r)); }
    IMPC_WF double rhob(int s) const { return R.of(bt[s]); }
    IMPC_WF double rhoib(int s) const { return R.inv(bt[s]); }
    IMPC_WF double rhog_(int s) const { return R.of(gt[s]); }
    IMPC_WF double rhoig_(int s) const { return R.inv(gt[s]); }

    // ADMM deltas of the last iteration (termination checks only): LDS or registers
    IMPC_WF double &dxv(int s) { if constexpr (LD::ONCHIP) return lds[LD::DLT_OFF + NL * s + L]; else return dxv_[s]; }
    IMPC_WF double &dyb(int s) {
        if constexpr (LD::ONCHIP) return lds[LD::DLT_OFF + LD::NMAX + NL * s + L]; else return dyb_[s];
    }
    IMPC_WF double &dyg(int s) {
        if constexpr (LD::ONCHIP) return lds[LD::DLT_OFF + 2 * LD::NMAX + NL * s + L]; else return dyg_[s];
    }
    // scaling vectors D, E (set by scale(), read at warm start, checks and unscaling): layout
    // [D n][E box n][E general mg], in LDS or in the per-QP HBM scratch
    IMPC_WF double *scal(int64_t b) {
        if constexpr (LD::ONCHIP) return lds + LD::SCL_OFF;
        else return T.scal_lds ? lds + LD::scl2_off(T) : io.scal + b * (int64_t)(2 * T.n + T.mg);
    }

    IMPC_WF double *F() { return lds + LD::F_OFF; }
    IMPC_WF double *rbuf() { return lds + LD::R_OFF; }
    IMPC_WF double *tbuf() { return lds + LD::T_OFF; }
    IMPC_WF double *ebuf() { return lds + LD::E_OFF; }
    IMPC_WF double *xbuf() { return lds + LD::X_OFF; }
    IMPC_WF double *pbuf() { return lds + LD::P_OFF; }

    // Chunked stage recursions of the long horizon (the compile-time W = 39 and W = 29 instances of
    // the three-slot shape).  That shape runs one team per CU, so the three wavefronts that wait out
    // a serial sweep leave their SIMDs idle.  Each W-step sweep runs as four chunks, CL = 2 ceil(W/8)
    // steps each and W - 3 CL in the last (W = 39: 10, 10, 10, 9; W = 29: 8, 8, 8, 5), one per
    // wavefront, in two rounds: wave 0 runs the first chunk from the true start while waves 1 and 2
    // run theirs from zero for the chunk-end values only; after a barrier each of waves 1..3 forms
    // its chunk's true start from those ends and the chunk operators (products of the chunk's -F_k,
    // or -F_k^T backward, built with the factorisation: a_{o+CL} = a^_{o+CL} + P a_o) in one 8-lane
    // reduction and runs its chunk again.  Dependent chain per sweep: W steps -> 2 CL steps and one
    // reduction.  Operators and ends live in the F region's tail (blocks >= W + 3, never read).
    // CL is even, so every chunk starts on an even stage (the sweeps' index parity).
    //
    // Five chunks (NCH = 5, the long shape's form since round 5; four: IMPC_CHUNK5=0 and the
    // default horizon's IMPC_CHUNK19 variant): CL = 2 ceil(W/10) and W - 4 CL in the
    // last (W = 39: 8, 8, 8, 8, 7; W = 29: 6, 6, 6, 6, 5).  Round 1: wave 0 the first chunk from the
    // true start, waves 1..3 chunks 1..3 from zero; round 2: waves 1..3 chunks 1..3 again from their
    // true starts and wave 0 the fifth, whose start a_4CL = a^_4CL + P3 a^_3CL + P3P2 a^_2CL +
    // P3P2P1 a_CL is still one 8-lane reduction.  Chain per sweep: 2 CL steps and one reduction
    // (W = 39: 16 instead of 20).
    static constexpr bool F3 = IMPC_FACT2 && IMPC_FACT3 && VS == 3;
    static constexpr int NCH = (WF > 0 && VS == 3 && IMPC_CHUNK5) ? 5 : 4;
    static constexpr bool CHUNK = WF > 0 && NL == 256 && (VS == 3 || (VS == 1 && IMPC_CHUNK19 != 0));
    static constexpr int CL = WF > 0 ? (NCH == 5 ? 2 * ((WF + 9) / 10) : 2 * ((WF + 7) / 8)) : 2;
    static constexpr int CLAST = WF - (NCH - 1) * CL;
    static constexpr int CH_OFF = LD::F_OFF + 64 * (WF + 3);
    enum { kChFP1 = 0, kChFP2 = 64, kChFP21 = 128, kChBT1 = 192, kChBT2 = 256, kChBT21 = 320 };
    // five chunks: forward P1 P2 P3 P2P1 P3P2 P3P2P1, then the same backward (+kCh5B), then the ends
    enum { kCh5P1 = 0, kCh5P2 = 64, kCh5P3 = 128, kCh5P21 = 192, kCh5P32 = 256, kCh5P321 = 320, kCh5B = 384 };
    static constexpr int kChEnd = NCH == 5 ? 768 : 384;
    static constexpr int kChEnds = NCH == 5 ? 24 : 16;  // chunk-end values per direction
    static_assert(!CHUNK || VS == 1 || CH_OFF + kChEnd + 2 * kChEnds <= LD::R_OFF,
                  "chunk operators do not fit the F region");
    static_assert(!CHUNK || VS != 1 || LD::CHX >= kChEnd + 2 * kChEnds, "chunk operator region");
    IMPC_WF double *chbuf() const { return lds + (VS == 1 ? LD::ch_off(T) : CH_OFF); }
    static_assert(!CHUNK || (CLAST >= 1 && CLAST <= CL), "chunk lengths");

    // zero the exchange vectors (their tails are the zero slots read by padded entries)
    IMPC_WF void clear_exchange() {
        for (int i = L; i < 4 * LD::NP; i += NL) lds[LD::R_OFF + i] = 0.0;
        wv.sync();
    }

    // ------------------------------------------------------------------ load + scaling
    IMPC_WF void load(int64_t b) {
        const int n = T.n, m = T.m;
        const int64_t bn = b * n, bm = b * m, bP = io.shared ? 0 : b * T.nnzP, bA = io.shared ? 0 : b * T.nnzA;
        // A value at CSC position p of this QP (shared-structure batches: the per-QP override)
        auto Aval = [&](int p) -> double {
            if (io.shared) {
                const int32_t v = io.vmap[p];
                return v >= 0 ? io.Ax_var[b * io.nvar + v] : io.Ax[p];
            }
            return io.Ax[bA + p];
        };
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            int v = NL * s + L;
            vok[s] = v < n;
            vs_[s] = vok[s] ? v / 13 : 0;
            vr_[s] = vok[s] ? v % 13 : 0;
            hid_[s] = TIER && vok[s] ? T.col_hid[v] : -1;  // second products tier (TIER batches)
            x[s] = q[s] = pd[s] = ab[s] = zb[s] = yb[s] = lb[s] = ub[s] = dxv_[s] = dyb_[s] = 0.0;
            bt[s] = 0;
            // the branch-free phases read a slot's factor rows whether or not it holds a variable
            _Pragma("unroll") for (int cc = 0; cc < 13; cc++) ainv[s][cc] = 0.0;
            _Pragma("unroll") for (int cc = 0; cc < 8; cc++) cp[s][cc] = 0.0;
            if (vok[s]) {
                int ov = T.var_orig[v];
                q[s] = (io.q_scale ? io.q_scale : io.q)[bn + ov];
                int pp = T.var_pdiag[v];
                pd[s] = pp >= 0 ? io.Px[bP + pp] : 0.0;
                ab[s] = Aval(T.var_boxpos[v]);
                int br = T.var_boxrow[v];
                lb[s] = dmin(dmax(io.l[bm + br], -kInf), kInf);
                ub[s] = dmin(dmax(io.u[bm + br], -kInf), kInf);
            }
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            int g = NL * s + L;
            gok[s] = g < T.mg;
            z[s] = y[s] = lg[s] = ug[s] = dyg_[s] = 0.0;
            gt[s] = 0;
            const int16_t *gs = (const int16_t *)(lds + LD::GSLOT_OFF);
            const int pz = LD::p_size(T);
            _Pragma("unroll") for (int e = 0; e < 4; e++) {
                a[s][e] = 0.0;
                gc[s][e] = (pz << 16) | LD::NMAX;  // discard slot / zero tail of the x exchange
            }
            if (gok[s]) {
                _Pragma("unroll") for (int e = 0; e < 4; e++) {
                    int col = T.gen_col[4 * g + e], pos = T.gen_pos[4 * g + e];
                    if (col >= 0) {
                        gc[s][e] = ((int)gs[4 * g + e] << 16) | col;
                        a[s][e] = Aval(pos);
                    }
                }
                int row = T.gen_row[g];
                lg[s] = dmin(dmax(io.l[bm + row], -kInf), kInf);
                ug[s] = dmin(dmax(io.u[bm + row], -kInf), kInf);
            }
        }
        if constexpr (LD::ONCHIP) {  // deltas read by a check before any ADMM step (max_iter = 0)
            _Pragma("unroll") for (int s = 0; s < VS; s++) dxv(s) = dyb(s) = 0.0;
            _Pragma("unroll") for (int s = 0; s < GS; s++) dyg(s) = 0.0;
        }
    }

    // Per-workgroup tables (once per launch): the product slot of every general-row entry
    // (mpc_structure colg inverted into the column-slot layout, int16 in LDS; padded entries get
    // the discard slot), and a zeroed products region (slots no entry maps to must read 0).
    static IMPC_WF void load_tables(WV &w, const WaveTables &T, double *lds) {
        int16_t *gs = (int16_t *)(lds + LD::GSLOT_OFF);
        const int pz = LD::p_size(T);
        for (int e = w.lane(); e < 4 * NL * GS; e += NL) gs[e] = (int16_t)pz;
        double *pb = lds + LD::P_OFF;
        for (int e = w.lane(); e < pz + 8; e += NL) pb[e] = 0.0;
        w.sync();
        for (int e = w.lane(); e < T.n * T.CG; e += NL) {
            const int v = e / T.CG, t = e % T.CG, id = T.colg[e];
            if (id >= 0)
                gs[id] = (int16_t)(t < T.T1r ? t * LD::stride(T.n) + v
                                             : T.T1r * LD::stride(T.n) + (t - T.T1r) * LD::hsp(T.HS) + T.col_hid[v]);
        }
        w.sync();
    }

    IMPC_WF void zero_products() {
        double *pb = pbuf();
        const int cnt = LD::p_size(T) + 8;
        for (int i = L; i < cnt; i += NL) pb[i] = 0.0;
        wv.sync();
    }

    // column index / product slot of general entry e of slot s (packed: slot << 16 | column)
    IMPC_WF int gcol(int s, int e) const { return gc[s][e] & 0xFFFF; }
    IMPC_WF int gdst(int s, int e) const { return gc[s][e] >> 16; }

    // col_gather's loop for C4 = 4 NG: s = 0 + group 0 + group 1 + ..., each group (p0+p1)+(p2+p3)
    template <int NG>
    IMPC_WF static double gather_n(const double *pb, int sd) {
        double p[4 * NG];
        _Pragma("unroll") for (int t = 0; t < 4 * NG; t++) p[t] = pb[t * sd];
        double s = 0.0;
        _Pragma("unroll") for (int g = 0; g < NG; g++) s += (p[4 * g] + p[4 * g + 1]) + (p[4 * g + 2] + p[4 * g + 3]);
        return s;
    }

    // gather sum over the general entries of column v (column-slot layout, independent reads;
    // the sums add groups of four in entry order).  TIER: the first T1 rows, then -- for a heavy
    // column, h = its second-tier index (hid_, -1 for a light column) -- the second tier
    IMPC_WF double col_gather(int v, int h) {
        const double *pb = pbuf() + v;
        // (a compile-time horizon's products stride is a constant, n = 13 (WF + 1) - 5, so the
        // gather's reads take immediate offsets instead of per-read address arithmetic)
        const int C4 = c4_, sd = WF ? LD::stride(13 * (WF + 1) - 5) : sd_;
        double s = 0.0;
        if constexpr (!TIER) {
            (void)h;
            // the same sum, every read of the column issued before the first add (C4 is uniform)
            switch (C4) {
                case 4: return gather_n<1>(pb, sd);
                case 8: return gather_n<2>(pb, sd);
                case 12: return gather_n<3>(pb, sd);
                case 16: return gather_n<4>(pb, sd);
                case 20: return gather_n<5>(pb, sd);
                default: break;
            }
            for (int t = 0; t < C4; t += 4) {
                const double p0 = pb[t * sd], p1 = pb[(t + 1) * sd], p2 = pb[(t + 2) * sd], p3 = pb[(t + 3) * sd];
                s += (p0 + p1) + (p2 + p3);
            }
        } else {
            static_assert(LD::T1 == 4, "one first-tier group");
            s += (pb[0] + pb[sd]) + (pb[2 * sd] + pb[3 * sd]);
            if (h >= 0) {
                const int hp = LD::hsp(T.HS);
                const double *q = pbuf() + LD::T1 * sd + h;
                for (int t = 0; t < C4 - LD::T1; t += 4)
                    s += (q[t * hp] + q[(t + 1) * hp]) + (q[(t + 2) * hp] + q[(t + 3) * hp]);
            }
        }
        return s;
    }
    IMPC_WF double col_gather_max(int v, int h) {
        const double *pb = pbuf() + v;
        const int C4 = c4_, sd = sd_;
        double s = 0.0;
        for (int t = 0; t < (TIER ? LD::T1 : C4); t++) s = dmax(pb[t * sd], s);
        if (TIER && h >= 0) {
            const int hp = LD::hsp(T.HS);
            const double *q = pbuf() + LD::T1 * sd + h;
            for (int t = 0; t < C4 - LD::T1; t++) s = dmax(q[t * hp], s);
        }
        return s;
    }

    // scale_data (scaling.h:21): Ruiz equilibration + cost scaling; D, E kept in registers here,
    // written to the per-QP scratch at the end.
    // ps: the QP's persistent record (or null): the Ruiz passes' cost factors are stored there,
    // or replayed from it when resuming
    IMPC_WF void scale(int64_t b, double D[VS], double Eb[VS], double Eg[GS], double *ps) {
        const int n = T.n;
        _Pragma("unroll") for (int s = 0; s < VS; s++) D[s] = Eb[s] = 1.0;
        _Pragma("unroll") for (int s = 0; s < GS; s++) Eg[s] = 1.0;
        c = 1.0;
        double *pb = pbuf(), *xb = xbuf();
#if IMPC_FACT2
        // |A| entries of the general rows -> products buffer: pass 0's here, each later pass's at
        // the end of the pass before (after its scaling), ordered by that pass's team reduction
        if (st.scaling > 0) {
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (gok[s])
                    _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = fabs(a[s][e]);
            }
            wv.sync();
        }
#endif
        for (int it = 0; it < st.scaling; it++) {
#if !IMPC_FACT2
            // |A| entries of general rows -> products buffer
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (gok[s])
                    _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = fabs(a[s][e]);
            }
            wv.sync();
#endif
            double Dt[VS], Etb[VS], Etg[GS];
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                // colnorm_sym(P) (diagonal), max with colnorm(A) = max(box, general entries)
                double d = fabs(pd[s]);
                double an = dmax(fabs(ab[s]), 0.0);
                if (vok[s]) an = dmax(col_gather_max(NL * s + L, hid_[s]), an);
                d = dmax(d, an);
                d = d < kMinScaling ? 1.0 : d;
                d = d > kMaxScaling ? kMaxScaling : d;
                Dt[s] = 1.0 / sqrt(d);
                double e = fabs(ab[s]);
                e = e < kMinScaling ? 1.0 : e;
                e = e > kMaxScaling ? kMaxScaling : e;
                Etb[s] = 1.0 / sqrt(e);
            }
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                double e = 0.0;
                _Pragma("unroll") for (int k = 0; k < 4; k++) e = dmax(fabs(a[s][k]), e);
                e = e < kMinScaling ? 1.0 : e;
                e = e > kMaxScaling ? kMaxScaling : e;
                Etg[s] = 1.0 / sqrt(e);
            }
            // D_temp of every column to LDS for the general rows
            _Pragma("unroll") for (int s = 0; s < VS; s++)
                if (vok[s]) xb[NL * s + L] = Dt[s];
            wv.sync();
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                pd[s] = (pd[s] * Dt[s]) * Dt[s];
                ab[s] = (ab[s] * Etb[s]) * Dt[s];
                q[s] = Dt[s] * q[s];
                D[s] = D[s] * Dt[s];
                Eb[s] = Eb[s] * Etb[s];
            }
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                _Pragma("unroll") for (int e = 0; e < 4; e++) a[s][e] = (a[s][e] * Etg[s]) * xb[gcol(s, e)];
                Eg[s] = Eg[s] * Etg[s];
            }
#if IMPC_FACT2
            // the next pass's |A| (every read of this pass's came before the D_temp barrier)
            if (it + 1 < st.scaling)
                _Pragma("unroll") for (int s = 0; s < GS; s++) {
                    if (gok[s])
                        _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = fabs(a[s][e]);
                }
#endif
            // cost normalisation
            double psum = 0.0, qn = 0.0;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (vok[s]) {
                    psum += fabs(pd[s]);
                    qn = dmax(fabs(q[s]), qn);
                }
            }
#if IMPC_FACT2
            // both cost norms in one team reduction (the same combine orders as sum / max)
            double mx1[1] = {qn}, sm1[1] = {psum};
            wv.max_sum_n(mx1, sm1);
            double ct = sm1[0] / (double)n;
            qn = mx1[0];
#else
            double ct = wv.sum(psum) / (double)n;
            qn = wv.max(qn);
#endif
            qn = qn < kMinScaling ? 1.0 : qn;
            qn = qn > kMaxScaling ? kMaxScaling : qn;
            ct = dmax(ct, qn);
            ct = ct < kMinScaling ? 1.0 : ct;
            ct = ct > kMaxScaling ? kMaxScaling : ct;
            ct = 1. / ct;
            if (ps) {
                if (io.resume == 1)  // replay; resume 2 (new P / A: osqp_update_P / _A) scales afresh
                    ct = ps[it];
                else if (L == 0)
                    ps[it] = ct;
            }
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                pd[s] *= ct;
                q[s] *= ct;
            }
            c *= ct;
#if !IMPC_FACT2
            wv.sync();  // (redundant: the team reduction's barriers already order this pass's reads
                        // of pb / xb before the next pass's writes)
#endif
        }
        c = wv.uniform(c);
        cinv = 1. / c;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            lb[s] = Eb[s] * lb[s];
            ub[s] = Eb[s] * ub[s];
            bt[s] = row_type(lb[s], ub[s]);
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            lg[s] = Eg[s] * lg[s];
            ug[s] = Eg[s] * ug[s];
            gt[s] = row_type(lg[s], ug[s]);
        }
        double *sc = scal(b);
        _Pragma("unroll") for (int s = 0; s < VS; s++)
            if (vok[s]) {
                sc[NL * s + L] = D[s];
                sc[T.n + NL * s + L] = Eb[s];
            }
        _Pragma("unroll") for (int s = 0; s < GS; s++)
            if (gok[s]) sc[2 * T.n + NL * s + L] = Eg[s];
    }

    // ------------------------------------------------------------ block factorisation
    // Returns 1 if a pivot is not positive (OSQP_NONCVX_ERROR).
    // the factorisation assembly's destination of slot r = L + NL u (0 <= r < kStageDests): the
    // identity, or (IMPC_FACT3) slots 0..63 on the 8 x 8 Schur block M[i][j] (13 i + j, lane 8 i + j),
    // the rest in order over the other 209 (M rows 0..7 columns 8..12, M rows 8..12, then B)
    IMPC_WF static int stage_dest(int r) {
        if constexpr (F3) {
            if (r < 64) return 13 * (r >> 3) + (r & 7);
            const int c = r - 64;
            return c < 40 ? 13 * (c / 5) + 8 + c % 5 : 104 + (c - 40);
        }
        return r;
    }

    IMPC_WF int factorize() {
        const int n = T.n, W = Wst(), N = W + 1;
        double *w = pbuf(), *rhog = pbuf() + 4 * T.mg, *diagx = lds + LD::DIAGX;
        double *A = lds + LD::FA, *Li = lds + LD::FL, *Ai = lds + LD::FI, *Bb = lds + LD::FB, *G = lds + LD::FG,
               *E = lds + LD::FE, *Fm = F();
        double e_reg = 0.0;  // F3: E_k-1[L >> 3][L & 7] (lanes < 64)
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            int g = NL * s + L;
            if (gok[s]) {
                _Pragma("unroll") for (int e = 0; e < 4; e++) w[4 * g + e] = a[s][e];
                rhog[g] = rhog_(s);
            }
        }
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (vok[s]) {
                double rb = rhob(s);
                diagx[NL * s + L] = (pd[s] + st.sigma) + rb * ab[s] * ab[s];
            }
        }
        wv.sync();
        int bad = 0;
#if IMPC_FACT2
        // the assembly program's range of each of this lane's destinations, one stage ahead (a
        // global load; the long shape runs one team per CU, so nothing hides its latency)
        constexpr int ND = (kStageDests + NL - 1) / NL;
        int32_t tp[ND][2];
        auto load_tp = [&](int k) {
            _Pragma("unroll") for (int u = 0; u < ND; u++) {
                const int d = stage_dest(L + NL * u);
                const bool ok = d < kStageDests && k < N;
                tp[u][0] = ok ? T.term_ptr[(int64_t)k * kStageDests + d] : 0;
                tp[u][1] = ok ? T.term_ptr[(int64_t)k * kStageDests + d + 1] : 0;
            }
        };
        load_tp(0);
#endif
        for (int k = 0; k < N; k++) {
            const int sz = k < W ? 13 : 8;
            if constexpr (F3) Bb = lds + ((k & 1) ? LD::FB2 : LD::FB);
            // assemble M_kk and Bbar_k
#if IMPC_FACT2
            int32_t tc[ND][2];
            _Pragma("unroll") for (int u = 0; u < ND; u++) tc[u][0] = tp[u][0], tc[u][1] = tp[u][1];
            load_tp(k + 1);
            _Pragma("unroll") for (int u = 0; u < ND; u++) {
                if (L + NL * u >= kStageDests) continue;
                const int d = stage_dest(L + NL * u);
#else
            for (int d = L; d < kStageDests; d += NL) {
#endif
                const bool isB = d >= 169;
                if (isB && k == W) continue;
                const int dd = isB ? d - 169 : d;
                const int r = dd / 13, cc = dd % 13;
                double val = 0.0;
                if (isB || (r < sz && cc < sz)) {
#if IMPC_FACT2
                    // the codes four at a time, their LDS operands before the products (the sum
                    // keeps its term order)
                    const int32_t t0 = tc[u][0], t1 = tc[u][1];
                    for (int32_t t = t0; t < t1; t += IMPC_F2B) {
                        int32_t cd[IMPC_F2B];
                        _Pragma("unroll") for (int v = 0; v < IMPC_F2B; v++) cd[v] = t + v < t1 ? T.term[t + v] : 0;
                        double rg[IMPC_F2B], we[IMPC_F2B], wf[IMPC_F2B];
                        _Pragma("unroll") for (int v = 0; v < IMPC_F2B; v++) {
                            const int32_t g = cd[v] >> 4, e = (cd[v] >> 2) & 3, f = cd[v] & 3;
                            rg[v] = rhog[g];
                            we[v] = w[4 * g + e];
                            wf[v] = w[4 * g + f];
                        }
                        _Pragma("unroll") for (int v = 0; v < IMPC_F2B; v++)
                            if (t + v < t1) val += rg[v] * we[v] * wf[v];
                    }
#else
                    const int32_t t0 = T.term_ptr[(int64_t)k * kStageDests + d];
                    const int32_t t1 = T.term_ptr[(int64_t)k * kStageDests + d + 1];
                    for (int32_t t = t0; t < t1; t++) {
                        int32_t code = T.term[t];
                        int32_t g = code >> 4, e = (code >> 2) & 3, f = code & 3;
                        val += rhog[g] * w[4 * g + e] * w[4 * g + f];
                    }
#endif
                    if (!isB && r == cc) val += diagx[13 * k + r];
                    if (!isB && k > 0 && r < 8 && cc < 8)  // Schur complement (F3: this lane's E)
                        val -= F3 ? e_reg : E[8 * r + cc];
                }
                if (isB)
                    Bb[dd] = val;
                else
                    A[dd] = val;
            }
            wv.sync();
            IMPC_SEC(kSecFAsm);
            // Ahat_k^{-1} by Gauss-Jordan elimination: one element per lane, the pivots in order
            // (SPD, no pivoting needed; a non-positive-definite pivot flags the factorisation as
            // failed, as a failed Cholesky did), ping-pong between two LDS buffers so every step
            // is one barrier.  The last step writes the lower triangle to both halves of Ai
            // (exactly symmetric).
            {
                double *src = A, *dst = Li;
                // two pivots per step (2x2 block pivot Q = P^-1, P = S[J][J], J = {j, j+1}):
                //   D[J][J] = Q, D[J][c] = Q S[J][c], D[i][J] = -S[i][J] Q,
                //   D[i][c] = S[i][c] - (S[i][J] Q) S[J][c]; a non-PD pivot block flags failure
                for (int j = 0; j < sz; j += 2) {
                    const bool two = j + 1 < sz, last = j + (two ? 2 : 1) >= sz;
                    // element (gi, gc) of the 13 x 13 block per lane (a team of fewer than 169 lanes
                    // takes several)
                    for (int el = L; el < 169; el += NL) {
                        const int gi = el / 13, gc = el % 13;
                        if (gi >= sz || gc >= sz) continue;
                        const int i = last && gc > gi ? gc : gi, c = last && gc > gi ? gi : gc;
                        double v;
#if IMPC_FACT2
                        // every operand read at once (one LDS round trip per step), the lane's
                        // case selected after: the same expressions as below
                        const double p00 = src[13 * j + j], p01 = src[13 * j + (two ? j + 1 : j)];
                        const double p10 = src[13 * (two ? j + 1 : j) + j], p11 = src[13 * (two ? j + 1 : j) + (two ? j + 1 : j)];
                        const double s0 = src[13 * j + c], s1 = src[13 * (two ? j + 1 : j) + c];
                        const double a0 = src[13 * i + j], a1 = src[13 * i + (two ? j + 1 : j)];
                        const double sic = src[13 * i + c];
                        if (two) {
                            const double det = p00 * p11 - p01 * p10;
                            if (!(p00 > 0.0) || !(det > 0.0)) bad = 1;
                            const double rd = 1.0 / det;
                            const double q00 = p11 * rd, q01 = -(p01 * rd), q10 = -(p10 * rd), q11 = p00 * rd;
                            const int ri = i - j, ci = c - j;
                            const bool iJ = ri == 0 || ri == 1, cJ = ci == 0 || ci == 1;
                            const double vq = ri == 0 ? (ci == 0 ? q00 : q01) : (ci == 0 ? q10 : q11);
                            const double vr = ri == 0 ? q00 * s0 + q01 * s1 : q10 * s0 + q11 * s1;
                            const double u0 = a0 * q00 + a1 * q10, u1 = a0 * q01 + a1 * q11;
                            const double vc = -(ci == 0 ? u0 : u1);
                            const double vi = sic - (u0 * s0 + u1 * s1);
                            v = iJ ? (cJ ? vq : vr) : (cJ ? vc : vi);
                        } else {
                            if (!(p00 > 0.0)) bad = 1;
                            const double r = 1.0 / p00;
                            v = i == j ? (c == j ? r : s0 * r) : (c == j ? -(a0 * r) : sic - (a0 * r) * s0);
                        }
#else
                        if (two) {
                            const double p00 = src[13 * j + j], p01 = src[13 * j + j + 1];
                            const double p10 = src[13 * (j + 1) + j], p11 = src[13 * (j + 1) + j + 1];
                            const double det = p00 * p11 - p01 * p10;
                            if (!(p00 > 0.0) || !(det > 0.0)) bad = 1;
                            const double rd = 1.0 / det;
                            const double q00 = p11 * rd, q01 = -(p01 * rd), q10 = -(p10 * rd), q11 = p00 * rd;
                            const int ri = i - j, ci = c - j;
                            const bool iJ = ri == 0 || ri == 1, cJ = ci == 0 || ci == 1;
                            if (iJ && cJ) {
                                v = ri == 0 ? (ci == 0 ? q00 : q01) : (ci == 0 ? q10 : q11);
                            } else if (iJ) {
                                const double s0 = src[13 * j + c], s1 = src[13 * (j + 1) + c];
                                v = ri == 0 ? q00 * s0 + q01 * s1 : q10 * s0 + q11 * s1;
                            } else {
                                const double a0 = src[13 * i + j], a1 = src[13 * i + j + 1];
                                const double u0 = a0 * q00 + a1 * q10, u1 = a0 * q01 + a1 * q11;
                                if (cJ)
                                    v = -(ci == 0 ? u0 : u1);
                                else
                                    v = src[13 * i + c] - (u0 * src[13 * j + c] + u1 * src[13 * (j + 1) + c]);
                            }
                        } else {
                            const double p = src[13 * j + j];
                            if (!(p > 0.0)) bad = 1;
                            const double r = 1.0 / p;
                            if (i == j && c == j)
                                v = r;
                            else if (i == j)
                                v = src[13 * j + c] * r;
                            else if (c == j)
                                v = -(src[13 * i + j] * r);
                            else
                                v = src[13 * i + c] - (src[13 * i + j] * r) * src[13 * j + c];
                        }
#endif
                        (last ? Ai : dst)[13 * gi + gc] = v;
                    }
                    wv.sync();
                    double *t = src;
                    src = dst;
                    dst = t;
                }
            }
            _Pragma("unroll") for (int s = 0; s < VS; s++)
                if (vok[s] && vs_[s] == k)
                    _Pragma("unroll") for (int cc = 0; cc < 13; cc++) ainv[s][cc] = cc < sz ? Ai[13 * vr_[s] + cc] : 0.0;
            if (k < W) {
                for (int p = L; p < 104; p += NL) {
                    int i = p / 13, cc = p % 13;
                    double s = 0.0;
#if IMPC_FACT2 && IMPC_F2U == 0
                    _Pragma("unroll")
#elif IMPC_FACT2
                    IMPC_PRAGMA(unroll IMPC_F2U)
#endif
                    for (int t = 0; t < 13; t++) s += Bb[13 * i + t] * Ai[13 * t + cc];
                    G[p] = s;
                }
                wv.sync();
                if (L < 64) {
                    int i = L >> 3, j = L & 7;
                    double s = 0.0;
#if IMPC_FACT2 && IMPC_F2U == 0
                    _Pragma("unroll")
#elif IMPC_FACT2
                    IMPC_PRAGMA(unroll IMPC_F2U)
#endif
                    for (int t = 0; t < 13; t++) s += G[13 * i + t] * Bb[13 * j + t];
                    if constexpr (F3)
                        e_reg = s;
                    else
                        E[8 * i + j] = s;
                    // recursion layout: lane (i,j) of step k reads F_k[j][i] when the column index
                    // sits on i (k even), F_k[i][j] otherwise
                    Fm[64 * k + 8 * i + j] = !(k & 1) ? G[13 * j + i] : G[13 * i + j];
                }
                _Pragma("unroll") for (int s = 0; s < VS; s++) {
                    if (!vok[s]) continue;
                    if (vs_[s] == k && vr_[s] >= 8)
                        _Pragma("unroll") for (int j = 0; j < 8; j++) cp[s][j] = G[13 * j + vr_[s]];
                    if (vs_[s] == k + 1 && vr_[s] < 8)
                        _Pragma("unroll") for (int j = 0; j < 8; j++) cp[s][j] = j < 5 ? G[13 * vr_[s] + 8 + j] : 0.0;
                }
                if constexpr (!F3) wv.sync();
            }
            IMPC_SEC(kSecFDense);
        }
        _Pragma("unroll") for (int s = 0; s < VS; s++)
            if (vok[s] && vs_[s] == 0 && vr_[s] < 8)
                _Pragma("unroll") for (int j = 0; j < 8; j++) cp[s][j] = 0.0;
        if constexpr (CHUNK) chunk_ops();
        bad = (int)wv.max((double)bad);  // set by lane 0 only: team-wide, so every wavefront agrees
        clear_exchange();
        zero_products();  // the (4g + e) factorisation scratch shared the products region
        (void)n;
        return bad;
    }

    // F_k[r][c] from the recursion layout (factorize stores even stages' blocks transposed)
    IMPC_WF static double f_el(const double *Fm, int k, int r, int c) {
        return !(k & 1) ? Fm[64 * k + 8 * c + r] : Fm[64 * k + 8 * r + c];
    }

    // The chunk operators (CHUNK): wave 0 / 1 the forward chunks 1 / 2 (steps CL..2CL-1 /
    // 2CL..3CL-1, P <- -F_k P with k ascending), wave 2 / 3 the backward chunks 1 / 2 (steps
    // 3CL-1..2CL / 2CL-1..CL, P <- -F_k^T P with k descending); lane (i, j) holds P[i][j].  Then the
    // two-chunk operators of the last chunk's start, P2 P1, forward and backward.
    IMPC_WF void chunk_ops() {
        if constexpr (NCH == 5) {
            chunk_ops5();
            return;
        }
        const double *Fm = F();
        double *C = chbuf();
        const int w = L >> 6, l = L & 63, i = l >> 3, j = l & 7;
        const bool fwd = w < 2;
        const int o = (w == 0 || w == 3) ? CL : 2 * CL;
        double *P = C + (fwd ? kChFP1 + 64 * w : kChBT1 + 64 * (w - 2));
        P[l] = i == j ? 1.0 : 0.0;
        wv.wsync();
        for (int s = 0; s < CL; s++) {
            const int k = fwd ? o + s : o + CL - 1 - s;
            double pc[8];
            _Pragma("unroll") for (int m = 0; m < 8; m++) pc[m] = P[8 * m + j];
            double v = 0.0;
            _Pragma("unroll") for (int m = 0; m < 8; m++) v -= (fwd ? f_el(Fm, k, i, m) : f_el(Fm, k, m, i)) * pc[m];
            wv.wsync();
            P[l] = v;
            wv.wsync();
        }
        wv.sync();
        if (w == 0 || w == 2) {
            const double *P1 = C + (w == 0 ? kChFP1 : kChBT1), *P2 = C + (w == 0 ? kChFP2 : kChBT2);
            double v = 0.0;
            _Pragma("unroll") for (int m = 0; m < 8; m++) v += P2[8 * i + m] * P1[8 * m + j];
            C[(w == 0 ? kChFP21 : kChBT21) + l] = v;
        }
        wv.sync();
    }

    // P = the product of one chunk's step operators on one wavefront (lane (i, j) holds P[i][j]):
    // forward steps o..o+CL-1, P <- -F_k P with k ascending; backward steps o+CL-1..o, P <- -F_k^T P
    // with k descending
    IMPC_WF void chunk_prod(bool fwd, int o, double *P, int l) {
        const double *Fm = F();
        const int i = l >> 3, j = l & 7;
        P[l] = i == j ? 1.0 : 0.0;
        wv.wsync();
        for (int s = 0; s < CL; s++) {
            const int k = fwd ? o + s : o + CL - 1 - s;
            double pc[8];
            _Pragma("unroll") for (int m = 0; m < 8; m++) pc[m] = P[8 * m + j];
            double v = 0.0;
            _Pragma("unroll") for (int m = 0; m < 8; m++) v -= (fwd ? f_el(Fm, k, i, m) : f_el(Fm, k, m, i)) * pc[m];
            wv.wsync();
            P[l] = v;
            wv.wsync();
        }
    }
    IMPC_WF static void mat8(const double *A, const double *B, double *out, int l) {  // out = A B
        const int i = l >> 3, j = l & 7;
        double v = 0.0;
        _Pragma("unroll") for (int m = 0; m < 8; m++) v += A[8 * i + m] * B[8 * m + j];
        out[l] = v;
    }
    // The five-chunk operators: forward chunks c = 1..3 start at c CL; backward chunks c = 1..3 (in
    // sweep order) cover steps (5 - c) CL - 1 .. (4 - c) CL.  Six chunk products on four wavefronts,
    // then the two-chunk products, then the three-chunk ones.
    IMPC_WF void chunk_ops5() {
        double *C = chbuf(), *Bk = C + kCh5B;
        const int w = L >> 6, l = L & 63;
        if (w < 3)
            chunk_prod(true, (w + 1) * CL, C + kCh5P1 + 64 * w, l);
        else
            chunk_prod(false, 3 * CL, Bk + kCh5P1, l);
        if (w < 2) chunk_prod(false, (2 - w) * CL, Bk + kCh5P2 + 64 * w, l);
        wv.sync();
        // w 0 / 1: forward P2 P1 / P3 P2; w 2 / 3: backward P2 P1 / P3 P2
        double *X = w < 2 ? C : Bk;
        mat8(X + kCh5P2 + 64 * (w & 1), X + kCh5P1 + 64 * (w & 1), X + kCh5P21 + 64 * (w & 1), l);
        wv.sync();
        if (w < 2) {  // w 0: forward P3 P2 P1, w 1: backward
            double *Y = w ? Bk : C;
            mat8(Y + kCh5P3, Y + kCh5P21, Y + kCh5P321, l);
        }
        wv.sync();
    }

    // One step of a stage recursion on the 8x8 lane grid: returns c - F v as R(c / 8 - f v), R the
    // strided (STRIDE) or contiguous 8-lane sum.  The sweeps' inputs c come pre-scaled by 1/8
    // (exact: S1 stores t / 8, S3 the state part of e / 8), so the subtraction rides in the
    // product's FMA: one instruction and one dependent operation less per step on the serial chain.
    template <bool STRIDE>
    IMPC_WF double rstep(double f, double c8, double v) {
        const double p = __builtin_fma(-f, v, c8);
        return STRIDE ? wv.sum_stride8(p) : wv.sum_contig8(p);
    }

    // Sweeps with a compile-time step count WC (= WSPEC) are fully unrolled: every LDS wait is
    // exact and the step results stay in registers until the sweep ends, instead of an LDS store
    // per step whose completion the next step's wait would include (measured 195 -> 157 cycles
    // per step, tools/probe/recur_probe.hip).  Step m's result sits in the 8 lanes sharing its
    // output index; of those the lane whose other index is (m/2) mod 8 keeps it, in slot m/16 of
    // the even- or odd-step array (a compile-time lane mask, one v_cndmask pair per step).
    static constexpr int CQ = LD::WSPEC / 16 + 1;
    IMPC_WF static void cap(double (&c)[CQ], double r, int m, int other) {
        if (((m >> 1) & 7) == other) c[m >> 4] = r;
    }
    // cap with the lane test as a compile-time lane mask (OI: `other` is the lane's i = l >> 3, else
    // j = l & 7; lane l = 8 i + j of the recursion wavefront): the select by that constant mask in
    // an SGPR pair instead of a v_cmp per step (the CPU emulation takes the plain test)
    template <bool OI>
    IMPC_WF static void capm(double (&c)[CQ], double r, int m, int other) {
#if defined(__HIP_DEVICE_COMPILE__)
        (void)other;
        const int v = (m >> 1) & 7;
        const uint64_t msk = OI ? (0xFFull << (8 * v)) : (0x0101010101010101ull << v);
        double &d = c[m >> 4];
        int lo = __double2loint(d), hi = __double2hiint(d);
        asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(lo) : "v"(__double2loint(r)), "s"(msk));
        asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(hi) : "v"(__double2hiint(r)), "s"(msk));
        d = __hiloint2double(hi, lo);
#else
        cap(c, r, m, other);
#endif
    }
    // Store a sweep's W captured steps: even steps' outputs sit at index j (EJ) or i, odd steps'
    // at the other; step m is stage m + 1 (forward) or W - 1 - m (backward).
    template <bool EJ>
    IMPC_WF static void cap_store(const double (&c0)[CQ], const double (&c1)[CQ], double *buf, int W, bool fwd,
                                  int i, int j) {
        const int o0 = EJ ? i : j, e0 = EJ ? j : i;
        _Pragma("unroll") for (int q = 0; q < CQ; q++) {
            const int m0 = 16 * q + 2 * o0, m1 = 16 * q + 2 * e0 + 1;
            if (m0 < W) buf[13 * (fwd ? m0 + 1 : W - 1 - m0) + e0] = c0[q];
            if (m1 < W) buf[13 * (fwd ? m1 + 1 : W - 1 - m1) + o0] = c1[q];
        }
    }

    // Forward steps o .. o + WC - 1 (o even) from a_o = a at index i, fully unrolled: the results
    // a_{o+1} .. a_{o+WC} stored to rb when CAP, the last one returned (every lane (i, j) holds
    // a_{o+WC}[i] or [j] by its parity).
    template <int WC, bool CAP>
    IMPC_WF double fwd_run(const double *tb, double *rb, int o, double a) {
        const double *Fm = lds + LD::F_OFF + 64 * o;
        tb += 13 * o;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;  // opaque: see lane_o
        // (F, t) of the next even / odd step, loaded two steps ahead (reads past the last stage
        // stay inside the LDS buffers and are never used)
        double fe = Fm[l], te = tb[13 + j], fo = Fm[64 + l], to = tb[26 + i];
        double c0[CQ], c1[CQ];
        _Pragma("unroll") for (int q = 0; q < CQ; q++) c0[q] = c1[q] = 0.0;
        _Pragma("unroll") for (int k = 0; k < WC; k += 2) {
            const double f0 = fe, t0 = te;
            fe = Fm[64 * (k + 2) + l];
            te = tb[13 * (k + 3) + j];
            a = rstep<true>(f0, t0, a);
            if constexpr (CAP) capm<true>(c0, a, k, i);
            if (k + 1 < WC) {
                const double f1 = fo, t1 = to;
                fo = Fm[64 * (k + 3) + l];
                to = tb[13 * (k + 4) + i];
                a = rstep<false>(f1, t1, a);
                if constexpr (CAP) capm<false>(c1, a, k + 1, j);
            }
        }
        if constexpr (CAP) cap_store<true>(c0, c1, rb + 13 * o, WC, true, i, j);
        return a;
    }

    // S2 body: a_{k+1} = t_{k+1} - F_k a_k for k = 0..W-1 (WC = W, or 0 for a runtime W).
    template <int WC>
    IMPC_WF void fwd_sweep(const double *tb, double *rb, int W) {
        const double *Fm = lds + LD::F_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;  // opaque: see lane_o
        double a = 8.0 * tb[i];  // a_0 = t_0 (tb holds t / 8)
        // (F, t) of the next even / odd step, loaded two steps ahead (reads past the last stage
        // stay inside the LDS buffers and are never used)
        double fe = Fm[l], te = tb[13 + j], fo = Fm[64 + l], to = tb[26 + i];
        if constexpr (WC > 0) {
            double c0[CQ], c1[CQ];
            _Pragma("unroll") for (int q = 0; q < CQ; q++) c0[q] = c1[q] = 0.0;
            _Pragma("unroll") for (int k = 0; k < WC; k += 2) {
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
                a = rstep<true>(f0, t0, a);
                capm<true>(c0, a, k, i);
                if (k + 1 < WC) {
                    const double f1 = fo, t1 = to;
                    fo = Fm[64 * (k + 3) + l];
                    to = tb[13 * (k + 4) + i];
                    a = rstep<false>(f1, t1, a);
                    capm<false>(c1, a, k + 1, j);
                }
            }
            cap_store<true>(c0, c1, rb, WC, true, i, j);
        } else {
            // one lane per element writes, the rest write to discard slots (no divergent branch)
            double *junk = lds + LD::JUNK_OFF + lo;
            const bool wri = j == 0, wrj = i == 0;
            for (int k = 0; k < W; k += 2) {
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
                a = rstep<true>(f0, t0, a);
                *(wrj ? rb + 13 * (k + 1) + j : junk) = a;
                if (k + 1 >= W) break;
                const double f1 = fo, t1 = to;
                fo = Fm[64 * (k + 3) + l];
                to = tb[13 * (k + 4) + i];
                a = rstep<false>(f1, t1, a);
                *(wri ? rb + 13 * (k + 2) + i : junk) = a;
            }
        }
    }

    // Backward steps o + WC - 1 .. o (o even, the first of parity ODD) from x_{o+WC} = x, fully
    // unrolled: x_{o+WC-1} .. x_o stored to xb when CAP, x_o returned.
    template <bool ODD, int WC, bool CAP>
    IMPC_WF double bwd_run(const double *eb, double *xb, int o, double x) {
        const double *Fm = lds + LD::F_OFF + 64 * o;
        eb += 13 * o;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        constexpr int k1 = WC - 2 > 0 ? WC - 2 : 0;
        double fa = Fm[64 * (WC - 1) + l], ea = eb[13 * (WC - 1) + (ODD ? j : i)];
        double fb = Fm[64 * k1 + l], ebv = eb[13 * k1 + (ODD ? i : j)];
        double c0[CQ], c1[CQ];
        _Pragma("unroll") for (int q = 0; q < CQ; q++) c0[q] = c1[q] = 0.0;
        _Pragma("unroll") for (int m = 0; m < WC; m += 2) {
            const int k = WC - 1 - m;
            const int k2 = k - 2 > 0 ? k - 2 : 0, k3 = k - 3 > 0 ? k - 3 : 0;
            const double f0 = fa, e0 = ea;
            fa = Fm[64 * k2 + l];
            ea = eb[13 * k2 + (ODD ? j : i)];
            x = rstep<ODD>(f0, e0, x);
            if constexpr (CAP) capm<ODD>(c0, x, m, ODD ? i : j);
            if (m + 1 < WC) {
                const double f1 = fb, e1 = ebv;
                fb = Fm[64 * k3 + l];
                ebv = eb[13 * k3 + (ODD ? i : j)];
                x = rstep<!ODD>(f1, e1, x);
                if constexpr (CAP) capm<!ODD>(c1, x, m + 1, ODD ? j : i);
            }
        }
        if constexpr (CAP) cap_store<ODD>(c0, c1, xb + 13 * o, WC, false, i, j);
        return x;
    }

    // S4 body for a first step k = W-1 of parity ODD: steps alternate strided (odd k) and
    // contiguous (even k) reductions; x_k sits at index j (odd k) / i (even k).  WC as above.
    template <bool ODD, int WC>
    IMPC_WF void bwd_sweep(const double *eb, double *xb, int W) {
        const double *Fm = lds + LD::F_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        if constexpr (WC > 0) W = WC;
        // x_W = e_W: W = (W-1)+1 has the opposite parity of the first step (eb holds e[:8] / 8)
        double x = 8.0 * eb[13 * W + (ODD ? i : j)];
        const int k1 = W - 2 > 0 ? W - 2 : 0;
        double fa = Fm[64 * (W - 1) + l], ea = eb[13 * (W - 1) + (ODD ? j : i)];
        double fb = Fm[64 * k1 + l], ebv = eb[13 * k1 + (ODD ? i : j)];
        if constexpr (WC > 0) {
            double c0[CQ], c1[CQ];
            _Pragma("unroll") for (int q = 0; q < CQ; q++) c0[q] = c1[q] = 0.0;
            _Pragma("unroll") for (int m = 0; m < WC; m += 2) {
                const int k = WC - 1 - m;
                const int k2 = k - 2 > 0 ? k - 2 : 0, k3 = k - 3 > 0 ? k - 3 : 0;
                const double f0 = fa, e0 = ea;
                fa = Fm[64 * k2 + l];
                ea = eb[13 * k2 + (ODD ? j : i)];
                x = rstep<ODD>(f0, e0, x);
                capm<ODD>(c0, x, m, ODD ? i : j);
                if (m + 1 < WC) {
                    const double f1 = fb, e1 = ebv;
                    fb = Fm[64 * k3 + l];
                    ebv = eb[13 * k3 + (ODD ? i : j)];
                    x = rstep<!ODD>(f1, e1, x);
                    capm<!ODD>(c1, x, m + 1, ODD ? j : i);
                }
            }
            cap_store<ODD>(c0, c1, xb, WC, false, i, j);
        } else {
            double *junk = lds + LD::JUNK_OFF + lo;
            const bool wri = j == 0, wrj = i == 0;
            for (int k = W - 1; k >= 0; k -= 2) {
                const int k2 = k - 2 > 0 ? k - 2 : 0, k3 = k - 3 > 0 ? k - 3 : 0;
                const double f0 = fa, e0 = ea;
                fa = Fm[64 * k2 + l];
                ea = eb[13 * k2 + (ODD ? j : i)];
                x = rstep<ODD>(f0, e0, x);
                *(ODD ? (wrj ? xb + 13 * k + j : junk) : (wri ? xb + 13 * k + i : junk)) = x;
                if (k - 1 < 0) break;
                const double f1 = fb, e1 = ebv;
                fb = Fm[64 * k3 + l];
                ebv = eb[13 * k3 + (ODD ? i : j)];
                x = rstep<!ODD>(f1, e1, x);
                *(ODD ? (wri ? xb + 13 * (k - 1) + i : junk) : (wrj ? xb + 13 * (k - 1) + j : junk)) = x;
            }
        }
    }

    // S2 in chunks (CHUNK; see CH_OFF): steps 0..CL-1 / CL..2CL-1 / 2CL..3CL-1 / 3CL..W-1 on waves
    // 0..3.  a_2CL = a^_2CL + P1 a_CL, a_3CL = a^_3CL + P2 a^_2CL + P2 P1 a_CL (a^: the chunk run from
    // zero); chunk starts are even stages, so a_CL sits at index i (captured by wave 0 in rb).
    IMPC_WF void fwd_chunked(const double *tb, double *rb) {
        const double *C = chbuf();
        double *ends = chbuf() + kChEnd;
        const int w = L >> 6, l = lane_o() & 63, i = l >> 3, j = l & 7;
        constexpr int A1 = 13 * CL;  // a_CL in rb
        for (int rep_ = 0; rep_ < (IMPC_CHDUP == 1 ? 2 : 1); rep_++)
        if (w == 0) {
            (void)fwd_run<CL, true>(tb, rb, 0, 8.0 * tb[i]);  // a_0 = t_0 (tb holds t / 8)
        } else if (w == 1) {
            const double e = fwd_run<CL, false>(tb, rb, CL, 0.0);
            if (j == 0) ends[i] = e;
        } else if (w == 2) {
            const double e = fwd_run<CL, false>(tb, rb, 2 * CL, 0.0);
            if (j == 0) ends[8 + i] = e;
        }
        wv.lsync();
        for (int rep_ = 0; rep_ < (IMPC_CHDUP == 2 ? 2 : 1); rep_++)
        if (w == 1) {
            (void)fwd_run<CL, true>(tb, rb, CL, rb[A1 + i]);
        } else if (w == 2) {
            const double a = wv.sum_contig8(__builtin_fma(C[kChFP1 + l], rb[A1 + j], 0.125 * ends[i]));
            (void)fwd_run<CL, true>(tb, rb, 2 * CL, a);
        } else if (w == 3) {
            const double p = __builtin_fma(C[kChFP2 + l], ends[j],
                                           __builtin_fma(C[kChFP21 + l], rb[A1 + j], 0.125 * ends[8 + i]));
            (void)fwd_run<CLAST, true>(tb, rb, 3 * CL, wv.sum_contig8(p));
        }
    }

    // S4 in chunks: steps W-1..3CL / 3CL-1..2CL / 2CL-1..CL / CL-1..0 on waves 0..3, from x_W /
    // x_3CL / x_2CL / x_CL (x_2CL = x^_2CL + P1 x_3CL, x_CL = x^_CL + P2 x^_2CL + P2 P1 x_3CL).
    IMPC_WF void bwd_chunked(const double *eb, double *xb) {
        const double *C = chbuf();
        double *ends = chbuf() + kChEnd + kChEnds;
        const int w = L >> 6, l = lane_o() & 63, i = l >> 3, j = l & 7;
        constexpr int X3 = 13 * 3 * CL;     // x_3CL in xb (even stage: index i)
        constexpr bool LODD = (WF - 1) & 1;  // parity of the last chunk's first step W - 1
        for (int rep_ = 0; rep_ < (IMPC_CHDUP == 1 ? 2 : 1); rep_++)
        if (w == 0) {
            // x_W = e_W: at index j for odd W, i for even W
            (void)bwd_run<LODD, CLAST, true>(eb, xb, 3 * CL, 8.0 * eb[13 * WF + (LODD ? i : j)]);
        } else if (w == 1) {
            const double e = bwd_run<true, CL, false>(eb, xb, 2 * CL, 0.0);
            if (j == 0) ends[i] = e;
        } else if (w == 2) {
            const double e = bwd_run<true, CL, false>(eb, xb, CL, 0.0);
            if (j == 0) ends[8 + i] = e;
        }
        wv.lsync();
        for (int rep_ = 0; rep_ < (IMPC_CHDUP == 2 ? 2 : 1); rep_++)
        if (w == 1) {
            (void)bwd_run<true, CL, true>(eb, xb, 2 * CL, xb[X3 + i]);
        } else if (w == 2) {
            const double x = wv.sum_contig8(__builtin_fma(C[kChBT1 + l], xb[X3 + j], 0.125 * ends[i]));
            (void)bwd_run<true, CL, true>(eb, xb, CL, x);
        } else if (w == 3) {
            const double p = __builtin_fma(C[kChBT2 + l], ends[j],
                                           __builtin_fma(C[kChBT21 + l], xb[X3 + j], 0.125 * ends[8 + i]));
            (void)bwd_run<true, CL, true>(eb, xb, 0, wv.sum_contig8(p));
        }
    }

    // S2 in five chunks (NCH = 5): steps c CL .. c CL + CL - 1 (c = 0..3) and 4 CL .. W - 1; waves
    // 1..3 run chunks 1..3 twice, wave 0 chunk 0 in round 1 and chunk 4 in round 2.
    IMPC_WF void fwd_chunked5(const double *tb, double *rb) {
        const double *C = chbuf();
        double *ends = chbuf() + kChEnd;
        const int w = L >> 6, l = lane_o() & 63, i = l >> 3, j = l & 7;
        constexpr int A1 = 13 * CL;  // a_CL in rb (even stage: index i)
        if (w == 0) {
            (void)fwd_run<CL, true>(tb, rb, 0, 8.0 * tb[i]);  // a_0 = t_0 (tb holds t / 8)
        } else {
            const double e = fwd_run<CL, false>(tb, rb, w * CL, 0.0);
            if (j == 0) ends[8 * (w - 1) + i] = e;
        }
        wv.lsync();
        if (w == 1) {
            (void)fwd_run<CL, true>(tb, rb, CL, rb[A1 + i]);
        } else if (w == 2) {
            const double a = wv.sum_contig8(__builtin_fma(C[kCh5P1 + l], rb[A1 + j], 0.125 * ends[i]));
            (void)fwd_run<CL, true>(tb, rb, 2 * CL, a);
        } else if (w == 3) {
            const double p = __builtin_fma(C[kCh5P2 + l], ends[j],
                                           __builtin_fma(C[kCh5P21 + l], rb[A1 + j], 0.125 * ends[8 + i]));
            (void)fwd_run<CL, true>(tb, rb, 3 * CL, wv.sum_contig8(p));
        } else {
            const double p = __builtin_fma(
                C[kCh5P3 + l], ends[8 + j],
                __builtin_fma(C[kCh5P32 + l], ends[j], __builtin_fma(C[kCh5P321 + l], rb[A1 + j], 0.125 * ends[16 + i])));
            (void)fwd_run<CLAST, true>(tb, rb, 4 * CL, wv.sum_contig8(p));
        }
    }

    // S4 in five chunks: steps W-1..4CL (wave 0, round 1, from x_W), 4CL-1..3CL / 3CL-1..2CL /
    // 2CL-1..CL (waves 1..3, both rounds), CL-1..0 (wave 0, round 2).
    IMPC_WF void bwd_chunked5(const double *eb, double *xb) {
        const double *C = chbuf() + kCh5B;
        double *ends = chbuf() + kChEnd + kChEnds;
        const int w = L >> 6, l = lane_o() & 63, i = l >> 3, j = l & 7;
        constexpr int X4 = 13 * 4 * CL;      // x_4CL in xb (even stage: index i)
        constexpr bool LODD = (WF - 1) & 1;  // parity of the first chunk's first step W - 1
        if (w == 0) {
            (void)bwd_run<LODD, CLAST, true>(eb, xb, 4 * CL, 8.0 * eb[13 * WF + (LODD ? i : j)]);
        } else {
            const double e = bwd_run<true, CL, false>(eb, xb, (4 - w) * CL, 0.0);
            if (j == 0) ends[8 * (w - 1) + i] = e;
        }
        wv.lsync();
        if (w == 1) {
            (void)bwd_run<true, CL, true>(eb, xb, 3 * CL, xb[X4 + i]);
        } else if (w == 2) {
            const double x = wv.sum_contig8(__builtin_fma(C[kCh5P1 + l], xb[X4 + j], 0.125 * ends[i]));
            (void)bwd_run<true, CL, true>(eb, xb, 2 * CL, x);
        } else if (w == 3) {
            const double p = __builtin_fma(C[kCh5P2 + l], ends[j],
                                           __builtin_fma(C[kCh5P21 + l], xb[X4 + j], 0.125 * ends[8 + i]));
            (void)bwd_run<true, CL, true>(eb, xb, CL, wv.sum_contig8(p));
        } else {
            const double p = __builtin_fma(
                C[kCh5P3 + l], ends[8 + j],
                __builtin_fma(C[kCh5P32 + l], ends[j], __builtin_fma(C[kCh5P321 + l], xb[X4 + j], 0.125 * ends[16 + i])));
            (void)bwd_run<true, CL, true>(eb, xb, 0, wv.sum_contig8(p));
        }
    }

    // v = rho z - y products of the general rows for the next rhs
    IMPC_WF void write_v_products() {
        double *pb = pbuf();
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            // (an empty slot writes a zero product to the discard slot)
            double vv = rhog_(s) * z[s] - y[s];
            _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = a[s][e] * vv;
        }
        wv.lsync();
    }

    // --------------------------------------------------------------- one ADMM iteration
    IMPC_WF void iterate(bool need_delta) {
        const int W = Wst();
        double *rb = rbuf(), *tb = tbuf(), *eb = ebuf(), *xb = xbuf();
        const double sigma = sig_;
        IMPC_REP(kSecRhs) {
            // rhs = sigma x - q + A' v   (stage order; an empty slot's iterates, bounds and column
            // are zero, so it writes 0)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                int v = NL * s + L;
                double vb = rhob(s) * zb[s] - yb[s];
                double r = sigma * x[s] - q[s];
                r += ab[s] * vb;
                r += col_gather(v, hid_[s]);
                rb[v] = r;
            }
            wv.lsync();
        }
        IMPC_SEC(kSecRhs);
        IMPC_REP(kSecS1) {
            // S1: t_k = r_k[:8] - G_{k-1}[:, 8:] r_{k-1}[8:]  (every lane, without branches: a
            // stage-0 or empty slot has zero coupling coefficients, a control lane's t lands in a
            // slot nothing reads)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                int v = NL * s + L;
                double t = rb[v];
                // (stage 0: the zero tail of the x exchange, not LDS below rb -- past the horizon's
                // last F block that is another QP's data or uninitialised)
                const double *rp = lds + (vs_[s] > 0 ? LD::R_OFF + 13 * (vs_[s] - 1) + 8 : LD::X_OFF + LD::NMAX);
                double rv[5];
                _Pragma("unroll") for (int cc = 0; cc < 5; cc++) rv[cc] = rp[cc];
                IMPC_LOADS_FIRST(5, 12);
                _Pragma("unroll") for (int cc = 0; cc < 5; cc++) t -= cp[s][cc] * rv[cc];
                tb[v] = 0.125 * t;  // the forward sweep's input, pre-scaled (rstep)
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS1);
        IMPC_REP(kSecFwd) {
            // S2: forward 8-dim recursion a_{k+1} = t_{k+1} - F_k a_k on the 8x8 lane grid of each
            // wavefront (lane l = 8i + j).  Vectors of even stages sit at index i, of odd stages at
            // index j; F_k is stored as F_k[j][i] (k even) / F_k[i][j] (k odd), so even steps reduce
            // over i (strided: DPP row_ror 8, permlane16/32 swaps) and odd steps over j (contiguous
            // DPP), all in the VALU, with no transpose.  The next F and t are loaded two steps ahead.
            // One wavefront of the team (rw) runs it -- the others go straight to the barrier and
            // leave their SIMD's issue slots to the co-resident team.
            // (a_0 = t_0 = r_0[:8] is already in rb: stage 0 has no coupling, so S1 left it as is)
            // The long horizon's W = 39 instance runs it in chunks on all four wavefronts (CHUNK).
            if constexpr (CHUNK && NCH == 5) {
                fwd_chunked5(tb, rb);
            } else if constexpr (CHUNK) {
                fwd_chunked(tb, rb);
            } else if ((L >> 6) == rw) {
                IMPC_PRIO_UP();
                if (W == LD::WSPEC)
                    fwd_sweep<LD::WSPEC>(tb, rb, W);
                else
                    fwd_sweep<0>(tb, rb, W);
                IMPC_PRIO_DOWN();
            }
            wv.lsync();
        }
        IMPC_SEC(kSecFwd);
        IMPC_REP(kSecS3) {
            // S3: e_k = Ahat_k^{-1} rhat_k
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                const double *rk = lds + LD::R_OFF + 13 * vs_[s];
                double rv[13];
                _Pragma("unroll") for (int cc = 0; cc < 13; cc++) rv[cc] = rk[cc];
                IMPC_LOADS_FIRST(7, 20);
                double e = 0.0;
                _Pragma("unroll") for (int cc = 0; cc < 13; cc++) e += ainv[s][cc] * rv[cc];
                // the state part pre-scaled for the backward sweep (rstep); S5 reads the controls' e
                eb[NL * s + L] = vr_[s] < 8 ? 0.125 * e : e;
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS3);
        IMPC_REP(kSecBwd) {
            // S4: backward 8-dim recursion x_k[:8] = e_k[:8] - F_k' x_{k+1}[:8] on the same grid and
            // stored layout: even steps reduce over j (contiguous), odd steps over i (strided).
            if (L < 8) xb[13 * W + L] = 8.0 * eb[13 * W + L];
            if constexpr (CHUNK && NCH == 5) {
                bwd_chunked5(eb, xb);
            } else if constexpr (CHUNK) {
                bwd_chunked(eb, xb);
            } else if ((L >> 6) == rw) {
                IMPC_PRIO_UP();
                if (W == LD::WSPEC)
                    bwd_sweep<((LD::WSPEC - 1) & 1) != 0, LD::WSPEC>(eb, xb, W);
                else if ((W - 1) & 1)
                    bwd_sweep<true, 0>(eb, xb, W);
                else
                    bwd_sweep<false, 0>(eb, xb, W);
                IMPC_PRIO_DOWN();
            }
            wv.lsync();
        }
        IMPC_SEC(kSecBwd);
        IMPC_REP(kSecS5) {
            // S5: controls x_k[8:] = e_k[8:] - G_k[:, 8:]' x_{k+1}[:8]  (every lane, the state lanes'
            // and empty slots' results to their discard slots)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                const double *xn = lds + LD::X_OFF + 13 * (vs_[s] + 1);
                double t = eb[NL * s + L];
                double xv[8];
                _Pragma("unroll") for (int j = 0; j < 8; j++) xv[j] = xn[j];
                IMPC_LOADS_FIRST(5, 16);
                _Pragma("unroll") for (int j = 0; j < 8; j++) t -= cp[s][j] * xv[j];
                *(vok[s] && vr_[s] >= 8 ? xb + NL * s + L : lds + LD::JUNK_OFF + L) = t;
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS5);
        update_and_products(need_delta);
    }

    // project_z (auxil.h): min(max(v, l), u), as v_max_f64 / v_min_f64 -- the same value as the
    // reference's c_max / c_min except the sign of a zero when v equals a zero bound
    IMPC_WF static double clampz(double v, double l, double u) { return __builtin_fmin(__builtin_fmax(v, l), u); }

    // update_x and the box rows (update_z / project / update_y), the general rows, and the
    // products of the next rhs (the end of every ADMM iteration).  need_delta: the check-iteration
    // deltas are written.
    IMPC_WF void update_and_products(bool need_delta) {
        double *xb = xbuf();
        const double alpha = alp_, oma = (double)1.0 - alp_;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            double xt = xb[NL * s + L];
            double xn = alpha * xt + oma * x[s];
            if (need_delta) dxv(s) = xn - x[s];
            x[s] = xn;
            double zt = ab[s] * xt;
            double zr = alpha * zt + oma * zb[s];
            double zn = clampz(zr + rhoib(s) * yb[s], lb[s], ub[s]);
            double dy = rhob(s) * (zr - zn);
            yb[s] += dy;
            if (need_delta) dyb(s) = dy;
            zb[s] = zn;
        }
        // general rows, without a per-slot branch: an empty slot's columns are the zero tail of the
        // x exchange, its A values, bounds and iterates zero, so it computes zeros
        double xg[GS][4];
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            _Pragma("unroll") for (int e = 0; e < 4; e++) xg[s][e] = xb[gcol(s, e)];
        }
        IMPC_LOADS_FIRST(4 * GS, 8 * GS);
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            double zt = 0.0;
            _Pragma("unroll") for (int e = 0; e < 4; e++) zt += a[s][e] * xg[s][e];
            double zr = alpha * zt + oma * z[s];
            double zn = clampz(zr + rhoig_(s) * y[s], lg[s], ug[s]);
            double dy = rhog_(s) * (zr - zn);
            y[s] += dy;
            if (need_delta) dyg(s) = dy;
            z[s] = zn;
        }
        // no barrier: the products go to their own LDS region, which nothing above reads, and
        // write_v_products ends with the barrier the next rhs gather needs
        IMPC_SEC(kSecUpdate);
        IMPC_REP(kSecProducts) write_v_products();
        IMPC_SEC(kSecProducts);
    }

    // ------------------------------------------------------------ update_info + checks
    struct Info {
        double pri_res, dua_res, pri_norm_u, dua_norm_u, pri_norm_s, dua_norm_s, pri_plain, dua_plain;
        // the infeasibility tests' first stages (is_primal_infeasible: ||E P(dy)||, u'P(dy)_+ +
        // l'P(dy)_-; is_dual_infeasible: ||D dx||, q'dx, and its ||D^-1 P dx||), reduced with the
        // norms above
        double pinf_nrm, pinf_lhs, dinf_nrm, dinf_qdx, dinf_pdx;
    };

    IMPC_WF void load_scal(int64_t b, double D[VS], double Eb[VS], double Eg[GS]) {
        const double *sc = scal(b);
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            D[s] = vok[s] ? sc[NL * s + L] : 1.0;
            Eb[s] = vok[s] ? sc[T.n + NL * s + L] : 1.0;
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) Eg[s] = gok[s] ? sc[2 * T.n + NL * s + L] : 1.0;
    }

    IMPC_WF void update_info(Info &inf, const double D[VS], const double Eb[VS], const double Eg[GS]) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        double *xb = xbuf(), *pb = pbuf();
        _Pragma("unroll") for (int s = 0; s < VS; s++)
            if (vok[s]) xb[NL * s + L] = x[s];
        // A'y products of the general rows
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (gok[s])
                _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = a[s][e] * y[s];
        }
        wv.sync();
        double pr_u = 0, z_u = 0, ax_u = 0, pr_p = 0, z_p = 0, ax_p = 0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            double ax = ab[s] * x[s], r = ax + -1 * zb[s], ei = 1. / Eb[s];
            pr_p = dmax(pr_p, fabs(r));
            z_p = dmax(z_p, fabs(zb[s]));
            ax_p = dmax(ax_p, fabs(ax));
            pr_u = dmax(pr_u, fabs(ei * r));
            z_u = dmax(z_u, fabs(ei * zb[s]));
            ax_u = dmax(ax_u, fabs(ei * ax));
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (!gok[s]) continue;
            double ax = 0.0;
            _Pragma("unroll") for (int e = 0; e < 4; e++) ax += a[s][e] * xb[gcol(s, e)];
            double r = ax + -1 * z[s], ei = 1. / Eg[s];
            pr_p = dmax(pr_p, fabs(r));
            z_p = dmax(z_p, fabs(z[s]));
            ax_p = dmax(ax_p, fabs(ax));
            pr_u = dmax(pr_u, fabs(ei * r));
            z_u = dmax(z_u, fabs(ei * z[s]));
            ax_u = dmax(ax_u, fabs(ei * ax));
        }
        double dr_u = 0, q_u = 0, aty_u = 0, px_u = 0, dr_p = 0, q_p = 0, aty_p = 0, px_p = 0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            double aty = ab[s] * yb[s] + col_gather(NL * s + L, hid_[s]);
            double px = pd[s] * x[s];
            double r = q[s] + 1 * px;
            r = r + 1 * aty;
            double di = 1. / D[s];
            dr_p = dmax(dr_p, fabs(r));
            q_p = dmax(q_p, fabs(q[s]));
            aty_p = dmax(aty_p, fabs(aty));
            px_p = dmax(px_p, fabs(px));
            dr_u = dmax(dr_u, fabs(di * r));
            q_u = dmax(q_u, fabs(di * q[s]));
            aty_u = dmax(aty_u, fabs(di * aty));
            px_u = dmax(px_u, fabs(di * px));
        }
        {
            // the infeasibility tests' lane-local parts too (the check needs them whenever it does
            // not terminate): one team reduction for 16 maxima and 2 sums
            double pn, pl, dn, dq, dp;
            pinf_partials(Eb, Eg, pn, pl);
            dinf_partials(D, dn, dq, dp);
            double r[17] = {pr_u, z_u, ax_u, pr_p, z_p, ax_p, dr_u, q_u, aty_u, px_u, dr_p, q_p, aty_p, px_p, pn, dn, dp};
            double sm[2] = {pl, dq};
            wv.max_sum_n(r, sm);
            pr_u = r[0], z_u = r[1], ax_u = r[2], pr_p = r[3], z_p = r[4], ax_p = r[5], dr_u = r[6];
            q_u = r[7], aty_u = r[8], px_u = r[9], dr_p = r[10], q_p = r[11], aty_p = r[12], px_p = r[13];
            inf.pinf_nrm = r[14];
            inf.dinf_nrm = r[15];
            inf.dinf_pdx = r[16];
            inf.pinf_lhs = sm[0];
            inf.dinf_qdx = sm[1];
        }
        inf.pri_plain = pr_p;
        inf.dua_plain = dr_p;
        inf.pri_norm_s = dmax(z_p, ax_p);
        inf.dua_norm_s = dmax(dmax(q_p, aty_p), px_p);
        if (unsc) {
            inf.pri_res = T.m == 0 ? 0.0 : pr_u;
            inf.dua_res = cinv * dr_u;
            inf.pri_norm_u = dmax(z_u, ax_u);
            inf.dua_norm_u = dmax(dmax(q_u, aty_u), px_u) * cinv;
        } else {
            inf.pri_res = T.m == 0 ? 0.0 : pr_p;
            inf.dua_res = dr_p;
            inf.pri_norm_u = inf.pri_norm_s;
            inf.dua_norm_u = inf.dua_norm_s;
        }
        // (no barrier: the reduction's last one already follows every read of the exchange
        // buffers above)
    }

    // is_primal_infeasible's projection of dy onto the normal cone of the bounds (OSQP projects
    // delta_y in place; the next ADMM step overwrites it, so only the test's second stage sees it)
    IMPC_WF static double pinf_proj(double d, double l, double u) {
        if (u > kInf * kMinScaling) return (l < -kInf * kMinScaling) ? 0.0 : dmin(d, 0.0);
        if (l < -kInf * kMinScaling) return dmax(d, 0.0);
        return d;
    }
    // is_primal_infeasible, lane-local part: ||E P(dy)||_inf and u' max(P(dy), 0) + l' min(P(dy), 0)
    IMPC_WF void pinf_partials(const double Eb[VS], const double Eg[GS], double &nrm_o, double &lhs_o) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        double nrm = 0.0, lhs = 0.0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            const double d = pinf_proj(dyb(s), lb[s], ub[s]);
            nrm = dmax(nrm, fabs(unsc ? Eb[s] * d : d));
            lhs += ub[s] * dmax(d, 0) + lb[s] * dmin(d, 0);
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (!gok[s]) continue;
            const double d = pinf_proj(dyg(s), lg[s], ug[s]);
            nrm = dmax(nrm, fabs(unsc ? Eg[s] * d : d));
            lhs += ug[s] * dmax(d, 0) + lg[s] * dmin(d, 0);
        }
        nrm_o = nrm;
        lhs_o = lhs;
    }
    // ... and the rest, from the team-reduced norm and sum
    IMPC_WF int pinf_stage2(double eps, double nrm, double lhs, const double D[VS]) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        int res = 0;
        if (nrm > kDivTol && lhs < eps * nrm) {
            IMPC_COUNT(0);
            double *pb = pbuf();
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (gok[s]) {
                    const double d = pinf_proj(dyg(s), lg[s], ug[s]);
                    _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = a[s][e] * d;
                }
            }
            wv.sync();
            double mx = 0.0;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                double t = ab[s] * pinf_proj(dyb(s), lb[s], ub[s]) + col_gather(NL * s + L, hid_[s]);
                if (unsc) t = (1. / D[s]) * t;
                mx = dmax(mx, fabs(t));
            }
            mx = wv.max(mx);
            res = mx < eps * nrm;
            wv.sync();
        }
        return res;
    }

    // is_dual_infeasible, lane-local part: ||D dx||_inf, q' dx and ||D^-1 P dx||_inf
    IMPC_WF void dinf_partials(const double D[VS], double &nrm_o, double &qdx_o, double &pdx_o) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        double nrm = 0.0, qdx = 0.0, pdx = 0.0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            nrm = dmax(nrm, fabs(unsc ? D[s] * dxv(s) : dxv(s)));
            qdx += q[s] * dxv(s);
            double pv = pd[s] * dxv(s);
            if (unsc) pv = (1. / D[s]) * pv;
            pdx = dmax(pdx, fabs(pv));
        }
        nrm_o = nrm;
        qdx_o = qdx;
        pdx_o = pdx;
    }
    IMPC_WF int dinf_stage2(double eps, double nrm, double qdx, double mx, const double Eb[VS], const double Eg[GS]) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        const double cs = unsc ? c : 1.0;
        int res = 0;
        if (nrm > kDivTol && qdx < cs * eps * nrm) {
            IMPC_COUNT(1);
            if (mx < cs * eps * nrm) {
                IMPC_COUNT(2);
                double *xb = xbuf();
                _Pragma("unroll") for (int s = 0; s < VS; s++)
                    if (vok[s]) xb[NL * s + L] = dxv(s);
                wv.sync();
                double viol = 0.0;
                _Pragma("unroll") for (int s = 0; s < VS; s++) {
                    if (!vok[s]) continue;
                    double t = ab[s] * dxv(s);
                    if (unsc) t = (1. / Eb[s]) * t;
                    if ((ub[s] < kInf * kMinScaling && t > eps * nrm) || (lb[s] > -kInf * kMinScaling && t < -eps * nrm))
                        viol = 1.0;
                }
                _Pragma("unroll") for (int s = 0; s < GS; s++) {
                    if (!gok[s]) continue;
                    double t = 0.0;
                    _Pragma("unroll") for (int e = 0; e < 4; e++) t += a[s][e] * xb[gcol(s, e)];
                    if (unsc) t = (1. / Eg[s]) * t;
                    if ((ug[s] < kInf * kMinScaling && t > eps * nrm) || (lg[s] > -kInf * kMinScaling && t < -eps * nrm))
                        viol = 1.0;
                }
                viol = wv.max(viol);
                res = viol == 0.0;
                wv.sync();
            }
        }
        return res;
    }

    IMPC_WF int check_termination(const Info &inf, int approximate, int64_t &status, double &obj, const double D[VS],
                                  const double Eb[VS], const double Eg[GS]) {
        if ((inf.pri_res > kInf) || (inf.dua_res > kInf)) {
            status = IMPC_NON_CVX;
            obj = kNan;
            return 1;
        }
        double eps_abs = st.eps_abs, eps_rel = st.eps_rel, eps_pinf = st.eps_prim_inf, eps_dinf = st.eps_dual_inf;
        if (approximate) {
            eps_abs *= 10;
            eps_rel *= 10;
            eps_pinf *= 10;
            eps_dinf *= 10;
        }
        int prim_ok = 0, dual_ok = 0, prim_inf = 0, dual_inf = 0;
        const bool ptest = T.m != 0 && !(inf.pri_res < eps_abs + eps_rel * inf.pri_norm_u);
        prim_ok = !ptest;
        dual_ok = inf.dua_res < eps_abs + eps_rel * inf.dua_norm_u;
        // the first stages' norms and sums were reduced with the residual norms (update_info)
        IMPC_COUNT(3);
        if (ptest) IMPC_COUNT(4);
        if (!dual_ok) IMPC_COUNT(5);
        if (ptest) prim_inf = pinf_stage2(eps_pinf, inf.pinf_nrm, inf.pinf_lhs, D);
        if (!dual_ok) dual_inf = dinf_stage2(eps_dinf, inf.dinf_nrm, inf.dinf_qdx, inf.dinf_pdx, Eb, Eg);
        if (prim_ok && dual_ok) {
            status = approximate ? IMPC_SOLVED_INACCURATE : IMPC_SOLVED;
            return 1;
        } else if (prim_inf) {
            status = approximate ? IMPC_PRIMAL_INFEASIBLE_INACCURATE : IMPC_PRIMAL_INFEASIBLE;
            obj = kInf;
            return 1;
        } else if (dual_inf) {
            status = approximate ? IMPC_DUAL_INFEASIBLE_INACCURATE : IMPC_DUAL_INFEASIBLE;
            obj = -kInf;
            return 1;
        }
        return 0;
    }

    IMPC_WF double rho_estimate(const Info &inf) const {
        double pri = inf.pri_plain / (inf.pri_norm_s + kDivTol);
        double dua = inf.dua_plain / (inf.dua_norm_s + kDivTol);
        double est = R.rho * sqrt(pri / (dua + kDivTol));
        return dmin(dmax(est, kRhoMin), kRhoMax);
    }

    // ------------------------------------------------------------------ whole solve
    // The scaling vectors D, E live in the per-QP global scratch (written by scale()) and are
    // reloaded only where OSQP needs them (warm start, termination checks, unscaling), so they do
    // not occupy registers across the ADMM loop.
    // the persistent workspace (WaveIO::persist) from the registers: rho and the scaled iterates
    IMPC_WF void write_persist(double *ps) {
        const int n = T.n;
        double *it = ps + kPersistHdr;
        if (L == 0) ps[kPersistHdr - 1] = R.rho;
        _Pragma("unroll") for (int s = 0; s < VS; s++)
            if (vok[s]) {
                const int v = NL * s + L;
                it[v] = x[s];
                it[n + v] = zb[s];
                it[2 * n + v] = yb[s];
            }
        _Pragma("unroll") for (int s = 0; s < GS; s++)
            if (gok[s]) {
                const int g = NL * s + L;
                it[3 * n + g] = z[s];
                it[3 * n + T.mg + g] = y[s];
            }
    }

    IMPC_WF void solve(int64_t b) {
        const int n = T.n, m = T.m;
        // time_limit clock: from the start of the QP's setup (load, scaling, factorisation), as
        // OSQP 0.6.2 counts setup_time + solve time on a first run (every solveTraj call is one);
        // the profiling record (qpt) starts at the same tick, so a QP stopped by its limit always
        // shows a recorded latency of at least that limit.  A persistent-workspace resume (OSQP's
        // non-first run) counts from the same tick: OSQP then counts update_time + solve time, and
        // here the update work (the scaling replay, the row types, the refactorisation) runs at the
        // start of the resumed solve -- one difference: OSQP refactors on osqp_update_bounds only
        // when a row changes type, the resume always does (its time counts against the limit)
        const uint64_t t0 = device_clock();
        rw = (int)(b % (NL / 64));  // spread the serial recursions of co-resident QPs over SIMDs
#if defined(__HIP_DEVICE_COMPILE__)
        // recursion wave from the hardware placement (HW_REG_HW_ID: WAVE_ID [3:0], SIMD_ID [5:4]):
        // the wave on SIMD (wave slot of the team's wave 0) mod 4, so co-resident teams, which sit
        // in different wave slots, run their recursions on different SIMDs; the QP-index choice
        // above when no wave of the team is on that SIMD
        if ((L & 63) == 0) lds[LD::JUNK_OFF + (L >> 6)] = (double)(__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0x3f);
#endif
        IMPC_SEC_START();
        clear_exchange();
#if defined(__HIP_DEVICE_COMPILE__)
        {
            const int target = (int)lds[LD::JUNK_OFF] & 3;
            _Pragma("unroll") for (int w = NL / 64 - 1; w >= 0; w--)
                if (((int)lds[LD::JUNK_OFF + w] >> 4) == target) rw = w;
        }
#endif
        load(b);
        double *ps = io.persist ? io.persist + b * persist_stride(T.n, T.mg) : nullptr;
        {
            double D[VS], Eb[VS], Eg[GS];
            scale(b, D, Eb, Eg, ps);
            if (ps && ((io.resume == 1 && io.q_updated) || io.q_scale))  // osqp_update_lin_cost: q = c (D q)
                _Pragma("unroll") for (int s = 0; s < VS; s++)
                    if (vok[s]) q[s] = (D[s] * io.q[b * n + T.var_orig[NL * s + L]]) * c;
        }
        set_rho(ps && io.resume ? ps[kPersistHdr - 1] : dmin(dmax(st.rho, kRhoMin), kRhoMax));
        IMPC_SEC(kSecSetup);
        int bad = 0;
        IMPC_REP(kSecFactor) bad = factorize();  // (phase-cost experiments only)
        IMPC_SEC(kSecFactor);
        impc_info *out = io.info + b;
        if (bad) {
            _Pragma("unroll") for (int s = 0; s < VS; s++)
                if (vok[s]) io.xo[b * n + T.var_orig[NL * s + L]] = kNan;
            _Pragma("unroll") for (int s = 0; s < VS; s++)
                if (vok[s]) io.yo[b * m + T.var_boxrow[NL * s + L]] = kNan;
            _Pragma("unroll") for (int s = 0; s < GS; s++)
                if (gok[s]) io.yo[b * m + T.gen_row[NL * s + L]] = kNan;
            if (L == 0) {
                out->iter = 0;
                out->status_val = IMPC_NON_CVX;
                out->rho_updates = 0;
                out->setup_exitflag = IMPC_NONCVX_ERROR;
                out->obj_val = kNan;
                out->pri_res = out->dua_res = 0.0;
                out->rho_estimate = R.rho;
            }
            // a first setup that fails its factorisation leaves a defined workspace: the settings'
            // rho and zero iterates (osqp_setup's cold_start; load() zeroed them), so a resume after a
            // matrix update (impc_batch_update_matrices) starts as a fresh setup would; a failed
            // resume keeps the workspace it had (OSQP keeps work->x, z, y when osqp_update_P / _A
            // fails to refactor)
            if (ps && io.resume == 0) write_persist(ps);
            wv.sync();
            return;
        }
        // iterates: zero, then osqp_warm_start (x <- Dinv x, y <- c Einv y, z <- A x)
        if (ps && io.resume && !io.has_ws && st.warm_start) {  // OSQP keeps its iterates between solves
            const double *it = ps + kPersistHdr;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                const int v = NL * s + L;
                x[s] = it[v];
                zb[s] = it[n + v];
                yb[s] = it[2 * n + v];
            }
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (!gok[s]) continue;
                const int g = NL * s + L;
                z[s] = it[3 * n + g];
                y[s] = it[3 * n + T.mg + g];
            }
        } else if (io.has_ws) {
            double D[VS], Eb[VS], Eg[GS];
            load_scal(b, D, Eb, Eg);
            double *xb = xbuf();
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                int ov = T.var_orig[NL * s + L];
                double xv = io.xws[b * n + ov];
                x[s] = st.scaling > 0 ? (1. / D[s]) * xv : xv;
                double yv = io.has_ws == 1 ? io.yws[b * m + T.var_boxrow[NL * s + L]] : 0.0;
                if (st.scaling > 0) {
                    yv = (1. / Eb[s]) * yv;
                    yv *= c;
                }
                yb[s] = yv;
                zb[s] = ab[s] * x[s];
                xb[NL * s + L] = x[s];
            }
            wv.sync();
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (!gok[s]) continue;
                double yv = io.has_ws == 1 ? io.yws[b * m + T.gen_row[NL * s + L]] : 0.0;
                if (st.scaling > 0) {
                    yv = (1. / Eg[s]) * yv;
                    yv *= c;
                }
                y[s] = yv;
                double zz = 0.0;
                _Pragma("unroll") for (int e = 0; e < 4; e++) zz += a[s][e] * xb[gcol(s, e)];
                z[s] = zz;
            }
            wv.sync();
            clear_exchange();
        }
        write_v_products();
        IMPC_SEC(kSecWarm);

        int64_t status = IMPC_UNSOLVED, rho_updates = 0;
        int32_t iter;
        double obj = 0.0, rho_est = R.rho;
        Info inf{};
        int64_t info_iter = 0;
        const int chk = st.check_termination;
        int can_check = 0;
        // counters of the next check / rho update instead of iter % interval
        // the loop's settings read once into registers (the batch's settings live in global memory
        // for a grouped launch: read in the loop they cost a scalar-memory round trip each
        // iteration, after every barrier)
        int32_t max_iter = st.max_iter;  // (dropped to 0 by a failed refactorisation, below)
        const int32_t rho_int = st.adaptive_rho ? st.rho_interval : 0;
        // team-uniform, in scalar registers (io.tlim: the QP's own limit)
        const double tl = wv.uniform(io.tlim ? io.tlim[b] : st.time_limit), tick = st.tick_s;
        const bool tlim = tl > 0;
        int32_t chk_left = chk, rho_left = rho_int;
        // The refactorisation after an adaptive-rho update runs between two passes of the inner
        // iteration loop rather than inside it: the register allocator then places the spills the
        // factorisation's temporaries force around that (rare) call, outside the hot loop.
        bool refac = false;
        iter = 1;
        for (;;) {
            if (refac) {
                refac = false;
                // osqp_solve: a failed rho update ends the solve with exitflag 1.  It leaves the loop
                // through the loop's one exit -- the pass bound drops to 0, the status register
                // carries the mark -- so no second exit edge (and its live values) burdens the
                // register allocation of the passes (round 6: 217.5 -> 213.9 ms per config-3 launch)
                if (factorize()) {
                    max_iter = 0;
                    status = kRefailMark;
                }
                write_v_products();
                IMPC_SEC(kSecFactor);
            }
            // the hot loop: ADMM steps up to the next termination check / rho update (or the end);
            // the check and the update run between two passes of it, so their code and registers
            // sit outside it (the operations are those of one loop, in the same order)
            bool chk_now = false, rho_now = false, stop = false;
            // the pass runs to its next event nxt = min(iterations left, chk_left, rho_left) (counted
            // once per pass, not per iteration); only its last iteration can be a check /
            // rho-update / max_iter one.  osqp_solve's time-limit test sits after the ADMM steps,
            // before can_check is recomputed (so a stop keeps the previous iteration's value); one
            // team-wide decision
            if (iter <= max_iter) {
                int nxt = max_iter - iter + 1;
                if (chk && chk_left < nxt) nxt = chk_left;
                if (rho_int && rho_left < nxt) nxt = rho_left;
                const bool ce = chk && chk_left == nxt, re = rho_int && rho_left == nxt;
                const bool nd_last = ce || iter + nxt - 1 == max_iter || tlim;
                for (int t = 1;; t++) {
                    iterate(t == nxt ? nd_last : tlim);
                    if (tlim) {
                        const double el = wv.max((double)(device_clock() - t0) * tick);
                        if (el >= tl) {
                            status = IMPC_TIME_LIMIT_REACHED;
                            stop = true;
                            if (t > 1) can_check = 0;  // the previous iteration was no check
                            break;
                        }
                    }
                    if (t == nxt) break;
                    iter++;
                }
                if (!stop) {
                    chk_now = ce;
                    rho_now = re;
                    if (chk) chk_left = ce ? chk : chk_left - nxt;
                    if (rho_int) rho_left = re ? rho_int : rho_left - nxt;
                    can_check = chk_now;
                    if (!(chk_now || rho_now)) iter++;
                }
            }
            if (stop || iter > max_iter) break;
            if (can_check) {
                IMPC_SEC_START();
                double D[VS], Eb[VS], Eg[GS];
                load_scal(b, D, Eb, Eg);
                int done = 0;
                IMPC_REP(kSecChecks) {  // (phase-cost experiments only: the check is idempotent)
                    update_info(inf, D, Eb, Eg);
                    done = check_termination(inf, 0, status, obj, D, Eb, Eg);
                }
                info_iter = iter;
                write_v_products();
                IMPC_SEC(kSecChecks);
                if (done) break;
            }
            if (rho_now) {
                if (!can_check) {
                    double D[VS], Eb[VS], Eg[GS];
                    load_scal(b, D, Eb, Eg);
                    update_info(inf, D, Eb, Eg);
                    info_iter = iter;
                    write_v_products();
                }
                double rn = rho_estimate(inf);
                rho_est = rn;
                if ((rn > R.rho * st.adaptive_rho_tolerance) || (rn < R.rho / st.adaptive_rho_tolerance)) {
                    IMPC_SEC(kSecChecks);
                    set_rho(dmin(dmax(rn, kRhoMin), kRhoMax));
                    rho_updates += 1;
                    refac = true;
                }
            }
            iter++;  // this iteration is complete; the next pass starts at the next one
        }
        if (status == kRefailMark) {
            // OSQP 0.6.2 jumps to exit: no termination check, no stored solution (the outputs keep
            // the previous solve's), status stays UNSOLVED, info.iter is the last update_info's;
            // the workspace keeps the new rho and its iterates as they are
            if (ps) write_persist(ps);
            if (L == 0) {
                out->iter = info_iter;
                out->status_val = IMPC_UNSOLVED;
                out->rho_updates = rho_updates;
                out->setup_exitflag = 0;
                out->pri_res = inf.pri_res;
                out->dua_res = inf.dua_res;
                out->rho_estimate = rho_est;
            }
            wv.sync();
            return;
        }
        IMPC_SEC_START();
        double D[VS], Eb[VS], Eg[GS];
        load_scal(b, D, Eb, Eg);
        if (!can_check) {  // post-loop update_info / check, as osqp_solve
            update_info(inf, D, Eb, Eg);
            info_iter = iter - 1;
            check_termination(inf, 0, status, obj, D, Eb, Eg);
        }
        const bool has_sol = status != IMPC_PRIMAL_INFEASIBLE && status != IMPC_PRIMAL_INFEASIBLE_INACCURATE &&
                             status != IMPC_DUAL_INFEASIBLE && status != IMPC_DUAL_INFEASIBLE_INACCURATE &&
                             status != IMPC_NON_CVX;
        if (has_sol) {
            double qf = 0.0;
            _Pragma("unroll") for (int s = 0; s < VS; s++)
                if (vok[s]) qf += (double).5 * pd[s] * x[s] * x[s] + q[s] * x[s];
            obj = wv.sum(qf);
            if (st.scaling > 0) obj *= cinv;
        }
        if (status == IMPC_UNSOLVED) {
            if (!check_termination(inf, 1, status, obj, D, Eb, Eg)) status = IMPC_MAX_ITER_REACHED;
        }
        rho_est = rho_estimate(inf);
        const bool has_sol2 = status != IMPC_PRIMAL_INFEASIBLE && status != IMPC_PRIMAL_INFEASIBLE_INACCURATE &&
                              status != IMPC_DUAL_INFEASIBLE && status != IMPC_DUAL_INFEASIBLE_INACCURATE &&
                              status != IMPC_NON_CVX;
        const bool scaled = st.scaling > 0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            int v = NL * s + L;
            io.xo[b * n + T.var_orig[v]] = has_sol2 ? (scaled ? D[s] * x[s] : x[s]) : kNan;
            double yv = has_sol2 ? (scaled ? (Eb[s] * yb[s]) * cinv : yb[s]) : kNan;
            io.yo[b * m + T.var_boxrow[v]] = yv;
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (!gok[s]) continue;
            double yv = has_sol2 ? (scaled ? (Eg[s] * y[s]) * cinv : y[s]) : kNan;
            io.yo[b * m + T.gen_row[NL * s + L]] = yv;
        }
        if (ps) {  // the workspace after osqp_solve: rho and the scaled iterates -- zero when the
                   // solve ended without a solution (store_solution's cold_start, auxil.c)
            if (!has_sol2) {
                _Pragma("unroll") for (int s = 0; s < VS; s++) x[s] = zb[s] = yb[s] = 0.0;
                _Pragma("unroll") for (int s = 0; s < GS; s++) z[s] = y[s] = 0.0;
            }
            write_persist(ps);
        }
        if (L == 0 && io.qpt) {
            io.qpt[2 * b] = t0;
            io.qpt[2 * b + 1] = device_clock();
        }
        if (L == 0) {
            out->iter = info_iter;
            out->status_val = status;
            out->rho_updates = rho_updates;
            out->setup_exitflag = 0;
            out->obj_val = obj;
            out->pri_res = inf.pri_res;
            out->dua_res = inf.dua_res;
            out->rho_estimate = rho_est;
        }
        wv.sync();
#if defined(IMPC_SECTION_PROF) && defined(__HIP_DEVICE_COMPILE__)
        IMPC_SEC(kSecOutput);
        if (L == 0 && io.sec) {
            sec_acc[kSecIters] = (uint64_t)info_iter;
            _Pragma("unroll") for (int i = 0; i < kSecCount; i++) atomicAdd(io.sec + i, (unsigned long long)sec_acc[i]);
        }
#endif
    }
};

}  // namespace impc
