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
#ifndef IMPC_DUP
#define IMPC_DUP -1
#endif
#define IMPC_REP(X) for (int rep_ = 0; rep_ < (IMPC_DUP == (X) ? 2 : 1); rep_++)

#ifndef IMPC_HWRW  // recursion wave from the waves' SIMD placement: +0.5-1 % (profiles/r02/exp/README.md,
#define IMPC_HWRW 1  // profiles/r03/exp/README.md); re-validated on the GPU suite in round 3, on
#endif
#ifndef IMPC_NOCHUNK
#define IMPC_NOCHUNK 1
#endif

#ifndef IMPC_LDSBAR  // LDS-only barriers inside the ADMM iteration (GpuTeam::lsync)
#define IMPC_LDSBAR 0
#endif
#ifndef IMPC_PRIO  // raise the wave priority of the stage-recursion wavefront during its sweeps
#define IMPC_PRIO 0
#endif
#ifndef IMPC_PRIO_INV  // the inverse: every wave at this priority, the recursion wavefront drops to 0
#define IMPC_PRIO_INV 0  // during its sweeps (the parallel phases win the SIMD's issue arbitration)
#endif
#if IMPC_PRIO
#define IMPC_PRIO_HI() __builtin_amdgcn_s_setprio(IMPC_PRIO)
#define IMPC_PRIO_LO() __builtin_amdgcn_s_setprio(0)
#elif IMPC_PRIO_INV && defined(__HIP_DEVICE_COMPILE__)
#define IMPC_PRIO_HI() __builtin_amdgcn_s_setprio(0)
#define IMPC_PRIO_LO() __builtin_amdgcn_s_setprio(IMPC_PRIO_INV)
#else
#define IMPC_PRIO_HI() ((void)0)
#define IMPC_PRIO_LO() ((void)0)
#endif
#ifndef IMPC_RFOLD  // fold the recursion's subtraction into the first product (rstep): measured slower, off
#define IMPC_RFOLD 0
#endif
#ifndef IMPC_PSTRIDE_PAD
#define IMPC_PSTRIDE_PAD 1
#endif
#ifndef IMPC_TWIST  // twisted (two-ended) block elimination on the default horizon (WaveQP::TWIST):
#define IMPC_TWIST 0  // built, parity green, measured slower (profiles/r03/exp/README.md), off
#endif
#ifndef IMPC_TWOPQ  // twisted chains: one address register per prefetch (no ds_read2 merging)
#define IMPC_TWOPQ 0
#endif
#ifndef IMPC_PAIR  // pair-blocked stage recursions on the default horizon (WaveLds::PAIR): built,
#define IMPC_PAIR 0  // measured slower (profiles/r02/exp/README.md), off
#endif
// Scheduling hint for the parallel phases' LDS reads: under the kernel's register pressure the
// machine scheduler otherwise issues them one ds_read2 at a time, each followed by its own
// lgkmcnt wait (S3 = 7 serialised LDS round trips); this asks for the phase's reads first, then
// its arithmetic, so the round trips overlap.
#ifndef IMPC_SGB
#define IMPC_SGB 1
#endif
#if IMPC_SGB && defined(__HIP_DEVICE_COMPILE__)
#define IMPC_LOADS_FIRST(NR, NV)                            \
    do {                                                    \
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0); \
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0); \
    } while (0)
#else
#define IMPC_LOADS_FIRST(NR, NV) ((void)0)
#endif
#ifndef IMPC_GJ  // stage inverses by Gauss-Jordan with 2x2 (2) or 1x1 (1) pivots, or Cholesky +
#define IMPC_GJ 2  // L^-1 + L^-T L^-1 (0)
#endif
#ifndef IMPC_PCAP_REG  // pair sweeps: keep the stage results in registers until the sweep ends (1)
#define IMPC_PCAP_REG 0  // or store each one as it is produced (0: measured faster, fewer spills)
#endif
// Round-3 iteration-latency experiments (tools/exp.sh, profiles/r03/exp/README.md "Branch-free
// general rows and the other phase / sweep variants"): only IMPC_GFREE paid (-1.9..-2.2 % kernel
// time, identical iterations) and is on; the rest were measured slower alone or beside it, off.
#ifndef IMPC_GFREE  // general-row update / products without per-slot branches (the GS slots'
#define IMPC_GFREE 1  // chains interleave; an empty slot computes zeros into the discard slot)
#endif
#ifndef IMPC_GUNROLL  // rhs column gather: the groups of a compile-time group count issued at once
#define IMPC_GUNROLL 1  // (dispatch on CG4) instead of one LDS round trip per group of four (on, with
#endif                  // IMPC_SDC: -1.3 %; measured neutral before the branch-free phases)
#ifndef IMPC_TREE  // S1 / S3 / S5 / general-row dot products as two to four partial chains
#define IMPC_TREE 0
#endif
#ifndef IMPC_PFREE  // rhs / S1 / S3 / S5 without the per-lane variable-kind branches (on: -0.6 %)
#define IMPC_PFREE 1
#endif
#ifndef IMPC_DPPRED  // team max / sum (checks, infeasibility tests): the in-wave butterfly by DPP /
#define IMPC_DPPRED 1  // permlane / swizzle exchanges instead of ds_bpermute (bitwise the same; on: -1.6 %)
#endif
#ifndef IMPC_CHKRED  // termination check: both infeasibility tests' first stages in one team reduction
#define IMPC_CHKRED 1  // (bitwise the same values; on)
#endif
#ifndef IMPC_CMASK  // sweep captures selected by compile-time lane masks (SGPR constants; on: -0.3..-0.6 %)
#define IMPC_CMASK 1
#endif
#ifndef IMPC_OBASE  // S1 / S3 / S5 reads from one opaque per-lane base with immediate offsets
#define IMPC_OBASE 0  // (measured +1.3 %, off)
#endif
#ifndef IMPC_SDC  // default-horizon instances: the products stride as a compile-time constant, so
#define IMPC_SDC 1  // the gather's reads take immediate offsets (on)
#endif
#ifndef IMPC_VMAX  // the iteration's projections by v_max_f64 / v_min_f64 instead of compare + selects
#define IMPC_VMAX 1  // (on: -1.2 %; with PFREE -1.7 %)
#endif
#ifndef IMPC_LOOPC  // the inner loop counts to the pass's next event (check / rho update / max_iter)
#define IMPC_LOOPC 1  // computed once per pass, instead of per-iteration countdown bookkeeping
#endif
#ifndef IMPC_NDT  // the check-iteration deltas: update phase instantiated with and without them
#define IMPC_NDT 0
#endif
#ifndef IMPC_HCAP  // default-horizon sweeps: every step's output kept in its own register (no
#define IMPC_HCAP 0  // per-step capture select), stored by one lane row / column after the sweep
#endif
#ifndef IMPC_SSTORE  // default-horizon sweeps: every stage result stored as produced by all lanes
#define IMPC_SSTORE 0  // (same value, same address per output index) instead of register captures
#endif
#ifndef IMPC_SFOLD  // stage recursions carry (c, S) with a = c - S: the next product is
#define IMPC_SFOLD 0  // fma(-f, S, f c), one dependent operation per step fewer
#endif

template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

struct WaveTables {
    int32_t n, m, mg, N, W, CG, nnzP, nnzA;
    const int32_t *var_orig, *var_pdiag, *var_boxrow, *var_boxpos;
    const int32_t *gen_row, *gen_col, *gen_pos, *colg, *term_ptr, *term;
    int32_t HS;               // heavy columns (second products tier), MpcStructure::HS; 0: one tier
    const int32_t *col_hid;   // [n] heavy-column index or -1 (stage order)
    int32_t T1r;              // first-tier rows: cg4(CG) (one tier) or kProdTier1 (two tiers)
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
    // iterates x, z (box), y (box), z (general), y (general).  resume = 1: scale with the stored
    // factors (the same D, E, c and scaled P, A as the first setup), start from the stored rho and
    // iterates, and -- when q_updated -- scale q as osqp_update_lin_cost does ((D q) c).
    double *persist = nullptr;
    int32_t resume = 0, q_updated = 0;
    // per-QP time limits [B] (impc_batch_set_time_limits: each solveTraj call sets its own), or
    // nullptr for the settings' time_limit
    const double *tlim = nullptr;
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

// LDS doubles per wave for (VS, GS)
template <int NL, int VS, int GS>
struct WaveLds {
    static constexpr int NMAX = NL * VS;
    static constexpr int WMAX = (NMAX + 5) / 13 - 1;       // max control stages
    // stage count whose recursions are fully unrolled (the reference's default horizon N = 20
    // for the one-variable-per-lane shape, N = 40 for the long-horizon shape)
    static constexpr int WSPEC = VS == 1 ? 19 : 39;
    // exchange vector length: zero tail past NMAX, and room for the factorisation scratch
    // (the sweeps' two-steps-ahead prefetches read at most 13 (W + 4) + 8 past the start), and
    // room for the factorisation's dense stage scratch (FA .. DIAGX below)
    static constexpr int NP = (NMAX + 48 > (779 + NMAX + 3) / 4) ? NMAX + 48 : (779 + NMAX + 3) / 4;
    static constexpr int F_OFF = 0;                         // [WMAX][64]
    static constexpr int R_OFF = F_OFF + WMAX * 64;         // rbuf
    static constexpr int T_OFF = R_OFF + NP;                // tbuf
    static constexpr int E_OFF = T_OFF + NP;                // ebuf
    static constexpr int X_OFF = E_OFF + NP;                // xbuf
    static constexpr int RED_OFF = X_OFF + NP;              // team reduction scratch
    static constexpr int JUNK_OFF = RED_OFF + 64;           // per-lane discard slots [NL]
    static constexpr int GSLOT_OFF = JUNK_OFF + NL;         // int16 [4 NL GS]: general entry -> product slot
    // Chunked stage recursions (default horizon of the one-variable-per-lane shape): the W + 1
    // stages split into 4 chunks [S(c), S(c+1)), one per wavefront; the chunk-entry operators
    // Psi_k (forward) / Phi_k (backward) and two cross-chunk products live here.
    static constexpr bool CHUNK = VS == 1 && NL == 256 && !IMPC_NOCHUNK;
    static IMPC_WF constexpr int S(int c) { return (c * (WSPEC + 1) + 2) / 4; }
    static constexpr int NPF = WSPEC + 1 - S(1), NPB = S(3);   // Psi_k, k in [S1, W]; Phi_k, k in [0, S3)
    static constexpr int PSI_OFF = GSLOT_OFF + NL * GS;     // [NPF + NPB + 2][64], row-major 8x8
    static constexpr int PSI_N = CHUNK ? 64 * (NPF + NPB + 2) : 0;
    // One-variable-per-lane shape: the Ruiz scaling vectors D, E and the ADMM deltas of the
    // termination checks live here (the long-horizon shape keeps them in HBM / registers: its LDS
    // is full).  Layout of each: [var slots NMAX][box rows NMAX][general slots NL GS].
#ifndef IMPC_OFFCHIP_SCL  // experiment: D, E in the per-QP HBM scratch and the deltas in registers also
#define IMPC_OFFCHIP_SCL 0  // for the one-variable-per-lane shape (frees 2 x VEC_N doubles of LDS)
#endif
    static constexpr bool ONCHIP = VS == 1 && !IMPC_OFFCHIP_SCL;
    static constexpr int VEC_N = 2 * NMAX + NL * GS;
    // Pair-blocked stage recursions (default horizon of the one-variable-per-lane shape): the
    // 8-dim recursions step over two stages at a time along the even stages, with the products
    // H_k = F_{k+1} F_k and M_k = F_{k+1} G_k[:, 8:] (k = 0, 2, .., WSPEC - 3) formed by the
    // factorisation; the odd stages come off the chain as independent side products.
    static constexpr bool PAIR = VS == 1 && NL == 256 && IMPC_PAIR && !CHUNK;
    static constexpr int NH = (WSPEC - 1) / 2;              // chain steps (9 at WSPEC = 19)
    static_assert(!PAIR || (WSPEC & 1), "pair blocking needs an odd stage count");
    static constexpr int H_OFF = PSI_OFF + PSI_N;           // [NH][64] H_k, recursion layout
    static constexpr int M_OFF = H_OFF + (PAIR ? 64 * NH : 0);  // [NH][40] M_k, row-major 8 x 5
    static constexpr int SCL_OFF = M_OFF + (PAIR ? 40 * NH : 0);  // D, E (scaling)
    static constexpr int DLT_OFF = SCL_OFF + (ONCHIP ? VEC_N : 0);  // dx, dy (check iterations)
    // Twisted (two-ended) elimination of the default horizon (IMPC_TWIST, WaveQP::TWIST): the middle
    // stage's state lanes' G_{KM-1}[:, 8:] rows ([8][5]; their cp registers hold Abar^-1 Bbar' rows)
    static constexpr bool TW = VS == 1 && NL == 256 && IMPC_TWIST && !CHUNK && !PAIR;
    static constexpr int MID_OFF = DLT_OFF + (ONCHIP ? VEC_N : 0);
    // ... and the coupling-row table (int32 per general-row slot: (upper entry << 16) | upper
    // column for rows coupling stages k, k + 1 > KM, else -1), set per batch by load_tables
    static constexpr int CPL_OFF = MID_OFF + (TW ? 40 : 0);
    static constexpr int P_OFF = CPL_OFF + (TW ? NL * GS / 2 : 0);  // products, column-slot layout (size below)
    // chunk-boundary exchange of the recursions (inside the team reduction scratch, past red[0..3])
    static constexpr int XF_OFF = RED_OFF + 8;              // forward: a^_{S(c+1)-1}, c = 0..2
    static constexpr int XB_OFF = RED_OFF + 32;             // backward: x^_{S(c)}, c = 1..3
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
    static constexpr IMPC_WF int stride(int n) { return ((n + 63) & ~63) + IMPC_PSTRIDE_PAD; }
    // the factorisation uses it as (4g + e) scratch followed by the general rows' rho (RHOG_P)
    static IMPC_WF int hsp(int HS) { return HS + 1; }  // second-tier row length
    static IMPC_WF int p_size(int CG, int n, int HS, int mg, int T1r) {
        const int c = T1r * stride(n) + (cg4(CG) > T1r ? (cg4(CG) - T1r) * hsp(HS) : 0), f = 5 * mg;
        return c > f ? c : f;
    }
    static IMPC_WF int p_size(const WaveTables &T) { return p_size(T.CG, T.n, T.HS, T.mg, T.T1r); }
    static IMPC_WF int size(const WaveTables &T) { return P_OFF + p_size(T) + 8; }
    // factorisation aliases (inside R..X region and the products buffer)
    static constexpr int FA = R_OFF, FL = FA + 169, FI = FL + 169, FB = FI + 169, FG = FB + 104, FE = FG + 104,
                         DIAGX = FE + 64;
    // twisted elimination: Acheck_{k+1}^{-1}[:8, :8] of the stage eliminated last from the bottom
    static constexpr int FEB = DIAGX + NMAX;
    // general rows' rho during the factorisation: products region + 4 mg
    static_assert(FEB + 64 <= RED_OFF, "factorisation scratch does not fit");
};

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

// a * b rounded on its own (never contracted into a following add), so the symmetric
// cross-lane sums that consume it give bitwise-identical results in every lane of a group
IMPC_WF double prod_nc(double a, double b) {
    // contract(off) drops the multiply's contraction flag, so it never fuses into the add that
    // consumes it (an empty volatile asm would do the same but also pin the instruction order)
#pragma clang fp contract(off)
    return a * b;
}

// WF: the stage count W fixed at compile time (LD::WSPEC, the default horizon: every stage loop
// and LDS offset becomes a constant and no runtime-W code path shares the kernel's registers), or 0
// for any W read from the tables.
// TIER: the batch uses the two-tier products layout (WaveLds, T1r = kProdTier1); a one-tier
// batch (T1r = CG4) runs the TIER = false instance, whose gathers are the plain CG4-row loops.
template <class WV, int NL, int VS, int GS, int WF = 0, bool TIER = false>
struct WaveQP {
    using LD = WaveLds<NL, VS, GS>;
    static_assert(WF == 0 || WF == LD::WSPEC, "WF is 0 or the shape's default horizon");
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
    // Twisted (two-ended) block elimination, default horizon of the one-variable-per-lane shape:
    // stages 0 .. KM-1 are eliminated top-down (the Schur complements Ahat_k, F_k as in the
    // one-ended scheme), stages W .. KM+1 bottom-up (Acheck_k = M_kk - Bbar_k' Acheck_{k+1}^-1[:8,:8]
    // Bbar_k, H_k = (Acheck_k^-1 Bbar_k')[:8, :]), and the middle stage KM takes both
    // (Abar = M - E_{KM-1} - Bbar_KM' Acheck_{KM+1}^-1[:8,:8] Bbar_KM).  Each solve then runs its
    // 8-dim recursions as two concurrent chains of (W - 1) / 2 steps on two wavefronts -- top-down
    // and bottom-up, then outward from the middle -- instead of one chain of W steps.
    static constexpr bool TWIST = LD::TW && WF == LD::WSPEC;
    static constexpr int KM = (LD::WSPEC - 1) / 2;
    // (the coupling-row table lives in LDS, WaveLds::CPL_OFF: kept in registers it was spilled and
    // reloaded from scratch every iteration)
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

    // IMPC_OBASE: a phase's per-lane LDS base formed as one opaque offset, so its reads take
    // immediate offsets (a ds_read2 offset reaches 255 doubles) instead of one address add each
    IMPC_WF const double *lds_at(int off) const {
#if IMPC_OBASE
        opaque(off);
#endif
        return lds + off;
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
        else return io.scal + b * (int64_t)(2 * T.n + T.mg);
    }

    IMPC_WF double *F() { return lds + LD::F_OFF; }
    IMPC_WF double *rbuf() { return lds + LD::R_OFF; }
    IMPC_WF double *tbuf() { return lds + LD::T_OFF; }
    IMPC_WF double *ebuf() { return lds + LD::E_OFF; }
    IMPC_WF double *xbuf() { return lds + LD::X_OFF; }
    IMPC_WF double *pbuf() { return lds + LD::P_OFF; }

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
#if IMPC_PFREE
            // the branch-free phases read a slot's factor rows whether or not it holds a variable
            _Pragma("unroll") for (int cc = 0; cc < 13; cc++) ainv[s][cc] = 0.0;
            _Pragma("unroll") for (int cc = 0; cc < 8; cc++) cp[s][cc] = 0.0;
#endif
            if (vok[s]) {
                int ov = T.var_orig[v];
                q[s] = io.q[bn + ov];
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
        if constexpr (TWIST) {
            // coupling rows: entries in stages k and k + 1 > KM, one of them in stage k + 1
            // (MpcStructure::twist_ok, checked on the host) -- the upper entry, last in column order
            int32_t *cpl = (int32_t *)(lds + LD::CPL_OFF);
            for (int g = w.lane(); g < NL * GS; g += NL) {
                int hi = -1, lo = 1 << 30, eu = 0, cu = 0;
                for (int e = 0; e < 4 && g < T.mg; e++) {
                    const int c = T.gen_col[4 * g + e];
                    if (c < 0) continue;
                    const int st_ = c / 13;
                    if (st_ > hi) hi = st_, eu = e, cu = c;
                    lo = st_ < lo ? st_ : lo;
                }
                cpl[g] = g < T.mg && hi == lo + 1 && hi > KM ? (eu << 16) | cu : -1;
            }
        }
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
        // (IMPC_SDC: the compile-time horizon's products stride, n = 13 (WF + 1) - 5, so the gather's
        // reads take immediate offsets instead of per-read address arithmetic)
        const int C4 = c4_, sd = (IMPC_SDC && WF) ? LD::stride(13 * (WF + 1) - 5) : sd_;
        double s = 0.0;
        if constexpr (!TIER) {
            (void)h;
#if IMPC_GUNROLL
            // the same sum, every read of the column issued before the first add (C4 is uniform)
            switch (C4) {
                case 4: return gather_n<1>(pb, sd);
                case 8: return gather_n<2>(pb, sd);
                case 12: return gather_n<3>(pb, sd);
                case 16: return gather_n<4>(pb, sd);
                case 20: return gather_n<5>(pb, sd);
                default: break;
            }
#endif
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
        for (int it = 0; it < st.scaling; it++) {
            // |A| entries of general rows -> products buffer
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (gok[s])
                    _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = fabs(a[s][e]);
            }
            wv.sync();
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
            // cost normalisation
            double psum = 0.0, qn = 0.0;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (vok[s]) {
                    psum += fabs(pd[s]);
                    qn = dmax(fabs(q[s]), qn);
                }
            }
            double ct = wv.sum(psum) / (double)n;
            qn = wv.max(qn);
            qn = qn < kMinScaling ? 1.0 : qn;
            qn = qn > kMaxScaling ? kMaxScaling : qn;
            ct = dmax(ct, qn);
            ct = ct < kMinScaling ? 1.0 : ct;
            ct = ct > kMaxScaling ? kMaxScaling : ct;
            ct = 1. / ct;
            if (ps) {
                if (io.resume)
                    ct = ps[it];
                else if (L == 0)
                    ps[it] = ct;
            }
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                pd[s] *= ct;
                q[s] *= ct;
            }
            c *= ct;
            wv.sync();
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
    IMPC_WF int factorize() {
        if constexpr (TWIST) return factorize_tw();
        const int n = T.n, W = Wst(), N = W + 1;
        double *w = pbuf(), *rhog = pbuf() + 4 * T.mg, *diagx = lds + LD::DIAGX;
        const bool pair = LD::PAIR && W == LD::WSPEC;
        double *A = lds + LD::FA, *Li = lds + LD::FL, *Ai = lds + LD::FI, *Bb = lds + LD::FB, *G = lds + LD::FG,
               *E = lds + LD::FE, *Fm = F();
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
        for (int k = 0; k < N; k++) {
            const int sz = k < W ? 13 : 8;
            // assemble M_kk and Bbar_k
            for (int d = L; d < kStageDests; d += NL) {
                const bool isB = d >= 169;
                if (isB && k == W) continue;
                const int dd = isB ? d - 169 : d;
                const int r = dd / 13, cc = dd % 13;
                double val = 0.0;
                if (isB || (r < sz && cc < sz)) {
                    const int32_t t0 = T.term_ptr[(int64_t)k * kStageDests + d];
                    const int32_t t1 = T.term_ptr[(int64_t)k * kStageDests + d + 1];
                    for (int32_t t = t0; t < t1; t++) {
                        int32_t code = T.term[t];
                        int32_t g = code >> 4, e = (code >> 2) & 3, f = code & 3;
                        val += rhog[g] * w[4 * g + e] * w[4 * g + f];
                    }
                    if (!isB && r == cc) val += diagx[13 * k + r];
#if IMPC_GJ
                    if (!isB && k > 0 && r < 8 && cc < 8) val -= E[8 * r + cc];  // Schur complement
#endif
                }
                if (isB)
                    Bb[dd] = val;
                else
                    A[dd] = val;
            }
            wv.sync();
            IMPC_SEC(kSecFAsm);
#if IMPC_GJ
            // Ahat_k^{-1} by Gauss-Jordan elimination: one element per lane, the pivots in order
            // (SPD, no pivoting needed; a non-positive-definite pivot flags the factorisation as
            // failed, as a failed Cholesky did), ping-pong between two LDS buffers so every step
            // is one barrier.  The last step writes the lower triangle to both halves of Ai
            // (exactly symmetric).
            {
                double *src = A, *dst = Li;
                const int gi = L / 13, gc = L % 13;
                const bool act = L < 169 && gi < sz && gc < sz;
#if IMPC_GJ == 2
                // two pivots per step (2x2 block pivot Q = P^-1, P = S[J][J], J = {j, j+1}):
                //   D[J][J] = Q, D[J][c] = Q S[J][c], D[i][J] = -S[i][J] Q,
                //   D[i][c] = S[i][c] - (S[i][J] Q) S[J][c]; a non-PD pivot block flags failure
                for (int j = 0; j < sz; j += 2) {
                    const bool two = j + 1 < sz, last = j + (two ? 2 : 1) >= sz;
                    if (act) {
                        const int i = last && gc > gi ? gc : gi, c = last && gc > gi ? gi : gc;
                        double v;
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
                        (last ? Ai : dst)[13 * gi + gc] = v;
                    }
                    wv.sync();
                    double *t = src;
                    src = dst;
                    dst = t;
                }
#else
                for (int j = 0; j < sz; j++) {
                    const bool last = j == sz - 1;
                    if (act) {
                        const int i = last && gc > gi ? gc : gi, c = last && gc > gi ? gi : gc;
                        const double p = src[13 * j + j];
                        if (!(p > 0.0)) bad = 1;
                        const double r = 1.0 / p;
                        double v;
                        if (i == j && c == j)
                            v = r;
                        else if (i == j)
                            v = src[13 * j + c] * r;
                        else if (c == j)
                            v = -(src[13 * i + j] * r);
                        else
                            v = src[13 * i + c] - (src[13 * i + j] * r) * src[13 * j + c];
                        (last ? Ai : dst)[13 * gi + gc] = v;
                    }
                    wv.sync();
                    double *t = src;
                    src = dst;
                    dst = t;
                }
#endif
            }
#else
            if (k > 0) {
                if (L < 64) {
                    int i = L >> 3, j = L & 7;
                    A[13 * i + j] -= E[8 * i + j];
                }
                wv.sync();
            }
            // Cholesky of A (sz x sz, stride 13)
            for (int j = 0; j < sz; j++) {
                if (L == 0) {
                    double dj = A[13 * j + j];
                    if (!(dj > 0.0)) bad = 1;
                    A[13 * j + j] = sqrt(dj);
                }
                wv.sync();
                if (L > j && L < sz) A[13 * L + j] /= A[13 * j + j];
                wv.sync();
                const int rem = sz - 1 - j, cnt = rem * (rem + 1) / 2;
                for (int p = L; p < cnt; p += NL) {
                    // p -> (i, cc) with j < cc <= i < sz, row-major over i
                    int i = j + 1, off = p;
                    while (off >= i - j) {
                        off -= i - j;
                        i++;
                    }
                    int cc = j + 1 + off;
                    A[13 * i + cc] -= A[13 * i + j] * A[13 * cc + j];
                }
                wv.sync();
            }
            // Linv column by column (lane = column)
            if (L < sz) {
                const int cc = L;
                Li[13 * cc + cc] = 1.0 / A[13 * cc + cc];
                for (int i = cc + 1; i < sz; i++) {
                    double s = 0.0;
                    for (int t = cc; t < i; t++) s += A[13 * i + t] * Li[13 * t + cc];
                    Li[13 * i + cc] = -s / A[13 * i + i];
                }
            }
            wv.sync();
            // Ainv = Linv' Linv
            for (int p = L; p < sz * sz; p += NL) {
                int r = p / sz, cc = p % sz;
                int t0 = r > cc ? r : cc;
                double s = 0.0;
                for (int t = t0; t < sz; t++) s += Li[13 * t + r] * Li[13 * t + cc];
                Ai[13 * r + cc] = s;
            }
            wv.sync();
#endif
            _Pragma("unroll") for (int s = 0; s < VS; s++)
                if (vok[s] && vs_[s] == k)
                    _Pragma("unroll") for (int cc = 0; cc < 13; cc++) ainv[s][cc] = cc < sz ? Ai[13 * vr_[s] + cc] : 0.0;
            if (k < W) {
                for (int p = L; p < 104; p += NL) {
                    int i = p / 13, cc = p % 13;
                    double s = 0.0;
                    for (int t = 0; t < 13; t++) s += Bb[13 * i + t] * Ai[13 * t + cc];
                    G[p] = s;
                }
                wv.sync();
                if (L < 64) {
                    int i = L >> 3, j = L & 7;
                    double s = 0.0;
                    for (int t = 0; t < 13; t++) s += G[13 * i + t] * Bb[13 * j + t];
                    E[8 * i + j] = s;
                    // recursion layout: lane (i,j) of step k reads F_k[j][i] when the column index
                    // sits on i (k even, or pair_col_i(k) when pair-blocked), F_k[i][j] otherwise
                    const bool ci = pair ? pair_col_i(k) : !(k & 1);
                    Fm[64 * k + 8 * i + j] = ci ? G[13 * j + i] : G[13 * i + j];
                } else if (pair && L < 104 && !(k & 1) && k < 2 * LD::NH) {
                    // G_k[:, 8:] of the even stages, for M_k = F_{k+1} G_k[:, 8:] once F_{k+1} exists
                    const int p = L - 64, q = p / 5, cc = p % 5;
                    lds[LD::M_OFF + 40 * (k >> 1) + p] = G[13 * q + 8 + cc];
                }
                _Pragma("unroll") for (int s = 0; s < VS; s++) {
                    if (!vok[s]) continue;
                    if (vs_[s] == k && vr_[s] >= 8)
                        _Pragma("unroll") for (int j = 0; j < 8; j++) cp[s][j] = G[13 * j + vr_[s]];
                    if (vs_[s] == k + 1 && vr_[s] < 8)
                        _Pragma("unroll") for (int j = 0; j < 8; j++) cp[s][j] = j < 5 ? G[13 * vr_[s] + 8 + j] : 0.0;
                }
                wv.sync();
            }
            IMPC_SEC(kSecFDense);
        }
        _Pragma("unroll") for (int s = 0; s < VS; s++)
            if (vok[s] && vs_[s] == 0 && vr_[s] < 8)
                _Pragma("unroll") for (int j = 0; j < 8; j++) cp[s][j] = 0.0;
        if constexpr (LD::CHUNK)
            if (W == LD::WSPEC) chunk_operators();
        if constexpr (LD::PAIR)
            if (pair) pair_operators();
        bad = (int)wv.max((double)bad);  // set by lane 0 only: team-wide, so every wavefront agrees
        clear_exchange();
        zero_products();  // the (4g + e) factorisation scratch shared the products region
        (void)n;
        return bad;
    }

    // ---------------------------------------------------- pair-blocked stage recursions
    // Forward: a_{k+1} = t_{k+1} - F_k a_k.  Over two stages, a_{k+2} = u_{k+2} + H_k a_k with
    // u_{k+2} = t_{k+2} - F_{k+1} t_{k+1} (formed in S1) and H_k = F_{k+1} F_k, so the dependent
    // chain runs over the even stages (a_0 -> a_2 -> .. -> a_{W-1}: (W - 1) / 2 steps) and each step
    // also yields the odd stage a_{k+1} = t_{k+1} - F_k a_k from the same input: an independent
    // second reduction that fills the chain's latency.  Backward likewise: x_k = v_k + H_k' x_{k+2}
    // with v_k = e_k - F_k' e_{k+1} (the V phase) and the side x_{k+1} = e_{k+1} - F_{k+1}' x_{k+2}.
    // Layout: the vector of even stage k = 2c sits at index i when c is even (j when odd); the
    // matrices of stages k and k + 1 are stored with their column index on that index
    // (pair_col_i), so every step reduces over its input's index and lands on the other one.
    static IMPC_WF constexpr bool pair_col_i(int k) { return ((k >> 1) & 1) == 0; }
    // F_k[r][c] in the pair layout
    IMPC_WF double Fp(int k, int r, int c) const {
        return pair_col_i(k) ? lds[LD::F_OFF + 64 * k + 8 * c + r] : lds[LD::F_OFF + 64 * k + 8 * r + c];
    }

    // H_k = F_{k+1} F_k (in the layout of step k) and M_k = F_{k+1} G_k[:, 8:] (row-major; the M
    // slots hold G_k[:, 8:] until here), k = 0, 2, .., 2 (NH - 1)
    IMPC_WF void pair_operators() {
        wv.sync();
        double *Hm = lds + LD::H_OFF, *Mm = lds + LD::M_OFF;
        for (int p = L; p < 64 * LD::NH; p += NL) {
            const int c = p >> 6, e = p & 63, k = 2 * c, i = e >> 3, j = e & 7;
            const int r = pair_col_i(k) ? j : i, col = pair_col_i(k) ? i : j;
            double a = 0.0;
            for (int q = 0; q < 8; q++) a += Fp(k + 1, r, q) * Fp(k, q, col);
            Hm[p] = a;
        }
        constexpr int NM = 40 * LD::NH, MR = (NM + NL - 1) / NL;
        double mv[MR];
        _Pragma("unroll") for (int t = 0; t < MR; t++) {
            const int p = L + NL * t;
            double a = 0.0;
            if (p < NM) {
                const int c = p / 40, e = p % 40, r = e / 5, cc = e % 5;
                for (int q = 0; q < 8; q++) a += Fp(2 * c + 1, r, q) * Mm[40 * c + 5 * q + cc];
            }
            mv[t] = a;
        }
        wv.sync();
        _Pragma("unroll") for (int t = 0; t < MR; t++)
            if (L + NL * t < NM) Mm[L + NL * t] = mv[t];
        wv.sync();
    }

    // Stage s's value r sits in the 8 lanes that share its index.  IMPC_PCAP_REG = 0: the lane
    // whose other index is 0 stores it to buf right away (the others to their discard slot).
    // IMPC_PCAP_REG = 1: the lane whose other index is s mod 8 keeps it in slot s / 8 of the array
    // for values on index i (ci) or j (cj) and pcap_store writes them after the sweep (no LDS
    // store per step, but 6 more live doubles: measured slower through register spills).
    static constexpr int PQ = (LD::WSPEC + 8) / 8;
    template <bool OUT_I>
    IMPC_WF void pcap(double (&ci)[PQ], double (&cj)[PQ], double r, int s, int i, int j, double *buf, double *junk) {
#if IMPC_PCAP_REG
        (void)buf, (void)junk;
        if (OUT_I) {
            if (j == (s & 7)) ci[s >> 3] = r;
        } else {
            if (i == (s & 7)) cj[s >> 3] = r;
        }
#else
        (void)ci, (void)cj;
        if (OUT_I)
            *(j == 0 ? buf + 13 * s + i : junk) = r;
        else
            *(i == 0 ? buf + 13 * s + j : junk) = r;
#endif
    }
    // store the captured stages s0 .. s1 (stage s at 13 s + its index; out_i(s): on index i)
    template <class OUTI>
    IMPC_WF void pcap_store(const double (&ci)[PQ], const double (&cj)[PQ], double *buf, int s0, int s1, int i,
                            int j, OUTI out_i) {
        if (!IMPC_PCAP_REG) return;
        double *junk = lds + LD::JUNK_OFF + lane_o();
        _Pragma("unroll") for (int q = 0; q < PQ; q++) {
            const int si = 8 * q + j, sj = 8 * q + i;
            *((si >= s0 && si <= s1 && out_i(si)) ? buf + 13 * si + i : junk) = ci[q];
            *((sj >= s0 && sj <= s1 && !out_i(sj)) ? buf + 13 * sj + j : junk) = cj[q];
        }
    }

    // S2, pair-blocked (W = WSPEC): from a_0 = t_0 (index i), stages 1 .. W into rb; tb holds
    // u_k on the even stages k >= 2 (S1).  Operands are loaded two steps ahead.
    IMPC_WF void fwd_pair(const double *tb, double *rb) {
        constexpr int NH = LD::NH, W = LD::WSPEC;
        constexpr bool last_on_i = (NH & 1) == 0;  // input index of the final side step
        const double *Fm = F(), *Hm = lds + LD::H_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double *junk = lds + LD::JUNK_OFF + lo;
        double ci[PQ], cj[PQ];
        if (IMPC_PCAP_REG) _Pragma("unroll") for (int q = 0; q < PQ; q++) ci[q] = cj[q] = 0.0;
        double a = tb[i];
        // operands of step c: H_{2c}, F_{2c}, u_{2c+2}, t_{2c+1} (u, t on the step's output index);
        // step NH is the final side step (F_{W-1}, t_W)
        auto ld = [&](int c, double &h, double &f, double &u, double &t) {
            const int k = 2 * c, xo = (c & 1) == 0 ? j : i;
            if (c < NH) {
                h = Hm[64 * c + l];
                f = Fm[64 * k + l];
                u = tb[13 * (k + 2) + xo];
                t = tb[13 * (k + 1) + xo];
            } else if (c == NH) {
                f = Fm[64 * (W - 1) + l];
                t = tb[13 * W + xo];
            }
        };
        double h0 = 0, f0 = 0, u0 = 0, t0 = 0, h1 = 0, f1 = 0, u1 = 0, t1 = 0;
        ld(0, h0, f0, u0, t0);
        ld(1, h1, f1, u1, t1);
        _Pragma("unroll") for (int c = 0; c < NH; c++) {
            const int k = 2 * c;
            const bool on_i = (c & 1) == 0;  // this step's input index (its outputs: the other)
            const double h = h0, f = f0, u = u0, t = t0;
            h0 = h1, f0 = f1, u0 = u1, t0 = t1;
            ld(c + 2, h1, f1, u1, t1);
            const double pc = prod_nc(h, a), ps = prod_nc(f, a);
            double rc, rs;
            if (on_i) {
                rc = wv.sum_stride8(pc);
                rs = wv.sum_stride8(ps);
            } else {
                rc = wv.sum_contig8(pc);
                rs = wv.sum_contig8(ps);
            }
            const double as = t - rs;  // a_{k+1}
            a = u + rc;                // a_{k+2}
            if (on_i) {
                pcap<false>(ci, cj, as, k + 1, i, j, rb, junk);
                pcap<false>(ci, cj, a, k + 2, i, j, rb, junk);
            } else {
                pcap<true>(ci, cj, as, k + 1, i, j, rb, junk);
                pcap<true>(ci, cj, a, k + 2, i, j, rb, junk);
            }
        }
        const double ps = prod_nc(f0, a);
        const double aw = t0 - (last_on_i ? wv.sum_stride8(ps) : wv.sum_contig8(ps));
        pcap<!last_on_i>(ci, cj, aw, W, i, j, rb, junk);
        pcap_store(ci, cj, rb, 1, W, i, j, [](int s) { return s == W ? !last_on_i : (((s - 1) >> 1) & 1) == 1; });
    }

    // S4, pair-blocked (W = WSPEC): from x_W = e_W, stages W-1 .. 0 into xb; eb holds v_k on the
    // even stages k <= W - 3 (V phase).  Operands are loaded two steps ahead.
    IMPC_WF void bwd_pair(const double *eb, double *xb) {
        constexpr int NH = LD::NH, W = LD::WSPEC;
        constexpr bool last_on_i = (NH & 1) == 0;  // x_{W-1} sits on index i (else j)
        const double *Fm = F(), *Hm = lds + LD::H_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double *junk = lds + LD::JUNK_OFF + lo;
        double ci[PQ], cj[PQ];
        if (IMPC_PCAP_REG) _Pragma("unroll") for (int q = 0; q < PQ; q++) ci[q] = cj[q] = 0.0;
        // operands of step c (x_{2c+2} -> x_{2c}, x_{2c+1}): H_{2c}, F_{2c+1}, v_{2c}, e_{2c+1}, on
        // the step's output index (i for even c)
        auto ld = [&](int c, double &h, double &f, double &v, double &e) {
            if (c < 0) return;
            const int xo = (c & 1) == 0 ? i : j;
            h = Hm[64 * c + l];
            f = Fm[64 * (2 * c + 1) + l];
            v = eb[13 * (2 * c) + xo];
            e = eb[13 * (2 * c + 1) + xo];
        };
        double h0 = 0, f0 = 0, v0 = 0, e0 = 0, h1 = 0, f1 = 0, v1 = 0, e1 = 0;
        ld(NH - 1, h0, f0, v0, e0);
        ld(NH - 2, h1, f1, v1, e1);
        // x_{W-1} = e_{W-1} - F_{W-1}' x_W, reduced over x_W's index
        double x;
        {
            const double xW = eb[13 * W + (last_on_i ? j : i)], ew = eb[13 * (W - 1) + (last_on_i ? i : j)];
            const double p = prod_nc(Fm[64 * (W - 1) + l], xW);
            x = ew - (last_on_i ? wv.sum_contig8(p) : wv.sum_stride8(p));
            pcap<last_on_i>(ci, cj, x, W - 1, i, j, xb, junk);
        }
        _Pragma("unroll") for (int c = NH - 1; c >= 0; c--) {
            const bool out_i = (c & 1) == 0;
            const double h = h0, f = f0, v = v0, e = e0;
            h0 = h1, f0 = f1, v0 = v1, e0 = e1;
            ld(c - 2, h1, f1, v1, e1);
            const double pc = prod_nc(h, x), ps = prod_nc(f, x);
            double rc, rs;
            if (out_i) {  // input on index j
                rc = wv.sum_contig8(pc);
                rs = wv.sum_contig8(ps);
            } else {
                rc = wv.sum_stride8(pc);
                rs = wv.sum_stride8(ps);
            }
            const double xs = e - rs;  // x_{2c+1}
            x = v + rc;                // x_{2c}
            if (out_i) {
                pcap<true>(ci, cj, xs, 2 * c + 1, i, j, xb, junk);
                pcap<true>(ci, cj, x, 2 * c, i, j, xb, junk);
            } else {
                pcap<false>(ci, cj, xs, 2 * c + 1, i, j, xb, junk);
                pcap<false>(ci, cj, x, 2 * c, i, j, xb, junk);
            }
        }
        pcap_store(ci, cj, xb, 0, W - 1, i, j, [](int s) { return s == W - 1 ? last_on_i : ((s >> 1) & 1) == 0; });
    }

    // ------------------------------------------------------- chunked stage recursions
    // The forward recursion a_{k+1} = t_{k+1} - F_k a_k is linear in the chunk's entry value: for a
    // chunk [S, E] entered from a_{S-1}, a_k = a^_k + Psi_k a_{S-1} with a^ the recursion started
    // from a^_S = t_S, Psi_S = -F_{S-1}, Psi_{k+1} = -F_k Psi_k.  Likewise backward, x_k = x^_k +
    // Phi_k x_{E+1} with x^_E = e_E, Phi_E = -F_E', Phi_k = -F_k' Phi_{k+1}.  Each wavefront runs
    // its chunk's local recursion (phase A, S(c+1) - S(c) - 1 dependent steps), the boundary values
    // meet in LDS, then every wavefront forms its entry value from the earlier chunks' boundary
    // values (at most two independent 8x8 products, with the precomputed Psi_{S3-1} Psi_{S2-1} /
    // Phi_{S1} Phi_{S2}) and corrects its stages with independent 8x8 products (phase B).  The
    // dependent chain drops from W steps to 4 + 2.  Psi / Phi depend only on the factorisation.
    IMPC_WF static double Fget(const double *Fm, int k, int r, int c) {  // F_k[r][c] (parity layout)
        return (k & 1) ? Fm[64 * k + 8 * r + c] : Fm[64 * k + 8 * c + r];
    }
    IMPC_WF double *PF(int k) { return lds + LD::PSI_OFF + 64 * (k - LD::S(1)); }  // Psi_k, row-major
    IMPC_WF double *PB(int k) { return lds + LD::PSI_OFF + 64 * (LD::NPF + k); }   // Phi_k
    IMPC_WF double *PIF() { return lds + LD::PSI_OFF + 64 * (LD::NPF + LD::NPB); }
    IMPC_WF double *PIB() { return PIF() + 64; }

    IMPC_WF void chunk_operators() {
        const double *Fm = F();
        constexpr int CL = LD::S(4) - LD::S(3) > LD::S(1) ? LD::S(4) - LD::S(3) : LD::S(1);
        static_assert(LD::S(2) - LD::S(1) <= CL && LD::S(3) - LD::S(2) <= CL, "chunk length");
        for (int st = 0; st < CL; st++) {
            for (int p = L; p < 6 * 64; p += NL) {
                const int mtx = p >> 6, e = p & 63, r = e >> 3, cc = e & 7;
                if (mtx < 3) {  // Psi_k of chunk c = mtx + 1
                    const int c = mtx + 1, k = LD::S(c) + st;
                    if (k >= LD::S(c + 1)) continue;
                    double v;
                    if (st == 0) {
                        v = -Fget(Fm, k - 1, r, cc);
                    } else {
                        const double *Pp = PF(k - 1);
                        double a = 0.0;
                        for (int q = 0; q < 8; q++) a += Fget(Fm, k - 1, r, q) * Pp[8 * q + cc];
                        v = -a;
                    }
                    PF(k)[e] = v;
                } else {  // Phi_k of chunk c = mtx - 3
                    const int c = mtx - 3, k = LD::S(c + 1) - 1 - st;
                    if (k < LD::S(c)) continue;
                    double v;
                    if (st == 0) {
                        v = -Fget(Fm, k, cc, r);
                    } else {
                        const double *Pn = PB(k + 1);
                        double a = 0.0;
                        for (int q = 0; q < 8; q++) a += Fget(Fm, k, q, r) * Pn[8 * q + cc];
                        v = -a;
                    }
                    PB(k)[e] = v;
                }
            }
            wv.sync();
        }
        for (int p = L; p < 128; p += NL) {
            const int e = p & 63, r = e >> 3, cc = e & 7;
            const double *X = p < 64 ? PF(LD::S(3) - 1) : PB(LD::S(1));
            const double *Y = p < 64 ? PF(LD::S(2) - 1) : PB(LD::S(2));
            double a = 0.0;
            for (int q = 0; q < 8; q++) a += X[8 * r + q] * Y[8 * q + cc];
            (p < 64 ? PIF() : PIB())[e] = a;
        }
        wv.sync();
    }

    // y = M v on the wavefront's 8x8 grid (M row-major in LDS): v at index i -> y at index j
    // (l: the lane within the wavefront, formed once by the caller)
    IMPC_WF double mv_i(const double *M, double v, int l) {
        return wv.sum_stride8(prod_nc(M[8 * (l & 7) + (l >> 3)], v));
    }
    // v at index j -> y at index i
    IMPC_WF double mv_j(const double *M, double v, int l) { return wv.sum_contig8(prod_nc(M[l], v)); }

    // Phase A forward, chunk [K0, K1): a^_{K0} = t_{K0}; stores a^_k, K0 < k < K1, to rb and
    // a^_{K1-1} to xo (XO).  Stage k's vector sits at index i (k even) / j (k odd).
    template <int K0, int K1, bool XO>
    IMPC_WF void fwd_chunk(const double *tb, double *rb, double *xo) {
        const double *Fm = F();
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double *junk = lds + LD::JUNK_OFF + lo;
        constexpr int NS = K1 - 1 - K0;
        double a = tb[13 * K0 + ((K0 & 1) ? j : i)];
        double cs = 0.0, cc = 0.0;  // step m kept by lane i == m (strided steps) / j == m (contiguous)
        _Pragma("unroll") for (int k = K0; k < K1 - 1; k++) {
            const double f = Fm[64 * k + l], t = tb[13 * (k + 1) + ((k & 1) ? i : j)];
            if ((k & 1) == 0) {
                a = rstep<true>(f, t, a);
                cs = i == k - K0 ? a : cs;
            } else {
                a = rstep<false>(f, t, a);
                cc = j == k - K0 ? a : cc;
            }
        }
        const int ke = K0 + i, ko = K0 + j;
        *((i < NS && !(ke & 1)) ? rb + 13 * (ke + 1) + j : junk) = cs;
        *((j < NS && (ko & 1)) ? rb + 13 * (ko + 1) + i : junk) = cc;
        if constexpr (XO) {
            if constexpr (((K1 - 1) & 1) == 0)
                *(j == 0 ? xo + i : junk) = a;
            else
                *(i == 0 ? xo + j : junk) = a;
        }
    }

    // Phase B forward, chunk C >= 1: entry a_{S(C)-1} from the boundary values, then the stages
    template <int C>
    IMPC_WF void fwd_fix(const double *tb, double *rb) {
        const double *X = lds + LD::XF_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double *junk = lds + LD::JUNK_OFF + lo;
        double v = X[8 * (C - 1) + j];
        if constexpr (C >= 2) v = v + mv_i(PF(LD::S(C) - 1), X[8 * (C - 2) + i], l);
        if constexpr (C == 3) v = v + mv_i(PIF(), X[i], l);
        constexpr int K0 = LD::S(C), K1 = LD::S(C + 1);
        double r[K1 - K0];
        _Pragma("unroll") for (int k = K0; k < K1; k++) r[k - K0] = mv_j(PF(k), v, l);
        _Pragma("unroll") for (int k = K0; k < K1; k++) {
            const double ah = k == K0 ? tb[13 * k + i] : rb[13 * k + i];
            *(j == 0 ? rb + 13 * k + i : junk) = ah + r[k - K0];
        }
    }

    // Phase A backward, chunk [KB, KT]: x^_{KT} = e_{KT}; stores x^_k, KB <= k < KT, to xb and
    // x^_{KB} to xo (XO)
    template <int KB, int KT, bool XO>
    IMPC_WF void bwd_chunk(const double *eb, double *xb, double *xo) {
        const double *Fm = F();
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double *junk = lds + LD::JUNK_OFF + lo;
        constexpr int NS = KT - KB;
        double x = eb[13 * KT + ((KT & 1) ? j : i)];
        double cs = 0.0, cc = 0.0;
        _Pragma("unroll") for (int k = KT - 1; k >= KB; k--) {
            const double f = Fm[64 * k + l], e = eb[13 * k + ((k & 1) ? j : i)];
            if (k & 1) {
                x = rstep<true>(f, e, x);
                cs = i == KT - 1 - k ? x : cs;
            } else {
                x = rstep<false>(f, e, x);
                cc = j == KT - 1 - k ? x : cc;
            }
        }
        const int ks = KT - 1 - i, kc = KT - 1 - j;
        *((i < NS && (ks & 1)) ? xb + 13 * ks + j : junk) = cs;
        *((j < NS && !(kc & 1)) ? xb + 13 * kc + i : junk) = cc;
        if constexpr (XO) {
            if constexpr ((KB & 1) == 0)
                *(j == 0 ? xo + i : junk) = x;
            else
                *(i == 0 ? xo + j : junk) = x;
        }
    }

    // Phase B backward, chunk C <= 2: entry x_{S(C+1)}, then the stages
    template <int C>
    IMPC_WF void bwd_fix(const double *eb, double *xb) {
        const double *X = lds + LD::XB_OFF;  // x^_{S(c)} at X + 8 (c - 1)
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double *junk = lds + LD::JUNK_OFF + lo;
        double v = X[8 * C + j];
        if constexpr (C <= 1) v = v + mv_i(PB(LD::S(C + 1)), X[8 * (C + 1) + i], l);
        if constexpr (C == 0) v = v + mv_i(PIB(), X[16 + i], l);
        constexpr int K0 = LD::S(C), K1 = LD::S(C + 1);
        double r[K1 - K0];
        _Pragma("unroll") for (int k = K0; k < K1; k++) r[k - K0] = mv_j(PB(k), v, l);
        _Pragma("unroll") for (int k = K0; k < K1; k++) {
            const double xh = k == K1 - 1 ? eb[13 * k + i] : xb[13 * k + i];
            *(j == 0 ? xb + 13 * k + i : junk) = xh + r[k - K0];
        }
    }

    IMPC_WF void fwd_chunked(const double *tb, double *rb) {
        double *X = lds + LD::XF_OFF;
        const int w = L >> 6;
        if (w == 0) fwd_chunk<LD::S(0), LD::S(1), true>(tb, rb, X);
        else if (w == 1) fwd_chunk<LD::S(1), LD::S(2), true>(tb, rb, X + 8);
        else if (w == 2) fwd_chunk<LD::S(2), LD::S(3), true>(tb, rb, X + 16);
        else fwd_chunk<LD::S(3), LD::S(4), false>(tb, rb, X);
        wv.sync();
        if (w == 1) fwd_fix<1>(tb, rb);
        else if (w == 2) fwd_fix<2>(tb, rb);
        else if (w == 3) fwd_fix<3>(tb, rb);
    }

    IMPC_WF void bwd_chunked(const double *eb, double *xb) {
        double *X = lds + LD::XB_OFF;
        const int w = L >> 6;
        if (w == 0) bwd_chunk<LD::S(0), LD::S(1) - 1, false>(eb, xb, X);
        else if (w == 1) bwd_chunk<LD::S(1), LD::S(2) - 1, true>(eb, xb, X);
        else if (w == 2) bwd_chunk<LD::S(2), LD::S(3) - 1, true>(eb, xb, X + 8);
        else bwd_chunk<LD::S(3), LD::S(4) - 1, true>(eb, xb, X + 16);
        wv.sync();
        if (w == 0) bwd_fix<0>(eb, xb);
        else if (w == 1) bwd_fix<1>(eb, xb);
        else if (w == 2) bwd_fix<2>(eb, xb);
    }

    // One step of a stage recursion on the 8x8 lane grid: returns c - R(F v), R the strided
    // (STRIDE) or contiguous 8-lane sum.
    template <bool STRIDE>
    IMPC_WF double rstep(double f, double c, double v) {
#if IMPC_RFOLD
        // c - sum_q f_q v_q with c folded into the products: the lane at reduction index 0 forms
        // fma(f, -v, c), the others f (-v); the select acts on the prefetched c, off the chain,
        // and the chain loses its final subtraction.
        const int l = L & 63;
        const bool own = STRIDE ? (l >> 3) == 0 : (l & 7) == 0;
        const double p = __builtin_fma(f, -v, own ? c : 0.0);
        return STRIDE ? wv.sum_stride8(p) : wv.sum_contig8(p);
#else
        const double p = prod_nc(f, v);
        return c - (STRIDE ? wv.sum_stride8(p) : wv.sum_contig8(p));
#endif
    }

    // IMPC_SFOLD: a step's state is (c, S) with v = c - S (c the step's t / e value, S its 8-lane
    // sum); the next step's product f v is formed as fma(-f, S, f c), with f c off the chain, so
    // the subtraction leaves the dependent chain (v itself is formed only for the stores)
    template <bool STRIDE>
    IMPC_WF double fstep(double f, double c, double S) {
        const double p = __builtin_fma(-f, S, prod_nc(f, c));
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
    // j = l & 7; lane l = 8 i + j of the recursion wavefront): IMPC_CMASK selects by that constant
    // mask in an SGPR pair instead of a v_cmp per step
    template <bool OI>
    IMPC_WF static void capm(double (&c)[CQ], double r, int m, int other) {
#if IMPC_CMASK && defined(__HIP_DEVICE_COMPILE__)
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

    // S2 body: a_{k+1} = t_{k+1} - F_k a_k for k = 0..W-1 (WC = W, or 0 for a runtime W).
    template <int WC>
    IMPC_WF void fwd_sweep(const double *tb, double *rb, int W) {
        const double *Fm = lds + LD::F_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;  // opaque: see lane_o
        double a = tb[i];
        // (F, t) of the next even / odd step, loaded two steps ahead (reads past the last stage
        // stay inside the LDS buffers and are never used)
        double fe = Fm[l], te = tb[13 + j], fo = Fm[64 + l], to = tb[26 + i];
#if IMPC_SFOLD
        double S = 0.0;  // a_0 = t_0 - 0
#endif
        // one step: a <- t - R(f a); SFOLD: (a, S) <- (t, R(fma(-f, S, f a))), the value t - S
        auto step = [&](auto stride, double f, double t) -> double {
#if IMPC_SFOLD
            S = fstep<decltype(stride)::value>(f, a, S);
            a = t;
            return t - S;
#else
            a = rstep<decltype(stride)::value>(f, t, a);
            return a;
#endif
        };
        using ST = BoolC<true>;
        using SC = BoolC<false>;
        if constexpr (WC > 0) {
            double c0[CQ], c1[CQ];
            _Pragma("unroll") for (int q = 0; q < CQ; q++) c0[q] = c1[q] = 0.0;
#if IMPC_SSTORE
            // each stage stored as produced by all 64 lanes: the 8 lanes of an output index hold
            // bitwise the same value and write it to the same address (no lane mask, no capture)
            double *rj = rb + j, *ri = rb + i;
#elif IMPC_HCAP
            double hist[WC];  // every step's output in registers (constant indices), stored after
#endif
            _Pragma("unroll") for (int k = 0; k < WC; k += 2) {
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
#if IMPC_SSTORE
                rj[13 * (k + 1)] = step(ST{}, f0, t0);
#elif IMPC_HCAP
                hist[k] = step(ST{}, f0, t0);
#else
                capm<true>(c0, step(ST{}, f0, t0), k, i);
#endif
                if (k + 1 < WC) {
                    const double f1 = fo, t1 = to;
                    fo = Fm[64 * (k + 3) + l];
                    to = tb[13 * (k + 4) + i];
#if IMPC_SSTORE
                    ri[13 * (k + 2)] = step(SC{}, f1, t1);
#elif IMPC_HCAP
                    hist[k + 1] = step(SC{}, f1, t1);
#else
                    capm<false>(c1, step(SC{}, f1, t1), k + 1, j);
#endif
                }
            }
#if IMPC_HCAP
            // even steps' outputs (index j) from the lanes i == 0, odd steps' (index i) from j == 0
            if (i == 0) _Pragma("unroll") for (int k = 0; k < WC; k += 2) rb[13 * (k + 1) + j] = hist[k];
            if (j == 0) _Pragma("unroll") for (int k = 1; k < WC; k += 2) rb[13 * (k + 1) + i] = hist[k];
#elif !IMPC_SSTORE
            cap_store<true>(c0, c1, rb, WC, true, i, j);
#endif
        } else {
            // one lane per element writes, the rest write to discard slots (no divergent branch)
            double *junk = lds + LD::JUNK_OFF + lo;
            const bool wri = j == 0, wrj = i == 0;
            for (int k = 0; k < W; k += 2) {
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
                *(wrj ? rb + 13 * (k + 1) + j : junk) = step(ST{}, f0, t0);
                if (k + 1 >= W) break;
                const double f1 = fo, t1 = to;
                fo = Fm[64 * (k + 3) + l];
                to = tb[13 * (k + 4) + i];
                *(wri ? rb + 13 * (k + 2) + i : junk) = step(SC{}, f1, t1);
            }
        }
    }

    // S4 body for a first step k = W-1 of parity ODD: steps alternate strided (odd k) and
    // contiguous (even k) reductions; x_k sits at index j (odd k) / i (even k).  WC as above.
    template <bool ODD, int WC>
    IMPC_WF void bwd_sweep(const double *eb, double *xb, int W) {
        const double *Fm = lds + LD::F_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        if constexpr (WC > 0) W = WC;
        // x_W: W = (W-1)+1 has the opposite parity of the first step
        double x = eb[13 * W + (ODD ? i : j)];
        const int k1 = W - 2 > 0 ? W - 2 : 0;
        double fa = Fm[64 * (W - 1) + l], ea = eb[13 * (W - 1) + (ODD ? j : i)];
        double fb = Fm[64 * k1 + l], ebv = eb[13 * k1 + (ODD ? i : j)];
#if IMPC_SFOLD
        double S = 0.0;  // x_W = e_W - 0
#endif
        auto step = [&](auto stride, double f, double e) -> double {
#if IMPC_SFOLD
            S = fstep<decltype(stride)::value>(f, x, S);
            x = e;
            return e - S;
#else
            x = rstep<decltype(stride)::value>(f, e, x);
            return x;
#endif
        };
        using SA = BoolC<ODD>;
        using SB = BoolC<!ODD>;
        if constexpr (WC > 0) {
            double c0[CQ], c1[CQ];
            _Pragma("unroll") for (int q = 0; q < CQ; q++) c0[q] = c1[q] = 0.0;
#if IMPC_SSTORE
            double *xe = xb + (ODD ? j : i), *xo = xb + (ODD ? i : j);  // even / odd steps' outputs
#elif IMPC_HCAP
            double hist[WC];
#endif
            _Pragma("unroll") for (int m = 0; m < WC; m += 2) {
                const int k = WC - 1 - m;
                const int k2 = k - 2 > 0 ? k - 2 : 0, k3 = k - 3 > 0 ? k - 3 : 0;
                const double f0 = fa, e0 = ea;
                fa = Fm[64 * k2 + l];
                ea = eb[13 * k2 + (ODD ? j : i)];
#if IMPC_SSTORE
                xe[13 * k] = step(SA{}, f0, e0);
#elif IMPC_HCAP
                hist[m] = step(SA{}, f0, e0);
#else
                capm<ODD>(c0, step(SA{}, f0, e0), m, ODD ? i : j);
#endif
                if (m + 1 < WC) {
                    const double f1 = fb, e1 = ebv;
                    fb = Fm[64 * k3 + l];
                    ebv = eb[13 * k3 + (ODD ? i : j)];
#if IMPC_SSTORE
                    xo[13 * (k - 1)] = step(SB{}, f1, e1);
#elif IMPC_HCAP
                    hist[m + 1] = step(SB{}, f1, e1);
#else
                    capm<!ODD>(c1, step(SB{}, f1, e1), m + 1, ODD ? j : i);
#endif
                }
            }
#if IMPC_HCAP
            // step m is stage WC - 1 - m; even steps' outputs at index j (ODD) / i, odd steps' at the other
            if ((ODD ? i : j) == 0)
                _Pragma("unroll") for (int m = 0; m < WC; m += 2) xb[13 * (WC - 1 - m) + (ODD ? j : i)] = hist[m];
            if ((ODD ? j : i) == 0)
                _Pragma("unroll") for (int m = 1; m < WC; m += 2) xb[13 * (WC - 1 - m) + (ODD ? i : j)] = hist[m];
#elif !IMPC_SSTORE
            cap_store<ODD>(c0, c1, xb, WC, false, i, j);
#endif
        } else {
            double *junk = lds + LD::JUNK_OFF + lo;
            const bool wri = j == 0, wrj = i == 0;
            for (int k = W - 1; k >= 0; k -= 2) {
                const int k2 = k - 2 > 0 ? k - 2 : 0, k3 = k - 3 > 0 ? k - 3 : 0;
                const double f0 = fa, e0 = ea;
                fa = Fm[64 * k2 + l];
                ea = eb[13 * k2 + (ODD ? j : i)];
                *(ODD ? (wrj ? xb + 13 * k + j : junk) : (wri ? xb + 13 * k + i : junk)) = step(SA{}, f0, e0);
                if (k - 1 < 0) break;
                const double f1 = fb, e1 = ebv;
                fb = Fm[64 * k3 + l];
                ebv = eb[13 * k3 + (ODD ? i : j)];
                *(ODD ? (wri ? xb + 13 * (k - 1) + i : junk) : (wrj ? xb + 13 * (k - 1) + j : junk)) = step(SB{}, f1, e1);
            }
        }
    }

    // v = rho z - y products of the general rows for the next rhs
    IMPC_WF void write_v_products() {
        double *pb = pbuf();
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (IMPC_GFREE || gok[s]) {  // an empty slot writes a zero product to the discard slot
                double vv = rhog_(s) * z[s] - y[s];
                _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = a[s][e] * vv;
            }
        }
        wv.lsync();
    }

    // --------------------------------------------------------------- one ADMM iteration
    IMPC_WF void iterate(bool need_delta) {
        if constexpr (TWIST) {
            iterate_tw(need_delta);
            return;
        }
        const int W = Wst();
        const bool pair = LD::PAIR && W == LD::WSPEC;
        double *rb = rbuf(), *tb = tbuf(), *eb = ebuf(), *xb = xbuf();
        const double sigma = sig_;
        IMPC_REP(kSecRhs) {
            // rhs = sigma x - q + A' v   (stage order; IMPC_PFREE: an empty slot's iterates, bounds
            // and column are zero, so it writes 0)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!IMPC_PFREE && !vok[s]) continue;
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
            // S1: t_k = r_k[:8] - G_{k-1}[:, 8:] r_{k-1}[8:]  (IMPC_PFREE: every lane; a stage-0 or
            // empty slot has zero coupling coefficients, a control lane's t lands in a slot nothing
            // reads)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!IMPC_PFREE && (!vok[s] || vr_[s] >= 8)) continue;
                int v = NL * s + L;
                double t = rb[v];
                if (IMPC_PFREE || vs_[s] > 0) {
                    // (PFREE, stage 0: the zero tail of the x exchange, not LDS below rb -- past the
                    // horizon's last F block that is another QP's data or uninitialised)
                    const double *rp = lds_at(!IMPC_PFREE || vs_[s] > 0 ? LD::R_OFF + 13 * (vs_[s] - 1) + 8 : LD::X_OFF + LD::NMAX);
                    double rv[5];
                    _Pragma("unroll") for (int cc = 0; cc < 5; cc++) rv[cc] = rp[cc];
                    IMPC_LOADS_FIRST(5, 12);
#if IMPC_TREE
                    double tb2 = cp[s][1] * rv[1];
                    tb2 += cp[s][3] * rv[3];
                    t -= cp[s][0] * rv[0];
                    t -= cp[s][2] * rv[2];
                    t -= cp[s][4] * rv[4];
                    t -= tb2;
#else
                    _Pragma("unroll") for (int cc = 0; cc < 5; cc++) t -= cp[s][cc] * rv[cc];
#endif
                }
                if constexpr (LD::PAIR) {
                    // pair-blocked forward: on the even stages k >= 2 the chain takes
                    // u_k = t_k - F_{k-1} t_{k-1} = t_k - F_{k-1} r_{k-1}[:8] + M_{k-2} r_{k-2}[8:]
                    int k = vs_[s];
                    if (pair && k >= 2 && !(k & 1)) {
                        int r = vr_[s];
                        opaque(k);  // per-lane addresses formed here, not hoisted out of the ADMM loop
                        opaque(r);
                        const double *r1 = rb + 13 * (k - 1), *r2 = rb + 13 * (k - 2) + 8;
                        const double *Mk = lds + LD::M_OFF + 40 * ((k - 2) >> 1) + 5 * r;
                        double fa = 0.0, fb = 0.0, mb = 0.0;
                        _Pragma("unroll") for (int q = 0; q < 4; q++) fa += Fp(k - 1, r, q) * r1[q];
                        _Pragma("unroll") for (int q = 4; q < 8; q++) fb += Fp(k - 1, r, q) * r1[q];
                        _Pragma("unroll") for (int cc = 0; cc < 5; cc++) mb += Mk[cc] * r2[cc];
                        t = (t - (fa + fb)) + mb;
                    }
                }
                tb[v] = t;
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
            if (L < 8) rb[L] = tb[L];
            if (LD::CHUNK && W == LD::WSPEC) {
                if constexpr (LD::CHUNK) fwd_chunked(tb, rb);
            } else if ((L >> 6) == rw) {
                IMPC_PRIO_HI();
                if constexpr (LD::PAIR) {
                    if (pair) fwd_pair(tb, rb);
                    else if (W == LD::WSPEC)
                        fwd_sweep<LD::WSPEC>(tb, rb, W);
                    else
                        fwd_sweep<0>(tb, rb, W);
                } else if (W == LD::WSPEC)
                    fwd_sweep<LD::WSPEC>(tb, rb, W);
                else
                    fwd_sweep<0>(tb, rb, W);
                IMPC_PRIO_LO();
            }
            wv.lsync();
        }
        IMPC_SEC(kSecFwd);
        IMPC_REP(kSecS3) {
            // S3: e_k = Ahat_k^{-1} rhat_k
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!IMPC_PFREE && !vok[s]) continue;
                const double *rk = lds_at(LD::R_OFF + 13 * vs_[s]);
                double rv[13];
                _Pragma("unroll") for (int cc = 0; cc < 13; cc++) rv[cc] = rk[cc];
                IMPC_LOADS_FIRST(7, 20);
#if IMPC_TREE
                double ea[4];
                _Pragma("unroll") for (int u = 0; u < 4; u++) ea[u] = ainv[s][u] * rv[u];
                _Pragma("unroll") for (int cc = 4; cc < 13; cc++) ea[cc & 3] += ainv[s][cc] * rv[cc];
                const double e = (ea[0] + ea[1]) + (ea[2] + ea[3]);
#else
                double e = 0.0;
                _Pragma("unroll") for (int cc = 0; cc < 13; cc++) e += ainv[s][cc] * rv[cc];
#endif
                eb[NL * s + L] = e;
            }
            wv.lsync();
            if constexpr (LD::PAIR) {
                // V: v_k = e_k - F_k' e_{k+1} on the even stages k <= W - 3 (pair-blocked backward
                // chain), in place: each lane reads only the odd stage k + 1 besides its own value
                if (pair) {
                    _Pragma("unroll") for (int s = 0; s < VS; s++) {
                        int k = vs_[s], r = vr_[s];
                        if (!vok[s] || r >= 8 || (k & 1) || k > W - 3) continue;
                        opaque(k);
                        opaque(r);
                        const double *e1 = eb + 13 * (k + 1);
                        double va = 0.0, vb = 0.0;
                        _Pragma("unroll") for (int q = 0; q < 4; q++) va += Fp(k, q, r) * e1[q];
                        _Pragma("unroll") for (int q = 4; q < 8; q++) vb += Fp(k, q, r) * e1[q];
                        eb[NL * s + L] = eb[NL * s + L] - (va + vb);
                    }
                    wv.lsync();
                }
            }
        }
        IMPC_SEC(kSecS3);
        IMPC_REP(kSecBwd) {
            // S4: backward 8-dim recursion x_k[:8] = e_k[:8] - F_k' x_{k+1}[:8] on the same grid and
            // stored layout: even steps reduce over j (contiguous), odd steps over i (strided).
            if (L < 8) xb[13 * W + L] = eb[13 * W + L];
            if (LD::CHUNK && W == LD::WSPEC) {
                if constexpr (LD::CHUNK) bwd_chunked(eb, xb);
            } else if ((L >> 6) == rw) {
                IMPC_PRIO_HI();
                if (LD::PAIR && pair) {
                    if constexpr (LD::PAIR) bwd_pair(eb, xb);
                } else if (W == LD::WSPEC)
                    bwd_sweep<((LD::WSPEC - 1) & 1) != 0, LD::WSPEC>(eb, xb, W);
                else if ((W - 1) & 1)
                    bwd_sweep<true, 0>(eb, xb, W);
                else
                    bwd_sweep<false, 0>(eb, xb, W);
                IMPC_PRIO_LO();
            }
            wv.lsync();
        }
        IMPC_SEC(kSecBwd);
        IMPC_REP(kSecS5) {
            // S5: controls x_k[8:] = e_k[8:] - G_k[:, 8:]' x_{k+1}[:8]  (IMPC_PFREE: every lane, the
            // state lanes' and empty slots' results to their discard slots)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!IMPC_PFREE && (!vok[s] || vr_[s] < 8)) continue;
                const double *xn = lds_at(LD::X_OFF + 13 * (vs_[s] + 1));
                double t = eb[NL * s + L];
                double xv[8];
                _Pragma("unroll") for (int j = 0; j < 8; j++) xv[j] = xn[j];
                IMPC_LOADS_FIRST(5, 16);
#if IMPC_TREE
                double tb2 = cp[s][1] * xv[1];
                _Pragma("unroll") for (int j = 3; j < 8; j += 2) tb2 += cp[s][j] * xv[j];
                _Pragma("unroll") for (int j = 0; j < 8; j += 2) t -= cp[s][j] * xv[j];
                t -= tb2;
#else
                _Pragma("unroll") for (int j = 0; j < 8; j++) t -= cp[s][j] * xv[j];
#endif
#if IMPC_PFREE
                *(vok[s] && vr_[s] >= 8 ? xb + NL * s + L : lds + LD::JUNK_OFF + L) = t;
#else
                xb[NL * s + L] = t;
#endif
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS5);
        update_and_products(need_delta);
    }

    // project_z (auxil.h): min(max(v, l), u) as c_max / c_min, or (IMPC_VMAX) as v_max_f64 /
    // v_min_f64 -- the same value except the sign of a zero when v equals a zero bound
    IMPC_WF static double clampz(double v, double l, double u) {
#if IMPC_VMAX
        return __builtin_fmin(__builtin_fmax(v, l), u);
#else
        return dmin(dmax(v, l), u);
#endif
    }

    IMPC_WF void update_and_products(bool need_delta) {
#if IMPC_NDT
        if (need_delta)
            update_and_products_t<true>();
        else
            update_and_products_t<false>();
#else
        update_and_products_t<false>(need_delta);
#endif
    }

    // update_x and the box rows (update_z / project / update_y), the general rows, and the
    // products of the next rhs (the end of every ADMM iteration).  ND: the check-iteration deltas
    // are written (IMPC_NDT: a compile-time instance each; otherwise the runtime flag nd).
    template <bool ND>
    IMPC_WF void update_and_products_t(bool nd = ND) {
        const bool need_delta = ND || nd;
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
        // general rows (IMPC_GFREE: an empty slot's columns are the zero tail of the x exchange, its
        // A values, bounds and iterates zero, so it computes zeros, without a per-slot branch)
        double xg[GS][4];
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            _Pragma("unroll") for (int e = 0; e < 4; e++) xg[s][e] = (IMPC_GFREE || gok[s]) ? xb[gcol(s, e)] : 0.0;
        }
        IMPC_LOADS_FIRST(4 * GS, 8 * GS);
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (!IMPC_GFREE && !gok[s]) continue;
#if IMPC_TREE
            const double zt = (a[s][0] * xg[s][0] + a[s][1] * xg[s][1]) + (a[s][2] * xg[s][2] + a[s][3] * xg[s][3]);
#else
            double zt = 0.0;
            _Pragma("unroll") for (int e = 0; e < 4; e++) zt += a[s][e] * xg[s][e];
#endif
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

    // ------------------------------------------------------ twisted elimination (TWIST)
    // One 8-dim chain of S steps on the recursion grid (lane l = 8i + j of the calling wavefront):
    //   v <- c - B v  (TR: c - B' v),  B = the stored block of stage k(m) = K0 + D m.
    // F slot k holds its block with the column index on i for even k (factorize), so a plain
    // product of an even stage reduces over i (input at i, output at j) and a transposed one over j,
    // odd stages the other way round: consecutive steps alternate without moving data.  c of step m
    // is read at cb + 13 (k + CO) + (output index); the result goes to ob + 13 (k + OO) + (output
    // index), captured in registers during the sweep (each lane keeps at most one even and one odd
    // step) and stored after it.  v: the input of step 0, at its index.
    static IMPC_WF constexpr bool strd(int k, bool tr) { return ((k & 1) == 0) != tr; }
    template <int S, int K0, int D, bool TR, int CO, int OO>
    IMPC_WF void chain(const double *cb, double *ob, double v) {
        static_assert(S >= 1 && S <= 16, "captures hold one even and one odd step per lane");
        const double *Fm = lds + LD::F_OFF;
        const int lo = lane_o(), l = lo & 63, i = l >> 3, j = l & 7;
        double fq[2], cq[2], cap0 = 0.0, cap1 = 0.0;
        // each prefetch from its own (opaque) address register: merged into one ds_read2 with the
        // next prefetch of the same parity, a load would issue two steps late and its wait would
        // sit on the chain (IMPC_TWOPQ)
        auto ldF = [&](int k) {
            int o = 64 * k + l;
            if (IMPC_TWOPQ) opaque(o);
            return Fm[o];
        };
        auto ldC = [&](int k) {
            int o = 13 * (k + CO) + (strd(k, TR) ? j : i);
            if (IMPC_TWOPQ) opaque(o);
            return cb[o];
        };
        _Pragma("unroll") for (int m = 0; m < 2 && m < S; m++) {
            const int k = K0 + D * m;
            fq[m] = ldF(k);
            cq[m] = ldC(k);
        }
        _Pragma("unroll") for (int m = 0; m < S; m++) {
            const int k = K0 + D * m;
            const double f0 = fq[m & 1], c0 = cq[m & 1];
            if (m + 2 < S) {  // the next step of this parity, two steps ahead
                fq[m & 1] = ldF(k + 2 * D);
                cq[m & 1] = ldC(k + 2 * D);
            }
            if (strd(k, TR)) {
                v = rstep<true>(f0, c0, v);
                if (((m >> 1) & 7) == i) (m & 1 ? cap1 : cap0) = v;
            } else {
                v = rstep<false>(f0, c0, v);
                if (((m >> 1) & 7) == j) (m & 1 ? cap1 : cap0) = v;
            }
        }
        // even steps: output index (strd(K0) ? j : i), kept by the lane whose other index is m / 2
        const bool se = strd(K0, TR), so = strd(K0 + D, TR);
        const int me = 2 * (se ? i : j), mo = 2 * (so ? i : j) + 1;
        if (me < S) ob[13 * (K0 + D * me + OO) + (se ? j : i)] = cap0;
        if (mo < S) ob[13 * (K0 + D * mo + OO) + (so ? j : i)] = cap1;
    }

    // One ADMM iteration with the twisted solve.  Exchange vectors per stage k (13 slots each):
    //   rb: r (rhs); a_k in [:8] for top stages 1..KM; u_{k-1} = Bbar_{k-1} x_{k-1} in [:8] for
    //       bottom stages (written after r is consumed)
    //   tb: t_k (top, k <= KM) / s_k = Acheck_k^-1[:8,:] r_k (bottom) in [:8]; then c_{k-1} =
    //       Bbar_{k-1} zhat_{k-1} (bottom, k - 1 > KM) in [:8]
    //   eb: e_k = Ahat_k^-1 (a_k, r_k[8:]) (top) / zhat_k = Acheck_k^-1 (r_k - Bbar_k' w_{k+1}) (bottom)
    //   xb: w_k = (zhat_k)[:8] (bottom, chain A), then the solution x
    IMPC_WF void iterate_tw(bool need_delta) {
        constexpr int W = WF;
        double *rb = rbuf(), *tb = tbuf(), *eb = ebuf(), *xb = xbuf();
        const double sigma = sig_;
        const int wave = L >> 6, rw2 = (rw + 2) & 3;
        // rhs = sigma x - q + A' v   (stage order)
        IMPC_REP(kSecRhs) {
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                const int v = NL * s + L;
                const double vb = rhob(s) * zb[s] - yb[s];
                double r = sigma * x[s] - q[s];
                r += ab[s] * vb;
                r += col_gather(v, hid_[s]);
                rb[v] = r;
            }
            wv.lsync();
        }
        IMPC_SEC(kSecRhs);
        IMPC_REP(kSecS1) {
            // P1: t_k = r_k[:8] - G_{k-1}[:, 8:] r_{k-1}[8:] (top and middle), s_k = Acheck_k^-1[:8,:] r_k (bottom)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s] || vr_[s] >= 8) continue;
                const int v = NL * s + L, k = vs_[s];
                double t;
                if (k <= KM) {
                    t = rb[v];
                    if (k > 0) {
                        const double *rp = rb + 13 * (k - 1) + 8, *mc = lds + LD::MID_OFF + 5 * vr_[s];
                        double rv[5];
                        _Pragma("unroll") for (int cc = 0; cc < 5; cc++) rv[cc] = rp[cc];
                        // the middle stage's lanes hold Abar^-1 Bbar' rows in cp: their G_{KM-1}[:, 8:]
                        // rows live in LDS
                        _Pragma("unroll") for (int cc = 0; cc < 5; cc++) t -= (k == KM ? mc[cc] : cp[s][cc]) * rv[cc];
                    }
                } else {
                    const double *rk = rb + 13 * k;
                    double rv[13];
                    _Pragma("unroll") for (int cc = 0; cc < 13; cc++) rv[cc] = rk[cc];
                    t = 0.0;
                    _Pragma("unroll") for (int cc = 0; cc < 13; cc++) t += ainv[s][cc] * rv[cc];
                }
                tb[v] = t;
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS1);
        IMPC_REP(kSecFwd) {
            // chains A: a_{k+1} = t_{k+1} - F_k a_k (k = 0..KM-1) and w_k = s_k - H_k w_{k+1}
            // (k = W-1..KM+1, w_W = s_W), on two wavefronts at once
            if (L < 8) rb[L] = tb[L];                      // a_0 = t_0
            if (L >= 64 && L < 72) xb[13 * W + L - 64] = tb[13 * W + L - 64];  // w_W = s_W
            if (wave == rw) {
                const int l = lane_o() & 63;
                chain<KM, 0, 1, false, 1, 1>(tb, rb, tb[strd(0, false) ? (l >> 3) : (l & 7)]);
            } else if (wave == rw2) {
                const int l = lane_o() & 63;
                chain<W - 1 - KM, W - 1, -1, false, 0, 0>(tb, xb,
                                                           tb[13 * W + (strd(W - 1, false) ? (l >> 3) : (l & 7))]);
            }
            wv.lsync();
        }
        IMPC_SEC(kSecFwd);
        IMPC_REP(kSecS3) {
            // P3: e_k (top), x_KM = Abar^-1 ((a_KM, r_KM[8:]) - Bbar_KM' w_{KM+1}) (middle),
            // zhat_k = Acheck_k^-1 r_k - (Acheck_k^-1 Bbar_k') w_{k+1} (bottom)
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                const int v = NL * s + L, k = vs_[s];
                // the coupling term first, kept apart from the 13-term product by a scheduling
                // barrier, so the two operand sets are not live at once
                double g = 0.0;
                if (k >= KM && k < W) {
                    const double *w1 = xb + 13 * (k + 1);
                    double wv_[8];
                    _Pragma("unroll") for (int p = 0; p < 8; p++) wv_[p] = w1[p];
                    _Pragma("unroll") for (int p = 0; p < 8; p++) g += cp[s][p] * wv_[p];
                }
#if defined(__HIP_DEVICE_COMPILE__)
                __builtin_amdgcn_sched_barrier(0);
#endif
                const double *rk = rb + 13 * k;
                double rv[13];
                _Pragma("unroll") for (int cc = 0; cc < 13; cc++) rv[cc] = rk[cc];
                IMPC_LOADS_FIRST(7, 20);
                double e = 0.0;
                _Pragma("unroll") for (int cc = 0; cc < 13; cc++) e += ainv[s][cc] * rv[cc];
                e -= g;
                (k == KM ? xb : eb)[v] = e;
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS3);
        IMPC_REP(kSecFAsm) {
            // P3b: u_KM = Bbar_KM x_KM and c_k = Bbar_k zhat_k (k > KM), one coupling row per state:
            // Bbar_k row i = rho a_up a_(k, .) of the row whose stage-(k+1) entry is state i
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                const int cp_ = ((const int32_t *)(lds + LD::CPL_OFF))[NL * s + L];
                if (cp_ < 0) continue;
                const int cu = cp_ & 0xFFFF, eu = cp_ >> 16;
                const bool m0 = cu / 13 == KM + 1;
                const double *src = m0 ? xb : eb;
                double acc = 0.0, au = 0.0;
                _Pragma("unroll") for (int e = 0; e < 4; e++) {
                    const bool up = e == eu;
                    au = up ? a[s][e] : au;
                    acc += up ? 0.0 : a[s][e] * src[gcol(s, e)];
                }
                (m0 ? rb : tb)[cu] = (rhog_(s) * au) * acc;
            }
            wv.lsync();
        }
        IMPC_REP(kSecBwd) {
            // chains B: x_k[:8] = e_k[:8] - F_k' x_{k+1}[:8] (k = KM-1..0) and
            // u_k = c_k - H_k' u_{k-1} (k = KM+1..W-1)
            if (wave == rw) {
                const int l = lane_o() & 63;
                chain<KM, KM - 1, -1, true, 0, 0>(eb, xb, xb[13 * KM + (strd(KM - 1, true) ? (l >> 3) : (l & 7))]);
            } else if (wave == rw2) {
                const int l = lane_o() & 63;
                chain<W - 1 - KM, KM + 1, 1, true, 1, 1>(tb, rb,
                                                          rb[13 * (KM + 1) + (strd(KM + 1, true) ? (l >> 3) : (l & 7))]);
            }
            wv.lsync();
        }
        IMPC_SEC(kSecBwd);
        IMPC_REP(kSecS5) {
            // P5: controls of the top stages (S5), all of a bottom stage: x_k = zhat_k - Acheck_k^-1[:, :8] u_{k-1}
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                const int v = NL * s + L, k = vs_[s];
                if (k < KM && vr_[s] >= 8) {
                    const double *xn = xb + 13 * (k + 1);
                    double t = eb[v], xv[8];
                    _Pragma("unroll") for (int jj = 0; jj < 8; jj++) xv[jj] = xn[jj];
                    _Pragma("unroll") for (int jj = 0; jj < 8; jj++) t -= cp[s][jj] * xv[jj];
                    xb[v] = t;
                } else if (k > KM) {
                    const double *uu = rb + 13 * k;
                    double t = eb[v], uv[8];
                    _Pragma("unroll") for (int jj = 0; jj < 8; jj++) uv[jj] = uu[jj];
                    _Pragma("unroll") for (int jj = 0; jj < 8; jj++) t -= ainv[s][jj] * uv[jj];
                    xb[v] = t;
                }
            }
            wv.lsync();
        }
        IMPC_SEC(kSecS5);
        update_and_products(need_delta);
    }

    // The twisted factorisation (TWIST): top stages 0..KM-1 as the one-ended scheme, bottom stages
    // W..KM+1 from the bottom up, then the middle stage with both Schur complements.
    IMPC_WF int factorize_tw() {
        constexpr int W = WF, N = W + 1;
        double *w = pbuf(), *rhog = pbuf() + 4 * T.mg, *diagx = lds + LD::DIAGX;
        double *A = lds + LD::FA, *Li = lds + LD::FL, *Ai = lds + LD::FI, *Bb = lds + LD::FB, *G = lds + LD::FG,
               *E = lds + LD::FE, *EB = lds + LD::FEB, *Fm = F();
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            const int g = NL * s + L;
            if (gok[s]) {
                _Pragma("unroll") for (int e = 0; e < 4; e++) w[4 * g + e] = a[s][e];
                rhog[g] = rhog_(s);
            }
        }
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (vok[s]) {
                const double rb = rhob(s);
                diagx[NL * s + L] = (pd[s] + st.sigma) + rb * ab[s] * ab[s];
            }
        }
        wv.sync();
        int bad = 0;
        for (int it = 0; it < N; it++) {
            const int k = it < KM ? it : it < N - 1 ? W - (it - KM) : KM;
            const int sz = k < W ? 13 : 8;
            const bool top = k < KM, mid = k == KM;
            // assemble M_kk (the top Schur complement E_{k-1} folded in for k <= KM) and Bbar_k
            for (int d = L; d < kStageDests; d += NL) {
                const bool isB = d >= 169;
                if (isB && k == W) continue;
                const int dd = isB ? d - 169 : d;
                const int r = dd / 13, cc = dd % 13;
                double val = 0.0;
                if (isB || (r < sz && cc < sz)) {
                    const int32_t t0 = T.term_ptr[(int64_t)k * kStageDests + d];
                    const int32_t t1 = T.term_ptr[(int64_t)k * kStageDests + d + 1];
                    for (int32_t t = t0; t < t1; t++) {
                        const int32_t code = T.term[t];
                        const int32_t g = code >> 4, e = (code >> 2) & 3, f = code & 3;
                        val += rhog[g] * w[4 * g + e] * w[4 * g + f];
                    }
                    if (!isB && r == cc) val += diagx[13 * k + r];
                    if (!isB && k > 0 && k <= KM && r < 8 && cc < 8) val -= E[8 * r + cc];
                }
                if (isB)
                    Bb[dd] = val;
                else
                    A[dd] = val;
            }
            wv.sync();
            IMPC_SEC(kSecFAsm);
            if (!top && k < W) {
                // bottom Schur complement: A -= Bbar_k' (Acheck_{k+1}^-1[:8,:8]) Bbar_k (T = EB Bbar_k in Li)
                for (int p = L; p < 104; p += NL) {
                    const int ii = p / 13, cc = p % 13;
                    double sacc = 0.0;
                    for (int qq = 0; qq < 8; qq++) sacc += EB[8 * ii + qq] * Bb[13 * qq + cc];
                    Li[p] = sacc;
                }
                wv.sync();
                for (int d = L; d < 169; d += NL) {
                    const int r = d / 13, cc = d % 13;
                    double sacc = 0.0;
                    for (int p = 0; p < 8; p++) sacc += Bb[13 * p + r] * Li[13 * p + cc];
                    A[d] -= sacc;
                }
                wv.sync();
            }
            // A^-1 by Gauss-Jordan with 2x2 pivot blocks (as factorize)
            {
                double *src = A, *dst = Li;
                const int gi = L / 13, gc = L % 13;
                const bool act = L < 169 && gi < sz && gc < sz;
                for (int j = 0; j < sz; j += 2) {
                    const bool two = j + 1 < sz, last = j + (two ? 2 : 1) >= sz;
                    if (act) {
                        const int i = last && gc > gi ? gc : gi, c = last && gc > gi ? gi : gc;
                        double v;
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
            if (top) {
                // G_k = Bbar_k Ahat_k^-1, E_k = G_k Bbar_k', F_k (recursion layout), cp rows (S5 / S1)
                for (int p = L; p < 104; p += NL) {
                    const int ii = p / 13, cc = p % 13;
                    double sacc = 0.0;
                    for (int t = 0; t < 13; t++) sacc += Bb[13 * ii + t] * Ai[13 * t + cc];
                    G[p] = sacc;
                }
                wv.sync();
                if (L < 64) {
                    const int ii = L >> 3, jj = L & 7;
                    double sacc = 0.0;
                    for (int t = 0; t < 13; t++) sacc += G[13 * ii + t] * Bb[13 * jj + t];
                    E[8 * ii + jj] = sacc;
                    Fm[64 * k + 8 * ii + jj] = !(k & 1) ? G[13 * jj + ii] : G[13 * ii + jj];
                }
                _Pragma("unroll") for (int s = 0; s < VS; s++) {
                    if (!vok[s]) continue;
                    if (vs_[s] == k && vr_[s] >= 8)
                        _Pragma("unroll") for (int jj = 0; jj < 8; jj++) cp[s][jj] = G[13 * jj + vr_[s]];
                    if (vs_[s] == k + 1 && vr_[s] < 8 && k + 1 < KM)
                        _Pragma("unroll") for (int jj = 0; jj < 8; jj++) cp[s][jj] = jj < 5 ? G[13 * vr_[s] + 8 + jj] : 0.0;
                }
                if (k + 1 == KM && L < 40) lds[LD::MID_OFF + L] = G[13 * (L / 5) + 8 + L % 5];  // [8][5]
                wv.sync();
            } else if (k < W) {
                // G'_k = A^-1 Bbar_k' (13 x 8, row-major at G[8 r + p]); bottom: H_k = G'_k[:8, :] in F
                // slot k (recursion layout) and the stage's cp rows; middle: G'_KM to LDS
                for (int p = L; p < 104; p += NL) {
                    const int r = p >> 3, qq = p & 7;
                    double sacc = 0.0;
                    for (int cc = 0; cc < 13; cc++) sacc += Ai[13 * r + cc] * Bb[13 * qq + cc];
                    G[p] = sacc;
                }
                wv.sync();
                if (!mid && L < 64) {
                    const int ii = L >> 3, jj = L & 7;
                    Fm[64 * k + 8 * ii + jj] = !(k & 1) ? G[8 * jj + ii] : G[8 * ii + jj];
                }
                _Pragma("unroll") for (int s = 0; s < VS; s++)
                    if (vok[s] && vs_[s] == k)
                        _Pragma("unroll") for (int jj = 0; jj < 8; jj++) cp[s][jj] = G[8 * vr_[s] + jj];
            }
            if (!top && !mid) {
                // Acheck_k^-1[:8, :8] for the next stage up
                if (L < 64) EB[L] = Ai[13 * (L >> 3) + (L & 7)];
            }
            wv.sync();
            IMPC_SEC(kSecFDense);
        }
        _Pragma("unroll") for (int s = 0; s < VS; s++)
            if (vok[s] && vs_[s] == 0 && vr_[s] < 8)
                _Pragma("unroll") for (int jj = 0; jj < 8; jj++) cp[s][jj] = 0.0;
        bad = (int)wv.max((double)bad);
        clear_exchange();
        zero_products();
        return bad;
    }

    // ------------------------------------------------------------ update_info + checks
    struct Info {
        double pri_res, dua_res, pri_norm_u, dua_norm_u, pri_norm_s, dua_norm_s, pri_plain, dua_plain;
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
            double r[14] = {pr_u, z_u, ax_u, pr_p, z_p, ax_p, dr_u, q_u, aty_u, px_u, dr_p, q_p, aty_p, px_p};
            wv.max_n(r);  // one team reduction for all 14 norms
            pr_u = r[0], z_u = r[1], ax_u = r[2], pr_p = r[3], z_p = r[4], ax_p = r[5], dr_u = r[6];
            q_u = r[7], aty_u = r[8], px_u = r[9], dr_p = r[10], q_p = r[11], aty_p = r[12], px_p = r[13];
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
        wv.sync();
    }

    // is_primal_infeasible (projects dy in place)
    IMPC_WF int primal_infeasible(double eps, const double D[VS], const double Eb[VS], const double Eg[GS]) {
        double nrm, lhs;
        pinf_partials(Eb, Eg, nrm, lhs);
        nrm = wv.max(nrm);
        lhs = wv.sum(lhs);
        return pinf_stage2(eps, nrm, lhs, D);
    }
    // its lane-local part: the projected dy, ||E dy||_inf and u' max(dy, 0) + l' min(dy, 0)
    IMPC_WF void pinf_partials(const double Eb[VS], const double Eg[GS], double &nrm_o, double &lhs_o) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        double nrm = 0.0, lhs = 0.0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            double d = dyb(s);
            if (ub[s] > kInf * kMinScaling)
                d = (lb[s] < -kInf * kMinScaling) ? 0.0 : dmin(d, 0.0);
            else if (lb[s] < -kInf * kMinScaling)
                d = dmax(d, 0.0);
            dyb(s) = d;
            nrm = dmax(nrm, fabs(unsc ? Eb[s] * d : d));
            lhs += ub[s] * dmax(d, 0) + lb[s] * dmin(d, 0);
        }
        _Pragma("unroll") for (int s = 0; s < GS; s++) {
            if (!gok[s]) continue;
            double d = dyg(s);
            if (ug[s] > kInf * kMinScaling)
                d = (lg[s] < -kInf * kMinScaling) ? 0.0 : dmin(d, 0.0);
            else if (lg[s] < -kInf * kMinScaling)
                d = dmax(d, 0.0);
            dyg(s) = d;
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
            double *pb = pbuf();
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (gok[s])
                    _Pragma("unroll") for (int e = 0; e < 4; e++) pb[gdst(s, e)] = a[s][e] * dyg(s);
            }
            wv.sync();
            double mx = 0.0;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                double t = ab[s] * dyb(s) + col_gather(NL * s + L, hid_[s]);
                if (unsc) t = (1. / D[s]) * t;
                mx = dmax(mx, fabs(t));
            }
            mx = wv.max(mx);
            res = mx < eps * nrm;
            wv.sync();
        }
        return res;
    }

    // is_dual_infeasible
    IMPC_WF int dual_infeasible(double eps, const double D[VS], const double Eb[VS], const double Eg[GS]) {
        double nrm, qdx;
        dinf_partials(D, nrm, qdx);
        nrm = wv.max(nrm);
        qdx = wv.sum(qdx);
        return dinf_stage2(eps, nrm, qdx, D, Eb, Eg);
    }
    // its lane-local part: ||D dx||_inf and q' dx
    IMPC_WF void dinf_partials(const double D[VS], double &nrm_o, double &qdx_o) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        double nrm = 0.0, qdx = 0.0;
        _Pragma("unroll") for (int s = 0; s < VS; s++) {
            if (!vok[s]) continue;
            nrm = dmax(nrm, fabs(unsc ? D[s] * dxv(s) : dxv(s)));
            qdx += q[s] * dxv(s);
        }
        nrm_o = nrm;
        qdx_o = qdx;
    }
    IMPC_WF int dinf_stage2(double eps, double nrm, double qdx, const double D[VS], const double Eb[VS],
                            const double Eg[GS]) {
        const bool unsc = st.scaling > 0 && !st.scaled_termination;
        const double cs = unsc ? c : 1.0;
        int res = 0;
        if (nrm > kDivTol && qdx < cs * eps * nrm) {
            double mx = 0.0;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                double pv = pd[s] * dxv(s);
                if (unsc) pv = (1. / D[s]) * pv;
                mx = dmax(mx, fabs(pv));
            }
            mx = wv.max(mx);
            if (mx < cs * eps * nrm) {
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
#if IMPC_CHKRED
        // the same tests as below, the two infeasibility tests' first-stage norms and sums reduced
        // over the team in one exchange (bitwise the values of the separate reductions)
        const bool ptest = T.m != 0 && !(inf.pri_res < eps_abs + eps_rel * inf.pri_norm_u);
        prim_ok = !ptest;
        dual_ok = inf.dua_res < eps_abs + eps_rel * inf.dua_norm_u;
        if (ptest || !dual_ok) {
            double mx[2] = {0.0, 0.0}, sm[2] = {0.0, 0.0};
            if (ptest) pinf_partials(Eb, Eg, mx[0], sm[0]);
            if (!dual_ok) dinf_partials(D, mx[1], sm[1]);
            wv.max_sum_n(mx, sm);
            if (ptest) prim_inf = pinf_stage2(eps_pinf, mx[0], sm[0], D);
            if (!dual_ok) dual_inf = dinf_stage2(eps_dinf, mx[1], sm[1], D, Eb, Eg);
        }
#else
        if (T.m == 0) {
            prim_ok = 1;
        } else {
            if (inf.pri_res < eps_abs + eps_rel * inf.pri_norm_u)
                prim_ok = 1;
            else
                prim_inf = primal_infeasible(eps_pinf, D, Eb, Eg);
        }
        if (inf.dua_res < eps_abs + eps_rel * inf.dua_norm_u)
            dual_ok = 1;
        else
            dual_inf = dual_infeasible(eps_dinf, D, Eb, Eg);
#endif
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
    IMPC_WF void solve(int64_t b) {
        const int n = T.n, m = T.m;
        // time_limit clock: from the start of the QP's setup (load, scaling, factorisation), as
        // OSQP 0.6.2 counts setup_time + solve time on a first run (every solveTraj call is one);
        // the profiling record (qpt) starts at the same tick, so a QP stopped by its limit always
        // shows a recorded latency of at least that limit
        const uint64_t t0 = device_clock();
#if IMPC_PRIO_INV && defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_s_setprio(IMPC_PRIO_INV);
#endif
        rw = (int)(b % (NL / 64));  // spread the serial recursions of co-resident QPs over SIMDs
#if IMPC_HWRW && defined(__HIP_DEVICE_COMPILE__)
        // recursion wave from the hardware placement (HW_REG_HW_ID: WAVE_ID [3:0], SIMD_ID [5:4]):
        // the wave on SIMD (wave slot of the team's wave 0) mod 4, so co-resident teams, which sit
        // in different wave slots, run their recursions on different SIMDs; the QP-index choice
        // above when no wave of the team is on that SIMD
        if ((L & 63) == 0) lds[LD::JUNK_OFF + (L >> 6)] = (double)(__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0x3f);
#endif
        IMPC_SEC_START();
        clear_exchange();
#if IMPC_HWRW && defined(__HIP_DEVICE_COMPILE__)
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
            if (ps && io.resume && io.q_updated)  // osqp_update_lin_cost: q = c (D q)
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
        // countdowns instead of iter % interval (no integer division in the loop)
        // the loop's settings read once into registers (the batch's settings live in global memory
        // for a grouped launch: read in the loop they cost a scalar-memory round trip each
        // iteration, after every barrier)
        const int32_t max_iter = st.max_iter, rho_int = st.adaptive_rho ? st.rho_interval : 0;
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
                factorize();
                write_v_products();
                IMPC_SEC(kSecFactor);
            }
            // the hot loop: ADMM steps up to the next termination check / rho update (or the end);
            // the check and the update run between two passes of it, so their code and registers
            // sit outside it (the operations are those of one loop, in the same order)
            bool chk_now = false, rho_now = false, stop = false;
#if IMPC_LOOPC
            // the same iterations, flags and counters as the countdown loop below: the pass runs to
            // its next event nxt = min(iterations left, chk_left, rho_left); only its last iteration
            // can be a check / rho-update / max_iter one
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
#else
            for (; iter <= max_iter; iter++) {
                chk_now = chk && --chk_left == 0;
                if (chk_now) chk_left = chk;
                rho_now = rho_int && --rho_left == 0;
                if (rho_now) rho_left = rho_int;
                const bool need_delta = chk_now || iter == max_iter || tlim;
                iterate(need_delta);
                // osqp_solve (PROFILING build): checked after the ADMM steps, before can_check is
                // recomputed (so it keeps the previous iteration's value); one team-wide decision
                if (tlim) {
                    const double el = wv.max((double)(device_clock() - t0) * tick);
                    if (el >= tl) {
                        status = IMPC_TIME_LIMIT_REACHED;
                        stop = true;
                        break;
                    }
                }
                can_check = chk_now;
                if (chk_now || rho_now) break;
            }
#endif
            if (stop || iter > max_iter) break;
            if (can_check) {
                IMPC_SEC_START();
                double D[VS], Eb[VS], Eg[GS];
                load_scal(b, D, Eb, Eg);
                update_info(inf, D, Eb, Eg);
                info_iter = iter;
                int done = check_termination(inf, 0, status, obj, D, Eb, Eg);
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
        if (ps) {  // the workspace after osqp_solve: rho and the scaled iterates
            double *it = ps + kPersistHdr;
            if (L == 0) ps[kPersistHdr - 1] = R.rho;
            _Pragma("unroll") for (int s = 0; s < VS; s++) {
                if (!vok[s]) continue;
                const int v = NL * s + L;
                it[v] = x[s];
                it[n + v] = zb[s];
                it[2 * n + v] = yb[s];
            }
            _Pragma("unroll") for (int s = 0; s < GS; s++) {
                if (!gok[s]) continue;
                const int g = NL * s + L;
                it[3 * n + g] = z[s];
                it[3 * n + T.mg + g] = y[s];
            }
        }
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
