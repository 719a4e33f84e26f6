// impc_qp.hip -- libimpc_qp.so: C-ABI (include/impc_qp.h), device memory management and the
// gfx950 kernels of the batched OSQP-equivalent solver.
//
// Two device paths, both OSQP 0.6.2 ADMM in FP64:
//   STRUCTURED  k_mpc_wave<VS,GS>: one mpcPlanner QP per 64-lane wavefront, all per-QP state in
//               VGPRs/LDS, waves pull QPs from a work queue (mpc_wave.hpp).  Used when the
//               pattern is the stage-structured MPC QP (mpc_structure.hpp).
//   GENERIC     k_setup + k_solve: any sparsity pattern, one QP per lane, batch-interleaved state
//               in HBM, sparse LDL^T of the reduced KKT (admm_core.hpp, symbolic.hpp).  Also
//               backs the persistent update calls.
// Inputs are kept QP-major on the device (the layout the C-ABI receives them in); the generic
// path interleaves them (LDS-tiled transpose) at setup.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/impc_qp.h"
#include "../../include/impc_select.h"
#include "../../include/impc_mpc.h"
#include "../../include/impc_fanout.h"
#include "../../include/impc_predict.h"
#include "../../include/impc_comm.h"
#include "../../include/impc_replan.h"
#include "lib_internal.hpp"
#include "mpc_qp_internal.hpp"
#include "admm_core.hpp"
#include "mpc_structure.hpp"
#include "mpc_wave.hpp"
#include "queue.hpp"
#include "symbolic.hpp"

#ifndef IMPC_BUILD_ID  // set by the Makefile: hash of the compiled sources and flags
#define IMPC_BUILD_ID "src-unknown"
#endif
#ifndef IMPC_GIT_REV
#define IMPC_GIT_REV "unknown"
#endif
#define IMPC_VERSION "impc_qp 0.3.0 (OSQP 0.6.2 semantics, gfx950, git " IMPC_GIT_REV ")"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define HIP_OK(expr)                                                                             \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail(IMPC_DEVICE_ERROR, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kBlock = 64;  // generic path: one wavefront per workgroup, one QP per lane
constexpr int kTile = 64;   // transpose tile edge
// Structured path team shapes, keyed by the variable slots per lane VS:
//   VS = 1  team shape: one QP per 256-lane workgroup (one variable per lane), two teams per CU
//           (n <= 256: the reference's default horizon N = 20)
//   VS = 3  long shape: 256 lanes, three variables per lane, one team per CU (n <= 768)
//   VS = 4  wavefront shape (built only with IMPC_WAVEFRONT=1: measured slower):
//           one QP per 64-lane wavefront (four variables and up to six general rows per lane, D / E
//           and the check deltas off LDS), one wavefront per SIMD, four QPs per CU
#ifndef IMPC_WAVEFRONT
#define IMPC_WAVEFRONT 0
#endif
constexpr int kWaveVS = 1, kWaveVSLong = 3, kWaveVSFront = 4;
template <int VS>
struct Shape {
    static constexpr int NL = VS == kWaveVSFront ? 64 : 256;  // lanes per QP
    static constexpr int WPS = VS == kWaveVS ? 2 : 1;         // waves per SIMD (launch bound: registers)
    static constexpr int GMAX = VS == kWaveVSFront ? 6 : 4;   // general-row slots per lane
    // the two-tier products instances (mpc_wave.hpp WaveLds): general-row slot counts that have them
    static constexpr int TIER_GMAX = VS == kWaveVSFront ? 6 : VS == kWaveVS ? 3 : 1;
    static constexpr int PER_CU = 4 * WPS / (NL / 64);        // resident QPs per CU by waves
};

// ------------------------------------------------------------------ layout transposes
// dst[e * S + b] = src[b * len + e]; 64x64 tile through LDS so both sides are coalesced.
__global__ __launch_bounds__(256) void k_interleave(const double *__restrict__ src, double *__restrict__ dst,
                                                    int64_t len, int64_t B, int64_t S) {
    __shared__ double tile[kTile][kTile + 1];
    const int64_t e0 = (int64_t)blockIdx.x * kTile, b0 = (int64_t)blockIdx.y * kTile;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < kTile; r += 4) {
        int64_t b = b0 + r, e = e0 + tx;
        tile[r][tx] = (b < B && e < len) ? src[b * len + e] : 0.0;
    }
    __syncthreads();
    for (int r = ty; r < kTile; r += 4) {
        int64_t e = e0 + r, b = b0 + tx;
        if (e < len && b < S) dst[e * S + b] = tile[tx][r];
    }
}

// dst[b * len + e] = src[e * S + b]
__global__ __launch_bounds__(256) void k_deinterleave(const double *__restrict__ src, double *__restrict__ dst,
                                                      int64_t len, int64_t B, int64_t S) {
    __shared__ double tile[kTile][kTile + 1];
    const int64_t e0 = (int64_t)blockIdx.x * kTile, b0 = (int64_t)blockIdx.y * kTile;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < kTile; r += 4) {
        int64_t e = e0 + r, b = b0 + tx;
        tile[r][tx] = (e < len && b < B) ? src[e * S + b] : 0.0;
    }
    __syncthreads();
    for (int r = ty; r < kTile; r += 4) {
        int64_t b = b0 + r, e = e0 + tx;
        if (b < B && e < len) dst[b * len + e] = tile[tx][r];
    }
}

// ------------------------------------------------------------------ generic path kernels
__global__ __launch_bounds__(kBlock) void k_setup(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st, int64_t B,
                                                  int has_ws) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    const int64_t S = wk.S;
    const uint64_t t0 = impc::device_clock();
    impc::qp_setup(sy, wk, st, lane, has_ws);
    // osqp_setup's own duration (setup_time): a first solve's time limit counts it, not the time
    // the workspace then waits for the solve
    IMPC_AT(wk.scal, impc::SC_TSETUP) = (double)(impc::device_clock() - t0);
}

// first_run: the first solve after k_setup (its time limit counts the setup time, OSQP 0.6.2)
__global__ __launch_bounds__(kBlock) void k_solve(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st,
                                                  int64_t B, int first_run) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    impc::qp_solve(sy, wk, st, lane, lane, 0, first_run);
}

// impc_ctx_clock_check: spin until the device clock has advanced `ticks` (one wavefront)
__global__ __launch_bounds__(64) void k_clock_spin(uint64_t ticks) {
    const uint64_t t0 = impc::device_clock();
    while (impc::device_clock() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// osqp_warm_start (osqp.h:157) on a set-up workspace: scaling, rho and factor stay
__global__ __launch_bounds__(kBlock) void k_warm_start(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st,
                                                        int64_t B) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    const int64_t S = wk.S;
    impc::apply_warm_start(sy, wk, st, IMPC_AT(wk.scal, impc::SC_C), lane);
    impc::refresh_v(sy, wk, lane);
}

// osqp_update_lin_cost (osqp.h:114): q <- c * D q
__global__ __launch_bounds__(kBlock) void k_update_q(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st,
                                                     int64_t B) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    const int64_t S = wk.S;
    const double c = IMPC_AT(wk.scal, impc::SC_C);
    for (int32_t j = 0; j < sy.n; j++) {
        double qj = IMPC_AT(wk.q, j);
        if (st.scaling > 0) {
            qj = IMPC_AT(wk.D, j) * qj;
            qj *= c;
        }
        IMPC_AT(wk.qs, j) = qj;
    }
}

// osqp_update_bounds (osqp.h:125) + update_rho_vec (auxil.h:43): refactor only when a
// constraint changes type.
__global__ __launch_bounds__(kBlock) void k_update_bounds(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st,
                                                          int64_t B) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    const int64_t S = wk.S;
    const double rho = IMPC_AT(wk.scal, impc::SC_RHO);
    int changed = 0;
    for (int32_t i = 0; i < sy.m; i++) {
        double li = impc::dmin(impc::dmax(IMPC_AT(wk.l, i), -impc::kInf), impc::kInf);
        double ui = impc::dmin(impc::dmax(IMPC_AT(wk.u, i), -impc::kInf), impc::kInf);
        if (st.scaling > 0) {
            li = IMPC_AT(wk.E, i) * li;
            ui = IMPC_AT(wk.E, i) * ui;
        }
        IMPC_AT(wk.ls, i) = li;
        IMPC_AT(wk.us, i) = ui;
        double t, r;
        if ((li < -impc::kInf * impc::kMinScaling) && (ui > impc::kInf * impc::kMinScaling)) {
            t = -1.0;
            r = impc::kRhoMin;
        } else if (ui - li < impc::kRhoTol) {
            t = 1.0;
            r = rho * impc::kRhoEqOverIneq;
        } else {
            t = 0.0;
            r = rho;
        }
        if (IMPC_AT(wk.ctype, i) != t) {
            IMPC_AT(wk.ctype, i) = t;
            IMPC_AT(wk.rho, i) = r;
            IMPC_AT(wk.rhoinv, i) = 1. / r;
            changed = 1;
        }
    }
    if (changed) {
        int bad = impc::assemble_and_factor(sy, wk, st, lane);
        if (bad) IMPC_AT(wk.scal, impc::SC_SETUP_ERR) = (double)IMPC_NONCVX_ERROR;
    }
    impc::refresh_v(sy, wk, lane);
}

// ---------------------------------------------------------------- structured path kernel
// Team policy of mpc_wave.hpp on gfx950: one QP per workgroup of NL threads (NL/64 wavefronts);
// LDS exchange + workgroup barrier, readlane broadcast inside a wavefront, butterfly reductions
// inside a wavefront combined across wavefronts through LDS in a fixed order (bitwise uniform).
template <int NL>
struct GpuTeam {
    double *red;  // >= NL/64 doubles of LDS
    __device__ int lane() const { return (int)threadIdx.x; }
    // A one-wavefront team (NL = 64) needs no workgroup barrier: a wavefront's LDS operations
    // execute in issue order, so a read issued after a write sees it; only code motion across the
    // exchange point is ruled out (wavefront-scope fence, no wait for outstanding LDS operations)
    __device__ static void wave_sync() {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    __device__ void sync() {
        if constexpr (NL == 64) wave_sync();
        else __syncthreads();
    }
    // exchange point inside the caller's wavefront only (the long horizon's chunk operators)
    __device__ static void wsync() { wave_sync(); }
    // barrier of the ADMM iteration's LDS exchanges (an LDS-only wait was measured slower)
    __device__ void lsync() { sync(); }
    __device__ double bcast(double v, int src) {
        int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
        int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
        return __hiloint2double(hi, lo);
    }
    // a value every lane holds identically, moved to scalar registers
    __device__ static double uniform(double v) {
        int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
        int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
        return __hiloint2double(hi, lo);
    }
    // v of lane src (per-lane) of the caller's wavefront: ds_bpermute on both halves
    __device__ double shfl(double v, int src) {
        const int addr = src << 2;
        int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
        int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
        return __hiloint2double(hi, lo);
    }
    template <int CTRL>
    __device__ static double dpp(double v) {
        // every control used reads a valid lane of the same row: no "old" operand to initialise
        int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
        int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
        return __hiloint2double(hi, lo);
    }
    // sum over lanes {8i, .., 8i+7}: quad_perm xor 1, quad_perm xor 2, row_half_mirror.  Every
    // stage adds a commuted operand pair, so all 8 lanes hold bitwise the same
    // ((v0+v1)+(v2+v3)) + ((v4+v5)+(v6+v7)).
    __device__ double sum_contig8(double v) {
        v = v + dpp<0xB1>(v);   // quad_perm [1,0,3,2]
        v = v + dpp<0x4E>(v);   // quad_perm [2,3,0,1]
        v = v + dpp<0x141>(v);  // row_half_mirror
        return v;
    }
    // x + y computed a second time into its own register, out of CSE's sight: the permlane swaps
    // need their operand in two registers, and a second add issued beside the first is off the
    // chain where a two-v_mov copy of the result was on it.  (The hazard recognizer pads the
    // gfx950 "VALU write -> v_permlane read" distance after the asm itself: checked in the .s.)
    __device__ static double add_dup(double x, double y) {
        double r;
        asm("v_add_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
        return r;
    }
    // pair_sum of a value held (bitwise identically) in two registers a, b; returns the sum and,
    // when DUP, its second copy
    template <bool P32, bool DUP>
    __device__ static double pair_sum2(double a, double b, double *dup) {
        const int al = __double2loint(a), ah = __double2hiint(a), bl = __double2loint(b), bh = __double2hiint(b);
        auto rl = P32 ? __builtin_amdgcn_permlane32_swap(al, bl, false, false)
                      : __builtin_amdgcn_permlane16_swap(al, bl, false, false);
        auto rh = P32 ? __builtin_amdgcn_permlane32_swap(ah, bh, false, false)
                      : __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
        const double x = __hiloint2double(rh[0], rl[0]), y = __hiloint2double(rh[1], rl[1]);
        if (DUP) *dup = add_dup(x, y);
        return x + y;
    }
    // sum over lanes {j, j+8, .., j+56}: row_ror 8 (xor 8), then xor 16 and xor 32 pair sums,
    // low + high in both partners: ((v0+v1)+(v2+v3)) + ((v4+v5)+(v6+v7)) over the 8 rows i
    __device__ double sum_stride8(double v) {
        const double d = dpp<0x128>(v);  // row_ror:8
        const double a = v + d, b = add_dup(v, d);
        double c2;
        const double c = pair_sum2<false, true>(a, b, &c2);
        return pair_sum2<true, false>(c, c2, nullptr);
    }
    // lane l's value paired with lane l ^ 4 (ds_swizzle bit mode: and 0x1f, xor 4; no LDS access)
    __device__ static double xor4(double v) {
        const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), (4 << 10) | 0x1F);
        const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), (4 << 10) | 0x1F);
        return __hiloint2double(hi, lo);
    }
    // team maximum: the in-wave exchanges by DPP / permlane (max is order-independent), one LDS
    // round across wavefronts
    __device__ double max(double v) {
        double mv[1] = {v};
        reduce<1, 0>(mv, nullptr);
        return mv[0];
    }
    // K team maxima at once (one LDS round across wavefronts)
    template <int K>
    __device__ void max_n(double (&v)[K]) {
        reduce<K, 0>(v, nullptr);
    }
    template <int KM, int KS>
    __device__ void max_sum_n(double (&mx)[KM], double (&sm)[KS]) {
        reduce<KM, KS>(mx, sm);
    }
    // the 64-bit permlane swaps (V_PERMLANE32_SWAP / V_PERMLANE16_SWAP on both halves): lanes of the
    // lower 32 (even 16-lane row) end with x from their partner l + 32 (l + 16) in y, the upper
    // (odd) ones with y from their partner in x -- so max(x, y) is, in every lane, the pair's
    // maximum of x (lower / even lanes) or of y (upper / odd lanes)
    template <bool P32>
    __device__ static void swap64(double &x, double &y) {
        const int xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
        auto rl = P32 ? __builtin_amdgcn_permlane32_swap(xl, yl, false, false)
                      : __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
        auto rh = P32 ? __builtin_amdgcn_permlane32_swap(xh, yh, false, false)
                      : __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
        x = __hiloint2double(rh[0], rl[0]);
        y = __hiloint2double(rh[1], rl[1]);
    }
    // KM team maxima and KS team sums at once, each bitwise the value max() / sum() gives, over one
    // LDS round.  Maxima: reduce-scatter inside the wavefront -- the permlane32 swap pairs value k
    // with value k + K1 (lower 32 lanes keep the first K1 values, upper 32 the rest), the permlane16
    // swap halves each half again per 16-lane row, then DPP butterflies inside the rows over the K2
    // values left: every lane of row r ends with values (r >> 1) K1 + (r & 1) K2 + k (max is exact,
    // so the order does not matter; 3 instructions per value and level instead of 30 per value
    // for a full butterfly of each).  Sums: the xor butterfly of wave_sum, wavefronts added in order.
    template <int KM, int KS>
    __device__ void reduce(double (&mx)[KM], double *sm) {
        constexpr int K1 = (KM + 1) / 2, K2 = (K1 + 1) / 2, KT = KM + KS;
        static_assert(KT * (NL / 64) <= impc::kRedLen, "team reduction scratch (WaveLds RED_OFF)");
        auto vmax = [](double a, double b) { return b > a ? b : a; };
        double h[K1], q[K2];
        _Pragma("unroll") for (int k = 0; k < K1; k++) {
            double x = mx[k], y = k + K1 < KM ? mx[k + K1] : mx[k];
            swap64<true>(x, y);
            h[k] = vmax(x, y);
        }
        _Pragma("unroll") for (int k = 0; k < K2; k++) {
            double x = h[k], y = k + K2 < K1 ? h[k + K2] : h[k];
            swap64<false>(x, y);
            double t = vmax(x, y);
            t = vmax(t, dpp<0xB1>(t));   // quad_perm [1,0,3,2]
            t = vmax(t, dpp<0x4E>(t));   // quad_perm [2,3,0,1]
            t = vmax(t, dpp<0x141>(t));  // row_half_mirror
            q[k] = vmax(t, dpp<0x128>(t));  // row_ror:8
        }
        _Pragma("unroll") for (int k = 0; k < KS; k++) sm[k] = wave_sum(sm[k]);
        const int w = (int)threadIdx.x >> 6, row = ((int)threadIdx.x >> 4) & 3;
        if ((threadIdx.x & 15) == 0) {
            _Pragma("unroll") for (int k = 0; k < K2; k++) {
                const int sub = (row & 1) * K2 + k, idx = (row >> 1) * K1 + sub;
                if (sub < K1 && idx < KM) red[w * KT + idx] = q[k];
            }
        }
        if ((threadIdx.x & 63) == 0) _Pragma("unroll") for (int k = 0; k < KS; k++) red[w * KT + KM + k] = sm[k];
        __syncthreads();
        _Pragma("unroll") for (int k = 0; k < KM; k++) {
            double r = red[k];
            for (int u = 1; u < NL / 64; u++) r = vmax(r, red[u * KT + k]);
            mx[k] = r;
        }
        _Pragma("unroll") for (int k = 0; k < KS; k++) {
            double r = red[KM + k];
            for (int u = 1; u < NL / 64; u++) r = r + red[u * KT + KM + k];
            sm[k] = r;
        }
        __syncthreads();
    }
    // sum() inside one wavefront: the xor butterfly (partners l ^ 32, 16, 8, 4, 2, 1, each level
    // adding a commuted pair, so every lane holds bitwise the same value), exchanges by permlane /
    // DPP / swizzle
    __device__ double wave_sum(double v) {
        {
            const int lo = __double2loint(v), hi = __double2hiint(v);
            auto ql = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
            auto qh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
            v = __hiloint2double(qh[0], ql[0]) + __hiloint2double(qh[1], ql[1]);
        }
        {
            const int lo = __double2loint(v), hi = __double2hiint(v);
            auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
            auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
            v = __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
        }
        v = v + dpp<0x128>(v);  // row_ror:8 = lane ^ 8 within a row of 16
        v = v + xor4(v);
        v = v + dpp<0x4E>(v);   // quad_perm [2,3,0,1] = lane ^ 2
        v = v + dpp<0xB1>(v);   // quad_perm [1,0,3,2] = lane ^ 1
        return v;
    }
    // team sum: the in-wave xor butterfly (wave_sum, every lane bitwise the same), wavefronts
    // added in order through LDS
    __device__ double sum(double v) {
        v = wave_sum(v);
        v = bcast(v, 0);
        if (NL == 64) return v;
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
        __syncthreads();
        double r = red[0];
        for (int w = 1; w < NL / 64; w++) r = r + red[w];
        __syncthreads();
        return r;
    }
};

// One batch of a grouped launch (impc_batch_solve_group): its tables, I/O, settings and the
// index of its first QP in the group's work queue.
struct GroupEntry {
    impc::WaveTables T;
    impc::WaveIO io;
    impc::DevSettings st;
    int64_t first;
    // the batch's active QP count in device memory (impc_lib::batch_set_active_device), or null:
    // io.B QPs.  A launch with device counts dequeues through a permutation that puts every
    // active QP first, and stops after the sum of the counts.
    const int64_t *dcount;
};

// Several structured batches in one persistent launch: one work queue over all their QPs, so
// the long-running QPs at the end of one batch overlap the next batch's work instead of leaving
// CUs idle between launches.  A workgroup reloads the pattern tables when it crosses batches.
template <int NL, int VS, int GS, int WPS, int WF, bool TIER>
__global__ __launch_bounds__(NL, WPS) void k_mpc_wave_group(const GroupEntry *__restrict__ g, int count,
                                                            int64_t total, unsigned *counter,
                                                            const uint32_t *__restrict__ ord, int devcnt) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    using LD = impc::WaveLds<NL, VS, GS>;
    GpuTeam<NL> wv{smem + LD::RED_OFF};
    __shared__ unsigned next;
    int cur = -1;
    if (devcnt) {  // device-side active counts: the queue's length is their sum (ord puts them first)
        int64_t t = 0;
        for (int e = 0; e < count; e++) {
            const int64_t c = g[e].dcount ? *g[e].dcount : g[e].io.B;
            t += c < g[e].io.B ? (c > 0 ? c : 0) : g[e].io.B;
        }
        total = t;
    }
    for (;;) {
        if (threadIdx.x == 0) next = atomicAdd(counter, 1u);
        __syncthreads();
        const unsigned pos = next;
        __syncthreads();
        if ((int64_t)pos >= total) break;
        // queue order (impc_batch_set_queue_order): a permutation of the launch's QPs
        const unsigned b = ord ? ord[pos] : pos;
        int e = 0;
        while (e + 1 < count && (int64_t)b >= g[e + 1].first) e++;
        if (e != cur) {
            impc::WaveQP<GpuTeam<NL>, NL, VS, GS, WF, TIER>::load_tables(wv, g[e].T, smem);
            cur = e;
        }
        impc::WaveQP<GpuTeam<NL>, NL, VS, GS, WF, TIER> qp(wv, g[e].T, g[e].io, g[e].st, smem);
        qp.solve((int64_t)b - g[e].first);
    }
}

}  // namespace

struct impc_ctx_s {
    int device = 0;
    int num_cu = 256;
    hipStream_t stream = nullptr;
    // the device clock of time limits and latencies: seconds per tick (hipDeviceAttributeWallClockRate)
    double tick_s = 1e-8;
    // grouped launches: device copies of the entry tables of the last few distinct groups (a
    // pipeline alternates between batch sets), each with its host copy; reused while unchanged
    struct GroupTable {
        GroupEntry *d = nullptr;
        int cap = 0;
        std::vector<GroupEntry> h;
        uint64_t used = 0;
    };
    std::vector<GroupTable> groups;
    uint64_t group_clock = 0;
    // caller-stream bookkeeping (ctx_order_launch / ctx_note_launch / ctx_quiesce)
    hipEvent_t ev_order = nullptr;
    std::vector<hipEvent_t> ev_pool, ev_pending;
    std::vector<hipEvent_t> timer_marks;  // impc_ctx_timer_mark
    // released batches (impc_batch_acquire / impc_batch_release), with their pattern hashes
    std::vector<std::pair<uint64_t, impc_batch_s *>> pool;
};

// Every host->device transfer and fill below goes through the context's stream and has finished
// when the call returns: the solver's kernels run on that stream, which is non-blocking, so the
// legacy null stream of a plain hipMemcpy / hipMemset would not be ordered before them (a pageable
// hipMemcpy may also return before its DMA lands).
static int h2d_sync(hipStream_t st, void *dst, const void *src, size_t bytes) {
    if (!bytes) return IMPC_OK;
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
    return IMPC_OK;
}
static int fill0_sync(hipStream_t st, void *dst, size_t bytes) {
    if (!bytes) return IMPC_OK;
    HIP_OK(hipMemsetAsync(dst, 0, bytes, st));
    HIP_OK(hipStreamSynchronize(st));
    return IMPC_OK;
}
#define IMPC_TRY(expr)          \
    do {                        \
        int rc_ = (expr);       \
        if (rc_) return rc_;    \
    } while (0)

// Caller streams (impc_batch_setup / _solve / _solve_group accept one) are ordered against the
// context's own stream in both directions: a launch on a caller stream first waits for what is
// already queued on the context stream (device-to-device value copies, in-place updates and warm
// starts), and every entry point that rewrites batch inputs, workspaces or the group-entry table
// first waits for every launch issued on a caller stream (an event recorded after each one), so
// no kernel in flight on another stream reads half-replaced data.
static int ctx_order_launch(impc_ctx ctx, hipStream_t st) {
    if (st == ctx->stream) return IMPC_OK;
    if (!ctx->ev_order) HIP_OK(hipEventCreateWithFlags(&ctx->ev_order, hipEventDisableTiming));
    HIP_OK(hipEventRecord(ctx->ev_order, ctx->stream));
    HIP_OK(hipStreamWaitEvent(st, ctx->ev_order, 0));
    return IMPC_OK;
}
// st waits for every launch noted on any caller stream (ctx_note_launch) as well as for the
// context stream: for consumers of results that may have been produced on another stream (the
// cost gather) and of scratch an earlier call on another stream may still be reading
static int ctx_order_after_all(impc_ctx ctx, hipStream_t st) {
    if (st != ctx->stream) IMPC_TRY(ctx_order_launch(ctx, st));
    for (hipEvent_t e : ctx->ev_pending) HIP_OK(hipStreamWaitEvent(st, e, 0));
    return IMPC_OK;
}
static int ctx_note_launch(impc_ctx ctx, hipStream_t st) {
    if (st == ctx->stream) return IMPC_OK;
    // recycle the events of launches that have completed (keeps the pending list short)
    for (size_t k = 0; k < ctx->ev_pending.size();) {
        if (hipEventQuery(ctx->ev_pending[k]) == hipSuccess) {
            ctx->ev_pool.push_back(ctx->ev_pending[k]);
            ctx->ev_pending[k] = ctx->ev_pending.back();
            ctx->ev_pending.pop_back();
        } else {
            k++;
        }
    }
    hipEvent_t e = nullptr;
    if (!ctx->ev_pool.empty()) {
        e = ctx->ev_pool.back();
        ctx->ev_pool.pop_back();
    } else {
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIP_OK(hipEventRecord(e, st));
    ctx->ev_pending.push_back(e);
    return IMPC_OK;
}
static int ctx_quiesce(impc_ctx ctx) {
    HIP_OK(hipStreamSynchronize(ctx->stream));
    for (hipEvent_t e : ctx->ev_pending) HIP_OK(hipEventSynchronize(e));
    ctx->ev_pool.insert(ctx->ev_pool.end(), ctx->ev_pending.begin(), ctx->ev_pending.end());
    ctx->ev_pending.clear();
    return IMPC_OK;
}

struct impc_batch_s {
    impc_ctx ctx = nullptr;
    int64_t n = 0, m = 0, nnzP = 0, nnzA = 0;
    std::vector<int64_t> Pp, Pi, Ap, Ai;  // pattern (host copy)
    int64_t B = 0, S = 0;
    int64_t Bact = 0;  // QPs the solves take (impc_batch_set_active): the first Bact of B
    // or the count in device memory (impc_lib::batch_set_active_device; Bact = B while set): the
    // batch's producer decides it on the device, no host round trip before the solve
    const int64_t *d_active = nullptr;
    impc_settings settings{};
    impc::DevSettings dst{};
    int kernel_req = IMPC_KERNEL_AUTO;
    // QP-major inputs on the device
    double *d_in = nullptr;
    double *in_Px = nullptr, *in_q = nullptr, *in_Ax = nullptr, *in_l = nullptr, *in_u = nullptr, *in_xws = nullptr,
           *in_yws = nullptr;
    double *d_xout = nullptr, *d_yout = nullptr;
    impc_info *d_info = nullptr;
    int64_t device_bytes = 0;
    bool values_set = false, has_ws = false;
    bool ws_y = false;  // the warm start carries duals (else y = 0: nothing uploaded or read)
    unsigned long long *d_qpt = nullptr;  // profiling: per-QP (start, end) device clock
    double *d_tlim = nullptr;  // per-QP time limits (impc_batch_set_time_limits), or none
    bool tlim_on = false;
    // persistent workspace of the structured kernel (impc_batch_set_persistent)
    double *d_persist = nullptr;
    bool persist_on = false, persist_valid = false, q_by_update = false;
    bool rescale = false;  // new P / A values on a persistent workspace (impc_batch_update_matrices)
    bool q_after = false;  // ... and q updated after them: d_qsnap holds the q at the matrix update
    double *d_qsnap = nullptr;
    bool qpt_valid = false;
    // shared-structure values (impc_batch_set_values_shared)
    bool shared = false, shared_expanded = false;
    int64_t nvar = 0, nvar_cap = -1;
    double *d_shPx = nullptr, *d_shAx = nullptr, *d_Axv = nullptr;
    int32_t *d_vmap = nullptr;
    // ---- structured path
    std::unique_ptr<impc::MpcStructure> ms;
    bool structured_ok = false;
    bool tier = false;  // two-tier products layout (grouped-kernel instances only)
    int gs = 0;  // general-row slots per lane of the structured kernel
    int vs = 1;  // variable slots per lane (kWaveVS, or kWaveVSLong for long horizons)
    void *d_tables = nullptr;
    double *d_scal = nullptr;
    unsigned *d_counter = nullptr;
    unsigned long long *d_sec = nullptr;  // section-profiling build only
    impc::WaveTables wt{};
    // ---- generic path (allocated on first use)
    std::unique_ptr<impc::Symbolic> sym;
    void *d_sym = nullptr;
    double *d_work = nullptr;
    impc::DevSym dsym{};
    impc::DevWork dwk{};
    bool generic_dirty = true, generic_setup_done = false, generic_first_run = false;
    // work-queue order of the structured kernel's persistent launches (impc_batch_set_queue_order)
    int queue_mode = IMPC_QUEUE_FIFO;
    double queue_qw = 0.0;
    int32_t *d_csr = nullptr;  // CSR of A's pattern: row_ptr [m + 1], column [nnzA], CSC entry [nnzA]
    // order scratch of the launches this batch heads: keys, sorted keys, indices, order, sort temp
    void *d_qscr = nullptr;
    int64_t qscr_cap = 0;
    size_t qtmp_bytes = 0;
    // profiling
    bool profile = false;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool ev_setup = false, ev_solve = false;
    // small batches: pinned host staging of the inputs, warm start and results (one DMA each way
    // instead of a pageable copy + synchronisation per array), regions [inputs][x ws][y ws][x][y][info].
    // impc_batch_set_values / _warm_start only fill the staging (in_dirty / ws_dirty); the first call
    // that needs them on the device queues one DMA for both (flush_staged)
    double *h_stage = nullptr;
    hipEvent_t ev_in = nullptr;  // the last staged DMA (the staging is rewritten only after it)
    bool in_pending = false;
    bool in_dirty = false, ws_dirty = false;
    size_t ws_len = 0;  // doubles of the staged warm start (x, or x and y)
    uint64_t pool_hash = 0;
};

namespace {

int to_dev_settings(const impc_settings *s, impc::DevSettings *d) {
    if (s->rho <= 0.0 || s->sigma <= 0.0 || s->scaling < 0 || (s->adaptive_rho != 0 && s->adaptive_rho != 1) ||
        s->adaptive_rho_interval < 0 || s->adaptive_rho_fraction <= 0 || s->adaptive_rho_tolerance < 1.0 ||
        s->max_iter <= 0 || s->eps_abs < 0 || s->eps_rel < 0 || (s->eps_abs == 0 && s->eps_rel == 0) ||
        s->eps_prim_inf <= 0 || s->eps_dual_inf <= 0 || s->alpha <= 0 || s->alpha >= 2 || s->delta <= 0 ||
        (s->polish != 0 && s->polish != 1) || s->polish_refine_iter < 0 || (s->verbose != 0 && s->verbose != 1) ||
        (s->scaled_termination != 0 && s->scaled_termination != 1) || s->check_termination < 0 ||
        (s->warm_start != 0 && s->warm_start != 1) || s->time_limit < 0)
        return fail(IMPC_SETTINGS_VALIDATION_ERROR, "invalid settings (OSQP validate_settings)");
    if (s->polish) return fail(IMPC_UNSUPPORTED, "solution polishing is not supported (the reference never enables it)");
    if (s->max_iter > INT32_MAX || s->check_termination > INT32_MAX || s->adaptive_rho_interval > INT32_MAX ||
        s->scaling > INT32_MAX)
        return fail(IMPC_SETTINGS_VALIDATION_ERROR, "integer setting out of range");
    d->rho = s->rho;
    d->sigma = s->sigma;
    d->adaptive_rho_tolerance = s->adaptive_rho_tolerance;
    d->eps_abs = s->eps_abs;
    d->eps_rel = s->eps_rel;
    d->eps_prim_inf = s->eps_prim_inf;
    d->eps_dual_inf = s->eps_dual_inf;
    d->alpha = s->alpha;
    d->time_limit = s->time_limit;
    d->scaling = (int32_t)s->scaling;
    d->adaptive_rho = (int32_t)s->adaptive_rho;
    // adaptive_rho_interval == 0 ("automatic", wall-clock based in the reference): resolved to the
    // interval the reference's own timer produces on these problems.
    d->rho_interval = s->adaptive_rho_interval
                          ? (int32_t)s->adaptive_rho_interval
                          : (int32_t)(s->check_termination ? s->check_termination : 25);
    d->max_iter = (int32_t)s->max_iter;
    d->scaled_termination = (int32_t)s->scaled_termination;
    d->check_termination = (int32_t)s->check_termination;
    d->warm_start = (int32_t)s->warm_start;
    return IMPC_OK;
}

hipStream_t pick(impc_batch b, void *stream) { return stream ? (hipStream_t)stream : b->ctx->stream; }

bool use_structured(impc_batch b) {
    if (b->kernel_req == IMPC_KERNEL_GENERIC) return false;
    return b->structured_ok;
}

int interleave(impc_batch b, const double *src_dev, double *dst, int64_t len, hipStream_t st) {
    if (len <= 0) return IMPC_OK;
    dim3 grid((unsigned)((len + kTile - 1) / kTile), (unsigned)((b->S + kTile - 1) / kTile));
    hipLaunchKernelGGL(k_interleave, grid, dim3(256), 0, st, src_dev, dst, len, b->B, b->S);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int deinterleave(impc_batch b, const double *src, double *dst_dev, int64_t len, hipStream_t st) {
    if (len <= 0) return IMPC_OK;
    // only the active rows: rows >= Bact keep their results (impc_batch_set_active)
    dim3 grid((unsigned)((len + kTile - 1) / kTile), (unsigned)((b->Bact + kTile - 1) / kTile));
    hipLaunchKernelGGL(k_deinterleave, grid, dim3(256), 0, st, src, dst_dev, len, b->Bact, b->S);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

// The structured kernel's view of a batch's inputs / outputs.
impc::WaveIO wave_io(impc_batch b) {
    impc::WaveIO io{b->Bact,     b->shared ? b->d_shPx : b->in_Px, b->in_q, b->shared ? b->d_shAx : b->in_Ax,
                    b->in_l,     b->in_u,   b->in_xws, b->in_yws, b->has_ws ? (b->ws_y ? 1 : 2) : 0, b->d_xout, b->d_yout,
                    b->d_scal,   b->d_info};
    if (b->profile && b->d_qpt) io.qpt = b->d_qpt;
#ifdef IMPC_SECTION_PROF
    io.sec = b->d_sec;
#endif
    if (b->tlim_on) io.tlim = b->d_tlim;
    if (b->persist_on && b->d_persist) {
        io.persist = b->d_persist;
        io.resume = b->persist_valid ? (b->rescale ? 2 : 1) : 0;
        if (b->persist_valid && b->rescale && b->q_after) io.q_scale = b->d_qsnap;
        io.q_updated = b->q_by_update ? 1 : 0;
    }
    b->qpt_valid = io.qpt != nullptr;
    if (b->shared) {
        io.shared = 1;
        io.nvar = b->nvar;
        io.vmap = b->d_vmap;
        io.Ax_var = b->d_Axv;
    }
    return io;
}

// Shared-structure values expanded into the QP-major input arrays (the generic kernel's input)
__global__ void k_expand_shared(const double *Px, const double *Ax, const int32_t *vmap, const double *Axv,
                                int64_t nvar, int64_t nnzP, int64_t nnzA, int64_t B, double *oPx, double *oAx) {
    const int64_t tot = B * (nnzP + nnzA);
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        if (e < B * nnzP) {
            oPx[e] = Px[e % nnzP];
        } else {
            const int64_t f = e - B * nnzP, b = f / nnzA, p = f % nnzA;
            const int32_t v = vmap[p];
            oAx[f] = v >= 0 ? Axv[b * nvar + v] : Ax[p];
        }
    }
}

// ---- generic path: symbolic analysis + interleaved workspace, allocated on first use
int ensure_generic(impc_batch b) {
    if (b->d_work) return IMPC_OK;
    b->sym.reset(new impc::Symbolic());
    std::string err = b->sym->build(b->n, b->m, b->Pp.data(), b->Pi.data(), b->Ap.data(), b->Ai.data());
    if (!err.empty()) return fail(IMPC_DATA_VALIDATION_ERROR, err);
    const impc::Symbolic &s = *b->sym;
    std::vector<const std::vector<int32_t> *> arrs = {&s.Pp, &s.Pi, &s.Ap, &s.Ai, &s.Arp, &s.Arpos, &s.Arcol,
                                                      &s.Arcolf, &s.perm, &s.iperm, &s.Mp, &s.Mi, &s.Mdiag,
                                                      &s.Pt_dest, &s.Pt_src, &s.At_dest, &s.At_a, &s.At_b,
                                                      &s.At_r, &s.Lp, &s.Li, &s.Lrp, &s.Lrc, &s.Lrpos,
                                                      &s.upd_ptr, &s.upd_c, &s.upd_js, &s.upd_je, &s.upd_w};
    std::vector<size_t> offs;
    size_t tot = 0;
    for (auto *a : arrs) {
        offs.push_back(tot);
        tot += (a->size() + 63) / 64 * 64;
    }
    std::vector<int32_t> hsym(tot + 64, 0);
    for (size_t k = 0; k < arrs.size(); k++)
        if (!arrs[k]->empty()) std::memcpy(hsym.data() + offs[k], arrs[k]->data(), arrs[k]->size() * 4);
    HIP_OK(hipMalloc(&b->d_sym, hsym.size() * 4));
    IMPC_TRY(h2d_sync(b->ctx->stream, b->d_sym, hsym.data(), hsym.size() * 4));
    const int32_t *base = (const int32_t *)b->d_sym;
    impc::DevSym &d = b->dsym;
    d.n = s.n;
    d.m = s.m;
    d.nnzP = s.nnzP;
    d.nnzA = s.nnzA;
    d.nnzM = (int32_t)s.nnzM;
    d.nnzL = (int32_t)s.nnzL;
    d.nPt = (int32_t)s.Pt_dest.size();
    d.nAt = (int32_t)s.At_dest.size();
    const int32_t **dst_ptrs[] = {&d.Pp, &d.Pi, &d.Ap, &d.Ai, &d.Arp, &d.Arpos, &d.Arcol, &d.Arcolf,
                                  &d.perm, &d.iperm, &d.Mp, &d.Mi, &d.Mdiag, &d.Pt_dest, &d.Pt_src,
                                  &d.At_dest, &d.At_a, &d.At_b, &d.At_r, &d.Lp, &d.Li, &d.Lrp, &d.Lrc,
                                  &d.Lrpos, &d.upd_ptr, &d.upd_c, &d.upd_js, &d.upd_je, &d.upd_w};
    for (size_t k = 0; k < arrs.size(); k++) *dst_ptrs[k] = base + offs[k];

    const int64_t n_ = s.n, m_ = s.m, nP = s.nnzP, nA = s.nnzA, nM = s.nnzM, nL = s.nnzL;
    struct Slot {
        double **dst;
        int64_t len;
    };
    impc::DevWork &w = b->dwk;
    w.S = b->S;
    double *Px_, *q_, *Ax_, *l_, *u_, *xws_, *yws_;
    std::vector<Slot> slots = {
        {&Px_, nP}, {&q_, n_}, {&Ax_, nA}, {&l_, m_}, {&u_, m_}, {&xws_, n_}, {&yws_, m_},
        {&w.Ps, nP}, {&w.qs, n_}, {&w.As, nA}, {&w.ls, m_}, {&w.us, m_}, {&w.D, n_}, {&w.Dinv, n_},
        {&w.E, m_}, {&w.Einv, m_}, {&w.rho, m_}, {&w.rhoinv, m_}, {&w.ctype, m_}, {&w.scal, impc::SC_NSCAL},
        {&w.x, n_}, {&w.z, m_}, {&w.y, m_}, {&w.v, m_}, {&w.w, n_}, {&w.dx, n_}, {&w.dy, m_},
        {&w.Mval, nM}, {&w.Lx, nL}, {&w.Dinvf, n_}, {&w.yf, n_}, {&w.tn1, n_}, {&w.tm1, m_},
        {&w.xo, n_}, {&w.yo, m_}};
    int64_t per_qp = 0;
    for (auto &sl : slots) per_qp += std::max<int64_t>(sl.len, 1);
    const size_t work_bytes = sizeof(double) * (size_t)per_qp * (size_t)b->S;
    if (hipMalloc((void **)&b->d_work, work_bytes) != hipSuccess) {
        b->d_work = nullptr;
        return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(generic workspace) failed: batch too large for device memory");
    }
    IMPC_TRY(fill0_sync(b->ctx->stream, b->d_work, work_bytes));
    int64_t off = 0;
    for (auto &sl : slots) {
        *sl.dst = b->d_work + off * b->S;
        off += std::max<int64_t>(sl.len, 1);
    }
    w.Px = Px_;
    w.q = q_;
    w.Ax = Ax_;
    w.l = l_;
    w.u = u_;
    w.xws = xws_;
    w.yws = yws_;
    w.info = b->d_info;
    b->device_bytes += (int64_t)(work_bytes + hsym.size() * 4);
    return IMPC_OK;
}

int generic_setup(impc_batch b, hipStream_t st) {
    int rc = ensure_generic(b);
    if (rc) return rc;
    if (b->shared && !b->shared_expanded) {
        const int64_t tot = b->B * (b->nnzP + b->nnzA);
        const int64_t blocks = std::min<int64_t>((tot + 255) / 256, (int64_t)b->ctx->num_cu * 16);
        hipLaunchKernelGGL(k_expand_shared, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, b->d_shPx,
                           b->d_shAx, b->d_vmap, b->d_Axv, b->nvar, b->nnzP, b->nnzA, b->B, b->in_Px, b->in_Ax);
        HIP_OK(hipGetLastError());
        b->shared_expanded = true;
    }
    impc::DevWork &w = b->dwk;
    if ((rc = interleave(b, b->in_Px, const_cast<double *>(w.Px), b->nnzP, st))) return rc;
    if ((rc = interleave(b, b->in_q, const_cast<double *>(w.q), b->n, st))) return rc;
    if ((rc = interleave(b, b->in_Ax, const_cast<double *>(w.Ax), b->nnzA, st))) return rc;
    if ((rc = interleave(b, b->in_l, const_cast<double *>(w.l), b->m, st))) return rc;
    if ((rc = interleave(b, b->in_u, const_cast<double *>(w.u), b->m, st))) return rc;
    if (b->has_ws) {
        if ((rc = interleave(b, b->in_xws, const_cast<double *>(w.xws), b->n, st))) return rc;
        if (!b->ws_y && b->m) HIP_OK(hipMemsetAsync(b->in_yws, 0, sizeof(double) * b->m * b->B, st));
        if ((rc = interleave(b, b->in_yws, const_cast<double *>(w.yws), b->m, st))) return rc;
    }
    if (b->profile) HIP_OK(hipEventRecord(b->ev[0], st));
    hipLaunchKernelGGL(k_setup, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk, b->dst, b->Bact,
                       b->has_ws ? 1 : 0);
    HIP_OK(hipGetLastError());
    if (b->profile) {
        HIP_OK(hipEventRecord(b->ev[1], st));
        b->ev_setup = true;
    }
    b->generic_dirty = false;
    b->generic_setup_done = true;
    b->generic_first_run = true;
    return IMPC_OK;
}

int generic_solve(impc_batch b, hipStream_t st) {
    b->qpt_valid = false;  // per-QP latency is recorded by the structured kernel only
    if (b->generic_dirty) {
        int rc = generic_setup(b, st);
        if (rc) return rc;
    }
    const int first_run = b->generic_first_run ? 1 : 0;
    b->generic_first_run = false;
    b->dwk.tlim = b->tlim_on ? b->d_tlim : nullptr;
    if (b->profile) HIP_OK(hipEventRecord(b->ev[2], st));
    hipLaunchKernelGGL(k_solve, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk, b->dst, b->Bact,
                       first_run);
    HIP_OK(hipGetLastError());
    if (b->profile) HIP_OK(hipEventRecord(b->ev[3], st));
    int rc = deinterleave(b, b->dwk.xo, b->d_xout, b->n, st);
    if (!rc) rc = deinterleave(b, b->dwk.yo, b->d_yout, b->m, st);
    if (!rc && b->profile) {
        HIP_OK(hipEventRecord(b->ev[4], st));
        b->ev_solve = true;
    }
    return rc;
}

// ---- structured path
// The raised dynamic-LDS limit is set once per kernel instantiation (grow-only).
template <class K>
int ensure_lds_attr(K kernel, size_t lds) {
    static size_t attr_bytes = 0;
    if (lds > attr_bytes) {
        HIP_OK(hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_bytes = lds;
    }
    return IMPC_OK;
}

// resident workgroups per CU: the waves-per-SIMD budget of the shape, and LDS
template <int VS>
int64_t resident_groups(int num_cu, size_t lds, int64_t work) {
    const int per_cu = std::max<int>(1, std::min<int>(Shape<VS>::PER_CU, (int)((160 * 1024 - 1024) / lds)));
    return std::min<int64_t>(work, (int64_t)num_cu * per_cu);
}

// the compile-time horizon instance that takes the batch: its W when the shape has one for it
// (WSPEC: the default horizon of the shape; WSPEC2: the long shape's N = 30), else 0 (runtime W)
int spec_w(impc_batch b) {
    using LL = impc::WaveLds<256, kWaveVSLong, 2>;
    using LD1 = impc::WaveLds<256, kWaveVS, 2>;
    const int W = b->ms->W;
    if (b->vs == kWaveVSLong) return (W == LL::WSPEC || (LL::WSPEC2 && W == LL::WSPEC2)) ? W : 0;
    return (W == LD1::WSPEC || (LD1::WSPEC2 && W == LD1::WSPEC2)) ? W : 0;
}

// ---- work-queue order (impc_batch_set_queue_order, csrc/queue.hpp)
// CSR of A's pattern with each entry's CSC index, built once per batch on the host
int build_queue_csr(impc_batch b) {
    if (b->d_csr) return IMPC_OK;
    const int64_t m = b->m, nnz = b->nnzA;
    std::vector<int32_t> h((size_t)(m + 1 + 2 * nnz), 0);
    int32_t *rp = h.data(), *col = rp + m + 1, *ent = col + nnz;
    for (int64_t k = 0; k < nnz; k++) rp[b->Ai[(size_t)k] + 1]++;
    for (int64_t r = 0; r < m; r++) rp[r + 1] += rp[r];
    std::vector<int32_t> fill(rp, rp + m);
    for (int64_t j = 0; j < b->n; j++)
        for (int64_t k = b->Ap[(size_t)j]; k < b->Ap[(size_t)j + 1]; k++) {
            const int32_t at = fill[(size_t)b->Ai[(size_t)k]]++;
            col[at] = (int32_t)j;
            ent[at] = (int32_t)k;
        }
    HIP_OK(hipMalloc((void **)&b->d_csr, sizeof(int32_t) * h.size()));
    b->device_bytes += (int64_t)(sizeof(int32_t) * h.size());
    return h2d_sync(b->ctx->stream, b->d_csr, h.data(), sizeof(int32_t) * h.size());
}

// The queue order of one persistent launch over bs[0 .. count) (bs[k]'s QPs at launch-wide queue
// indices firsts[k] ..): when any of them asks for IMPC_QUEUE_LONGEST_FIRST, every QP's key on the
// device (each batch with its own q_weight), sorted descending (stable: ties in queue order).
// *ord = the permutation (scratch of bs[0]), or nullptr for the plain FIFO queue.
int queue_order(impc_batch *bs, const int64_t *firsts, int count, int64_t total, hipStream_t st,
                const uint32_t **ord) {
    *ord = nullptr;
    bool any = false, devcnt = false;
    for (int k = 0; k < count; k++) {
        any = any || bs[k]->queue_mode == IMPC_QUEUE_LONGEST_FIRST;
        devcnt = devcnt || bs[k]->d_active != nullptr;
    }
    // device-side active counts: always a permutation, active QPs first (FIFO order among them
    // unless a batch asks for the longest-first order), the inactive rows' keys -inf
    if (!devcnt && (!any || total < 2)) return IMPC_OK;
    // the radix sort takes an int item count
    if (total > (int64_t)INT32_MAX) return fail(IMPC_UNSUPPORTED, "queue order: too many QPs in one launch");
    impc_batch h = bs[0];
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, (const double *)nullptr, (double *)nullptr,
                                                        (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)total,
                                                        0, 64, st));
    auto bytes_for = [](int64_t cap, size_t t) { return (size_t)cap * (2 * sizeof(double) + 2 * sizeof(uint32_t)) + t; };
    if (total > h->qscr_cap || tmp > h->qtmp_bytes) {
        IMPC_TRY(ctx_quiesce(h->ctx));  // no launch in flight reads the order being replaced
        if (h->d_qscr) {
            HIP_OK(hipFree(h->d_qscr));
            h->device_bytes -= (int64_t)bytes_for(h->qscr_cap, h->qtmp_bytes);
        }
        h->d_qscr = nullptr;
        h->qscr_cap = std::max(total, h->qscr_cap);
        h->qtmp_bytes = std::max(tmp, h->qtmp_bytes);
        HIP_OK(hipMalloc(&h->d_qscr, bytes_for(h->qscr_cap, h->qtmp_bytes)));
        h->device_bytes += (int64_t)bytes_for(h->qscr_cap, h->qtmp_bytes);
    }
    double *key = (double *)h->d_qscr, *key2 = key + h->qscr_cap;
    uint32_t *idx = (uint32_t *)(key2 + h->qscr_cap), *out = idx + h->qscr_cap;
    void *t = (void *)(out + h->qscr_cap);
    for (int k = 0; k < count; k++) {
        impc_batch b = bs[k];
        if (b->Bact == 0) continue;
        IMPC_TRY(build_queue_csr(b));
        impc::QueueKeyArgs a{};
        a.B = b->Bact, a.n = b->n, a.m = b->m, a.first = firsts[k];
        a.row_ptr = b->d_csr, a.row_col = b->d_csr + b->m + 1, a.row_ent = b->d_csr + b->m + 1 + b->nnzA;
        a.shared = b->shared ? 1 : 0;
        a.Ax = b->shared ? b->d_shAx : b->in_Ax;
        a.nvar = b->nvar, a.vmap = b->d_vmap, a.Ax_var = b->d_Axv;
        a.q = b->in_q, a.l = b->in_l, a.u = b->in_u, a.xws = b->in_xws, a.has_ws = b->has_ws ? 1 : 0;
        a.q_weight = b->queue_qw;
        a.dcount = b->d_active;
        a.fifo = any ? 0 : 1;
        const unsigned grid = (unsigned)std::min<int64_t>(b->Bact, 4096);
        hipLaunchKernelGGL(impc::k_queue_key, dim3(grid), dim3(256), 0, st, a, key, idx);
        HIP_OK(hipGetLastError());
    }
    HIP_OK(hipcub::DeviceRadixSort::SortPairsDescending(t, tmp, key, key2, idx, out, (int)total, 0, 64, st));
    *ord = out;
    return IMPC_OK;
}

// runtime (VS, GS, TIER) -> the instantiated kernel class: f(VS, GS, TIER) as integral constants
template <int V, int G, bool TR, class F>
int shape_call(F &&f) {
    return f(std::integral_constant<int, V>{}, std::integral_constant<int, G>{}, std::integral_constant<bool, TR>{});
}
template <int V, bool TR, class F>
int with_gs(int gs, F &&f) {
    constexpr int gmax = TR ? Shape<V>::TIER_GMAX : Shape<V>::GMAX;
    switch (gs) {
        case 2: if constexpr (gmax >= 2) return shape_call<V, 2, TR>(f); break;
        case 3: if constexpr (gmax >= 3) return shape_call<V, 3, TR>(f); break;
        case 4: if constexpr (gmax >= 4) return shape_call<V, 4, TR>(f); break;
        case 5: if constexpr (gmax >= 5) return shape_call<V, 5, TR>(f); break;
        case 6: if constexpr (gmax >= 6) return shape_call<V, 6, TR>(f); break;
        default: break;
    }
    return fail(IMPC_UNSUPPORTED, "no structured kernel for this size");
}
template <class F>
int with_shape(int vs, int gs, bool tier, F &&f) {
    switch (vs) {
        case kWaveVSFront:
            if constexpr (IMPC_WAVEFRONT != 0)
                return tier ? with_gs<kWaveVSFront, true>(gs, f) : with_gs<kWaveVSFront, false>(gs, f);
            break;
        case kWaveVS: return tier ? with_gs<kWaveVS, true>(gs, f) : with_gs<kWaveVS, false>(gs, f);
        case kWaveVSLong: return tier ? with_gs<kWaveVSLong, true>(gs, f) : with_gs<kWaveVSLong, false>(gs, f);
        default: break;
    }
    return fail(IMPC_UNSUPPORTED, "no structured kernel for this size");
}

// After a structured solve of a persistent batch: its workspace holds the scaled iterates, and an
// explicit warm start has been consumed (OSQP applies osqp_warm_start once).
void structured_solved(impc_batch b) {
    if (!b->persist_on) return;
    b->persist_valid = true;
    b->rescale = b->q_after = false;
    b->has_ws = false;
}

// One batch's structured solve: a grouped launch of one entry (the entry table is cached, so
// repeated solves of a batch upload nothing)
int structured_solve(impc_batch b, hipStream_t st) {
#ifdef IMPC_SECTION_PROF
    if (!b->d_sec) {
        HIP_OK(hipMalloc((void **)&b->d_sec, sizeof(unsigned long long) * impc::kSecCount));
        HIP_OK(hipMemsetAsync(b->d_sec, 0, sizeof(unsigned long long) * impc::kSecCount, st));
    }
#endif
    return impc_batch_solve_group(&b, 1, st);
}

template <int VS, int GS, int WF, bool TIER>
int launch_group_w(impc_ctx ctx, hipStream_t st, const GroupEntry *entries, int count, int64_t total, size_t lds,
                   unsigned *counter, const uint32_t *ord, int devcnt) {
    using S = Shape<VS>;
    if (int rc = ensure_lds_attr(k_mpc_wave_group<S::NL, VS, GS, S::WPS, WF, TIER>, lds)) return rc;
    const int64_t groups = resident_groups<VS>(ctx->num_cu, lds, total);
    hipLaunchKernelGGL((k_mpc_wave_group<S::NL, VS, GS, S::WPS, WF, TIER>), dim3((unsigned)groups), dim3(S::NL), lds,
                       st, entries, count, total, counter, ord, devcnt);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}
// spec: the compile-time horizon every batch of the launch shares (spec_w), or 0
template <int VS, int GS, bool TIER = false>
int launch_group(impc_ctx ctx, hipStream_t st, const GroupEntry *entries, int count, int64_t total, size_t lds,
                 unsigned *counter, int spec, const uint32_t *ord, int devcnt) {
    using LD = impc::WaveLds<Shape<VS>::NL, VS, GS>;
    constexpr int WS = LD::WSPEC, WS2 = LD::WSPEC2;
    if (spec && spec == WS)
        return launch_group_w<VS, GS, WS, TIER>(ctx, st, entries, count, total, lds, counter, ord, devcnt);
    if constexpr (WS2 != 0)
        if (spec == WS2)
            return launch_group_w<VS, GS, WS2, TIER>(ctx, st, entries, count, total, lds, counter, ord, devcnt);
    return launch_group_w<VS, GS, 0, TIER>(ctx, st, entries, count, total, lds, counter, ord, devcnt);
}

// dynamic LDS bytes of the structured kernel for a shape (team VS, GS) and pattern (CG, n); 0 if
// the shape has no kernel for GS
size_t wave_lds_bytes(int vs, int gs, const impc::WaveTables &T) {
    size_t bytes = 0;
    (void)with_shape(vs, gs, false, [&](auto v, auto g, auto) {
        constexpr int V = decltype(v)::value;
        bytes = sizeof(double) * (size_t)impc::WaveLds<Shape<V>::NL, V, decltype(g)::value>::size(T);
        return IMPC_OK;
    });
    return bytes;
}

// A library built with the wavefront shape uses it unless IMPC_WAVEFRONT_SHAPE=0 is in the
// environment when the batch is created (A/B in one process).
// The scaling vectors of the wavefront / long shapes in LDS where it has the room (WaveTables::
// scal_lds) unless IMPC_SCAL_LDS=0 is in the environment when the batch is created (A/B).
bool scal_lds_on() {
    const char *e = std::getenv("IMPC_SCAL_LDS");
    return !(e && e[0] == '0');
}

bool wavefront_shape_on() {
    const char *e = std::getenv("IMPC_WAVEFRONT_SHAPE");
    return IMPC_WAVEFRONT != 0 && !(e && e[0] == '0');
}

// Shape selection: (when built) the wavefront shape if the pattern fits it with four QPs per CU,
// else the team shape (n <= 256), else the long shape.  Sets b->vs, b->gs, b->tier and the tables' layout
// fields; false if no structured shape takes the pattern.
bool choose_shape(impc_batch b) {
    const impc::MpcStructure &s = *b->ms;
    impc::WaveTables &t = b->wt;
    t.n = s.n;
    t.m = s.m;
    t.mg = s.mg;
    t.N = s.N;
    t.W = s.W;
    t.CG = s.CG;
    t.nnzP = s.nnzP;
    t.nnzA = s.nnzA;
    auto fit = [&](int vs, int nl, int gmax, int tier_gmax, int per_cu, bool need_full) -> bool {
        if (s.n > nl * vs) return false;
        const int g = std::max(2, (s.mg + nl - 1) / nl);  // general-row slots per lane
        if (g > gmax) return false;
        const size_t budget = (160 * 1024 - 1024) / (size_t)per_cu;
        // products layout (mpc_wave.hpp WaveLds): one tier unless it would cost the shape a resident
        // team per CU, then the heavy columns' overflow in a second tier
        t.HS = 0;
        t.T1r = impc::WaveLds<256, kWaveVS, 2>::cg4(s.CG);
        if (g <= tier_gmax && wave_lds_bytes(vs, g, t) > budget) {
            t.HS = s.HS;
            t.T1r = impc::kProdTier1;
        }
        const size_t lds = wave_lds_bytes(vs, g, t);
        if (!lds || lds > (need_full ? budget : (size_t)(160 * 1024 - 1024))) return false;
        b->vs = vs;
        b->gs = g;
        // D, E in LDS when the shape keeps them in HBM and the room costs no resident team
        t.scal_lds = 0;
        if (!(vs == kWaveVS && impc::WaveLds<256, kWaveVS, 2>::ONCHIP) && scal_lds_on()) {
            impc::WaveTables t2 = t;
            t2.scal_lds = 1;
            const size_t cap = 160 * 1024 - 1024, l2 = wave_lds_bytes(vs, g, t2);
            if (l2 && l2 <= cap && cap / l2 >= std::min<size_t>(cap / lds, (size_t)per_cu)) t.scal_lds = 1;
        }
        b->tier = t.T1r < impc::WaveLds<256, kWaveVS, 2>::cg4(s.CG);
        return true;
    };
    using F = Shape<kWaveVSFront>;
    using T1 = Shape<kWaveVS>;
    using L = Shape<kWaveVSLong>;
    if (wavefront_shape_on() && fit(kWaveVSFront, F::NL, F::GMAX, F::TIER_GMAX, F::PER_CU, true)) return true;
    if (fit(kWaveVS, T1::NL, T1::GMAX, T1::TIER_GMAX, T1::PER_CU, false)) return true;
    return fit(kWaveVSLong, L::NL, L::GMAX, L::TIER_GMAX, L::PER_CU, false);
}

int prepare_structured(impc_batch b) {
    b->ms.reset(new impc::MpcStructure());
    std::string why = b->ms->analyse(b->n, b->m, b->Pp.data(), b->Pi.data(), b->Ap.data(), b->Ai.data());
    if (!why.empty() || b->ms->CG > impc::WaveLds<256, kWaveVS, 2>::CGM || !choose_shape(b)) {
        b->structured_ok = false;  // the generic kernel takes it
        return IMPC_OK;
    }
    const impc::MpcStructure &s = *b->ms;
    impc::WaveTables &t = b->wt;
    std::vector<const std::vector<int32_t> *> arrs = {&s.var_orig, &s.var_pdiag, &s.var_boxrow, &s.var_boxpos,
                                                      &s.gen_row,  &s.gen_col,   &s.gen_pos,    &s.colg,
                                                      &s.term_ptr, &s.term,      &s.col_hid};
    std::vector<size_t> offs;
    size_t tot = 0;
    for (auto *a : arrs) {
        offs.push_back(tot);
        tot += (a->size() + 63) / 64 * 64;
    }
    std::vector<int32_t> h(tot + 64, 0);
    for (size_t k = 0; k < arrs.size(); k++)
        if (!arrs[k]->empty()) std::memcpy(h.data() + offs[k], arrs[k]->data(), arrs[k]->size() * 4);
    HIP_OK(hipMalloc(&b->d_tables, h.size() * 4));
    IMPC_TRY(h2d_sync(b->ctx->stream, b->d_tables, h.data(), h.size() * 4));
    const int32_t *base = (const int32_t *)b->d_tables;
    const int32_t **dst_ptrs[] = {&t.var_orig, &t.var_pdiag, &t.var_boxrow, &t.var_boxpos, &t.gen_row,
                                  &t.gen_col,  &t.gen_pos,   &t.colg,       &t.term_ptr,   &t.term,
                                  &t.col_hid};
    for (size_t k = 0; k < arrs.size(); k++) *dst_ptrs[k] = base + offs[k];
    // per-QP HBM scratch for the scaling vectors: the wavefront and long shapes (the team shape keeps
    // them in LDS, mpc_wave.hpp WaveLds::ONCHIP)
    const bool onchip = (b->vs == kWaveVS && impc::WaveLds<256, kWaveVS, 2>::ONCHIP) || t.scal_lds;
    const size_t scal_bytes = onchip ? 0 : sizeof(double) * (size_t)b->B * (size_t)(2 * s.n + s.mg);
    if (scal_bytes) HIP_OK(hipMalloc((void **)&b->d_scal, scal_bytes));
    HIP_OK(hipMalloc((void **)&b->d_counter, 256));
    b->device_bytes += (int64_t)(scal_bytes + h.size() * 4 + 256);
    b->structured_ok = true;
    return IMPC_OK;
}

// ---- pinned staging of small batches (impc_batch_set_values / _warm_start / _get)
constexpr size_t kStageMax = (size_t)8 << 20;  // bytes: inputs + warm start + results of the batch
size_t stage_in_len(const impc_batch_s *b) { return (size_t)b->B * (size_t)(b->nnzP + b->n + b->nnzA + 2 * b->m); }
size_t stage_len(const impc_batch_s *b) {
    return stage_in_len(b) + (size_t)b->B * (size_t)(2 * (b->n + b->m)) + (size_t)b->B * sizeof(impc_info) / 8;
}
bool stage_ok(const impc_batch_s *b) { return 8 * stage_len(b) <= kStageMax; }
double *stage_xws(impc_batch b) { return b->h_stage + stage_in_len(b); }
double *stage_xout(impc_batch b) { return stage_xws(b) + (size_t)b->B * (size_t)(b->n + b->m); }
int stage_ensure(impc_batch b) {
    if (b->h_stage) return IMPC_OK;
    HIP_OK(hipHostMalloc((void **)&b->h_stage, 8 * stage_len(b), hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&b->ev_in, hipEventDisableTiming));
    return IMPC_OK;
}
// before the host rewrites the staging: the last DMA from it has completed
int stage_wait(impc_batch b) {
    if (b->in_pending) HIP_OK(hipEventSynchronize(b->ev_in));
    b->in_pending = false;
    return IMPC_OK;
}
// the staged inputs and / or warm start to the device: one DMA on the context stream, after every
// launch (on any stream) that may still read the arrays it replaces.  The device regions
// [inputs][x ws][y ws] are contiguous in the staging's order, so both go in one copy.  Called by
// every entry point that reads or rewrites the device inputs.
int flush_staged(impc_batch b) {
    if (!b->in_dirty && !b->ws_dirty) return IMPC_OK;
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    IMPC_TRY(ctx_order_after_all(b->ctx, st));
    const size_t in_len = stage_in_len(b);
    const size_t off = b->in_dirty ? 0 : in_len, end = b->ws_dirty ? in_len + b->ws_len : in_len;
    HIP_OK(hipMemcpyAsync(b->in_Px + off, b->h_stage + off, sizeof(double) * (end - off), hipMemcpyHostToDevice, st));
    HIP_OK(hipEventRecord(b->ev_in, st));
    b->in_pending = true;
    b->in_dirty = b->ws_dirty = false;
    return IMPC_OK;
}

// the state impc_batch_create leaves (a batch taken from the workspace pool)
void reset_batch(impc_batch b) {
    impc_default_settings(&b->settings);
    to_dev_settings(&b->settings, &b->dst);
    b->dst.tick_s = b->ctx->tick_s;
    b->kernel_req = IMPC_KERNEL_AUTO;
    b->values_set = b->has_ws = b->ws_y = b->tlim_on = false;
    b->persist_on = b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;
    b->profile = b->qpt_valid = b->ev_setup = b->ev_solve = false;
    b->queue_mode = IMPC_QUEUE_FIFO;
    b->queue_qw = 0.0;
    b->Bact = b->B;
    b->shared = b->shared_expanded = false;
    b->generic_dirty = true;
    b->generic_setup_done = b->generic_first_run = false;
    b->in_dirty = b->ws_dirty = false;
}

uint64_t pattern_hash(int64_t n, int64_t m, int64_t batch, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                      const int64_t *Ai) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const int64_t *a, int64_t len) {
        for (int64_t k = 0; k < len; k++) h = (h ^ (uint64_t)a[k]) * 1099511628211ull;
    };
    const int64_t hdr[3] = {n, m, batch};
    mix(hdr, 3);
    mix(Pp, n + 1);
    if (Pi) mix(Pi, Pp[n]);
    mix(Ap, n + 1);
    mix(Ai, Ap[n]);
    return h;
}

}  // namespace

extern "C" {

void impc_default_settings(impc_settings *s) {
    if (!s) return;
    s->rho = 0.1;                     // constants.h:59
    s->sigma = 1e-06;                 // :60
    s->scaling = 10;                  // :85
    s->adaptive_rho = 1;              // :109
    s->adaptive_rho_interval = 0;     // :110
    s->adaptive_rho_tolerance = 5;    // :114
    s->adaptive_rho_fraction = 0.4;   // :111
    s->max_iter = 4000;               // :61
    s->eps_abs = 1e-3;                // :62
    s->eps_rel = 1e-3;                // :63
    s->eps_prim_inf = 1e-4;           // :64
    s->eps_dual_inf = 1e-4;           // :65
    s->alpha = 1.6;                   // :66
    s->linsys_solver = 0;             // QDLDL_SOLVER
    s->delta = 1e-6;                  // :71
    s->polish = 0;                    // :72
    s->polish_refine_iter = 3;        // :73
    s->verbose = 1;                   // :74
    s->scaled_termination = 0;        // :82
    s->check_termination = 25;        // :83
    s->warm_start = 1;                // :84
    s->time_limit = 0;                // :117
}

const char *impc_last_error(void) { return g_last_error.c_str(); }
const char *impc_version(void) { return IMPC_VERSION; }
const char *impc_build_id(void) { return IMPC_BUILD_ID; }

int impc_ctx_create(int device, impc_ctx *out) {
    if (!out) return fail(IMPC_INVALID_ARGUMENT, "null output pointer");
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0)
        return fail(IMPC_DEVICE_ERROR, "no HIP device available: the batched solver runs only on the GPU");
    if (device < 0 || device >= count) return fail(IMPC_INVALID_ARGUMENT, "device index out of range");
    HIP_OK(hipSetDevice(device));
    impc_ctx c = new impc_ctx_s();
    c->device = device;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
        c->num_cu = ncu;
    int khz = 0;  // rate of the constant-rate clock the kernels read (s_memrealtime), kHz
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) {
        delete c;
        return fail(IMPC_DEVICE_ERROR, "hipDeviceAttributeWallClockRate unavailable: time limits cannot be measured");
    }
    c->tick_s = 1.0 / (1e3 * (double)khz);
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(IMPC_DEVICE_ERROR, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = c;
    return IMPC_OK;
}

int impc_ctx_destroy(impc_ctx ctx) {
    if (!ctx) return IMPC_OK;
    (void)hipSetDevice(ctx->device);
    (void)ctx_quiesce(ctx);
    auto pool = std::move(ctx->pool);  // (impc_batch_destroy looks the batch up in ctx->pool)
    ctx->pool.clear();
    for (auto &e : pool) (void)impc_batch_destroy(e.second);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    for (auto &g : ctx->groups)
        if (g.d) (void)hipFree(g.d);
    for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->ev_pending) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->timer_marks) (void)hipEventDestroy(e);
    if (ctx->ev_order) (void)hipEventDestroy(ctx->ev_order);
    delete ctx;
    return IMPC_OK;
}

void *impc_ctx_stream(impc_ctx ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int impc_ctx_synchronize(impc_ctx ctx) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    HIP_OK(hipDeviceSynchronize());
    return IMPC_OK;
}

int impc_batch_create(impc_ctx ctx, int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                      const int64_t *Ai, int64_t batch, impc_batch *out) {
    if (!ctx || !out) return fail(IMPC_INVALID_ARGUMENT, "null context or output");
    *out = nullptr;
    if (batch <= 0 || batch > (int64_t)1 << 30) return fail(IMPC_INVALID_ARGUMENT, "batch must be in [1, 2^30]");
    if (n <= 0 || m < 0 || !Pp || !Ap) return fail(IMPC_DATA_VALIDATION_ERROR, "invalid dimensions or pattern");
    // validate the pattern once (OSQP validate_data: P upper triangular, indices in range)
    impc::Symbolic check;
    std::string err = check.build(n, m, Pp, Pi, Ap, Ai);
    if (!err.empty()) return fail(IMPC_DATA_VALIDATION_ERROR, err);
    HIP_OK(hipSetDevice(ctx->device));
    std::unique_ptr<impc_batch_s> b(new impc_batch_s());
    b->ctx = ctx;
    b->n = n;
    b->m = m;
    b->nnzP = Pp[n];
    b->nnzA = Ap[n];
    b->Pp.assign(Pp, Pp + n + 1);
    b->Pi.assign(Pi ? Pi : Pp, Pi ? Pi + b->nnzP : Pp);
    b->Ap.assign(Ap, Ap + n + 1);
    b->Ai.assign(Ai, Ai + b->nnzA);
    b->B = b->Bact = batch;
    b->S = (batch + kBlock - 1) / kBlock * kBlock;
    impc_default_settings(&b->settings);
    to_dev_settings(&b->settings, &b->dst);
    b->dst.tick_s = ctx->tick_s;
    const int64_t B = batch;
    const int64_t in_len = b->nnzP + b->n + b->nnzA + 2 * b->m + b->n + b->m;
    const size_t in_bytes = sizeof(double) * (size_t)(in_len * B + 8);
    if (hipMalloc((void **)&b->d_in, in_bytes) != hipSuccess)
        return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(inputs) failed: batch too large for device memory");
    double *p = b->d_in;
    b->in_Px = p;
    p += b->nnzP * B;
    b->in_q = p;
    p += b->n * B;
    b->in_Ax = p;
    p += b->nnzA * B;
    b->in_l = p;
    p += b->m * B;
    b->in_u = p;
    p += b->m * B;
    b->in_xws = p;
    p += b->n * B;
    b->in_yws = p;
    IMPC_TRY(fill0_sync(ctx->stream, b->d_in, in_bytes));
    // results [x][y][info] in one allocation, so a small batch's results come back in one DMA
    // (impc_batch_get; the staging's result regions have the same order)
    const size_t xo_len = (size_t)n * (size_t)B, yo_len = (size_t)std::max<int64_t>(m, 1) * (size_t)B;
    if (hipMalloc((void **)&b->d_xout, sizeof(double) * (xo_len + yo_len) + sizeof(impc_info) * (size_t)B) != hipSuccess)
        return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(results) failed");
    b->d_yout = b->d_xout + xo_len;
    b->d_info = (impc_info *)(b->d_yout + yo_len);
    IMPC_TRY(fill0_sync(ctx->stream, b->d_info, sizeof(impc_info) * (size_t)B));
    b->device_bytes = (int64_t)(in_bytes + sizeof(double) * (n + m) * B + sizeof(impc_info) * B);
    int rc = prepare_structured(b.get());
    if (rc) return rc;
    *out = b.release();
    return IMPC_OK;
}

int impc_batch_destroy(impc_batch b) {
    if (!b) return IMPC_OK;
    if (b->ctx) {
        (void)hipSetDevice(b->ctx->device);
        (void)ctx_quiesce(b->ctx);
        // a released batch destroyed by its holder leaves the pool (no second destroy at ctx_destroy)
        auto &pool = b->ctx->pool;
        for (size_t k = 0; k < pool.size(); k++)
            if (pool[k].second == b) {
                pool.erase(pool.begin() + (std::ptrdiff_t)k);
                break;
            }
    }
    for (hipEvent_t e : b->ev)
        if (e) (void)hipEventDestroy(e);
    if (b->ev_in) (void)hipEventDestroy(b->ev_in);
    if (b->h_stage) (void)hipHostFree(b->h_stage);
    void *ptrs[] = {b->d_in,     b->d_xout,  b->d_tables, b->d_scal, b->d_counter,
                    b->d_sym,    b->d_work,  b->d_sec,   b->d_shPx,  b->d_shAx,   b->d_Axv,  b->d_vmap,
                    b->d_qpt,    b->d_persist, b->d_tlim, b->d_csr, b->d_qscr, b->d_qsnap};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete b;
    return IMPC_OK;
}

int impc_batch_acquire(impc_ctx ctx, int64_t n, int64_t m, const int64_t *Pp, const int64_t *Pi, const int64_t *Ap,
                       const int64_t *Ai, int64_t batch, impc_batch *out) {
    if (!ctx || !out) return fail(IMPC_INVALID_ARGUMENT, "null context or output");
    *out = nullptr;
    if (n <= 0 || m < 0 || !Pp || !Ap || batch <= 0) return fail(IMPC_DATA_VALIDATION_ERROR, "invalid dimensions or pattern");
    const uint64_t h = pattern_hash(n, m, batch, Pp, Pi, Ap, Ai);
    for (size_t k = ctx->pool.size(); k-- > 0;) {
        impc_batch b = ctx->pool[k].second;
        if (ctx->pool[k].first != h || b->n != n || b->m != m || b->B != batch || b->nnzP != Pp[n] ||
            b->nnzA != Ap[n])
            continue;
        if (!std::equal(b->Pp.begin(), b->Pp.end(), Pp) || (b->nnzP && !std::equal(b->Pi.begin(), b->Pi.end(), Pi)) ||
            !std::equal(b->Ap.begin(), b->Ap.end(), Ap) || !std::equal(b->Ai.begin(), b->Ai.end(), Ai))
            continue;
        ctx->pool.erase(ctx->pool.begin() + (std::ptrdiff_t)k);
        reset_batch(b);
        *out = b;
        return IMPC_OK;
    }
    int rc = impc_batch_create(ctx, n, m, Pp, Pi, Ap, Ai, batch, out);
    if (!rc) (*out)->pool_hash = h;
    return rc;
}

int impc_batch_release(impc_batch b) {
    if (!b) return IMPC_OK;
    impc_ctx ctx = b->ctx;
    if (!b->pool_hash)  // a batch of impc_batch_create: hash it now
        b->pool_hash = pattern_hash(b->n, b->m, b->B, b->Pp.data(), b->nnzP ? b->Pi.data() : nullptr, b->Ap.data(),
                                    b->Ai.data());
    for (const auto &e : ctx->pool)
        if (e.second == b) return fail(IMPC_INVALID_ARGUMENT, "batch released twice");
    constexpr size_t kPoolMax = 64;  // released batches kept per context (oldest freed first)
    if (ctx->pool.size() >= kPoolMax) {
        // out of the pool first: impc_batch_destroy would otherwise look it up and erase it itself
        impc_batch old = ctx->pool.front().second;
        ctx->pool.erase(ctx->pool.begin());
        (void)impc_batch_destroy(old);
    }
    ctx->pool.emplace_back(b->pool_hash, b);
    return IMPC_OK;
}

int impc_ctx_pool_stats(impc_ctx ctx, int64_t *batches, int64_t *device_bytes) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    int64_t bytes = 0;
    for (const auto &e : ctx->pool) bytes += e.second->device_bytes;
    if (batches) *batches = (int64_t)ctx->pool.size();
    if (device_bytes) *device_bytes = bytes;
    return IMPC_OK;
}

int impc_batch_set_kernel(impc_batch b, int kernel) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (kernel != IMPC_KERNEL_AUTO && kernel != IMPC_KERNEL_GENERIC && kernel != IMPC_KERNEL_STRUCTURED)
        return fail(IMPC_INVALID_ARGUMENT, "unknown kernel id");
    if (kernel == IMPC_KERNEL_STRUCTURED && !b->structured_ok)
        return fail(IMPC_UNSUPPORTED, "pattern is not a stage-structured MPC QP within the wave kernel's limits");
    b->kernel_req = kernel;
    return IMPC_OK;
}

int impc_batch_set_settings(impc_batch b, const impc_settings *s) {
    if (!b || !s) return fail(IMPC_INVALID_ARGUMENT, "null batch or settings");
    impc::DevSettings d{};
    int rc = to_dev_settings(s, &d);
    if (rc) return rc;
    d.tick_s = b->ctx->tick_s;
    if (b->persist_on && s->scaling > impc::kPersistMaxScaling)
        return fail(IMPC_UNSUPPORTED, "persistent workspaces support scaling <= 20 Ruiz passes");
    if (s->rho != b->settings.rho || s->sigma != b->settings.sigma || s->scaling != b->settings.scaling) {
        b->generic_dirty = true;
        b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;  // a different setup: the next solve starts over
    }
    b->settings = *s;
    b->dst = d;
    return IMPC_OK;
}

int impc_batch_set_values(impc_batch b, const double *Px, const double *q, const double *Ax, const double *l,
                          const double *u) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if ((b->nnzP && !Px) || !q || (b->nnzA && !Ax) || (b->m && (!l || !u)))
        return fail(IMPC_INVALID_ARGUMENT, "null value array");
    for (int64_t k = 0; k < b->m * b->B; k++)
        if (l[k] > u[k]) {
            char msg[160];
            std::snprintf(msg, sizeof msg, "lower bound greater than upper bound (QP %lld, row %lld)",
                          (long long)(k / b->m), (long long)(k % b->m));
            return fail(IMPC_DATA_VALIDATION_ERROR, msg);
        }
    HIP_OK(hipSetDevice(b->ctx->device));
    const size_t B = (size_t)b->B;
    if (stage_ok(b)) {
        // small batch: the five arrays packed into pinned staging (the device inputs Px, q, Ax, l, u
        // are contiguous in that order), one DMA queued after every launch that may still read
        // the inputs -- no host synchronisation
        IMPC_TRY(stage_ensure(b));
        IMPC_TRY(stage_wait(b));
        double *s = b->h_stage;
        const size_t len[5] = {(size_t)b->nnzP * B, (size_t)b->n * B, (size_t)b->nnzA * B, (size_t)b->m * B,
                               (size_t)b->m * B};
        const double *src[5] = {Px, q, Ax, l, u};
        for (int k = 0; k < 5; k++) {
            if (len[k]) std::memcpy(s, src[k], sizeof(double) * len[k]);
            s += len[k];
        }
        b->in_dirty = true;  // uploaded with the warm start by the next call that needs them (flush_staged)
        b->shared = false;
        b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;
        b->values_set = true;
        b->generic_dirty = true;
        return IMPC_OK;
    }
    IMPC_TRY(ctx_quiesce(b->ctx));  // no solve in flight on any stream reads the arrays replaced below
    IMPC_TRY(h2d_sync(b->ctx->stream, b->in_Px, Px, sizeof(double) * b->nnzP * B));
    IMPC_TRY(h2d_sync(b->ctx->stream, b->in_q, q, sizeof(double) * b->n * B));
    IMPC_TRY(h2d_sync(b->ctx->stream, b->in_Ax, Ax, sizeof(double) * b->nnzA * B));
    if (b->m) {
        IMPC_TRY(h2d_sync(b->ctx->stream, b->in_l, l, sizeof(double) * b->m * B));
        IMPC_TRY(h2d_sync(b->ctx->stream, b->in_u, u, sizeof(double) * b->m * B));
    }
    b->shared = false;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;  // new data: the next solve sets up from scratch
    b->values_set = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_set_values_shared(impc_batch b, const double *Px, const double *Ax, int64_t nvar,
                                 const int64_t *var_pos, const double *Ax_var, const double *q, const double *l,
                                 const double *u) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if ((b->nnzP && !Px) || !q || (b->nnzA && !Ax) || (b->m && (!l || !u)) || nvar < 0 || nvar > b->nnzA ||
        (nvar && (!var_pos || !Ax_var)))
        return fail(IMPC_INVALID_ARGUMENT, "null value array or bad nvar");
    std::vector<int32_t> vmap((size_t)std::max<int64_t>(b->nnzA, 1), -1);
    for (int64_t k = 0; k < nvar; k++) {
        if (var_pos[k] < 0 || var_pos[k] >= b->nnzA || (k && var_pos[k] <= var_pos[k - 1]))
            return fail(IMPC_DATA_VALIDATION_ERROR, "var_pos must be ascending positions in [0, nnzA)");
        vmap[(size_t)var_pos[k]] = (int32_t)k;
    }
    for (int64_t k = 0; k < b->m * b->B; k++)
        if (l[k] > u[k]) {
            char msg[160];
            std::snprintf(msg, sizeof msg, "lower bound greater than upper bound (QP %lld, row %lld)",
                          (long long)(k / b->m), (long long)(k % b->m));
            return fail(IMPC_DATA_VALIDATION_ERROR, msg);
        }
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    IMPC_TRY(ctx_quiesce(b->ctx));  // no solve in flight on any stream reads the arrays replaced below
    b->in_dirty = false;            // staged inputs of impc_batch_set_values are superseded
    if (!b->d_shPx) {
        HIP_OK(hipMalloc((void **)&b->d_shPx, sizeof(double) * std::max<int64_t>(b->nnzP, 1)));
        HIP_OK(hipMalloc((void **)&b->d_shAx, sizeof(double) * std::max<int64_t>(b->nnzA, 1)));
        HIP_OK(hipMalloc((void **)&b->d_vmap, sizeof(int32_t) * vmap.size()));
    }
    if (nvar > b->nvar_cap) {
        if (b->d_Axv) HIP_OK(hipFree(b->d_Axv));
        b->d_Axv = nullptr;
        HIP_OK(hipMalloc((void **)&b->d_Axv, sizeof(double) * (size_t)std::max<int64_t>(nvar, 1) * (size_t)b->B));
        b->nvar_cap = nvar;
    }
    const size_t B = (size_t)b->B;
    IMPC_TRY(h2d_sync(st, b->d_shPx, Px, sizeof(double) * b->nnzP));
    IMPC_TRY(h2d_sync(st, b->d_shAx, Ax, sizeof(double) * b->nnzA));
    IMPC_TRY(h2d_sync(st, b->d_vmap, vmap.data(), sizeof(int32_t) * vmap.size()));
    IMPC_TRY(h2d_sync(st, b->d_Axv, Ax_var, sizeof(double) * (size_t)nvar * B));
    IMPC_TRY(h2d_sync(st, b->in_q, q, sizeof(double) * b->n * B));
    if (b->m) {
        IMPC_TRY(h2d_sync(st, b->in_l, l, sizeof(double) * b->m * B));
        IMPC_TRY(h2d_sync(st, b->in_u, u, sizeof(double) * b->m * B));
    }
    b->nvar = nvar;
    b->shared = true;
    b->shared_expanded = false;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;
    b->values_set = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_set_values_device(impc_batch b, const double *Px, const double *q, const double *Ax, const double *l,
                                 const double *u) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if ((b->nnzP && !Px) || !q || (b->nnzA && !Ax) || (b->m && (!l || !u)))
        return fail(IMPC_INVALID_ARGUMENT, "null value array");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));  // the copies below are ordered on the context stream only
    b->in_dirty = false;            // staged inputs of impc_batch_set_values are superseded
    hipStream_t st = b->ctx->stream;
    const size_t B = (size_t)b->B;
    if (b->nnzP) HIP_OK(hipMemcpyAsync(b->in_Px, Px, sizeof(double) * b->nnzP * B, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemcpyAsync(b->in_q, q, sizeof(double) * b->n * B, hipMemcpyDeviceToDevice, st));
    if (b->nnzA) HIP_OK(hipMemcpyAsync(b->in_Ax, Ax, sizeof(double) * b->nnzA * B, hipMemcpyDeviceToDevice, st));
    if (b->m) {
        HIP_OK(hipMemcpyAsync(b->in_l, l, sizeof(double) * b->m * B, hipMemcpyDeviceToDevice, st));
        HIP_OK(hipMemcpyAsync(b->in_u, u, sizeof(double) * b->m * B, hipMemcpyDeviceToDevice, st));
    }
    b->shared = false;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;  // new data: the next solve sets up from scratch
    b->values_set = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_warm_start(impc_batch b, const double *x, const double *y) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (!x) {
        b->has_ws = false;
        b->generic_dirty = true;
        return IMPC_OK;
    }
    const size_t B = (size_t)b->B;
    if (stage_ok(b)) {  // x (and y) through the pinned staging, stream-ordered, one DMA
        IMPC_TRY(stage_ensure(b));
        IMPC_TRY(stage_wait(b));
        double *s = stage_xws(b);
        std::memcpy(s, x, sizeof(double) * b->n * B);
        if (b->m && y) std::memcpy(s + (size_t)b->n * B, y, sizeof(double) * b->m * B);  // in_yws follows in_xws
        b->ws_len = (size_t)b->n * B + (b->m && y ? (size_t)b->m * B : 0);
        b->ws_dirty = true;  // uploaded by the next call that needs it (flush_staged)
    } else {
        IMPC_TRY(ctx_quiesce(b->ctx));  // no solve in flight on any stream reads the arrays replaced below
        IMPC_TRY(h2d_sync(b->ctx->stream, b->in_xws, x, sizeof(double) * b->n * B));
        // y = 0 (the solveTraj warm start, mpcPlanner.cpp:480-497): nothing is uploaded, the
        // structured kernel reads no duals (WaveIO::has_ws == 2) and the generic path zero-fills
        if (b->m && y) IMPC_TRY(h2d_sync(b->ctx->stream, b->in_yws, y, sizeof(double) * b->m * B));
    }
    b->ws_y = y != nullptr;
    // osqp_warm_start turns the warm_start setting on (osqp.c, oracle ora_warm_start)
    b->settings.warm_start = 1;
    b->dst.warm_start = 1;
    if (!use_structured(b) && b->generic_setup_done && !b->generic_dirty) {
        // a set-up generic workspace takes the warm start in place, keeping scaling, rho and factor
        IMPC_TRY(flush_staged(b));
        hipStream_t st = b->ctx->stream;
        int rc = interleave(b, b->in_xws, const_cast<double *>(b->dwk.xws), b->n, st);
        if (!rc && !b->ws_y && b->m) rc = fill0_sync(st, b->in_yws, sizeof(double) * b->m * b->B);
        if (!rc) rc = interleave(b, b->in_yws, const_cast<double *>(b->dwk.yws), b->m, st);
        if (rc) return rc;
        hipLaunchKernelGGL(k_warm_start, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk,
                           b->dst, b->Bact);
        HIP_OK(hipGetLastError());
        return IMPC_OK;
    }
    b->has_ws = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_set_values_async(impc_batch b, const double *Ax_var, const double *q, const double *l, const double *u,
                                const double *x_ws, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!b->shared || !b->d_Axv) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "impc_batch_set_values_shared first");
    if (!q || (b->m && (!l || !u)) || (b->nvar && !Ax_var)) return fail(IMPC_INVALID_ARGUMENT, "null value array");
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->ctx->stream;
    const size_t B = (size_t)b->B;
    auto h2d = [&](double *dst, const double *src, size_t len) -> hipError_t {
        return len ? hipMemcpyAsync(dst, src, sizeof(double) * len, hipMemcpyHostToDevice, st) : hipSuccess;
    };
    // staged uploads these copies supersede are dropped (a DMA of them on the context stream would
    // not be ordered with this stream's copies)
    b->in_dirty = false;
    if (x_ws) b->ws_dirty = false;
    HIP_OK(h2d(b->d_Axv, Ax_var, (size_t)b->nvar * B));
    HIP_OK(h2d(b->in_q, q, (size_t)b->n * B));
    HIP_OK(h2d(b->in_l, l, (size_t)b->m * B));
    HIP_OK(h2d(b->in_u, u, (size_t)b->m * B));
    if (x_ws) HIP_OK(h2d(b->in_xws, x_ws, (size_t)b->n * B));
    b->has_ws = x_ws != nullptr;
    b->ws_y = false;
    if (x_ws) b->settings.warm_start = b->dst.warm_start = 1;
    b->shared_expanded = false;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;
    b->values_set = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_get_async(impc_batch b, double *x, double *y, impc_info *info, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->ctx->stream;
    const size_t B = (size_t)b->B;
    if (x) HIP_OK(hipMemcpyAsync(x, b->d_xout, sizeof(double) * b->n * B, hipMemcpyDeviceToHost, st));
    if (y && b->m) HIP_OK(hipMemcpyAsync(y, b->d_yout, sizeof(double) * b->m * B, hipMemcpyDeviceToHost, st));
    if (info) HIP_OK(hipMemcpyAsync(info, b->d_info, sizeof(impc_info) * B, hipMemcpyDeviceToHost, st));
    return IMPC_OK;
}

int impc_batch_warm_start_device(impc_batch b, const double *x, const double *y) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (!x) return impc_batch_warm_start(b, nullptr, nullptr);
    hipStream_t st = b->ctx->stream;
    // queued after every launch on every stream this context has used: none of them still reads
    // the warm-start arrays when the copies land
    IMPC_TRY(ctx_order_after_all(b->ctx, st));
    b->ws_dirty = false;  // a staged host warm start is superseded
    const size_t B = (size_t)b->B;
    HIP_OK(hipMemcpyAsync(b->in_xws, x, sizeof(double) * b->n * B, hipMemcpyDeviceToDevice, st));
    if (b->m && y) HIP_OK(hipMemcpyAsync(b->in_yws, y, sizeof(double) * b->m * B, hipMemcpyDeviceToDevice, st));
    b->ws_y = y != nullptr;
    b->settings.warm_start = 1;  // as impc_batch_warm_start (osqp_warm_start)
    b->dst.warm_start = 1;
    if (!use_structured(b) && b->generic_setup_done && !b->generic_dirty) {
        int rc = interleave(b, b->in_xws, const_cast<double *>(b->dwk.xws), b->n, st);
        if (!rc && !b->ws_y && b->m) HIP_OK(hipMemsetAsync(b->in_yws, 0, sizeof(double) * b->m * B, st));
        if (!rc) rc = interleave(b, b->in_yws, const_cast<double *>(b->dwk.yws), b->m, st);
        if (rc) return rc;
        hipLaunchKernelGGL(k_warm_start, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk,
                           b->dst, b->Bact);
        HIP_OK(hipGetLastError());
        return IMPC_OK;
    }
    b->has_ws = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_set_active(impc_batch b, int64_t count) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (count < 1 || count > b->B) return fail(IMPC_INVALID_ARGUMENT, "active count must be in [1, B]");
    b->d_active = nullptr;
    if (count != b->Bact) {
        b->Bact = count;
        b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;  // the stored workspaces cover other QPs
        b->generic_dirty = true;
    }
    return IMPC_OK;
}

int impc_batch_setup(impc_batch b, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!b->values_set) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "values not set");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (use_structured(b)) return IMPC_OK;  // the wave kernel runs setup and solve per QP in one launch
    IMPC_TRY(flush_staged(b));
    hipStream_t st = pick(b, stream);
    IMPC_TRY(ctx_order_launch(b->ctx, st));
    IMPC_TRY(generic_setup(b, st));
    return ctx_note_launch(b->ctx, st);
}

int impc_batch_solve(impc_batch b, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!b->values_set) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "values not set");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(flush_staged(b));
    hipStream_t st = pick(b, stream);
    IMPC_TRY(ctx_order_launch(b->ctx, st));
    IMPC_TRY(use_structured(b) ? structured_solve(b, st) : generic_solve(b, st));
    return ctx_note_launch(b->ctx, st);
}

int impc_batch_solve_group(impc_batch *bs, int count, void *stream) {
    if (!bs || count < 1) return fail(IMPC_INVALID_ARGUMENT, "empty group");
    impc_batch b0 = bs[0];
    if (!b0) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    impc_ctx ctx = b0->ctx;
    for (int k = 0; k < count; k++) {
        impc_batch b = bs[k];
        if (!b || b->ctx != ctx) return fail(IMPC_INVALID_ARGUMENT, "group batches must share a context");
        if (!b->values_set) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "values not set");
        if (!use_structured(b)) return fail(IMPC_UNSUPPORTED, "grouped solves need structured batches");
    }
    for (int k = 0; k < count; k++) IMPC_TRY(flush_staged(bs[k]));
    // One persistent launch per kernel class (team shape VS, general-row slots per lane GS, products
    // tiers): a bucket never runs in a wider instance than it needs (more registers, spills) and each
    // launch's LDS is sized by its own batches, so mixed obstacle counts (config 4, K = 0..21) keep
    // the narrow kernels for most buckets.  Classes run back to back on the stream, entries contiguous.
    std::vector<int> order((size_t)count);
    for (int k = 0; k < count; k++) order[(size_t)k] = k;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
        if (bs[x]->vs != bs[y]->vs) return bs[x]->vs > bs[y]->vs;  // wavefront shape first
        return bs[x]->gs != bs[y]->gs ? bs[x]->gs < bs[y]->gs : (int)bs[x]->tier < (int)bs[y]->tier;
    });
    struct Launch {
        int vs, gs;
        bool tier;
        int first, count;
        int64_t total;
        size_t lds;
        int spec;  // the launch's compile-time horizon (-1: no batch yet; 0: runtime W)
        unsigned *counter;
        bool devcnt;  // some batch's active count is in device memory
    };
    std::vector<Launch> launches;
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    std::vector<GroupEntry> entries((size_t)count);
    std::memset((void *)entries.data(), 0, sizeof(GroupEntry) * (size_t)count);  // comparable bytes
    for (int p = 0; p < count; p++) {
        impc_batch b = bs[order[(size_t)p]];
        if (launches.empty() || launches.back().vs != b->vs || launches.back().gs != b->gs ||
            launches.back().tier != b->tier)
            launches.push_back(Launch{b->vs, b->gs, b->tier, p, 0, 0, 0, -1, b->d_counter, false});
        Launch &L = launches.back();
        L.count++;
        L.lds = std::max(L.lds, wave_lds_bytes(b->vs, b->gs, b->wt));
        L.spec = L.spec < 0 ? spec_w(b) : (L.spec == spec_w(b) ? L.spec : 0);
        GroupEntry &e = entries[(size_t)p];
        e.T = b->wt;
        e.io = wave_io(b);
        e.st = b->dst;
        e.first = L.total;
        e.dcount = b->d_active;
        L.devcnt = L.devcnt || b->d_active != nullptr;
        L.total += b->Bact;
        b->ev_solve = false;
        b->ev_setup = false;
    }
    for (const Launch &L : launches)
        if (L.lds > 160 * 1024 - 1024) return fail(IMPC_UNSUPPORTED, "grouped batches exceed the LDS of a CU");
    // the entry table: a cached device copy of these very entries (repeated solves of one group,
    // or of the few groups a pipeline alternates between), else a fresh table -- uploaded on the
    // launch stream; replacing a cached table that a launch in flight may read waits for every
    // launch on every stream this context has used
    constexpr size_t kGroupTables = 8;
    const size_t ebytes = sizeof(GroupEntry) * (size_t)count;
    impc_ctx_s::GroupTable *tab = nullptr;
    for (auto &g : ctx->groups)
        if (g.h.size() == entries.size() && std::memcmp(g.h.data(), entries.data(), ebytes) == 0) tab = &g;
    IMPC_TRY(ctx_order_launch(ctx, st));
    if (!tab) {
        if (ctx->groups.size() < kGroupTables) {
            ctx->groups.emplace_back();
            tab = &ctx->groups.back();
        } else {
            IMPC_TRY(ctx_quiesce(ctx));
            tab = &*std::min_element(ctx->groups.begin(), ctx->groups.end(),
                                     [](const impc_ctx_s::GroupTable &a, const impc_ctx_s::GroupTable &c) {
                                         return a.used < c.used;
                                     });
        }
        if (count > tab->cap) {
            if (tab->d) HIP_OK(hipFree(tab->d));
            tab->d = nullptr;
            HIP_OK(hipMalloc((void **)&tab->d, ebytes));
            tab->cap = count;
        }
        tab->h = entries;  // the host copy stays alive: the stream-ordered upload reads it
        HIP_OK(hipMemcpyAsync(tab->d, tab->h.data(), ebytes, hipMemcpyHostToDevice, st));
    }
    tab->used = ++ctx->group_clock;
    if (b0->profile) HIP_OK(hipEventRecord(b0->ev[2], st));
    for (const Launch &L : launches) {
        if (L.total == 0) continue;
        HIP_OK(hipMemsetAsync(L.counter, 0, 256, st));
        const GroupEntry *E = tab->d + L.first;
        std::vector<impc_batch> lb((size_t)L.count);
        std::vector<int64_t> lf((size_t)L.count);
        for (int k = 0; k < L.count; k++) {
            lb[(size_t)k] = bs[order[(size_t)(L.first + k)]];
            lf[(size_t)k] = entries[(size_t)(L.first + k)].first;
        }
        const uint32_t *ord = nullptr;
        IMPC_TRY(queue_order(lb.data(), lf.data(), L.count, L.total, st, &ord));
        const int rc = with_shape(L.vs, L.gs, L.tier, [&](auto vs, auto gs, auto tr) {
            return launch_group<decltype(vs)::value, decltype(gs)::value, decltype(tr)::value>(
                ctx, st, E, L.count, L.total, L.lds, L.counter, L.spec, ord, L.devcnt ? 1 : 0);
        });
        if (rc) return rc;
    }
    IMPC_TRY(ctx_note_launch(ctx, st));
    for (int k = 0; k < count; k++) structured_solved(bs[k]);
    if (b0->profile) {
        HIP_OK(hipEventRecord(b0->ev[3], st));
        HIP_OK(hipEventRecord(b0->ev[4], st));
        b0->ev_solve = true;
    }
    return IMPC_OK;
}

int impc_batch_get(impc_batch b, double *x, double *y, impc_info *info) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (stage_ok(b)) {  // results through the pinned staging: three DMAs, one synchronisation
        IMPC_TRY(stage_ensure(b));
        hipStream_t st = b->ctx->stream;
        IMPC_TRY(ctx_order_after_all(b->ctx, st));  // after the solves, on whichever stream
        double *sx = stage_xout(b), *sy = sx + (size_t)b->B * b->n;
        impc_info *si = (impc_info *)(sy + (size_t)b->B * b->m);
        const size_t B = (size_t)b->B;
        if (x && y && info && b->m) {  // the device regions [x][y][info] are contiguous as in the staging
            HIP_OK(hipMemcpyAsync(sx, b->d_xout, sizeof(double) * (b->n + b->m) * B + sizeof(impc_info) * B,
                                  hipMemcpyDeviceToHost, st));
        } else {
            if (x) HIP_OK(hipMemcpyAsync(sx, b->d_xout, sizeof(double) * b->n * B, hipMemcpyDeviceToHost, st));
            if (y && b->m) HIP_OK(hipMemcpyAsync(sy, b->d_yout, sizeof(double) * b->m * B, hipMemcpyDeviceToHost, st));
            if (info) HIP_OK(hipMemcpyAsync(si, b->d_info, sizeof(impc_info) * B, hipMemcpyDeviceToHost, st));
        }
        IMPC_TRY(ctx_quiesce(b->ctx));
        if (x) std::memcpy(x, sx, sizeof(double) * b->n * B);
        if (y && b->m) std::memcpy(y, sy, sizeof(double) * b->m * B);
        if (info) std::memcpy(info, si, sizeof(impc_info) * B);
        return IMPC_OK;
    }
    HIP_OK(hipStreamSynchronize(b->ctx->stream));
    HIP_OK(hipDeviceSynchronize());
    if (x) HIP_OK(hipMemcpy(x, b->d_xout, sizeof(double) * b->n * b->B, hipMemcpyDeviceToHost));
    if (y && b->m) HIP_OK(hipMemcpy(y, b->d_yout, sizeof(double) * b->m * b->B, hipMemcpyDeviceToHost));
    if (info) HIP_OK(hipMemcpy(info, b->d_info, sizeof(impc_info) * b->B, hipMemcpyDeviceToHost));
    return IMPC_OK;
}

int impc_batch_device_results(impc_batch b, double **x, double **y, impc_info **info) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (x) *x = b->d_xout;
    if (y) *y = b->d_yout;
    if (info) *info = b->d_info;
    return IMPC_OK;
}

static int upload_interleaved(impc_batch b, const double *host, double *qp_major, double *dst, int64_t len) {
    IMPC_TRY(h2d_sync(b->ctx->stream, qp_major, host, sizeof(double) * len * b->B));
    int rc = interleave(b, qp_major, dst, len, b->ctx->stream);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(b->ctx->stream));
    return IMPC_OK;
}

int impc_batch_update_lin_cost(impc_batch b, const double *q) {
    if (!b || !q) return fail(IMPC_INVALID_ARGUMENT, "null batch or q");
    IMPC_TRY(flush_staged(b));  // the staged values go first, the update overwrites q after them
    if (use_structured(b)) {  // the next structured solve resumes the workspace with this q
        if (!b->persist_on || !b->persist_valid)
            return fail(IMPC_WORKSPACE_NOT_INIT_ERROR,
                        "structured kernel: impc_batch_set_persistent(b, 1) and one solve before updates");
        HIP_OK(hipSetDevice(b->ctx->device));
        IMPC_TRY(ctx_quiesce(b->ctx));
        IMPC_TRY(h2d_sync(b->ctx->stream, b->in_q, q, sizeof(double) * b->n * b->B));
        b->q_by_update = true;
        b->q_after = b->rescale;
        b->generic_dirty = true;
        return IMPC_OK;
    }
    if (!b->generic_setup_done || b->generic_dirty)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "setup has not run on current data");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));
    int rc = upload_interleaved(b, q, b->in_q, const_cast<double *>(b->dwk.q), b->n);
    if (rc) return rc;
    hipLaunchKernelGGL(k_update_q, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, b->ctx->stream, b->dsym, b->dwk,
                       b->dst, b->Bact);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int impc_batch_update_bounds(impc_batch b, const double *l, const double *u) {
    if (!b || (b->m && (!l || !u))) return fail(IMPC_INVALID_ARGUMENT, "null batch or bounds");
    IMPC_TRY(flush_staged(b));
    if (use_structured(b)) {  // the next structured solve resumes the workspace with these bounds
        if (!b->persist_on || !b->persist_valid)
            return fail(IMPC_WORKSPACE_NOT_INIT_ERROR,
                        "structured kernel: impc_batch_set_persistent(b, 1) and one solve before updates");
        for (int64_t k = 0; k < b->m * b->B; k++)
            if (l[k] > u[k]) return fail(IMPC_DATA_VALIDATION_ERROR, "lower bound greater than upper bound");
        HIP_OK(hipSetDevice(b->ctx->device));
        IMPC_TRY(ctx_quiesce(b->ctx));
        if (b->m) {
            IMPC_TRY(h2d_sync(b->ctx->stream, b->in_l, l, sizeof(double) * b->m * b->B));
            IMPC_TRY(h2d_sync(b->ctx->stream, b->in_u, u, sizeof(double) * b->m * b->B));
        }
        b->generic_dirty = true;
        return IMPC_OK;
    }
    if (!b->generic_setup_done || b->generic_dirty)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "setup has not run on current data");
    for (int64_t k = 0; k < b->m * b->B; k++)
        if (l[k] > u[k]) return fail(IMPC_DATA_VALIDATION_ERROR, "lower bound greater than upper bound");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));
    int rc = upload_interleaved(b, l, b->in_l, const_cast<double *>(b->dwk.l), b->m);
    if (!rc) rc = upload_interleaved(b, u, b->in_u, const_cast<double *>(b->dwk.u), b->m);
    if (rc) return rc;
    hipLaunchKernelGGL(k_update_bounds, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, b->ctx->stream, b->dsym,
                       b->dwk, b->dst, b->Bact);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int impc_batch_update_lin_cost_device(impc_batch b, const double *q) {
    if (!b || !q) return fail(IMPC_INVALID_ARGUMENT, "null batch or q");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(flush_staged(b));
    hipStream_t st = b->ctx->stream;
    const size_t bytes = sizeof(double) * (size_t)(b->n * b->B);
    if (use_structured(b)) {
        if (!b->persist_on || !b->persist_valid)
            return fail(IMPC_WORKSPACE_NOT_INIT_ERROR,
                        "structured kernel: impc_batch_set_persistent(b, 1) and one solve before updates");
        IMPC_TRY(ctx_order_after_all(b->ctx, st));
        HIP_OK(hipMemcpyAsync(b->in_q, q, bytes, hipMemcpyDeviceToDevice, st));
        b->q_by_update = true;
        b->q_after = b->rescale;
        b->generic_dirty = true;
        return IMPC_OK;
    }
    if (!b->generic_setup_done || b->generic_dirty)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "setup has not run on current data");
    IMPC_TRY(ctx_order_after_all(b->ctx, st));
    HIP_OK(hipMemcpyAsync(b->in_q, q, bytes, hipMemcpyDeviceToDevice, st));
    IMPC_TRY(interleave(b, b->in_q, const_cast<double *>(b->dwk.q), b->n, st));
    hipLaunchKernelGGL(k_update_q, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk, b->dst, b->Bact);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int impc_batch_update_bounds_device(impc_batch b, const double *l, const double *u) {
    if (!b || (b->m && (!l || !u))) return fail(IMPC_INVALID_ARGUMENT, "null batch or bounds");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(flush_staged(b));
    hipStream_t st = b->ctx->stream;
    const size_t bytes = sizeof(double) * (size_t)(b->m * b->B);
    if (use_structured(b)) {
        if (!b->persist_on || !b->persist_valid)
            return fail(IMPC_WORKSPACE_NOT_INIT_ERROR,
                        "structured kernel: impc_batch_set_persistent(b, 1) and one solve before updates");
        IMPC_TRY(ctx_order_after_all(b->ctx, st));
        if (bytes) {
            HIP_OK(hipMemcpyAsync(b->in_l, l, bytes, hipMemcpyDeviceToDevice, st));
            HIP_OK(hipMemcpyAsync(b->in_u, u, bytes, hipMemcpyDeviceToDevice, st));
        }
        b->generic_dirty = true;
        return IMPC_OK;
    }
    if (!b->generic_setup_done || b->generic_dirty)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "setup has not run on current data");
    IMPC_TRY(ctx_order_after_all(b->ctx, st));
    if (bytes) {
        HIP_OK(hipMemcpyAsync(b->in_l, l, bytes, hipMemcpyDeviceToDevice, st));
        HIP_OK(hipMemcpyAsync(b->in_u, u, bytes, hipMemcpyDeviceToDevice, st));
    }
    IMPC_TRY(interleave(b, b->in_l, const_cast<double *>(b->dwk.l), b->m, st));
    IMPC_TRY(interleave(b, b->in_u, const_cast<double *>(b->dwk.u), b->m, st));
    hipLaunchKernelGGL(k_update_bounds, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk, b->dst,
                       b->Bact);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

// The q of the workspace at a matrix update (OSQP's scale_data normalises the cost with it; a later
// matrix update rescales again with the q current then): kept for the next solve in case q is
// updated before it (impc_batch_update_lin_cost after the matrices)
static int snapshot_q(impc_batch b, hipStream_t st) {
    if (!b->d_qsnap) {
        HIP_OK(hipMalloc((void **)&b->d_qsnap, sizeof(double) * (size_t)(b->n * b->B)));
        b->device_bytes += (int64_t)sizeof(double) * b->n * b->B;
    }
    HIP_OK(hipMemcpyAsync(b->d_qsnap, b->in_q, sizeof(double) * (size_t)(b->n * b->B), hipMemcpyDeviceToDevice, st));
    b->q_after = false;
    return IMPC_OK;
}

int impc_batch_update_matrices(impc_batch b, const double *Px, const double *Ax) {
    if (!b || (!Px && !Ax)) return fail(IMPC_INVALID_ARGUMENT, "null batch, or neither P nor A values");
    IMPC_TRY(flush_staged(b));
    if (!use_structured(b))
        return fail(IMPC_UNSUPPORTED, "generic kernel: no in-place matrix update (impc_batch_set_values + warm start)");
    if (!b->persist_on || !b->persist_valid)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR,
                    "structured kernel: impc_batch_set_persistent(b, 1) and one solve before updates");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));  // no launch in flight reads the arrays replaced below
    hipStream_t st = b->ctx->stream;
    if (b->shared) {  // the kept half of the values into the per-QP arrays first
        const int64_t tot = b->B * (b->nnzP + b->nnzA);
        const int64_t blocks = std::min<int64_t>((tot + 255) / 256, (int64_t)b->ctx->num_cu * 16);
        hipLaunchKernelGGL(k_expand_shared, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, b->d_shPx,
                           b->d_shAx, b->d_vmap, b->d_Axv, b->nvar, b->nnzP, b->nnzA, b->B, b->in_Px, b->in_Ax);
        HIP_OK(hipGetLastError());
        b->shared = false;
    }
    if (Px && b->nnzP) IMPC_TRY(h2d_sync(st, b->in_Px, Px, sizeof(double) * b->nnzP * b->B));
    if (Ax && b->nnzA) IMPC_TRY(h2d_sync(st, b->in_Ax, Ax, sizeof(double) * b->nnzA * b->B));
    IMPC_TRY(snapshot_q(b, st));
    b->rescale = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_update_matrices_device(impc_batch b, const double *Px, const double *Ax) {
    if (!b || (!Px && !Ax)) return fail(IMPC_INVALID_ARGUMENT, "null batch, or neither P nor A values");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(flush_staged(b));
    if (!use_structured(b))
        return fail(IMPC_UNSUPPORTED, "generic kernel: no in-place matrix update (impc_batch_set_values + warm start)");
    if (!b->persist_on || !b->persist_valid)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR,
                    "structured kernel: impc_batch_set_persistent(b, 1) and one solve before updates");
    hipStream_t st = b->ctx->stream;
    IMPC_TRY(ctx_order_after_all(b->ctx, st));  // after every launch that may still read the values
    if (b->shared) {
        const int64_t tot = b->B * (b->nnzP + b->nnzA);
        const int64_t blocks = std::min<int64_t>((tot + 255) / 256, (int64_t)b->ctx->num_cu * 16);
        hipLaunchKernelGGL(k_expand_shared, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, b->d_shPx,
                           b->d_shAx, b->d_vmap, b->d_Axv, b->nvar, b->nnzP, b->nnzA, b->B, b->in_Px, b->in_Ax);
        HIP_OK(hipGetLastError());
        b->shared = false;
    }
    if (Px && b->nnzP)
        HIP_OK(hipMemcpyAsync(b->in_Px, Px, sizeof(double) * b->nnzP * b->B, hipMemcpyDeviceToDevice, st));
    if (Ax && b->nnzA)
        HIP_OK(hipMemcpyAsync(b->in_Ax, Ax, sizeof(double) * b->nnzA * b->B, hipMemcpyDeviceToDevice, st));
    IMPC_TRY(snapshot_q(b, st));
    b->rescale = true;
    b->generic_dirty = true;
    return IMPC_OK;
}

int impc_batch_get_stats(impc_batch b, impc_batch_stats *out) {
    if (!b || !out) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    std::memset(out, 0, sizeof(*out));
    out->n = b->n;
    out->m = b->m;
    out->nnzP = b->nnzP;
    out->nnzA = b->nnzA;
    out->batch = b->B;
    out->batch_stride = b->S;
    if (b->sym) {
        out->nnzL = b->sym->nnzL;
        out->nnzLcol = b->sym->nnzL;
        out->n_terms = (int64_t)b->sym->At_dest.size();
        out->bandwidth = b->sym->max_row_L;
    }
    out->device_bytes = b->device_bytes;
    out->kernel = use_structured(b) ? IMPC_KERNEL_STRUCTURED : IMPC_KERNEL_GENERIC;
    out->structured_ok = b->structured_ok ? 1 : 0;
    if (b->structured_ok) {
        out->team_lanes = b->vs == kWaveVSFront ? Shape<kWaveVSFront>::NL : Shape<kWaveVS>::NL;
        out->var_slots = b->vs;
        out->row_slots = b->gs;
    }
    return IMPC_OK;
}

int impc_batch_set_profiling(impc_batch b, int on) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (on && !b->ev[0])
        for (hipEvent_t &e : b->ev) HIP_OK(hipEventCreate(&e));
    if (on && !b->d_qpt) HIP_OK(hipMalloc((void **)&b->d_qpt, sizeof(unsigned long long) * 2 * (size_t)b->B));
    b->profile = on != 0;
    return IMPC_OK;
}

int impc_batch_set_persistent(impc_batch b, int on) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (on && !b->structured_ok) return fail(IMPC_UNSUPPORTED, "persistent workspaces are a structured-kernel mode");
    if (on && b->settings.scaling > impc::kPersistMaxScaling)
        return fail(IMPC_UNSUPPORTED, "persistent workspaces support scaling <= 20 Ruiz passes");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (on && !b->d_persist) {
        const size_t bytes = sizeof(double) * (size_t)b->B * (size_t)impc::persist_stride((int)b->n, b->ms->mg);
        if (hipMalloc((void **)&b->d_persist, bytes) != hipSuccess) {
            b->d_persist = nullptr;
            return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(persistent workspace) failed");
        }
        b->device_bytes += (int64_t)bytes;
        // defined contents before any solve writes them (rho and iterates of a fresh workspace are
        // written by the first solve, including one whose factorisation fails)
        HIP_OK(hipMemsetAsync(b->d_persist, 0, bytes, b->ctx->stream));
    }
    b->persist_on = on != 0;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;  // the next solve sets up from scratch
    return IMPC_OK;
}

int impc_batch_get_persistent(impc_batch b, double *rho, double *x, double *z, double *y) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!b->persist_on || !b->persist_valid || !b->d_persist)
        return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "no persistent workspace solved yet (impc_batch_set_persistent + solve)");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));
    const impc::MpcStructure &ms = *b->ms;
    const int64_t n = b->n, m = b->m, mg = ms.mg, stride = impc::persist_stride((int)n, (int)mg);
    std::vector<double> h((size_t)(b->B * stride));
    HIP_OK(hipMemcpy(h.data(), b->d_persist, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
    // the kernel's layout (mpc_wave.hpp WaveIO::persist): [hdr | x, z_box, y_box (stage order) |
    // z_gen, y_gen (general-row order)] -> OSQP's variable and row order
    for (int64_t k = 0; k < b->B; k++) {
        const double *p = h.data() + k * stride, *it = p + impc::kPersistHdr;
        if (rho) rho[k] = p[impc::kPersistHdr - 1];
        for (int64_t v = 0; v < n; v++) {
            if (x) x[k * n + ms.var_orig[v]] = it[v];
            if (z) z[k * m + ms.var_boxrow[v]] = it[n + v];
            if (y) y[k * m + ms.var_boxrow[v]] = it[2 * n + v];
        }
        for (int64_t g = 0; g < mg; g++) {
            if (z) z[k * m + ms.gen_row[g]] = it[3 * n + g];
            if (y) y[k * m + ms.gen_row[g]] = it[3 * n + mg + g];
        }
    }
    return IMPC_OK;
}

int impc_batch_get_qp_latency(impc_batch b, double *ms) {
    if (!b || !ms) return fail(IMPC_INVALID_ARGUMENT, "null batch or output");
    if (!b->qpt_valid) return fail(IMPC_INVALID_ARGUMENT, "no profiled structured-kernel solve");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));
    std::vector<unsigned long long> t((size_t)b->B * 2);
    HIP_OK(hipMemcpy(t.data(), b->d_qpt, sizeof(unsigned long long) * t.size(), hipMemcpyDeviceToHost));
    const double tick_ms = b->ctx->tick_s * 1e3;
    for (int64_t k = 0; k < b->B; k++) ms[k] = (double)(t[2 * k + 1] - t[2 * k]) * tick_ms;
    return IMPC_OK;
}

int impc_batch_set_time_limits(impc_batch b, const double *time_limit) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!time_limit) {
        b->tlim_on = false;
        return IMPC_OK;
    }
    for (int64_t k = 0; k < b->B; k++)
        if (!(time_limit[k] >= 0.0)) return fail(IMPC_SETTINGS_VALIDATION_ERROR, "time limits must be >= 0");
    HIP_OK(hipSetDevice(b->ctx->device));
    IMPC_TRY(ctx_quiesce(b->ctx));  // no launch in flight reads the array being replaced
    if (!b->d_tlim) {
        HIP_OK(hipMalloc((void **)&b->d_tlim, sizeof(double) * (size_t)b->B));
        b->device_bytes += (int64_t)sizeof(double) * b->B;
    }
    IMPC_TRY(h2d_sync(b->ctx->stream, b->d_tlim, time_limit, sizeof(double) * (size_t)b->B));
    b->tlim_on = true;
    return IMPC_OK;
}

int impc_batch_set_queue_order(impc_batch b, int mode, double q_weight) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (mode != IMPC_QUEUE_FIFO && mode != IMPC_QUEUE_LONGEST_FIRST)
        return fail(IMPC_INVALID_ARGUMENT, "unknown queue order");
    if (!(q_weight >= 0.0 && q_weight < 1e300)) return fail(IMPC_INVALID_ARGUMENT, "q_weight must be finite, >= 0");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (mode == IMPC_QUEUE_LONGEST_FIRST) IMPC_TRY(build_queue_csr(b));
    b->queue_mode = mode;
    b->queue_qw = q_weight;
    return IMPC_OK;
}

int impc_ctx_clock_rate(impc_ctx ctx, double *hz) {
    if (!ctx || !hz) return fail(IMPC_INVALID_ARGUMENT, "null context or output");
    *hz = 1.0 / ctx->tick_s;
    return IMPC_OK;
}

int impc_ctx_clock_check(impc_ctx ctx, double seconds, double *event_seconds) {
    if (!ctx || !event_seconds) return fail(IMPC_INVALID_ARGUMENT, "null context or output");
    if (!(seconds > 0.0 && seconds <= 10.0)) return fail(IMPC_INVALID_ARGUMENT, "seconds must be in (0, 10]");
    HIP_OK(hipSetDevice(ctx->device));
    IMPC_TRY(ctx_quiesce(ctx));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    const uint64_t ticks = (uint64_t)(seconds / ctx->tick_s + 0.5);
    hipError_t err = hipEventRecord(e0, ctx->stream);
    if (err == hipSuccess) {
        hipLaunchKernelGGL(k_clock_spin, dim3(1), dim3(64), 0, ctx->stream, ticks);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipEventRecord(e1, ctx->stream);
    if (err == hipSuccess) err = hipEventSynchronize(e1);
    float ms = 0.f;
    if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (err != hipSuccess) return fail(IMPC_DEVICE_ERROR, std::string("clock check: ") + hipGetErrorString(err));
    *event_seconds = 1e-3 * (double)ms;
    return IMPC_OK;
}

int impc_batch_get_timings(impc_batch b, double *setup_ms, double *solve_ms, double *output_ms) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!b->profile) return fail(IMPC_INVALID_ARGUMENT, "profiling is off");
    float t = 0.f;
    if (setup_ms) {
        *setup_ms = 0.0;
        if (b->ev_setup) {
            HIP_OK(hipEventSynchronize(b->ev[1]));
            HIP_OK(hipEventElapsedTime(&t, b->ev[0], b->ev[1]));
            *setup_ms = t;
        }
    }
    if (b->ev_solve) HIP_OK(hipEventSynchronize(b->ev[4]));
    if (solve_ms) {
        *solve_ms = 0.0;
        if (b->ev_solve) {
            HIP_OK(hipEventElapsedTime(&t, b->ev[2], b->ev[3]));
            *solve_ms = t;
        }
    }
    if (output_ms) {
        *output_ms = 0.0;
        if (b->ev_solve) {
            HIP_OK(hipEventElapsedTime(&t, b->ev[3], b->ev[4]));
            *output_ms = t;
        }
    }
    return IMPC_OK;
}

#ifdef IMPC_SECTION_PROF
// Profiling build only (not part of include/impc_qp.h): cycle sums per section since the first
// structured solve of this batch (enum kSec* in mpc_wave.hpp), then resets them.
extern "C" int impc_debug_sections(impc_batch b, unsigned long long *out) {
    if (!b || !out) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    for (int i = 0; i < impc::kSecCount; i++) out[i] = 0;
    if (!b->d_sec) return IMPC_OK;
    HIP_OK(hipStreamSynchronize(b->ctx->stream));
    HIP_OK(hipMemcpy(out, b->d_sec, sizeof(unsigned long long) * impc::kSecCount, hipMemcpyDeviceToHost));
    IMPC_TRY(fill0_sync(b->ctx->stream, b->d_sec, sizeof(unsigned long long) * impc::kSecCount));
    return IMPC_OK;
}
#endif

int impc_batch_get_perm(impc_batch b, int64_t *perm) {
    if (!b || !perm) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    int rc = ensure_generic(b);
    if (rc) return rc;
    for (int32_t k = 0; k < b->sym->n; k++) perm[k] = b->sym->perm[k];
    return IMPC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device memory utilities
int impc_device_alloc(impc_ctx ctx, int64_t bytes, void **out) {
    if (!ctx || !out || bytes < 0) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    *out = nullptr;
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipMalloc(out, (size_t)std::max<int64_t>(bytes, 1)));
    return IMPC_OK;
}
int impc_device_free(impc_ctx ctx, void *ptr) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    if (!ptr) return IMPC_OK;
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipFree(ptr));
    return IMPC_OK;
}
int impc_copy_to_device(impc_ctx ctx, void *dst, const void *src, int64_t bytes) {
    if (!ctx || (bytes > 0 && (!dst || !src)) || bytes < 0) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    HIP_OK(hipSetDevice(ctx->device));
    IMPC_TRY(ctx_quiesce(ctx));
    IMPC_TRY(h2d_sync(ctx->stream, dst, src, (size_t)bytes));
    return IMPC_OK;
}
int impc_host_alloc(impc_ctx ctx, int64_t bytes, void **out) {
    if (!ctx || !out || bytes < 0) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    *out = nullptr;
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    return IMPC_OK;
}
int impc_host_free(impc_ctx ctx, void *ptr) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    if (ptr) HIP_OK(hipHostFree(ptr));
    return IMPC_OK;
}
int impc_stream_create(impc_ctx ctx, void **stream) {
    if (!ctx || !stream) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t s = nullptr;
    HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void *)s;
    return IMPC_OK;
}
int impc_stream_destroy(impc_ctx ctx, void *stream) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    if (stream) {
        HIP_OK(hipStreamSynchronize((hipStream_t)stream));
        HIP_OK(hipStreamDestroy((hipStream_t)stream));
    }
    return IMPC_OK;
}
int impc_stream_wait(impc_ctx ctx, void *waiter, void *signaler) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    HIP_OK(hipSetDevice(ctx->device));
    hipStream_t w = waiter ? (hipStream_t)waiter : ctx->stream, s = signaler ? (hipStream_t)signaler : ctx->stream;
    if (w == s) return IMPC_OK;
    hipEvent_t e = nullptr;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipError_t err = hipEventRecord(e, s);
    if (err == hipSuccess) err = hipStreamWaitEvent(w, e, 0);
    (void)hipEventDestroy(e);  // released once the wait has been satisfied
    if (err != hipSuccess) return fail(IMPC_DEVICE_ERROR, std::string("impc_stream_wait: ") + hipGetErrorString(err));
    return IMPC_OK;
}
int impc_stream_synchronize(impc_ctx ctx, void *stream) {
    if (!ctx) return fail(IMPC_INVALID_ARGUMENT, "null context");
    HIP_OK(hipSetDevice(ctx->device));
    HIP_OK(hipStreamSynchronize(stream ? (hipStream_t)stream : ctx->stream));
    return IMPC_OK;
}

int impc_copy_to_host(impc_ctx ctx, void *dst, const void *src, int64_t bytes) {
    if (!ctx || (bytes > 0 && (!dst || !src)) || bytes < 0) return fail(IMPC_INVALID_ARGUMENT, "invalid argument");
    HIP_OK(hipSetDevice(ctx->device));
    IMPC_TRY(ctx_quiesce(ctx));
    if (bytes) HIP_OK(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToHost));
    return IMPC_OK;
}

// ---------------------------------------------------------------- candidate scoring / selection
#include "select.hpp"

// ---------------------------------------------------------------- intent-hypothesis fan-out
#include "fanout.hpp"

// ---------------------------------------------------------------- obstacle intent probabilities
#include "predict.hpp"

// ---------------------------------------------------------------- on-device MPC -> QP assembly
#include "mpc_build.hpp"

// ---------------------------------------------------------------- RCCL communicator, step timer
#include "comm.hpp"

// ---------------------------------------------------------------- reference trajectory (getXRef)
#include "reftraj.hpp"

// ---------------------------------------------------------------- replan state (impc_replan.h)
#include "replan.hpp"

// ---------------------------------------------------------------- hooks for the library's other
// translation units (lib_internal.hpp; replan_run.hip): error reporting, stream ordering, and
// direct writes into a batch's device input arrays
namespace impc_lib {
int set_error(int code, const std::string &msg) { return fail(code, msg); }
int num_cu(impc_ctx ctx) { return ctx->num_cu; }
int device(impc_ctx ctx) { return ctx->device; }
hipStream_t stream(impc_ctx ctx) { return ctx->stream; }
int order_after_all(impc_ctx ctx) {
    HIP_OK(hipSetDevice(ctx->device));
    return ctx_order_after_all(ctx, ctx->stream);
}
int batch_inputs_begin(impc_batch b, BatchInputs *out) {
    if (!b || !out) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    IMPC_TRY(order_after_all(b->ctx));  // no launch on any stream still reads the arrays handed out
    b->in_dirty = b->ws_dirty = false;   // staged host copies are superseded
    out->Px = b->in_Px, out->q = b->in_q, out->Ax = b->in_Ax, out->l = b->in_l, out->u = b->in_u;
    out->xws = b->in_xws;
    out->n = b->n, out->m = b->m, out->nnzP = b->nnzP, out->nnzA = b->nnzA, out->B = b->B;
    return IMPC_OK;
}
int batch_inputs_view(impc_batch b, BatchInputs *out) {
    if (!b || !out) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    out->Px = b->in_Px, out->q = b->in_q, out->Ax = b->in_Ax, out->l = b->in_l, out->u = b->in_u;
    out->xws = b->in_xws;
    out->n = b->n, out->m = b->m, out->nnzP = b->nnzP, out->nnzA = b->nnzA, out->B = b->B;
    return IMPC_OK;
}
int batch_set_active_device(impc_batch b, const int64_t *d_count) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (d_count && !use_structured(b))
        return fail(IMPC_UNSUPPORTED, "device-side active counts need the structured kernel");
    b->d_active = d_count;
    b->Bact = b->B;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;
    b->generic_dirty = true;
    return IMPC_OK;
}
int batch_tlim_device(impc_batch b, double **out) {
    if (!b || !out) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (!b->d_tlim) {
        HIP_OK(hipMalloc((void **)&b->d_tlim, sizeof(double) * (size_t)b->B));
        b->device_bytes += (int64_t)sizeof(double) * b->B;
        IMPC_TRY(fill0_sync(b->ctx->stream, b->d_tlim, sizeof(double) * (size_t)b->B));
    }
    b->tlim_on = true;
    *out = b->d_tlim;
    return IMPC_OK;
}
double tick_s(impc_ctx ctx) { return ctx->tick_s; }
int build_rows(impc_mpc_builder bd, int64_t cap, const int64_t *dcount, const int32_t *row_inst, const int64_t *osrc,
               const double *pos, const double *vel, const double *xref, const double *lin, const double *pred_pos,
               const double *pred_size, const double *held_pos, const double *held_size, const double *st_centroid,
               const double *st_size, const double *st_yaw, const BatchInputs &out, hipStream_t st) {
    if (!bd || cap < 1) return fail(IMPC_INVALID_ARGUMENT, "build_rows: null builder or empty capacity");
    if (bd->S > 0 && (!st_centroid || !st_size || !st_yaw))
        return fail(IMPC_INVALID_ARGUMENT, "build_rows: static obstacles required by the builder");
    impc_build::Args a{cap, bd->n, bd->m, bd->nnzP, bd->nnzA, bd->obs_off, bd->N, bd->W, bd->S, bd->Kd, bd->K, bd->L,
                       bd->p.dynamic_safety_dist, bd->p.static_safety_dist, bd->p.position_weight,
                       bd->p.velocity_weight, bd->d_tPx, bd->d_tAx, bd->d_tl, bd->d_tu, bd->d_slot, pos, vel, xref,
                       lin, st_centroid, st_size, st_yaw, pred_pos, pred_size, out.Px, out.q, out.Ax, out.l, out.u};
    a.dcount = dcount, a.row_inst = row_inst, a.osrc = osrc, a.hp = held_pos, a.hs = held_size;
    const int64_t groups = std::min<int64_t>(cap, (int64_t)bd->ctx->num_cu * 8);
    hipLaunchKernelGGL(impc_build::k_build, dim3((unsigned)groups), dim3(256), 0, st, a);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}
int batch_inputs_end(impc_batch b, bool warm_x) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    b->shared = false;
    b->persist_valid = b->q_by_update = b->rescale = b->q_after = false;  // new data: the next solve sets up from scratch
    b->values_set = true;
    b->generic_dirty = true;
    b->has_ws = warm_x;
    b->ws_y = false;  // zero duals (solveTraj's warm start, mpcPlanner.cpp:480-497)
    if (warm_x) b->settings.warm_start = b->dst.warm_start = 1;
    return IMPC_OK;
}
}  // namespace impc_lib
