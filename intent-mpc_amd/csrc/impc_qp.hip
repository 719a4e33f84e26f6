// impc_qp.hip -- libimpc_qp.so: C-ABI (include/impc_qp.h), device memory management and the
// gfx950 kernels of the batched OSQP-equivalent solver.
//
// Kernels (one QP per lane, batch-interleaved storage, see admm_core.hpp):
//   k_interleave   QP-major -> interleaved (LDS-tiled transpose), used for inputs
//   k_setup        osqp_setup numeric part + osqp_warm_start           (admm_core: qp_setup)
//   k_solve        osqp_solve: ADMM, termination, adaptive rho, unscale (admm_core: qp_solve)
//   k_deinterleave interleaved -> QP-major, used for outputs
//   k_update_q / k_update_bounds  osqp_update_lin_cost / osqp_update_bounds
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/impc_qp.h"
#include "admm_core.hpp"
#include "symbolic.hpp"

#define IMPC_VERSION "impc_qp 0.1.0 (OSQP 0.6.2 semantics, gfx950)"

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

constexpr int kBlock = 64;       // one wavefront per workgroup: one QP per lane
constexpr int kTile = 64;        // transpose tile edge

// dst[e * S + b] = src[b * len + e]  for b < B, e < len.  64x64 tile through LDS so both the
// global read (along e) and the global write (along b) are coalesced.
__global__ __launch_bounds__(256) void k_interleave(const double *__restrict__ src, double *__restrict__ dst,
                                                    int64_t len, int64_t B, int64_t S) {
    __shared__ double tile[kTile][kTile + 1];
    const int64_t e0 = (int64_t)blockIdx.x * kTile, b0 = (int64_t)blockIdx.y * kTile;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
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

__global__ __launch_bounds__(kBlock) void k_setup(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st, int64_t B,
                                                  int has_ws) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    impc::qp_setup(sy, wk, st, lane, has_ws);
}

__global__ __launch_bounds__(kBlock) void k_solve(impc::DevSym sy, impc::DevWork wk, impc::DevSettings st,
                                                  int64_t B) {
    const int lane = blockIdx.x * kBlock + threadIdx.x;
    if (lane >= B) return;
    impc::qp_solve(sy, wk, st, lane, lane, 0);
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

struct DevBuf {
    void *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct impc_ctx_s {
    int device = 0;
    hipStream_t stream = nullptr;
};

struct impc_batch_s {
    impc_ctx ctx = nullptr;
    impc::Symbolic sym;
    int64_t B = 0, S = 0;
    impc_settings settings{};
    impc::DevSettings dst{};
    // device allocations
    void *d_sym = nullptr;      // all int32 symbolic arrays
    double *d_work = nullptr;   // all interleaved per-QP arrays
    double *d_xout = nullptr;   // QP-major results
    double *d_yout = nullptr;
    impc_info *d_info = nullptr;
    double *d_stage = nullptr;  // QP-major staging for inputs
    int64_t stage_len = 0;
    int64_t device_bytes = 0;
    impc::DevSym dsym{};
    impc::DevWork dwk{};
    bool values_set = false, dirty = true, has_ws = false, setup_done = false;
    // profiling: events around k_setup, k_solve, output transposes
    bool profile = false;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool ev_setup = false, ev_solve = false;
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

int interleave(impc_batch b, const double *src_dev, double *dst, int64_t len, hipStream_t st) {
    if (len <= 0) return IMPC_OK;
    dim3 grid((unsigned)((len + kTile - 1) / kTile), (unsigned)((b->S + kTile - 1) / kTile));
    hipLaunchKernelGGL(k_interleave, grid, dim3(256), 0, st, src_dev, dst, len, b->B, b->S);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int deinterleave(impc_batch b, const double *src, double *dst_dev, int64_t len, hipStream_t st) {
    if (len <= 0) return IMPC_OK;
    dim3 grid((unsigned)((len + kTile - 1) / kTile), (unsigned)((b->B + kTile - 1) / kTile));
    hipLaunchKernelGGL(k_deinterleave, grid, dim3(256), 0, st, src, dst_dev, len, b->B, b->S);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

// host QP-major array -> staging (H2D) -> interleaved destination
int upload(impc_batch b, const double *host, double *dst, int64_t len) {
    if (len <= 0) return IMPC_OK;
    hipStream_t st = b->ctx->stream;
    HIP_OK(hipMemcpyAsync(b->d_stage, host, sizeof(double) * (size_t)(len * b->B), hipMemcpyHostToDevice, st));
    int rc = interleave(b, b->d_stage, dst, len, st);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(st));  // staging buffer is reused by the next upload
    return IMPC_OK;
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
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
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
    HIP_OK(hipSetDevice(ctx->device));
    impc_batch b = new impc_batch_s();
    b->ctx = ctx;
    std::string err = b->sym.build(n, m, Pp, Pi, Ap, Ai);
    if (!err.empty()) {
        delete b;
        return fail(IMPC_DATA_VALIDATION_ERROR, err);
    }
    const impc::Symbolic &s = b->sym;
    b->B = batch;
    b->S = (batch + kBlock - 1) / kBlock * kBlock;
    impc_default_settings(&b->settings);
    to_dev_settings(&b->settings, &b->dst);

    // ---- symbolic arrays: one int32 allocation
    std::vector<const std::vector<int32_t> *> arrs = {&s.Pp, &s.Pi, &s.Ap, &s.Ai, &s.Arp, &s.Arpos, &s.Arcol,
                                                      &s.Arcolf, &s.perm, &s.iperm, &s.Mp, &s.Mi, &s.Mdiag,
                                                      &s.Pt_dest, &s.Pt_src, &s.At_dest, &s.At_a, &s.At_b,
                                                      &s.At_r, &s.Lp, &s.Li, &s.Lrp, &s.Lrc, &s.Lrpos,
                                                      &s.upd_ptr, &s.upd_c, &s.upd_js, &s.upd_je, &s.upd_w};
    std::vector<size_t> offs;
    size_t tot = 0;
    for (auto *a : arrs) {
        offs.push_back(tot);
        tot += (a->size() + 63) / 64 * 64;  // 256-B aligned sub-arrays
    }
    std::vector<int32_t> hsym(tot + 64, 0);
    for (size_t k = 0; k < arrs.size(); k++)
        if (!arrs[k]->empty()) std::memcpy(hsym.data() + offs[k], arrs[k]->data(), arrs[k]->size() * 4);
    hipError_t he = hipMalloc(&b->d_sym, hsym.size() * 4);
    if (he != hipSuccess) {
        delete b;
        return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(symbolic) failed");
    }
    he = hipMemcpy(b->d_sym, hsym.data(), hsym.size() * 4, hipMemcpyHostToDevice);
    if (he != hipSuccess) {
        impc_batch_destroy(b);
        return fail(IMPC_DEVICE_ERROR, "hipMemcpy(symbolic) failed");
    }
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

    // ---- interleaved per-QP arrays: one double allocation, each sub-array len * S doubles
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
    he = hipMalloc((void **)&b->d_work, work_bytes);
    if (he != hipSuccess) {
        impc_batch_destroy(b);
        return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(work) failed: batch too large for device memory");
    }
    (void)hipMemset(b->d_work, 0, work_bytes);
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
    b->stage_len = std::max<int64_t>({nP, nA, n_, m_, 1});
    he = hipMalloc((void **)&b->d_stage, sizeof(double) * (size_t)(b->stage_len * b->B));
    if (he == hipSuccess) he = hipMalloc((void **)&b->d_xout, sizeof(double) * (size_t)(std::max<int64_t>(n_, 1) * b->B));
    if (he == hipSuccess) he = hipMalloc((void **)&b->d_yout, sizeof(double) * (size_t)(std::max<int64_t>(m_, 1) * b->B));
    if (he == hipSuccess) he = hipMalloc((void **)&b->d_info, sizeof(impc_info) * (size_t)b->B);
    if (he != hipSuccess) {
        impc_batch_destroy(b);
        return fail(IMPC_MEM_ALLOC_ERROR, "hipMalloc(staging/results) failed");
    }
    (void)hipMemset(b->d_info, 0, sizeof(impc_info) * (size_t)b->B);
    w.info = b->d_info;
    b->device_bytes = (int64_t)(work_bytes + hsym.size() * 4 + sizeof(double) * b->stage_len * b->B +
                                sizeof(double) * (n_ + m_) * b->B + sizeof(impc_info) * b->B);
    *out = b;
    return IMPC_OK;
}

int impc_batch_destroy(impc_batch b) {
    if (!b) return IMPC_OK;
    if (b->ctx) {
        (void)hipSetDevice(b->ctx->device);
        (void)hipStreamSynchronize(b->ctx->stream);
    }
    for (hipEvent_t e : b->ev)
        if (e) (void)hipEventDestroy(e);
    void *ptrs[] = {b->d_sym, b->d_work, b->d_xout, b->d_yout, b->d_info, b->d_stage};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete b;
    return IMPC_OK;
}

int impc_batch_set_settings(impc_batch b, const impc_settings *s) {
    if (!b || !s) return fail(IMPC_INVALID_ARGUMENT, "null batch or settings");
    impc::DevSettings d;
    int rc = to_dev_settings(s, &d);
    if (rc) return rc;
    // settings that change the setup phase invalidate it (OSQP takes them at osqp_setup)
    if (s->rho != b->settings.rho || s->sigma != b->settings.sigma || s->scaling != b->settings.scaling)
        b->dirty = true;
    b->settings = *s;
    b->dst = d;
    return IMPC_OK;
}

int impc_batch_set_values(impc_batch b, const double *Px, const double *q, const double *Ax, const double *l,
                          const double *u) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    const impc::Symbolic &s = b->sym;
    if ((s.nnzP && !Px) || !q || (s.nnzA && !Ax) || (s.m && (!l || !u)))
        return fail(IMPC_INVALID_ARGUMENT, "null value array");
    for (int64_t k = 0; k < (int64_t)s.m * b->B; k++)
        if (l[k] > u[k]) {
            char msg[160];
            std::snprintf(msg, sizeof msg, "lower bound greater than upper bound (QP %lld, row %lld)",
                          (long long)(k / s.m), (long long)(k % s.m));
            return fail(IMPC_DATA_VALIDATION_ERROR, msg);
        }
    HIP_OK(hipSetDevice(b->ctx->device));
    int rc;
    if ((rc = upload(b, Px, const_cast<double *>(b->dwk.Px), s.nnzP))) return rc;
    if ((rc = upload(b, q, const_cast<double *>(b->dwk.q), s.n))) return rc;
    if ((rc = upload(b, Ax, const_cast<double *>(b->dwk.Ax), s.nnzA))) return rc;
    if ((rc = upload(b, l, const_cast<double *>(b->dwk.l), s.m))) return rc;
    if ((rc = upload(b, u, const_cast<double *>(b->dwk.u), s.m))) return rc;
    b->values_set = true;
    b->dirty = true;
    return IMPC_OK;
}

int impc_batch_set_values_device(impc_batch b, const double *Px, const double *q, const double *Ax, const double *l,
                                 const double *u) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    const impc::Symbolic &s = b->sym;
    if ((s.nnzP && !Px) || !q || (s.nnzA && !Ax) || (s.m && (!l || !u)))
        return fail(IMPC_INVALID_ARGUMENT, "null value array");
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = b->ctx->stream;
    int rc;
    if ((rc = interleave(b, Px, const_cast<double *>(b->dwk.Px), s.nnzP, st))) return rc;
    if ((rc = interleave(b, q, const_cast<double *>(b->dwk.q), s.n, st))) return rc;
    if ((rc = interleave(b, Ax, const_cast<double *>(b->dwk.Ax), s.nnzA, st))) return rc;
    if ((rc = interleave(b, l, const_cast<double *>(b->dwk.l), s.m, st))) return rc;
    if ((rc = interleave(b, u, const_cast<double *>(b->dwk.u), s.m, st))) return rc;
    b->values_set = true;
    b->dirty = true;
    return IMPC_OK;
}

int impc_batch_warm_start(impc_batch b, const double *x, const double *y) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (!x) {
        b->has_ws = false;
        b->dirty = true;
        return IMPC_OK;
    }
    int rc = upload(b, x, const_cast<double *>(b->dwk.xws), b->sym.n);
    if (rc) return rc;
    if (y) {
        rc = upload(b, y, const_cast<double *>(b->dwk.yws), b->sym.m);
        if (rc) return rc;
    } else if (b->sym.m) {
        HIP_OK(hipMemsetAsync(const_cast<double *>(b->dwk.yws), 0, sizeof(double) * b->sym.m * b->S, b->ctx->stream));
    }
    b->has_ws = true;
    b->dirty = true;
    return IMPC_OK;
}

int impc_batch_setup(impc_batch b, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (!b->values_set) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "values not set");
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = pick(b, stream);
    if (b->profile) HIP_OK(hipEventRecord(b->ev[0], st));
    hipLaunchKernelGGL(k_setup, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk, b->dst, b->B,
                       b->has_ws ? 1 : 0);
    HIP_OK(hipGetLastError());
    if (b->profile) {
        HIP_OK(hipEventRecord(b->ev[1], st));
        b->ev_setup = true;
    }
    b->dirty = false;
    b->setup_done = true;
    return IMPC_OK;
}

int impc_batch_solve(impc_batch b, void *stream) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    if (b->dirty) {
        int rc = impc_batch_setup(b, stream);
        if (rc) return rc;
    }
    HIP_OK(hipSetDevice(b->ctx->device));
    hipStream_t st = pick(b, stream);
    if (b->profile) HIP_OK(hipEventRecord(b->ev[2], st));
    hipLaunchKernelGGL(k_solve, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, st, b->dsym, b->dwk, b->dst, b->B);
    HIP_OK(hipGetLastError());
    if (b->profile) HIP_OK(hipEventRecord(b->ev[3], st));
    int rc = deinterleave(b, b->dwk.xo, b->d_xout, b->sym.n, st);
    if (!rc) rc = deinterleave(b, b->dwk.yo, b->d_yout, b->sym.m, st);
    if (!rc && b->profile) {
        HIP_OK(hipEventRecord(b->ev[4], st));
        b->ev_solve = true;
    }
    return rc;
}

int impc_batch_get(impc_batch b, double *x, double *y, impc_info *info) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    HIP_OK(hipStreamSynchronize(b->ctx->stream));
    HIP_OK(hipDeviceSynchronize());
    if (x) HIP_OK(hipMemcpy(x, b->d_xout, sizeof(double) * b->sym.n * b->B, hipMemcpyDeviceToHost));
    if (y && b->sym.m) HIP_OK(hipMemcpy(y, b->d_yout, sizeof(double) * b->sym.m * b->B, hipMemcpyDeviceToHost));
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

int impc_batch_update_lin_cost(impc_batch b, const double *q) {
    if (!b || !q) return fail(IMPC_INVALID_ARGUMENT, "null batch or q");
    if (!b->setup_done || b->dirty) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "setup has not run on current data");
    int rc = upload(b, q, const_cast<double *>(b->dwk.q), b->sym.n);
    if (rc) return rc;
    hipLaunchKernelGGL(k_update_q, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, b->ctx->stream, b->dsym, b->dwk,
                       b->dst, b->B);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int impc_batch_update_bounds(impc_batch b, const double *l, const double *u) {
    if (!b || (b->sym.m && (!l || !u))) return fail(IMPC_INVALID_ARGUMENT, "null batch or bounds");
    if (!b->setup_done || b->dirty) return fail(IMPC_WORKSPACE_NOT_INIT_ERROR, "setup has not run on current data");
    for (int64_t k = 0; k < (int64_t)b->sym.m * b->B; k++)
        if (l[k] > u[k]) return fail(IMPC_DATA_VALIDATION_ERROR, "lower bound greater than upper bound");
    int rc = upload(b, l, const_cast<double *>(b->dwk.l), b->sym.m);
    if (!rc) rc = upload(b, u, const_cast<double *>(b->dwk.u), b->sym.m);
    if (rc) return rc;
    hipLaunchKernelGGL(k_update_bounds, dim3((unsigned)(b->S / kBlock)), dim3(kBlock), 0, b->ctx->stream, b->dsym,
                       b->dwk, b->dst, b->B);
    HIP_OK(hipGetLastError());
    return IMPC_OK;
}

int impc_batch_get_stats(impc_batch b, impc_batch_stats *out) {
    if (!b || !out) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    out->n = b->sym.n;
    out->m = b->sym.m;
    out->nnzP = b->sym.nnzP;
    out->nnzA = b->sym.nnzA;
    out->batch = b->B;
    out->batch_stride = b->S;
    out->nnzL = b->sym.nnzL;
    out->nnzLcol = b->sym.nnzL;
    out->n_terms = (int64_t)b->sym.At_dest.size();
    out->bandwidth = b->sym.max_row_L;
    out->device_bytes = b->device_bytes;
    return IMPC_OK;
}

int impc_batch_set_profiling(impc_batch b, int on) {
    if (!b) return fail(IMPC_INVALID_ARGUMENT, "null batch");
    HIP_OK(hipSetDevice(b->ctx->device));
    if (on && !b->ev[0])
        for (hipEvent_t &e : b->ev) HIP_OK(hipEventCreate(&e));
    b->profile = on != 0;
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

int impc_batch_get_perm(impc_batch b, int64_t *perm) {
    if (!b || !perm) return fail(IMPC_INVALID_ARGUMENT, "null argument");
    for (int32_t k = 0; k < b->sym.n; k++) perm[k] = b->sym.perm[k];
    return IMPC_OK;
}

}  // extern "C"
