// Cycles per step of the structured kernel's 8-dim stage recursion a_{k+1} = t_{k+1} - F_k a_k
// (W = 19 steps, F and t in LDS), in several formulations, on gfx950.  Run with 1 wavefront per
// SIMD (64-lane blocks) and with 2 (512-lane blocks: waves w and w+4 share a SIMD).
//
//   0  lane grid 8x8, alternating strided/contiguous 8-lane sums, update_dpp(old = 0), an LDS
//      store of each stage (the kernel as of round 1)
//   1  as 0 with mov_dpp (bound_ctrl, no old operand)
//   2  as 1, results captured in registers (v_cndmask per step) instead of stored
//   3  as 1 without any store (the bare chain: lower bound of the lane-grid form)
//   4  broadcast form: lane i < 8 holds row i of F_k, a_k in SGPRs (v_readlane), products and a
//      depth-3 add tree in the lane (same rounding as the lane-grid sums); store per step
//   5  as 4 without the store
//   6  as 1, recursion fully unrolled up to the maximum W (runtime W, break past it): exact
//      waitcnts, exec-masked store of each stage
//   7  as 6, stages captured in registers with compile-time lane masks, stored after the sweep
//   8  row-broadcast form: lane l holds row (l & 7) of F_k (8 copies per wave), a_k lane i;
//      the 8 operands by v_mov_b64_dpp row_newbcast, 4 mul + 4 fma + depth-2 adds in the lane;
//      fully unrolled, captured in registers (copy l >> 3 keeps step m when m % 8 == l >> 3)
//   9  as 8 with an LDS store of each stage by lanes 0..7 (runtime loop)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 19, REP = 32;

template <int CTRL, bool BC>
__device__ double dpp(double v) {
    int lo, hi;
    if (BC) {
        lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
        hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
    } else {
        lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
        hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    }
    return __hiloint2double(hi, lo);
}
template <bool P32>
__device__ double pair_sum(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    if (P32) {
        auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
    }
    auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
}
template <bool BC>
__device__ double contig(double v) {
    v = v + dpp<0xB1, BC>(v);
    v = v + dpp<0x4E, BC>(v);
    return v + dpp<0x141, BC>(v);
}
template <bool BC>
__device__ double strided(double v) {
    v = v + dpp<0x128, BC>(v);
    v = pair_sum<false>(v);
    return pair_sum<true>(v);
}
template <int N>
__device__ double nbc(double v) { return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + N, 0xF, 0xF, false); }
__device__ double rowdot(const double (&f)[8], double a) {
    const double s0 = fma(f[1], nbc<1>(a), f[0] * nbc<0>(a)), s1 = fma(f[3], nbc<3>(a), f[2] * nbc<2>(a));
    const double s2 = fma(f[5], nbc<5>(a), f[4] * nbc<4>(a)), s3 = fma(f[7], nbc<7>(a), f[6] * nbc<6>(a));
    return (s0 + s1) + (s2 + s3);
}
__device__ double prod_nc(double a, double b) {
    double p = a * b;
    asm volatile("" : "+v"(p));
    return p;
}
__device__ double bcast(double v, int src) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ void kr(double *o, unsigned long long *cyc, int Wr) {
    __shared__ double F[8][64 * (W + 3)];
    __shared__ double t[8][13 * (W + 4)], out[8][13 * (W + 4)], junk[8][64];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, i = l >> 3, j = l & 7;
    for (int p = l; p < 64 * (W + 3); p += 64) F[wv][p] = 0.01 * ((p * 37) % 17) - 0.08;
    for (int p = l; p < 13 * (W + 4); p += 64) t[wv][p] = 0.1 * ((p * 11) % 7) - 0.3;
    __syncthreads();
    const double *Fm = F[wv], *tb = t[wv];
    double *rb = out[wv], *jk = junk[wv] + l;
    double acc = 0.0;
    unsigned long long c0 = 0;
    for (int rep = -1; rep < REP; rep++) {
        if (rep == 0) c0 = __builtin_amdgcn_s_memtime();
        if (MODE == 10) {
            // two independent chains (different starts) interleaved in one instruction stream:
            // is a step issue-bound or latency-bound at this occupancy?
            double a = tb[i], b = tb[26 + i];
            double fe = Fm[l], te = tb[13 + j], fo = Fm[64 + l], to = tb[26 + i];
            for (int k = 0; k < W; k += 2) {
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
                a = t0 - strided<true>(prod_nc(f0, a));
                b = 0.5 * t0 - strided<true>(prod_nc(f0, b));
                if (k + 1 >= W) break;
                const double f1 = fo, t1 = to;
                fo = Fm[64 * (k + 3) + l];
                to = tb[13 * (k + 4) + i];
                a = t1 - contig<true>(prod_nc(f1, a));
                b = 0.5 * t1 - contig<true>(prod_nc(f1, b));
            }
            acc += a + b;
        } else if (MODE >= 8) {
            const int r = l & 7, cp = l >> 3;
            double a = tb[r], f[8], fn[8], tn = tb[13 + r];
            double cap[3] = {0, 0, 0};
            _Pragma("unroll") for (int q = 0; q < 8; q++) f[q] = Fm[8 * r + q];
            if (MODE == 8) {
                _Pragma("unroll") for (int k = 0; k < W; k++) {
                    _Pragma("unroll") for (int q = 0; q < 8; q++) fn[q] = Fm[64 * (k + 1) + 8 * r + q];
                    const double tc = tn;
                    tn = tb[13 * (k + 2) + r];
                    a = tc - rowdot(f, a);
                    if ((k & 7) == cp) cap[k >> 3] = a;
                    _Pragma("unroll") for (int q = 0; q < 8; q++) f[q] = fn[q];
                }
                _Pragma("unroll") for (int qq = 0; qq < 3; qq++) {
                    const int k = 8 * qq + cp;
                    if (k < W) rb[13 * (k + 1) + r] = cap[qq];
                }
            } else {
                for (int k = 0; k < Wr; k++) {
                    _Pragma("unroll") for (int q = 0; q < 8; q++) fn[q] = Fm[64 * (k + 1) + 8 * r + q];
                    const double tc = tn;
                    tn = tb[13 * (k + 2) + r];
                    a = tc - rowdot(f, a);
                    *(l < 8 ? rb + 13 * (k + 1) + r : jk) = a;
                    _Pragma("unroll") for (int q = 0; q < 8; q++) f[q] = fn[q];
                }
            }
            acc += a;
        } else if (MODE <= 3) {
            constexpr bool BC = MODE >= 1;
            double co0 = 0, co1 = 0, ce0 = 0, ce1 = 0;
            double a = tb[i];
            double fe = Fm[l], te = tb[13 + j], fo = Fm[64 + l], to = tb[26 + i];
            for (int k = 0; k < W; k += 2) {
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
                a = t0 - strided<BC>(prod_nc(f0, a));
                if (MODE <= 1) *(i == 0 ? rb + 13 * (k + 1) + j : jk) = a;
                if (MODE == 2) {
                    const bool h = (((k + 1) >> 1) & 7) == i;
                    co0 = (h && (k + 1) < 16) ? a : co0;
                    co1 = (h && (k + 1) >= 16) ? a : co1;
                }
                if (k + 1 >= W) break;
                const double f1 = fo, t1 = to;
                fo = Fm[64 * (k + 3) + l];
                to = tb[13 * (k + 4) + i];
                a = t1 - contig<BC>(prod_nc(f1, a));
                if (MODE <= 1) *(j == 0 ? rb + 13 * (k + 2) + i : jk) = a;
                if (MODE == 2) {
                    const bool h = (((k + 2) >> 1) & 7) == j;
                    ce0 = (h && (k + 2) < 16) ? a : ce0;
                    ce1 = (h && (k + 2) >= 16) ? a : ce1;
                }
            }
            acc += a + co0 + co1 + ce0 + ce1;
        } else if (MODE >= 6) {
            double co[2] = {0, 0}, ce[2] = {0, 0};
            double a = tb[i];
            double fe = Fm[l], te = tb[13 + j], fo = Fm[64 + l], to = tb[26 + i];
            _Pragma("unroll") for (int k = 0; k < W; k += 2) {
                if (k >= Wr) continue;
                const double f0 = fe, t0 = te;
                fe = Fm[64 * (k + 2) + l];
                te = tb[13 * (k + 3) + j];
                a = t0 - strided<true>(prod_nc(f0, a));
                if (MODE == 6) {
                    if (i == 0) rb[13 * (k + 1) + j] = a;
                } else if ((((k + 1) >> 1) & 7) == i) {
                    co[(k + 1) >> 4] = a;
                }
                if (k + 1 >= Wr) continue;
                const double f1 = fo, t1 = to;
                fo = Fm[64 * (k + 3) + l];
                to = tb[13 * (k + 4) + i];
                a = t1 - contig<true>(prod_nc(f1, a));
                if (MODE == 6) {
                    if (j == 0) rb[13 * (k + 2) + i] = a;
                } else if ((((k + 2) >> 1) & 7) == j) {
                    ce[(k + 2) >> 4] = a;
                }
            }
            if (MODE == 7) {
                _Pragma("unroll") for (int qq = 0; qq < 2; qq++) {
                    const int so = 2 * (8 * qq + i) + 1, se = 2 * (8 * qq + j);
                    if (so <= Wr) rb[13 * so + j] = co[qq];
                    if (se >= 1 && se <= Wr) rb[13 * se + i] = ce[qq];
                }
            }
            acc += a;
        } else {
            // broadcast form: lane r = l & 7 holds row r of F_k (row-major layout in this probe)
            const int r = l & 7;
            double av[8];
            _Pragma("unroll") for (int q = 0; q < 8; q++) av[q] = tb[q];
            double f[8], tn = tb[13 + r];
            _Pragma("unroll") for (int q = 0; q < 8; q++) f[q] = Fm[8 * r + q];
            for (int k = 0; k < W; k++) {
                double fc[8];
                _Pragma("unroll") for (int q = 0; q < 8; q++) fc[q] = f[q];
                const double tc = tn;
                _Pragma("unroll") for (int q = 0; q < 8; q++) f[q] = Fm[64 * (k + 1) + 8 * r + q];
                tn = tb[13 * (k + 2) + r];
                double p[8];
                _Pragma("unroll") for (int q = 0; q < 8; q++) p[q] = prod_nc(fc[q], av[q]);
                const double s = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
                const double res = tc - s;
                if (MODE == 4) *(l < 8 ? rb + 13 * (k + 1) + r : jk) = res;
                _Pragma("unroll") for (int q = 0; q < 8; q++) av[q] = bcast(res, q);
            }
            acc += av[0];
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    o[threadIdx.x] = acc + rb[l];
    if (threadIdx.x == 0) cyc[MODE] = (c1 - c0) / (REP * W);
}

int main() {
    double *o;
    unsigned long long *c, h[11] = {};
    if (hipMalloc(&o, 512 * sizeof(double)) || hipMalloc(&c, sizeof(h))) return 1;
    const char *nm[] = {"grid, update_dpp, store", "grid, mov_dpp, store", "grid, mov_dpp, capture",
                        "grid, mov_dpp, bare", "broadcast, store", "broadcast, bare", "unrolled, masked store",
                        "unrolled, const-mask capture", "row-bcast, unrolled capture", "row-bcast, store",
                        "grid, two chains interleaved"};
    for (int threads : {64, 512}) {
        for (int it = 0; it < 2; it++) {
            hipLaunchKernelGGL(kr<0>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<1>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<2>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<3>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<4>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<5>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<6>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<7>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<8>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<9>, 1, threads, 0, 0, o, c, W);
            hipLaunchKernelGGL(kr<10>, 1, threads, 0, 0, o, c, W);
        }
        if (hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost)) return 1;
        printf("-- %d lanes (%d wave(s) per SIMD)\n", threads, threads > 256 ? 2 : 1);
        for (int m = 0; m < 11; m++) printf("%-28s %llu cyc/step\n", nm[m], h[m]);
    }
    return 0;
}
