// Cycles per step of the 8-dim stage recursion a_{k+1} = t_{k+1} - F_k a_k (W = 19 steps, F and t
// in LDS) on gfx950: the structured kernel's lane-grid form (8x8 lanes, product + 8-lane DPP /
// permlane sums, results captured in registers) against an MFMA form -- two dependent
// v_mfma_f64_16x16x4_f64 per step:
//     D = C + A0 B0 + A1 B1,  A = -F_k (rows 0..7, cols 0..3 / 4..7), B = a_k replicated over the 16
//     columns, C = t_{k+1}
// whose D registers 0 / 1 (rows (lane >> 4) + 4 r, col lane & 15) ARE the next step's B operands
// (row lane >> 4 of the 4 x 16 B, chunk 0 / 1): no cross-lane move on the chain.  Also checks the
// MFMA chain against a sequential fma reference (max abs difference) and the backward form
// x_k = e_k - F_k' x_{k+1} (A read transposed).
//
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_recur_probe.hip -o mfma_recur_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

constexpr int W = 19, REP = 32;
typedef double d4 __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ double dpp(double v) {
    int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
    int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
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
__device__ double contig(double v) {
    v = v + dpp<0xB1>(v);
    v = v + dpp<0x4E>(v);
    return v + dpp<0x141>(v);
}
__device__ double strided(double v) {
    v = v + dpp<0x128>(v);
    v = pair_sum<false>(v);
    return pair_sum<true>(v);
}
__device__ double prod_nc(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}

// MODE 0: lane grid (the kernel's form), MODE 1: MFMA forward, MODE 2: MFMA backward
template <int MODE>
__global__ void kr(double *o, unsigned long long *cyc) {
    __shared__ double F[64 * (W + 3)];
    __shared__ double t[13 * (W + 4)], out[13 * (W + 4)], Fn[64 * (W + 3)];
    const int l = threadIdx.x & 63, i = l >> 3, j = l & 7;
    for (int p = l; p < 64 * (W + 3); p += 64) F[p] = 0.01 * ((p * 37) % 17) - 0.08;
    for (int p = l; p < 64 * (W + 3); p += 64) Fn[p] = -F[p];
    for (int p = l; p < 13 * (W + 4); p += 64) t[p] = 0.1 * ((p * 11) % 7) - 0.3;
    for (int p = l; p < 13 * (W + 4); p += 64) out[p] = 0.0;
    __syncthreads();
    double acc = 0.0;
    unsigned long long c0 = 0;
    const int r16 = l & 15, g = l >> 4;
    for (int rep = -1; rep < REP; rep++) {
        if (rep == 0) c0 = __builtin_amdgcn_s_memtime();
        if (MODE == 0) {
            double a = t[i];
            double fe = F[l], te = t[13 + j], fo = F[64 + l], to = t[26 + i];
            double c0v = 0, c1v = 0;
            for (int k = 0; k < W; k += 2) {
                const double f0 = fe, t0 = te;
                fe = F[64 * (k + 2) + l];
                te = t[13 * (k + 3) + j];
                a = t0 - strided(prod_nc(f0, a));
                if ((((k + 1) >> 1) & 7) == i) c0v = a;
                if (k + 1 >= W) break;
                const double f1 = fo, t1 = to;
                fo = F[64 * (k + 3) + l];
                to = t[13 * (k + 4) + i];
                a = t1 - contig(prod_nc(f1, a));
                if ((((k + 2) >> 1) & 7) == j) c1v = a;
            }
            acc += a + c0v + c1v;
        } else {
            // B operands: a_k[g] (chunk 0) and a_k[4 + g] (chunk 1), replicated over the 16 columns
            double b0 = t[g], b1 = t[4 + g];
            // A operands of step k: -F_k[r16][g], -F_k[r16][4 + g] (forward, F row-major) or
            // -F_k[g][r16], -F_k[4 + g][r16] (backward, transposed); prefetched one step ahead
            // (the kernel would store -F_k; rows 8..15 of A read row r16 - 8 again: their D rows,
            // registers 2 and 3, are never used, so no select sits between the load and the MFMA)
            const int rr = r16 & 7;
            auto ldA = [&](int k, double &a0, double &a1) {
                const double *Fk = Fn + 64 * k;
                if (MODE == 1) {
                    a0 = Fk[8 * rr + g];
                    a1 = Fk[8 * rr + 4 + g];
                } else {
                    a0 = Fk[8 * g + rr];
                    a1 = Fk[8 * (4 + g) + rr];
                }
            };
            double A0, A1, nA0, nA1;
            ldA(0, A0, A1);
            double tc0 = t[13 + g], tc1 = t[13 + 4 + g];
            double cap0[2] = {0, 0}, cap1[2] = {0, 0};
            _Pragma("unroll") for (int k = 0; k < W; k++) {
                ldA(k + 1, nA0, nA1);
                const double nt0 = t[13 * (k + 2) + g], nt1 = t[13 * (k + 2) + 4 + g];
                d4 c = {tc0, tc1, 0.0, 0.0};
                c = __builtin_amdgcn_mfma_f64_16x16x4f64(A0, b0, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f64_16x16x4f64(A1, b1, c, 0, 0, 0);
                b0 = c[0];
                b1 = c[1];
                if ((k & 15) == r16) {
                    cap0[k >> 4] = b0;
                    cap1[k >> 4] = b1;
                }
                A0 = nA0, A1 = nA1, tc0 = nt0, tc1 = nt1;
            }
            _Pragma("unroll") for (int q = 0; q < 2; q++) {
                const int k = 16 * q + r16;
                if (k < W) {
                    out[13 * (k + 1) + g] = cap0[q];
                    out[13 * (k + 1) + 4 + g] = cap1[q];
                }
            }
            acc += b0 + b1;
        }
    }
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    o[l] = acc;
    if (l == 0) cyc[0] = (c1 - c0) / REP;
    // reference: sequential fma chain in lane 0 (double), compared with what the sweep stored
    if (MODE != 0 && l == 0) {
        double a[8], an[8], md = 0.0;
        for (int r = 0; r < 8; r++) a[r] = t[r];
        for (int k = 0; k < W; k++) {
            for (int r = 0; r < 8; r++) {
                double s = t[13 * (k + 1) + r];
                for (int c = 0; c < 8; c++) s -= (MODE == 1 ? F[64 * k + 8 * r + c] : F[64 * k + 8 * c + r]) * a[c];
                an[r] = s;
            }
            for (int r = 0; r < 8; r++) {
                a[r] = an[r];
                md = fmax(md, fabs(out[13 * (k + 1) + r] - a[r]));
            }
        }
        o[64] = md;
    }
}

int main() {
    double *o, h[65] = {};
    unsigned long long *c, hc = 0;
    if (hipMalloc(&o, 65 * sizeof(double)) || hipMalloc(&c, sizeof(hc))) return 1;
    const char *nm[] = {"lane grid (kernel form)", "mfma f64 16x16x4, forward", "mfma f64 16x16x4, backward"};
    for (int mode = 0; mode < 3; mode++) {
        for (int it = 0; it < 2; it++) {
            if (mode == 0) hipLaunchKernelGGL(kr<0>, 1, 64, 0, 0, o, c);
            if (mode == 1) hipLaunchKernelGGL(kr<1>, 1, 64, 0, 0, o, c);
            if (mode == 2) hipLaunchKernelGGL(kr<2>, 1, 64, 0, 0, o, c);
        }
        if (hipMemcpy(&hc, c, sizeof(hc), hipMemcpyDeviceToHost) || hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost))
            return 1;
        std::printf("%-30s %6.1f cycles/step  (sweep %llu)%s", nm[mode], (double)hc / W, hc, mode ? "" : "\n");
        if (mode) std::printf("  max |mfma - fma chain| = %.3e\n", h[64]);
    }
    return 0;
}
