// Cycles per step of the 8-dim stage recursion a_{k+1} = t_{k+1} - F_k a_k (W = 19 steps, F and t
// in LDS) in two formulations, on gfx950, with 1 and 2 wavefronts per SIMD:
//
//   A  the kernel's lane grid (lane 8i + j holds F_k[i][j]; alternating strided / contiguous
//      8-lane sums by DPP / permlane), results captured in registers
//   B  row-broadcast with fused operands: lane l holds row r = l & 7 of -F_k (8 copies of the
//      grid per wave, two per 16-lane DPP row) and a_k in lane r of every DPP row; each term is
//      one v_fmac_f64 whose a operand comes from lane q of the row by DPP row_newbcast:q (the
//      64-bit DPP control gfx950 has), two accumulation chains of four, one add
//
// Output: cycles per step (s_memtime), and the largest |A - B| over the run (the two sum in
// different orders, so they agree to rounding, not bitwise).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

constexpr int W = 19, REP = 64;

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

// acc += (lane q of this DPP row's a) * f; NOP: the 2 wait states a VALU write of a needs
// before a DPP read of it (the hazard recognizer cannot see the DPP inside the asm)
template <int Q, bool NOP = false>
__device__ void fmac_bc(double &acc, double a, double f) {
    if (NOP)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc)
            : "v"(a), "v"(f), "n"(Q));
    else
        asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc)
            : "v"(a), "v"(f), "n"(Q));
}

template <int MODE>
__global__ void kr(double *o, unsigned long long *cyc) {
    // per wave: F_k row-major [W + 3][8][8] (-F_k for MODE B), t [W + 4][8]
    __shared__ double F[8][64 * (W + 3)], t[8][8 * (W + 4)];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int p = l; p < 64 * (W + 3); p += 64) {
        const double f = 0.01 * ((p * 37) % 17) - 0.08;
        F[wv][p] = MODE == 0 ? f : -f;  // MODE B keeps -F_k
    }
    for (int p = l; p < 8 * (W + 4); p += 64) t[wv][p] = 0.1 * ((p * 11) % 7) - 0.3;
    __syncthreads();
    const double *Fm = F[wv], *Nm = F[wv], *tb = t[wv];
    double acc_out = 0.0;
    unsigned long long c0 = 0;
    for (int rep = -1; rep < REP; rep++) {
        if (rep == 0) c0 = __builtin_amdgcn_s_memtime();
        if (MODE == 0) {
            // lane grid: i = l >> 3, j = l & 7; even steps reduce over i (F_k[i][j] a_i -> index j),
            // odd steps over j (F_k[j][i] stored transposed ... here: F read as [j][i] for odd k)
            const int i = l >> 3, j = l & 7;
            double a = tb[i];
            _Pragma("unroll") for (int k = 0; k < W; k++) {
                if ((k & 1) == 0) {
                    const double f = Fm[64 * k + 8 * j + i];  // F_k[j][i] at lane (i, j): sum over i -> y_j
                    a = tb[8 * (k + 1) + j] - strided(prod_nc(f, a));
                } else {
                    const double f = Fm[64 * k + 8 * i + j];  // F_k[i][j]: sum over j -> y_i
                    a = tb[8 * (k + 1) + i] - contig(prod_nc(f, a));
                }
            }
            // a is y at index j (W odd: last step k = 18 even -> index j)
            acc_out += a;
        } else {
            const int r = l & 7;
            double a = tb[r];
            double fr[8], fn[8];
            _Pragma("unroll") for (int q = 0; q < 8; q++) fr[q] = Nm[8 * r + q];
            _Pragma("unroll") for (int k = 0; k < W; k++) {
                _Pragma("unroll") for (int q = 0; q < 8; q++) fn[q] = Nm[64 * (k + 1) + 8 * r + q];
                double acc0 = tb[8 * (k + 1) + r], acc1 = 0.0;
                fmac_bc<0, true>(acc0, a, fr[0]);
                fmac_bc<4>(acc1, a, fr[4]);
                fmac_bc<1>(acc0, a, fr[1]);
                fmac_bc<5>(acc1, a, fr[5]);
                fmac_bc<2>(acc0, a, fr[2]);
                fmac_bc<6>(acc1, a, fr[6]);
                fmac_bc<3>(acc0, a, fr[3]);
                fmac_bc<7>(acc1, a, fr[7]);
                a = acc0 + acc1;
                _Pragma("unroll") for (int q = 0; q < 8; q++) fr[q] = fn[q];
            }
            acc_out += a;
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    o[threadIdx.x] = acc_out;
    if (threadIdx.x == 0) cyc[MODE] = (c1 - c0) / (REP * W);
}

int main() {
    double *o;
    unsigned long long *c, h[2] = {};
    if (hipMalloc(&o, 2 * 512 * sizeof(double)) || hipMalloc(&c, sizeof(h))) return 1;
    double ho[2][512];
    for (int threads : {64, 512}) {
        for (int it = 0; it < 2; it++) {
            hipLaunchKernelGGL(kr<0>, 1, threads, 0, 0, o, c);
            hipLaunchKernelGGL(kr<1>, 1, threads, 0, 0, o + 512, c);
        }
        if (hipDeviceSynchronize() || hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost) ||
            hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost))
            return 1;
        // compare the final vectors: A holds y at index j = l & 7, B at index r = l & 7
        double md = 0.0;
        for (int l = 0; l < 64; l++) md = fmax(md, fabs(ho[0][l] - ho[1][l]));
        printf("-- %d lanes (%d wave(s) per SIMD): lane grid %llu cyc/step, row-broadcast fmac %llu cyc/step, max |A-B| %.3g (A %.6f B %.6f)\n",
               threads, threads > 256 ? 2 : 1, h[0], h[1], md, ho[0][3], ho[1][3]);
    }
    return 0;
}
