// Dependent-chain latency (cycles per op, one wave on the chip) of the instruction mixes used by
// the structured kernel's stage recursions on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ double dpp(double v) {
    int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ double p16(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double(rh[0], rl[0]) + __hiloint2double(rh[1], rl[1]);
}
__device__ double bperm(double v, int src) {
    int lo = __builtin_amdgcn_ds_bpermute(src << 2, __double2loint(v));
    int hi = __builtin_amdgcn_ds_bpermute(src << 2, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ void k(double *o, unsigned long long *cyc, double seed) {
    double v = seed + threadIdx.x * 1e-3, w = 1.0000001;
    const int REP = 256;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REP; r++) {
        if (MODE == 0) v = v * w;                         // f64 mul chain
        if (MODE == 1) v = v + w;                         // f64 add chain
        if (MODE == 2) v = __builtin_fma(v, w, 1e-9);     // f64 fma chain
        if (MODE == 3) v = v + dpp<0xB1>(v);              // dpp mov pair + add
        if (MODE == 4) v = p16(v) * 0.5;                  // permlane16 pair + add + mul
        if (MODE == 5) v = bperm(v, (threadIdx.x + 1) & 63) + w;  // ds_bpermute pair + add
        if (MODE == 6) { int x = __builtin_amdgcn_readlane(__double2loint(v), 3); v = v + (double)x; }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    o[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[MODE] = (t1 - t0) / REP;
}

int main() {
    double *o;
    unsigned long long *c, h[8] = {};
    if (hipMalloc(&o, 64 * sizeof(double)) || hipMalloc(&c, sizeof(h))) return 1;
    for (int it = 0; it < 2; it++) {
        hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, o, c, 1.0);
        hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, o, c, 1.0);
        hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, o, c, 1.0);
        hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, o, c, 1.0);
        hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, o, c, 1.0);
        hipLaunchKernelGGL(k<5>, 1, 64, 0, 0, o, c, 1.0);
        hipLaunchKernelGGL(k<6>, 1, 64, 0, 0, o, c, 1.0);
    }
    if (hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost)) return 1;
    const char *nm[] = {"mul_f64", "add_f64", "fma_f64", "dpp pair + add_f64", "permlane16 pair + add + mul",
                        "ds_bpermute pair + add", "readlane + cvt + add"};
    for (int i = 0; i < 7; i++) printf("%-32s %llu cyc/step\n", nm[i], h[i]);
    return 0;
}
