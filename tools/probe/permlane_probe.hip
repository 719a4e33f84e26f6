// Prints the lane mapping of v_permlane16_swap / v_permlane32_swap (gfx950) for one wavefront.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *o) {
    int v = threadIdx.x;
    int w = 100 + threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(v, w, false, false);
    auto q = __builtin_amdgcn_permlane16_swap(v, w, false, false);
    o[4 * threadIdx.x + 0] = r[0];
    o[4 * threadIdx.x + 1] = r[1];
    o[4 * threadIdx.x + 2] = q[0];
    o[4 * threadIdx.x + 3] = q[1];
}
int main() {
    int *d, h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l = 0; l < 64; l++) printf("lane %2d: p32 (%3d,%3d)  p16 (%3d,%3d)\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
    return hipFree(d) == hipSuccess ? 0 : 1;
}
