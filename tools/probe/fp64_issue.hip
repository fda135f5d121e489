// Probe: issue cost of fp64 VALU forms on gfx950 for ONE wavefront (cycles per instruction, s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
__global__ void probe(unsigned long long* out, double* d) {
    double a0 = d[threadIdx.x], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    double nl = d[threadIdx.x + 64];
    unsigned long long t0, t1, t2, t3, t4, t5;
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; it++) {
        REP8(asm volatile("v_fmac_f64 %0, %8, %0\n\tv_fmac_f64 %1, %8, %1\n\tv_fmac_f64 %2, %8, %2\n\tv_fmac_f64 %3, %8, %3\n\tv_fmac_f64 %4, %8, %4\n\tv_fmac_f64 %5, %8, %5\n\tv_fmac_f64 %6, %8, %6\n\tv_fmac_f64 %7, %8, %7"
             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(nl));)
    }
    t1 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; it++) {
        REP8(asm volatile("v_fmac_f64_dpp %0, %0, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %1, %1, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %2, %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %3, %3, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %4, %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %5, %5, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %6, %6, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %7, %7, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf"
             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(nl));)
    }
    t2 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; it++) {   // dependent chain of plain fmac
        REP8(asm volatile("v_fmac_f64 %0, %1, %0" : "+v"(a0) : "v"(nl));)
    }
    t3 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; it++) {   // dependent rcp + fma chain
        REP8(asm volatile("v_rcp_f64 %0, %0\n\ts_nop 0\n\tv_fma_f64 %0, %0, %1, %0" : "+v"(a1) : "v"(nl));)
    }
    t4 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; it++) {   // dependent dpp-fmac chain
        REP8(asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a2) : "v"(nl));)
    }
    t5 = __builtin_amdgcn_s_memtime();
    d[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4; }
}
int main() {
    unsigned long long* o; double* d;
    hipMalloc(&o, 64); hipMalloc(&d, 128 * 8); hipMemset(d, 0, 128 * 8);
    unsigned long long h[5];
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o, d);
        hipMemcpy(h, o, 40, hipMemcpyDeviceToHost);
    }
    printf("cycles per instr: fmac_f64 (8 indep) %.2f | fmac_f64_dpp (8 indep) %.2f | fmac_f64 dep chain %.2f | rcp+fma dep pair %.2f | s_nop1+dpp-fmac dep chain %.2f\n",
           h[0] / 4096.0, h[1] / 4096.0, h[2] / 512.0, h[3] / 512.0, h[4] / 512.0);
    return 0;
}
