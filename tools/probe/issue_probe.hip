// Probe: issue THROUGHPUT of integer / packed-16 VALU, SALU and mixed streams on gfx950 with
// W wavefronts per SIMD (every CU filled): cycles per instruction per SIMD from s_memtime.
// Answers whether fast_cells' VALU mix (v_pk_*_u16, v_perm, v_mbcnt, v_add) issues at 2 or 4 cycles
// per wave64 instruction and whether the scalar unit is per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
#define NIT 256

template <int K>
__global__ __launch_bounds__(64) void probe(unsigned long long* out, unsigned* d) {
    unsigned a0 = d[threadIdx.x], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned c = d[threadIdx.x + 64];
    unsigned s0 = __builtin_amdgcn_readfirstlane(a0), s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NIT; it++) {
        if (K == 0) {   // 64 packed u16 max
            REP8(asm volatile("v_pk_max_u16 %0, %0, %8\n\tv_pk_max_u16 %1, %1, %8\n\tv_pk_max_u16 %2, %2, %8\n\tv_pk_max_u16 %3, %3, %8\n\tv_pk_max_u16 %4, %4, %8\n\tv_pk_max_u16 %5, %5, %8\n\tv_pk_max_u16 %6, %6, %8\n\tv_pk_max_u16 %7, %7, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));)
        } else if (K == 1) {   // 64 v_add_u32
            REP8(asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\tv_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));)
        } else if (K == 2) {   // 64 v_perm_b32
            REP8(asm volatile("v_perm_b32 %0, %0, %8, %8\n\tv_perm_b32 %1, %1, %8, %8\n\tv_perm_b32 %2, %2, %8, %8\n\tv_perm_b32 %3, %3, %8, %8\n\tv_perm_b32 %4, %4, %8, %8\n\tv_perm_b32 %5, %5, %8, %8\n\tv_perm_b32 %6, %6, %8, %8\n\tv_perm_b32 %7, %7, %8, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));)
        } else if (K == 3) {   // 64 s_add_u32 (4 chains)
            REP8(asm volatile("s_mul_i32 %0, %0, 3\n\ts_mul_i32 %1, %1, 3\n\ts_mul_i32 %2, %2, 3\n\ts_mul_i32 %3, %3, 3\n\ts_mul_i32 %0, %0, 3\n\ts_mul_i32 %1, %1, 3\n\ts_mul_i32 %2, %2, 3\n\ts_mul_i32 %3, %3, 3"
                              : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) : : "scc");)
        } else if (K == 4) {   // 32 v_pk_max_u16 + 32 s_add_u32 interleaved
            REP8(asm volatile("v_pk_max_u16 %0, %0, %8\n\ts_mul_i32 %4, %4, 3\n\tv_pk_max_u16 %1, %1, %8\n\ts_mul_i32 %5, %5, 3\n\tv_pk_max_u16 %2, %2, %8\n\ts_mul_i32 %6, %6, 3\n\tv_pk_max_u16 %3, %3, %8\n\ts_mul_i32 %7, %7, 3"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) : "v"(c) : "scc");)
        } else if (K == 5) {   // 64 v_mbcnt_lo
            REP8(asm volatile("v_mbcnt_lo_u32_b32 %0, %9, %0\n\tv_mbcnt_lo_u32_b32 %1, %9, %1\n\tv_mbcnt_lo_u32_b32 %2, %9, %2\n\tv_mbcnt_lo_u32_b32 %3, %9, %3\n\tv_mbcnt_lo_u32_b32 %4, %9, %4\n\tv_mbcnt_lo_u32_b32 %5, %9, %5\n\tv_mbcnt_lo_u32_b32 %6, %9, %6\n\tv_mbcnt_lo_u32_b32 %7, %9, %7"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c), "s"(s0));)
        } else if (K == 6) {   // 64 v_cmp_ne_u16 -> SGPR pair (ballot-like)
            unsigned long long m0, m1;
            REP8(asm volatile("v_cmp_ne_u16_e64 %0, %2, %3\n\tv_cmp_ne_u16_e64 %1, %3, %2\n\tv_cmp_ne_u16_e64 %0, %2, %3\n\tv_cmp_ne_u16_e64 %1, %3, %2\n\tv_cmp_ne_u16_e64 %0, %2, %3\n\tv_cmp_ne_u16_e64 %1, %3, %2\n\tv_cmp_ne_u16_e64 %0, %2, %3\n\tv_cmp_ne_u16_e64 %1, %3, %2"
                              : "=s"(m0), "=s"(m1) : "v"(a0), "v"(c));)
            a1 += (unsigned)m0 + (unsigned)m1;
        } else if (K == 7) {   // 64 v_alignbyte
            REP8(asm volatile("v_alignbyte_b32 %0, %0, %8, 1\n\tv_alignbyte_b32 %1, %1, %8, 1\n\tv_alignbyte_b32 %2, %2, %8, 1\n\tv_alignbyte_b32 %3, %3, %8, 1\n\tv_alignbyte_b32 %4, %4, %8, 1\n\tv_alignbyte_b32 %5, %5, %8, 1\n\tv_alignbyte_b32 %6, %6, %8, 1\n\tv_alignbyte_b32 %7, %7, %8, 1"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));)
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    d[threadIdx.x + 128] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s0 + s1 + s2 + s3;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, unsigned long long* o, unsigned* d, unsigned long long* h, int ncu) {
    const int ninstr = NIT * 64;
    printf("%-22s", name);
    for (int W : {1, 2, 4, 8}) {
        const int nb = ncu * 4 * W;
        for (int rep = 0; rep < 2; rep++) probe<K><<<nb, 64>>>(o, d);
        hipDeviceSynchronize();
        hipMemcpy(h, o, nb * 8, hipMemcpyDeviceToHost);
        unsigned long long mx = 0, sum = 0;
        for (int b = 0; b < nb; b++) { mx = h[b] > mx ? h[b] : mx; sum += h[b]; }
        // all W waves of a SIMD run concurrently: cycles per SIMD-instruction = elapsed / (W * ninstr)
        printf("  W=%d: %.2f (avg %.2f)", W, (double)mx / (W * ninstr), (double)sum / nb / (W * ninstr));
    }
    printf("\n");
    fflush(stdout);
}

int main() {
    unsigned long long* o; unsigned* d;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    hipMalloc(&o, 1 << 20); hipMalloc(&d, 4096); hipMemset(d, 1, 4096);
    static unsigned long long h[1 << 17];
    printf("CUs %d; cycles (s_memtime ticks) per wave64 instruction per SIMD, max over waves\n", ncu);
    run<0>("v_pk_max_u16", o, d, h, ncu);
    run<1>("v_add_u32", o, d, h, ncu);
    run<2>("v_perm_b32", o, d, h, ncu);
    run<3>("s_mul_i32", o, d, h, ncu);
    run<4>("pk_max+s_mul (per pair)", o, d, h, ncu);
    run<5>("v_mbcnt_lo", o, d, h, ncu);
    run<6>("v_cmp_ne_u16_e64", o, d, h, ncu);
    run<7>("v_alignbyte", o, d, h, ncu);
    return 0;
}
