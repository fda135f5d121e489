// Probe 2: is the VOP3 / VOP3P issue cost on gfx950 (≈3.5-4 cycles per wave64 instruction at
// 8 waves per SIMD, against ≈2 for VOP2 v_add_u32 in issue_probe) the encoding size (8 bytes) or the
// operation?  256-thread workgroups (one wave per SIMD), W workgroups per CU, time from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP8(X) X X X X X X X X
#define NIT 256
#define B8(I) I " %0, %0, %8\n\t" I " %1, %1, %8\n\t" I " %2, %2, %8\n\t" I " %3, %3, %8\n\t" I " %4, %4, %8\n\t" I " %5, %5, %8\n\t" I " %6, %6, %8\n\t" I " %7, %7, %8"
#define OPS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c)

template <int K>
__global__ __launch_bounds__(256) void probe(unsigned long long* out, unsigned* d) {
    const int t = threadIdx.x & 63;
    unsigned a0 = d[t], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned c = d[t + 64];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NIT; it++) {
        if (K == 0) { REP8(asm volatile(B8("v_add_u32_e32") OPS);) }
        if (K == 1) { REP8(asm volatile(B8("v_add_u32_e64") OPS);) }
        if (K == 2) { REP8(asm volatile("v_add_u32 %0, 0x12345, %0\n\tv_add_u32 %1, 0x12345, %1\n\tv_add_u32 %2, 0x12345, %2\n\tv_add_u32 %3, 0x12345, %3\n\tv_add_u32 %4, 0x12345, %4\n\tv_add_u32 %5, 0x12345, %5\n\tv_add_u32 %6, 0x12345, %6\n\tv_add_u32 %7, 0x12345, %7" OPS);) }
        if (K == 3) { REP8(asm volatile(B8("v_pk_max_u16") OPS);) }
        if (K == 4) { REP8(asm volatile(B8("v_max_u16_e32") OPS);) }
        if (K == 5) { REP8(asm volatile("v_max_u16_sdwa %0, %0, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %1, %1, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %2, %2, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %3, %3, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %4, %4, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %5, %5, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %6, %6, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\tv_max_u16_sdwa %7, %7, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1" OPS);) }
        if (K == 6) { REP8(asm volatile("v_add_u32_dpp %0, %8, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %1, %8, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %2, %8, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %3, %8, %3 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %4, %8, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %5, %8, %5 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %6, %8, %6 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_u32_dpp %7, %8, %7 row_shr:1 row_mask:0xf bank_mask:0xf" OPS);) }
        if (K == 7) { REP8(asm volatile(B8("v_and_b32_e32") OPS);) }
        if (K == 8) { REP8(asm volatile("v_lshl_or_b32 %0, %0, 3, %8\n\tv_lshl_or_b32 %1, %1, 3, %8\n\tv_lshl_or_b32 %2, %2, 3, %8\n\tv_lshl_or_b32 %3, %3, 3, %8\n\tv_lshl_or_b32 %4, %4, 3, %8\n\tv_lshl_or_b32 %5, %5, 3, %8\n\tv_lshl_or_b32 %6, %6, 3, %8\n\tv_lshl_or_b32 %7, %7, 3, %8" OPS);) }
        if (K == 9) { REP8(asm volatile("v_pk_max_u16 %0, %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_pk_max_u16 %2, %2, %8\n\tv_add_u32_e32 %3, %3, %8\n\tv_pk_max_u16 %4, %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_pk_max_u16 %6, %6, %8\n\tv_add_u32_e32 %7, %7, %8" OPS);) }
        if (K == 10) { REP8(asm volatile(B8("v_pk_add_u16") OPS);) }
        if (K == 11) { REP8(asm volatile(B8("v_max_u32_e32") OPS);) }
        if (K == 12) { REP8(asm volatile(B8("v_max_u32_e64") OPS);) }
        if (K == 13) { REP8(asm volatile("v_max3_u32 %0, %0, %8, %1\n\tv_max3_u32 %1, %1, %8, %2\n\tv_max3_u32 %2, %2, %8, %3\n\tv_max3_u32 %3, %3, %8, %4\n\tv_max3_u32 %4, %4, %8, %5\n\tv_max3_u32 %5, %5, %8, %6\n\tv_max3_u32 %6, %6, %8, %7\n\tv_max3_u32 %7, %7, %8, %0" OPS);) }
        if (K == 14) { REP8(asm volatile(B8("v_pk_max_i16") OPS);) }
        if (K == 15) { REP8(asm volatile(B8("v_xor_b32_e32") OPS);) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    d[t + 128] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (t == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int K>
void run(const char* name, unsigned long long* o, unsigned* d, unsigned long long* h, int ncu) {
    const int ninstr = NIT * 64;
    printf("%-16s", name);
    for (int W : {1, 4, 8}) {
        const int nb = ncu * W;
        for (int rep = 0; rep < 2; rep++) probe<K><<<nb, 256>>>(o, d);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, o, nb * 4 * 8, hipMemcpyDeviceToHost);
        unsigned long long mx = 0, sum = 0;
        for (int b = 0; b < nb * 4; b++) { mx = h[b] > mx ? h[b] : mx; sum += h[b]; }
        printf("  W=%d: %.2f (avg %.2f)", W, (double)mx / (W * ninstr), (double)sum / (nb * 4) / (W * ninstr));
    }
    printf("\n");
    fflush(stdout);
}

int main() {
    unsigned long long* o; unsigned* d;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipMalloc(&o, 1 << 20); (void)hipMalloc(&d, 4096); (void)hipMemset(d, 1, 4096);
    static unsigned long long h[1 << 17];
    printf("CUs %d; cycles per wave64 instruction per SIMD (W waves per SIMD), max (avg) over waves\n", ncu);
    run<0>("add_e32", o, d, h, ncu);
    run<1>("add_e64", o, d, h, ncu);
    run<2>("add_e32+lit", o, d, h, ncu);
    run<3>("pk_max_u16", o, d, h, ncu);
    run<4>("max_u16_e32", o, d, h, ncu);
    run<5>("max_u16_sdwa", o, d, h, ncu);
    run<6>("add_dpp", o, d, h, ncu);
    run<7>("and_e32", o, d, h, ncu);
    run<8>("lshl_or", o, d, h, ncu);
    run<9>("pk_max/add_e32", o, d, h, ncu);
    run<10>("pk_add_u16", o, d, h, ncu);
    run<11>("max_u32_e32", o, d, h, ncu);
    run<12>("max_u32_e64", o, d, h, ncu);
    run<13>("max3_u32", o, d, h, ncu);
    run<14>("pk_max_i16", o, d, h, ncu);
    run<15>("xor_e32", o, d, h, ncu);
    return 0;
}
