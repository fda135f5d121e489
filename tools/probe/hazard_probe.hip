// Hazard probe (gfx950): instruction pairs the compiler's hazard recognizer does not see when they sit in
// inline asm, each run many times over the whole chip and checked against the host, to learn which ones
// the hardware does NOT order by itself (VERDICT r04 "Next round" 3: the round-4 describe builds whose
// descriptors differed between identical runs).
//   T0  control: the same VALU ops with 4 s_nop wait states between writer and reader;
//   T1  v_mov_b32 x2 writing a VGPR pair, v_fmac_f64 reading it as the accumulator, 0 wait states
//       (DESIGN §4 describe round 4: the fma-sincos build's v_fmac_f64_e32 read a pair written by two
//       v_mov_b32 one or two instructions earlier);
//   T2  the same with the pair as src0 instead of the accumulator;
//   T3  v_mfma_i32_16x16x64_i8 with D exactly over A (the pattern tools/mfma_overlap.py reports in
//       describe_kernel), result read after 18 wait states, vs a D elsewhere;
//   T5  v_mfma_i32_16x16x64_i8 result read by a VALU K wait states after issue: the hardware's window;
//   T6/T7  WAR: a VALU overwrites the MFMA's SrcA / SrcC K wait states after its issue;
//   T8/T9  D partially over SrcA / SrcB (the DESC_ANGLE_MFMA=0 build's allocation);
//   T10/T11  an LDS load (VALU write) over SrcA of an MFMA queued behind 0-3 others (the angold build);
//   T4  positive control: VALU write -> DPP read of the same VGPR with 0 wait states (a documented
//       hazard: 2 wait states required) -- shows the probe can see a hazard at all.
// Every lane computes a known answer; the kernel counts lanes whose result differs.  No scalar stores.
// Build: hipcc --offload-arch=gfx950 -O2 hazard_probe.hip -o hazard_probe ; run: ./hazard_probe [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

typedef int i4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double fmac_pair_acc(double a, double b, unsigned clo, unsigned chi, int nop) {
    double r;
    if (nop)
        asm volatile(
            "v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\ts_nop 4\n\t"
            "v_fmac_f64_e32 v[40:41], %3, %4\n\ts_nop 4\n\tv_mov_b64 %0, v[40:41]\n\ts_nop 4"
            : "=v"(r) : "v"(clo), "v"(chi), "v"(a), "v"(b) : "v40", "v41");
    else
        asm volatile(
            "v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\t"
            "v_fmac_f64_e32 v[40:41], %3, %4\n\ts_nop 4\n\tv_mov_b64 %0, v[40:41]\n\ts_nop 4"
            : "=v"(r) : "v"(clo), "v"(chi), "v"(a), "v"(b) : "v40", "v41");
    return r;
}

__device__ __forceinline__ double fmac_pair_src(double c, double b, unsigned alo, unsigned ahi, int nop) {
    double r = c;
    if (nop)
        asm volatile(
            "v_mov_b32 v42, %1\n\tv_mov_b32 v43, %2\n\ts_nop 4\n\t"
            "v_fmac_f64_e32 %0, v[42:43], %3\n\ts_nop 4"
            : "+v"(r) : "v"(alo), "v"(ahi), "v"(b) : "v42", "v43");
    else
        asm volatile(
            "v_mov_b32 v42, %1\n\tv_mov_b32 v43, %2\n\t"
            "v_fmac_f64_e32 %0, v[42:43], %3\n\ts_nop 4"
            : "+v"(r) : "v"(alo), "v"(ahi), "v"(b) : "v42", "v43");
    return r;
}

// D over A exactly (overlap 1) or D elsewhere (overlap 0); C = 0.  The result is read 18+ wait states later.
__device__ __forceinline__ i4v mfma_da(i4v a, i4v b, int overlap) {
    i4v r;
    if (overlap)
        asm volatile(
            "v_mov_b32 v44, %1\n\tv_mov_b32 v45, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t"
            "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v50, %7\n\tv_mov_b32 v51, %8\n\ts_nop 4\n\t"
            "v_mfma_i32_16x16x64_i8 v[44:47], v[44:47], v[48:51], 0\n\t"
            "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
            "v_mov_b32 %0, v44\n\ts_nop 4"
            : "=v"(r.x) : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
            : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
    else
        asm volatile(
            "v_mov_b32 v44, %1\n\tv_mov_b32 v45, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t"
            "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v50, %7\n\tv_mov_b32 v51, %8\n\ts_nop 4\n\t"
            "v_mfma_i32_16x16x64_i8 v[52:55], v[44:47], v[48:51], 0\n\t"
            "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
            "v_mov_b32 %0, v52\n\ts_nop 4"
            : "=v"(r.x) : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
            : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");
    r.y = r.z = r.w = 0;
    return r;
}

// MFMA result read by a VALU K wait states after the MFMA issue (the MFMA's inputs settled 5 wait states
// before it).  K = 0 .. 18: the window the hardware needs for v_mfma_i32_16x16x64_i8 (D in VGPRs).
#define MFMA_RAW(K, NOPS)                                                                                   \
    __device__ __noinline__ int mfma_raw_##K(i4v a, i4v b) {                                               \
        int r;                                                                                              \
        asm volatile("v_mov_b32 v44, %1\n\tv_mov_b32 v45, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t"  \
                     "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v50, %7\n\tv_mov_b32 v51, %8\n\t"  \
                     "v_mov_b32 v52, 0\n\tv_mov_b32 v53, 0\n\tv_mov_b32 v54, 0\n\tv_mov_b32 v55, 0\n\ts_nop 4\n\t" \
                     "v_mfma_i32_16x16x64_i8 v[52:55], v[44:47], v[48:51], v[52:55]\n\t" NOPS                 \
                     "v_mov_b32 %0, v52\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"                                   \
                     : "=v"(r) : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w) \
                     : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");     \
        return r;                                                                                           \
    }
MFMA_RAW(0, "")
MFMA_RAW(2, "s_nop 1\n\t")
MFMA_RAW(4, "s_nop 3\n\t")
MFMA_RAW(6, "s_nop 5\n\t")
MFMA_RAW(8, "s_nop 7\n\t")
MFMA_RAW(9, "s_nop 7\n\ts_nop 0\n\t")
MFMA_RAW(10, "s_nop 7\n\ts_nop 1\n\t")
MFMA_RAW(11, "s_nop 7\n\ts_nop 2\n\t")
MFMA_RAW(12, "s_nop 7\n\ts_nop 3\n\t")
MFMA_RAW(14, "s_nop 7\n\ts_nop 5\n\t")
MFMA_RAW(16, "s_nop 7\n\ts_nop 7\n\t")
MFMA_RAW(20, "s_nop 7\n\ts_nop 7\n\ts_nop 3\n\t")
__device__ __forceinline__ int mfma_raw(int k, i4v a, i4v b) {
    switch (k) {
        case 0: return mfma_raw_0(a, b);
        case 2: return mfma_raw_2(a, b);
        case 4: return mfma_raw_4(a, b);
        case 6: return mfma_raw_6(a, b);
        case 8: return mfma_raw_8(a, b);
        case 9: return mfma_raw_9(a, b);
        case 10: return mfma_raw_10(a, b);
        case 11: return mfma_raw_11(a, b);
        case 12: return mfma_raw_12(a, b);
        case 14: return mfma_raw_14(a, b);
        case 16: return mfma_raw_16(a, b);
        default: return mfma_raw_20(a, b);
    }
}

// WAR: a VALU overwrites an MFMA source K wait states after the MFMA issue -- SrcA (v44) for T6, SrcC (v52,
// D elsewhere) for T7; the product is read 24+ wait states later and compared with the undisturbed one.
#define MFMA_WAR(K, NOPS)                                                                                   \
    __device__ __noinline__ int mfma_war_a_##K(i4v a, i4v b) {                                             \
        int r;                                                                                              \
        asm volatile("v_mov_b32 v44, %1\n\tv_mov_b32 v45, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t"  \
                     "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v50, %7\n\tv_mov_b32 v51, %8\n\ts_nop 4\n\t" \
                     "v_mfma_i32_16x16x64_i8 v[56:59], v[44:47], v[48:51], 0\n\t" NOPS                        \
                     "v_mov_b32 v44, 0x5a5a5a5a\n\tv_mov_b32 v47, 0x12345678\n\t"                            \
                     "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\tv_mov_b32 %0, v56\n\ts_nop 4"                        \
                     : "=v"(r) : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w) \
                     : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v56", "v57", "v58", "v59");     \
        return r;                                                                                           \
    }                                                                                                       \
    __device__ __noinline__ int mfma_war_c_##K(i4v a, i4v b) {                                             \
        int r;                                                                                              \
        asm volatile("v_mov_b32 v44, %1\n\tv_mov_b32 v45, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t"  \
                     "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v50, %7\n\tv_mov_b32 v51, %8\n\t"  \
                     "v_mov_b32 v52, 0x8000\n\tv_mov_b32 v53, 0x8000\n\tv_mov_b32 v54, 0x8000\n\tv_mov_b32 v55, 0x8000\n\ts_nop 4\n\t" \
                     "v_mfma_i32_16x16x64_i8 v[56:59], v[44:47], v[48:51], v[52:55]\n\t" NOPS                 \
                     "v_mov_b32 v52, 0x77777\n\tv_mov_b32 v55, 0x33333\n\t"                                    \
                     "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\tv_mov_b32 %0, v56\n\ts_nop 4"                        \
                     : "=v"(r) : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w) \
                     : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", \
                       "v57", "v58", "v59");                                                                    \
        return r;                                                                                           \
    }
MFMA_WAR(0, "")
MFMA_WAR(2, "s_nop 1\n\t")
MFMA_WAR(4, "s_nop 3\n\t")
MFMA_WAR(8, "s_nop 7\n\t")
MFMA_WAR(12, "s_nop 7\n\ts_nop 3\n\t")
MFMA_WAR(20, "s_nop 7\n\ts_nop 7\n\ts_nop 3\n\t")
__device__ __forceinline__ int mfma_war(int c, int k, i4v a, i4v b) {
    switch (k) {
        case 0: return c ? mfma_war_c_0(a, b) : mfma_war_a_0(a, b);
        case 2: return c ? mfma_war_c_2(a, b) : mfma_war_a_2(a, b);
        case 4: return c ? mfma_war_c_4(a, b) : mfma_war_a_4(a, b);
        case 8: return c ? mfma_war_c_8(a, b) : mfma_war_a_8(a, b);
        case 12: return c ? mfma_war_c_12(a, b) : mfma_war_a_12(a, b);
        default: return c ? mfma_war_c_20(a, b) : mfma_war_a_20(a, b);
    }
}

// D partially over a source: D = v[46:49] over SrcA v[44:47] (T8), D = v[50:53] over SrcB v[48:51] (T9),
// vs D = v[52:55] (no overlap); C = 0.  The allocation of the DESC_ANGLE_MFMA=0 describe build
// (`v_mfma_i32_16x16x64_i8 v[14:17], v[16:19], v[6:9], ...`), the one build that reproduces the
// round-4 nondeterminism.  Every D element compared.
#define MFMA_PART(NAME, D, D0, D1, D2, D3, ...)                                                           \
    __device__ __noinline__ i4v NAME(i4v a, i4v b) {                                                       \
        i4v r;                                                                                              \
        asm volatile("v_mov_b32 v44, %4\n\tv_mov_b32 v45, %5\n\tv_mov_b32 v46, %6\n\tv_mov_b32 v47, %7\n\t"  \
                     "v_mov_b32 v48, %8\n\tv_mov_b32 v49, %9\n\tv_mov_b32 v50, %10\n\tv_mov_b32 v51, %11\n\ts_nop 4\n\t" \
                     "v_mfma_i32_16x16x64_i8 " D ", v[44:47], v[48:51], 0\n\t"                                \
                     "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"                                                      \
                     "v_mov_b32 %0, " D0 "\n\tv_mov_b32 %1, " D1 "\n\tv_mov_b32 %2, " D2 "\n\tv_mov_b32 %3, " D3 "\n\ts_nop 4" \
                     : "=v"(r.x), "=v"(r.y), "=v"(r.z), "=v"(r.w)                                           \
                     : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)       \
                     : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", __VA_ARGS__);                  \
        return r;                                                                                           \
    }
MFMA_PART(mfma_part_a, "v[46:49]", "v46", "v47", "v48", "v49", "v52")
MFMA_PART(mfma_part_b, "v[50:53]", "v50", "v51", "v52", "v53", "v54")
MFMA_PART(mfma_part_none, "v[52:55]", "v52", "v53", "v54", "v55", "v56")

// The DESC_ANGLE_MFMA=0 describe build (the reproducible nondeterministic one) issues three MFMAs back to
// back and then a `ds_read_b128` whose destination overlaps the third MFMA's SrcA:
//     v_mfma v[32:35], v[16:19], ... ; v_mfma v[36:39], v[16:19], ... ; v_mfma v[14:17], v[16:19], ...
//     ds_read_b128 v[18:21], v40 offset:1536
// T10: NPRE MFMAs (0-3) on other registers, then the victim MFMA reading SrcA v[44:47], then an LDS load
// (or a VALU write for T11) into v[46:49] K wait states later; the victim's D vs the undisturbed product.
#define MFMA_LDS_WAR(NAME, PRE, OVW)                                                                         \
    __device__ __noinline__ int NAME(i4v a, i4v b, unsigned lds_addr) {                                    \
        int r;                                                                                               \
        asm volatile("v_mov_b32 v44, %1\n\tv_mov_b32 v45, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t"   \
                     "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v50, %7\n\tv_mov_b32 v51, %8\n\t"   \
                     "v_mov_b32 v60, %5\n\tv_mov_b32 v61, %6\n\tv_mov_b32 v62, %7\n\tv_mov_b32 v63, %8\n\ts_nop 4\n\t" \
                     PRE                                                                                      \
                     "v_mfma_i32_16x16x64_i8 v[52:55], v[44:47], v[60:63], 0\n\t"                              \
                     OVW                                                                                      \
                     "s_waitcnt lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"               \
                     "v_mov_b32 %0, v52\n\ts_nop 4"                                                           \
                     : "=v"(r)                                                                                \
                     : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(lds_addr) \
                     : "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56",  \
                       "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",  \
                       "v70", "v71", "memory");                                                               \
        return r;                                                                                            \
    }
#define PRE0 ""
#define PRE1 "v_mfma_i32_16x16x64_i8 v[64:67], v[48:51], v[60:63], 0\n\t"
#define PRE3 "v_mfma_i32_16x16x64_i8 v[64:67], v[48:51], v[60:63], 0\n\tv_mfma_i32_16x16x64_i8 v[68:71], v[48:51], v[60:63], 0\n\tv_mfma_i32_16x16x64_i8 v[56:59], v[48:51], v[60:63], 0\n\t"
#define OVW_LDS "ds_read_b128 v[46:49], %9\n\t"
#define OVW_LDS4 "s_nop 3\n\tds_read_b128 v[46:49], %9\n\t"
#define OVW_LDS16 "s_nop 7\n\ts_nop 7\n\tds_read_b128 v[46:49], %9\n\t"
#define OVW_VALU "v_mov_b32 v46, 0x5a5a5a5a\n\tv_mov_b32 v47, 0x12345678\n\t"
#define OVW_NONE ""
MFMA_LDS_WAR(war_lds_p0, PRE0, OVW_LDS)
MFMA_LDS_WAR(war_lds_p1, PRE1, OVW_LDS)
MFMA_LDS_WAR(war_lds_p3, PRE3, OVW_LDS)
MFMA_LDS_WAR(war_lds_p3k4, PRE3, OVW_LDS4)
MFMA_LDS_WAR(war_lds_p3k16, PRE3, OVW_LDS16)
MFMA_LDS_WAR(war_valu_p3, PRE3, OVW_VALU)
MFMA_LDS_WAR(war_none_p3, PRE3, OVW_NONE)

// T12: the DESC_ANGLE_MFMA=0 describe sequence (tools/ab lib_angold): three MFMAs reading the same SrcA,
// the third writing D partly over that SrcA, then an LDS load over the rest of SrcA.  Returns the 12
// result elements (three D's) folded into 4 sums of distinct weights.
#define MFMA3_LDS(NAME, D3, OVW)                                                                              \
    __device__ __noinline__ i4v NAME(i4v a, i4v b, unsigned lds_addr) {                                     \
        i4v r;                                                                                               \
        asm volatile("v_mov_b32 v44, %4\n\tv_mov_b32 v45, %5\n\tv_mov_b32 v46, %6\n\tv_mov_b32 v47, %7\n\t"   \
                     "v_mov_b32 v72, %8\n\tv_mov_b32 v73, %9\n\tv_mov_b32 v74, %10\n\tv_mov_b32 v75, %11\n\t" \
                     "v_mov_b32 v60, %9\n\tv_mov_b32 v61, %8\n\tv_mov_b32 v62, %11\n\tv_mov_b32 v63, %10\n\t" \
                     "v_mov_b32 v56, %11\n\tv_mov_b32 v57, %10\n\tv_mov_b32 v58, %9\n\tv_mov_b32 v59, %8\n\ts_nop 4\n\t" \
                     "v_mfma_i32_16x16x64_i8 v[64:67], v[44:47], v[72:75], 0\n\t"                              \
                     "v_mov_b32 v76, 1\n\tv_mov_b32 v77, 2\n\tv_mov_b32 v78, 3\n\tv_mov_b32 v79, 4\n\t"     \
                     "v_mfma_i32_16x16x64_i8 v[68:71], v[44:47], v[60:63], 0\n\t"                              \
                     "v_mov_b32 v76, 5\n\tv_mov_b32 v77, 6\n\tv_mov_b32 v78, 7\n\tv_mov_b32 v79, 8\n\t"     \
                     "v_mfma_i32_16x16x64_i8 " D3 ", v[44:47], v[56:59], 0\n\t"                                \
                     OVW                                                                                      \
                     "s_waitcnt lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"               \
                     "v_add3_u32 %0, v64, v68, v42\n\tv_add3_u32 %1, v65, v69, v43\n\t"                         \
                     "v_add3_u32 %2, v66, v70, v44\n\tv_add3_u32 %3, v67, v71, v45\n\ts_nop 4"                  \
                     : "=v"(r.x), "=v"(r.y), "=v"(r.z), "=v"(r.w)                                             \
                     : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(lds_addr) \
                     : "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v56", "v57", "v58", "v59", "v60",  \
                       "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73",  \
                       "v74", "v75", "v76", "v77", "v78", "v79", "memory");                                   \
        return r;                                                                                            \
    }
// (the D elsewhere forms copy their D into v[42:45] so the folds compare the same elements)
#define D3_OVER "v[42:45]"
#define D3_ELSE "v[42:45]"
#define OVW12 "ds_read_b128 v[46:49], %12\n\t"
#define OVW12_16 "s_nop 7\n\ts_nop 7\n\tds_read_b128 v[46:49], %12\n\t"
#define OVW12_OFF "ds_read_b128 v[48:51], %12\n\t"
MFMA3_LDS(m3_lds, D3_OVER, OVW12)
MFMA3_LDS(m3_lds16, D3_OVER, OVW12_16)
MFMA3_LDS(m3_lds_off, D3_OVER, OVW12_OFF)
MFMA3_LDS(m3_none, D3_OVER, "")

__global__ __launch_bounds__(256) void probe_war12(int variant, int iters, const double* __restrict__ da,
                                                  const double* __restrict__ db, unsigned long long* __restrict__ bad,
                                                  unsigned long long* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) unsigned lds[256 * 4];
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < 4; k++) lds[threadIdx.x * 4 + k] = 0xdeadbeefu ^ (threadIdx.x * 4 + k) * 0x9e3779b9u;
    __syncthreads();
    const unsigned addr = (unsigned)(threadIdx.x * 16);
    unsigned long long nb = 0, acc = 0;
    for (int it = 0; it < iters; it++) {
        const int i = (t * 7 + it * 131) & 4095;
        const unsigned long long ab = __double_as_longlong(da[i]), bb = __double_as_longlong(db[i]);
        const i4v A = {(int)ab, (int)(ab >> 32), (int)(ab * 3), (int)(bb ^ ab)};
        const i4v B = {(int)bb, (int)(bb >> 32), (int)(bb * 5), (int)(ab + bb)};
        const i4v r = variant == 0 ? m3_lds(A, B, addr) : variant == 1 ? m3_lds16(A, B, addr) : m3_lds_off(A, B, addr);
        const i4v e = m3_none(A, B, addr);
        nb += (r.x != e.x) + (r.y != e.y) + (r.z != e.z) + (r.w != e.w);
        acc += (unsigned)r.x;
    }
    if (nb) atomicAdd(bad, nb);
    sink[t & 1023] = acc;
}

// VALU write then DPP read of the written VGPR (quad_perm [1,0,3,2]), 0 or 4 wait states
__device__ __forceinline__ unsigned dpp_after_write(unsigned v, int nop) {
    unsigned r;
    if (nop)
        asm volatile("v_add_u32 v56, %1, 1\n\ts_nop 4\n\tv_mov_b32_dpp %0, v56 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\ts_nop 4"
                     : "=v"(r) : "v"(v) : "v56");
    else
        asm volatile("v_add_u32 v56, %1, 1\n\tv_mov_b32_dpp %0, v56 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\ts_nop 4"
                     : "=v"(r) : "v"(v) : "v56");
    return r;
}

__global__ __launch_bounds__(256) void probe_war(int variant, int iters, const double* __restrict__ da,
                                                const double* __restrict__ db, unsigned long long* __restrict__ bad,
                                                unsigned long long* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) unsigned lds[256 * 4];
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < 4; k++) lds[threadIdx.x * 4 + k] = 0xdeadbeefu ^ (threadIdx.x * 4 + k) * 0x9e3779b9u;
    __syncthreads();
    const unsigned addr = (unsigned)(threadIdx.x * 16);
    unsigned long long nb = 0, acc = 0;
    for (int it = 0; it < iters; it++) {
        const int i = (t * 7 + it * 131) & 4095;
        const unsigned long long ab = __double_as_longlong(da[i]), bb = __double_as_longlong(db[i]);
        const i4v A = {(int)ab, (int)(ab >> 32), (int)(ab * 3), (int)(bb ^ ab)};
        const i4v B = {(int)bb, (int)(bb >> 32), (int)(bb * 5), (int)(ab + bb)};
        int r;
        switch (variant) {
            case 0: r = war_lds_p0(A, B, addr); break;
            case 1: r = war_lds_p1(A, B, addr); break;
            case 2: r = war_lds_p3(A, B, addr); break;
            case 3: r = war_lds_p3k4(A, B, addr); break;
            case 4: r = war_lds_p3k16(A, B, addr); break;
            default: r = war_valu_p3(A, B, addr); break;
        }
        const int e = war_none_p3(A, B, addr);
        nb += r != e;
        acc += (unsigned)r;
    }
    if (nb) atomicAdd(bad, nb);
    sink[t & 1023] = acc;
}

__global__ __launch_bounds__(256) void probe(int test, int nop, int iters, const double* __restrict__ da,
                                            const double* __restrict__ db, const double* __restrict__ dc,
                                            unsigned long long* __restrict__ bad, unsigned long long* __restrict__ sink) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    unsigned long long nb = 0, acc = 0;
    for (int it = 0; it < iters; it++) {
        const int i = (t * 7 + it * 131) & 4095;
        const double a = da[i], b = db[i], c = dc[i];
        if (test == 1) {
            const unsigned long long cb = __double_as_longlong(c);
            const double r = fmac_pair_acc(a, b, (unsigned)cb, (unsigned)(cb >> 32), nop);
            const double e = fma(a, b, c);
            nb += __double_as_longlong(r) != __double_as_longlong(e);
            acc += __double_as_longlong(r);
        } else if (test == 2) {
            const unsigned long long ab = __double_as_longlong(a);
            const double r = fmac_pair_src(c, b, (unsigned)ab, (unsigned)(ab >> 32), nop);
            const double e = fma(a, b, c);
            nb += __double_as_longlong(r) != __double_as_longlong(e);
            acc += __double_as_longlong(r);
        } else if (test == 3) {
            const unsigned long long ab = __double_as_longlong(a), bb = __double_as_longlong(b);
            const i4v A = {(int)ab, (int)(ab >> 32), (int)(ab * 3), (int)(bb ^ ab)};
            const i4v B = {(int)bb, (int)(bb >> 32), (int)(bb * 5), (int)(ab + bb)};
            const i4v r1 = mfma_da(A, B, nop ? 0 : 1);   // nop != 0: the non-overlapping reference form
            const i4v r0 = mfma_da(A, B, 0);
            nb += r1.x != r0.x;
            acc += (unsigned)r1.x;
        } else if (test == 5) {
            const unsigned long long ab = __double_as_longlong(a), bb = __double_as_longlong(b);
            const i4v A = {(int)ab, (int)(ab >> 32), (int)(ab * 3), (int)(bb ^ ab)};
            const i4v B = {(int)bb, (int)(bb >> 32), (int)(bb * 5), (int)(ab + bb)};
            const int r = mfma_raw(nop, A, B), e = mfma_raw(20, A, B);
            nb += r != e;
            acc += (unsigned)r;
        } else if (test == 6 || test == 7) {
            const unsigned long long ab = __double_as_longlong(a), bb = __double_as_longlong(b);
            const i4v A = {(int)ab, (int)(ab >> 32), (int)(ab * 3), (int)(bb ^ ab)};
            const i4v B = {(int)bb, (int)(bb >> 32), (int)(bb * 5), (int)(ab + bb)};
            const int r = mfma_war(test == 7, nop, A, B), e = mfma_war(test == 7, 20, A, B);
            nb += r != e;
            acc += (unsigned)r;
        } else if (test == 8 || test == 9) {
            const unsigned long long ab = __double_as_longlong(a), bb = __double_as_longlong(b);
            const i4v A = {(int)ab, (int)(ab >> 32), (int)(ab * 3), (int)(bb ^ ab)};
            const i4v B = {(int)bb, (int)(bb >> 32), (int)(bb * 5), (int)(ab + bb)};
            const i4v r = test == 8 ? mfma_part_a(A, B) : mfma_part_b(A, B);
            const i4v e = mfma_part_none(A, B);
            nb += (r.x != e.x) + (r.y != e.y) + (r.z != e.z) + (r.w != e.w);
            acc += (unsigned)r.x;
        } else if (test == 4) {
            const unsigned v = (unsigned)__double_as_longlong(a) + (unsigned)it;
            const unsigned r = dpp_after_write(v, nop);
            const unsigned e = __shfl_xor(v + 1u, 1);
            nb += r != e;
            acc += r;
        }
    }
    if (nb) atomicAdd(bad, nb);
    sink[t & 1023] = acc;   // keep the work
    (void)lane;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    std::vector<double> a(4096), b(4096), c(4096);
    srand(1);
    for (int i = 0; i < 4096; i++) {
        a[i] = (rand() / (double)RAND_MAX - 0.5) * 1e3;
        b[i] = (rand() / (double)RAND_MAX - 0.5) * 1e-2;
        c[i] = (rand() / (double)RAND_MAX - 0.5) * 7;
    }
    double *da, *db, *dc;
    unsigned long long *bad, *sink;
    hipMalloc(&da, 4096 * 8); hipMalloc(&db, 4096 * 8); hipMalloc(&dc, 4096 * 8);
    hipMalloc(&bad, 8); hipMalloc(&sink, 1024 * 8);
    hipMemcpy(da, a.data(), 4096 * 8, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), 4096 * 8, hipMemcpyHostToDevice);
    hipMemcpy(dc, c.data(), 4096 * 8, hipMemcpyHostToDevice);
    const char* names[] = {"", "T1 v_mov x2 -> v_fmac_f64 acc", "T2 v_mov x2 -> v_fmac_f64 src0",
                           "T3 mfma i8 D==A (vs D elsewhere)", "T4 VALU -> DPP read (positive control)"};
    const int blocks = 256 * 8;   // 8 workgroups of 4 waves per CU
    for (int test = 1; test <= 4; test++)
        for (int nop = 0; nop <= 1; nop++) {
            hipMemset(bad, 0, 8);
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, test, nop, iters, da, db, dc, bad, sink);
            if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
            unsigned long long nb = 0;
            hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
            printf("%-42s %s: %llu mismatches of %llu\n", names[test], nop ? (test == 3 ? "reference" : "4 nops ") : "0 nops ",
                   nb, (unsigned long long)blocks * 256 * iters);
        }
    const int ks[] = {0, 2, 4, 6, 8, 9, 10, 11, 12, 14, 16};
    for (int k : ks) {
        hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, 5, k, iters / 4, da, db, dc, bad, sink);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
        unsigned long long nb = 0;
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        printf("T5 mfma i8 16x16x64 -> VALU read after %2d wait states: %llu mismatches of %llu\n", k, nb,
               (unsigned long long)blocks * 256 * (iters / 4));
    }
    for (int test = 8; test <= 9; test++) {
        hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, test, 0, iters, da, db, dc, bad, sink);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
        unsigned long long nb = 0;
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        printf("T%d mfma i8 16x16x64, D partially over Src%s: %llu element mismatches of %llu\n", test, test == 8 ? "A" : "B",
               nb, 4ull * blocks * 256 * iters);
    }
    const char* wn[] = {"T10 LDS load over SrcA right after the MFMA, no MFMA ahead",
                        "T10 LDS load over SrcA right after the MFMA, 1 MFMA ahead",
                        "T10 LDS load over SrcA right after the MFMA, 3 MFMAs ahead",
                        "T10 LDS load over SrcA 4 wait states after, 3 MFMAs ahead",
                        "T10 LDS load over SrcA 16 wait states after, 3 MFMAs ahead",
                        "T11 VALU write over SrcA right after the MFMA, 3 MFMAs ahead"};
    for (int v = 0; v < 6; v++) {
        hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(probe_war, dim3(blocks), dim3(256), 0, 0, v, iters, da, db, bad, sink);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
        unsigned long long nb = 0;
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        printf("%-64s: %llu mismatches of %llu\n", wn[v], nb, (unsigned long long)blocks * 256 * iters);
    }
    const char* wn12[] = {"T12 angold: 3 MFMAs on one SrcA, D3 over its first half, LDS load over the rest",
                          "T12 the same, the LDS load 16 wait states later",
                          "T12 the same, the LDS load into registers no MFMA reads"};
    for (int v = 0; v < 3; v++) {
        hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(probe_war12, dim3(blocks), dim3(256), 0, 0, v, iters, da, db, bad, sink);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
        unsigned long long nb = 0;
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        printf("%-84s: %llu element mismatches of %llu\n", wn12[v], nb, 4ull * blocks * 256 * iters);
    }
    const int kw[] = {0, 2, 4, 8, 12};
    for (int test = 6; test <= 7; test++)
        for (int k : kw) {
            hipMemset(bad, 0, 8);
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, test, k, iters / 4, da, db, dc, bad, sink);
            if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
            unsigned long long nb = 0;
            hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
            printf("T%d mfma i8 16x16x64, VALU overwrites Src%s after %2d wait states: %llu mismatches of %llu\n", test,
                   test == 6 ? "A" : "C", k, nb, (unsigned long long)blocks * 256 * (iters / 4));
        }
    return 0;
}
