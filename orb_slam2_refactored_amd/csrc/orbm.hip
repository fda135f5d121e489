// orbm.hip — ORBmatcher Hamming kernels for gfx950.
//
//  * hamming_top2_mfma_kernel: brute-force best / second-best over all pairs with the reference's
//    scan semantics (SearchByBoW inner loop, src/ORBmatcher.cc:477-498) as an int8 MFMA
//    contraction: Hamming = |a| + |b| - 2<a, b> on 0/1-expanded bits (DescriptorDistance,
//    :1449-1457), exact in int32; running top-2 kept as packed (distance, index) keys.
//  * triangulation_kernel: SearchForTriangulation (:768-866) — per query, the last candidate
//    with the minimum distance <= TH_LOW that passes the epipole and epipolar gates
//    (CheckDistEpipolarLine :384-404).  `matched2` is never set by the reference (§0.5), so
//    queries are independent and map one per lane.
#include <cstring>
#include <vector>

#include "common.h"
#include "qt_sort.h"

namespace orbamd {

// ---------------------------------------------------------------------------------------------
// Brute-force top-2 on the matrix cores.  For 0/1 bit vectors, Hamming(a, b) = |a| + |b| -
// 2<a, b>, and <a, b> over the 256 bits is an exact int32 dot product of bytes: bits are expanded
// to 0/1 bytes in registers and fed to v_mfma_i32_16x16x64_i8 (4 k-steps per 256 bits).  Any k
// permutation applied identically to the A and B fragments leaves the dot product unchanged, so
// lane l (group g = l >> 4) simply takes descriptor bytes 8g..8g+7 and k-step s their bits
// 16s..16s+15.  A's bits are expanded to int8 0 / -128, B's to 0 / 2, and the accumulator starts
// at 128 (|b| + 256) + t for column tile t of a 2048-column chunk, so the MFMA yields the key
// 128 S + t with S = d - |a| + 256 in [0, 512] directly (a lane holds one column class, so t is
// its column).  The running best key is the minimum (lowest j on equal d, as the reference's
// strict-< scan) and the running second key the second order statistic.  Chunk keys become global
// keys S << 16 | j for the cross-lane merge; after it d = S - 256 + |a|; keys with d >= 256
// (d == 256 and the padding columns) never displace a real candidate and are mapped back to
// (256, -1), which is the reference's bestDist = 256 / bestIdx = -1 initialisation.
typedef int i4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i4v expand16(uint32_t b) {   // bit k of b -> byte k (0 / 1)
    i4v r;
    r.x = (int)(((b & 0xfu) * 0x00204081u) & 0x01010101u);
    r.y = (int)((((b >> 4) & 0xfu) * 0x00204081u) & 0x01010101u);
    r.z = (int)((((b >> 8) & 0xfu) * 0x00204081u) & 0x01010101u);
    r.w = (int)((((b >> 12) & 0xfu) * 0x00204081u) & 0x01010101u);
    return r;
}

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// The same median, ordered after `dep`.  `key` is an MFMA result: the compiler's hazard recognizer
// does not see reads inside inline asm, so the asm must come after a compiler-generated read of
// the same register (the `min` that produces `dep`), which carries the MFMA -> VALU wait states.
__device__ __forceinline__ uint32_t umed3_after(uint32_t a, uint32_t key, uint32_t c, uint32_t dep) {
    uint32_t r;
    asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(key), "v"(c), "v"(dep));
    return r;
}

__device__ __forceinline__ uint32_t chunk16(uint2 v, int s) {
    return ((s < 2 ? v.x : v.y) >> (16 * (s & 1))) & 0xffffu;
}

__device__ __forceinline__ int popc_row(const uint8_t* r) {
    const uint4 a = reinterpret_cast<const uint4*>(r)[0], b = reinterpret_cast<const uint4*>(r)[1];
    return __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w) + __popc(b.x) + __popc(b.y) + __popc(b.z) +
           __popc(b.w);
}

#ifndef MM_RT_DEF
#define MM_RT_DEF 2
#endif
constexpr int MM_RT = MM_RT_DEF;          // 16-row tiles per wavefront
constexpr int MM_WROWS = 16 * MM_RT;      // query rows per wavefront
constexpr int MM_ROWS = 4 * MM_WROWS;     // query rows per workgroup (4 wavefronts)
constexpr int MM_CHUNK = 2048;                // columns per chunk key range (128 tiles of 16)

template <bool MULTI>   // MULTI: more than MM_CHUNK columns (chunked, global keys kept across chunks)
__global__ __launch_bounds__(256) void hamming_top2_mfma_kernel(
    const uint8_t* __restrict__ A, const int32_t* __restrict__ nA_arr, int nA_fixed, int strideA,
    const uint8_t* __restrict__ B, const int32_t* __restrict__ nB_arr, int nB_fixed, int strideB,
    const int32_t* __restrict__ pair_b, float nnratio, int th_low, int32_t* __restrict__ best_idx,
    int32_t* __restrict__ best, int32_t* __restrict__ second, int32_t* __restrict__ match) {
    extern __shared__ __attribute__((aligned(16))) int mm_sm[];   // pa[MM_ROWS] | pb[nB padded to 32] | expanded B [2][2][4][64]
    int* s_pa = mm_sm;
    int* s_pb = mm_sm + MM_ROWS;
    const int p = blockIdx.y;
    const int q = pair_b ? pair_b[p] : p;
    const int nA = nA_arr ? nA_arr[p] : nA_fixed;
    const int nB = nB_arr ? nB_arr[q] : nB_fixed;
    const int row_base = blockIdx.x * MM_ROWS;
    if (row_base >= nA) return;   // block-uniform
    const uint8_t* Ap = A + (long long)p * strideA * 32;
    const uint8_t* Bp = B + (long long)q * strideB * 32;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c16 = lane & 15, g = lane >> 4;
    const int nBt = (nB + 31) & ~31;   // whole pairs of 16-column tiles
    const bool live = __builtin_amdgcn_readfirstlane(row_base + MM_WROWS * w < nA ? 1 : 0) != 0;
    for (int j = tid; j < nBt; j += blockDim.x) s_pb[j] = 128 * ((j < nB ? popc_row(Bp + (long long)j * 32) : 256) + 256);
    {
        const int row = row_base + tid;
        if (tid < MM_ROWS) s_pa[tid] = row < nA ? popc_row(Ap + (long long)row * 32) : 0;
    }
    // A fragments: tile rt rows row_base + 64w + 16rt + c16, bytes 8g..8g+7
    i4v af[MM_RT][4];
#pragma unroll
    for (int rt = 0; rt < MM_RT; rt++) {
        const int row = min(row_base + MM_WROWS * w + 16 * rt + c16, nA - 1);
        const uint2 v = *reinterpret_cast<const uint2*>(Ap + (long long)row * 32 + 8 * g);
#pragma unroll
        for (int s2 = 0; s2 < 4; s2++) af[rt][s2] = expand16(chunk16(v, s2)) * 0x80;   // bit -> int8 0 / -128
    }
    __syncthreads();
    // Inside a chunk of 128 tiles the MFMA itself yields the chunk key 128 S + t (t = tile in the
    // chunk, S = |b| + 256 - 2<a, b> = d - |a| + 256 in [0, 512]): A is expanded to 0 / -128, B
    // to 0 / 2, and the accumulator starts at 128 (|b| + 256) + t.  A lane holds one column class
    // c16 (j = chunk base + 16 t + c16), so the chunk key orders the lane's candidates by (S, j)
    // with no per-value key build.  With MULTI, global keys (S << 16 | j) carry the top-2 across
    // chunks.
    uint32_t bk[MM_RT][4], sk[MM_RT][4], lb[MM_RT][4], ls[MM_RT][4];
#pragma unroll
    for (int rt = 0; rt < MM_RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) bk[rt][r] = sk[rt][r] = 0xffffffffu;
    // Column tiles of 16, consumed in pairs.  The 0/1 byte expansion of a tile pair is shared by the
    // 4 wavefronts (all of them need the same columns): wavefront w expands k-step w of both tiles
    // of the next pair into an LDS double buffer while this pair is consumed, one barrier per pair.
    i4v* xb = reinterpret_cast<i4v*>(mm_sm + ((MM_ROWS + nBt + 16 + 3) & ~3));   // [2][2][4][64]
    auto ldb = [&](int jj) -> uint2 {
        return jj < nB ? *reinterpret_cast<const uint2*>(Bp + (long long)jj * 32 + 8 * g) : make_uint2(0, 0);
    };
    {
        const uint2 b0 = ldb(c16), b1 = ldb(16 + c16);
        xb[(0 * 4 + w) * 64 + lane] = expand16(chunk16(b0, w)) * 2;
        xb[(1 * 4 + w) * 64 + lane] = expand16(chunk16(b1, w)) * 2;
    }
    uint2 bn0 = ldb(32 + c16), bn1 = ldb(48 + c16);
    __syncthreads();
    for (int c0 = 0; c0 < nB; c0 += MM_CHUNK) {
#pragma unroll
        for (int rt = 0; rt < MM_RT; rt++)
#pragma unroll
            for (int r = 0; r < 4; r++) lb[rt][r] = ls[rt][r] = 0xffffffffu;
        const int c1 = min(nB, c0 + MM_CHUNK);
        for (int j0 = c0; j0 < c1; j0 += 32) {
            const int cur = (j0 >> 5) & 1;
            if (j0 + 32 < nB) {   // block-uniform
                xb[(((cur ^ 1) * 2 + 0) * 4 + w) * 64 + lane] = expand16(chunk16(bn0, w)) * 2;   // bit -> 0 / 2
                xb[(((cur ^ 1) * 2 + 1) * 4 + w) * 64 + lane] = expand16(chunk16(bn1, w)) * 2;
                bn0 = ldb(j0 + 64 + c16);
                bn1 = ldb(j0 + 80 + c16);
            }
            const int t = (j0 - c0) >> 4;
            // a wavefront whose rows all lie past nA (the last workgroup of a frame is mostly
            // empty) only expands its share of the next pair
#pragma unroll
            for (int tt = 0; tt < 2; tt++) {
                if (!live) break;   // wavefront-uniform
                const int ci = s_pb[j0 + 16 * tt + c16] + t + tt;
                const i4v cinit = {ci, ci, ci, ci};
                i4v bf[4];
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) bf[s2] = xb[((cur * 2 + tt) * 4 + s2) * 64 + lane];
#pragma unroll
                for (int rt = 0; rt < MM_RT; rt++) {
                    i4v acc = cinit;
#pragma unroll
                    for (int s2 = 0; s2 < 4; s2++)
                        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[rt][s2], bf[s2], acc, 0, 0, 0);
                    const int sv[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t key = (uint32_t)sv[r];
                        // lb <= ls always, so the new second order statistic min(ls, max(lb, key))
                        // is the median of the three
                        const uint32_t nb = min(lb[rt][r], key);
                        ls[rt][r] = umed3_after(lb[rt][r], key, ls[rt][r], nb);
                        lb[rt][r] = nb;
                    }
                }
            }
            __syncthreads();   // pair expanded into `cur ^ 1`; buffer `cur` free for the pair after
        }
        // the chunk's top-2 as global keys
        const uint32_t jb = (uint32_t)(c0 + c16);
#pragma unroll
        for (int rt = 0; rt < MM_RT; rt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                auto glob = [&](uint32_t k) {
                    return k == 0xffffffffu ? k : ((k >> 7) << 16) | (jb + 16 * (k & 127u));
                };
                const uint32_t b2 = glob(lb[rt][r]), s2v = glob(ls[rt][r]);
                if (MULTI) {
                    sk[rt][r] = min(min(sk[rt][r], s2v), max(bk[rt][r], b2));
                    bk[rt][r] = min(bk[rt][r], b2);
                } else {
                    bk[rt][r] = b2;
                    sk[rt][r] = s2v;
                }
            }
        if (!MULTI) break;
    }
    // merge the 16 column classes of each row (lanes with the same g)
#pragma unroll
    for (int rt = 0; rt < MM_RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint32_t b1 = bk[rt][r], s1 = sk[rt][r];
            // top-2 merge is associative and commutative, so the 16 lanes of a row combine in any
            // tree: DPP quad_perm [1,0,3,2], [2,3,0,1], then row_ror 4 and 8
            auto merge = [&](uint32_t b2, uint32_t s2v) {
                s1 = min(min(s1, s2v), max(b1, b2));
                b1 = min(b1, b2);
            };
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0xB1, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0xB1, 0xf, 0xf, false));
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0x4E, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0x4E, 0xf, 0xf, false));
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0x124, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0x124, 0xf, 0xf, false));
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0x128, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0x128, 0xf, 0xf, false));
            const int row = row_base + MM_WROWS * w + 16 * rt + 4 * g + r;
            if (c16 == 0 && row < nA) {
                const int pa = s_pa[MM_WROWS * w + 16 * rt + 4 * g + r];
                const int bdr = (int)(b1 >> 16) - 256 + pa, sdr = (int)(s1 >> 16) - 256 + pa;
                const int bd = bdr >= 256 ? 256 : bdr;
                const int bi = bdr >= 256 ? -1 : (int)(b1 & 0xffffu);
                const int sd = sdr >= 256 ? 256 : sdr;
                const long long o = (long long)p * strideA + row;
                if (best_idx) best_idx[o] = bi;
                if (best) best[o] = bd;
                if (second) second[o] = sd;
                if (match) match[o] = (bd <= th_low && (float)bd < nnratio * (float)sd) ? bi : -1;
            }
        }
}

// The same top-2 on the block-scaled FP4 matrix path (v_mfma_scale_f32_16x16x128_f8f6f4, e2m1
// operands: K = 128 per instruction, twice the i8 form's K at the same issue cost, and half the
// expanded bytes).  A bit becomes a nibble: A's 1 -> -4 with block scale 2^6 (-256), B's 1 -> 1.0
// with scale 2^0, so a common bit contributes -256 and, with the f32 accumulator started at
// 128 (|b| + 256) + t (exact: every value is an integer below 2^17), the MFMA again yields the chunk
// key 128 S + t, now as an f32.  The keys are non-negative, so their bit patterns order as the
// values: the running min / median run on the raw bits, converted to integers once per chunk.
// Lane group g takes descriptor bytes 8g..8g+7; k-step m its bits 32m..32m+31 (any k permutation
// shared by A and B leaves the dot product unchanged).
typedef int i8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t spread8(uint32_t b) {   // bit i of the low byte -> bit 4i
    uint32_t x = b & 0xffu;
    x = (x | (x << 12)) & 0x000f000fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x;
}
__device__ __forceinline__ i4v expand32_nib(uint32_t b, uint32_t nib) {   // bit k of b -> nibble k (0 / nib)
    i4v r;
    r.x = (int)(spread8(b) * nib);
    r.y = (int)(spread8(b >> 8) * nib);
    r.z = (int)(spread8(b >> 16) * nib);
    r.w = (int)(spread8(b >> 24) * nib);
    return r;
}
constexpr uint32_t FP4_NEG4 = 0xEu, FP4_ONE = 0x2u;    // e2m1: -4.0, 1.0
constexpr int FP4_SCALE_A = 0x85858585, FP4_SCALE_B = 0x7f7f7f7f;   // e8m0: 2^6, 2^0

__device__ __forceinline__ f4v mfma_fp4(i4v a, i4v b, f4v c) {
    const i8v a8 = __builtin_shufflevector(a, a, 0, 1, 2, 3, -1, -1, -1, -1);
    const i8v b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, -1, -1, -1, -1);
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, c, 4, 4, 0, FP4_SCALE_A, 0, FP4_SCALE_B);
}

#ifndef FP_RT_DEF
#define FP_RT_DEF 3
#endif
constexpr int FP_RT = FP_RT_DEF;       // 16-row tiles per wavefront (89 VGPRs: 5 wavefronts per SIMD; 4 tiles: 114, 4)
constexpr int FP_WROWS = 16 * FP_RT;
constexpr int FP_ROWS = 4 * FP_WROWS;
template <bool MULTI>
__global__ __launch_bounds__(256) void hamming_top2_fp4_kernel(
    const uint8_t* __restrict__ A, const int32_t* __restrict__ nA_arr, int nA_fixed, int strideA,
    const uint8_t* __restrict__ B, const int32_t* __restrict__ nB_arr, int nB_fixed, int strideB,
    const int32_t* __restrict__ pair_b, float nnratio, int th_low, int32_t* __restrict__ best_idx,
    int32_t* __restrict__ best, int32_t* __restrict__ second, int32_t* __restrict__ match) {
    extern __shared__ __attribute__((aligned(16))) int mm_sm[];   // pa[FP_ROWS] | pb[nB padded to 32] | expanded B [2][2][2][64]
    int* s_pa = mm_sm;
    int* s_pb = mm_sm + FP_ROWS;
    const int p = blockIdx.y;
    const int q = pair_b ? pair_b[p] : p;
    const int nA = nA_arr ? nA_arr[p] : nA_fixed;
    const int nB = nB_arr ? nB_arr[q] : nB_fixed;
    const int row_base = blockIdx.x * FP_ROWS;
    if (row_base >= nA) return;   // block-uniform
    const uint8_t* Ap = A + (long long)p * strideA * 32;
    const uint8_t* Bp = B + (long long)q * strideB * 32;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c16 = lane & 15, g = lane >> 4;
    const int nBt = (nB + 31) & ~31;   // whole pairs of 16-column tiles
    const bool live = __builtin_amdgcn_readfirstlane(row_base + FP_WROWS * w < nA ? 1 : 0) != 0;
    for (int j = tid; j < nBt; j += blockDim.x) s_pb[j] = 128 * ((j < nB ? popc_row(Bp + (long long)j * 32) : 256) + 256);
    {
        const int row = row_base + tid;
        if (tid < FP_ROWS) s_pa[tid] = row < nA ? popc_row(Ap + (long long)row * 32) : 0;
    }
    i4v af[FP_RT][2];
#pragma unroll
    for (int rt = 0; rt < FP_RT; rt++) {
        const int row = min(row_base + FP_WROWS * w + 16 * rt + c16, nA - 1);
        const uint2 v = *reinterpret_cast<const uint2*>(Ap + (long long)row * 32 + 8 * g);
        af[rt][0] = expand32_nib(v.x, FP4_NEG4);
        af[rt][1] = expand32_nib(v.y, FP4_NEG4);
    }
    __syncthreads();
    uint32_t bk[FP_RT][4], sk[FP_RT][4], lb[FP_RT][4], ls[FP_RT][4];
#pragma unroll
    for (int rt = 0; rt < FP_RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) bk[rt][r] = sk[rt][r] = 0xffffffffu;
    // Column tiles of 16, consumed in pairs.  Wavefront w expands k-step (w & 1) of tile (w >> 1) of
    // the next pair into an LDS double buffer while this pair is consumed, one barrier per pair.
    i4v* xb = reinterpret_cast<i4v*>(mm_sm + ((FP_ROWS + nBt + 16 + 3) & ~3));   // [2][2][2][64]
    const int xt = w >> 1, xs = w & 1;
    auto ldb = [&](int jj) -> uint32_t {
        return jj < nB ? *reinterpret_cast<const uint32_t*>(Bp + (long long)jj * 32 + 8 * g + 4 * xs) : 0u;
    };
    xb[((0 * 2 + xt) * 2 + xs) * 64 + lane] = expand32_nib(ldb(16 * xt + c16), FP4_ONE);
    uint32_t bn = ldb(32 + 16 * xt + c16);
    __syncthreads();
    for (int c0 = 0; c0 < nB; c0 += MM_CHUNK) {
#pragma unroll
        for (int rt = 0; rt < FP_RT; rt++)
#pragma unroll
            for (int r = 0; r < 4; r++) lb[rt][r] = ls[rt][r] = 0xffffffffu;
        const int c1 = min(nB, c0 + MM_CHUNK);
        for (int j0 = c0; j0 < c1; j0 += 32) {
            const int cur = (j0 >> 5) & 1;
            if (j0 + 32 < nB) {   // block-uniform
                xb[(((cur ^ 1) * 2 + xt) * 2 + xs) * 64 + lane] = expand32_nib(bn, FP4_ONE);
                bn = ldb(j0 + 64 + 16 * xt + c16);
            }
            const int t = (j0 - c0) >> 4;
#pragma unroll
            for (int tt = 0; tt < 2; tt++) {
                if (!live) break;   // wavefront-uniform
                const float ci = (float)(s_pb[j0 + 16 * tt + c16] + t + tt);
                const f4v cinit = {ci, ci, ci, ci};
                const i4v b0 = xb[((cur * 2 + tt) * 2 + 0) * 64 + lane];
                const i4v b1 = xb[((cur * 2 + tt) * 2 + 1) * 64 + lane];
#pragma unroll
                for (int rt = 0; rt < FP_RT; rt++) {
                    f4v acc = mfma_fp4(af[rt][0], b0, cinit);
                    acc = mfma_fp4(af[rt][1], b1, acc);
                    const float sv[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t key = __float_as_uint(sv[r]);   // >= 0: bits order as values
                        const uint32_t nb = min(lb[rt][r], key);
                        ls[rt][r] = umed3_after(lb[rt][r], key, ls[rt][r], nb);
                        lb[rt][r] = nb;
                    }
                }
            }
            __syncthreads();   // pair expanded into `cur ^ 1`; buffer `cur` free for the pair after
        }
        // the chunk's top-2 as global keys (chunk keys back to integers first)
        const uint32_t jb = (uint32_t)(c0 + c16);
#pragma unroll
        for (int rt = 0; rt < FP_RT; rt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                auto glob = [&](uint32_t kb) {
                    if (kb == 0xffffffffu) return kb;
                    const uint32_t k = (uint32_t)__uint_as_float(kb);
                    return ((k >> 7) << 16) | (jb + 16 * (k & 127u));
                };
                const uint32_t b2 = glob(lb[rt][r]), s2v = glob(ls[rt][r]);
                if (MULTI) {
                    sk[rt][r] = min(min(sk[rt][r], s2v), max(bk[rt][r], b2));
                    bk[rt][r] = min(bk[rt][r], b2);
                } else {
                    bk[rt][r] = b2;
                    sk[rt][r] = s2v;
                }
            }
        if (!MULTI) break;
    }
#pragma unroll
    for (int rt = 0; rt < FP_RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint32_t b1 = bk[rt][r], s1 = sk[rt][r];
            auto merge = [&](uint32_t b2, uint32_t s2v) {
                s1 = min(min(s1, s2v), max(b1, b2));
                b1 = min(b1, b2);
            };
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0xB1, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0xB1, 0xf, 0xf, false));
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0x4E, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0x4E, 0xf, 0xf, false));
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0x124, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0x124, 0xf, 0xf, false));
            merge((uint32_t)__builtin_amdgcn_update_dpp(0, (int)b1, 0x128, 0xf, 0xf, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0x128, 0xf, 0xf, false));
            const int row = row_base + FP_WROWS * w + 16 * rt + 4 * g + r;
            if (c16 == 0 && row < nA) {
                const int pa = s_pa[FP_WROWS * w + 16 * rt + 4 * g + r];
                const int bdr = (int)(b1 >> 16) - 256 + pa, sdr = (int)(s1 >> 16) - 256 + pa;
                const int bd = bdr >= 256 ? 256 : bdr;
                const int bi = bdr >= 256 ? -1 : (int)(b1 & 0xffffu);
                const int sd = sdr >= 256 ? 256 : sdr;
                const long long o = (long long)p * strideA + row;
                if (best_idx) best_idx[o] = bi;
                if (best) best[o] = bd;
                if (second) second[o] = sd;
                if (match) match[o] = (bd <= th_low && (float)bd < nnratio * (float)sd) ? bi : -1;
            }
        }
}

static int mm_fp4() {   // ORBM_FP4=0 selects the i8 kernel (read per launch: tests switch it)
    const char* e = getenv("ORBM_FP4");
    return e ? atoi(e) : 1;
}

static int tri_split() {   // kf2 column parts per query block of the matrix-core path (ORBM_TRI_SPLIT)
    const char* e = getenv("ORBM_TRI_SPLIT");
    return e ? std::max(1, std::min(8, atoi(e))) : 1;
}

static int tri_mm() {   // ORBM_TRI_MM=0 selects the per-lane scan for the all-pairs triangulation search
    const char* e = getenv("ORBM_TRI_MM");
    return e ? atoi(e) : 1;
}

static void launch_top2(const uint8_t* A, const int32_t* nA_arr, int nA_fixed, int strideA, const uint8_t* B,
                        const int32_t* nB_arr, int nB_fixed, int strideB, const int32_t* pair_b, int n_pairs,
                        float nnratio, int th_low, int32_t* bi, int32_t* bd, int32_t* sd, int32_t* mt,
                        hipStream_t st) {
    const bool fp4 = mm_fp4() != 0;
    const int rows = fp4 ? FP_ROWS : MM_ROWS;
    const size_t lds = (size_t)(((rows + ((strideB + 31) & ~31) + 16 + 3) & ~3) + 2 * 2 * (fp4 ? 2 : 4) * 64 * 4) * sizeof(int);
    auto kern = fp4 ? (strideB <= MM_CHUNK ? hamming_top2_fp4_kernel<false> : hamming_top2_fp4_kernel<true>)
                    : (strideB <= MM_CHUNK ? hamming_top2_mfma_kernel<false> : hamming_top2_mfma_kernel<true>);
    hipLaunchKernelGGL(kern, dim3((unsigned)((strideA + rows - 1) / rows), (unsigned)n_pairs),
                       dim3(256), lds, st, A, nA_arr, nA_fixed, strideA, B, nB_arr, nB_fixed, strideB, pair_b,
                       nnratio, th_low, bi, bd, sd, mt);
}

// ---------------------------------------------------------------------------------------------
// CheckOrientation (src/ORBmatcher.cc:249-309) on a query-indexed brute-force result, applied the
// way SearchForInitialization applies it (:676-686): matchIds = (bestIdx2, idx1) for every accepted
// query in ascending idx1, keypoints1 = frame B, keypoints2 = frame A, so a match's bin is
// diffToBin(angleB[j] - angleA[i]) and erasing sets match[i] = -1.  The histogram's 30 bins are
// sorted by size with libstdc++'s unstable std::sort (qt_sort.h reproduces its move sequence, so
// equal-size bins land where the reference puts them), then the bins from eraseBin on are erased.
// One workgroup per pair: counts into LDS, one lane sorts 30 items, then the erase pass.
constexpr int HISTO_LENGTH = 30;

__device__ __forceinline__ int rot_bin(float angB, float angA) {
    float diff = angB - angA;
    if (diff < 0) diff += 360.f;
    int bin = __float2int_rn((1.f / HISTO_LENGTH) * diff);   // cvRound: round half to even
    if (bin == HISTO_LENGTH) bin = 0;
    return min(max(bin, 0), HISTO_LENGTH - 1);   // angles outside [0, 360) (the reference asserts)
}

__global__ __launch_bounds__(256) void check_orientation_kernel(
    const float* __restrict__ angA, int kstrideA, int capA, const int32_t* __restrict__ nA_arr,
    const float* __restrict__ angB, int kstrideB, int capB, const int32_t* __restrict__ pair_b,
    int32_t* __restrict__ match, int strideM, int32_t* __restrict__ nmatch, const int32_t* __restrict__ pair_a) {
    __shared__ int hist[HISTO_LENGTH];
    __shared__ uint32_t keep;
    const int p = blockIdx.x, q = pair_b ? pair_b[p] : p, tid = threadIdx.x;
    const int pa = pair_a ? pair_a[p] : p;   // A frame of pair p (SearchByBoW(KeyFrame, KeyFrame): kf1 slots)
    const int n = nA_arr[pa];
    const float* aA = angA + (long long)pa * capA * kstrideA;
    const float* aB = angB + (long long)q * capB * kstrideB;
    int32_t* m = match + (long long)p * strideM;
    if (tid < HISTO_LENGTH) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        const int j = m[i];
        if (j >= 0) atomicAdd(&hist[rot_bin(aB[(long long)j * kstrideB], aA[(long long)i * kstrideA])], 1);
    }
    __syncthreads();
    if (tid == 0) {
        QtItem it[HISTO_LENGTH];
        for (int b = 0; b < HISTO_LENGTH; b++) it[b] = QtItem{hist[b], b};
        qt_sort(it, it + HISTO_LENGTH);
        const double max1 = it[0].size, max2 = it[1].size, max3 = it[2].size;
        const int eraseBin = max2 < 0.1 * max1 ? 1 : (max3 < 0.1 * max1 ? 2 : 3);
        uint32_t k = 0;
        int kept = 0;
        for (int r = 0; r < eraseBin; r++) {
            k |= 1u << it[r].node;
            kept += it[r].size;
        }
        keep = k;
        if (nmatch) nmatch[p] = kept;   // matchIds.size() - reduction
    }
    __syncthreads();
    const uint32_t k = keep;
    for (int i = tid; i < n; i += blockDim.x) {
        const int j = m[i];
        if (j >= 0 && !((k >> rot_bin(aB[(long long)j * kstrideB], aA[(long long)i * kstrideA])) & 1u)) m[i] = -1;
    }
}

struct TriQuery {
    int idx1;
    int beg2, end2;   // candidate range in the kf2 index list
};

__global__ __launch_bounds__(256) void triangulation_kernel(const TriQuery* __restrict__ q, int nq,
                                                            const float* __restrict__ xy1, const uint8_t* __restrict__ d1,
                                                            const float* __restrict__ xy2, const int32_t* __restrict__ oct2,
                                                            const float* __restrict__ ur2, const uint8_t* __restrict__ mp2,
                                                            const uint8_t* __restrict__ d2, const int32_t* __restrict__ idx2,
                                                            const float* __restrict__ ur1, const float* F,
                                                            float ep2x, float ep2y, const float* __restrict__ scale2,
                                                            const float* __restrict__ sigma2, int only_stereo,
                                                            int32_t* __restrict__ match12) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq) return;
    const TriQuery Q = q[t];
    const int i1 = Q.idx1;
    const bool st1 = ur1[i1] >= 0;
    const uint4 a0 = reinterpret_cast<const uint4*>(d1)[2 * i1], a1 = reinterpret_cast<const uint4*>(d1)[2 * i1 + 1];
    const float x1 = xy1[2 * i1], y1 = xy1[2 * i1 + 1];
    // epipolar line l = x1' F12 (:391-393)
    const float la = x1 * F[0] + y1 * F[3] + F[6];
    const float lb = x1 * F[1] + y1 * F[4] + F[7];
    const float lc = x1 * F[2] + y1 * F[5] + F[8];
    int bd = 50, bi = -1;   // TH_LOW
    for (int u = Q.beg2; u < Q.end2; u++) {
        const int i2 = idx2[u];
        if (mp2[i2]) continue;
        const bool st2 = ur2[i2] >= 0;
        if (only_stereo && !st2) continue;
        const uint4 b0 = reinterpret_cast<const uint4*>(d2)[2 * i2], b1 = reinterpret_cast<const uint4*>(d2)[2 * i2 + 1];
        const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                      __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
        if (d > 50 || d > bd) continue;
        const float x2 = xy2[2 * i2], y2 = xy2[2 * i2 + 1];
        const int o2 = oct2[i2];
        if (!st1 && !st2) {
            const float dx = ep2x - x2, dy = ep2y - y2;
            if (dx * dx + dy * dy < 100 * scale2[o2]) continue;
        }
        const float num = la * x2 + lb * y2 + lc;
        const float den = la * la + lb * lb;
        if (den == 0) continue;
        const float dsqr = num * num / den;
        if ((double)dsqr < 3.84 * (double)sigma2[o2]) {
            bi = i2;
            bd = d;
        }
    }
    match12[i1] = bi;
}

// ---------------------------------------------------------------------------------------------
// Batched SearchForTriangulation on extractor output (orbm_search_for_triangulation_batch_device).
// Per query the reference keeps the LAST candidate (in kf2's index order) whose distance equals
// the minimum over the gate-passing candidates with d <= TH_LOW: bestDist starts at TH_LOW, a
// candidate is considered iff d <= bestDist (:823) and, if it passes the epipole / epipolar gates,
// becomes the best.  `matched2` is never set (§0.5), so queries are independent.
struct TriTables {
    float scale2[ORBM_TRI_MAX_LEVELS];
    float sigma2[ORBM_TRI_MAX_LEVELS];
    int n_levels;
};

struct TriArgs {
    const orbx_keypoint* kps1;
    const uint8_t* desc1;
    const int32_t* counts1;
    const float* ur1;
    const uint8_t* mp1;
    const orbx_keypoint* kps2;
    const uint8_t* desc2;
    const int32_t* counts2;
    const float* ur2;
    const uint8_t* mp2;
    const int32_t* frame1;
    const int32_t* frame2;
    const float* F12;
    const float* ep2;
    const uint32_t* fvn1;
    const int32_t* fvo1;
    const int32_t* fvi1;
    const int32_t* fvc1;
    const uint32_t* fvn2;
    const int32_t* fvo2;
    const int32_t* fvi2;
    const int32_t* fvc2;
    int cap1, cap2, fvcap1, fvcap2, only_stereo;
    int32_t* match12;
    int32_t* nmatches;
};

// Epipole (mono-mono pairs, :828-833) and epipolar-line (CheckDistEpipolarLine, :384-404) gates.
// ep2 may be non-finite (a kf1 centre on kf2's principal plane, e.g. a rectified stereo pair): the
// squared distance is then NaN or inf and the comparisons fall as in the reference.
__device__ __forceinline__ bool tri_gates(float la, float lb, float lc, bool st1, bool st2, float x2, float y2, int o2,
                                          float ep2x, float ep2y, const TriTables& t) {
    o2 = min(max(o2, 0), t.n_levels - 1);
    if (!st1 && !st2) {
        const float dx = ep2x - x2, dy = ep2y - y2;
        if (dx * dx + dy * dy < 100 * t.scale2[o2]) return false;
    }
    const float num = la * x2 + lb * y2 + lc;
    const float den = la * la + lb * lb;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)t.sigma2[o2];
}

__device__ __forceinline__ int hamming8(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

constexpr int TRI_SEG = 256;   // kf2 candidates per workgroup

// Single BoW node holding every keypoint of both keyframes (no vocabulary): every
// query scans all of kf2.  The reference keeps the gate-passing candidate of minimum distance
// <= TH_LOW and, among equal distances, the largest index (its ascending scan replaces the best on
// d <= bestDist: the last minimum wins) — an order-independent minimum of the key
// (d << 16) | (0xFFFF - j).  So kf2 is cut into segments of 256 candidates, one workgroup per
// (256 queries, segment, pair) scans its segment with one lane per query (descriptors and gate
// operands staged in LDS, read as wavefront broadcasts) and merges its best key into match12 with
// atomicMin; tri_finalize_kernel turns the keys into indices.
__global__ __launch_bounds__(256) void tri_all_kernel(TriArgs a, TriTables t, int nqb) {
    __shared__ uint4 sd[TRI_SEG * 2];
    __shared__ float4 sk[TRI_SEG];   // x, y, octave bits, stereo flag
    __shared__ uint32_t sv[TRI_SEG / 32];
    const int p = blockIdx.y, tid = threadIdx.x;
    const int qb = blockIdx.x % nqb, c0 = (blockIdx.x / nqb) * TRI_SEG;
    const int f1 = a.frame1 ? a.frame1[p] : p, f2 = a.frame2 ? a.frame2[p] : p;
    const int n1 = a.counts1[f1], n2 = a.counts2[f2];
    if (qb * 256 >= n1 || c0 >= n2) return;   // block-uniform
    const int i1 = qb * 256 + tid;
    const long long g1 = (long long)f1 * a.cap1 + i1;
    const bool in = i1 < n1;
    const bool st1 = in && a.ur1 && a.ur1[g1] >= 0;
    const bool act = in && !(a.mp1 && a.mp1[g1]) && (!a.only_stereo || st1);
    const long long base2 = (long long)f2 * a.cap2;
    {
        const int j = c0 + tid;
        bool v = false;
        if (j < n2) {
            const long long g2 = base2 + j;
            sd[2 * tid] = reinterpret_cast<const uint4*>(a.desc2)[2 * g2];
            sd[2 * tid + 1] = reinterpret_cast<const uint4*>(a.desc2)[2 * g2 + 1];
            const orbx_keypoint& kp = a.kps2[g2];
            const bool st2 = a.ur2 && a.ur2[g2] >= 0;
            sk[tid] = make_float4(kp.x, kp.y, __int_as_float(kp.octave), st2 ? 1.f : 0.f);
            v = !(a.mp2 && a.mp2[g2]) && (!a.only_stereo || st2);
        }
        const uint64_t bal = __ballot(v);
        if ((tid & 63) == 0) {
            sv[2 * (tid >> 6)] = (uint32_t)bal;
            sv[2 * (tid >> 6) + 1] = (uint32_t)(bal >> 32);
        }
    }
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    float la = 0, lb = 0, lc = 0;
    if (act) {
        a0 = reinterpret_cast<const uint4*>(a.desc1)[2 * g1];
        a1 = reinterpret_cast<const uint4*>(a.desc1)[2 * g1 + 1];
        const float x1 = a.kps1[g1].x, y1 = a.kps1[g1].y;
        const float* F = a.F12 + 9 * (long long)p;
        la = x1 * F[0] + y1 * F[3] + F[6];   // l = x1' F12 (:391-393)
        lb = x1 * F[1] + y1 * F[4] + F[7];
        lc = x1 * F[2] + y1 * F[5] + F[8];
    }
    const float ep2x = a.ep2[2 * p], ep2y = a.ep2[2 * p + 1];
    __syncthreads();
    if (!act) return;
    int bd = 50, bi = -1;   // TH_LOW
    // kf2 descriptors through the scalar path (uniform addresses in the constant address space:
    // s_load_dwordx8, XORed as SGPR operands), four candidates per batch; the validity mask and
    // the gate operands only on the rare d <= bd branch
    typedef const uint32_t __attribute__((address_space(4))) cu32;
    const cu32* D2 = (const cu32*)(a.desc2 + (base2 + c0) * 32);
    const int m = min(TRI_SEG, n2 - c0);
    auto ham = [&](const cu32* dk) {
        return __popc(a0.x ^ dk[0]) + __popc(a0.y ^ dk[1]) + __popc(a0.z ^ dk[2]) + __popc(a0.w ^ dk[3]) +
               __popc(a1.x ^ dk[4]) + __popc(a1.y ^ dk[5]) + __popc(a1.z ^ dk[6]) + __popc(a1.w ^ dk[7]);
    };
    auto consider = [&](int k, int d) {
        if (d > bd) return;
        if (!((sv[k >> 5] >> (k & 31)) & 1u)) return;
        const float4 kp2 = sk[k];
        if (tri_gates(la, lb, lc, st1, kp2.w != 0.f, kp2.x, kp2.y, __float_as_int(kp2.z), ep2x, ep2y, t)) {
            bi = c0 + k;
            bd = d;
        }
    };
    int k = 0;
    for (; k + 4 <= m; k += 4) {
        const int d0 = ham(D2 + 8 * k), d1 = ham(D2 + 8 * k + 8), d2 = ham(D2 + 8 * k + 16), d3 = ham(D2 + 8 * k + 24);
        consider(k, d0);
        consider(k + 1, d1);
        consider(k + 2, d2);
        consider(k + 3, d3);
    }
    for (; k < m; k++) consider(k, ham(D2 + 8 * k));
    if (bi >= 0)
        atomicMin(reinterpret_cast<unsigned*>(a.match12) + (long long)p * a.cap1 + i1, ((unsigned)bd << 16) | (0xFFFFu - (unsigned)bi));
}

// The all-pairs search on the FP4 matrix path (hamming_top2_fp4_kernel's tiling): a workgroup owns
// 256 queries of one pair and streams all of kf2 through the MFMA.  A key 128 S (S = d - |a| + 256,
// the accumulator started at 128 (|b| + 256)) below the row's threshold 128 (307 - |a|) is a
// candidate with d <= TH_LOW; it is appended to the wavefront's LDS event pool as (row, d, j)
// (slots from a wave-uniform count and the lane's rank in the ballot: no atomics).  After the
// stream the wavefront's 64 lanes share its events: a candidate whose key (d << 16) | (0xFFFF - j)
// is below the row's current best is checked for validity and the gates and merged into the row's
// best with an LDS atomicMin (the order-independent form of the reference's scan, see
// tri_all_kernel).  Rows whose events did not fit are rescanned exactly by the whole workgroup.
// Rows the reference skips (a MapPoint, onlyStereo) get threshold 0: no events, result -1.
#ifndef TRI_POOL_DEF
#define TRI_POOL_DEF 1024
#endif
#ifndef TRI_RT_DEF
#define TRI_RT_DEF 4
#endif
constexpr int TRI_POOL = TRI_POOL_DEF;   // events per wavefront
constexpr int TRI_RT = TRI_RT_DEF;       // 16-row tiles per wavefront
constexpr int TRI_WROWS = 16 * TRI_RT, TRI_ROWS = 4 * TRI_WROWS;
__device__ __forceinline__ bool tri_valid2(const TriArgs& a, long long g2, bool* st2) {
    *st2 = a.ur2 && a.ur2[g2] >= 0;
    return !(a.mp2 && a.mp2[g2]) && (!a.only_stereo || *st2);
}

__global__ __launch_bounds__(256) void tri_mm_kernel(TriArgs a, TriTables t, int nsplit) {
    extern __shared__ __attribute__((aligned(16))) int mm_sm[];   // row | best | ovf | pa | ev | xb | pb
    float4* s_row = reinterpret_cast<float4*>(mm_sm);                  // la, lb, lc, st1 (per WG row)
    uint32_t* s_best = reinterpret_cast<uint32_t*>(mm_sm + 4 * TRI_ROWS);
    int* s_ovf = mm_sm + 5 * TRI_ROWS;
    int* s_pa = mm_sm + 6 * TRI_ROWS;
    uint32_t* s_ev = reinterpret_cast<uint32_t*>(mm_sm + 7 * TRI_ROWS);   // [4 waves][TRI_POOL]
    i4v* xb = reinterpret_cast<i4v*>(mm_sm + 7 * TRI_ROWS + 4 * TRI_POOL);   // [2][2][2][64]
    int* s_pb = mm_sm + 7 * TRI_ROWS + 4 * TRI_POOL + 2 * 2 * 2 * 64 * 4;
    __shared__ int s_anyovf;
    const int p = blockIdx.y;
    const int f1 = a.frame1 ? a.frame1[p] : p, f2 = a.frame2 ? a.frame2[p] : p;
    const int nA = a.counts1[f1], nB = a.counts2[f2];
    const int row_base = (blockIdx.x / nsplit) * TRI_ROWS;
    // this workgroup's kf2 columns [jlo, jhi) (a multiple of 32 wide except the last part)
    const int span = ((nB + nsplit - 1) / nsplit + 31) & ~31;
    const int jlo = (blockIdx.x % nsplit) * span, jhi = min(nB, jlo + span);
    if (row_base >= nA || (nsplit > 1 && jlo >= jhi)) return;   // block-uniform (one part: rows get -1 below)
    const uint8_t* Ap = a.desc1 + (long long)f1 * a.cap1 * 32;
    const uint8_t* Bp = a.desc2 + (long long)f2 * a.cap2 * 32;
    const long long base2 = (long long)f2 * a.cap2;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c16 = lane & 15, g = lane >> 4;
    const int jht = jlo + ((jhi - jlo + 31) & ~31);
    const float ep2x = a.ep2[2 * p], ep2y = a.ep2[2 * p + 1];
    for (int j = jlo + tid; j < jht; j += blockDim.x)   // columns past jhi: padding (S = 512, never an event)
        s_pb[j - jlo] = 128 * ((j < jhi ? popc_row(Bp + (long long)j * 32) : 256) + 256);
    if (tid < TRI_ROWS) {
        const int row = row_base + tid;
        int pa = -1;   // -1: no events for this row
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < nA) {
            const long long g1 = (long long)f1 * a.cap1 + row;
            const bool st1 = a.ur1 && a.ur1[g1] >= 0;
            if (!(a.mp1 && a.mp1[g1]) && (!a.only_stereo || st1)) {
                pa = popc_row(Ap + (long long)row * 32);
                const float x1 = a.kps1[g1].x, y1 = a.kps1[g1].y;
                const float* F = a.F12 + 9 * (long long)p;
                rv = make_float4(x1 * F[0] + y1 * F[3] + F[6], x1 * F[1] + y1 * F[4] + F[7],
                                 x1 * F[2] + y1 * F[5] + F[8], st1 ? 1.f : 0.f);   // l = x1' F12 (:391-393)
            }
        }
        s_row[tid] = rv;
        s_best[tid] = 0xffffffffu;
        s_ovf[tid] = 0;
        s_pa[tid] = pa;
    }
    if (tid == 0) s_anyovf = 0;
    const bool live = __builtin_amdgcn_readfirstlane(row_base + TRI_WROWS * w < nA ? 1 : 0) != 0;
    i4v af[TRI_RT][2];
#pragma unroll
    for (int rt = 0; rt < TRI_RT; rt++) {
        const int row = min(row_base + TRI_WROWS * w + 16 * rt + c16, nA - 1);
        const uint2 v = *reinterpret_cast<const uint2*>(Ap + (long long)row * 32 + 8 * g);
        af[rt][0] = expand32_nib(v.x, FP4_NEG4);
        af[rt][1] = expand32_nib(v.y, FP4_NEG4);
    }
    const int xt = w >> 1, xs = w & 1;
    auto ldb = [&](int jj) -> uint32_t {
        return jj < jhi ? *reinterpret_cast<const uint32_t*>(Bp + (long long)jj * 32 + 8 * g + 4 * xs) : 0u;
    };
    xb[((0 * 2 + xt) * 2 + xs) * 64 + lane] = expand32_nib(ldb(jlo + 16 * xt + c16), FP4_ONE);
    uint32_t bn = ldb(jlo + 32 + 16 * xt + c16);
    __syncthreads();
    float thr[TRI_RT][4];   // 128 (307 - |a|): key < thr <=> d <= TH_LOW
#pragma unroll
    for (int rt = 0; rt < TRI_RT; rt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int pa = s_pa[TRI_WROWS * w + 16 * rt + 4 * g + r];
            thr[rt][r] = pa < 0 ? 0.f : (float)(128 * (307 - pa));
        }
    int nev = 0;   // wave-uniform
    uint32_t* ev = s_ev + w * TRI_POOL;
    for (int j0 = jlo; j0 < jhi; j0 += 32) {
        const int cur = ((j0 - jlo) >> 5) & 1;
        if (j0 + 32 < jhi) {   // block-uniform
            xb[(((cur ^ 1) * 2 + xt) * 2 + xs) * 64 + lane] = expand32_nib(bn, FP4_ONE);
            bn = ldb(j0 + 64 + 16 * xt + c16);
        }
#pragma unroll
        for (int tt = 0; tt < 2; tt++) {
            if (!live) break;   // wavefront-uniform
            const float ci = (float)s_pb[j0 - jlo + 16 * tt + c16];
            const f4v cinit = {ci, ci, ci, ci};
            const i4v b0 = xb[((cur * 2 + tt) * 2 + 0) * 64 + lane];
            const i4v b1 = xb[((cur * 2 + tt) * 2 + 1) * 64 + lane];
#pragma unroll
            for (int rt = 0; rt < TRI_RT; rt++) {
                f4v acc = mfma_fp4(af[rt][0], b0, cinit);
                acc = mfma_fp4(af[rt][1], b1, acc);
                const float kv[4] = {acc.x, acc.y, acc.z, acc.w};
                const bool any = (kv[0] < thr[rt][0]) | (kv[1] < thr[rt][1]) | (kv[2] < thr[rt][2]) | (kv[3] < thr[rt][3]);
                if (__builtin_amdgcn_read_exec() & __ballot(any)) {   // wavefront-uniform, rare
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const bool e = kv[r] < thr[rt][r];
                        const uint64_t bal = __ballot(e);
                        if (e) {
                            const int rw = 16 * rt + 4 * g + r;   // row within the wavefront
                            // d = S - 256 + |a|, |a| = 307 - thr / 128
                            const int d = ((int)kv[r] >> 7) + 51 - ((int)thr[rt][r] >> 7);
                            const int j = j0 + 16 * tt + c16;
                            const int slot = nev + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                            if (slot < TRI_POOL) ev[slot] = ((uint32_t)rw << 22) | ((uint32_t)d << 16) | (uint32_t)j;
                            else s_ovf[TRI_WROWS * w + rw] = 1;
                        }
                        nev += (int)__popcll(bal);
                    }
                }
            }
        }
        __syncthreads();   // pair expanded into `cur ^ 1`; buffer `cur` free for the pair after
    }
    // the wavefront's events, shared by its lanes: validity, gates, row best (LDS atomicMin)
    for (int e = lane; e < min(nev, TRI_POOL); e += 64) {
        const uint32_t v = ev[e];
        const int rl = TRI_WROWS * w + (int)(v >> 22), d = (int)((v >> 16) & 63u), j = (int)(v & 0xffffu);
        const uint32_t key = ((uint32_t)d << 16) | (0xffffu - (uint32_t)j);
        if (key >= s_best[rl]) continue;
        bool st2;
        const long long g2 = base2 + j;
        if (!tri_valid2(a, g2, &st2)) continue;
        const float4 rv = s_row[rl];
        const orbx_keypoint& kp2 = a.kps2[g2];
        if (tri_gates(rv.x, rv.y, rv.z, rv.w != 0.f, st2, kp2.x, kp2.y, kp2.octave, ep2x, ep2y, t))
            atomicMin(&s_best[rl], key);
    }
    if (nev > TRI_POOL && lane == 0) s_anyovf = 1;
    __syncthreads();
    if (s_anyovf) {   // block-uniform, rare: rows whose events did not fit, rescanned by the workgroup
        for (int rl = 0; rl < TRI_ROWS; rl++) {
            if (!s_ovf[rl]) continue;   // block-uniform
            const int row = row_base + rl;
            const float4 rv = s_row[rl];
            const uint4 a0 = reinterpret_cast<const uint4*>(Ap)[2 * row], a1 = reinterpret_cast<const uint4*>(Ap)[2 * row + 1];
            if (tid == 0) s_best[rl] = 0xffffffffu;
            __syncthreads();
            for (int j = jlo + tid; j < jhi; j += blockDim.x) {
                const int d = hamming8(a0, a1, reinterpret_cast<const uint4*>(Bp)[2 * j], reinterpret_cast<const uint4*>(Bp)[2 * j + 1]);
                if (d > 50) continue;
                bool st2;
                if (!tri_valid2(a, base2 + j, &st2)) continue;
                const orbx_keypoint& kp2 = a.kps2[base2 + j];
                if (tri_gates(rv.x, rv.y, rv.z, rv.w != 0.f, st2, kp2.x, kp2.y, kp2.octave, ep2x, ep2y, t))
                    atomicMin(&s_best[rl], ((uint32_t)d << 16) | (0xffffu - (uint32_t)j));
            }
            __syncthreads();
        }
    }
    const int row = row_base + tid;
    bool got = false;
    if (tid < TRI_ROWS && row < nA) {
        const uint32_t best = s_best[tid];
        got = best != 0xffffffffu;
        if (nsplit > 1) {   // column parts merge their keys; tri_finalize_kernel decodes
            if (got) atomicMin(reinterpret_cast<unsigned*>(a.match12) + (long long)p * a.cap1 + row, best);
            return;
        }
        a.match12[(long long)p * a.cap1 + row] = got ? (int32_t)(0xffffu - (best & 0xffffu)) : -1;
    }
    if (nsplit > 1) return;
    const uint64_t bal = __ballot(got);
    if ((tid & 63) == 0 && bal) atomicAdd(a.nmatches + p, (int)__popcll(bal));
}

// match12 keys -> kf2 indices (-1 where no candidate passed), and the per-pair match count.
__global__ __launch_bounds__(256) void tri_finalize_kernel(int32_t* __restrict__ match12, int cap1,
                                                           int32_t* __restrict__ nmatches) {
    const int p = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    bool got = false;
    if (i < cap1) {
        const unsigned key = reinterpret_cast<unsigned*>(match12)[(long long)p * cap1 + i];
        got = key != 0xFFFFFFFFu;
        match12[(long long)p * cap1 + i] = got ? (int32_t)(0xFFFFu - (key & 0xFFFFu)) : -1;
    }
    const uint64_t bal = __ballot(got);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(nmatches + p, (int)__popcll(bal));
}

// General DBoW2 FeatureVectors (orbv_transform_batch_device layout): FeatureVectorIterator
// (:406-450) pairs equal node ids; each wavefront takes kf1 nodes in turn, finds the node in kf2's
// ascending list by binary search, and maps the node's queries one per lane over the node's kf2
// candidates (ascending, as stored).
__global__ __launch_bounds__(256) void tri_fv_kernel(TriArgs a, TriTables t) {
    const int p = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int f1 = a.frame1 ? a.frame1[p] : p, f2 = a.frame2 ? a.frame2[p] : p;
    const int nn1 = a.fvc1[f1], nn2 = a.fvc2[f2];
    const uint32_t* node1 = a.fvn1 + (long long)f1 * a.fvcap1;
    const uint32_t* node2 = a.fvn2 + (long long)f2 * a.fvcap2;
    const int32_t* off1 = a.fvo1 + (long long)f1 * (a.fvcap1 + 1);
    const int32_t* off2 = a.fvo2 + (long long)f2 * (a.fvcap2 + 1);
    const int32_t* idx1 = a.fvi1 + (long long)f1 * a.fvcap1;
    const int32_t* idx2 = a.fvi2 + (long long)f2 * a.fvcap2;
    const long long base1 = (long long)f1 * a.cap1, base2 = (long long)f2 * a.cap2;
    const float* F = a.F12 + 9 * (long long)p;
    const float ep2x = a.ep2[2 * p], ep2y = a.ep2[2 * p + 1];
    int found = 0;
    for (int na = w; na < nn1; na += 4) {
        const uint32_t id = node1[na];
        int lo = 0, hi = nn2;   // lower_bound
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (node2[mid] < id) lo = mid + 1;
            else hi = mid;
        }
        if (lo >= nn2 || node2[lo] != id) continue;
        const int c0 = off2[lo], c1 = off2[lo + 1];
        for (int u = off1[na] + lane; u < off1[na + 1]; u += 64) {
            const int i1 = idx1[u];
            const long long g1 = base1 + i1;
            const bool st1 = a.ur1 && a.ur1[g1] >= 0;
            if ((a.mp1 && a.mp1[g1]) || (a.only_stereo && !st1)) continue;
            const uint4 a0 = reinterpret_cast<const uint4*>(a.desc1)[2 * g1];
            const uint4 a1 = reinterpret_cast<const uint4*>(a.desc1)[2 * g1 + 1];
            const float x1 = a.kps1[g1].x, y1 = a.kps1[g1].y;
            const float la = x1 * F[0] + y1 * F[3] + F[6];
            const float lb = x1 * F[1] + y1 * F[4] + F[7];
            const float lc = x1 * F[2] + y1 * F[5] + F[8];
            int bd = 50, bi = -1;
            for (int v = c0; v < c1; v++) {
                const int i2 = idx2[v];
                const long long g2 = base2 + i2;
                if (a.mp2 && a.mp2[g2]) continue;
                const bool st2 = a.ur2 && a.ur2[g2] >= 0;
                if (a.only_stereo && !st2) continue;
                const uint4* b = reinterpret_cast<const uint4*>(a.desc2) + 2 * g2;
                const int d = hamming8(a0, a1, b[0], b[1]);
                if (d > bd) continue;
                const orbx_keypoint kp2 = a.kps2[g2];
                if (tri_gates(la, lb, lc, st1, st2, kp2.x, kp2.y, kp2.octave, ep2x, ep2y, t)) {
                    bi = i2;
                    bd = d;
                }
            }
            if (bi >= 0) {
                a.match12[(long long)p * a.cap1 + i1] = bi;
                found++;
            }
        }
    }
    const int tot = __reduce_add_sync(~0ull, found);
    if (lane == 0 && tot) atomicAdd(a.nmatches + p, tot);
}

// SearchByBoW(KeyFrame*, Frame&) (src/ORBmatcher.cc:452-516).  A frame feature belongs to one
// FeatureVector node, so the claims (`if (matches[idx2]) continue`, :483) of different common nodes
// never interact: one wavefront per common node walks the node's keyframe features in stored order
// (the reference's order inside the node), lanes over the node's frame candidates (64 per chunk).
// Per query every lane keeps its best key (d << 16 | candidate position: the lowest position wins
// a tie, as the strict '<' of :488) and its second distance; the wave minimum of the keys is the
// best, the minimum of the other lanes' bests and the winner's second is secondBestDist (the
// second order statistic the sequential update produces).  A claim sets the winner lane's bit.
struct BowArgs {
    const uint8_t* desc1;
    const uint8_t* mp1;
    const int32_t* frame1;
    const uint8_t* desc2;
    const uint32_t* fvn1; const int32_t* fvo1; const int32_t* fvi1; const int32_t* fvc1;
    const uint32_t* fvn2; const int32_t* fvo2; const int32_t* fvi2; const int32_t* fvc2;
    int cap1, cap2, fvcap1, fvcap2;
    float nnratio;
    int32_t* match;
    int32_t* nmatches;
    const uint8_t* mp2;      // KeyFrame-KeyFrame form: candidate MapPoint valid (NULL: all)
    const int32_t* frame2;   // KeyFrame-KeyFrame form: kf2 slot of pair p (NULL: p)
    int kf;                  // 1: SearchByBoW(KeyFrame*, KeyFrame*) (:696-766), matches12 by idx1
};
constexpr int BOW_MAX_CAND = 64 * 64;   // frame candidates per node: one claim bit per lane and chunk

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}

__global__ __launch_bounds__(256) void search_by_bow_kernel(BowArgs a) {
    const int p = blockIdx.y, lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), nwv = gridDim.x * 4;
    const int f1 = a.frame1 ? a.frame1[p] : p, f2 = a.frame2 ? a.frame2[p] : p;
    const int nn1 = a.fvc1[f1], nn2 = a.fvc2[f2];
    const uint32_t* node1 = a.fvn1 + (long long)f1 * a.fvcap1;
    const uint32_t* node2 = a.fvn2 + (long long)f2 * a.fvcap2;
    const int32_t* off1 = a.fvo1 + (long long)f1 * (a.fvcap1 + 1);
    const int32_t* off2 = a.fvo2 + (long long)f2 * (a.fvcap2 + 1);
    const int32_t* idx1 = a.fvi1 + (long long)f1 * a.fvcap1;
    const int32_t* idx2 = a.fvi2 + (long long)f2 * a.fvcap2;
    const long long base1 = (long long)f1 * a.cap1, base2 = (long long)f2 * a.cap2;
    const uint4* D1 = reinterpret_cast<const uint4*>(a.desc1);
    const uint4* D2 = reinterpret_cast<const uint4*>(a.desc2);
    // Frame form: matches[idx2] = idx1 (pair p's frame slots); KeyFrame form: matches12[idx1] = idx2
    int32_t* out = a.match + (long long)p * (a.kf ? a.cap1 : a.cap2);
    const int th_ok = a.kf ? 49 : 50;   // bestDist < TH_LOW (:750) / bestDist <= TH_LOW (:500)
    int found = 0;
    for (int na = wv; na < nn1; na += nwv) {
        const uint32_t id = node1[na];
        int lo = 0, hi = nn2;   // lower_bound (the iterator's join, :419-442)
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (node2[mid] < id) lo = mid + 1;
            else hi = mid;
        }
        if (lo >= nn2 || node2[lo] != id) continue;
        const int c0 = off2[lo], n2 = min(off2[lo + 1] - c0, BOW_MAX_CAND);
        const int nch = (n2 + 63) >> 6;
        unsigned long long claimed = 0;   // bit k: candidate 64k + lane
        // the first 64 candidates stay in registers for all of the node's queries (their index and
        // descriptor loads are off the per-query dependency chain)
        uint4 cd0 = make_uint4(0, 0, 0, 0), cd1 = cd0;
        bool ok0 = false;
        if (lane < n2) {
            const long long g2 = base2 + idx2[c0 + lane];
            ok0 = !a.mp2 || a.mp2[g2];
            cd0 = D2[2 * g2];
            cd1 = D2[2 * g2 + 1];
        }
        // the next query's index, MapPoint flag and descriptor are loaded while this one is matched
        const int u1 = off1[na + 1];
        int i1n = 0;
        bool vn = false;
        uint4 qn0 = make_uint4(0, 0, 0, 0), qn1 = qn0;
        auto fetch = [&](int uu) {
            i1n = idx1[uu];
            const long long g = base1 + i1n;
            vn = !a.mp1 || a.mp1[g];
            qn0 = D1[2 * g];
            qn1 = D1[2 * g + 1];
        };
        if (off1[na] < u1) fetch(off1[na]);
        for (int u = off1[na]; u < u1; u++) {
            const int i1 = i1n;
            const bool valid = vn;
            const uint4 q0 = qn0, q1 = qn1;
            if (u + 1 < u1) fetch(u + 1);
            if (!valid) continue;   // !mappoint1 || mappoint1->isBad() (:472)
            uint32_t k1 = 0xffffffffu;
            int d2 = 256;
            for (int k = 0; k < nch; k++) {
                const int pos = 64 * k + lane;
                bool ok;
                uint4 b0, b1;
                if (k == 0) {
                    ok = ok0;
                    b0 = cd0;
                    b1 = cd1;
                } else {
                    const long long g2 = pos < n2 ? base2 + idx2[c0 + pos] : 0;
                    ok = pos < n2 && (!a.mp2 || a.mp2[g2]);
                    if (ok) {
                        b0 = D2[2 * g2];
                        b1 = D2[2 * g2 + 1];
                    }
                }
                if (ok && !((claimed >> k) & 1ull)) {   // matched2 / mappoint2 (:733)
                    const int d = hamming8(q0, q1, b0, b1);
                    const uint32_t key = ((uint32_t)d << 16) | (uint32_t)pos;
                    if (key < k1) {
                        d2 = min(d2, (int)(k1 >> 16));
                        k1 = key;
                    } else if (d < d2) {
                        d2 = d;
                    }
                }
            }
            const uint32_t K = wave_min_u32(k1);
            if (K == 0xffffffffu) continue;   // no unclaimed candidate: bestDist stays 256
            const int sd = (int)wave_min_u32((uint32_t)(k1 == K ? d2 : min((int)(k1 >> 16), 256)));
            const int bd = (int)(K >> 16);
            if (bd <= th_ok && (float)bd < a.nnratio * (float)sd) {   // :500 / :750
                const int pos = (int)(K & 0xffffu);
                if ((pos & 63) == lane) {
                    claimed |= 1ull << (pos >> 6);
                    if (a.kf) out[i1] = idx2[c0 + pos];
                    else out[idx2[c0 + pos]] = i1;
                    found++;
                }
            }
        }
    }
    const int tot = __reduce_add_sync(~0ull, found);
    if (lane == 0 && tot) atomicAdd(a.nmatches + p, tot);
}

}  // namespace orbamd

using namespace orbamd;

namespace {
struct HostScratch {
    DevBuf a, b, o1, o2, o3, o4;
};
thread_local HostScratch g_scratch;
}  // namespace

extern "C" {

int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

int orbm_hamming_top2_device(const uint8_t* d_A, int nA, const uint8_t* d_B, int nB, int32_t* d_best_idx,
                             int32_t* d_best, int32_t* d_second, void* stream) {
    ORB_CHECK_ARG(nA >= 0 && nB >= 0 && (nA == 0 || d_A) && (nB == 0 || d_B), "bad matcher arguments");
    if (nA == 0) return ORB_OK;
    launch_top2(d_A, nullptr, nA, nA, d_B, nullptr, nB, std::max(nB, 1), nullptr, 1, 0.6f, 50, d_best_idx, d_best,
                d_second, nullptr, (hipStream_t)stream);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

int orbm_bf_match_batch_device(const uint8_t* d_A, const int32_t* d_nA, int strideA, const uint8_t* d_B,
                               const int32_t* d_nB, int strideB, const int32_t* d_pair_b, int n_pairs, float nnratio,
                               int th_low, int32_t* d_best_idx, int32_t* d_best, int32_t* d_second,
                               int32_t* d_match, void* stream) {
    ORB_CHECK_ARG(d_A && d_B && d_nA && d_nB && n_pairs >= 0 && strideA > 0 && strideB > 0, "bad matcher arguments");
    if (n_pairs == 0) return ORB_OK;
    ORB_CHECK_ARG(n_pairs <= 65535, "too many pairs in one launch");
    launch_top2(d_A, d_nA, 0, strideA, d_B, d_nB, 0, strideB, d_pair_b, n_pairs, nnratio, th_low, d_best_idx, d_best,
                d_second, d_match, (hipStream_t)stream);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

int orbm_bf_match(const uint8_t* A, int nA, const uint8_t* B, int nB, float nnratio, int th_low, int32_t* best_idx,
                  int32_t* best, int32_t* second, int32_t* match) {
    ORB_CHECK_ARG(nA >= 0 && nB >= 0, "negative sizes");
    if (nA == 0) return ORB_OK;
    ORB_CHECK_ARG(A && (nB == 0 || B), "null descriptors");
    HostScratch& s = g_scratch;
    int rc;
    if ((rc = s.a.reserve((size_t)nA * 32))) return rc;
    if ((rc = s.b.reserve((size_t)std::max(nB, 1) * 32))) return rc;
    if ((rc = s.o1.reserve((size_t)nA * 16))) return rc;
    int32_t* o = s.o1.as<int32_t>();
    ORB_HIP_TRY(hipMemcpy(s.a.ptr, A, (size_t)nA * 32, hipMemcpyHostToDevice));
    if (nB) ORB_HIP_TRY(hipMemcpy(s.b.ptr, B, (size_t)nB * 32, hipMemcpyHostToDevice));
    launch_top2(s.a.as<uint8_t>(), nullptr, nA, nA, s.b.as<uint8_t>(), nullptr, nB, std::max(nB, 1), nullptr, 1, nnratio,
                th_low, o, o + nA, o + 2 * nA, o + 3 * nA, (hipStream_t)0);
    ORB_HIP_TRY(hipGetLastError());
    std::vector<int32_t> h((size_t)nA * 4);
    ORB_HIP_TRY(hipMemcpy(h.data(), o, (size_t)nA * 16, hipMemcpyDeviceToHost));
    for (int i = 0; i < nA; i++) {
        if (best_idx) best_idx[i] = h[i];
        if (best) best[i] = h[nA + i];
        if (second) second[i] = h[2 * nA + i];
        if (match) match[i] = h[3 * nA + i];
    }
    return ORB_OK;
}

int orbm_check_orientation_batch_device(const float* d_angA, int kstrideA, int capA, const int32_t* d_nA,
                                        const float* d_angB, int kstrideB, int capB, const int32_t* d_pair_b,
                                        int n_pairs, int32_t* d_match, int strideM, int32_t* d_nmatches,
                                        void* stream) {
    ORB_CHECK_ARG(n_pairs >= 0 && kstrideA > 0 && kstrideB > 0 && capA > 0 && capB > 0 && strideM > 0,
                  "bad CheckOrientation arguments");
    if (n_pairs == 0) return ORB_OK;
    ORB_CHECK_ARG(d_angA && d_angB && d_nA && d_match, "null CheckOrientation argument");
    hipLaunchKernelGGL(check_orientation_kernel, dim3((unsigned)n_pairs), dim3(256), 0, (hipStream_t)stream, d_angA,
                       kstrideA, capA, d_nA, d_angB, kstrideB, capB, d_pair_b, d_match, strideM, d_nmatches,
                       (const int32_t*)nullptr);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

int orbm_check_orientation(const float* angA, int nA, const float* angB, int nB, int32_t* match, int32_t* nmatches) {
    ORB_CHECK_ARG(nA >= 0 && nB >= 0 && match && (nA == 0 || angA), "bad CheckOrientation arguments");
    for (int i = 0; i < nA; i++) {
        ORB_CHECK_ARG(match[i] < nB && match[i] >= -1, "match index out of range");
        ORB_CHECK_ARG(!(match[i] >= 0) || (angA[i] >= 0.f && angA[i] < 360.f && angB[match[i]] >= 0.f &&
                                           angB[match[i]] < 360.f),
                      "keypoint angle outside [0, 360) (CV_Assert in CheckOrientation)");
    }
    if (nmatches) *nmatches = 0;
    if (nA == 0) return ORB_OK;
    HostScratch& s = g_scratch;
    int rc;
    const size_t offB = align_up((size_t)nA * 4, 256);
    if ((rc = s.o3.reserve(offB + (size_t)std::max(nB, 1) * 4))) return rc;
    if ((rc = s.o4.reserve((size_t)nA * 4 + 8))) return rc;   // matches | nA | match count
    float* dA = s.o3.as<float>();
    float* dB = reinterpret_cast<float*>(s.o3.as<char>() + offB);
    int32_t* dM = s.o4.as<int32_t>();
    ORB_HIP_TRY(hipMemcpy(dA, angA, (size_t)nA * 4, hipMemcpyHostToDevice));
    if (nB) ORB_HIP_TRY(hipMemcpy(dB, angB, (size_t)nB * 4, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(dM, match, (size_t)nA * 4, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(dM + nA, &nA, 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(check_orientation_kernel, dim3(1), dim3(256), 0, (hipStream_t)0, dA, 1, nA, dM + nA, dB, 1,
                       std::max(nB, 1), nullptr, dM, nA, dM + nA + 1, (const int32_t*)nullptr);
    ORB_HIP_TRY(hipGetLastError());
    ORB_HIP_TRY(hipMemcpy(match, dM, (size_t)nA * 4, hipMemcpyDeviceToHost));
    int32_t nm = 0;
    ORB_HIP_TRY(hipMemcpy(&nm, dM + nA + 1, 4, hipMemcpyDeviceToHost));
    if (nmatches) *nmatches = nm;
    return ORB_OK;
}

static int search_by_bow(const orbm_bow_batch* b, int kf, int32_t* d_match, int32_t* d_nmatches, void* stream) {
    ORB_CHECK_ARG(b && d_match && d_nmatches, "null argument");
    ORB_CHECK_ARG(b->n_pairs >= 0 && b->cap1 > 0 && b->cap2 > 0, "bad pair count / capacities");
    if (b->n_pairs == 0) return ORB_OK;
    ORB_CHECK_ARG(b->n_pairs <= 65535, "too many pairs in one launch");
    ORB_CHECK_ARG(b->cap2 <= BOW_MAX_CAND, "SearchByBoW: frame capacity above 4096 keypoints");
    ORB_CHECK_ARG(b->desc1 && b->desc2 && b->counts2, "null keyframe / frame arrays");
    ORB_CHECK_ARG(b->fv_node1 && b->fv_off1 && b->fv_idx1 && b->fv_n_nodes1 && b->fv_node2 && b->fv_off2 && b->fv_idx2 &&
                      b->fv_n_nodes2 && b->fv_cap1 > 0 && b->fv_cap2 > 0,
                  "SearchByBoW needs both FeatureVectors");
    ORB_CHECK_ARG(!b->check_orientation || (b->kps1 && b->kps2), "CheckOrientation needs the keypoint slots");
    ORB_CHECK_ARG(kf || (!b->frame2 && !b->mp_valid2), "frame2 / mp_valid2 belong to the KeyFrame-KeyFrame form");
    ORB_CHECK_ARG(!kf || !b->check_orientation || b->counts1, "CheckOrientation needs counts1");
    BowArgs a{b->desc1, b->mp_valid1, b->frame1, b->desc2, b->fv_node1, b->fv_off1, b->fv_idx1, b->fv_n_nodes1,
              b->fv_node2, b->fv_off2, b->fv_idx2, b->fv_n_nodes2, b->cap1, b->cap2, b->fv_cap1, b->fv_cap2, b->nnratio,
              d_match, d_nmatches, b->mp_valid2, b->frame2, kf};
    hipStream_t st = (hipStream_t)stream;
    ORB_HIP_TRY(hipMemsetAsync(d_nmatches, 0, (size_t)b->n_pairs * 4, st));
    ORB_HIP_TRY(hipMemsetAsync(d_match, 0xff, (size_t)b->n_pairs * (kf ? b->cap1 : b->cap2) * 4, st));
    const int gx = (std::min(b->fv_cap1, 256) + 3) / 4;   // wavefronts stride over the keyframe's nodes
    hipLaunchKernelGGL(search_by_bow_kernel, dim3((unsigned)gx, (unsigned)b->n_pairs), dim3(256), 0, st, a);
    ORB_HIP_TRY(hipGetLastError());
    if (b->check_orientation && !kf) {
        // CheckOrientation(keyframe->keypointsUn, frame.keypointsUn, matchIds, matches) (:512-513) on the
        // frame-indexed result: bin of angle1[idx1] - angle2[idx2], matches[idx2] erased
        hipLaunchKernelGGL(check_orientation_kernel, dim3((unsigned)b->n_pairs), dim3(256), 0, st, &b->kps2[0].angle, 7,
                           b->cap2, b->counts2, &b->kps1[0].angle, 7, b->cap1, b->frame1, d_match, b->cap2, d_nmatches,
                           (const int32_t*)nullptr);
        ORB_HIP_TRY(hipGetLastError());
    } else if (b->check_orientation) {
        // CheckOrientation(keypoints2, keypoints1, matchIds = (bestIdx2, idx1), matches12) (:762-763): bin of
        // angle2[idx2] - angle1[idx1], matches12[idx1] erased (the query-indexed form, A = kf1)
        hipLaunchKernelGGL(check_orientation_kernel, dim3((unsigned)b->n_pairs), dim3(256), 0, st, &b->kps1[0].angle, 7,
                           b->cap1, b->counts1, &b->kps2[0].angle, 7, b->cap2, b->frame2, d_match, b->cap1, d_nmatches,
                           b->frame1);
        ORB_HIP_TRY(hipGetLastError());
    }
    return ORB_OK;
}

int orbm_search_by_bow_batch_device(const orbm_bow_batch* b, int32_t* d_match, int32_t* d_nmatches, void* stream) {
    return search_by_bow(b, 0, d_match, d_nmatches, stream);
}

int orbm_search_by_bow_kf_batch_device(const orbm_bow_batch* b, int32_t* d_match12, int32_t* d_nmatches, void* stream) {
    return search_by_bow(b, 1, d_match12, d_nmatches, stream);
}

int orbm_search_for_triangulation_batch_device(const orbm_tri_batch* b, int32_t* d_match12, int32_t* d_nmatches,
                                               void* stream) {
    ORB_CHECK_ARG(b && d_match12 && d_nmatches, "null argument");
    ORB_CHECK_ARG(b->n_pairs >= 0 && b->cap1 > 0 && b->cap2 > 0, "bad pair count / capacities");
    ORB_CHECK_ARG(b->n_levels > 0 && b->n_levels <= ORBM_TRI_MAX_LEVELS && b->scale_factors2 && b->sigma2,
                  "n_levels must be 1..ORBM_TRI_MAX_LEVELS with host scale / sigma2 tables");
    if (b->n_pairs == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kps1 && b->desc1 && b->counts1 && b->kps2 && b->desc2 && b->counts2 && b->F12 && b->ep2,
                  "null keyframe arrays");
    const bool fv1 = b->fv_node1 || b->fv_off1 || b->fv_idx1 || b->fv_n_nodes1;
    const bool fv2 = b->fv_node2 || b->fv_off2 || b->fv_idx2 || b->fv_n_nodes2;
    ORB_CHECK_ARG(fv1 == fv2, "give FeatureVectors for both keyframe sets or for neither");
    if (fv1)
        ORB_CHECK_ARG(b->fv_node1 && b->fv_off1 && b->fv_idx1 && b->fv_n_nodes1 && b->fv_node2 && b->fv_off2 &&
                          b->fv_idx2 && b->fv_n_nodes2 && b->fv_cap1 > 0 && b->fv_cap2 > 0,
                      "incomplete FeatureVector arrays");
    ORB_CHECK_ARG(b->n_pairs <= 65535, "too many pairs in one launch");
    TriTables t{};
    for (int l = 0; l < b->n_levels; l++) {
        t.scale2[l] = b->scale_factors2[l];
        t.sigma2[l] = b->sigma2[l];
    }
    t.n_levels = b->n_levels;
    TriArgs a{b->kps1, b->desc1, b->counts1, b->uright1, b->has_mappoint1, b->kps2, b->desc2, b->counts2, b->uright2,
              b->has_mappoint2, b->frame1, b->frame2, b->F12, b->ep2, b->fv_node1, b->fv_off1, b->fv_idx1,
              b->fv_n_nodes1, b->fv_node2, b->fv_off2, b->fv_idx2, b->fv_n_nodes2, b->cap1, b->cap2, b->fv_cap1,
              b->fv_cap2, b->only_stereo ? 1 : 0, d_match12, d_nmatches};
    hipStream_t st = (hipStream_t)stream;
    ORB_HIP_TRY(hipMemsetAsync(d_nmatches, 0, (size_t)b->n_pairs * 4, st));
    if (fv1) {
        ORB_HIP_TRY(hipMemsetAsync(d_match12, 0xff, (size_t)b->n_pairs * b->cap1 * 4, st));
        hipLaunchKernelGGL(tri_fv_kernel, dim3((unsigned)b->n_pairs), dim3(256), 0, st, a, t);
    } else {
        ORB_CHECK_ARG(b->cap2 <= 65535, "cap2 must be <= 65535 for the all-pairs search");
        if (tri_mm() && b->cap2 <= 8192) {   // matrix-core path
            const int nsplit = tri_split();
            const size_t lds = (size_t)(7 * TRI_ROWS + 4 * TRI_POOL + 2 * 2 * 2 * 64 * 4 + ((b->cap2 + 31) & ~31)) * 4;
            const int nqb = (b->cap1 + TRI_ROWS - 1) / TRI_ROWS;
            if (nsplit > 1) ORB_HIP_TRY(hipMemsetAsync(d_match12, 0xff, (size_t)b->n_pairs * b->cap1 * 4, st));
            hipLaunchKernelGGL(tri_mm_kernel, dim3((unsigned)(nqb * nsplit), (unsigned)b->n_pairs), dim3(256), lds, st, a,
                               t, nsplit);
            ORB_HIP_TRY(hipGetLastError());
            if (nsplit > 1) {
                hipLaunchKernelGGL(tri_finalize_kernel, dim3((unsigned)((b->cap1 + 255) / 256), (unsigned)b->n_pairs),
                                   dim3(256), 0, st, d_match12, b->cap1, d_nmatches);
                ORB_HIP_TRY(hipGetLastError());
            }
            return ORB_OK;
        }
        // keys (d << 16) | (0xFFFF - j) merged with atomicMin from 0xFFFFFFFF (no candidate)
        ORB_HIP_TRY(hipMemsetAsync(d_match12, 0xff, (size_t)b->n_pairs * b->cap1 * 4, st));
        const int nqb = (b->cap1 + 255) / 256, nseg = (b->cap2 + TRI_SEG - 1) / TRI_SEG;
        hipLaunchKernelGGL(tri_all_kernel, dim3((unsigned)(nqb * nseg), (unsigned)b->n_pairs), dim3(256), 0, st, a, t,
                           nqb);
        ORB_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(tri_finalize_kernel, dim3((unsigned)nqb, (unsigned)b->n_pairs), dim3(256), 0, st, d_match12,
                           b->cap1, d_nmatches);
    }
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

int orbm_search_for_triangulation(const orbm_tri_frame* kf1, const orbm_tri_frame* kf2, const float* F12,
                                  const float* ep2, const float* scale2, const float* sigma2, int n_levels,
                                  int only_stereo, int32_t* match12, int32_t* nmatches) {
    ORB_CHECK_ARG(kf1 && kf2 && F12 && ep2 && scale2 && sigma2 && match12 && n_levels > 0, "null argument");
    for (int i = 0; i < kf1->n; i++) match12[i] = -1;
    if (nmatches) *nmatches = 0;
    // FeatureVectorIterator (:406-450): walk the two ascending node lists; queries are the
    // kf1 features of shared nodes without a MapPoint (and stereo when onlyStereo).
    std::vector<TriQuery> qs;
    int a = 0, b = 0;
    while (a < kf1->n_nodes && b < kf2->n_nodes) {
        if (kf1->node_id[a] == kf2->node_id[b]) {
            for (int u = kf1->node_off[a]; u < kf1->node_off[a + 1]; u++) {
                const int i1 = kf1->indices[u];
                ORB_CHECK_ARG(i1 >= 0 && i1 < kf1->n, "kf1 feature index out of range");
                if (kf1->has_mappoint[i1]) continue;
                if (only_stereo && !(kf1->uright[i1] >= 0)) continue;
                qs.push_back(TriQuery{i1, kf2->node_off[b], kf2->node_off[b + 1]});
            }
            a++;
            b++;
        } else if (kf1->node_id[a] < kf2->node_id[b]) {
            a++;
        } else {
            b++;
        }
    }
    for (int o = 0; o < kf2->n; o++) ORB_CHECK_ARG(kf2->octave[o] >= 0 && kf2->octave[o] < n_levels, "bad octave");
    if (qs.empty()) return ORB_OK;
    const int n1 = kf1->n, n2 = kf2->n, ni2 = kf2->node_off[kf2->n_nodes];
    // one device slab: queries | kf1 xy,ur,desc | kf2 xy,oct,ur,mp,desc,idx | F | scale | sigma | out
    std::vector<size_t> sz = {qs.size() * sizeof(TriQuery), (size_t)n1 * 8, (size_t)n1 * 4, (size_t)n1 * 32,
                              (size_t)n2 * 8, (size_t)n2 * 4, (size_t)n2 * 4, (size_t)n2, (size_t)n2 * 32,
                              (size_t)std::max(ni2, 1) * 4, 36, (size_t)n_levels * 4, (size_t)n_levels * 4,
                              (size_t)n1 * 4};
    std::vector<size_t> off(sz.size());
    size_t tot = 0;
    for (size_t i = 0; i < sz.size(); i++) { off[i] = tot; tot += align_up(std::max<size_t>(sz[i], 1), 256); }
    DevBuf& s = g_scratch.o2;
    int rc;
    if ((rc = s.reserve(tot))) return rc;
    char* base = s.as<char>();
    const void* src[] = {qs.data(), kf1->kp_xy, kf1->uright, kf1->desc, kf2->kp_xy, kf2->octave, kf2->uright,
                         kf2->has_mappoint, kf2->desc, kf2->indices, F12, scale2, sigma2};
    for (int i = 0; i < 13; i++)
        if (sz[i]) ORB_HIP_TRY(hipMemcpy(base + off[i], src[i], sz[i], hipMemcpyHostToDevice));
    const int nq = (int)qs.size();
    ORB_HIP_TRY(hipMemset(base + off[13], 0xff, sz[13]));   // -1: no match
    hipLaunchKernelGGL(triangulation_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, (hipStream_t)0,
                       (const TriQuery*)(base + off[0]), nq, (const float*)(base + off[1]),
                       (const uint8_t*)(base + off[3]), (const float*)(base + off[4]),
                       (const int32_t*)(base + off[5]), (const float*)(base + off[6]),
                       (const uint8_t*)(base + off[7]), (const uint8_t*)(base + off[8]),
                       (const int32_t*)(base + off[9]), (const float*)(base + off[2]), (const float*)(base + off[10]),
                       ep2[0], ep2[1], (const float*)(base + off[11]), (const float*)(base + off[12]), only_stereo,
                       (int32_t*)(base + off[13]));
    ORB_HIP_TRY(hipGetLastError());
    ORB_HIP_TRY(hipMemcpy(match12, base + off[13], (size_t)n1 * 4, hipMemcpyDeviceToHost));
    int nm = 0;
    for (int i = 0; i < n1; i++) nm += match12[i] >= 0;
    if (nmatches) *nmatches = nm;
    return ORB_OK;
}

}  // extern "C"
