// orbx.hip — ORBextractor::Extract as gfx950 HIP kernels.
//
// Pipeline for a batch of F frames of identical size (one launch per stage, all frames at once):
//   1. pyramid_level_kernel  x (nlevels-1): cascaded cv::resize INTER_LINEAR 8U
//                             (src/ORBextractor.cc:455-470).  Level 0 is the caller's image.
//   2. fast_cells_kernel     : one workgroup per (frame, 30-px cell): crop -> LDS, FAST-9/16
//                             corner score, cell-local 3x3 NMS at iniThFAST, retry at minThFAST
//                             when the cell is empty (DetectFAST :489-540, cv::FAST [ext]).
//   3. quadtree_kernel       : one workgroup per (frame, level): QuadTreeSuppression (:542-693)
//                             with the reference's std::list order and libstdc++ introsort ties
//                             (qt_sort.h); partitions run wave-parallel, list bookkeeping in LDS.
//   4. describe_kernel       : one wave per kept keypoint: IC_Angle on the raw level (:74-101),
//                             GaussianBlur 7x7 s2 Q8 REFLECT_101 of the 43x43 neighbourhood in
//                             LDS (:799), rotated rBRIEF (:103-140) packed with wave ballots,
//                             octave / size / scale written in the reference's output order.
// Compiled with -ffp-contract=off so every float expression rounds like the reference's
// ISO C++14 build (no FMA contraction).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include <hip/hip_ext.h>

#include "common.h"
#include "qt_sort.h"
#include "sincos_f.h"
#include "stereo.h"

namespace orbamd {

constexpr int MAX_LEVELS = 16;
constexpr int MAX_ZONE = 64;            // max FAST detection-zone side (cellw <= 59 always)
constexpr int MAX_ROOTS = 32;
constexpr int PATCH = 43;               // raw neighbourhood: +-21 (rBRIEF reach 18 + blur 3)
constexpr int HBLUR_W = 37;             // horizontally blurred columns: +-18
constexpr int HBS = 40;                 // LDS row stride of the blurred rows (u16): 20 dwords, 8-byte aligned rows
static_assert(HBLUR_W + 3 <= HBS, "the blur's fourth-column tiles store up to column 39");

__constant__ int c_umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
constexpr int c_umax_h[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};   // compile-time copy
__constant__ int c_gauss[7] = {18, 34, 48, 56, 48, 34, 18};   // OpenCV 4.x bit-exact Q8 taps
// FAST circle (cv::FAST makeOffsets, pattern 16): compile-time so LDS reads use immediate offsets
constexpr int c_circle_dx_h[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int c_circle_dy_h[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

struct LevelDev {
    int w, h, stride;
    long long off;          // byte offset of this level in a frame's pyramid slab (l >= 1)
    int rx, ry, rw, rh;     // ROI = level inset by BORDER 16 (:755-760)
    int ncells, cell_base;
    long long cand_base;    // offset of this level's candidate array in a frame's slab
    int cand_cap;
    int quota, out_cap, out_base;
    int nroots;
    double hx;
    float scale, size;
    int xtab_off, ytab_off;         // resize coefficient tables (l >= 1)
    int tail_x;                     // first column of VResizeLinear's scalar tail (l >= 1; w: none)
    int mt_off;                     // first 16-column block in the matrix-core resize tables (-1: none)
    double ssx, ssy;                // (double)w[l-1] / w[l], (double)h[l-1] / h[l] (l >= 1)
};
// 128 bytes: g.lv[l] is a shift, and the kernels' scalar registers stay where round 4 had them (a
// 136-byte LevelDev made fast_cells' level indexing a multiply and moved its SGPR spills: +3.7 %)
static_assert(sizeof(LevelDev) == 128, "LevelDev stays 128 bytes");

struct Geom {
    int nlevels;
    int ncells_total;
    long long pyr_frame_bytes;
    long long slot_frame;     // candidate slots per frame (sum of per-cell capacities)
    long long cand_frame;     // contiguous candidate entries per frame
    int out_frame;            // selected keypoints per frame (sum of out_cap)
    unsigned of_m;            // n / out_frame = (t + ((n - t) >> of_s1)) >> of_s2, t = mulhi(n, of_m)
    int of_s1, of_s2;         // (round-up magic, exact for every n < 2^31; divmod_of)
    // describe's slot -> level: level q's first slot as u16 field q (q = 0 and unused levels 0x7fff);
    // the level of slot s is the number of fields <= s (SWAR, describe_level)
    unsigned lv_start[MAX_LEVELS / 2];
    LevelDev lv[MAX_LEVELS];
};

// n / g.out_frame for 0 <= n < 2^31 by the host's round-up magic (scalar multiply-high, no
// reciprocal round trip): the describe grid is out_frame selection slots per frame.
__device__ __forceinline__ int divmod_of(const Geom& g, int n) {
    const unsigned t = __umulhi((unsigned)n, g.of_m);
    return (int)((t + (((unsigned)n - t) >> g.of_s1)) >> g.of_s2);
}

// cell_cnt entries: the cell's kept corner count, plus a hint bit for fast_cells' next launch
constexpr int CELL_CNT_MASK = 0xffff, CELL_CNT_INI = 1 << 30;

struct CellDev {
    int level;
    int x0y0;     // x0 | y0 << 16 (crop origin, level coords)
    int zwzh;     // detection zone width | height << 16
    int slot;     // first slot (per-frame candidate-slot index)
};

// ------------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ unsigned long long lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ __forceinline__ int popc64(unsigned long long m) { return __popcll(m); }
// popc(m & lanemask_lt) without a lane mask held in VGPRs: v_mbcnt_lo / v_mbcnt_hi
__device__ __forceinline__ int rank64(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ const uint8_t* level_base(const Geom& g, int l, int f, const uint8_t* in,
                                                      long long in_fstride, int in_step, const uint8_t* pyr,
                                                      int* step) {
    if (l == 0) {
        *step = in_step;
        return in + (long long)f * in_fstride;
    }
    *step = g.lv[l].stride;
    return pyr + (long long)f * g.pyr_frame_bytes + g.lv[l].off;
}

// Orders this wavefront's LDS accesses across lanes (LDS ops of one wave complete in order).
// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs (linear id % 8), each
// with its own 4 MiB L2.  Remap so XCD x runs one contiguous 1/8 of the logical blocks: neighbouring
// cells / tiles / keypoints of a frame then share that XCD's L2 for their overlapping rows instead
// of fetching the same 128-B lines from the fabric on several XCDs.  Bijective for any nb.
__device__ __forceinline__ int xcd_swizzle(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
    return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

// Sum of an int over the 64 lanes, wave-uniform result: DPP within each row of 16 (quad xor 1, xor 2,
// row rotate 4, 8), then the four row sums by v_readlane.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false); }
__device__ __forceinline__ int wave_sum_i32(int v) {
    v += dpp_i32<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_i32<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_i32<0x124>(v);   // row_ror:4
    v += dpp_i32<0x128>(v);   // row_ror:8
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

// v_writelane_b32 (the LLVM intrinsic; this clang has no builtin for it): a wave-uniform value into
// one lane of a register, with the compiler's own hazard handling
extern "C" __device__ uint32_t writelane_u32(uint32_t v, uint32_t lane, uint32_t old) __asm("llvm.amdgcn.writelane.i32");

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Wave-inclusive scan of ints (64 lanes) on DPP: Hillis-Steele inside each row of 16 (row_shr 1, 2,
// 4, 8 with zero fill), then row 1 / 3 add lane 15 of the row before (row_bcast:15) and rows 2 / 3
// add lane 31 (row_bcast:31).  No LDS round trips (a ds_bpermute scan costs six).
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// Block-wide exclusive scan for any blockDim.x that is a multiple of 64 (<= 8 waves). `tmp` >= 8 ints of LDS.
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
    const int w = threadIdx.x >> 6, l = lane_id();
    const int inc = wave_incl_scan(v);
    if (l == 63) tmp[w] = inc;
    __syncthreads();
    int base = 0, tot = 0;
    const int nw = blockDim.x >> 6;
    for (int i = 0; i < nw; i++) {
        if (i < w) base += tmp[i];
        tot += tmp[i];
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// The quadtree's group primitives for its two forms: WV = false, the whole workgroup on one tree
// (workgroup barrier, block scan); WV = true (round 6), one wavefront per tree (no barrier: a wavefront
// runs in lockstep, so an LDS / global write is visible to the wavefront's next read once issued and
// the compiler is kept from reordering across the point; the fence orders global memory as the
// workgroup barrier's does).
template <bool WV>
__device__ __forceinline__ void qt_sync() {
    if constexpr (WV) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
        __syncthreads();
    }
}
template <bool WV>
__device__ __forceinline__ int grp_excl_scan(int v, int* tmp, int* total) {
    if constexpr (WV) {
        const int inc = wave_incl_scan(v);
        *total = __builtin_amdgcn_readlane(inc, 63);
        return inc - v;
    } else {
        return block_excl_scan(v, tmp, total);
    }
}

// ------------------------------------------------------------------------------------------
// 1. pyramid
// ------------------------------------------------------------------------------------------
// cv::resize INTER_LINEAR CV_8UC1 [ext]: horizontal 11-bit fixed point (exact int32), vertical
// with the universal-intrinsics rounding ((b0*(S0>>4))>>16 + (b1*(S1>>4))>>16 + 2) >> 2 up to the
// level's tail_x and (S0*b0 + S1*b1 + 2^21) >> 22 from there.  Default tail mode 0: tail_x = w, the
// vector rounding on every column (OpenCV's uchar VResizeLinear specialisation uses it in its scalar
// tail too); the other modes are sensitivity switches (orbx_set_opencv_compat, oracle resize_tail_x).
// xtab[dx] = {sx0 | sx1 << 16, a0 | a1 << 16}; ytab[dy] = {sy0 | sy1 << 16, b0 | b1 << 16}.
// One workgroup = a 64 x 16 tile of level l (256 threads, 4 output pixels each).  The source
// rectangle of level l-1 it needs is staged in LDS with dword loads; coefficients come from the
// per-level tables.
typedef unsigned short us2 __attribute__((ext_vector_type(2)));   // packed u16 pair

// Vertical taps ((h >> 4) * b) >> 16 on the full-rate 24-bit multiplier: with h4 = (h >> 4) << 4
// (h < 2^20) and b12 = b << 12 (b <= 2048), mulhi(h4, b12) = ((h >> 4) * b * 2^16) >> 32, and the
// masks tell the compiler both operands fit in 24 bits (v_mul_hi_u32_u24 instead of the
// quarter-rate v_mul_hi_u32).
__device__ __forceinline__ uint32_t htap24(uint32_t h) { return h & 0xffff0u; }
// v_mul_hi_u32_u24 on operands the compiler cannot see are < 2^24 (table coefficients b << 12, the
// matrix-core pass's sums): no mask instruction to prove it
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
#ifdef PYR_MULHI_MASK_DIAG   // diagnostic A/B only: the masked compiler form
    return __umulhi(a & 0xffffffu, b & 0xffffffu);
#else
    uint32_t r;
    asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#endif
}
__device__ __forceinline__ uint32_t vcoef24(int b) { return ((uint32_t)b & 0xfffu) << 12; }
// VResizeLinear's scalar loop, FixedPtCast<int, uchar, 22>: (S0*b0 + S1*b1 + 2^21) >> 22 on the full
// horizontal sums (S < 2^20, b <= 2048: both products and the sum fit 32 bits); b24 = b << 12
__device__ __forceinline__ uint32_t vtail(uint32_t h0, uint32_t h1, uint32_t b0_24, uint32_t b1_24) {
    return (__umul24(h0, b0_24 >> 12) + __umul24(h1, b1_24 >> 12) + (1u << 21)) >> 22;
}

// two u8 taps of the 8-byte window (hi:lo) picked by a v_perm selector, as a packed u16 pair
__device__ __forceinline__ us2 pyr_tap(uint32_t hi, uint32_t lo, uint32_t sel) {
    const uint32_t r = __builtin_amdgcn_perm(hi, lo, sel);
    return *reinterpret_cast<const us2*>(&r);
}

constexpr int PYR_TW = 64, PYR_TH = 64;
constexpr int PYR_SW = 144, PYR_SH = 128;   // LDS source tile capacity (scale factor <= ~1.9)

// A tile row's vertical taps, built once per workgroup (round 4): the byte offsets of its two source rows
// in the staged rectangle (first row sy_lo, row stride PYR_SW) and the two coefficients in mulhi24 form
// (b << 12), so a row costs one ds_read_b128 and the address adds instead of ~11 VALU of decoding.
__device__ __forceinline__ int4 pyr_row_taps(int2 yv, int sy_lo) {
    return make_int4(((yv.x & 0xffff) - sy_lo) * PYR_SW, ((yv.x >> 16) - sy_lo) * PYR_SW, (int)vcoef24(yv.y),
                     (int)vcoef24(yv.y >> 16));
}

// Level-l output tile (tx0, ty0, tw x th) from the staged source rectangle S (row stride PYR_SW,
// first byte column xa), the tile's column taps xs_t and its row taps ys_t (pyr_row_taps).  Every
// thread of the workgroup must call it (block-wide vote inside); no barrier follows the vote.
__device__ __forceinline__ void pyr_tile_compute(const Geom& g, const LevelDev& L, int f, uint8_t* pyr,
                                                 const uint8_t* S, const int2* xs_t, const int4* ys_t, int tx0,
                                                 int ty0, int tw, int th, int xa) {
    {
        // 16 threads per 64-px output row (4 px each: two pairs), 16 rows per pass (round 4: the row's
        // table read, address and loop control once per 4 pixels instead of 2).  Both pixels of a pair
        // have their four taps in the 8 LDS bytes from the pair's dword wd (scale <= ~3), so a pair costs
        // two dword reads per source row; v_perm packs a pixel's taps as u16 (S0, S1) and v_dot2_u32_u16
        // with the packed (a0, a1) gives S0*a0 + S1*a1 exactly.  (h >> 4 <= 32640 and the result <= 255:
        // OpenCV's saturations cannot trigger for coefficients summing to 2048.)
        const int q0 = (threadIdx.x & 15) * 4;
        uint32_t sel0[2], sel1[2];
        int wdb[2];
        us2 a0[2], a1[2];
        bool fits = true;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int2 xv0 = xs_t[min(q0 + 2 * j, tw - 1)], xv1 = xs_t[min(q0 + 2 * j + 1, tw - 1)];
            const int s00 = (xv0.x & 0xffff) - xa, s01 = (xv0.x >> 16) - xa;
            const int s10 = (xv1.x & 0xffff) - xa, s11 = (xv1.x >> 16) - xa;
            const int wd = s00 >> 2;
            const int e00 = s00 - 4 * wd, e01 = s01 - 4 * wd, e10 = s10 - 4 * wd, e11 = s11 - 4 * wd;
            fits = fits && max(e01, e11) <= 7 && min(e00, e10) >= 0;
            sel0[j] = (uint32_t)e00 | 0x0c00u | ((uint32_t)e01 << 16) | 0x0c000000u;
            sel1[j] = (uint32_t)e10 | 0x0c00u | ((uint32_t)e11 << 16) | 0x0c000000u;
            wdb[j] = 4 * wd;
            a0[j] = *reinterpret_cast<const us2*>(&xv0.y);
            a1[j] = *reinterpret_cast<const us2*>(&xv1.y);
        }
        if (!__syncthreads_or(!fits)) {   // block-uniform: every thread's taps fit its 8-byte windows
            if (q0 >= tw) return;   // after the block-wide vote: no barrier follows
            const bool full = q0 + 3 < tw;
            uint8_t* dst = pyr + (long long)f * g.pyr_frame_bytes + L.off + tx0 + q0 +
                           (long long)(ty0 + (int)(threadIdx.x >> 4)) * L.stride;
            const long long dstep = 16ll * L.stride;
            // this thread's first column in the scalar tail (<= 0: all four, >= 4: none); the tail
            // loop is a separate instantiation, so columns left of tail_x run the plain loop
            const int tcol = L.tail_x - (tx0 + q0);
            auto rows = [&](auto tail_c) {
                constexpr bool TAIL = decltype(tail_c)::value;
                for (int ty = threadIdx.x >> 4; ty < th; ty += 16, dst += dstep) {
                    const int4 yv = ys_t[ty];
                    const uint32_t b0 = (uint32_t)yv.z, b1 = (uint32_t)yv.w;   // b << 12 (pyr_row_taps)
                    uint32_t out = 0;
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const uint32_t* s0 = reinterpret_cast<const uint32_t*>(S + yv.x + wdb[j]);
                        const uint32_t* s1 = reinterpret_cast<const uint32_t*>(S + yv.y + wdb[j]);
                        const uint32_t w00 = s0[0], w01 = s0[1], w10 = s1[0], w11 = s1[1];
                        const uint32_t r0a = __builtin_amdgcn_udot2(pyr_tap(w01, w00, sel0[j]), a0[j], 0u, false);
                        const uint32_t r1a = __builtin_amdgcn_udot2(pyr_tap(w11, w10, sel0[j]), a0[j], 0u, false);
                        const uint32_t r0b = __builtin_amdgcn_udot2(pyr_tap(w01, w00, sel1[j]), a1[j], 0u, false);
                        const uint32_t r1b = __builtin_amdgcn_udot2(pyr_tap(w11, w10, sel1[j]), a1[j], 0u, false);
                        uint32_t va = (mulhi24(htap24(r0a), b0) + mulhi24(htap24(r1a), b1) + 2) >> 2;
                        uint32_t vb = (mulhi24(htap24(r0b), b0) + mulhi24(htap24(r1b), b1) + 2) >> 2;
                        if (TAIL) {
                            va = 2 * j >= tcol ? vtail(r0a, r1a, b0, b1) : va;
                            vb = 2 * j + 1 >= tcol ? vtail(r0b, r1b, b0, b1) : vb;
                        }
                        out |= (va | (vb << 8)) << (16 * j);
                    }
                    if (full) {
                        *reinterpret_cast<uint32_t*>(dst) = out;   // tx0 + q0 and the row stride: multiples of 4
                    } else {
                        for (int k = 0; k < 3; k++)
                            if (q0 + k < tw) dst[k] = (uint8_t)(out >> (8 * k));
                    }
                }
            };
            // block-uniform: only the tiles that reach the tail run the selecting loop (a per-thread choice
            // made the waves holding both kinds of lane run both loops)
#ifndef PYR_NO_TAIL_DIAG
            if (tx0 + tw > L.tail_x) rows(std::true_type{});
            else
#endif
                rows(std::false_type{});
            return;
        }
    }
    // generic path: 16 threads per 64-px output row segment (4 px each), 16 rows per pass
    const int q0 = (threadIdx.x & 15) * 4;
    if (q0 >= tw) return;
    // (cold path: the column coefficients are re-read from LDS per row to keep registers free for
    // pyramid_tiles_kernel's prefetch)
    uint8_t* dbase = pyr + (long long)f * g.pyr_frame_bytes + L.off + tx0 + q0;
#pragma nounroll
    for (int ty = threadIdx.x >> 4; ty < th; ty += 16) {
        const int4 yv = ys_t[ty];
        const int r0 = yv.x, r1 = yv.y;
        const int b0 = yv.z >> 12, b1 = yv.w >> 12;
        uint32_t packed = 0;
#pragma nounroll
        for (int k = 0; k < 4; k++) {
            const int2 xv = xs_t[min(q0 + k, tw - 1)];
            const int sx0 = (xv.x & 0xffff) - xa, sx1 = (xv.x >> 16) - xa, a0 = xv.y & 0xffff, a1 = xv.y >> 16;
            const int h0 = S[r0 + sx0] * a0 + S[r0 + sx1] * a1;
            const int h1 = S[r1 + sx0] * a0 + S[r1 + sx1] * a1;
            const int s0 = min(h0 >> 4, 32767), s1 = min(h1 >> 4, 32767);
            int v = (((s0 * b0) >> 16) + ((s1 * b1) >> 16) + 2) >> 2;
            if (tx0 + q0 + k >= L.tail_x) v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
            packed |= (uint32_t)(v > 255 ? 255 : v) << (8 * k);
        }
        uint8_t* dst = dbase + (long long)(ty0 + ty) * L.stride;
        if (q0 + 3 < tw) *reinterpret_cast<uint32_t*>(dst) = packed;   // stride % 16 == 0, tx0+q0 % 4 == 0
        else {   // q0 < tw <= q0 + 3
            dst[0] = (uint8_t)packed;
            if (q0 + 1 < tw) dst[1] = (uint8_t)(packed >> 8);
            if (q0 + 2 < tw) dst[2] = (uint8_t)(packed >> 16);
        }
    }
}

// 16-byte staging (every pyramid level; level 0 when the caller's base and step are multiples of
// 16): the source rectangle is fetched as 16-byte pieces with (row, piece) flattened over the 256
// threads, i.e. ~3 loads per thread instead of one dword load per source row.
constexpr int PYR_PF = 5;   // 16-byte pieces per thread: PYR_SH rows x PYR_SW / 16 pieces <= 5 x 256

struct PyrTile {
    int f, tx0, ty0, tw, th, sy_lo, xa, nc, items, mul;   // mul = ceil(2^20 / nc): row = item * mul >> 20
    const uint8_t* src;
    int sstep;
};

__device__ __forceinline__ PyrTile pyr_tile_geom(const Geom& g, int l, int t, int ntx, int nty, const uint8_t* in,
                                                 long long in_fstride, int in_step, uint8_t* pyr) {
    const LevelDev& L = g.lv[l];
    const LevelDev& Ls = g.lv[l - 1];
    PyrTile T;
    const int per = ntx * nty;
    T.f = t / per;
    const int r = t - T.f * per;
    T.ty0 = (r / ntx) * PYR_TH;
    T.tx0 = (r - (r / ntx) * ntx) * PYR_TW;
    T.tw = min(PYR_TW, L.w - T.tx0);
    T.th = min(PYR_TH, L.h - T.ty0);
    const int sx_lo = max(0, (int)floor((T.tx0 + 0.5) * L.ssx - 0.5) - 2);
    const int sx_hi = min(Ls.w - 1, (int)floor((T.tx0 + T.tw - 0.5) * L.ssx - 0.5) + 2);
    T.sy_lo = max(0, (int)floor((T.ty0 + 0.5) * L.ssy - 0.5) - 2);
    const int sy_hi = min(Ls.h - 1, (int)floor((T.ty0 + T.th - 0.5) * L.ssy - 0.5) + 2);
    T.xa = sx_lo & ~15;
    T.nc = ((sx_hi - T.xa) >> 4) + 1;
    T.items = (sy_hi - T.sy_lo + 1) * T.nc;
    T.mul = ((1 << 20) + T.nc - 1) / T.nc;
    T.src = level_base(g, l - 1, T.f, in, in_fstride, in_step, pyr, &T.sstep);
    // workgroup-uniform by construction: keep the tile in SGPRs, not in VGPRs across the compute
    auto u = [](int x) { return __builtin_amdgcn_readfirstlane(x); };
    T.f = u(T.f), T.tx0 = u(T.tx0), T.ty0 = u(T.ty0), T.tw = u(T.tw), T.th = u(T.th), T.sy_lo = u(T.sy_lo);
    T.xa = u(T.xa), T.nc = u(T.nc), T.items = u(T.items), T.mul = u(T.mul), T.sstep = u(T.sstep);
    const unsigned long long sp = (unsigned long long)(uintptr_t)T.src;
    T.src = (const uint8_t*)(uintptr_t)(((unsigned long long)(unsigned)u((int)(sp >> 32)) << 32) |
                                        (unsigned)u((int)(unsigned)sp));
    return T;
}

// piece i -> (row, 16-byte column): rr = (i * mul) >> 20 as a 24-bit high product (i < 2^11,
// mul <= 2^20), c = i - rr * nc as a 24-bit product (full-rate multipliers)
__device__ __forceinline__ int pyr_piece_row(const PyrTile& T, int i) {
    return (int)(__umulhi(((unsigned)i & 0x7ffu) << 12, (unsigned)T.mul & 0xffffffu) & 0x7ffu);
}
__device__ __forceinline__ int mul12(int a, int b) {   // a, b in [0, 4096): one v_mul_u32_u24
    return (int)(((unsigned)a & 0xfffu) * ((unsigned)b & 0xfffu));
}
__device__ __forceinline__ void pyr_piece_load(const PyrTile& T, int i, uint4& v) {
    if (i < T.items) {
        const int rr = pyr_piece_row(T, i), c = i - mul12(rr, T.nc);
        v = *reinterpret_cast<const uint4*>(T.src + __mul24(T.sy_lo + rr, T.sstep) + T.xa + 16 * c);
    }
}

__device__ __forceinline__ void pyr_fetch(const PyrTile& T, int tid, uint4& v0, uint4& v1, uint4& v2, uint4& v3,
                                          uint4& v4) {
    static_assert(PYR_PF == 5, "five pieces per thread");
    pyr_piece_load(T, tid, v0);
    pyr_piece_load(T, tid + 256, v1);
    pyr_piece_load(T, tid + 512, v2);
    pyr_piece_load(T, tid + 768, v3);
    pyr_piece_load(T, tid + 1024, v4);
}

__device__ __forceinline__ void pyr_stage(const PyrTile& T, int tid, uint8_t* S, const uint4& v, int k) {
    const int i = tid + 256 * k;
    if (i < T.items) {
        const int rr = pyr_piece_row(T, i), c = i - mul12(rr, T.nc);
        *reinterpret_cast<uint4*>(&S[mul12(rr, PYR_SW) + 16 * c]) = v;
    }
}

__global__ __launch_bounds__(256) void pyramid_level_kernel(Geom g, int l, const uint8_t* __restrict__ in,
                                                            long long in_fstride, int in_step, uint8_t* pyr,
                                                            const int2* __restrict__ xtab,
                                                            const int2* __restrict__ ytab) {
    __shared__ __attribute__((aligned(16))) uint8_t S[PYR_SH * PYR_SW + 16];   // +16: the 8-byte windows may read past the last row
    __shared__ int2 xs_t[PYR_TW];
    __shared__ int4 ys_t[PYR_TH];
    const LevelDev& L = g.lv[l];
    const LevelDev& Ls = g.lv[l - 1];
    const int gx = gridDim.x, gxy = gridDim.x * gridDim.y;
    const int lb = xcd_swizzle(blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z, gxy * gridDim.z);
    const int f = lb / gxy;
    const int tx0 = (lb % gx) * PYR_TW, ty0 = ((lb % gxy) / gx) * PYR_TH;
    const int tw = min(PYR_TW, L.w - tx0), th = min(PYR_TH, L.h - ty0);
    int sstep;
    const uint8_t* src = level_base(g, l - 1, f, in, in_fstride, in_step, pyr, &sstep);
    const int2* xt = xtab + L.xtab_off;
    const int2* yt = ytab + L.ytab_off;
    // coefficient tables -> LDS (independent of the image loads below)
    // conservative source rectangle from the scale (a superset of the tables' taps; no table
    // round trip before the image loads)
    const int sw = Ls.w, sh = Ls.h;
    const double scx = L.ssx, scy = L.ssy;
    const int sx_lo = max(0, (int)floor((tx0 + 0.5) * scx - 0.5) - 2);
    const int sx_hi = min(sw - 1, (int)floor((tx0 + tw - 0.5) * scx - 0.5) + 2);
    const int sy_lo = max(0, (int)floor((ty0 + 0.5) * scy - 0.5) - 2);
    if ((int)threadIdx.x < tw) xs_t[threadIdx.x] = xt[tx0 + threadIdx.x];
    if ((int)threadIdx.x >= 64 && (int)threadIdx.x - 64 < th)
        ys_t[threadIdx.x - 64] = pyr_row_taps(yt[ty0 + threadIdx.x - 64], sy_lo);
    const int sy_hi = min(sh - 1, (int)floor((ty0 + th - 0.5) * scy - 0.5) + 2);
    const int xa = sx_lo & ~3;
    const int nd = (sx_hi - xa + 4) >> 2;   // dwords per source row (<= PYR_SW / 4 < 64)
    const int nr = sy_hi - sy_lo + 1;
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) | (uintptr_t)sstep) & 3) == 0;
    if (((reinterpret_cast<uintptr_t>(src) | (uintptr_t)sstep) & 15) == 0 && sx_hi - (sx_lo & ~15) < PYR_SW) {
        const PyrTile T = pyr_tile_geom(g, l, lb, gx, gridDim.y, in, in_fstride, in_step, pyr);
        uint4 v0, v1, v2, v3, v4;
        pyr_fetch(T, threadIdx.x, v0, v1, v2, v3, v4);
        pyr_stage(T, threadIdx.x, S, v0, 0);
        pyr_stage(T, threadIdx.x, S, v1, 1);
        pyr_stage(T, threadIdx.x, S, v2, 2);
        pyr_stage(T, threadIdx.x, S, v3, 3);
        pyr_stage(T, threadIdx.x, S, v4, 4);
        __syncthreads();
        pyr_tile_compute(g, L, f, pyr, S, xs_t, ys_t, tx0, ty0, tw, th, T.xa);
        return;
    }
    if (aligned) {
        // wavefront w stages rows w, w + 4, ...; lane = dword of the row.  The row address is
        // wave-uniform (SGPR base + a per-lane column offset), so a load costs no VALU; all of a
        // lane's loads are issued before the LDS stores.
        constexpr int RPW = PYR_SH / 4;
        const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        const int ln = threadIdx.x & 63;
        const int col = min(xa + 4 * ln, (sw - 1) & ~3);   // in-row dword (row stride >= align4(w))
        const uint8_t* rbase = src + (long long)sy_lo * sstep + col;
        uint32_t v[RPW];
#pragma unroll
        for (int k = 0; k < RPW; k++) {   // unconditional (row clamped): straight-line loads
            const int rk = min(wv + 4 * k, nr - 1);
            v[k] = *reinterpret_cast<const uint32_t*>(rbase + (long long)rk * sstep);
        }
        if (ln < nd) {
            uint32_t* drow = reinterpret_cast<uint32_t*>(S) + wv * (PYR_SW / 4) + ln;
#pragma unroll
            for (int k = 0; k < RPW; k++)
                if (wv + 4 * k < nr) drow[k * PYR_SW] = v[k];   // row wv + 4k: (wv + 4k) * PYR_SW / 4 dwords
        }
    } else {   // unaligned caller image (level 0 with an odd base / step): byte loads
        for (int i = threadIdx.x; i < nd * nr; i += blockDim.x) {
            const int r = i / nd, d = i - r * nd;
            const uint8_t* rowp = src + (long long)(sy_lo + r) * sstep;
            const int x = xa + 4 * d;
            uint32_t v = 0;
            for (int q = 0; q < 4; q++)
                if (x + q < sw) v |= (uint32_t)rowp[x + q] << (8 * q);
            *reinterpret_cast<uint32_t*>(&S[r * PYR_SW + 4 * d]) = v;
        }
    }
    __syncthreads();
    pyr_tile_compute(g, L, f, pyr, S, xs_t, ys_t, tx0, ty0, tw, th, xa);
}

// Two cascaded levels in one launch: level l (from level l-1, both in the pyramid slab) and level
// l+1, one workgroup per 64x64 tile of level l+1.  The workgroup computes the level-l rectangle
// its tile's taps need (the conservative rectangle of pyramid_level_kernel, columns from a dword
// boundary) from a staged level-(l-1) rectangle, keeps it in LDS for the level-(l+1) tile and
// writes it to the slab.  Neighbouring workgroups' rectangles overlap by the tap margins; they
// write the same bytes there.  Removes the launch boundary between the two levels and the
// level-l re-read.
constexpr int PP_MAXP = 8;   // level-l row passes per thread
constexpr int PP_MAXC = 96, PP_MAXR = 96;   // level-l rectangle columns / rows the tables hold

__device__ __forceinline__ uint32_t pyr_px_generic(const uint8_t* S, int2 xv, int4 yv, int xa, bool tail) {
    const int r0 = yv.x, r1 = yv.y;
    const int sx0 = (xv.x & 0xffff) - xa, sx1 = (xv.x >> 16) - xa, a0 = xv.y & 0xffff, a1 = xv.y >> 16;
    const int b0 = yv.z >> 12, b1 = yv.w >> 12;
    const int h0 = S[r0 + sx0] * a0 + S[r0 + sx1] * a1;
    const int h1 = S[r1 + sx0] * a0 + S[r1 + sx1] * a1;
    const int s0 = min(h0 >> 4, 32767), s1 = min(h1 >> 4, 32767);
    int v = (((s0 * b0) >> 16) + ((s1 * b1) >> 16) + 2) >> 2;
    if (tail) v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    return (uint32_t)(v > 255 ? 255 : v);
}

__global__ __launch_bounds__(256) void pyramid_pair_kernel(Geom g, int l, const uint8_t* __restrict__ in,
                                                           long long in_fstride, int in_step, uint8_t* pyr,
                                                           const int2* __restrict__ xtab,
                                                           const int2* __restrict__ ytab) {
    __shared__ __attribute__((aligned(16))) uint8_t S[PYR_SH * PYR_SW + 16];
    __shared__ int2 xs1[PP_MAXC], xs2[PYR_TW];
    __shared__ int4 ys1[PP_MAXR], ys2[PYR_TH];
    const LevelDev& L0 = g.lv[l - 1];
    const LevelDev& L1 = g.lv[l];
    const LevelDev& L2 = g.lv[l + 1];
    const int tid = threadIdx.x;
    const int gx = gridDim.x, gxy = gridDim.x * gridDim.y;
    const int lb = xcd_swizzle(blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z, gxy * gridDim.z);
    const int f = lb / gxy;
    const int tx0 = (lb % gx) * PYR_TW, ty0 = ((lb % gxy) / gx) * PYR_TH;
    const int tw = min(PYR_TW, L2.w - tx0), th = min(PYR_TH, L2.h - ty0);
    auto u = [](int x) { return __builtin_amdgcn_readfirstlane(x); };
    // level-l rectangle [c0, c1] x [ay0, ay1] (c0 dword aligned)
    const int ax0 = max(0, (int)floor((tx0 + 0.5) * L2.ssx - 0.5) - 2);
    const int c1 = u(min(L1.w - 1, (int)floor((tx0 + tw - 0.5) * L2.ssx - 0.5) + 2));
    const int ay0 = u(max(0, (int)floor((ty0 + 0.5) * L2.ssy - 0.5) - 2));
    const int ay1 = u(min(L1.h - 1, (int)floor((ty0 + th - 0.5) * L2.ssy - 0.5) + 2));
    const int c0 = u(ax0 & ~3);
    const int ncol = c1 - c0 + 1, nrow = ay1 - ay0 + 1;
    // level-(l-1) rectangle for it, staged as 16-byte pieces
    PyrTile T;
    const int bx0 = max(0, (int)floor((c0 + 0.5) * L1.ssx - 0.5) - 2);
    const int bx1 = min(L0.w - 1, (int)floor((c1 + 0.5) * L1.ssx - 0.5) + 2);
    T.sy_lo = u(max(0, (int)floor((ay0 + 0.5) * L1.ssy - 0.5) - 2));
    const int by1 = min(L0.h - 1, (int)floor((ay1 + 0.5) * L1.ssy - 0.5) + 2);
    T.xa = u(bx0 & ~15);
    T.nc = u(((bx1 - T.xa) >> 4) + 1);
    T.items = u((by1 - T.sy_lo + 1) * T.nc);
    T.mul = u(((1 << 20) + T.nc - 1) / T.nc);
    T.src = level_base(g, l - 1, f, in, in_fstride, in_step, pyr, &T.sstep);   // 16-byte aligned (host)
    {
        uint4 v0, v1, v2, v3, v4;
        pyr_fetch(T, tid, v0, v1, v2, v3, v4);
        if (tid < ncol) xs1[tid] = xtab[L1.xtab_off + c0 + tid];
        if (tid < nrow) ys1[tid] = pyr_row_taps(ytab[L1.ytab_off + ay0 + tid], T.sy_lo);
        if (tid < tw) xs2[tid] = xtab[L2.xtab_off + tx0 + tid];
        if (tid < th) ys2[tid] = pyr_row_taps(ytab[L2.ytab_off + ty0 + tid], ay0);
        pyr_stage(T, tid, S, v0, 0);
        pyr_stage(T, tid, S, v1, 1);
        pyr_stage(T, tid, S, v2, 2);
        pyr_stage(T, tid, S, v3, 3);
        pyr_stage(T, tid, S, v4, 4);
    }
    __syncthreads();
    // level l: thread = (quad q of 4 columns, first row r0), rows r0 + p * rpp
    const int ncq = (ncol + 3) >> 2, rpp = 256 / ncq;
    const int q = tid % ncq, r0 = tid / ncq;
    const bool act = r0 < rpp;
    uint32_t out[PP_MAXP];
    if (act) {
        uint32_t sel0[2], sel1[2], wdv[2];
        us2 a0[2], a1[2];
        int2 xv[4];
        bool fits = true;
#pragma unroll
        for (int k = 0; k < 4; k++) xv[k] = xs1[min(4 * q + k, ncol - 1)];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int2 xv0 = xv[2 * j], xv1 = xv[2 * j + 1];
            const int s00 = (xv0.x & 0xffff) - T.xa, s01 = (xv0.x >> 16) - T.xa;
            const int s10 = (xv1.x & 0xffff) - T.xa, s11 = (xv1.x >> 16) - T.xa;
            const int wd = s00 >> 2;
            const int e00 = s00 - 4 * wd, e01 = s01 - 4 * wd, e10 = s10 - 4 * wd, e11 = s11 - 4 * wd;
            fits = fits && max(e01, e11) <= 7 && min(e00, e10) >= 0;
            sel0[j] = (uint32_t)e00 | 0x0c00u | ((uint32_t)e01 << 16) | 0x0c000000u;
            sel1[j] = (uint32_t)e10 | 0x0c00u | ((uint32_t)e11 << 16) | 0x0c000000u;
            wdv[j] = (uint32_t)wd;
            a0[j] = *reinterpret_cast<const us2*>(&xv0.y);
            a1[j] = *reinterpret_cast<const us2*>(&xv1.y);
        }
        // this thread's first level-l column in the scalar tail (<= 0: all four, >= 4: none)
        const int tcol = L1.tail_x - (c0 + 4 * q);
        auto rows = [&](auto tail_c) {
            constexpr bool TAIL = decltype(tail_c)::value;
#pragma unroll
            for (int pp = 0; pp < PP_MAXP; pp++) {
                const int r = r0 + pp * rpp;
                out[pp] = 0;
                if (r >= nrow) break;
                const int4 yv = ys1[r];
                if (fits) {
                    const uint32_t b0 = (uint32_t)yv.z, b1 = (uint32_t)yv.w;   // b << 12 (pyr_row_taps)
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const uint32_t* s0 = reinterpret_cast<const uint32_t*>(S + yv.x + 4 * (int)wdv[j]);
                        const uint32_t* s1 = reinterpret_cast<const uint32_t*>(S + yv.y + 4 * (int)wdv[j]);
                        const uint32_t w00 = s0[0], w01 = s0[1], w10 = s1[0], w11 = s1[1];
                        const uint32_t r0a = __builtin_amdgcn_udot2(pyr_tap(w01, w00, sel0[j]), a0[j], 0u, false);
                        const uint32_t r1a = __builtin_amdgcn_udot2(pyr_tap(w11, w10, sel0[j]), a0[j], 0u, false);
                        const uint32_t r0b = __builtin_amdgcn_udot2(pyr_tap(w01, w00, sel1[j]), a1[j], 0u, false);
                        const uint32_t r1b = __builtin_amdgcn_udot2(pyr_tap(w11, w10, sel1[j]), a1[j], 0u, false);
                        uint32_t va = (mulhi24(htap24(r0a), b0) + mulhi24(htap24(r1a), b1) + 2) >> 2;
                        uint32_t vb = (mulhi24(htap24(r0b), b0) + mulhi24(htap24(r1b), b1) + 2) >> 2;
                        if (TAIL) {
                            va = 2 * j >= tcol ? vtail(r0a, r1a, b0, b1) : va;
                            vb = 2 * j + 1 >= tcol ? vtail(r0b, r1b, b0, b1) : vb;
                        }
                        out[pp] |= (va | (vb << 8)) << (16 * j);
                    }
                } else {   // taps outside the 8-byte windows (not at the supported scale factors)
#pragma unroll
                    for (int k = 0; k < 4; k++) out[pp] |= pyr_px_generic(S, xv[k], yv, T.xa, k >= tcol) << (8 * k);
                }
            }
        };
#ifndef PYR_NO_TAIL_DIAG   // diagnostic A/B only (drops the tail's formula): the price of its instantiation
        if (c1 >= L1.tail_x) rows(std::true_type{});   // block-uniform, as in pyr_tile_compute
        else
#endif
            rows(std::false_type{});
    }
    __syncthreads();   // every read of the level-(l-1) rectangle done: S now takes the level-l one
    if (act) {
        uint8_t* lrow = pyr + (long long)f * g.pyr_frame_bytes + L1.off + c0 + 4 * q;
        // columns past c1 hold clamped-coefficient values: never written to the slab (a
        // neighbouring workgroup writes the true ones there)
        const bool full = c0 + 4 * q + 3 <= c1;
#pragma unroll
        for (int pp = 0; pp < PP_MAXP; pp++) {
            const int r = r0 + pp * rpp;
            if (r >= nrow) break;
            *reinterpret_cast<uint32_t*>(&S[r * PYR_SW + 4 * q]) = out[pp];
            uint8_t* dst = lrow + __mul24(ay0 + r, L1.stride);
            if (full) {
                *reinterpret_cast<uint32_t*>(dst) = out[pp];
            } else {
                for (int k = 0; k < 3; k++)
                    if (c0 + 4 * q + k <= c1) dst[k] = (uint8_t)(out[pp] >> (8 * k));
            }
        }
    }
    __syncthreads();
    pyr_tile_compute(g, L2, f, pyr, S, xs2, ys2, tx0, ty0, tw, th, c0);
}

// Host check of pyramid_pair_kernel's capacities at the level pair's scale factors (with margins
// for the floor / alignment slack of the conservative rectangles).
static bool pyr_pair_fits(const Geom& g, int l) {
    const double s1x = g.lv[l].ssx, s1y = g.lv[l].ssy, s2x = g.lv[l + 1].ssx, s2y = g.lv[l + 1].ssy;
    const int ncol = (int)std::ceil(PYR_TW * s2x) + 10, nrow = (int)std::ceil(PYR_TH * s2y) + 7;
    const int ncq = (ncol + 3) / 4, rpp = 256 / ncq;
    const int bw = (int)std::ceil(ncol * s1x) + 7 + 15, bh = (int)std::ceil(nrow * s1y) + 7;
    return ncol + 8 <= PYR_SW && nrow <= PYR_SH && ncol <= PP_MAXC && nrow <= PP_MAXR && (nrow + rpp - 1) / rpp <= PP_MAXP &&
           bw <= PYR_SW && bh <= PYR_SH &&
           bh * ((bw + 15) / 16) <= PYR_PF * 256;
}

// ---- the level pair with the horizontal pass on the matrix cores (round 5) ----
// VResizeLinear's horizontal sums for a block of 16 output columns (M) and 16 source rows (N) are
// one v_mfma_f32_16x16x32_f16 over K = 32 source columns from kb (the block's first tap rounded
// down to a dword):
//   A[m][k] = a0 at k = sx0 - kb, a1 at k = sx1 - kb (integers <= 2049: exact in f16),
//   B[k][n] = 1024 + pixel (the byte under an f16 0x64 high byte: one v_perm per two pixels),
//   C[m]    = 2^23 - 1024 (a0 + a1).
// Every partial sum is an integer below 2^24, so D = 2^23 + (S0 a0 + S1 a1) exactly and its float
// bits carry the horizontal sum in bits 0..19 (h < 2^19).  A source row's sums are computed once
// (the VALU form computes them for each of the ~1.7 output rows that read the row) into a
// per-wavefront ring of 48 rows; the vertical taps stay on the VALU (their per-term truncation is
// not a product).  A and C come from a per-level table built on the host (one 2 KiB entry per
// 16-column block); a wavefront owns one block at a time, so the ring needs no workgroup barrier.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float pf4v __attribute__((ext_vector_type(4)));
struct PyrMfmaLane { uint32_t a[4]; float c[4]; };   // one lane's A fragment (8 f16) and C (4 f32)
constexpr int PM_MAXB1 = 6;      // level-l rectangle blocks (96 columns)
constexpr int PM_TAB = PYR_SH;   // per-source-row table entries (rows of S)
constexpr int PM_MAXU1 = 12;     // level-l units (block, 15-row group) per wavefront


// One unit: source rows 15 k .. 15 k + 15 of S (16 rows, the last shared with the next group) x a
// 16-column block.  The product leaves lane (n, g) with the horizontal sums of source row 15 k + n,
// columns 4 g .. 4 g + 3; at scale factors >= 1 a source row is the upper tap sy0 of at most one
// output row, so lane n (n < 15) computes that output row from its own sums and lane n + 1's (DPP
// row_shl:1) -- the vertical pass needs no exchange through LDS.  sp: this lane's S address of
// group 0 (kb - S's first column + 8 g + n * PYR_SW); tab[r] = {byte offset of r's output row in the
// output level (-1: none), b0 << 12, b1 << 12, the row in the rectangle}.  Returns the lane's 4 pixels
// (meaningful when tab[15 k + n].x >= 0 and n < 15).
template <bool TAIL>
__device__ __forceinline__ uint32_t pyr_mfma_unit(const uint8_t* sp, int k, const h8v& A, const pf4v& C, const int4& t,
                                                  int tcol) {
    const int g = lane_id() >> 4;
    constexpr uint32_t hmask = TAIL ? 0xfffffu : 0xffff0u;   // the tail's formula needs the full sum
    const uint2 w = *reinterpret_cast<const uint2*>(sp + k * (15 * PYR_SW));
    const uint4 bu = make_uint4(__builtin_amdgcn_perm(0x64646464u, w.x, 0x04010400u),
                                __builtin_amdgcn_perm(0x64646464u, w.x, 0x04030402u),
                                __builtin_amdgcn_perm(0x64646464u, w.y, 0x04010400u),
                                __builtin_amdgcn_perm(0x64646464u, w.y, 0x04030402u));
    const pf4v d = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, __builtin_bit_cast(h8v, bu), C, 0, 0, 0);
    const uint32_t b0 = (uint32_t)t.y, b1 = (uint32_t)t.z;
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t h0 = __float_as_uint(d[j]) & hmask;
        const uint32_t h1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)h0, 0x101, 0xf, 0xf, true);   // row_shl:1 (lane 15: 0)
        uint32_t v;
        if (!TAIL) {
            v = (mulhi24(h0, b0) + mulhi24(h1, b1) + 2) >> 2;
        } else {
            v = (mulhi24(h0 & 0xffff0u, b0) + mulhi24(h1 & 0xffff0u, b1) + 2) >> 2;
            v = 4 * g + j >= tcol ? vtail(h0, h1, b0, b1) : v;
        }
        out |= v << (8 * j);
    }
    return out;
}

// A block's A / C fragments from the host table
__device__ __forceinline__ void pyr_mfma_frag(const PyrMfmaLane* tab, h8v& A, pf4v& C) {
    const PyrMfmaLane t = tab[lane_id()];
    A = __builtin_bit_cast(h8v, make_uint4(t.a[0], t.a[1], t.a[2], t.a[3]));
    C = pf4v{t.c[0], t.c[1], t.c[2], t.c[3]};
}

// The per-source-row table of pyr_mfma_unit: output rows [r0, r0 + nrow) of a level (row stride
// ostride) whose source rows start at S row 0 = sy_lo.  Thread y fills source rows sy0(y) ..
// sy0(y + 1) - 1 (thread 0 also the rows above sy0(0), the last thread the rows to PM_TAB).
__device__ __forceinline__ void pyr_mfma_tab(const int2* ytab, int r0, int nrow, int sy_lo, int ostride, int4* tab) {
    const int y = threadIdx.x;
    if (y < nrow) {
        const int2 v = ytab[r0 + y];
        const int s0 = (v.x & 0xffff) - sy_lo;
        const int s0n = y + 1 < nrow ? (ytab[r0 + y + 1].x & 0xffff) - sy_lo : PM_TAB;
        if (y == 0)
            for (int r = 0; r < s0; r++) tab[r] = make_int4(-1, 0, 0, -1);
        tab[s0] = make_int4((r0 + y) * ostride, (int)vcoef24(v.y), (int)vcoef24(v.y >> 16), y);
        for (int r = s0 + 1; r < min(s0n, PM_TAB); r++) tab[r] = make_int4(-1, 0, 0, -1);
    }
}

// 4 output pixels (one dword) at byte column col of a row; partial at the right edge (last: the
// last column that may be written)
__device__ __forceinline__ void pyr_store4(uint8_t* dst, uint32_t o, int col, int last) {
    if (col + 3 <= last) *reinterpret_cast<uint32_t*>(dst) = o;
    else
        for (int k = 0; k < 3; k++)
            if (col + k <= last) dst[k] = (uint8_t)(o >> (8 * k));
}

__global__ __launch_bounds__(256) void pyramid_pair_mfma_kernel(Geom g, int l, const uint8_t* __restrict__ in,
                                                                long long in_fstride, int in_step, uint8_t* pyr,
                                                                const int2* __restrict__ ytab,
                                                                const PyrMfmaLane* __restrict__ mt,
                                                                const int* __restrict__ mkb) {
    __shared__ __attribute__((aligned(16))) uint8_t S[PYR_SH * PYR_SW + 16];
    __shared__ int4 tab1[PM_TAB], tab2[PM_TAB];
    const LevelDev& L0 = g.lv[l - 1];
    const LevelDev& L1 = g.lv[l];
    const LevelDev& L2 = g.lv[l + 1];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gx = gridDim.x, gxy = gridDim.x * gridDim.y;
    const int lb = xcd_swizzle(blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z, gxy * gridDim.z);
    const int f = lb / gxy;
    const int tx0 = (lb % gx) * PYR_TW, ty0 = ((lb % gxy) / gx) * PYR_TH;
    const int tw = min(PYR_TW, L2.w - tx0), th = min(PYR_TH, L2.h - ty0);
    auto u = [](int x) { return __builtin_amdgcn_readfirstlane(x); };
    // level-l rectangle [c0, c1] x [ay0, ay1], c0 on a 16-column block boundary
    const int ax0 = max(0, (int)floor((tx0 + 0.5) * L2.ssx - 0.5) - 2);
    const int c1 = u(min(L1.w - 1, (int)floor((tx0 + tw - 0.5) * L2.ssx - 0.5) + 2));
    const int ay0 = u(max(0, (int)floor((ty0 + 0.5) * L2.ssy - 0.5) - 2));
    const int ay1 = u(min(L1.h - 1, (int)floor((ty0 + th - 0.5) * L2.ssy - 0.5) + 2));
    const int c0 = u(ax0 & ~15);
    const int ncol = c1 - c0 + 1, nrow = ay1 - ay0 + 1;
    PyrTile T;
    const int bx0 = max(0, (int)floor((c0 + 0.5) * L1.ssx - 0.5) - 2);
    const int bx1 = min(L0.w - 1, (int)floor((c1 + 0.5) * L1.ssx - 0.5) + 2);
    T.sy_lo = u(max(0, (int)floor((ay0 + 0.5) * L1.ssy - 0.5) - 2));
    const int by1 = u(min(L0.h - 1, (int)floor((ay1 + 0.5) * L1.ssy - 0.5) + 2));
    T.xa = u(bx0 & ~15);
    T.nc = u(((bx1 - T.xa) >> 4) + 1);
    T.items = u((by1 - T.sy_lo + 1) * T.nc);
    T.mul = u(((1 << 20) + T.nc - 1) / T.nc);
    T.src = level_base(g, l - 1, f, in, in_fstride, in_step, pyr, &T.sstep);   // 16-byte aligned (host)
    // at the level's last row the lower tap is clipped to the upper one (sy1 = sy0): S row sy0 + 1
    // then holds a copy of the last row, so the lane below always supplies the lower tap
    const int rep1 = by1 == L0.h - 1 ? by1 - T.sy_lo : -1;
    {
        uint4 v0, v1, v2, v3, v4;
        pyr_fetch(T, tid, v0, v1, v2, v3, v4);
        pyr_mfma_tab(ytab + L1.ytab_off, ay0, nrow, T.sy_lo, (int)L1.stride, tab1);
        pyr_mfma_tab(ytab + L2.ytab_off, ty0, th, ay0, (int)L2.stride, tab2);
        auto stage = [&](const uint4& v, int k) {
            const int i = tid + 256 * k;
            if (i < T.items) {
                const int rr = pyr_piece_row(T, i), c = i - mul12(rr, T.nc);
                *reinterpret_cast<uint4*>(&S[mul12(rr, PYR_SW) + 16 * c]) = v;
                if (rr == rep1) *reinterpret_cast<uint4*>(&S[mul12(rr + 1, PYR_SW) + 16 * c]) = v;
            }
        };
        stage(v0, 0);
        stage(v1, 1);
        stage(v2, 2);
        stage(v3, 3);
        stage(v4, 4);
    }
    __syncthreads();
    const int n = tid & 15, q = (tid >> 4) & 3;
    // level l: units (block b, group k) block-major, a contiguous range per wavefront; the rows
    // stay in registers until every wavefront is done reading the level-(l-1) rectangle
    const int nb1 = (ncol + 15) >> 4;
    const int g1 = u(((ytab[L1.ytab_off + ay1].x & 0xffff) - T.sy_lo) / 15 + 1);   // groups to the last output's sy0
    const int nu1 = nb1 * g1;
    const int ub = (nu1 * w) >> 2, ue = (nu1 * (w + 1)) >> 2;
    uint32_t o1[PM_MAXU1];
    uint8_t* lbase = pyr + (long long)f * g.pyr_frame_bytes + L1.off + c0 + 4 * q;
    {
        int cur = -1;
        h8v A;
        pf4v C;
        const uint8_t* sp = S;
        int tcol = 16;
#pragma unroll
        for (int i = 0; i < PM_MAXU1; i++) {
            const int un = ub + i;
            if (un >= ue) break;
            const int b = un / g1, k = un - b * g1;
            if (b != cur) {   // wavefront-uniform
                cur = b;
                const int blk = L1.mt_off + ((c0 >> 4) + b);
                pyr_mfma_frag(mt + (long long)blk * 64, A, C);
                sp = S + (mkb[blk] - T.xa + 8 * q + n * PYR_SW);
                tcol = L1.tail_x - (c0 + 16 * b);
            }
            const int4 t = tab1[15 * k + n];   // < PM_TAB (host check)
            o1[i] = tcol < 16 ? pyr_mfma_unit<true>(sp, k, A, C, t, tcol) : pyr_mfma_unit<false>(sp, k, A, C, t, tcol);
            const int col = c0 + 16 * b + 4 * q;
            if (t.x >= 0 && n < 15 && col <= c1) pyr_store4(lbase + 16 * b + t.x, o1[i], col, c1);
        }
    }
    __syncthreads();   // every read of the level-(l-1) rectangle done: S now takes the level-l one
    const int rep2 = ay1 == L1.h - 1 ? nrow - 1 : -1;
#pragma unroll
    for (int i = 0; i < PM_MAXU1; i++) {
        const int un = ub + i;
        if (un >= ue) break;
        const int b = un / g1, k = un - b * g1;
        const int4 t = tab1[15 * k + n];
        if (t.x >= 0 && n < 15) {
            *reinterpret_cast<uint32_t*>(&S[t.w * PYR_SW + 16 * b + 4 * q]) = o1[i];
            if (t.w == rep2) *reinterpret_cast<uint32_t*>(&S[(t.w + 1) * PYR_SW + 16 * b + 4 * q]) = o1[i];
        }
    }
    __syncthreads();
    // level l+1: wavefront w takes block w of the 64-column tile, all its groups
    if (16 * w < tw) {
        const int bc = tx0 + 16 * w;
        const int blk = L2.mt_off + (bc >> 4);
        h8v A;
        pf4v C;
        pyr_mfma_frag(mt + (long long)blk * 64, A, C);
        const uint8_t* sp = S + (mkb[blk] - c0 + 8 * q + n * PYR_SW);
        const int col = bc + 4 * q;
        const int tcol = L2.tail_x - bc;
        const int g2 = u(((ytab[L2.ytab_off + ty0 + th - 1].x & 0xffff) - ay0) / 15 + 1);
        uint8_t* dbase = pyr + (long long)f * g.pyr_frame_bytes + L2.off + col;
        const int last = tx0 + tw - 1;
        auto run = [&](auto tail_c) {
            constexpr bool TAIL = decltype(tail_c)::value;
            for (int k = 0; k < g2; k++) {
                const int4 t = tab2[15 * k + n];
                const uint32_t o = pyr_mfma_unit<TAIL>(sp, k, A, C, t, tcol);
                if (t.x >= 0 && n < 15 && col <= last) pyr_store4(dbase + t.x, o, col, last);
            }
        };
        if (tcol < 16) run(std::true_type{});
        else run(std::false_type{});
    }
}

// FAST's first-cell hint for the next launch: bit 31 of every strip descriptor = the CELL_CNT_INI bit of
// its first cell in frame 0 (cell_cnt's frame-0 slots).  One thread per strip, once per batch after every
// stage of it (launch_fast_hint).
__global__ void fast_hint_kernel(int2* __restrict__ strips, const int* __restrict__ cell_cnt, int nstrips) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nstrips) return;
    const int2 sd = strips[s];
    const unsigned bit = (cell_cnt[sd.x] & CELL_CNT_INI) ? 0x80000000u : 0u;
    strips[s].y = (int)(((unsigned)sd.y & 0x7fffffffu) | bit);
}

// f16 bits of an integer 0 <= v <= 2048 (exact: at most 11 significant bits)
static uint16_t f16_of_int(int v) {
    if (v <= 0) return 0;
    int e = 0;
    while ((2 << e) <= v) e++;   // v in [2^e, 2^(e+1))
    const int m = e >= 10 ? (v - (1 << e)) >> (e - 10) : (v - (1 << e)) << (10 - e);
    return (uint16_t)(((e + 15) << 10) | m);
}

// A / C fragments of pyramid_pair_mfma_kernel for one level's columns (xt: its xtab entries, dw
// columns), appended to mt / mkb; returns the level's first block, or -1 when a block's taps do
// not fit K = 32 from its dword-aligned first tap (scale factors above ~1.7).
static int pyr_mfma_tables(const int2* xt, int dw, std::vector<PyrMfmaLane>& mt, std::vector<int>& mkb) {
    const int nb = (dw + 15) / 16;
    std::vector<PyrMfmaLane> lanes((size_t)nb * 64);
    std::vector<int> kbs(nb);
    for (int j = 0; j < nb; j++) {
        const int kb = (xt[16 * j].x & 0xffff) & ~7;   // 8-byte aligned: the B fragments are ds_read_b64
        kbs[j] = kb;
        for (int ln = 0; ln < 64; ln++) {
            PyrMfmaLane& t = lanes[(size_t)j * 64 + ln];
            const int c = 16 * j + (ln & 15), gq = ln >> 4;
            uint16_t hv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (c < dw) {
                const int sx0 = xt[c].x & 0xffff, sx1 = xt[c].x >> 16, a0 = xt[c].y & 0xffff, a1 = xt[c].y >> 16;
                const int e0 = sx0 - kb, e1 = sx1 - kb;
                if (e0 < 0 || e1 < e0 || e1 > 31 || a0 < 0 || a1 < 0 || a0 + a1 > 4096) return -1;
                for (int k = 0; k < 8; k++) {
                    const int kk = 8 * gq + k;
                    const int wv = (kk == e0 ? a0 : 0) + (kk == e1 ? a1 : 0);
                    if (wv > 2048) return -1;
                    hv[k] = f16_of_int(wv);
                }
            }
            for (int k = 0; k < 4; k++) t.a[k] = (uint32_t)hv[2 * k] | ((uint32_t)hv[2 * k + 1] << 16);
            for (int r = 0; r < 4; r++) {
                const int cm = 16 * j + 4 * gq + r;
                const int sum = cm < dw ? (xt[cm].y & 0xffff) + (xt[cm].y >> 16) : 0;
                t.c[r] = (float)(8388608 - 1024 * sum);
            }
        }
    }
    const int off = (int)mkb.size();
    mt.insert(mt.end(), lanes.begin(), lanes.end());
    mkb.insert(mkb.end(), kbs.begin(), kbs.end());
    return off;
}

// pyramid_pair_mfma_kernel's geometry replayed for every tile of the pair (l, l+1): the staged
// rectangles fit S, every block's K window lies inside S's rows, one output row per source row, and
// the 15-row groups (and their tables) inside S.
static bool pyr_mfma_pair_fits(const Geom& g, int l, const std::vector<int>& mkb, const std::vector<int2>& ytab) {
    const LevelDev &L0 = g.lv[l - 1], &L1 = g.lv[l], &L2 = g.lv[l + 1];
    if (L1.mt_off < 0 || L2.mt_off < 0) return false;
    auto fl = [](double v) { return (int)std::floor(v); };
    int max_rows = 0, max_nc = 0, max_nb1 = 0, max_g1 = 0;
    for (int ty0 = 0; ty0 < L2.h; ty0 += PYR_TH) {
        const int th = std::min(PYR_TH, L2.h - ty0);
        const int ay0 = std::max(0, fl((ty0 + 0.5) * L2.ssy - 0.5) - 2);
        const int ay1 = std::min(L1.h - 1, fl((ty0 + th - 0.5) * L2.ssy - 0.5) + 2);
        const int nrow = ay1 - ay0 + 1;
        const int sy_lo = std::max(0, fl((ay0 + 0.5) * L1.ssy - 0.5) - 2);
        const int by1 = std::min(L0.h - 1, fl((ay1 + 0.5) * L1.ssy - 0.5) + 2);
        if (nrow > PP_MAXR || by1 - sy_lo + 1 > PYR_SH) return false;
        max_rows = std::max(max_rows, by1 - sy_lo + 1);
        max_g1 = std::max(max_g1, ((ytab[L1.ytab_off + ay1].x & 0xffff) - sy_lo) / 15 + 1);
        // per output row: sy0 strictly increasing (one output row per source row), sy1 = sy0 + 1 except
        // at the level's last row (clipped: S holds a copy there); the groups' rows and the copy in S
        auto rows_ok = [&](const LevelDev& L, const LevelDev& Ls, int r0, int nr, int lo, int staged) {
            int prev = -1;
            for (int y = 0; y < nr; y++) {
                const int2 v = ytab[L.ytab_off + r0 + y];
                const int s0 = (v.x & 0xffff) - lo, s1 = (v.x >> 16) - lo;
                if (s0 <= prev || s0 < 0 || !(s1 == s0 + 1 || (s1 == s0 && (v.x >> 16) == Ls.h - 1))) return false;
                if (s1 >= staged) return false;
                prev = s0;
            }
            const int groups = prev / 15 + 1;
            return 15 * groups < PM_TAB && 15 * groups < PYR_SH && staged + 1 <= PYR_SH;
        };
        if (!rows_ok(L1, L0, ay0, nrow, sy_lo, by1 - sy_lo + 1) || !rows_ok(L2, L1, ty0, th, ay0, nrow)) return false;
    }
    for (int tx0 = 0; tx0 < L2.w; tx0 += PYR_TW) {
        const int tw = std::min(PYR_TW, L2.w - tx0);
        const int ax0 = std::max(0, fl((tx0 + 0.5) * L2.ssx - 0.5) - 2);
        const int c1 = std::min(L1.w - 1, fl((tx0 + tw - 0.5) * L2.ssx - 0.5) + 2);
        const int c0 = ax0 & ~15;
        const int ncol = c1 - c0 + 1;
        const int bx0 = std::max(0, fl((c0 + 0.5) * L1.ssx - 0.5) - 2);
        const int bx1 = std::min(L0.w - 1, fl((c1 + 0.5) * L1.ssx - 0.5) + 2);
        const int xa = bx0 & ~15, nc = ((bx1 - xa) >> 4) + 1;
        if (ncol > 16 * PM_MAXB1 || 16 * nc > PYR_SW) return false;
        max_nb1 = std::max(max_nb1, (ncol + 15) / 16);
        max_nc = std::max(max_nc, nc);
        for (int b = 0; b < (ncol + 15) / 16; b++) {
            const int kbrel = mkb[L1.mt_off + (c0 >> 4) + b] - xa;
            if (kbrel < 0 || kbrel + 32 > PYR_SW) return false;
        }
        for (int b = 0; 16 * b < tw; b++) {   // (c0 is a multiple of 16: kb - c0 stays 8-byte aligned)
            const int kbrel = mkb[L2.mt_off + (tx0 >> 4) + b] - c0;
            if (kbrel < 0 || kbrel + 32 > PYR_SW) return false;
        }
    }
    return max_rows * max_nc <= PYR_PF * 256 && max_nb1 * max_g1 <= 4 * PM_MAXU1;
}

// ------------------------------------------------------------------------------------------
// 2. FAST per cell
// ------------------------------------------------------------------------------------------
// Corner strength M = max over the 16 nine-pixel arcs and both polarities of min |I_p - I_c|.
// A pixel is a FAST-9 corner at threshold t iff M > t, and cornerScore<16> == M - 1 for every
// detected corner (threshold-independent), so one M map serves both the iniThFAST pass and the
// minThFAST retry of DetectFAST.
//
// Cost model (PMC, tools/pmc_ab.sh): the kernel is issue-bound -- time follows the total count of
// instructions a wave issues (VALU + SALU + branch + LDS, about 2 cycles each per SIMD) and the VALU
// pipe's occupancy (v_pk_*, v_perm, v_alignbyte, v_mbcnt, v_cmp take 4 cycles, v_add/v_and/v_or/
// v_bitop3 and the unpacked 16-bit forms 2: tools/probe/issue_probe3).  So the tests below use the
// fewest instructions (packed u16, 2 pixels per instruction), not the cheapest ones, and avoid
// per-pixel branches.
template <int IMM>
__device__ __forceinline__ uint32_t bt3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, IMM); }
constexpr int BT_OR3 = 0xFE;   // a | b | c (truth tables over (a, b, c) = (0xF0, 0xCC, 0xAA))

// Two-of-four pre-test on packed u16 lanes.  A dword w of pixels x..x+3 is used as two words of
// u16 lanes: the even pixels (x, x+2) unpacked, w & 0x00ff00ff, and the odd pixels (x+1, x+3) in
// place, i.e. in each lane's high byte with the even pixel as a low byte.  The odd lanes' thresholds
// carry the low byte that makes the comparison depend on the high byte only:
//   p*256 + q > (v + t)*256 + 255  <=>  p > v + t     (saturated at 0xffff when v + t > 255)
//   (v - t)*256 > p*256 + q        <=>  p < v - t     (saturated at 0 when v < t)
// and max / min of such words order by the high byte first, so the same network serves both halves.
// Pass condition for four circle points at 90-degree steps (p1, p3 opposite; p2, p4 opposite): two
// circle-adjacent ones both brighter than v + t or both darker than v - t, which factors to
// (B1 | B3) & (B2 | B4):  min(max(p1, p3), max(p2, p4)) > hi  or  max(min(p1, p3), min(p2, p4)) < lo.
struct PkThr {
    us2 hi_e, lo_e, hi_o, lo_o;
};
__device__ __forceinline__ us2 u2us(uint32_t a) { return __builtin_bit_cast(us2, a); }
__device__ __forceinline__ uint32_t us2u(us2 a) { return __builtin_bit_cast(uint32_t, a); }
__device__ __forceinline__ us2 pk_even(uint32_t w) { return u2us(w & 0x00ff00ffu); }
__device__ __forceinline__ PkThr pk_thresholds(uint32_t wv, int t) {
    const unsigned short tc = (unsigned short)min(max(t, 0), 255);   // cv::FAST clamps the threshold
    const us2 t1 = {tc, tc}, t8 = {(unsigned short)(tc << 8), (unsigned short)(tc << 8)};
    PkThr r;
    const us2 ve = pk_even(wv);
    r.hi_e = ve + t1;                                                        // <= 510: no wrap
    r.lo_e = __builtin_elementwise_sub_sat(ve, t1);
    r.hi_o = __builtin_elementwise_add_sat(u2us(wv | 0x00ff00ffu), t8);      // (v + t)*256 + 255, saturated
    r.lo_o = __builtin_elementwise_sub_sat(u2us(wv & 0xff00ff00u), t8);      // (v - t)*256, saturated
    return r;
}
// non-zero u16 lanes where the pixel passes
__device__ __forceinline__ us2 pk_two_of_four(us2 p1, us2 p3, us2 p2, us2 p4, us2 hi, us2 lo) {
    const us2 bmax = __builtin_elementwise_min(__builtin_elementwise_max(p1, p3), __builtin_elementwise_max(p2, p4));
    const us2 dmin = __builtin_elementwise_max(__builtin_elementwise_min(p1, p3), __builtin_elementwise_min(p2, p4));
    return __builtin_elementwise_sub_sat(bmax, hi) | __builtin_elementwise_sub_sat(lo, dmin);
}

// Corner strength M (cornerScore<16> + 1, or 0 when not a corner at any threshold) on packed u16
// pairs: lane pair k holds circle positions (k, k + 8), so every min / max of the arc network covers
// two arcs at once; position j >= 8 is the swapped pair j - 8.  The network runs on the raw pixels:
// max over arcs of min(p) - v is the bright strength, v - min over arcs of max(p) the dark one.
__device__ __forceinline__ us2 swap2(us2 a) { return __builtin_shufflevector(a, a, 1, 0); }
// The 16 circle bytes as packed pairs (the compiler packs them with v_perm; ds_read_u8_d16_hi cannot
// be used: with SRAM ECC enabled, as on MI355X, d16 loads zero the other half of the register
// instead of preserving it -- a round-4 attempt failed tests/test_extractor_gpu.py exactly so).
template <int CS>
__device__ __forceinline__ void circle_pairs(const uint8_t* c, int cs, us2 (&D)[8]) {
    const int s = CS != 0 ? CS : cs;
#pragma unroll
    for (int k = 0; k < 8; k++)
        D[k] = us2{(unsigned short)c[c_circle_dy_h[k] * s + c_circle_dx_h[k]],
                   (unsigned short)c[c_circle_dy_h[k + 8] * s + c_circle_dx_h[k + 8]]};
}
template <int CS>
__device__ __forceinline__ int corner_strength_pk(const uint8_t* c, int cs) {
    us2 D[8];
    circle_pairs<CS>(c, cs, D);
    us2 l[8], h[8], l2[8], h2[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {   // arcs of 2
        const us2 n = k + 1 < 8 ? D[k + 1] : swap2(D[k - 7]);
        l[k] = __builtin_elementwise_min(D[k], n);
        h[k] = __builtin_elementwise_max(D[k], n);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {   // arcs of 4
        const us2 nl = k + 2 < 8 ? l[k + 2] : swap2(l[k - 6]);
        const us2 nh = k + 2 < 8 ? h[k + 2] : swap2(h[k - 6]);
        l2[k] = __builtin_elementwise_min(l[k], nl);
        h2[k] = __builtin_elementwise_max(h[k], nh);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {   // arcs of 8
        const us2 nl = k + 4 < 8 ? l2[k + 4] : swap2(l2[k - 4]);
        const us2 nh = k + 4 < 8 ? h2[k + 4] : swap2(h2[k - 4]);
        l[k] = __builtin_elementwise_min(l2[k], nl);
        h[k] = __builtin_elementwise_max(h2[k], nh);
    }
    // arcs of 9 = two overlapping arcs of 8, max / min over all 16, two windows at a time by the lattice
    // identities max(min(a, b), min(b, c)) = min(b, max(a, c)) and min(max(a, b), max(b, c)) =
    // max(b, min(a, c)): 22 packed ops instead of 32
    us2 A, B;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {   // windows starting at j and j + 1 (and j + 8, j + 9)
        const us2 cl = j + 2 < 8 ? l[j + 2] : swap2(l[0]);
        const us2 ch = j + 2 < 8 ? h[j + 2] : swap2(h[0]);
        const us2 wl = __builtin_elementwise_min(l[j + 1], __builtin_elementwise_max(l[j], cl));
        const us2 wh = __builtin_elementwise_max(h[j + 1], __builtin_elementwise_min(h[j], ch));
        A = j == 0 ? wl : __builtin_elementwise_max(A, wl);
        B = j == 0 ? wh : __builtin_elementwise_min(B, wh);
    }
    const int v = c[0];
    const int bright = (int)max(A.x, A.y) - v;   // max over arcs of min(p - v)
    const int dark = v - (int)min(B.x, B.y);     // max over arcs of min(v - p)
    return max(0, max(bright, dark));
}

// One wavefront per (cell, frame).  LDS (sized per launch from the largest cell): the crop
// (zone + 3-px apron, stored one byte right so zone column 0 is dword aligned), a zone map of
// corner strengths, a queue of pre-test passers and the ordered list of corners.
//   1. crop -> LDS with aligned dword loads issued together
//   2. compass pre-test, 4 pixels per lane (SWAR), groups with a passer queued in row-major order
//   3. diagonal pre-test on the queued groups' passers (SWAR), survivors queued per pixel; those get
//      the corner strength densely, 64 at a time; corners are appended in row-major order
//   4. corner strength M (cornerScore + 1) for the corner list; NMS at iniThFAST and minThFAST
//      over the list (3x3, cell-local: neighbours outside the zone count as 0)
//   5. emit the iniThFAST set, or the minThFAST set when it is empty (DetectFAST :527-530)
constexpr int GR_RING = 128;   // pre-test group ring (u32 entries; power of two, >= 64 + 64)
constexpr int FQ2_RING = 512;  // diagonal-filter passer ring (u16 entries; power of two, >= 64 + 256)
constexpr int FAST_CLIST_CAP = 256;   // ordered corner list (cells with more take the zone-scan NMS)

struct FastLds {
    int CS, ZS, crop_bytes, mz_bytes, qcap, ccap;
};

#ifdef ORB_FAST_STAMPS
// diagnostic build: phase stamps of every 64th logical wave (8 words each)
#define FAST_NSAMP 8192
__device__ unsigned long long g_fast_stamps[FAST_NSAMP * 8];
#define FAST_STAMP(k, v)                                                                               \
    do {                                                                                             \
        if (lane == 0 && (lb & 63) == 0 && (lb >> 6) < FAST_NSAMP) g_fast_stamps[(lb >> 6) * 8 + (k)] = (v); \
    } while (0)
#else
#define FAST_STAMP(k, v) do {} while (0)
#endif

// Crop staging.  LDS dword mm of crop row r holds crop cols 4mm-1 .. 4mm+2 (col c at byte c+1), i.e.
// the 4 image bytes starting at q = (y0+r)*step + x0 - 1 + 4mm, built with v_alignbyte from the two
// dword-aligned image words around q.  The (row, dword) pairs are walked flat over the wave's 64
// lanes; the first CROP_PF*64 of them are loaded into registers one cell ahead (the loads of cell
// i+1 are in flight while cell i is processed), the rest (cells wider or taller than ~40 px) are
// loaded and stored synchronously.
constexpr int CROP_PF = 8;
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

struct CropWalk {
    int row, mm, dr, dm, ndl;
    __device__ __forceinline__ CropWalk(int lane, int ndl_) : ndl(ndl_) {
        row = lane / ndl;
        mm = lane - row * ndl;
        dr = 64 / ndl;
        dm = 64 - dr * ndl;
    }
    __device__ __forceinline__ void next() {
        row += dr;
        mm += dm;
        if (mm >= ndl) { mm -= ndl; row++; }
    }
};

struct CropSrc {
    const uint8_t* img;   // level base of the frame (wave-uniform)
    int step, x0, y0, ch, ndl, h;   // h: the level's height
    __device__ __forceinline__ int q(const CropWalk& w) const { return (y0 + w.row) * step + x0 - 1 + 4 * w.mm; }
    __device__ __forceinline__ int mis(int q) const {
        return (int)(((uint32_t)reinterpret_cast<uintptr_t>(img) + (uint32_t)q) & 3u);
    }
    __device__ __forceinline__ u32x2a4 load(int q) const {
        return *reinterpret_cast<const u32x2a4*>(img + (q - mis(q)));
    }
};

__device__ __forceinline__ void crop_prefetch(const CropSrc& c, int lane, u32x2a4 (&v)[CROP_PF]) {
    CropWalk w(lane, c.ndl);
#pragma unroll
    for (int it = 0; it < CROP_PF; it++) {   // unconditional (row clamped): straight-line loads
        CropWalk wc = w;
        wc.row = min(w.row, c.ch - 1);
        v[it] = c.load(c.q(wc));
        w.next();
    }
}

__device__ __forceinline__ void crop_commit(const CropSrc& c, int lane, const u32x2a4 (&v)[CROP_PF], uint8_t* crop,
                                            int CSd) {
    CropWalk w(lane, c.ndl);
#pragma unroll
    for (int it = 0; it < CROP_PF; it++) {
        if (w.row < c.ch) {
            const int q = c.q(w);
            reinterpret_cast<uint32_t*>(crop + w.row * CSd)[w.mm] = __builtin_amdgcn_alignbyte(v[it].y, v[it].x, c.mis(q));
        }
        w.next();
    }
    while (w.row < c.ch) {   // rare: crops larger than CROP_PF*64 dwords
        const int q = c.q(w);
        const u32x2a4 t = c.load(q);
        reinterpret_cast<uint32_t*>(crop + w.row * CSd)[w.mm] = __builtin_amdgcn_alignbyte(t.y, t.x, c.mis(q));
        w.next();
    }
}

// Row-group staging: lanes per crop row LR = 16 (32, 64 for wider crops), row group k covers
// rows RPG*k .. RPG*k + RPG-1.  A group's source address is wave-uniform plus a per-lane constant,
// so a load costs no address VALU; only the realignment (v_alignbyte) and the LDS address remain.
constexpr int CROP_NG = 10;
constexpr int FAST_CROP_SLACK = 3;   // crop rows past the tallest crop: a partial last row group (RPG <= 4)
// groups whose loads are issued together (40 rows at LR = 16)
// LRS = log2(lanes per crop row), a template constant so that with a compile-time crop stride the
// CROP_NG row-group stores share one LDS base address (offset fields) instead of CROP_NG live
// per-lane addresses.
template <int LRS>   // 0: from the crop's row-dword count at run time
__device__ __forceinline__ void crop_stage_rows_t(const CropSrc& c, int lane, uint8_t* crop, int CSd) {
    const int lrs = LRS ? LRS : (c.ndl <= 16 ? 4 : (c.ndl <= 32 ? 5 : 6));   // 0: run time
    const int RPG = 64 >> lrs;
    const int roff = lane >> lrs, d = lane & ((1 << lrs) - 1);
    const bool dok = d < c.ndl;
    const int dd = dok ? d : 0;
    const uint8_t* g0 = c.img + (long long)c.y0 * c.step + (c.x0 - 1);   // wave-uniform
    const int ng = (c.ch + RPG - 1) >> (6 - lrs);
    if ((c.step & 3) == 0) {
        // dword-multiple row step (every pyramid level; level 0 unless the caller's step is odd):
        // the misalignment is one wave-uniform shift, the loads are buffer loads off a scalar
        // resource with a per-lane constant voffset and a per-group soffset (no address VALU),
        // and a partial last group writes into the crop's slack rows (FAST_CROP_SLACK).  The resource
        // ends with the level, so loads of groups past it return 0 instead of needing a clamp, and the
        // first batch stores all CROP_NG groups unconditionally (the crop buffer holds CROP_NG * 4 rows,
        // and groups past the crop only fill rows nothing reads): no per-group scalar control.
        const int m = __builtin_amdgcn_readfirstlane((int)(reinterpret_cast<uintptr_t>(g0) & 3u));
        const int avail = (c.h - c.y0) * c.step - (c.x0 - 1) + m;   // bytes from g0 - m to the level's end
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(g0 - m), 0, avail, 0x00020000);
        const int voff = roff * c.step + 4 * dd;
        uint32_t* lrow = reinterpret_cast<uint32_t*>(crop + roff * CSd) + d;
        const int gstep = RPG * c.step, lstep = RPG * CSd / 4;
        {
            u32x2a4 v[CROP_NG];
#pragma unroll
            for (int k = 0; k < CROP_NG; k++) {
                const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, k * gstep, 0);
                v[k] = u32x2a4{t[0], t[1]};
            }
            if (dok) {
#pragma unroll
                for (int k = 0; k < CROP_NG; k++) lrow[k * lstep] = __builtin_amdgcn_alignbyte(v[k].y, v[k].x, m);
            }
        }
        for (int k0 = CROP_NG; k0 < ng; k0 += CROP_NG) {   // crops taller than CROP_NG groups (rare)
            u32x2a4 v[CROP_NG];
#pragma unroll
            for (int k = 0; k < CROP_NG; k++) {
                const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, (k0 + k) * gstep, 0);
                v[k] = u32x2a4{t[0], t[1]};
            }
            if (dok) {
#pragma unroll
                for (int k = 0; k < CROP_NG; k++)
                    if (k0 + k < ng) lrow[(k0 + k) * lstep] = __builtin_amdgcn_alignbyte(v[k].y, v[k].x, m);
            }
        }
        return;
    }
    const int loff = roff * c.step + 4 * dd;                            // per-lane constant
    for (int k0 = 0; k0 < ng; k0 += CROP_NG) {
        u32x2a4 v[CROP_NG];
        int m[CROP_NG];
#pragma unroll
        for (int k = 0; k < CROP_NG; k++) {
            // group k's rows; a partial last group reads up to RPG-1 rows past the crop, which stay
            // inside the level (crops end >= 13 rows above its bottom edge); groups past the crop
            // re-read the last group
            const int gk = min(k0 + k, ng - 1);
            const uint8_t* p = g0 + (long long)(RPG * gk) * c.step + loff;
            m[k] = (int)(reinterpret_cast<uintptr_t>(p) & 3u);
            v[k] = *reinterpret_cast<const u32x2a4*>(p - m[k]);
        }
#pragma unroll
        for (int k = 0; k < CROP_NG; k++) {
            const int r = RPG * (k0 + k) + roff;
            if (dok && r < c.ch)
                reinterpret_cast<uint32_t*>(crop + r * CSd)[d] = __builtin_amdgcn_alignbyte(v[k].y, v[k].x, m[k]);
        }
    }
}

template <int CST>
__device__ __forceinline__ void crop_stage_rows(const CropSrc& c, int lane, uint8_t* crop, int CSd) {
    if (CST == 0) crop_stage_rows_t<0>(c, lane, crop, CSd);   // run-time stride: one generic copy
    else if (c.ndl <= 16) crop_stage_rows_t<4>(c, lane, crop, CSd);
    else if (c.ndl <= 32) crop_stage_rows_t<5>(c, lane, crop, CSd);
    else crop_stage_rows_t<6>(c, lane, crop, CSd);
}

// One wavefront processes `cpw` consecutive (frame, cell) items of the XCD-swizzled order; item
// i = f * ncells + cell.  LDS (sized per launch from the largest cell): the crop (zone + 3-px
// apron), a zone map of corner strengths, a queue of pre-test passers and the ordered corner list.
#ifndef FAST_WAVES_DEF
#define FAST_WAVES_DEF 6
#endif
// CST / ZST: the crop and zone-map row strides when known at compile time (the C1-C3 geometries:
// 48 / 36 and 52 / 40), so every LDS address off a row base folds into the instruction's offset
// field; 0 = read them from FastLds (any other geometry).
// PAIR (round 6, ORBX_FAST_PAIR=1): two vertically consecutive cells of the strip per pass, as one
// merged zone (one crop of zhA + zhB + 6 rows, one zone map with a zero separator row between the
// cells so the 3x3 NMS stays cell-local, one set of rings): the end-of-cell partial drains, partial
// strength batches, NMS chunks and emission loops happen once per pair instead of once per cell.
// Counts, the iniThFAST / minThFAST choice (:527-530), the slot capacity and the output stay per cell;
// a speculative pass is kept only when both cells keep an iniThFAST corner.
template <int CST, int ZST, bool PAIR>
__global__ __launch_bounds__(64, FAST_WAVES_DEF) void fast_cells_kernel(Geom g, const CellDev* __restrict__ cells,
                                                        const int2* __restrict__ strips,
                                                        const uint8_t* __restrict__ in, long long in_fstride,
                                                        int in_step, const uint8_t* __restrict__ pyr, int th_ini,
                                                        int th_min, uint32_t* __restrict__ slots,
                                                        int* __restrict__ cell_cnt, uint32_t* fault, FastLds fl,
                                                        int strip_beg, int nstrips, int spec_arg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t fsm[];
    uint8_t* crop = fsm;                                   // crop col c at byte 1 + c
    uint8_t* Mz = fsm + fl.crop_bytes;
    short* queue = reinterpret_cast<short*>(Mz + fl.mz_bytes);
    short* clist = queue + fl.qcap;
    unsigned long long* bal = reinterpret_cast<unsigned long long*>(clist + fl.ccap);
    const int CSd = CST ? CST : fl.CS, ZSd = ZST ? ZST : fl.ZS;

    const int lane = threadIdx.x;
    const int lb = xcd_swizzle(blockIdx.x, gridDim.x);
    FAST_STAMP(0, __builtin_amdgcn_s_memtime());
    // wavefront = (frame, column strip): up to fast_cpw vertically consecutive cells of one column
    const int f = lb / nstrips;
    const int2 sd = strips[strip_beg + lb - f * nstrips];
    const int i_beg = 0, i_end = sd.y & 255, cstride = (sd.y >> 8) & 0x7fffff;   // bit 31: the first-cell hint
    // every cell of a strip has the same level and zone width (host-checked): the crop's level
    // base, step and row-dword count and every per-lane quantity that depends on the zone width are
    // loop-invariant over the strip
    const CellDev c0 = cells[sd.x];
    const int zw = c0.zwzh & 0xffff;
    int lstep;
    const uint8_t* limg = level_base(g, c0.level, f, in, in_fstride, in_step, pyr, &lstep);
    const int lh = g.lv[c0.level].h;
    const int ndl = (zw + 6 + 1 + 3) >> 2;   // LDS dwords per crop row
    auto source = [&](int item, CellDev& cd, int& ci) {
        ci = sd.x + item * cstride;
        cd = cells[ci];
        CropSrc c;
        c.img = limg;
        c.step = lstep;
        c.x0 = cd.x0y0 & 0xffff;
        c.y0 = cd.x0y0 >> 16;
        c.ch = (cd.zwzh >> 16) + 6;
        c.ndl = ndl;
        c.h = lh;
        return c;
    };
    // Speculative iniThFAST pass: a cell whose predecessor in this wavefront (the cell above it in
    // the same column) kept >= spec_min corners at iniThFAST is first run with the pre-test,
    // the diagonal filter and the corner list at iniThFAST only.  When the NMS keeps one of them
    // that is DetectFAST's answer (:527); otherwise the cell is re-run at min(ini, min).  On
    // texture-rich frames most pixels pass at minThFAST but few at iniThFAST.
    // spec_arg: the threshold (-1: every cell), bit 29 (threshold > 0 only): a strip's first cell, which has
    // no predecessor, speculates when the strip's hint bit (bit 31 of its descriptor, set by
    // fast_hint_kernel from the CELL_CNT_INI bit its cell got in frame 0 of the previous launch) is set.
    // Consecutive batches of a sequence see the same texture there.  The hint costs the cell loop
    // nothing (the descriptor is already in SGPRs; the kernel is at its SGPR limit), and it only decides
    // whether to speculate, never the result.
    const int spec_min = spec_arg < 0 ? spec_arg : spec_arg & 0x1fffffff;
    int prev_ini = (spec_arg > 0 && ((spec_arg >> 29) & 1) && sd.y < 0) ? spec_min : 0;
    for (int item = i_beg; item < i_end; item += PAIR ? 2 : 1) {
    CellDev cell;
    int ci;
    CropSrc src = source(item, cell, ci);
    const int x0 = src.x0, y0 = src.y0;
    const int zhA = cell.zwzh >> 16;
    // PAIR: the second cell (the one below; zhB = 0 when the strip has an odd count) extends the zone
    const bool hasB = PAIR && item + 1 < i_end;
    CellDev cellB = cell;
    int ciB = ci, zhB = 0;
    if (hasB) {
        ciB = ci + cstride;
        cellB = cells[ciB];
        zhB = cellB.zwzh >> 16;
        src.ch += zhB;
    }
    const int zh = zhA + zhB;
    // zone-map row of zone row y: PAIR inserts a zero row between the cells
    auto mrow = [&](int y) { return PAIR ? y + (y >= zhA ? 1 : 0) : y; };
    {
        crop_stage_rows<CST>(src, lane, crop, CSd);
    }
    const int tlo = min(th_ini, th_min);
    bool spec = spec_min != 0 && th_ini > tlo && prev_ini >= spec_min;   // spec_min < 0: every cell
    uint8_t* Mc = Mz + ZSd + 1;   // zone (0, 0); the zero border makes out-of-zone neighbours read 0
    uint32_t* out = slots + (long long)f * g.slot_frame + cell.slot;
    const int cap = ((zw + 1) / 2) * ((zhA + 1) / 2);
    int n_ini = 0, n_min = 0, total = 0;
    int n_iniB = 0, totalB = 0;   // PAIR: the second cell
    for (;;) {   // passes: speculative (iniThFAST) and / or full (min(ini, min))
    for (int i = lane; i < ((zh + 2 + (PAIR ? 1 : 0)) * ZSd + 15) >> 4; i += 64) reinterpret_cast<uint4*>(Mz)[i] = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
    if (item == i_beg) FAST_STAMP(1, __builtin_amdgcn_s_memtime());

    const int tp = spec ? th_ini : tlo;   // threshold of this pass
    // lanes: QR quads per row (8 or 16), 64/QR rows per chunk
    const int qsh = zw <= 32 ? 3 : 4;
    const int QR = 1 << qsh, RPC = 64 >> qsh;
    const int qx = (lane & (QR - 1)) * 4, qy = lane >> qsh;
    // u16-lane masks (1 / 0) of the zone's columns: even lanes hold (qx, qx+2), odd lanes (qx+1, qx+3)
    const us2 pme = {(unsigned short)(qx < zw), (unsigned short)(qx + 2 < zw)};
    const us2 pmo = {(unsigned short)(qx + 1 < zw), (unsigned short)(qx + 3 < zw)};

    // Stage 1 (dense): the compass pre-test (points 0/4/8/12) on 4 pixels per lane; a lane whose group
    // of 4 has a passer appends one entry (pass bits 0, 1, 16, 17 = pixels qx .. qx+3, the group's
    // zone index (y << 8) | qx at bits 2-15) to a ring of GR_RING groups in row-major order.
    // Stage 2, whenever 64 groups are pending: the diagonal pre-test (points 2/6/10/14: a 9-arc also
    // holds two circle-adjacent ones of them) on the passers of 64 groups, survivors appended per pixel
    // to a second ring in row-major order (14 % -> 5 % of the pixels on the synthetic frames).
    // Stage 3, whenever 64 pixels are pending: the corner strength M densely.  Corners (M > the pass
    // threshold) get M in the zone map and are appended to the ordered corner list.
    // (pending groups < 64 + 64 <= GR_RING; pending pixels < 64 + 256 <= FQ2_RING.)
    uint32_t* gring = reinterpret_cast<uint32_t*>(queue);
    short* queue2 = queue + 2 * GR_RING;
    int qn = 0, head = 0, q2n = 0, h2 = 0, nc = 0;
    auto strength = [&](int n) {
        const int i = lane < n ? queue2[(h2 + lane) & (FQ2_RING - 1)] : -1;
        int M = 0;
        if (i >= 0) M = corner_strength_pk<CST>(&crop[__mul24((i >> 8) + 3, CSd) + 4 + (i & 255)], CSd);
#ifdef FAST_DUP_STRENGTH   // diagnostic: the strength network twice (result discarded)
        if (i >= 0) asm volatile("" ::"v"(corner_strength_pk<CST>(&crop[__mul24((i >> 8) + 4, CSd) + 4 + (i & 255)], CSd)));
#endif
        const bool c = M > tp;
        const unsigned long long bm = __ballot(c);
        if (c) {
            const int pos = nc + rank64(bm);
            if (pos < fl.ccap) clist[pos] = (short)i;   // past ccap: the cell takes the zone-scan NMS below
            Mc[__mul24(mrow(i >> 8), ZSd) + (i & 255)] = (uint8_t)min(M, 255);
        }
        nc += popc64(bm);
        h2 += n;
    };
    auto drain = [&](int n) {
        const uint32_t e = lane < n ? gring[(head + lane) & (GR_RING - 1)] : 0u;   // 0: no pass bits
        // zone index (y << 8) | x; PAIR: stored as (y << 6) | x at bits 18-30 (merged zones are taller
        // than the 64 rows bits 2-15 hold)
        const int i0 = PAIR ? (int)(((e >> 24) << 8) | ((e >> 18) & 63u)) : (int)((e >> 2) & 0x3fffu);
        const uint8_t* c = crop + __mul24((i0 >> 8) + 3, CSd) + 4 + (i0 & 255);   // zone (y, x): dword aligned
        const uint32_t* cp = reinterpret_cast<const uint32_t*>(c + 2 * CSd);
        const uint32_t* cm = reinterpret_cast<const uint32_t*>(c - 2 * CSd);
        const uint32_t wv = *reinterpret_cast<const uint32_t*>(c);
        const uint32_t ap = cp[-1], bp = cp[0], dp = cp[1], am = cm[-1], bm_ = cm[0], dm = cm[1];
        const uint32_t Lp = __builtin_amdgcn_alignbyte(bp, ap, 2), Rp = __builtin_amdgcn_alignbyte(dp, bp, 2);
        const uint32_t Lm = __builtin_amdgcn_alignbyte(bm_, am, 2), Rm = __builtin_amdgcn_alignbyte(dm, bm_, 2);
        // position 2 = (+2, +2): Rp, 10 = (-2, -2): Lm, 6 = (+2, -2): Rm, 14 = (-2, +2): Lp
        const PkThr T = pk_thresholds(wv, tp);
        const us2 se = __builtin_elementwise_min(
            pk_two_of_four(pk_even(Rp), pk_even(Lm), pk_even(Rm), pk_even(Lp), T.hi_e, T.lo_e), u2us(e & 0x00010001u));
        const us2 so = __builtin_elementwise_min(pk_two_of_four(u2us(Rp), u2us(Lm), u2us(Rm), u2us(Lp), T.hi_o, T.lo_o),
                                                 u2us((e >> 1) & 0x00010001u));
        // ordered compaction of up to 4 survivors per lane: one ballot per pixel slot, the lane's
        // position = the survivors of the lower lanes (mbcnt) + its own earlier slots
        const bool p0 = se.x != 0, p1 = so.x != 0, p2 = se.y != 0, p3 = so.y != 0;
        const unsigned long long b0 = __ballot(p0), b1 = __ballot(p1), b2 = __ballot(p2), b3 = __ballot(p3);
        unsigned pre = __builtin_amdgcn_mbcnt_hi((unsigned)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b0, 0u));
        pre = __builtin_amdgcn_mbcnt_hi((unsigned)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b1, pre));
        pre = __builtin_amdgcn_mbcnt_hi((unsigned)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b2, pre));
        pre = __builtin_amdgcn_mbcnt_hi((unsigned)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b3, pre));
        int pos = q2n + (int)pre;
        if (p0) queue2[pos++ & (FQ2_RING - 1)] = (short)i0;
        if (p1) queue2[pos++ & (FQ2_RING - 1)] = (short)(i0 + 1);
        if (p2) queue2[pos++ & (FQ2_RING - 1)] = (short)(i0 + 2);
        if (p3) queue2[pos & (FQ2_RING - 1)] = (short)(i0 + 3);
        q2n += popc64(b0) + popc64(b1) + popc64(b2) + popc64(b3);
        head += n;
        wave_lds_sync();
        while (q2n - h2 >= 64) strength(64);
    };
    // per-lane LDS address of zone (qy, qx) = crop (qy+3, qx+3) at byte qx+4 and the group's zone index
    // (qy << 8) | qx at bits 2-15, both stepped by a wave-uniform amount per chunk of RPC rows
    const uint8_t* rowq = crop + __mul24(qy + 3, CSd) + 4 + qx;
    const uint32_t e0s = PAIR ? (uint32_t)((qy << 6) | qx) << 18 : (uint32_t)((qy << 8) | qx) << 2;
    const bool qxin = qx < zw;
    for (int yb = 0, yoff = 0; yb < zh; yb += RPC, yoff += RPC * CSd) {
        const int y = yb + qy;
        us2 pe = {0, 0}, po = {0, 0};
        if (y < zh && qxin) {
            const uint8_t* rowc = rowq + yoff;   // zone (y, qx)
            const uint32_t wv = *reinterpret_cast<const uint32_t*>(rowc);
            const uint32_t wl = *reinterpret_cast<const uint32_t*>(rowc - 4);
            const uint32_t wr = *reinterpret_cast<const uint32_t*>(rowc + 4);
            const uint32_t wn = *reinterpret_cast<const uint32_t*>(rowc + 3 * CSd);   // (0,+3)
            const uint32_t ws = *reinterpret_cast<const uint32_t*>(rowc - 3 * CSd);   // (0,-3)
            const uint32_t we = __builtin_amdgcn_alignbyte(wr, wv, 3);   // (+3, 0): bytes qx+3..qx+6
            const uint32_t ww = __builtin_amdgcn_alignbyte(wv, wl, 1);   // (-3, 0): bytes qx-3..qx
            const PkThr T = pk_thresholds(wv, tp);
            pe = __builtin_elementwise_min(
                pk_two_of_four(pk_even(wn), pk_even(ws), pk_even(we), pk_even(ww), T.hi_e, T.lo_e), pme);
            po = __builtin_elementwise_min(pk_two_of_four(u2us(wn), u2us(ws), u2us(we), u2us(ww), T.hi_o, T.lo_o), pmo);
#ifdef FAST_DUP_PRETEST   // diagnostic: the pre-test arithmetic twice (result discarded)
            {
                const PkThr T2 = pk_thresholds(wv, tp ^ yb);
                asm volatile("" ::"v"(us2u(pk_two_of_four(pk_even(wn), pk_even(ws), pk_even(we), pk_even(ww), T2.hi_e, T2.lo_e))),
                             "v"(us2u(pk_two_of_four(u2us(wn), u2us(ws), u2us(we), u2us(ww), T2.hi_o, T2.lo_o))));
            }
#endif
        }
        const bool any = (us2u(pe) | us2u(po)) != 0;
        const unsigned long long bm = __ballot(any);
        if (any) {
            // ring slot = qn + the passers of the lower lanes (mbcnt accumulates qn)
            const unsigned pos = __builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, (unsigned)qn));
            gring[pos & (GR_RING - 1)] = bt3<BT_OR3>(us2u(pe), us2u(po) + us2u(po), e0s + ((uint32_t)yb << (PAIR ? 24 : 10)));
        }
        qn += popc64(bm);
        wave_lds_sync();
        if (qn - head >= 64) drain(64);
    }
    if (qn > head) drain(qn - head);
    if (q2n > h2) strength(q2n - h2);
    wave_lds_sync();
    if (item == i_beg) FAST_STAMP(3, __builtin_amdgcn_s_memtime());

    n_ini = 0;
    n_min = 0;
    n_iniB = 0;   // (a speculative pass that fell through left its counts)
    if constexpr (PAIR) {
        // Both cells' NMS in one walk (the list, or the zone map row by row for dense pairs), with a
        // third ballot per chunk marking the first cell's entries (row-major: a prefix), then each
        // cell's emission from its own threshold's ballots.  Ballots: 3 words per chunk / pass.
        const bool dense = nc > fl.ccap;
        const int rsh = zw <= 32 ? 5 : 6, RP = 64 >> rsh;
        const int zx = lane & ((1 << rsh) - 1), zr = lane >> rsh;
        unsigned long long* pb = dense ? reinterpret_cast<unsigned long long*>(queue) : bal;
        int nm_b = 0, nch = 0;
        const int nsteps = dense ? (zh + RP - 1) / RP : (nc + 63) >> 6;
        for (; nch < nsteps; nch++) {
            bool ki = false, km = false, inA = false;
            int y = -1, x = 0;
            if (dense) {
                if (zx < zw && zr + nch * RP < zh) { y = zr + nch * RP; x = zx; }
            } else if (nch * 64 + lane < nc) {
                const int i = clist[nch * 64 + lane];
                y = i >> 8;
                x = i & 255;
            }
            if (y >= 0) {
                inA = y < zhA;
                const uint8_t* c0 = Mc + __mul24(mrow(y), ZSd) + x;
                const int m = c0[0];
                if (m) {
                    const int n0 = max(max((int)c0[-ZSd - 1], (int)c0[-ZSd]), (int)c0[-ZSd + 1]);
                    const int n1 = max((int)c0[-1], (int)c0[1]);
                    const int n2 = max(max((int)c0[ZSd - 1], (int)c0[ZSd]), (int)c0[ZSd + 1]);
                    const bool top = max(max(n0, n1), n2) < m;
                    ki = top && m > th_ini;
                    km = top && m > th_min;
                }
            }
            const unsigned long long bi = __ballot(ki), bmn = __ballot(km), ba = __ballot(inA);
            if (lane == 0) { pb[3 * nch] = bi; pb[3 * nch + 1] = bmn; pb[3 * nch + 2] = ba; }
            n_ini += popc64(bi & ba);
            n_min += popc64(bmn & ba);
            n_iniB += popc64(bi & ~ba);
            nm_b += popc64(bmn & ~ba);
        }
        wave_lds_sync();
        if (spec && (n_ini == 0 || (hasB && n_iniB == 0))) goto full_pass;
        const int wA = n_ini > 0 ? 0 : 1, wB = n_iniB > 0 ? 0 : 1;
        total = wA == 0 ? n_ini : n_min;
        totalB = wB == 0 ? n_iniB : nm_b;
        uint32_t* outB = slots + (long long)f * g.slot_frame + cellB.slot;
        const int capB = ((zw + 1) / 2) * ((zhB + 1) / 2);
        const unsigned long long below = lanemask_lt();
        int runA = 0, runB = 0;
        for (int p = 0; p < nch; p++) {
            const unsigned long long ba = pb[3 * p + 2];
            const unsigned long long kA = pb[3 * p + wA] & ba, kB = pb[3 * p + wB] & ~ba;
            if (((kA | kB) >> lane) & 1) {
                const bool a = (kA >> lane) & 1;
                const int r = a ? runA + popc64(kA & below) : runB + popc64(kB & below);
                int y, x;
                if (dense) { y = zr + p * RP; x = zx; }
                else { const int i = clist[p * 64 + lane]; y = i >> 8; x = i & 255; }
                if (r < (a ? cap : capB))
                    (a ? out : outB)[r] = (uint32_t)(x0 + 3 + x) | ((uint32_t)(y0 + 3 + y) << 12) |
                                          ((uint32_t)(Mc[__mul24(mrow(y), ZSd) + x] - 1) << 24);
            }
            runA += popc64(kA);
            runB += popc64(kB);
        }
    } else if (nc > fl.ccap) {
        // Dense cell (more corners than the list holds, e.g. pure noise): NMS over the zone map in
        // row-major order, one zone row per pass (zw <= 64), the same keep rule: a corner is kept
        // at threshold t iff M > t and every neighbour is < M (for M > t, a neighbour q >= M is
        // also > t), so both thresholds share the neighbourhood maximum.  (The speculative pass's
        // map holds only the corners at iniThFAST: a neighbour with M <= ini < m never suppresses
        // at iniThFAST, so its iniThFAST set is the full pass's.)
        // Rows per pass: two 32-lane rows when the zone is at most 32 wide (every C1-C3 cell but the
        // widest cells of the smallest levels), else one 64-lane row.  The keep ballots of both
        // thresholds are computed once and kept in the (drained) passer ring for the emission pass;
        // lane order within a pass is row-major, so the emission order is the reference's.
        const int rsh = zw <= 32 ? 5 : 6, RP = 64 >> rsh;
        const int zx = lane & ((1 << rsh) - 1), zr = lane >> rsh;
        unsigned long long* dbal = reinterpret_cast<unsigned long long*>(queue);   // 2 per pass, <= 160
        int npass = 0;
        for (int yb = 0; yb < zh; yb += RP, npass++) {
            const int y = yb + zr;
            bool ki = false, km = false;
            if (zx < zw && y < zh) {
                const uint8_t* c0 = Mc + __mul24(y, ZSd) + zx;
                const int m = c0[0];
                if (m) {
                    const int n0 = max(max((int)c0[-ZSd - 1], (int)c0[-ZSd]), (int)c0[-ZSd + 1]);
                    const int n1 = max((int)c0[-1], (int)c0[1]);
                    const int n2 = max(max((int)c0[ZSd - 1], (int)c0[ZSd]), (int)c0[ZSd + 1]);
                    const int nmax = max(max(n0, n1), n2);
                    ki = m > th_ini && nmax < m;
                    km = m > th_min && nmax < m;
                }
            }
            const unsigned long long bi = __ballot(ki), bmn = __ballot(km);
            if (lane == 0) { dbal[2 * npass] = bi; dbal[2 * npass + 1] = bmn; }
            n_ini += popc64(bi);
            n_min += popc64(bmn);
        }
        wave_lds_sync();
        if (spec && n_ini == 0) goto full_pass;
        const int which = n_ini > 0 ? 0 : 1;
        total = which == 0 ? n_ini : n_min;
        int running = 0;
        for (int pp = 0; pp < npass; pp++) {
            const unsigned long long bm = dbal[2 * pp + which];
            if (bm & (1ull << lane)) {
                const int r = running + rank64(bm);
                const int y = pp * RP + zr;
                if (r < cap)
                    out[r] = (uint32_t)(x0 + 3 + zx) | ((uint32_t)(y0 + 3 + y) << 12) |
                             ((uint32_t)(Mc[__mul24(y, ZSd) + zx] - 1) << 24);
            }
            running += popc64(bm);
        }
    } else {
    for (int jb = 0, ch2 = 0; jb < nc; jb += 64, ch2++) {
        const int j = jb + lane;
        bool ki = false, km = false;
        if (j < nc) {   // 3x3 NMS at both thresholds from one read of the 8 neighbours: for M > t a
                        // neighbour q >= M is also > t, so both keep rules are M > t && max(q) < M
            const int i = clist[j];
            const uint8_t* c0 = Mc + __mul24(i >> 8, ZSd) + (i & 255);
            const int m = c0[0];
            const int n0 = max(max((int)c0[-ZSd - 1], (int)c0[-ZSd]), (int)c0[-ZSd + 1]);
            const int n1 = max((int)c0[-1], (int)c0[1]);
            const int n2 = max(max((int)c0[ZSd - 1], (int)c0[ZSd]), (int)c0[ZSd + 1]);
            const bool top = max(max(n0, n1), n2) < m;
            ki = top && m > th_ini;
            km = top && m > th_min;
        }
        const unsigned long long bi = __ballot(ki), bmn = __ballot(km);
        if (lane == 0) { bal[2 * ch2] = bi; bal[2 * ch2 + 1] = bmn; }
        n_ini += popc64(bi);
        n_min += popc64(bmn);
    }
    wave_lds_sync();
    if (spec && n_ini == 0) goto full_pass;

    const int which = n_ini > 0 ? 0 : 1;
    total = which == 0 ? n_ini : n_min;
    int running = 0;
    for (int jb = 0, ch2 = 0; jb < nc; jb += 64, ch2++) {
        const unsigned long long bm = bal[2 * ch2 + which];
        if (bm & (1ull << lane)) {
            const int r = running + rank64(bm);
            const int i = clist[jb + lane];
            if (r < cap) {
                const int zy = i >> 8, zx = i & 255;
                const uint32_t x = (uint32_t)(x0 + 3 + zx), yy = (uint32_t)(y0 + 3 + zy);
                out[r] = x | (yy << 12) | ((uint32_t)(Mc[__mul24(zy, ZSd) + zx] - 1) << 24);
            }
        }
        running += popc64(bm);
    }
    }   // list NMS
    break;
full_pass:   // the speculative pass kept no corner at iniThFAST: the full pass decides
    spec = false;
    }   // passes
    prev_ini = hasB ? n_iniB : n_ini;
    if (item == i_beg) FAST_STAMP(4, __builtin_amdgcn_s_memtime());
    if (lane == 0) {
        if (total > cap) atomicOr(fault, FAULT_CELL_CAP);
        // bit 30: this cell kept >= spec_min corners at iniThFAST (the next strips' first-cell hint;
        // the quadtree masks the count with CELL_CNT_MASK)
        cell_cnt[(long long)f * g.ncells_total + ci] = min(total, cap) | (n_ini >= spec_min ? CELL_CNT_INI : 0);
        if (hasB) {
            const int capB = ((zw + 1) / 2) * ((zhB + 1) / 2);
            if (totalB > capB) atomicOr(fault, FAULT_CELL_CAP);
            cell_cnt[(long long)f * g.ncells_total + ciB] = min(totalB, capB) | (n_iniB >= spec_min ? CELL_CNT_INI : 0);
        }
    }
    if (item == i_beg) {
        FAST_STAMP(2, __builtin_amdgcn_s_memtime());
        FAST_STAMP(6, ((unsigned long long)cell.level << 48) | ((unsigned long long)n_min << 16) | (unsigned)total);
    }
    wave_lds_sync();
    }   // items
    FAST_STAMP(5, __builtin_amdgcn_s_memtime());
    FAST_STAMP(7, (unsigned long long)(i_end - i_beg));
}

// ------------------------------------------------------------------------------------------
// 3. quadtree
// ------------------------------------------------------------------------------------------
struct QtNode {
    short tlx, tly, brx, bry;
    int beg, cnt;
};

__device__ __forceinline__ int kp_x(uint32_t k) { return (int)(k & 0xfff); }
__device__ __forceinline__ int kp_y(uint32_t k) { return (int)((k >> 12) & 0xfff); }
__device__ __forceinline__ int kp_s(uint32_t k) { return (int)(k >> 24); }

// QTreeNode::divide (:404-452): children TL/BR and the stable 4-way split of the node's points.
__device__ __forceinline__ void qt_child_geom(const QtNode& n, int c, QtNode& ch) {
    const int xm = n.tlx + (n.brx - n.tlx + 1) / 2;   // TL.x + RoundUp(0.5*(BR.x-TL.x)), d >= 0
    const int ym = n.tly + (n.bry - n.tly + 1) / 2;
    ch.tlx = (short)((c & 1) ? xm : n.tlx);
    ch.brx = (short)((c & 1) ? n.brx : xm);
    ch.tly = (short)((c & 2) ? ym : n.tly);
    ch.bry = (short)((c & 2) ? n.bry : ym);
}

// One wave splits one node: counts per child (returned) and stable scatter into T.  A node of at
// most 512 points is loaded once (8 independent loads per lane) and split from registers.
__device__ int4 qt_wave_split(const QtNode& n, const uint32_t* __restrict__ P, uint32_t* __restrict__ T) {
    const int xm = n.tlx + (n.brx - n.tlx + 1) / 2;
    const int ym = n.tly + (n.bry - n.tly + 1) / 2;
    int c[4] = {0, 0, 0, 0};
    if (n.cnt <= 512) {
        const int lane = lane_id();
        uint32_t k[8];
        int q[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int j = 64 * t + lane;
            k[t] = j < n.cnt ? P[n.beg + j] : 0u;
        }
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int j = 64 * t + lane;
            q[t] = j < n.cnt ? (kp_x(k[t]) < xm ? (kp_y(k[t]) < ym ? 0 : 2) : (kp_y(k[t]) < ym ? 1 : 3)) : -1;
            if (64 * t < n.cnt) {   // wave-uniform
#pragma unroll
                for (int qq = 0; qq < 4; qq++) c[qq] += popc64(__ballot(q[t] == qq));
            }
        }
        int o[4] = {n.beg, n.beg + c[0], n.beg + c[0] + c[1], n.beg + c[0] + c[1] + c[2]};
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if (64 * t >= n.cnt) break;   // wave-uniform
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const unsigned long long m = __ballot(q[t] == qq);
                if (q[t] == qq) T[o[qq] + rank64(m)] = k[t];
                o[qq] += popc64(m);
            }
        }
        return make_int4(c[0], c[1], c[2], c[3]);
    }
    for (int b = 0; b < n.cnt; b += 64) {
        const int j = b + lane_id();
        int q = -1;
        if (j < n.cnt) {
            const uint32_t k = P[n.beg + j];
            q = kp_x(k) < xm ? (kp_y(k) < ym ? 0 : 2) : (kp_y(k) < ym ? 1 : 3);
        }
#pragma unroll
        for (int qq = 0; qq < 4; qq++) c[qq] += popc64(__ballot(q == qq));
    }
    int o[4] = {n.beg, n.beg + c[0], n.beg + c[0] + c[1], n.beg + c[0] + c[1] + c[2]};
    for (int b = 0; b < n.cnt; b += 64) {
        const int j = b + lane_id();
        int q = -1;
        uint32_t k = 0;
        if (j < n.cnt) {
            k = P[n.beg + j];
            q = kp_x(k) < xm ? (kp_y(k) < ym ? 0 : 2) : (kp_y(k) < ym ? 1 : 3);
        }
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const unsigned long long m = __ballot(q == qq);
            if (q == qq) T[o[qq] + rank64(m)] = k;
            o[qq] += popc64(m);
        }
    }
    return make_int4(c[0], c[1], c[2], c[3]);
}

// A 16-lane group splits one node of at most 16 points (group = lane >> 4): the same stable 4-way
// scatter as qt_wave_split with the ballots cut to the group's 16 bits.  Every lane of the
// wavefront must call it (ballots); lanes of a group without a node pass cnt = 0.
template <bool SCATTER = true>
__device__ int4 qt_group16_split(const QtNode& n, int cnt, const uint32_t* __restrict__ P, uint32_t* __restrict__ T) {
    const int lane = lane_id(), sh = lane & 48, gl = lane & 15;
    const unsigned lt16 = (1u << gl) - 1u;
    const int xm = n.tlx + (n.brx - n.tlx + 1) / 2;
    const int ym = n.tly + (n.bry - n.tly + 1) / 2;
    int q = -1;
    uint32_t k = 0;
    if (gl < cnt) {
        k = P[n.beg + gl];
        q = kp_x(k) < xm ? (kp_y(k) < ym ? 0 : 2) : (kp_y(k) < ym ? 1 : 3);
    }
    unsigned m[4];
#pragma unroll
    for (int qq = 0; qq < 4; qq++) m[qq] = (unsigned)(__ballot(q == qq) >> sh) & 0xffffu;
    const int c0 = __popc(m[0]), c1 = __popc(m[1]), c2 = __popc(m[2]), c3 = __popc(m[3]);
    const int o[4] = {n.beg, n.beg + c0, n.beg + c0 + c1, n.beg + c0 + c1 + c2};
    if (SCATTER && q >= 0) T[o[q] + __popc(m[q] & lt16)] = k;
    return make_int4(c0, c1, c2, c3);
}

// quadtree_kernel's block size.  qt_block_split is written for exactly QT_THREADS threads (QT_WAVES
// wavefronts): its child counts are summed from QT_WAVES per-wave partials and its scatter tiles are
// 4 x QT_THREADS points with (u, child, wave) ballot counts.  Round 5's 64-thread experiment
// (ORBX_QT_SMALL=64) broke exactly this: with one wavefront the totals read three stale wave slots,
// the child offsets went wild and T was written out of bounds (the illegal access in
// test_fast_candidates_dense_cells[noise], whose dense root nodes take this split).  The kernel now
// checks its block size on entry and sets FAULT_BLOCK_SIZE instead of running (quadtree_kernel).
constexpr int QT_THREADS = 256, QT_WAVES = QT_THREADS / 64;
static_assert(QT_WAVES == 4, "qt_block_split's scratch layout (sc[16 u + 4 child + wave]) holds 4 wavefronts");
// All threads of the QT_THREADS block split one large node: child counts by a block reduction,
// then the stable scatter in tiles of 4 QT_THREADS points, point u*QT_THREADS + tid of a tile in
// thread tid, its position from the per-(u, child, wave) ballot counts of the tile.  sc: 64 ints of
// LDS scratch.  Every thread must call it; the counts are block-uniform.
// Phase-1 nodes above this size are split by the whole block (round 5: 2048 -> 512, quadtree
// -3 % on pan frames, +0.7 % textured: a level's first pass has a few root nodes of 500-2000
// points, and a wavefront per node left the other wavefronts idle)
#ifndef QT_BIG_DEF
#define QT_BIG_DEF 512
#endif
constexpr int QT_BIG = QT_BIG_DEF;
__device__ int4 qt_block_split(const QtNode& n, const uint32_t* __restrict__ P, uint32_t* __restrict__ T, int* sc) {
    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const int xm = n.tlx + (n.brx - n.tlx + 1) / 2;
    const int ym = n.tly + (n.bry - n.tly + 1) / 2;
    auto quad = [&](uint32_t k) { return kp_x(k) < xm ? (kp_y(k) < ym ? 0 : 2) : (kp_y(k) < ym ? 1 : 3); };
    int c[4] = {0, 0, 0, 0};
#ifndef QT_BS_CNT
#define QT_BS_CNT 4
#endif
    for (int b = 0; b < n.cnt; b += QT_THREADS * QT_BS_CNT) {   // (the counts: QT_BS_CNT points per thread per round)
        uint32_t k[QT_BS_CNT];
#pragma unroll
        for (int u = 0; u < QT_BS_CNT; u++) {
            const int j = b + QT_THREADS * u + tid;
            k[u] = j < n.cnt ? P[n.beg + j] : 0u;
        }
#pragma unroll
        for (int u = 0; u < QT_BS_CNT; u++) {
            const int q = b + QT_THREADS * u + tid < n.cnt ? quad(k[u]) : -1;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) c[qq] += q == qq;
        }
    }
#pragma unroll
    for (int qq = 0; qq < 4; qq++) {
        const int v = wave_sum_i32(c[qq]);
        if (lane == 0) sc[4 * w + qq] = v;
    }
    __syncthreads();
    int tot[4], o[4];
#pragma unroll
    for (int qq = 0; qq < 4; qq++) tot[qq] = sc[qq] + sc[4 + qq] + sc[8 + qq] + sc[12 + qq];   // QT_WAVES = 4 partials
    o[0] = n.beg;
    o[1] = o[0] + tot[0];
    o[2] = o[1] + tot[1];
    o[3] = o[2] + tot[2];
    __syncthreads();
#ifdef QT_BS_PF
    // the next tile's points are loaded before this tile's barrier (ranks kept as ints, so the
    // prefetch costs no registers over the 64-bit ballot masks)
    uint32_t k[4];
#pragma unroll
    for (int u = 0; u < 4; u++) k[u] = QT_THREADS * u + tid < n.cnt ? P[n.beg + QT_THREADS * u + tid] : 0u;
    for (int b = 0; b < n.cnt; b += 4 * QT_THREADS) {
        int q[4], rk[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            q[u] = b + QT_THREADS * u + tid < n.cnt ? quad(k[u]) : -1;
            rk[u] = 0;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const unsigned long long bm = __ballot(q[u] == qq);
                if (q[u] == qq) rk[u] = rank64(bm);
                if (lane == 0) sc[16 * u + 4 * qq + w] = popc64(bm);   // (u, child, wave)
            }
        }
        uint32_t kn[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int j = b + 4 * QT_THREADS + QT_THREADS * u + tid;
            kn[u] = j < n.cnt ? P[n.beg + j] : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (q[u] < 0) continue;
            const int* cq = sc + 4 * q[u];
            int off = o[q[u]];
            for (int uu = 0; uu < u; uu++) off += cq[16 * uu] + cq[16 * uu + 1] + cq[16 * uu + 2] + cq[16 * uu + 3];
            for (int ww = 0; ww < w; ww++) off += cq[16 * u + ww];
            T[off + rk[u]] = k[u];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) k[u] = kn[u];
#else
    for (int b = 0; b < n.cnt; b += 4 * QT_THREADS) {
        uint32_t k[4];
        int q[4];
        unsigned long long m[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int j = b + QT_THREADS * u + tid;
            k[u] = j < n.cnt ? P[n.beg + j] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            q[u] = b + QT_THREADS * u + tid < n.cnt ? quad(k[u]) : -1;
            m[u] = 0;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const unsigned long long bm = __ballot(q[u] == qq);
                if (q[u] == qq) m[u] = bm;
                if (lane == 0) sc[16 * u + 4 * qq + w] = popc64(bm);   // (u, child, wave)
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (q[u] < 0) continue;
            const int* cq = sc + 4 * q[u];
            int off = o[q[u]];
            for (int uu = 0; uu < u; uu++) off += cq[16 * uu] + cq[16 * uu + 1] + cq[16 * uu + 2] + cq[16 * uu + 3];
            for (int ww = 0; ww < w; ww++) off += cq[16 * u + ww];
            T[off + rank64(m[u])] = k[u];
        }
#endif
#pragma unroll
        for (int qq = 0; qq < 4; qq++)
#pragma unroll
            for (int u = 0; u < 4; u++)
                o[qq] += sc[16 * u + 4 * qq] + sc[16 * u + 4 * qq + 1] + sc[16 * u + 4 * qq + 2] + sc[16 * u + 4 * qq + 3];
        __syncthreads();
    }
    return make_int4(tot[0], tot[1], tot[2], tot[3]);
}

// Child counts of one node by a single thread (phase 2 only needs the counts of every divisible
// node to find where to stop; only the processed prefix is then split for real); 8 loads in flight.
__device__ __forceinline__ int4 qt_thread_count(const QtNode& n, const uint32_t* __restrict__ P) {
    const int xm = n.tlx + (n.brx - n.tlx + 1) / 2;
    const int ym = n.tly + (n.bry - n.tly + 1) / 2;
    int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int j0 = 0; j0 < n.cnt; j0 += 8) {
        uint32_t kk[8];
#pragma unroll
        for (int u = 0; u < 8; u++) kk[u] = j0 + u < n.cnt ? P[n.beg + j0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t k = kk[u];
            const bool in = j0 + u < n.cnt;
            const bool r = kp_x(k) >= xm, d = kp_y(k) >= ym;
            c0 += in && !r && !d;
            c1 += in && r && !d;
            c2 += in && !r && d;
            c3 += in && r && d;
        }
    }
    return make_int4(c0, c1, c2, c3);
}

__device__ __forceinline__ int ne4(int4 c) { return (c.x > 0) + (c.y > 0) + (c.z > 0) + (c.w > 0); }
__device__ __forceinline__ int dv4(int4 c) { return (c.x > 1) + (c.y > 1) + (c.z > 1) + (c.w > 1); }
__device__ __forceinline__ int c4(int4 c, int i) { return i == 0 ? c.x : i == 1 ? c.y : i == 2 ? c.z : c.w; }

// Appends item `j`'s children into the new list (group position `gpos`, children in push_front
// order c3..c0) and its divisible children into `divs` at `dpos` (child order c0..c3).
__device__ __forceinline__ void qt_emit_children(const QtNode& parent, int4 cc, int gpos, int dpos, QtNode* nb,
                                                 QtItem* divs, int NC) {
    int pos = gpos;
    for (int c = 3; c >= 0; c--) {
        const int n = c4(cc, c);
        if (n <= 0) continue;
        QtNode ch;
        qt_child_geom(parent, c, ch);
        int off = 0;
        for (int q = 0; q < c; q++) off += c4(cc, q);
        ch.beg = parent.beg + off;
        ch.cnt = n;
        if (pos < NC) nb[pos] = ch;
        pos++;
    }
    // positions: child c sits at gpos + #{nonempty c' > c}
    int d = dpos;
    for (int c = 0; c < 4; c++) {
        const int n = c4(cc, c);
        if (n <= 1) continue;
        int above = 0;
        for (int q = c + 1; q < 4; q++) above += c4(cc, q) > 0;
        if (d < NC) divs[d] = QtItem{n, gpos + above};
        d++;
    }
}

#ifndef QT_STAMP_LEVEL
#define QT_STAMP_LEVEL 0   // the level whose frame-0 workgroup records the phase stamps (ORB_QT_STAMPS)
#endif
#ifdef ORB_QT_STAMPS
__device__ unsigned long long g_qt_stamps[64];
__device__ unsigned long long g_qt_wg[4096 * 2];   // per (frame, level) WG: start, end
#define QT_STAMP(k)                                                                                \
    do {                                                                                           \
        if (blockIdx.x == 0 && lev0 + (int)blockIdx.y == QT_STAMP_LEVEL && threadIdx.x == 0 && (k) < 64)\
            g_qt_stamps[(k)] = __builtin_amdgcn_s_memtime();                                       \
    } while (0)
#ifndef QT_SUB_ITER
#define QT_SUB_ITER 5   // the phase-1 pass whose sub-phases are stamped (56-59)
#endif
#define QT_SUBSTAMP(k)                                                                             \
    do {                                                                                           \
        if (iter_no == QT_SUB_ITER + 1) QT_STAMP(k);                                               \
    } while (0)
#else
#define QT_SUBSTAMP(k) \
    do {               \
    } while (0)
#define QT_STAMP(k) \
    do {            \
    } while (0)
#endif


// std::sort(a, a+n, size-descending) as qt_sort_parallel_form() (qt_sort.h): each Hoare partition
// computed from ballot-compacted stopper lists by one wavefront.  Segments of one recursion round are disjoint
// and a partition (or the depth-0 heap sort) only moves items inside its own segment, so the
// rounds run one after another and a round's segments in parallel, one wavefront each; the
// result is identical to the sequential order.  All threads of the block must call it.
// Scratch: Ls, Rs, seg_lo, seg_len (n ints each), tmp (n items), lists (6 * list_cap ints),
// s_cnt (2 shared ints).  list_cap >= n / 17 + 1.
template <bool WV>
__device__ void qt_sort_block(QtItem* a, int n, int* Ls, int* Rs, int* seg_lo, int* seg_len, QtItem* tmp,
                              int* lists, int list_cap, int* s_cnt) {
    const int lane = lane_id(), w = WV ? 0 : (int)(threadIdx.x >> 6), nw = WV ? 1 : (int)(blockDim.x >> 6);
    const int gtid = WV ? lane : (int)threadIdx.x, gbd = WV ? 64 : (int)blockDim.x;
    if (n <= 0) return;
    int* cur = lists;
    int* nxt = lists + 3 * list_cap;
    if (gtid == 0) {
        s_cnt[0] = 0;
        s_cnt[1] = 0;
        if (n > 16) {
            cur[0] = 0; cur[1] = n; cur[2] = 2 * qt_lg(n);
            s_cnt[0] = 1;
        }
    }
    if (n <= 16)
        for (int i = gtid; i < n; i += gbd) { seg_lo[i] = 0; seg_len[i] = n; }
    qt_sync<WV>();
    while (true) {
        const int nc = s_cnt[0];
        if (nc == 0) break;
        for (int si = w; si < nc; si += nw) {
            const int lo = cur[3 * si], hi = cur[3 * si + 1];
            int depth = cur[3 * si + 2];
            if (depth == 0) {
                if (lane == 0) qt_heap_sort(a + lo, a + hi);
                for (int i = lo + lane; i < hi; i += 64) { seg_lo[i] = lo; seg_len[i] = -1; }
                wave_lds_sync();
                continue;
            }
            --depth;
            const int mid = lo + (hi - lo) / 2;
            if (lane == 0) qt_median_to_first(a + lo, a + lo + 1, a + mid, a + hi - 1);
            wave_lds_sync();
            const int pv = a[lo].size;
            int nl = 0, nr = 0;
            for (int base = lo + 1; base < hi; base += 64) {
                const int i = base + lane;
                const bool f = i < hi && a[i].size <= pv;
                const unsigned long long m = __ballot(f);
                if (f) Ls[lo + nl + rank64(m)] = i;
                nl += popc64(m);
            }
            for (int base = hi - 1; base >= lo; base -= 64) {
                const int j = base - lane;
                const bool f = j >= lo && a[j].size >= pv;
                const unsigned long long m = __ballot(f);
                if (f) Rs[lo + nr + rank64(m)] = j;
                nr += popc64(m);
            }
            wave_lds_sync();
            const int mn = min(nl, nr);
            int K = 0;
            for (int kb = 0; kb < mn; kb += 64) {
                const int k = kb + lane;
                const unsigned long long m = __ballot(k < mn && Ls[lo + k] < Rs[lo + k]);
                K += popc64(m);
                if (m != ~0ull) break;   // the predicate holds on a prefix of k
            }
            for (int k = lane; k < K; k += 64) {
                const int li = Ls[lo + k], ri = Rs[lo + k];
                const QtItem x = a[li], y = a[ri];
                a[li] = y;
                a[ri] = x;
            }
            wave_lds_sync();
            int cut;
            if (K == 0) cut = Ls[lo];
            else {
                const int c1 = K < nl ? Ls[lo + K] : hi;
                const int c2 = Rs[lo + K - 1];
                cut = c1 < c2 ? c1 : c2;
            }
            // children: > 16 go to the next round, the rest are final segments now
            const int clo[2] = {lo, cut}, chi[2] = {cut, hi};
#pragma unroll
            for (int c = 0; c < 2; c++) {
                if (chi[c] - clo[c] > 16) {
                    if (lane == 0) {
                        const int idx = atomicAdd(&s_cnt[1], 1);
                        nxt[3 * idx] = clo[c]; nxt[3 * idx + 1] = chi[c]; nxt[3 * idx + 2] = depth;
                    }
                } else {
                    for (int i = clo[c] + lane; i < chi[c]; i += 64) { seg_lo[i] = clo[c]; seg_len[i] = chi[c] - clo[c]; }
                }
            }
            wave_lds_sync();
        }
        qt_sync<WV>();
        if (gtid == 0) {
            s_cnt[0] = s_cnt[1];
            s_cnt[1] = 0;
        }
        int* t = cur; cur = nxt; nxt = t;
        qt_sync<WV>();
    }
    // final insertion pass == stable sort inside each final segment
    for (int i = gtid; i < n; i += gbd) {
        const QtItem v = a[i];
        if (seg_len[i] < 0) { tmp[i] = v; continue; }
        const int lo = seg_lo[i], hi = lo + seg_len[i];
        int r = 0;
        for (int j = lo; j < hi; j++) {
            const int sj = a[j].size;
            r += (sj > v.size) || (sj == v.size && j < i);
        }
        tmp[lo + r] = v;
    }
    qt_sync<WV>();
    for (int i = gtid; i < n; i += gbd) a[i] = tmp[i];
    qt_sync<WV>();
}

#ifndef QT_WAVES_DEF
#define QT_WAVES_DEF 4   // wavefronts per SIMD = workgroups per CU (4 wavefronts each)
#endif
// per node: na, nb (QtNode), cc (int4), divs, prev (QtItem), ia, ib (int) -- the host sizes the LDS with it
constexpr int QT_NODE_BYTES = 2 * (int)sizeof(QtNode) + (int)sizeof(int4) + 2 * (int)sizeof(QtItem) + 2 * (int)sizeof(int);
template <bool WV>
__global__ __launch_bounds__(QT_THREADS, QT_WAVES_DEF) void quadtree_kernel(Geom g, const int* __restrict__ cell_cnt,
                                                       const uint32_t* __restrict__ slots, const CellDev* cells,
                                                       uint32_t* __restrict__ Pbuf, uint32_t* __restrict__ Tbuf,
                                                       uint32_t* __restrict__ sel, int* __restrict__ sel_cnt, int NC,
                                                       int PTC, uint32_t* fault, int lev0, int nlev) {
    extern __shared__ __attribute__((aligned(16))) char smem_all[];
    // WV: wavefront q of the workgroup runs level lev0 + 4 blockIdx.y + q on its own LDS slice and its
    // own copy of the shared scalars; otherwise the workgroup runs level lev0 + blockIdx.y
    const int wslot = WV ? (int)(threadIdx.x >> 6) : 0;
    char* smem = smem_all + (WV ? (size_t)wslot * ((size_t)NC * QT_NODE_BYTES + (size_t)PTC * 8) : 0);
    QtNode* na = reinterpret_cast<QtNode*>(smem);
    QtNode* nb = na + NC;
    int4* cc = reinterpret_cast<int4*>(nb + NC);
    QtItem* divs = reinterpret_cast<QtItem*>(cc + NC);
    QtItem* prev = divs + NC;
    int* ia = reinterpret_cast<int*>(prev + NC);    // per-node scratch (flags / positions)
    int* ib = ia + NC;
    uint32_t* lds_P = reinterpret_cast<uint32_t*>(ib + NC);   // candidate arrays when they fit
    uint32_t* lds_T = lds_P + PTC;
    constexpr int NSC = WV ? QT_WAVES : 1;
    __shared__ int tmp_a[NSC][16];
    __shared__ int s_sc[NSC][8];
    __shared__ int s_sortcnt_a[NSC][2];
    __shared__ int s_split[64];
    __shared__ int rc_a[NSC][MAX_ROOTS];
    int* tmp = tmp_a[wslot];
    int& s_n = s_sc[wslot][0];
    int& s_ndiv = s_sc[wslot][1];
    int& s_state = s_sc[wslot][2];
    int& s_proc = s_sc[wslot][3];
    int& s_fail = s_sc[wslot][4];
    int& s_anybig = s_sc[wslot][5];
    int* s_sortcnt = s_sortcnt_a[wslot];
    int* rc = rc_a[wslot];

    const int f = blockIdx.x, l = WV ? lev0 + 4 * (int)blockIdx.y + wslot : lev0 + (int)blockIdx.y;
    if (blockDim.x != QT_THREADS) {   // block-uniform: a launch this kernel is not written for fails loudly
        if (threadIdx.x == 0) {
            atomicOr(fault, FAULT_BLOCK_SIZE);
            // describe then sees empty levels, never stale selections (WV: all four of the group)
            for (int q = 0; q < (WV ? 4 : 1); q++) {
                const int lq = WV ? lev0 + 4 * (int)blockIdx.y + q : l;
                if (!WV || lq < lev0 + nlev) sel_cnt[f * g.nlevels + lq] = 0;
            }
        }
        return;
    }
    if (WV && l >= lev0 + nlev) return;   // (wave-uniform; no workgroup barrier in this form)
    int* scnt = sel_cnt + f * g.nlevels + l;
    const LevelDev& L = g.lv[l];
    const int qtid = WV ? lane_id() : (int)threadIdx.x;   // thread index within the tree's group
    constexpr int QBD = WV ? 64 : QT_THREADS;               // the group's size
    const int w = WV ? 0 : (int)(threadIdx.x >> 6), nw = WV ? 1 : QT_WAVES;
    if (L.rw <= 0 || L.rh <= 0 || L.ncells == 0) {
        if (qtid == 0) *scnt = 0;
        return;
    }
    uint32_t* P = Pbuf + (long long)f * g.cand_frame + L.cand_base;
    uint32_t* T = Tbuf + (long long)f * g.cand_frame + L.cand_base;
    uint32_t* gP = P;
    const int* ccell = cell_cnt + (long long)f * g.ncells_total + L.cell_base;
    const uint32_t* fslots = slots + (long long)f * g.slot_frame;

    QT_STAMP(0);
    int p2_round = 0;
    (void)p2_round;
#ifdef ORB_QT_STAMPS
    const unsigned long long qt_t0 = __builtin_amdgcn_s_memtime();
#endif
    // ---- gather candidates in cell raster order (DetectFAST push_back order).  Pass 1: total count;
    //      the arrays live in LDS when they fit.  Pass 2: one lane per cell copies its points.
    // Root id of a keypoint (:562-569): (int)(((float)x - roi.x) / hx) in double; monotone in x.
    const int R = L.nroots;
    auto root_x = [&](int x) -> int {
        const float dx = (float)x - (float)L.rx;   // keypoint.pt.x - roi.x (float)
        return (int)((double)dx / L.hx);
    };
    if (qtid < MAX_ROOTS) rc[qtid] = 0;
    if (qtid == 0) s_fail = 0;
    int n_total = 0, carry = 0;
    bool parted = false;   // the gather below writes the root-partitioned order itself (round 5)
    if (L.ncells <= 4 * QBD && R <= 4) {
        // thread t owns cells cpt t .. cpt t + cpt - 1 (raster order): their counts and slot offsets are loaded
        // together and the points go straight to their root's segment.  A cell whose zone lies inside
        // one root (all but the cells on a root boundary) sends all its points there, a boundary cell
        // splits them by x; one block scan per root (R <= 4) of the threads' counts places the threads'
        // runs, so each segment keeps the gather order: the stable partition of :547-579 without the
        // round trip through T.  Every thread's first 8 points per cell are loaded in one batch.
        // Cells per thread: as few as the grid allows (a small level's 100-500 cells over 1-2 per
        // thread instead of 4), so a thread's chain of dependent slot loads is shorter (round 5);
        // thread order is still cell order.
#ifndef QT_GATHER_CPT4
        const int cpt = (L.ncells + QBD - 1) / QBD;   // 1..4
#else
        const int cpt = 4;
#endif
        const int i0 = cpt * qtid;
        int cv[4], cs[4], rl[4], rh[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int i = i0 + k;
            cv[k] = 0; cs[k] = 0; rl[k] = 0; rh[k] = 0;
            if (k < cpt && i < L.ncells) {
                const CellDev cd = cells[L.cell_base + i];
                cv[k] = ccell[i] & CELL_CNT_MASK;
                cs[k] = cd.slot;
                const int zx = (cd.x0y0 & 0xffff) + 3;            // the zone's first column
                rl[k] = root_x(zx);
                rh[k] = root_x(zx + (cd.zwzh & 0xffff) - 1);     // and its last
            }
        }
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 4; k++) bad |= cv[k] > 0 && (rl[k] < 0 || rh[k] >= R);
        if (bad) atomicOr(fault, FAULT_QT_ROOT);
        int cnt[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (rl[k] == rh[k]) {
#pragma unroll
                for (int rt = 0; rt < 4; rt++) cnt[rt] += rl[k] == rt ? cv[k] : 0;
            } else {   // a boundary cell (rare): its points' roots
                for (int q = 0; q < cv[k]; q++) {
                    const int rt = root_x(kp_x(fslots[cs[k] + q]));
#pragma unroll
                    for (int u = 0; u < 4; u++) cnt[u] += rt == u;
                }
            }
        }
        int run[4];
        int base = 0;
#pragma unroll
        for (int rt = 0; rt < 4; rt++) {
            if (rt >= R) { run[rt] = 0; continue; }   // block-uniform
            int tot;
            run[rt] = base + grp_excl_scan<WV>(cnt[rt], tmp, &tot);
            if (qtid == 0) rc[rt] = tot;
            base += tot;
        }
        n_total = base;
        if (n_total <= PTC) { P = lds_P; T = lds_T; }
        uint32_t r[4][8];
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int q = 0; q < 8; q++) r[k][q] = q < cv[k] ? fslots[cs[k] + q] : 0u;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (rl[k] == rh[k]) {
                int o = run[0];
#pragma unroll
                for (int rt = 1; rt < 4; rt++) o = rl[k] == rt ? run[rt] : o;
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (q < cv[k]) P[o + q] = r[k][q];
                for (int q0 = 8; q0 < cv[k]; q0 += 8) {   // > 8 points in a cell: batches of 8 loads
                    uint32_t r2[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) r2[q] = q0 + q < cv[k] ? fslots[cs[k] + q0 + q] : 0u;
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (q0 + q < cv[k]) P[o + q0 + q] = r2[q];
                }
#pragma unroll
                for (int rt = 0; rt < 4; rt++) run[rt] += rl[k] == rt ? cv[k] : 0;
            } else {
                for (int q = 0; q < cv[k]; q++) {
                    const uint32_t kk = fslots[cs[k] + q];
                    const int rt = root_x(kp_x(kk));
                    int o = run[0];
#pragma unroll
                    for (int u = 1; u < 4; u++) o = rt == u ? run[u] : o;
                    P[o] = kk;
#pragma unroll
                    for (int u = 0; u < 4; u++) run[u] += rt == u;
                }
            }
        }
        carry = n_total;
        parted = true;
    } else if (L.ncells <= 4 * QBD) {
        // (more than 4 roots: an aspect ratio above 4.5) the gather in raster order, partitioned below
        const int i0 = 4 * qtid;
        int cv[4], cs[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int i = i0 + k;
            cv[k] = i < L.ncells ? ccell[i] & CELL_CNT_MASK : 0;
            cs[k] = i < L.ncells ? cells[L.cell_base + i].slot : 0;
        }
        const int sum = cv[0] + cv[1] + cv[2] + cv[3];
        const int ex = grp_excl_scan<WV>(sum, tmp, &n_total);
        if (n_total <= PTC) { P = lds_P; T = lds_T; }
        int o = ex;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            for (int q0 = 0; q0 < cv[k]; q0 += 8) {
                uint32_t r2[8];
#pragma unroll
                for (int q = 0; q < 8; q++) r2[q] = q0 + q < cv[k] ? fslots[cs[k] + q0 + q] : 0u;
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (q0 + q < cv[k]) P[o + q0 + q] = r2[q];
            }
            o += cv[k];
        }
        carry = n_total;
    } else {
        {
            int part = 0;
            for (int i = qtid; i < L.ncells; i += QBD) part += ccell[i] & CELL_CNT_MASK;
            part = wave_sum_i32(part);
            if (lane_id() == 0) tmp[8 + w] = part;
            qt_sync<WV>();
            for (int q = 0; q < nw; q++) n_total += tmp[8 + q];
            qt_sync<WV>();
        }
        if (n_total <= PTC) { P = lds_P; T = lds_T; }
        for (int b = 0; b < L.ncells; b += QBD) {
            const int i = b + qtid;
            const int v = i < L.ncells ? ccell[i] & CELL_CNT_MASK : 0;
            int tot;
            const int ex = grp_excl_scan<WV>(v, tmp, &tot);
            if (v > 0) {
                const uint32_t* __restrict__ src = fslots + cells[L.cell_base + i].slot;
                uint32_t* dst = P + carry + ex;
                for (int j0 = 0; j0 < v; j0 += 8) {
                    uint32_t r[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) r[q] = j0 + q < v ? src[j0 + q] : 0;
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (j0 + q < v) dst[j0 + q] = r[q];
                }
            }
            carry += tot;
        }
    }
    qt_sync<WV>();
    const int n_src = carry;
    if (WV && !parted) {   // the host sends only levels the partitioned gather takes (<= 256 cells, <= 4 roots)
        if (qtid == 0) {
            atomicOr(fault, FAULT_BLOCK_SIZE);
            *scnt = 0;
        }
        return;
    }
    QT_STAMP(1);
    if (n_src == 0) {
        if (qtid == 0) *scnt = 0;
        return;
    }
    qt_sync<WV>();

    // ---- root nodes (:547-579): stable partition by root id (the large-grid gather's order; the
    //      small-grid gather above wrote the partitioned order itself)
    if (!parted) {   // block-uniform
    auto root_of = [&](uint32_t k) -> int { return root_x(kp_x(k)); };
    // every wave partitions a contiguous quarter (root ids kept in registers between the passes);
    // quarter q's base offset per root = that root's count over quarters < q -> stable overall
    __shared__ int s_rcnt[4][MAX_ROOTS];
    constexpr int QT_RPL = 32;   // points per lane held in registers (fallback loop past that)
    const int qlen = (n_src + nw - 1) / nw;
    const int q0 = min(n_src, w * qlen), q1 = min(n_src, q0 + qlen);
    int rid[QT_RPL];
    {
        int counts[MAX_ROOTS];
        for (int r = 0; r < R; r++) counts[r] = 0;
#pragma unroll
        for (int t = 0; t < QT_RPL; t++) {
            if (q0 + 64 * t >= q1) { rid[t] = -1; continue; }   // wave-uniform: past this quarter
            const int j = q0 + 64 * t + lane_id();
            int r = -1;
            if (j < q1) {
                r = root_of(P[j]);
                if (r < 0 || r >= R) atomicOr(fault, FAULT_QT_ROOT);
            }
            rid[t] = r;
            for (int q = 0; q < R; q++) counts[q] += popc64(__ballot(r == q));
        }
        for (int b = q0 + 64 * QT_RPL; b < q1; b += 256) {   // quarters longer than 64*QT_RPL points
            uint32_t kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = b + 64 * u + lane_id();
                kk[u] = j < q1 ? P[j] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = b + 64 * u + lane_id();
                const int r = j < q1 ? root_of(kk[u]) : -1;
                for (int q = 0; q < R; q++) counts[q] += popc64(__ballot(r == q));
            }
        }
        if (lane_id() == 0)
            for (int q = 0; q < R; q++) s_rcnt[w][q] = counts[q];
    }
    qt_sync<WV>();
    {
        int o[MAX_ROOTS];
        int acc = 0;
        for (int q = 0; q < R; q++) {
            int before = 0, tot = 0;
            for (int v = 0; v < nw; v++) {
                tot += s_rcnt[v][q];
                if (v < w) before += s_rcnt[v][q];
            }
            o[q] = acc + before;
            acc += tot;
            if (qtid == 0) rc[q] = tot;
        }
#pragma unroll
        for (int t = 0; t < QT_RPL; t++) {
            if (q0 + 64 * t >= q1) continue;   // wave-uniform
            const int j = q0 + 64 * t + lane_id();
            const uint32_t k = j < q1 ? P[j] : 0;
            const int r = rid[t];
            for (int q = 0; q < R; q++) {
                const unsigned long long m = __ballot(r == q);
                if (r == q) T[o[q] + rank64(m)] = k;
                o[q] += popc64(m);
            }
        }
        for (int b = q0 + 64 * QT_RPL; b < q1; b += 256) {
            uint32_t kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = b + 64 * u + lane_id();
                kk[u] = j < q1 ? P[j] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = b + 64 * u + lane_id();
                const uint32_t k = kk[u];
                const int r = j < q1 ? root_of(k) : -1;
                for (int q = 0; q < R; q++) {
                    const unsigned long long m = __ballot(r == q);
                    if (r == q) T[o[q] + rank64(m)] = k;
                    o[q] += popc64(m);
                }
            }
        }
    }
    qt_sync<WV>();
    {   // the partitioned copy becomes P (every thread swaps the same pointers)
        uint32_t* t = P;
        P = T;
        T = t;
    }
    }   // !parted
    if (qtid == 0) {
        int n = 0, acc = 0;
        for (int q = 0; q < R; q++) {
            if (rc[q] > 0) {
                QtNode r;
                r.tlx = (short)(int)(L.rx + L.hx * q);
                r.tly = (short)L.ry;
                r.brx = (short)(int)(L.rx + L.hx * (q + 1));
                r.bry = (short)(L.ry + L.rh);
                r.beg = acc;
                r.cnt = rc[q];
                na[n++] = r;
            }
            acc += rc[q];
        }
        s_n = n;
        s_state = 0;   // 0 = phase 1, 1 = phase 2, 2 = finished
        s_ndiv = 0;
        s_anybig = 0;
    }
    qt_sync<WV>();

    const int nfeat = L.quota;
    QT_STAMP(2);
    int iter_no = 0;
    (void)iter_no;
    (void)gP;
    // ---- main loop
    while (true) {
        const int n = s_n;
        const int state = s_state;
        QT_STAMP(3 + 2 * iter_no);
        if (qtid == 0 && blockIdx.x == 0 && l == QT_STAMP_LEVEL) {
#ifdef ORB_QT_STAMPS
            if (4 + 2 * iter_no < 60) g_qt_stamps[4 + 2 * iter_no] = ((unsigned long long)state << 32) | (unsigned)n;
#endif
        }
        iter_no++;
        if (state == 2) break;
        if (state == 0) {
            // Phase 1 pass (:588-630): split every divisible node in list order.
            // D positions via compaction
            int kdiv = 0, nnd = 0;   // (s_anybig was cleared before the last barrier)
            for (int b = 0; b < n; b += QBD) {
                const int i = b + qtid;
                const int dvf = (i < n && na[i].cnt > 1) ? 1 : 0;
                if (!WV && i < n && na[i].cnt > QT_BIG) s_anybig = 1;   // (WV: one wavefront per tree, no block split)
                int tot;
                const int ex = grp_excl_scan<WV>(dvf, tmp, &tot);
                if (i < n) {
                    if (dvf) ia[kdiv + ex] = i;               // D: divisible, processing order
                    else ib[i] = nnd + (i - b - ex);          // rank among non-divisible
                }
                nnd += min(QBD, n - b) - tot;
                kdiv += tot;
            }
            qt_sync<WV>();
            QT_SUBSTAMP(56);
            // nodes of <= 16 points: four per wavefront (16-lane groups); larger: one wavefront each
            for (int b = 4 * w; b < kdiv; b += 4 * nw) {   // wave-uniform trip count
                const int j = b + (lane_id() >> 4);
                QtNode nd{};
                int cnt = 0;
                if (j < kdiv) {
                    nd = na[ia[j]];
                    cnt = nd.cnt <= 16 ? nd.cnt : 0;
                }
                const int4 c = qt_group16_split(nd, cnt, P, T);
                if (cnt > 0 && (lane_id() & 15) == 0) cc[j] = c;
            }
            for (int j = w; j < kdiv; j += nw) {
                const int cn = na[ia[j]].cnt;
                if (cn <= 16 || (!WV && cn > QT_BIG)) continue;   // wave-uniform
                const int4 c = qt_wave_split(na[ia[j]], P, T);
                if (lane_id() == 0) cc[j] = c;
            }
            if (!WV && s_anybig) {   // block-uniform (set before the scans' barriers)
                for (int j = 0; j < kdiv; j++) {
                    if (na[ia[j]].cnt <= QT_BIG) continue;   // block-uniform
                    const int4 c = qt_block_split(na[ia[j]], P, T, s_split);
                    if (qtid == 0) cc[j] = c;
                }
            }
            qt_sync<WV>();
            QT_SUBSTAMP(57);
            // group positions: reverse processing order; divisibles: forward order.  The ne and dv counts
            // share one block scan (16-bit halves: a chunk's totals are <= 4 blockDim); with one chunk
            // (kdiv <= blockDim, every small level) the scan's total is the grand total the reverse
            // order needs, so the separate total pass and its two barriers are skipped (round 5)
            int ne_carry = 0, dv_carry = 0, ne_total = 0;
            if (kdiv > QBD) {   // block-uniform
                int part = 0;
                for (int j = qtid; j < kdiv; j += QBD) part += ne4(cc[j]);
                part = wave_sum_i32(part);
                if (lane_id() == 0) tmp[8 + w] = part;
                qt_sync<WV>();
                for (int q = 0; q < nw; q++) ne_total += tmp[8 + q];
                qt_sync<WV>();
            }
            for (int b = 0; b < kdiv; b += QBD) {
                const int j = b + qtid;
                const int4 c = j < kdiv ? cc[j] : make_int4(0, 0, 0, 0);
                int tt;
                const int ex = grp_excl_scan<WV>(ne4(c) | (dv4(c) << 16), tmp, &tt);
                const int t1 = tt & 0xffff, t2 = tt >> 16, ex_ne = ex & 0xffff, ex_dv = ex >> 16;
                if (kdiv <= QBD) ne_total = t1;
                if (j < kdiv) {
                    const int incl = ne_carry + ex_ne + ne4(c);
                    const int gpos = ne_total - incl;   // sum of ne over items after j
                    qt_emit_children(na[ia[j]], c, gpos, dv_carry + ex_dv, nb, divs, NC);
                }
                ne_carry += t1;
                dv_carry += t2;
            }
            const int n_new = ne_total + nnd;
            QT_SUBSTAMP(55);   // (thread 0: its emit done)
            for (int i = qtid; i < n; i += QBD)
                if (na[i].cnt <= 1 && ne_total + ib[i] < NC) nb[ne_total + ib[i]] = na[i];
            // commit: the single points of the non-divisible nodes join the split nodes' points in
            // T, which becomes P (every thread swaps the same pointers)
            for (int i = qtid; i < n; i += QBD)
                if (na[i].cnt == 1) T[na[i].beg] = P[na[i].beg];
            {
                uint32_t* t = P;
                P = T;
                T = t;
            }
            qt_sync<WV>();
            QT_SUBSTAMP(58);
            if (qtid == 0) {
                if (n_new > NC) { s_fail = 1; atomicOr(fault, FAULT_QT_NODES); }
                s_n = min(n_new, NC);
                s_ndiv = dv_carry;
                s_anybig = 0;
                if (n_new >= nfeat || n_new == n || s_fail) s_state = 2;
                else if (n_new + 3 * dv_carry > nfeat) s_state = 1;
            }
            qt_sync<WV>();
            QT_SUBSTAMP(59);
            QtNode* t = na; na = nb; nb = t;
        } else {
            // Phase 2 round (:632-672): split the previous round's divisible nodes, largest
            // first (std::sort, emulated), stopping as soon as the list reaches nfeat.
            const int m = s_ndiv;
            for (int j = qtid; j < m; j += QBD) prev[j] = divs[j];
            qt_sync<WV>();
            QT_STAMP(40 + 4 * min(p2_round, 5));
            {
                int* seg = reinterpret_cast<int*>(cc);   // cc (4 NC ints) is free until the splits below
                qt_sort_block<WV>(prev, m, ia, ib, seg, seg + NC, divs, seg + 2 * NC, NC / 3, s_sortcnt);
            }
            QT_STAMP(41 + 4 * min(p2_round, 5));
            for (int j = qtid; j < m; j += QBD) cc[j] = qt_thread_count(na[prev[j].node], P);
            for (int i = qtid; i < n; i += QBD) ia[i] = 0;   // erased flags
            if (qtid == 0) s_proc = m;
            qt_sync<WV>();
            // first sorted item whose split brings the list to nfeat (:666-667), by prefix sums
            {
                int carry2 = 0;
                for (int b = 0; b < m; b += QBD) {
                    const int j = b + qtid;
                    const int d = j < m ? ne4(cc[j]) - 1 : 0;
                    int tot;
                    const int ex = grp_excl_scan<WV>(d, tmp, &tot);
                    if (j < m && n + carry2 + ex + d >= nfeat) atomicMin(&s_proc, j + 1);
                    carry2 += tot;
                }
            }
            qt_sync<WV>();
            const int proc = s_proc;
            QT_STAMP(42 + 4 * min(p2_round, 5));
            for (int j = qtid; j < proc; j += QBD) ia[prev[j].node] = 1;
            // split the processed prefix only: small nodes one thread each, large ones one wave each
            for (int b = 4 * w; b < proc; b += 4 * nw) {   // <= 16 points: 16-lane groups
                const int j = b + (lane_id() >> 4);
                QtNode nd{};
                int cnt = 0;
                if (j < proc) {
                    nd = na[prev[j].node];
                    cnt = nd.cnt <= 16 ? nd.cnt : 0;
                }
                (void)qt_group16_split(nd, cnt, P, T);
            }
            for (int j = w; j < proc; j += nw)
                if (na[prev[j].node].cnt > 16) (void)qt_wave_split(na[prev[j].node], P, T);
            qt_sync<WV>();
            int ne_total = 0;   // (one packed scan; the total pass only for more than one chunk, as phase 1)
            if (proc > QBD) {   // block-uniform
                int part = 0;
                for (int j = qtid; j < proc; j += QBD) part += ne4(cc[j]);
                part = wave_sum_i32(part);
                if (lane_id() == 0) tmp[8 + w] = part;
                qt_sync<WV>();
                for (int q = 0; q < nw; q++) ne_total += tmp[8 + q];
                qt_sync<WV>();
            }
            int ne_carry = 0, dv_carry = 0;
            for (int b = 0; b < proc; b += QBD) {
                const int j = b + qtid;
                const int4 c = j < proc ? cc[j] : make_int4(0, 0, 0, 0);
                int tt;
                const int ex = grp_excl_scan<WV>(ne4(c) | (dv4(c) << 16), tmp, &tt);
                const int t1 = tt & 0xffff, t2 = tt >> 16, ex_ne = ex & 0xffff, ex_dv = ex >> 16;
                if (proc <= QBD) ne_total = t1;
                if (j < proc) {
                    const int gpos = ne_total - (ne_carry + ex_ne + ne4(c));
                    qt_emit_children(na[prev[j].node], c, gpos, dv_carry + ex_dv, nb, divs, NC);
                }
                ne_carry += t1;
                dv_carry += t2;
            }
            // survivors keep their order after the new groups
            int surv = 0;
            for (int b = 0; b < n; b += QBD) {
                const int i = b + qtid;
                const int keep = (i < n && !ia[i]) ? 1 : 0;
                int tot;
                const int ex = grp_excl_scan<WV>(keep, tmp, &tot);
                if (keep && ne_total + surv + ex < NC) nb[ne_total + surv + ex] = na[i];
                surv += tot;
            }
            for (int j = w; j < proc; j += nw) {
                const QtNode& p = na[prev[j].node];
                for (int q = lane_id(); q < p.cnt; q += 64) P[p.beg + q] = T[p.beg + q];
            }
            qt_sync<WV>();
            if (qtid == 0) {
                const int n_new = ne_total + surv;
                if (n_new > NC) { s_fail = 1; atomicOr(fault, FAULT_QT_NODES); }
                s_n = min(n_new, NC);
                s_ndiv = dv_carry;
                if (n_new >= nfeat || n_new == n || s_fail) s_state = 2;
            }
            qt_sync<WV>();
            QT_STAMP(43 + 4 * min(p2_round, 5));
            p2_round++;
            QtNode* t = na; na = nb; nb = t;
        }
    }

    // ---- retain the best point per node (:677-692): strict '>' => first maximum wins.  One lane
    //      per node (nodes are small at this point).
    const int n = s_n;
    uint32_t* out = sel + (long long)f * g.out_frame + L.out_base;
    if (n > L.out_cap && qtid == 0) atomicOr(fault, FAULT_OUT_CAP);
    for (int i = qtid; i < n && i < L.out_cap; i += QBD) {
        const QtNode nd = na[i];
        int bs = -1;
        uint32_t best = 0;
        for (int j0 = 0; j0 < nd.cnt; j0 += 4) {
            uint32_t r[4];
#pragma unroll
            for (int q = 0; q < 4; q++) r[q] = j0 + q < nd.cnt ? P[nd.beg + j0 + q] : 0;
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (j0 + q < nd.cnt && kp_s(r[q]) > bs) { bs = kp_s(r[q]); best = r[q]; }
        }
        out[i] = best;
    }
    if (qtid == 0) *scnt = min(n, L.out_cap);
    QT_STAMP(63);
#ifdef ORB_QT_STAMPS
    if (qtid == 0 && f * g.nlevels + l < 4096) {
        g_qt_wg[2 * (f * g.nlevels + l)] = qt_t0;
        g_qt_wg[2 * (f * g.nlevels + l) + 1] = __builtin_amdgcn_s_memtime();
    }
#endif
}

// ------------------------------------------------------------------------------------------
// 4. orientation + descriptor
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float fast_atan2_dev(float y, float x) {
    const float k = (float)(180 / M_PI);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    // the reference's two branches (ax >= ay: ay / ax, else 90 - f(ax / ay)) with one division:
    // the same operations on the same operands
    const float ax = fabsf(x), ay = fabsf(y);
    const bool xm = ax >= ay;
    const float c = (xm ? ay : ax) / ((xm ? ax : ay) + (float)DBL_EPSILON);
    const float c2 = c * c;
    float a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    if (!xm) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

constexpr int RS = 48;   // LDS raw-patch row stride (16-byte aligned rows for the blur's b128 reads)

// Horizontal Q8 blur as v_mfma_i32_16x16x64_i8 products C[m][n] = sum_k A[m][k] B[k][n]: m = blurred
// column, n = patch row, k = raw column; A = the 7-tap Toeplitz band A[m][k] = K[k - m]
// (K = 18 34 48 56 48 34 18), B = raw pixels as i8 (p - 128; sum K = 256, so the accumulator starts
// at 128 * 256).  Lane l holds A rows m = l % 16 (+16 mt), k = 16 (l / 16) .. +15 — the same k
// split as its B bytes, so the hardware's k order inside a lane group does not matter.
struct HBlurA { uint32_t v[3][64][4]; };   // [m tile][lane][dword]
constexpr HBlurA make_hblur_a() {
    HBlurA t{};
    const int K[7] = {18, 34, 48, 56, 48, 34, 18};
    for (int mt = 0; mt < 3; mt++)
        for (int l = 0; l < 64; l++)
            for (int d = 0; d < 4; d++) {
                uint32_t w = 0;
                for (int b = 0; b < 4; b++) {
                    const int o = 16 * (l >> 4) + 4 * d + b - (l & 15) - 16 * mt;
                    if (o >= 0 && o < 7) w |= (uint32_t)K[o] << (8 * b);
                }
                t.v[mt][l][d] = w;
            }
    return t;
}

// IC_Angle (:74-101) as the same i8 products on the blur's B fragments: D_t = A_t B_nt chained over
// the three row tiles, with A_t[m][k] = the disk weight of patch pixel (row m + 16 nt, column k) —
// u = k - 21 for m_10, v = m + 16 nt - 21 for m_01, 0 outside the disk |v| <= 15, |u| <= umax[|v|].
// The diagonal D[n][n] is then the weighted sum of patch row n (+16 nt), and its trace the moment.
// The disk is symmetric in u and in v, so sum(weights) = 0 and the i8 offset (p - 128) cancels.
struct AngleA { uint32_t v[3][2][64][4]; };   // [row tile][m_10, m_01][lane][dword]
constexpr AngleA make_angle_a() {
    AngleA t{};
    for (int nt = 0; nt < 3; nt++)
        for (int l = 0; l < 64; l++)
            for (int d = 0; d < 4; d++)
                for (int b = 0; b < 4; b++) {
                    const int v = (l & 15) + 16 * nt - 21, u = 16 * (l >> 4) + 4 * d + b - 21;
                    const int av = v < 0 ? -v : v, au = u < 0 ? -u : u;
                    if (av > 15 || au > c_umax_h[av]) continue;
                    t.v[nt][0][l][d] |= (uint32_t)(uint8_t)(int8_t)u << (8 * b);
                    t.v[nt][1][l][d] |= (uint32_t)(uint8_t)(int8_t)v << (8 * b);
                }
    return t;
}
// describe's constant tables in ONE symbol, read through one buffer resource (a lane's 16 bytes at
// lane * 16 + a compile-time offset): one address materialisation instead of one s_getpc + 64-bit add per
// table load (13 loads, ~39 SALU instructions per keypoint wave, in a kernel bound by SALU issue; round 6)
struct DescTabs {
    HBlurA hb;                              // 3 KiB
    AngleA an;                              // 6 KiB
    float pat[1024];                        // bit_pattern_31_ (:142-400) as floats (the samples' operands), 4 KiB
};
__constant__ __attribute__((aligned(16))) DescTabs c_desc_tabs = {make_hblur_a(), make_angle_a(), {
#include "orb_pattern31.inc"
}};
constexpr int DT_HB = 0, DT_AN = 3 * 1024, DT_PAT = 9 * 1024;
// the fdlibm sincos constants as a __constant__ copy: scalar loads instead of two s_mov_b32 per double
__constant__ __attribute__((aligned(16))) SincosK c_sincos_k = kSincosK;
static_assert(sizeof(HBlurA) == 3 * 1024 && sizeof(AngleA) == 6 * 1024, "table offsets");
typedef int i4v __attribute__((ext_vector_type(4)));

#ifdef ORB_DESC_STAMPS
// diagnostic build: phase stamps of every 16th describe wavefront (8 words each)
__device__ unsigned long long g_desc_stamps[1024 * 8];
#define DESC_STAMP(k)                                                                              \
    do {                                                                                           \
        if (lane == 0 && (lb & 15) == 0 && (lb >> 4) < 1024) g_desc_stamps[(lb >> 4) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define DESC_STAMP(k) do {} while (0)
#endif

// One workgroup = one wavefront = one selection slot (a kept keypoint or an empty slot).
constexpr int PATCH_DW = (PATCH + 3) / 4;                 // dwords staged per raw-patch row
#ifndef DESC_ANGLE_MFMA
#define DESC_ANGLE_MFMA 1   // IC_Angle as i8 products on the blur's B fragments (0: LDS disk reads; A/B)
#endif
#ifndef DESC_ANGLE_FIRST
#define DESC_ANGLE_FIRST 0   // A/B: the angle products before the blur's
#endif
#ifndef DESC_PAT_EARLY
#define DESC_PAT_EARLY 1   // the rBRIEF pattern loads issued before the angle chain (0: at the samples; A/B)
#endif
#ifndef DESC_SCALAR_PRE
#define DESC_SCALAR_PRE 1   // the slot's keypoint word and the frame's level counts by scalar loads (0: one vector load)
#endif
#ifndef DESC_HBT
#define DESC_HBT 1   // blurred patch column-major: a sample's 7 vertical taps in 4 dwords (0: row-major, 7 u16 reads)
#endif
// column-major blurred patch: column c (0..39) holds rows 0..47 at u16 c * HCS; 26 dwords per column
// put the 16 columns of one b64 store group on distinct bank pairs
constexpr int HCS = 52;
static_assert(HCS % 4 == 0 && HCS >= 48, "8-byte aligned columns of 48 rows (the tiles' slack rows)");
constexpr int HB_ELEMS = DESC_HBT ? 40 * HCS : 48 * HBS;

// One kept keypoint (level l, selection word k, output row o of the frame's slots): the raw 43x43 patch,
// IC_Angle, the 7x7 Q8 blur and the rBRIEF samples, written to kps / desc at row o.  One wavefront.
template <int TRIG>
__device__ __forceinline__ void describe_keypoint(const Geom& g, int l, int f, uint32_t k, long long o,
                                                  const uint8_t* __restrict__ in, long long in_fstride, int in_step,
                                                  const uint8_t* __restrict__ pyr, orbx_keypoint* __restrict__ kps,
                                                  uint8_t* __restrict__ desc, uint16_t* Hb, int lb) {
    const int lane = threadIdx.x;
    uint8_t* R = reinterpret_cast<uint8_t*>(Hb);
    const LevelDev& L = g.lv[l];
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<DescTabs*>(&c_desc_tabs), 0, (int)sizeof(DescTabs), 0x00020000);
    // a lane's 16 bytes of 1 KiB table row `row` (hb: mt; an: 2 nt + moment; pat: r), constant offsets
    auto tab16 = [&](int off) -> i4v {
        return __builtin_bit_cast(i4v, __builtin_amdgcn_raw_buffer_load_b128(trs, off + 16 * lane, 0, 0));
    };
    DESC_STAMP(0);
    // the blur's constant A fragments, in flight under the patch load
    i4v afr[3];
#pragma unroll
    for (int mt = 0; mt < 3; mt++) afr[mt] = tab16(DT_HB + 1024 * mt);

    const int kx = kp_x(k), ky = kp_y(k), score = kp_s(k);
    // the level's base and row step: both candidates' operands come with the kernel arguments' first
    // scalar round trip, and the selection is an s_cselect (no branch to a second round trip)
    const uint8_t* img0 = in + (long long)f * in_fstride;
    const uint8_t* imgl = pyr + (long long)f * g.pyr_frame_bytes + L.off;
    const uint8_t* img = l == 0 ? img0 : imgl;
    const int step = l == 0 ? in_step : L.stride;
    // 43x43 neighbourhood (reflect-101 outside the level, as the blur's BORDER_REFLECT_101)
    if (kx >= 21 && ky >= 21 && kx + 21 + 8 < L.w && ky + 21 < L.h) {
        // interior: 16 lanes per row (dword d of row 4k + lane/16), 11 row groups; all loads in
        // flight before the LDS stores
        constexpr int NG = (PATCH + 3) / 4;
        const uint8_t* base = img + (long long)(ky - 21) * step + (kx - 21);
        const int roff = lane >> 4, d = min(lane & 15, PATCH_DW - 1);
        uint32_t v[NG];
        if ((step & 3) == 0) {
            // dword-multiple row step (every pyramid level; level 0 unless the caller's step is
            // odd): one wave-uniform realignment, buffer loads off a scalar resource with a per-lane
            // constant voffset and a per-group soffset (no address VALU).  The resource ends at the
            // level's last pixel: row 43 of the last group (never stored) may lie past it and reads 0.
            const int m = __builtin_amdgcn_readfirstlane((int)(reinterpret_cast<uintptr_t>(base) & 3u));
            const int nrec = (L.h - 1 - (ky - 21)) * step + L.w - (kx - 21) + m;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base - m), 0, nrec, 0x00020000);
            const int voff = roff * step + 4 * d;
#pragma unroll
            for (int k = 0; k < NG; k++) {
                const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 4 * k * step, 0);
                v[k] = __builtin_amdgcn_alignbyte(t[1], t[0], m);
            }
        } else {
            // odd caller step: a per-lane realignment (v_alignbyte of the aligned dword pair)
            const int loff = roff * step + 4 * d;
            uint32_t lo[NG], hi[NG];
            int sh[NG];
#pragma unroll
            for (int k = 0; k < NG; k++) {
                const uint8_t* gb = base + (long long)min(4 * k, PATCH - 1 - roff) * step;   // rows <= 42
                const uint8_t* pbyte = gb + loff;
                const int m = (int)(reinterpret_cast<uintptr_t>(pbyte) & 3);
                const uint32_t* pw = reinterpret_cast<const uint32_t*>(pbyte - m);
                lo[k] = pw[0];
                hi[k] = pw[1];
                sh[k] = m;
            }
#pragma unroll
            for (int k = 0; k < NG; k++) v[k] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh[k]);
        }
        static_assert(4 * (NG - 1) + 3 == PATCH, "the last row group holds three patch rows");
        if ((lane & 15) < PATCH_DW) {
            uint32_t* rrow = reinterpret_cast<uint32_t*>(&R[roff * RS + 4 * d]);
#pragma unroll
            for (int k = 0; k < NG - 1; k++) rrow[k * RS] = v[k];   // row 4k + roff: (4k + roff) * RS / 4 dwords
            if (roff < 3) rrow[(NG - 1) * RS] = v[NG - 1];
        }
    } else if (lane < PATCH) {
        const int xx = reflect101(kx - 21 + lane, L.w);
        uint8_t v[PATCH];
#pragma unroll
        for (int r = 0; r < PATCH; r++) v[r] = img[(long long)reflect101(ky - 21 + r, L.h) * step + xx];
#pragma unroll
        for (int r = 0; r < PATCH; r++) R[r * RS + lane] = v[r];
    }
    __syncthreads();
    DESC_STAMP(1);

#if !DESC_ANGLE_MFMA   // the round-3 IC_Angle (LDS disk reads), for A/B builds
    // IC_Angle on the unblurred level, patch centre (21, 21).  Lane = (row parity, u + 15): lanes
    // 0-31 take rows +-v for odd v, lanes 32-63 for v + 1, so the 15 row pairs take 8 steps.
    int m10 = 0, m01 = 0;
    {
        const int hv = lane >> 5, u = (lane & 31) - 15;   // u = 16 on lanes 31 / 63: outside every umax
        const uint8_t* cp = R + 21 * RS + 21 + u + hv * RS;
        // every read unconditional (all inside the 43x43 patch) and issued together; the disk mask
        // is applied to the products
        int vp[8], vm[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int vv = 2 * t + 1;
            vp[t] = cp[vv * RS];
            vm[t] = cp[-(vv + 2 * hv) * RS];
        }
        const int c0 = R[21 * RS + 21 + u];
        m10 = (hv == 0 && u <= 15) ? u * c0 : 0;
        // the disk mask as lane-constant multipliers (branch-free multiply-adds)
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int vv = 2 * t + 1;
            const int v = vv + hv;
            const int um = hv ? (vv + 1 <= 15 ? c_umax_h[vv + 1] : -1) : c_umax_h[vv];
            const bool in = u >= -um && u <= um;
            const int vin = in ? v : 0, uin = in ? u : 0;
            m01 += vin * (vp[t] - vm[t]);
            m10 += uin * (vp[t] + vm[t]);
        }
    }
    m10 = wave_sum_i32(m10);
    m01 = wave_sum_i32(m01);
#endif
    // The raw rows as i8 B fragments (p - 128), shared by the angle and the blur products: lane
    // (n, g) holds columns 16 g .. +15 of patch row n + 16 nt.  Every read of R is issued before the
    // first Hb write (R aliases Hb; one wavefront's LDS operations complete in order).
    const int n = lane & 15, lg = lane >> 4;
    i4v bfr[3];
#pragma unroll
    for (int nt = 0; nt < 3; nt++) {
        bfr[nt] = *reinterpret_cast<const i4v*>(&R[(n + 16 * nt) * RS + 16 * lg]);
        bfr[nt] ^= (int)0x80808080u;
    }

#if DESC_ANGLE_MFMA
    // IC_Angle on the unblurred patch, centre (21, 21), as six more products (c_angle_a) chained
    // over the row tiles; the diagonal element D[n][n] sits in lane 20 (n / 4) + n % 4, register
    // n % 4: each lane takes register lane % 4, and the quads at row offset 4 (lane / 16) are summed.
    int m10 = 0, m01 = 0;
    auto angle_products = [&](const i4v (&au)[3], const i4v (&av)[3]) {
        i4v du = {0, 0, 0, 0}, dv = {0, 0, 0, 0};
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            du = __builtin_amdgcn_mfma_i32_16x16x64_i8(au[nt], bfr[nt], du, 0, 0, 0);
            dv = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[nt], bfr[nt], dv, 0, 0, 0);
        }
        const bool q1 = lane & 1, q2 = lane & 2;
        int tu = q2 ? (q1 ? du.w : du.z) : (q1 ? du.y : du.x);
        int tv = q2 ? (q1 ? dv.w : dv.z) : (q1 ? dv.y : dv.x);
        tu += dpp_i32<0xB1>(tu);   // quad_perm [1,0,3,2]
        tv += dpp_i32<0xB1>(tv);
        tu += dpp_i32<0x4E>(tu);   // quad_perm [2,3,0,1]
        tv += dpp_i32<0x4E>(tv);
        m10 = __builtin_amdgcn_readlane(tu, 0) + __builtin_amdgcn_readlane(tu, 20) +
              __builtin_amdgcn_readlane(tu, 40) + __builtin_amdgcn_readlane(tu, 60);
        m01 = __builtin_amdgcn_readlane(tv, 0) + __builtin_amdgcn_readlane(tv, 20) +
              __builtin_amdgcn_readlane(tv, 40) + __builtin_amdgcn_readlane(tv, 60);
    };
#if DESC_ANGLE_FIRST   // the angle products (and the atan / sincos chain) ahead of the blur's
    {
        i4v au[3], av[3];
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            au[nt] = tab16(DT_AN + 1024 * (2 * nt));
            av[nt] = tab16(DT_AN + 1024 * (2 * nt + 1));
        }
        angle_products(au, av);
    }
#endif
#endif

    // horizontal Q8 blur on the matrix cores (c_hblur_a): 3 x 3 tiles of 16 blurred columns x 16
    // rows; lane (n, g) of tile (mt, nt) gets columns 16 mt + 4 g .. +3 of row 16 nt + n.  Rows past
    // 42 (stored into slack rows) and columns past 36 are computed from neighbouring bytes and never
    // read; columns past 39 are not stored.
    {
#if defined(DESC_DIAG_NOPS) && DESC_DIAG_NOPS == 1   // diagnostic bisection only: drain before the products
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
        const i4v cinit = {128 * 256, 128 * 256, 128 * 256, 128 * 256};
        i4v acc[3][3];   // all nine products first: their results are not waited on one at a time
#pragma unroll
        for (int nt = 0; nt < 3; nt++)
#pragma unroll
            for (int mt = 0; mt < 3; mt++)
#if DESC_HBT
                // the transposed product (patch rows as A, the blur band as B: the same k pairing):
                // lane (n, g) gets rows 16 nt + 4 g .. +3 of blurred column 16 mt + n
                acc[nt][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bfr[nt], afr[mt], cinit, 0, 0, 0);
#else
                acc[nt][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr[mt], bfr[nt], cinit, 0, 0, 0);
#endif
#if defined(DESC_DIAG_NOPS) && DESC_DIAG_NOPS == 2   // diagnostic bisection only: drain after the products
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
#ifdef DESC_KEEPALIVE_DIAG
        // diagnostic only (tests/test_dpp_hazards.py): round 4's empty-asm keep-alives of the products'
        // operands, the build whose descriptors differed between identical runs
        asm volatile("" ::"v"(bfr[0]), "v"(bfr[1]), "v"(bfr[2]));
        asm volatile("" ::"v"(afr[0]), "v"(afr[1]), "v"(afr[2]));
#endif
        auto put = [&](int nt, int mt) {
            uint2 pk;
            pk.x = __builtin_amdgcn_perm((uint32_t)acc[nt][mt].y, (uint32_t)acc[nt][mt].x, 0x05040100u);
            pk.y = __builtin_amdgcn_perm((uint32_t)acc[nt][mt].w, (uint32_t)acc[nt][mt].z, 0x05040100u);
#if DESC_HBT
            *reinterpret_cast<uint2*>(&Hb[(16 * mt + n) * HCS + 16 * nt + 4 * lg]) = pk;   // rows 43..47: slack
#else
            *reinterpret_cast<uint2*>(&Hb[(16 * nt + n) * HBS + 16 * mt + 4 * lg]) = pk;   // rows 43..47: slack
#endif
        };
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            put(nt, 0);
            put(nt, 1);
        }
#if DESC_HBT
        if (n < 8) {   // columns 32..39 of the third tile
#else
        if (lg < 2) {   // columns 32..39 of the third tile (40..47 would wrap into the next row)
#endif
#pragma unroll
            for (int nt = 0; nt < 3; nt++) put(nt, 2);
        }
    }

#if DESC_PAT_EARLY
    // the lane's four pattern pairs, loaded before the angle / atan / sincos chain hides their latency
    float4 pat[4];
#pragma unroll
    for (int r = 0; r < 4; r++) pat[r] = __builtin_bit_cast(float4, tab16(DT_PAT + 1024 * r));
#endif
#if DESC_ANGLE_MFMA && !DESC_ANGLE_FIRST
    {
        i4v au[3], av[3];
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            au[nt] = tab16(DT_AN + 1024 * (2 * nt));
            av[nt] = tab16(DT_AN + 1024 * (2 * nt + 1));
        }
        angle_products(au, av);
    }
#endif
    const float angle = fast_atan2_dev((float)m01, (float)m10);
    DESC_STAMP(2);
    __syncthreads();

    const float factorPI = (float)(M_PI / 180.f);
    const float ang = angle * factorPI;
    float a, b;   // (float)::cos / ::sin((double)ang) or cosf / sinf, sincos_f.h (each checked on every float in range)
    DESC_STAMP(3);
#ifdef DESC_SINCOS_COST_DIAG   // diagnostic A/B only: hardware sin / cos (inexact) to price the exact path
    a = __cosf(ang);
    b = __sinf(ang);
#else
    if (TRIG) sincosf_glibc(ang, &b, &a);
    else sincos_f2d_k(ang, &b, &a, c_sincos_k);
#endif
    DESC_STAMP(4);
    auto sample = [&](float x, float y) -> int {
        // byte offset of blurred pixel (18 + dy, 18 + dx) from the rounded floats (exact integers)
        const float dy = rintf(x * b + y * a), dx = rintf(x * a - y * b);
#if DESC_HBT
        // u16 index of blurred pixel (18 + dy, 18 + dx) in the column-major map; its 7 vertical taps
        // (rows 18 + dy .. +6) are u16 q .. q + 6, inside dwords q / 2 .. q / 2 + 3, realigned by q's parity
        const int q = (int)fmaf(dx, (float)HCS, dy + (float)(18 * HCS + 18));
        const uint32_t* cw = reinterpret_cast<const uint32_t*>(Hb) + (q >> 1);
        const uint32_t d0 = cw[0], d1 = cw[1], d2 = cw[2], d3 = cw[3];
        const uint32_t sh = (uint32_t)(q & 1) * 2u;   // bytes
        const us2 p01 = u2us(__builtin_amdgcn_alignbyte(d1, d0, sh));
        const us2 p23 = u2us(__builtin_amdgcn_alignbyte(d2, d1, sh));
        const us2 p45 = u2us(__builtin_amdgcn_alignbyte(d3, d2, sh));
        const us2 p6x = u2us(__builtin_amdgcn_alignbyte(d3, d3, sh));   // tap 6 in the low half
        const us2 k01 = {18, 34}, k23 = {48, 56}, k45 = {48, 34}, k6x = {18, 0};
        unsigned acc = __builtin_amdgcn_udot2(p6x, k6x, 1u << 15, false);
        acc = __builtin_amdgcn_udot2(p01, k01, acc, false);
        acc = __builtin_amdgcn_udot2(p23, k23, acc, false);
        acc = __builtin_amdgcn_udot2(p45, k45, acc, false);
        return (int)(acc >> 16);
#else
        const int ob = (int)fmaf(dy, (float)(2 * HBS), fmaf(dx, 2.f, (float)(2 * (18 * HBS + 18))));
        const uint16_t* col = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(Hb) + ob);
        // vertical taps as u16 pairs (d16 / d16_hi loads) into v_dot2_u32_u16, rounding bias as the
        // accumulator: 18 c0 + 34 c1 + 48 c2 + 56 c3 + 48 c4 + 34 c5 + 18 c6 + 2^15
        const us2 p01 = {col[0], col[HBS]}, p23 = {col[2 * HBS], col[3 * HBS]}, p45 = {col[4 * HBS], col[5 * HBS]};
        const us2 k01 = {18, 34}, k23 = {48, 56}, k45 = {48, 34};
        unsigned acc = __builtin_amdgcn_udot2(p01, k01, 18u * col[6 * HBS] + (1u << 15), false);
        acc = __builtin_amdgcn_udot2(p23, k23, acc, false);
        acc = __builtin_amdgcn_udot2(p45, k45, acc, false);
        return (int)(acc >> 16);
#endif
    };
    unsigned long long words[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
#if DESC_PAT_EARLY
        const float4 q = pat[r];
#else
        const float4 q = __builtin_bit_cast(float4, tab16(DT_PAT + 1024 * r));   // pairs 2p, 2p + 1
#endif
        words[r] = __ballot(sample(q.x, q.y) < sample(q.z, q.w));
    }
    DESC_STAMP(5);
    // The 32 descriptor bytes and the 7-word keypoint record are wave-uniform: v_writelane places
    // them in lanes 0..7 / 0..6 of one register each (no per-lane selects or branches), one store each.
    uint32_t dv = 0, kv = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        dv = writelane_u32((uint32_t)words[r], 2 * r, dv);
        dv = writelane_u32((uint32_t)(words[r] >> 32), 2 * r + 1, dv);
    }
    const float ks = l > 0 ? L.scale : 1.f;   // (:812-815: pt *= scaleFactors_[s] above level 0; x * 1 = x)
    kv = writelane_u32(__float_as_uint((float)kx * ks), 0, kv);
    kv = writelane_u32(__float_as_uint((float)ky * ks), 1, kv);
    kv = writelane_u32(__float_as_uint(L.size), 2, kv);
    kv = writelane_u32(__float_as_uint(angle), 3, kv);
    kv = writelane_u32(__float_as_uint((float)score), 4, kv);
    kv = writelane_u32((uint32_t)l, 5, kv);
    kv = writelane_u32(0xffffffffu, 6, kv);
    if (lane < 8) reinterpret_cast<uint32_t*>(desc + o * 32)[lane] = dv;
    if (lane < 7) reinterpret_cast<uint32_t*>(kps + o)[lane] = kv;
    DESC_STAMP(6);
}

#ifndef DESC_SLOT_TAB
#define DESC_SLOT_TAB 1   // the slot's level from a host table and the level's output range from a per-frame prefix (0: SWAR + 16 counts)
#endif
constexpr int LVP = 32;   // per-frame stride (ints) of describe's level prefix (nlevels + 1 <= 17 used; 128 B rows)

// Per frame: the exclusive prefix of the kept counts over levels (lvl_pre[f][l] = first output row of level
// l, lvl_pre[f][nl] = the frame's total) and counts[f].  One thread per frame, between the quadtree and
// describe; it takes the per-level sums out of every describe wavefront's scalar preamble (round 6: the
// 16-count load, the level compare chain and the prefix sum were ~150 of a wave's ~330 SALU instructions,
// and describe was SALU-issue-bound, SALUBusy 83 %).
// stat[0]: the batch's largest frame total (atomicMax; the host sizes the next batch's dense describe grid
// from it).
__global__ __launch_bounds__(256) void describe_prefix_kernel(const int* __restrict__ sel_cnt, int nl, int F,
                                                              int* __restrict__ lvl_pre, int32_t* __restrict__ counts,
                                                              int* __restrict__ stat) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    int acc = 0;
    int* pre = lvl_pre + (long long)f * LVP;
    for (int q = 0; q < nl; q++) {
        pre[q] = acc;
        acc += sel_cnt[f * nl + q];
    }
    pre[nl] = acc;
    counts[f] = acc;
    atomicMax(stat, acc);
}

// The dense describe grid (round 6): launch slot s of frame f IS output row s.  Its level is the number of
// levels 1..nl whose first row is <= s (one vector load of the frame's prefix, one ballot), its rank in the
// level s - pre[l], its selection word sel[f][out_base_l + rank].  A launch of C slots per frame covers the
// frames with at most C keypoints; C comes from the previous batch's largest total (stat[0]), so the grid
// no longer carries every level's out_cap slack (2024 slots for ~1395 keypoints per C2 pan frame, 31 % of
// the wavefronts empty), and describe_overflow_kernel covers rows >= C of any frame that has more.
struct DescGrid {
    int C;                 // slots per frame in this launch
    unsigned m;            // lb / C by the round-up magic (as divmod_of)
    int s1, s2;
};
template <int TRIG>
__device__ __forceinline__ void describe_dense_slot(const Geom& g, int f, int s, const uint8_t* __restrict__ in,
                                                    long long in_fstride, int in_step, const uint8_t* __restrict__ pyr,
                                                    const uint32_t* __restrict__ sel, orbx_keypoint* __restrict__ kps,
                                                    uint8_t* __restrict__ desc, int cap, const int* __restrict__ lvl_pre,
                                                    uint16_t* Hb, int lb) {
    const int lane = threadIdx.x, nl = g.nlevels;
    const int pq = lane <= nl ? lvl_pre[(long long)f * LVP + lane] : 0x7fffffff;
    const int T = __builtin_amdgcn_readlane(pq, nl);
    if (s >= T || s >= cap) return;   // wave-uniform
    const int l = popc64(__ballot(lane >= 1 && lane <= nl && pq <= s));
    const int pre_l = __builtin_amdgcn_readlane(pq, l);
    const uint32_t k = sel[(long long)f * g.out_frame + g.lv[l].out_base + (s - pre_l)];
    describe_keypoint<TRIG>(g, l, f, k, (long long)f * cap + s, in, in_fstride, in_step, pyr, kps, desc, Hb, lb);
}

// Rows >= C of the frames whose total exceeds the dense launch's C: a fixed grid of one-wave workgroups
// loops over the frames (wave w: frames w, w + grid, ...) and their extra rows.  Exits at once when no
// frame overflows.
template <int TRIG>
__global__ __launch_bounds__(64) void describe_overflow_kernel(Geom g, const uint8_t* __restrict__ in,
                                                               long long in_fstride, int in_step,
                                                               const uint8_t* __restrict__ pyr,
                                                               const uint32_t* __restrict__ sel,
                                                               orbx_keypoint* __restrict__ kps,
                                                               uint8_t* __restrict__ desc, int cap,
                                                               const int* __restrict__ lvl_pre, int F, int C) {
    __shared__ __attribute__((aligned(16))) uint16_t Hb[HB_ELEMS];
    for (int f = blockIdx.x; f < F; f += gridDim.x) {
        const int T = min(lvl_pre[(long long)f * LVP + g.nlevels], cap);
        for (int s = C; s < T; s++) {
            describe_dense_slot<TRIG>(g, f, s, in, in_fstride, in_step, pyr, sel, kps, desc, cap, lvl_pre, Hb,
                                      (int)blockIdx.x);
            __syncthreads();   // Hb is reused by the next row
        }
    }
}

// One wavefront per selection slot of a frame; slots past their level's kept count exit at once.
// TRIG: ComputeOrbDescriptor's cos / sin (:107): 0 = (float)::cos((double)angle), 1 = cosf / sinf.
template <int TRIG>
__global__ __launch_bounds__(64) void describe_kernel(Geom g, const uint8_t* __restrict__ in, long long in_fstride,
                                                      int in_step, const uint8_t* __restrict__ pyr,
                                                      const uint32_t* __restrict__ sel,
                                                      const int* __restrict__ sel_cnt, orbx_keypoint* __restrict__ kps,
                                                      uint8_t* __restrict__ desc, int32_t* __restrict__ counts,
                                                      int cap, const uint32_t* __restrict__ slot_tab,
                                                      const int* __restrict__ lvl_pre, DescGrid dg) {
    // the raw patch R is dead once every lane holds its row for the horizontal blur (one
    // wavefront: its LDS reads complete before its later writes), so the blurred rows Hb reuse it
    __shared__ __attribute__((aligned(16))) uint16_t Hb[HB_ELEMS];   // 43 blurred rows + 5 rows of blur slack
    static_assert(47 * RS + 64 <= HB_ELEMS * 2, "R (and the blur's reads of rows 43..47) must fit in Hb");
    const int lane = threadIdx.x;
    const int lb = xcd_swizzle(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    DESC_STAMP(7);   // entry (diagnostic build): the preamble's loads are timed from here
    if (dg.C > 0) {   // the dense grid (DescGrid): slot = output row
        const unsigned t = __umulhi((unsigned)lb, dg.m);
        const int fd = (int)((t + (((unsigned)lb - t) >> dg.s1)) >> dg.s2);
        (void)sel_cnt; (void)counts; (void)slot_tab;
        describe_dense_slot<TRIG>(g, fd, lb - fd * dg.C, in, in_fstride, in_step, pyr, sel, kps, desc, cap, lvl_pre, Hb,
                                  lb);
        return;
    }
    const int f = divmod_of(g, lb);
    const int s = lb - f * g.out_frame;   // selection slot (level-major, out_cap slots per level)
#if DESC_SLOT_TAB
    // slot -> (level, rank in the level) from the host's table, the level's output rows from the frame's
    // prefix (describe_prefix_kernel, which also wrote counts[f]): three scalar loads, no sums
    (void)sel_cnt;
    (void)counts;
    (void)lane;
    const uint32_t e = slot_tab[s];
    const uint32_t k = sel[(long long)f * g.out_frame + s];
    // both words in one scalar round trip (the compiler would sink k's load past the exits below, into a
    // third dependent round trip on every kept keypoint's chain)
    asm volatile("" ::"s"(e), "s"(k), "s"(cap), "s"(in), "s"(in_fstride), "s"(in_step), "s"(pyr), "s"(g.pyr_frame_bytes));
    const int l = (int)(e & 255u), i = (int)(e >> 8);
    const int2 pr = *reinterpret_cast<const int2*>(lvl_pre + (long long)f * LVP + l);
    {   // the level's fields describe_keypoint reads, in the same round trip as the prefix (kernarg, CSE'd)
        const LevelDev& L = g.lv[l];
        asm volatile("" ::"s"(pr.x), "s"(pr.y), "s"(L.w), "s"(L.h), "s"(L.stride), "s"(L.off));
    }
    if (i >= pr.y - pr.x) return;   // slot past the level's kept count
    const int oidx = pr.x + i;      // output order: level-major list order
    if (oidx >= cap) return;
#else
    (void)slot_tab;
    (void)lvl_pre;
    // The slot's level and the frame's per-level counts without a dependent chain of loads: the
    // level is the number of level starts (kernarg) <= s, and the level's output base is the sum of
    // the counts of the levels before it.
    const int nl = g.nlevels;
    // every address here is wave-uniform: scalar loads (the scalar cache path, not queued behind the
    // other wavefronts' patch loads); 16 counts read unconditionally (the count buffer has 64 B of slack)
    const uint32_t k = sel[(long long)f * g.out_frame + s];
    const int* cf = sel_cnt + f * nl;
    int cnt16[MAX_LEVELS];
#pragma unroll
    for (int q = 0; q < MAX_LEVELS; q++) cnt16[q] = cf[q];
    // levels >= nlevels carry 0x7fff (host; out_frame < 0x7fff checked there): a field x <= s iff bit
    // 15 of (x | 0x8000) - (s + 1) is clear, and no field borrows from the next
    int l = MAX_LEVELS;
    {
        const unsigned s1 = (unsigned)(s + 1) * 0x00010001u;
#pragma unroll
        for (int d = 0; d < MAX_LEVELS / 2; d++) l -= __popc(((g.lv_start[d] | 0x80008000u) - s1) & 0x80008000u);
    }
    int total = 0, lbase = 0, cnt_l = 0;
#pragma unroll
    for (int q = 0; q < MAX_LEVELS; q++) {
        const int cq = q < nl ? cnt16[q] : 0;
        total += cq;
        lbase += q < l ? cq : 0;
        cnt_l = q == l ? cq : cnt_l;
    }
    if (s == 0 && lane == 0) counts[f] = total;
    const int i = s - g.lv[l].out_base;
    if (i >= cnt_l) return;   // slot past the level's kept count
    const int oidx = lbase + i;   // output order: level-major list order
    if (oidx >= cap) return;
#endif
    describe_keypoint<TRIG>(g, l, f, k, (long long)f * cap + oidx, in, in_fstride, in_step, pyr, kps, desc, Hb, lb);
}

__global__ __launch_bounds__(256) void qt_sort_test_kernel(QtItem* items, int n, int* scratch) {
    __shared__ int s_cnt[2];
    qt_sort_block<false>(items, n, scratch, scratch + n, scratch + 2 * n, scratch + 3 * n,
                  reinterpret_cast<QtItem*>(scratch + 4 * n), scratch + 6 * n, n / 3 + 2, s_cnt);
}

}  // namespace orbamd

// ==============================================================================================
// Host side: extractor object and C-ABI
// ==============================================================================================
using namespace orbamd;

struct orbx_extractor {
    orbx_params p;
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> quota;
    std::mutex mu;   // one instance is not re-entrant (as the reference's mutable members)

    // geometry for the current image size
    int g_rows = -1, g_cols = -1;
    Geom geom;
    std::vector<CellDev> cells;
    int NC = 0, PTC = 0;
    size_t qt_lds = 0;
    int qt_ptc0 = 0;        // ORBX_QT_PTC0 (tuning knob): level 0 in its own launch with this LDS point capacity
    size_t qt_lds0 = 0;
    // round 6: the small levels [qtw_l0, nlevels) as one tree per wavefront (quadtree_kernel<true>),
    // four per workgroup, each with its own node capacity / LDS point capacity (ORBX_QT_WAVE=1; exact,
    // measured: pan quadtree -2 %, textured +13 % -- off by default, DESIGN §4 quadtree round 6)
    int qt_wave = 0, qt_wave_wg = 2, qtw_l0 = 0, qtw_nc = 0, qtw_ptc = 0;
    size_t qtw_lds = 0;
    FastLds fl;
    size_t fast_lds = 0;
    int fast_cpw = 16;  // FAST cells per wavefront (4 -> 16: -2 % pan, -17 % textured: fewer first cells without a speculation hint; ORBX_FAST_CPW)
    // a cell runs the speculative iniThFAST pass when the wavefront's previous cell kept at least
    // fast_spec corners at iniThFAST (texture-rich regions); 0 = never (ORBX_FAST_SPEC)
    int fast_spec = 8;
    int fast_pair = 0;      // ORBX_FAST_PAIR=1: fast_cells_kernel<..., PAIR> (two cells per pass; round 6)
    bool fast_pair_on = false;   // requested and the geometry allows it (consecutive strip cells adjacent)
    // a strip's first cell (no predecessor) speculates when its cell kept >= fast_spec corners in frame 0
    // (cell_cnt's frame-0 slot; ORBX_FAST_SPEC_FIRST=0: never)
    int fast_spec_first = 1;
    int nsub = 1;       // sub-batches on side streams (launch_batch; ORBX_NSUB)
    int debug_nc = 0;
    int debug_qt_block = 0;   // test hook (ORBX_DEBUG_QT_BLOCK): launch quadtree_kernel with this block size (FAULT_BLOCK_SIZE)
    uint32_t fault_host = 0;   // test hook (ORBX_DEBUG_NC): shrink the quadtree node capacity to induce FAULT_QT_NODES
    int pyr_mfma = 0;   // ORBX_PYR_MFMA=1: pyramid_pair_mfma_kernel where the level pair's tables fit (measured slower: DESIGN §4)
    std::vector<char> pyr_mfma_ok;   // per level l: the pair (l, l+1) fits pyramid_pair_mfma_kernel
    DevBuf d_pyrmt, d_pyrkb;         // its A / C fragments per 16-column block, and the blocks' first tap column
    int pyr_pair = 2;   // pyramid_pair_kernel for levels (1,2), (3,4), (5,6) (level 0 16-byte aligned); 1: (2,3), (4,5), (6,7) (ORBX_PYR_PAIR)
    // OpenCV-build switches (orbx_set_opencv_compat; ORBX_TRIG / ORBX_RESIZE_TAIL)
    int trig_float = 0;    // ComputeOrbDescriptor's cos / sin: 0 ::cos(double), 1 cosf / sinf
    // the resize's tail mode V (0, default: the SIMD rounding on every column, as OpenCV's uchar
    // specialisation of VResizeLinear does in its unrolled and scalar tails too; 8-64: a tail with
    // FixedPtCast rounding after a V-byte vector loop; 1: FixedPtCast everywhere).  Parity unpinned.
    int resize_simd = 0;
    std::vector<std::pair<hipStream_t, hipEvent_t>> sub;
    hipEvent_t fork_ev = nullptr;
    // level-split overlap (launch_chunk): level 0's FAST + quadtree on a side stream.  Off by
    // default: measured no gain at C2 (the concurrent kernels share the CUs: pyramid 0.26 -> 0.42 ms,
    // wall time unchanged), and it keeps the per-kernel launch times uncontended.  ORBX_LEVEL_OVERLAP=1
    bool lvl_overlap = false;
    hipStream_t lvl_side = nullptr;
    hipEvent_t lvl_fork = nullptr, lvl_join = nullptr;
    DevBuf d_cells, d_xtab, d_ytab;
    DevBuf d_strips;                 // FAST work items: column strips of cells (fast_cells_kernel)
    DevBuf d_slottab;                // describe: selection slot -> level | rank << 8 (out_frame entries)
    DevBuf d_lvlpre;                 // describe: per-frame level prefix of the kept counts (LVP ints per frame)
    std::vector<int> strip_beg;      // first strip of each level (nlevels + 1 entries)

    // workspace for up to ws_frames frames
    int ws_frames = 0;
    DevBuf d_pyr, d_slots, d_cellcnt, d_P, d_T, d_sel, d_selcnt, d_fault;
    // single-frame host API buffers
    DevBuf d_img, d_kps, d_desc, d_counts;
    DevBuf d_stereo_sad;   // stereo scratch (orbx_stereo_matches_batch_device)
    // stage profiling (events on the launch stream)
    int prof = 0;   // bit k: time stage k's launches (orbx_profile_enable)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev[4];
    std::vector<hipEvent_t> ev_pool;
    // last batch (for GetImagePyramid)
    const uint8_t* last_in = nullptr;
    long long last_fstride = 0;
    size_t last_step = 0;
    int last_frames = 0;
    // dense describe grid (DescGrid): slots per frame from the previous batch's largest total
    int desc_dense = 0;         // ORBX_DESC_DENSE=1: the dense grid (measured no faster, DESIGN §4 describe round 6)
    int desc_force_c = 0;       // test hook (ORBX_DESC_C): this C for every batch (exercises the overflow kernel)
    int desc_c = 0;             // C of the next batch (0: unknown, out_frame)
    DevBuf d_dstat;             // stat[0] = the batch's largest frame total (describe_prefix_kernel)
    int32_t* h_dstat = nullptr; // pinned copy of it
    hipEvent_t dstat_ev = nullptr;
    bool dstat_pending = false;
    bool last_single = false;   // the last extraction was orbx_extract (outputs in d_kps / d_desc / d_counts)
    int last_kcap = 0;          // its output capacity (row stride of d_kps / d_desc)
    DevBuf d_stereo_out;        // orbx_stereo_matches_last: uright | depth on the device
    std::vector<uint8_t> h_stage;   // host staging of the pageable copies (one copy per level / call)
};

// First column that takes FixedPtCast<int, uchar, 22> rounding under tail mode V: after a V-byte
// vector loop ([ext] imgproc/src/resize.cpp VResizeLinearVec_32s8u: `for (; x <= w - V; x += V)` then
// `for (; x < w - V/2; x += V/2)`).  V = 0 (default): none -- the recalled uchar specialisation of
// VResizeLinear rounds its unrolled and scalar tails like the vector op, so every column takes the SIMD
// formula whatever the build's SIMD width.  V = 1: FixedPtCast everywhere.  Modes other than 0 model
// builds whose tail rounds differently; they are kept as sensitivity switches (parity unpinned).
static int resize_tail_x(int w, int V) {
    if (V <= 0) return w;
    if (V == 1) return 0;
    int x = 0;
    for (; x <= w - V; x += V) {}
    for (; x < w - V / 2; x += V / 2) {}
    return x;
}

static int cv_round_d(double v) { return (int)std::lrint(v); }
static int cv_round_f(float v) { return (int)std::lrintf(v); }

static void compute_tables(orbx_extractor* h) {
    const orbx_params& p = h->p;
    const int L = p.nlevels;
    h->scale.resize(L); h->inv_scale.resize(L); h->sigma2.resize(L); h->inv_sigma2.resize(L);
    h->quota.resize(L);
    float s = 1.f;
    for (int l = 0; l < L; l++) {   // ORBextractor::Init (:728-737)
        h->scale[l] = s;
        h->inv_scale[l] = 1.f / s;
        h->sigma2[l] = s * s;
        h->inv_sigma2[l] = 1.f / (s * s);
        s *= p.scaleFactor;
    }
    const double factor = 1 / p.scaleFactor;   // ComputeNumFeaturesPerScale (:472-487)
    double nf = p.nfeatures * (1 - factor) / (1 - std::pow(factor, L));
    int sum = 0;
    for (int l = 0; l < L - 1; l++) {
        h->quota[l] = cv_round_d(nf);
        sum += h->quota[l];
        nf *= factor;
    }
    h->quota[L - 1] = std::max(p.nfeatures - sum, 0);
}

// Level sizes, resize tables, FAST cell grid, buffer layout for a rows x cols input.
static int setup_geometry(orbx_extractor* h, int rows, int cols) {
    if (h->g_rows == rows && h->g_cols == cols) return ORB_OK;
    const int Lc = h->p.nlevels;
    Geom g;
    std::memset(&g, 0, sizeof(g));
    g.nlevels = Lc;
    for (int l = Lc; l < MAX_LEVELS; l++) g.lv[l].out_base = INT_MAX;   // describe's level count
    std::vector<int2> xtab, ytab;
    std::vector<PyrMfmaLane> mt;
    std::vector<int> mkb;
    std::vector<CellDev> cells;
    long long pyr_off = 0, slot = 0, cand = 0;
    int out = 0, NC = 64;
    int prev_w = cols, prev_h = rows;
    for (int l = 0; l < Lc; l++) {
        LevelDev& L = g.lv[l];
        if (l == 0) {
            L.w = cols; L.h = rows; L.stride = cols; L.off = -1; L.tail_x = cols; L.mt_off = -1;
        } else {
            L.h = cv_round_f(h->inv_scale[l] * rows);
            L.w = cv_round_f(h->inv_scale[l] * cols);
            if (L.w <= 0 || L.h <= 0) {
                set_error("pyramid level collapses to zero size");
                return ORB_EINVAL;
            }
            L.stride = (int)align_up(L.w, 16);
            L.off = pyr_off;
            pyr_off += (long long)align_up((size_t)L.stride * L.h, 256);
            // cv::resize tables (same arithmetic as the oracle / OpenCV)
            const int sw = prev_w, sh = prev_h, dw = L.w, dh = L.h;
            const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
            L.xtab_off = (int)xtab.size();
            L.ytab_off = (int)ytab.size();
            L.ssx = (double)sw / L.w;
            L.ssy = (double)sh / L.h;
            L.tail_x = resize_tail_x(L.w, h->resize_simd);
            int xmax = dw;
            std::vector<int> sxs(dw), a0s(dw), a1s(dw);
            for (int dx = 0; dx < dw; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = (int)std::floor(fx);
                fx -= sx;
                if (sx < 0) { fx = 0; sx = 0; }
                if (sx + 1 >= sw) {
                    xmax = std::min(xmax, dx);
                    if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
                }
                sxs[dx] = sx;
                a0s[dx] = std::min(std::max(cv_round_f((1.f - fx) * 2048), -32768), 32767);
                a1s[dx] = std::min(std::max(cv_round_f(fx * 2048), -32768), 32767);
            }
            for (int dx = 0; dx < dw; dx++) {
                int sx0 = sxs[dx], sx1 = std::min(sxs[dx] + 1, sw - 1), a0 = a0s[dx], a1 = a1s[dx];
                if (dx >= xmax) { sx1 = sx0; a0 = 2048; a1 = 0; }
                xtab.push_back(make_int2(sx0 | (sx1 << 16), (a0 & 0xffff) | (a1 << 16)));
            }
            L.mt_off = h->pyr_mfma ? pyr_mfma_tables(xtab.data() + L.xtab_off, dw, mt, mkb) : -1;
            for (int dy = 0; dy < dh; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = (int)std::floor(fy);
                fy -= sy;
                const int b0 = std::min(std::max(cv_round_f((1.f - fy) * 2048), -32768), 32767);
                const int b1 = std::min(std::max(cv_round_f(fy * 2048), -32768), 32767);
                auto clip = [&](int y) { return y < 0 ? 0 : (y >= sh ? sh - 1 : y); };
                ytab.push_back(make_int2(clip(sy) | (clip(sy + 1) << 16), (b0 & 0xffff) | (b1 << 16)));
            }
        }
        if (l > 0) {   // the pyramid kernel's LDS source tile must hold a 64x16 output tile's footprint
            const double sc = (double)prev_w / L.w, scy = (double)prev_h / L.h;
            if (sc * PYR_TW + 12 > PYR_SW || scy * PYR_TH + 6 > PYR_SH) {   // conservative rectangle + margins
                set_error("scaleFactor too large for the pyramid tile (max ~1.9)");
                return ORB_EINVAL;
            }
        }
        if (L.w >= 4096 || L.h >= 4096) {
            set_error("image dimensions must be < 4096");
            return ORB_EINVAL;
        }
        prev_w = L.w; prev_h = L.h;
        L.rx = 16; L.ry = 16; L.rw = L.w - 32; L.rh = L.h - 32;
        L.scale = h->scale[l];
        L.size = h->scale[l] * 31;
        L.quota = h->quota[l];
        L.cell_base = (int)cells.size();
        L.ncells = 0;
        L.cand_base = cand;
        L.cand_cap = 0;
        L.nroots = 0;
        L.out_base = out;
        L.out_cap = 0;
        if (L.rw > 0 && L.rh > 0) {
            const int gridw = L.rw / 30, gridh = L.rh / 30;
            if (gridw > 0 && gridh > 0) {
                const int cellw = (int)std::ceil(1. * L.rw / gridw), cellh = (int)std::ceil(1. * L.rh / gridh);
                const int maxx = L.rx + L.rw, maxy = L.ry + L.rh;
                for (int cy = 0, y0 = L.ry; cy < gridh && y0 + 6 < maxy; cy++, y0 += cellh)
                    for (int cx = 0, x0 = L.rx; cx < gridw && x0 + 6 < maxx; cx++, x0 += cellw) {
                        const int y1 = std::min(y0 + cellh + 6, maxy), x1 = std::min(x0 + cellw + 6, maxx);
                        const int zw = x1 - x0 - 6, zh = y1 - y0 - 6;
                        if (zw > MAX_ZONE || zh > MAX_ZONE) {
                            set_error("FAST cell larger than supported zone");
                            return ORB_EINVAL;
                        }
                        CellDev c;
                        c.level = l;
                        c.x0y0 = x0 | (y0 << 16);
                        c.zwzh = zw | (zh << 16);
                        c.slot = (int)slot;
                        const int cap = ((zw + 1) / 2) * ((zh + 1) / 2);
                        slot += cap;
                        L.cand_cap += cap;
                        cells.push_back(c);
                        L.ncells++;
                    }
                L.nroots = cv_round_d(1. * L.rw / L.rh);
                if (L.nroots <= 0 || L.nroots > MAX_ROOTS) {
                    set_error("unsupported aspect ratio (quadtree root count)");
                    return ORB_EINVAL;
                }
                L.hx = 1. * L.rw / L.nroots;
                L.out_cap = std::max(L.quota + 3, 4 * L.nroots) + 1;
                NC = std::max(NC, L.out_cap + 8);
            }
        }
        cand += L.cand_cap;
        out += L.out_cap;
    }
    g.ncells_total = (int)cells.size();
    g.pyr_frame_bytes = std::max<long long>(pyr_off, 256);
    g.slot_frame = std::max<long long>(slot, 1);
    g.cand_frame = std::max<long long>(cand, 1);
    g.out_frame = std::max(out, 1);
    if (g.out_frame >= 0x7fff) {   // describe's u16 level starts (a frame of > 32k selected keypoints)
        set_error("ORBextractor: more than 32766 selection slots per frame (nfeatures too large)");
        return ORB_EINVAL;
    }
    for (int d = 0; d < MAX_LEVELS / 2; d++) g.lv_start[d] = 0x7fff7fffu;
    for (int l = 1; l < Lc; l++)
        g.lv_start[l >> 1] = (g.lv_start[l >> 1] & ~(0xffffu << (16 * (l & 1)))) | ((unsigned)g.lv[l].out_base << (16 * (l & 1)));
    {   // round-up magic for n / out_frame (Granlund-Montgomery; d = 1: t = 0, shifts 0)
        const unsigned d = (unsigned)g.out_frame;
        int lg = 0;
        while ((1ull << lg) < d) lg++;
        g.of_m = (unsigned)((((1ull << lg) - d) << 32) / d + 1);
        g.of_s1 = lg > 0 ? 1 : 0;
        g.of_s2 = lg > 0 ? lg - 1 : 0;
    }
    NC = (int)align_up(std::max(NC, 256), 64);   // >= blockDim: the gather reuses the node scratch
    if (h->debug_nc > 0) NC = (int)align_up(std::max(h->debug_nc, 256), 64);
    // PTC: candidate points kept in LDS (P and T) when a level has at most this many (more: HBM).
    // Sized for workgroups per CU first: the largest multiple of 64 (<= 2048) that fits 4 of them
    // in the 160 KiB (123 VGPRs allow 4), else 3, else 2, each with at least 512 points.  At C2
    // (NC = 448) that is 960 points and 4 workgroups per CU instead of 2048 and 3: quadtree 1.44 ->
    // 1.14 ms per 2048 pan frames, 3.20 -> 2.82 ms per 1024 textured ones.
    const size_t node_lds = (size_t)NC * (2 * sizeof(QtNode) + sizeof(int4) + 2 * sizeof(QtItem) + 2 * sizeof(int));
    int PTC = 2048;
    {
        hipFuncAttributes fa{};
        const size_t stat = hipFuncGetAttributes(&fa, (const void*)quadtree_kernel<false>) == hipSuccess ? fa.sharedSizeBytes : 1024;
        for (int t = QT_WAVES_DEF; t >= 2; t--) {
            const long long room = (long long)(160 * 1024 / t) - (long long)stat - (long long)node_lds;
            const int p = (int)std::min<long long>(2048, room / 8) & ~63;
            if (p >= 512) { PTC = p; break; }
        }
    }
    if (const char* e = getenv("ORBX_QT_PTC")) PTC = std::max(256, std::min(4096, atoi(e)));   // tuning knob
    const size_t lds = node_lds + (size_t)PTC * 8;
    if (lds > 156 * 1024) {   // gfx950: 160 KiB LDS per workgroup
        set_error("nfeatures too large for the quadtree LDS budget (per-level quota <= ~2100)");
        return ORB_EINVAL;
    }
    int PTC0 = 0;
    size_t lds0 = 0;
    if (const char* e = getenv("ORBX_QT_PTC0")) {   // level 0 (the densest) in its own launch
        PTC0 = std::max(256, std::min(8192, atoi(e))) & ~63;
        lds0 = node_lds + (size_t)PTC0 * 8;
        if (lds0 > 156 * 1024) { PTC0 = 0; lds0 = 0; }
    }
    if (std::max(lds, lds0) > 48 * 1024)
        ORB_HIP_TRY(hipFuncSetAttribute((const void*)quadtree_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)std::max(lds, lds0)));
    // Wave-per-tree levels: the trailing levels whose cells the partitioned gather of one wavefront takes
    // (<= 4 x 64 cells, <= 4 roots); node capacity from their own quotas; LDS points so that
    // qt_wave_wg workgroups of four trees fit a CU (a level with more points keeps them in HBM).
    h->qtw_l0 = g.nlevels;
    if (h->qt_wave) {
        int l0w = g.nlevels;
        while (l0w > 0 && g.lv[l0w - 1].ncells <= 4 * 64 && g.lv[l0w - 1].nroots <= 4) l0w--;
        int ncw = 64;
        for (int l = l0w; l < g.nlevels; l++) ncw = std::max(ncw, g.lv[l].out_cap + 8);
        ncw = (int)align_up(ncw, 64);
        hipFuncAttributes fa{};
        const size_t stat = hipFuncGetAttributes(&fa, (const void*)quadtree_kernel<true>) == hipSuccess ? fa.sharedSizeBytes : 2048;
        const long long per_wave = ((long long)(160 * 1024 / std::max(1, h->qt_wave_wg)) - (long long)stat) / 4;
        const int ptcw = (int)std::min<long long>(2048, (per_wave - (long long)ncw * QT_NODE_BYTES) / 8) & ~63;
        if (l0w < g.nlevels && ptcw >= 64) {
            h->qtw_l0 = l0w;
            h->qtw_nc = ncw;
            h->qtw_ptc = ptcw;
            h->qtw_lds = 4 * ((size_t)ncw * QT_NODE_BYTES + (size_t)ptcw * 8);
            if (h->qtw_lds > 48 * 1024)
                ORB_HIP_TRY(hipFuncSetAttribute((const void*)quadtree_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                (int)h->qtw_lds));
        }
    }
    int rc;
    if ((rc = h->d_cells.reserve(std::max<size_t>(1, cells.size()) * sizeof(CellDev)))) return rc;
    if ((rc = h->d_xtab.reserve(std::max<size_t>(1, xtab.size()) * sizeof(int2)))) return rc;
    if ((rc = h->d_ytab.reserve(std::max<size_t>(1, ytab.size()) * sizeof(int2)))) return rc;
    if (!cells.empty())
        ORB_HIP_TRY(hipMemcpy(h->d_cells.ptr, cells.data(), cells.size() * sizeof(CellDev), hipMemcpyHostToDevice));
    if (!xtab.empty())
        ORB_HIP_TRY(hipMemcpy(h->d_xtab.ptr, xtab.data(), xtab.size() * sizeof(int2), hipMemcpyHostToDevice));
    if (!ytab.empty())
        ORB_HIP_TRY(hipMemcpy(h->d_ytab.ptr, ytab.data(), ytab.size() * sizeof(int2), hipMemcpyHostToDevice));
    {   // describe's slot table: slot s of level l's [out_base, out_base + out_cap) -> l | (s - out_base) << 8
        std::vector<uint32_t> st((size_t)g.out_frame, 0u);
        for (int l = 0; l < Lc; l++)
            for (int i = 0; i < g.lv[l].out_cap; i++) st[(size_t)g.lv[l].out_base + i] = (uint32_t)l | ((uint32_t)i << 8);
        if ((rc = h->d_slottab.reserve(st.size() * sizeof(uint32_t)))) return rc;
        ORB_HIP_TRY(hipMemcpy(h->d_slottab.ptr, st.data(), st.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    // (only with ORBX_PYR_MFMA=1: the default path allocates nothing for it)
    if (!mt.empty() && (rc = h->d_pyrmt.reserve(mt.size() * sizeof(PyrMfmaLane)))) return rc;
    if (!mkb.empty() && (rc = h->d_pyrkb.reserve(mkb.size() * sizeof(int)))) return rc;
    if (!mt.empty())
        ORB_HIP_TRY(hipMemcpy(h->d_pyrmt.ptr, mt.data(), mt.size() * sizeof(PyrMfmaLane), hipMemcpyHostToDevice));
    if (!mkb.empty())
        ORB_HIP_TRY(hipMemcpy(h->d_pyrkb.ptr, mkb.data(), mkb.size() * sizeof(int), hipMemcpyHostToDevice));
    h->pyr_mfma_ok.assign(Lc, 0);
    for (int l = 1; l + 1 < Lc; l++) h->pyr_mfma_ok[l] = h->pyr_mfma && pyr_mfma_pair_fits(g, l, mkb, ytab);
    h->geom = g;
    h->cells = cells;
    {   // FAST column strips: up to fast_cpw vertically consecutive cells of one column per wavefront
        // (the speculation hint comes from the cell above); consecutive strips are neighbouring
        // columns of the same row block, so the wavefronts running together read adjacent crops
        // and share their cache lines (rows of one level all have the same cell count).
        std::vector<int2> strips;
        h->strip_beg.assign(g.nlevels + 1, 0);
        const int cpw = std::max(1, std::min(h->fast_cpw, 255));
        for (int l = 0; l < g.nlevels; l++) {
            h->strip_beg[l] = (int)strips.size();
            const LevelDev& L = g.lv[l];
            if (L.ncells <= 0) continue;
            const int x00 = cells[L.cell_base].x0y0 & 0xffff;
            int ncx = 0;
            while (ncx < L.ncells && (cells[L.cell_base + ncx].x0y0 >> 16) == (cells[L.cell_base].x0y0 >> 16)) ncx++;
            const int ncy = L.ncells / ncx;
            if (ncx * ncy != L.ncells || (cells[L.cell_base + ncx - 1].x0y0 & 0xffff) < x00) {
                set_error("FAST cell grid is not a rectangle");
                return ORB_EINTERNAL;
            }
            for (int rb = 0; rb < ncy; rb += cpw)
                for (int cx = 0; cx < ncx; cx++) {
                    const int c0 = L.cell_base + rb * ncx + cx, n = std::min(cpw, ncy - rb);
                    for (int k = 1; k < n; k++)   // the kernel takes the zone width from the first cell
                        if ((cells[c0 + k * ncx].zwzh & 0xffff) != (cells[c0].zwzh & 0xffff)) {
                            set_error("FAST strip with unequal zone widths");
                            return ORB_EINTERNAL;
                        }
                    strips.push_back(make_int2(c0, n | (ncx << 8)));
                }
        }
        h->strip_beg[g.nlevels] = (int)strips.size();
        if ((rc = h->d_strips.reserve(std::max<size_t>(1, strips.size()) * sizeof(int2)))) return rc;
        if (!strips.empty())
            ORB_HIP_TRY(hipMemcpy(h->d_strips.ptr, strips.data(), strips.size() * sizeof(int2), hipMemcpyHostToDevice));
    }
    {
        int mzw = 1, mzh = 1;
        for (const CellDev& c : cells) { mzw = std::max(mzw, c.zwzh & 0xffff); mzh = std::max(mzh, c.zwzh >> 16); }
        if (mzw > 64 || mzh > (2 * GR_RING + FQ2_RING) / 8) {   // DetectFAST cells are < 60 px (:508-511)
            set_error("FAST cell larger than the kernel supports");
            return ORB_EINTERNAL;
        }
        // PAIR: every strip's consecutive cells adjacent (zone B starts where zone A ends, same x0), the
        // merged zone's rows within the 7 bits of the pair encoding, and a dense pair's 3 ballot words
        // per pass within the drained ring
        h->fast_pair_on = false;
        if (h->fast_pair) {
            bool ok = 2 * mzh < 128 && 24 * ((2 * mzh + 1) / (mzw <= 32 ? 2 : 1) + 1) <= 2 * (2 * GR_RING + FQ2_RING);
            for (int l = 0; l < g.nlevels && ok; l++) {
                const LevelDev& L = g.lv[l];
                if (L.ncells <= 0) continue;
                int ncx = 0;   // cells per grid row (the strips' cell stride)
                while (ncx < L.ncells && (cells[L.cell_base + ncx].x0y0 >> 16) == (cells[L.cell_base].x0y0 >> 16)) ncx++;
                for (int c = L.cell_base; c + ncx < L.cell_base + L.ncells && ok; c++) {
                    const CellDev &A = cells[c], &B = cells[c + ncx];
                    ok = (A.x0y0 & 0xffff) == (B.x0y0 & 0xffff) && (B.x0y0 >> 16) == (A.x0y0 >> 16) + (A.zwzh >> 16);
                }
            }
            h->fast_pair_on = ok;
        }
        const int zrows = h->fast_pair_on ? 2 * mzh + 1 : mzh;   // zone rows per pass (+ the separator)
        FastLds fl;
        fl.CS = (int)align_up(mzw + 6 + 8, 4);         // +1 shift, +4 dword over-read each side
        if (fl.CS < 4 * ((mzw + 6 + 1 + 3) / 4)) fl.CS = 4 * ((mzw + 6 + 1 + 3) / 4);
        fl.ZS = (int)align_up(mzw + 2, 4);             // zone map with a zero border of 1
        // rows: the tallest crop + slack, and at least the CROP_NG row groups of 4 rows the staging's first
        // batch always stores
        fl.crop_bytes = (int)align_up((size_t)fl.CS * std::max(zrows + 6 + FAST_CROP_SLACK, 4 * CROP_NG), 16);
        fl.mz_bytes = (int)align_up((size_t)fl.ZS * (zrows + 2), 16);
        fl.qcap = 2 * GR_RING + FQ2_RING;   // in u16 entries
        fl.ccap = std::min(FAST_CLIST_CAP, (int)align_up((size_t)mzw * mzh, 8));
        const int nbal = (fl.ccap + 63) / 64;
        h->fast_lds = (size_t)fl.crop_bytes + fl.mz_bytes + 2 * (size_t)(fl.qcap + fl.ccap) +
                      (h->fast_pair_on ? 24 : 16) * (size_t)nbal;
        h->fl = fl;
    }
    h->NC = NC;
    h->PTC = PTC;
    h->qt_lds = lds;
    h->qt_ptc0 = PTC0;
    h->qt_lds0 = lds0;
    h->g_rows = rows;
    h->g_cols = cols;
    h->ws_frames = 0;   // force workspace re-layout
    return ORB_OK;
}

static int reserve_workspace(orbx_extractor* h, int frames) {
    if (frames <= h->ws_frames) return ORB_OK;
    const Geom& g = h->geom;
    int rc;
    if ((rc = h->d_pyr.reserve((size_t)frames * g.pyr_frame_bytes))) return rc;
    if ((rc = h->d_slots.reserve((size_t)frames * g.slot_frame * 4))) return rc;
    if ((rc = h->d_cellcnt.reserve((size_t)frames * std::max(1, g.ncells_total) * 4))) return rc;
    if ((rc = h->d_P.reserve((size_t)frames * g.cand_frame * 4))) return rc;
    if ((rc = h->d_T.reserve((size_t)frames * g.cand_frame * 4))) return rc;
    if ((rc = h->d_sel.reserve((size_t)frames * g.out_frame * 4))) return rc;
    // + 64 B: describe reads 16 counts from a frame's first (scalar loads, past the last frame too)
    if ((rc = h->d_selcnt.reserve((size_t)frames * g.nlevels * 4 + 64))) return rc;
    if ((rc = h->d_lvlpre.reserve((size_t)frames * LVP * 4))) return rc;
    if (!h->d_fault.ptr) {   // sticky until read (orbx_batch_status / the host Extract)
        if ((rc = h->d_fault.reserve(16))) return rc;
        ORB_HIP_TRY(hipMemset(h->d_fault.ptr, 0, 16));
    }
    h->ws_frames = frames;
    return ORB_OK;
}

static hipEvent_t prof_event(orbx_extractor* h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

constexpr int ORBX_MIN_SUB_FRAMES = 16;

// Per-launch timing when profiling: hipExtLaunchKernel records the two events as part of the
// kernel's own dispatch (start / completion of that kernel, no marker packets in the stream), so a
// stage's time is the sum of its kernels' durations, as rocprofv3 reports them.
template <typename... KArgs, typename... Args>
static void launch_timed(orbx_extractor* h, int stage, void (*kernel)(KArgs...), dim3 grid, dim3 block,
                         uint32_t shmem, hipStream_t s, Args... args) {
    if (h->prof & (1 << stage)) {
        hipEvent_t a = prof_event(h), b = prof_event(h);
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, a, b, 0, static_cast<KArgs>(args)...);
        h->prof_ev[stage].push_back({a, b});
    } else {
        hipLaunchKernelGGL(kernel, grid, block, shmem, s, static_cast<KArgs>(args)...);
    }
}

// All four stages for frames [f0, f0 + F) of the workspace, enqueued on st.  Every kernel indexes
// its per-frame buffers from the frame index within the launch, so a chunk is launched with base
// pointers advanced by f0 frames.
static void launch_chunk(orbx_extractor* h, int f0, const uint8_t* d_imgs, int F, long long fstride, int step,
                         orbx_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap, hipStream_t st,
                         hipStream_t side = nullptr) {
    const Geom& g = h->geom;
    uint8_t* pyr = h->d_pyr.as<uint8_t>() + (long long)f0 * g.pyr_frame_bytes;
    d_imgs += (long long)f0 * fstride;
    d_kps += (long long)f0 * cap;
    d_desc += (long long)f0 * cap * 32;
    d_counts += f0;
    uint32_t* slots = h->d_slots.as<uint32_t>() + (long long)f0 * g.slot_frame;
    int* cellcnt = h->d_cellcnt.as<int>() + (long long)f0 * g.ncells_total;
    uint32_t* Pb = h->d_P.as<uint32_t>() + (long long)f0 * g.cand_frame;
    uint32_t* Tb = h->d_T.as<uint32_t>() + (long long)f0 * g.cand_frame;
    uint32_t* sel = h->d_sel.as<uint32_t>() + (long long)f0 * g.out_frame;
    int* selcnt = h->d_selcnt.as<int>() + (long long)f0 * g.nlevels;
    uint32_t* fault = h->d_fault.as<uint32_t>();
    auto fast = [&](int l0, int l1, hipStream_t s) {   // levels [l0, l1)
        const int sb = h->strip_beg[l0], ns = h->strip_beg[l1] - sb;
        if (ns <= 0) return;
        const FastLds& fl = h->fl;
        auto kern = h->fast_pair_on ? (fl.CS == 48 && fl.ZS == 36   ? fast_cells_kernel<48, 36, true>
                                       : fl.CS == 52 && fl.ZS == 40 ? fast_cells_kernel<52, 40, true>
                                                                    : fast_cells_kernel<0, 0, true>)
                                    : (fl.CS == 48 && fl.ZS == 36   ? fast_cells_kernel<48, 36, false>
                                       : fl.CS == 52 && fl.ZS == 40 ? fast_cells_kernel<52, 40, false>
                                                                    : fast_cells_kernel<0, 0, false>);
        launch_timed(h, 1, kern, dim3((unsigned)(ns * F)), dim3(64), (uint32_t)h->fast_lds, s,
                           g, h->d_cells.as<CellDev>(), h->d_strips.as<int2>(), d_imgs, fstride, step, pyr, h->p.iniThFAST,
                           h->p.minThFAST, slots, cellcnt, fault, h->fl, sb, ns,
                           h->fast_spec > 0 && h->fast_spec_first ? h->fast_spec | (1 << 29) : h->fast_spec);
    };
    const unsigned qt_block = h->debug_qt_block ? (unsigned)h->debug_qt_block : (unsigned)QT_THREADS;
    auto quadtree = [&](int l0, int nl, hipStream_t s) {
        if (nl <= 0) return;
        // levels from qtw_l0 on: one tree per wavefront, four per workgroup (quadtree_kernel<true>)
        const int lw = std::max(l0, h->qtw_l0), nw_lv = l0 + nl - lw;
        if (nw_lv > 0) {
            launch_timed(h, 2, quadtree_kernel<true>, dim3((unsigned)F, (unsigned)((nw_lv + 3) / 4)), dim3(qt_block),
                         (uint32_t)h->qtw_lds, s, g, cellcnt, slots, h->d_cells.as<CellDev>(), Pb, Tb, sel, selcnt, h->qtw_nc,
                         h->qtw_ptc, fault, lw, nw_lv);
            nl -= nw_lv;
            if (nl <= 0) return;
        }
        if (h->qt_ptc0 > 0 && l0 == 0) {   // tuning knob: level 0 alone, with its own LDS point capacity
            launch_timed(h, 2, quadtree_kernel<false>, dim3((unsigned)F, 1u), dim3(qt_block), (uint32_t)h->qt_lds0, s, g,
                         cellcnt, slots, h->d_cells.as<CellDev>(), Pb, Tb, sel, selcnt, h->NC, h->qt_ptc0, fault, 0, 1);
            l0 = 1;
            if (--nl <= 0) return;
        }
        launch_timed(h, 2, quadtree_kernel<false>, dim3((unsigned)F, (unsigned)nl), dim3(qt_block), (uint32_t)h->qt_lds, s,
                     g, cellcnt, slots, h->d_cells.as<CellDev>(), Pb, Tb, sel, selcnt, h->NC, h->PTC, fault, l0, nl);
    };
    // levels l and l+1 in one pyramid_pair_kernel launch where the shapes fit its LDS rectangles
    // (returns the number of extra levels built)
    auto pyramid = [&](int l) -> int {
        const int first = h->pyr_pair == 2 ? 1 : 2;   // pairs (1,2), (3,4), (5,6) or (2,3), (4,5), (6,7)
        const bool a16 = l > 1 || (((uintptr_t)d_imgs | (uintptr_t)fstride | (uintptr_t)step) & 15) == 0;
        if (h->pyr_pair && l >= first && (l - first) % 2 == 0 && l + 1 < g.nlevels && a16 && h->pyr_mfma &&
            h->pyr_mfma_ok[l]) {
            const int ntx = (g.lv[l + 1].w + PYR_TW - 1) / PYR_TW, nty = (g.lv[l + 1].h + PYR_TH - 1) / PYR_TH;
            launch_timed(h, 0, pyramid_pair_mfma_kernel, dim3((unsigned)ntx, (unsigned)nty, (unsigned)F), dim3(256), 0u,
                         st, g, l, d_imgs, fstride, step, pyr, h->d_ytab.as<int2>(), h->d_pyrmt.as<PyrMfmaLane>(),
                         h->d_pyrkb.as<int>());
            return 1;
        }
        if (h->pyr_pair && l >= first && (l - first) % 2 == 0 && l + 1 < g.nlevels && a16 && pyr_pair_fits(g, l)) {
            const int ntx = (g.lv[l + 1].w + PYR_TW - 1) / PYR_TW, nty = (g.lv[l + 1].h + PYR_TH - 1) / PYR_TH;
            launch_timed(h, 0, pyramid_pair_kernel, dim3((unsigned)ntx, (unsigned)nty, (unsigned)F), dim3(256), 0u, st,
                         g, l, d_imgs, fstride, step, pyr, h->d_xtab.as<int2>(), h->d_ytab.as<int2>());
            return 1;
        }
        const int ntx = (g.lv[l].w + PYR_TW - 1) / PYR_TW, nty = (g.lv[l].h + PYR_TH - 1) / PYR_TH;
        launch_timed(h, 0, pyramid_level_kernel, dim3((unsigned)ntx, (unsigned)nty, (unsigned)F), dim3(256), 0u, st, g, l,
                     d_imgs, fstride, step, pyr, h->d_xtab.as<int2>(), h->d_ytab.as<int2>());
        return 0;
    };
    const int nc0 = g.lv[0].ncells;
    if (side && nc0 > 0 && g.nlevels > 1) {
        // Level 0 needs no pyramid: its FAST + quadtree run on the side stream while the main
        // stream builds levels 1..7 (latency-bound cascade) and runs their FAST / quadtree, so the
        // level-0 tree's serial rounds overlap the FAST work of the other levels.
        (void)hipStreamWaitEvent(side, h->lvl_fork, 0);
        fast(0, 1, side);
        quadtree(0, 1, side);
        (void)hipEventRecord(h->lvl_join, side);
        {
            for (int l = 1; l < g.nlevels; l++) l += pyramid(l);
        }
        fast(1, g.nlevels, st);
        quadtree(1, g.nlevels - 1, st);
        (void)hipStreamWaitEvent(st, h->lvl_join, 0);
    } else {
        {
            for (int l = 1; l < g.nlevels; l++) l += pyramid(l);
        }
        fast(0, g.nlevels, st);
        quadtree(0, g.nlevels, st);
    }
    int* lvlpre = h->d_lvlpre.as<int>() + (long long)f0 * LVP;
    if (DESC_SLOT_TAB)
        hipLaunchKernelGGL(describe_prefix_kernel, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, st, (const int*)selcnt,
                           g.nlevels, F, lvlpre, d_counts, h->d_dstat.as<int>());
    // the dense grid: C slots per frame (from the previous batch's largest total), the overflow kernel for
    // rows >= C of any frame with more (DescGrid); or the slot-table grid (out_frame slots)
    const int rows_max = std::min(g.out_frame, cap);
    const int C = (DESC_SLOT_TAB && h->desc_dense) ? std::max(1, std::min(h->desc_c > 0 ? h->desc_c : rows_max, rows_max)) : 0;
    DescGrid dg{};
    if (C > 0) {
        dg.C = C;
        const unsigned d = (unsigned)C;
        int lg = 0;
        while ((1ull << lg) < d) lg++;
        dg.m = (unsigned)((((1ull << lg) - d) << 32) / d + 1);
        dg.s1 = lg > 0 ? 1 : 0;
        dg.s2 = lg > 0 ? lg - 1 : 0;
    }
    launch_timed(h, 3, h->trig_float ? describe_kernel<1> : describe_kernel<0>,
                 dim3((unsigned)(C > 0 ? C : g.out_frame), (unsigned)F), dim3(64), 0u, st, g, d_imgs, fstride, step, pyr,
                 sel, selcnt, d_kps, d_desc, d_counts, cap, h->d_slottab.as<uint32_t>(), lvlpre, dg);
    if (C > 0 && C < rows_max)
        launch_timed(h, 3, h->trig_float ? describe_overflow_kernel<1> : describe_overflow_kernel<0>,
                     dim3((unsigned)std::min(F, 2048)), dim3(64), 0u, st, g, d_imgs, fstride, step, pyr, sel, d_kps, d_desc,
                     cap, (const int*)lvlpre, F, C);
}

// The first-cell hint bits for the next launch (fast_hint_kernel): once per batch, on st after every
// sub-batch and side stream has joined, so no fast_cells launch of this batch is still reading the strip
// descriptors it rewrites, and frame 0's cell counts (the first chunk's) are final.
static int launch_fast_hint(orbx_extractor* h, hipStream_t st) {
    if (!(h->fast_spec > 0 && h->fast_spec_first)) return ORB_OK;
    const int ns = h->strip_beg[h->geom.nlevels];
    if (ns <= 0) return ORB_OK;
    hipLaunchKernelGGL(fast_hint_kernel, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, st, h->d_strips.as<int2>(),
                       h->d_cellcnt.as<int>(), ns);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

// Frames are split into sub-batches on the handle's side streams (fork/join with events on st) so
// that one sub-batch's latency-bound stages (the short pyramid levels, the quadtree's level-0 tail)
// overlap another's FAST / describe work.
// The dense describe grid's C for this batch: the previous batch's largest frame total (read back
// asynchronously; a copy not yet landed keeps the last C) plus a margin, rounded up to 64.
static int describe_grid_begin(orbx_extractor* h, hipStream_t st) {
    if (!h->dstat_ev) {
        ORB_HIP_TRY(hipEventCreateWithFlags(&h->dstat_ev, hipEventDisableTiming));
        ORB_HIP_TRY(hipHostMalloc((void**)&h->h_dstat, 64, hipHostMallocDefault));
        int rc;
        if ((rc = h->d_dstat.reserve(64))) return rc;
    }
    if (h->dstat_pending && hipEventQuery(h->dstat_ev) == hipSuccess) {
        const int mx = *h->h_dstat;
        h->desc_c = (int)align_up((size_t)std::max(mx + 32, 64), 64);
        h->dstat_pending = false;
    }
    if (h->desc_force_c > 0) h->desc_c = h->desc_force_c;
    ORB_HIP_TRY(hipMemsetAsync(h->d_dstat.ptr, 0, 4, st));
    return ORB_OK;
}
static int describe_grid_end(orbx_extractor* h, hipStream_t st) {
    if (h->dstat_pending) return ORB_OK;   // the previous read-back has not landed: keep its slot
    ORB_HIP_TRY(hipMemcpyAsync(h->h_dstat, h->d_dstat.ptr, 4, hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipEventRecord(h->dstat_ev, st));
    h->dstat_pending = true;
    return ORB_OK;
}

static int launch_batch(orbx_extractor* h, const uint8_t* d_imgs, int F, long long fstride, int step,
                        orbx_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap, hipStream_t st) {
    {
        const int rc = describe_grid_begin(h, st);
        if (rc) return rc;
    }
    int nsub = std::min(h->nsub, F / ORBX_MIN_SUB_FRAMES);
    if (nsub <= 1) {
        hipStream_t side = nullptr;
        if (h->lvl_overlap) {
            if (!h->lvl_side) {
                ORB_HIP_TRY(hipStreamCreateWithFlags(&h->lvl_side, hipStreamNonBlocking));
                ORB_HIP_TRY(hipEventCreateWithFlags(&h->lvl_fork, hipEventDisableTiming));
                ORB_HIP_TRY(hipEventCreateWithFlags(&h->lvl_join, hipEventDisableTiming));
            }
            ORB_HIP_TRY(hipEventRecord(h->lvl_fork, st));
            side = h->lvl_side;
        }
        launch_chunk(h, 0, d_imgs, F, fstride, step, d_kps, d_desc, d_counts, cap, st, side);
        ORB_HIP_TRY(hipGetLastError());
        const int rc = describe_grid_end(h, st);
        return rc ? rc : launch_fast_hint(h, st);
    }
    while ((int)h->sub.size() < nsub) {
        hipStream_t s2;
        ORB_HIP_TRY(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        hipEvent_t e;
        ORB_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        h->sub.push_back({s2, e});
    }
    if (!h->fork_ev) ORB_HIP_TRY(hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming));
    ORB_HIP_TRY(hipEventRecord(h->fork_ev, st));
    int f0 = 0;
    for (int i = 0; i < nsub; i++) {
        const int Fi = F / nsub + (i < F % nsub ? 1 : 0);
        ORB_HIP_TRY(hipStreamWaitEvent(h->sub[i].first, h->fork_ev, 0));
        launch_chunk(h, f0, d_imgs, Fi, fstride, step, d_kps, d_desc, d_counts, cap, h->sub[i].first);
        ORB_HIP_TRY(hipEventRecord(h->sub[i].second, h->sub[i].first));
        ORB_HIP_TRY(hipStreamWaitEvent(st, h->sub[i].second, 0));
        f0 += Fi;
    }
    ORB_HIP_TRY(hipGetLastError());
    const int rc = describe_grid_end(h, st);
    return rc ? rc : launch_fast_hint(h, st);
}

static int check_fault(orbx_extractor* h) {
    uint32_t f = 0;
    ORB_HIP_TRY(hipMemcpy(&f, h->d_fault.ptr, 4, hipMemcpyDeviceToHost));
    if (f) {
        ORB_HIP_TRY(hipMemset(h->d_fault.ptr, 0, 4));
        set_error("device capacity check failed (fault mask " + std::to_string(f) + ")");
        return ORB_EINTERNAL;
    }
    return ORB_OK;
}

namespace orbamd {
// One workgroup per frame: rows [0, counts[f]) of the frame's slots -> out rows from incl[f] - counts[f],
// each 32-byte row as two uint4 (lanes take consecutive 16-byte halves: coalesced both ways).
__global__ __launch_bounds__(256) void pack_rows_kernel(const uint4* __restrict__ desc, int cap,
                                                        const int* __restrict__ counts, const int* __restrict__ incl,
                                                        uint4* __restrict__ out, int out_rows) {
    const int f = blockIdx.x;
    const int c = counts[f];
    const int n = min(max(c, 0), cap);                // never read past the frame's slots
    const long long start = (long long)incl[f] - c;   // the caller's layout
    const long long r0 = max(start, 0ll), r1 = min(start + n, (long long)out_rows);   // never write past out
    const uint4* src = desc + (long long)f * cap * 2;
    for (long long i = 2 * r0 + threadIdx.x; i < 2 * r1; i += blockDim.x) out[i] = src[i - 2 * start];
}

}  // namespace orbamd

extern "C" {

int orbx_create(const orbx_params* params, int device, orbx_extractor** out) {
    ORB_CHECK_ARG(params && out, "null argument");
    ORB_CHECK_ARG(params->nlevels >= 1 && params->nlevels <= MAX_LEVELS, "nlevels must be in [1,16]");
    ORB_CHECK_ARG(params->nfeatures >= 0 && params->scaleFactor > 1.0f, "bad nfeatures / scaleFactor");
    int ndev = 0;
    ORB_HIP_TRY(hipGetDeviceCount(&ndev));
    ORB_CHECK_ARG(device >= 0 && device < ndev, "no such HIP device");
    ORB_HIP_TRY(hipSetDevice(device));
    orbx_extractor* h = new orbx_extractor();
    h->p = *params;
    h->device = device;
    if (const char* e = getenv("ORBX_FAST_CPW")) h->fast_cpw = std::max(1, std::min(64, atoi(e)));   // tuning knobs
    if (const char* e = getenv("ORBX_FAST_SPEC")) h->fast_spec = std::max(-1, atoi(e));   // -1: every cell
    if (const char* e = getenv("ORBX_FAST_PAIR")) h->fast_pair = atoi(e) != 0;
    if (const char* e = getenv("ORBX_QT_WAVE")) h->qt_wave = atoi(e) != 0;
    if (const char* e = getenv("ORBX_QT_WAVE_WG")) h->qt_wave_wg = std::max(1, std::min(4, atoi(e)));
    if (const char* e = getenv("ORBX_FAST_SPEC_FIRST")) h->fast_spec_first = atoi(e) != 0;

    if (const char* e = getenv("ORBX_NSUB")) h->nsub = std::max(1, std::min(8, atoi(e)));
    if (const char* e = getenv("ORBX_PYR_PAIR")) h->pyr_pair = std::max(0, std::min(2, atoi(e)));
    if (const char* e = getenv("ORBX_PYR_MFMA")) h->pyr_mfma = atoi(e) != 0;
    if (const char* e = getenv("ORBX_LEVEL_OVERLAP")) h->lvl_overlap = atoi(e) != 0;
    if (const char* e = getenv("ORBX_DEBUG_NC")) h->debug_nc = atoi(e);
    if (const char* e = getenv("ORBX_DESC_DENSE")) h->desc_dense = atoi(e) != 0;
    if (const char* e = getenv("ORBX_DESC_C")) h->desc_force_c = std::max(0, atoi(e));
    if (const char* e = getenv("ORBX_DEBUG_QT_BLOCK")) {
        const int b = atoi(e);
        if (b >= 64 && b <= QT_THREADS && b % 64 == 0) h->debug_qt_block = b;
    }
    // OpenCV-build switches (orbx_set_opencv_compat): ORBX_TRIG=double|float, ORBX_RESIZE_TAIL=V
    if (const char* e = getenv("ORBX_TRIG")) h->trig_float = (e[0] == 'f' || e[0] == '1') ? 1 : 0;
    if (const char* e = getenv("ORBX_RESIZE_TAIL")) {
        const int v = atoi(e);
        if (v == 0 || v == 1 || v == 8 || v == 16 || v == 32 || v == 64) h->resize_simd = v;
    }
    compute_tables(h);
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        set_error(std::string("hipStreamCreate: ") + hipGetErrorString(e));
        return ORB_EHIP;
    }
    *out = h;
    return ORB_OK;
}

int orbx_destroy(orbx_extractor* h) {
    if (!h) return ORB_OK;
    (void)hipSetDevice(h->device);
    DevBuf* bufs[] = {&h->d_cells, &h->d_strips, &h->d_xtab, &h->d_ytab, &h->d_pyr, &h->d_slots, &h->d_cellcnt, &h->d_P,
                      &h->d_T, &h->d_sel, &h->d_selcnt, &h->d_fault, &h->d_img, &h->d_kps, &h->d_desc,
                      &h->d_counts, &h->d_stereo_sad, &h->d_pyrmt, &h->d_pyrkb, &h->d_slottab, &h->d_lvlpre,
                      &h->d_stereo_out, &h->d_dstat};
    for (DevBuf* b : bufs) b->release();
    for (auto& v : h->prof_ev)
        for (auto& pr : v) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    for (auto& se : h->sub) { (void)hipStreamDestroy(se.first); (void)hipEventDestroy(se.second); }
    if (h->fork_ev) (void)hipEventDestroy(h->fork_ev);
    if (h->lvl_side) (void)hipStreamDestroy(h->lvl_side);
    if (h->lvl_fork) (void)hipEventDestroy(h->lvl_fork);
    if (h->lvl_join) (void)hipEventDestroy(h->lvl_join);
    if (h->dstat_ev) (void)hipEventDestroy(h->dstat_ev);
    if (h->h_dstat) (void)hipHostFree(h->h_dstat);
    delete h;
    return ORB_OK;
}

int orbx_set_opencv_compat(orbx_extractor* h, int trig_mode, int resize_simd) {
    ORB_CHECK_ARG(h, "null extractor");
    ORB_CHECK_ARG(trig_mode >= -1 && trig_mode <= 1, "trig_mode must be -1 (keep), 0 (double) or 1 (float)");
    ORB_CHECK_ARG(resize_simd == -1 || resize_simd == 0 || resize_simd == 1 || resize_simd == 8 || resize_simd == 16 ||
                      resize_simd == 32 || resize_simd == 64,
                  "resize_simd must be -1 (keep), 0, 1, 8, 16, 32 or 64");
    std::lock_guard<std::mutex> lk(h->mu);
    if (trig_mode >= 0) h->trig_float = trig_mode;
    if (resize_simd >= 0 && resize_simd != h->resize_simd) {
        h->resize_simd = resize_simd;
        h->g_rows = h->g_cols = -1;   // the levels' tail columns change: rebuild the geometry
    }
    return ORB_OK;
}

int orbx_get_opencv_compat(const orbx_extractor* h, int* trig_mode, int* resize_simd) {
    ORB_CHECK_ARG(h, "null extractor");
    if (trig_mode) *trig_mode = h->trig_float;
    if (resize_simd) *resize_simd = h->resize_simd;
    return ORB_OK;
}

int orbx_scale_tables(const orbx_extractor* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                      int32_t* features_per_level) {
    ORB_CHECK_ARG(h, "null extractor");
    for (int l = 0; l < h->p.nlevels; l++) {
        if (scale) scale[l] = h->scale[l];
        if (inv_scale) inv_scale[l] = h->inv_scale[l];
        if (sigma2) sigma2[l] = h->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = h->inv_sigma2[l];
        if (features_per_level) features_per_level[l] = h->quota[l];
    }
    return ORB_OK;
}

int orbx_max_keypoints(const orbx_extractor* hc, int rows, int cols, int32_t* cap) {
    ORB_CHECK_ARG(hc && cap && rows > 0 && cols > 0, "bad argument");
    orbx_extractor* h = const_cast<orbx_extractor*>(hc);
    std::lock_guard<std::mutex> lk(h->mu);
    ORB_HIP_TRY(hipSetDevice(h->device));
    int rc = setup_geometry(h, rows, cols);
    if (rc) return rc;
    int c = 0;
    for (int l = 0; l < h->geom.nlevels; l++) c += h->geom.lv[l].out_cap;
    *cap = c;
    return ORB_OK;
}

int orbx_extract_batch_device(orbx_extractor* h, const uint8_t* d_imgs, int n_frames, int rows, int cols,
                              size_t frame_stride, size_t step, orbx_keypoint* d_kps, uint8_t* d_desc,
                              int32_t* d_counts, int cap, void* stream) {
    ORB_CHECK_ARG(h && d_imgs && d_kps && d_desc && d_counts, "null argument");
    ORB_CHECK_ARG(n_frames > 0 && n_frames <= 65535 && rows > 0 && cols > 0, "bad batch shape");
    ORB_CHECK_ARG(step >= (size_t)cols && step < (1u << 31), "bad row step");
    std::lock_guard<std::mutex> lk(h->mu);
    ORB_HIP_TRY(hipSetDevice(h->device));
    int rc = setup_geometry(h, rows, cols);
    if (rc) return rc;
    int need = 0;
    for (int l = 0; l < h->geom.nlevels; l++) need += h->geom.lv[l].out_cap;
    if (cap < need) {
        set_error("cap < orbx_max_keypoints()");
        return ORB_ECAP;
    }
    if ((rc = reserve_workspace(h, n_frames))) return rc;
    hipStream_t st = (hipStream_t)stream;   // NULL = the default stream, like every HIP API
    h->last_in = d_imgs;
    h->last_single = false;
    h->last_fstride = (long long)frame_stride;
    h->last_step = step;
    h->last_frames = n_frames;
    return launch_batch(h, d_imgs, n_frames, (long long)frame_stride, (int)step, d_kps, d_desc, d_counts, cap, st);
}

int orbx_extract(orbx_extractor* h, const uint8_t* img, int rows, int cols, size_t step, orbx_keypoint* kps,
                 uint8_t* desc, int cap, int* n) {
    ORB_CHECK_ARG(h && img && n, "null argument");
    ORB_CHECK_ARG(rows > 0 && cols > 0 && step >= (size_t)cols, "image must be a non-empty CV_8U matrix");
    std::lock_guard<std::mutex> lk(h->mu);
    ORB_HIP_TRY(hipSetDevice(h->device));
    int rc = setup_geometry(h, rows, cols);
    if (rc) return rc;
    int kcap = 0;
    for (int l = 0; l < h->geom.nlevels; l++) kcap += h->geom.lv[l].out_cap;
    if ((rc = reserve_workspace(h, 1))) return rc;
    if ((rc = h->d_img.reserve((size_t)rows * cols))) return rc;
    if ((rc = h->d_kps.reserve((size_t)kcap * sizeof(orbx_keypoint)))) return rc;
    if ((rc = h->d_desc.reserve((size_t)kcap * 32))) return rc;
    if ((rc = h->d_counts.reserve(16))) return rc;
    hipStream_t st = h->stream;
    // a contiguous image (the usual cv::Mat) goes up in one 1D copy: a pitched copy from pageable memory
    // may be staged row by row
    if (step == (size_t)cols)
        ORB_HIP_TRY(hipMemcpyAsync(h->d_img.ptr, img, (size_t)rows * cols, hipMemcpyHostToDevice, st));
    else
        ORB_HIP_TRY(hipMemcpy2DAsync(h->d_img.ptr, cols, img, step, cols, rows, hipMemcpyHostToDevice, st));
    h->last_in = h->d_img.as<uint8_t>();
    h->last_fstride = (long long)rows * cols;
    h->last_step = cols;
    h->last_frames = 1;
    h->last_single = true;
    h->last_kcap = kcap;
    rc = launch_batch(h, h->d_img.as<uint8_t>(), 1, (long long)rows * cols, cols, h->d_kps.as<orbx_keypoint>(),
                      h->d_desc.as<uint8_t>(), h->d_counts.as<int32_t>(), kcap, st);
    if (rc) return rc;
    int32_t total = 0;
    ORB_HIP_TRY(hipMemcpyAsync(&total, h->d_counts.ptr, 4, hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipStreamSynchronize(st));
    if ((rc = check_fault(h))) return rc;
    *n = total;
    if (total == 0) return ORB_OK;   // reference: keypoints left untouched (:778-782)
    if (total > cap) {
        set_error("output capacity too small");
        return ORB_ECAP;
    }
    ORB_CHECK_ARG(kps && desc, "null output");
    ORB_HIP_TRY(hipMemcpyAsync(kps, h->d_kps.ptr, (size_t)total * sizeof(orbx_keypoint), hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipMemcpyAsync(desc, h->d_desc.ptr, (size_t)total * 32, hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipStreamSynchronize(st));
    return ORB_OK;
}

int orbx_batch_status(orbx_extractor* h, void* stream, uint32_t* fault_mask) {
    ORB_CHECK_ARG(h && fault_mask, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    ORB_HIP_TRY(hipSetDevice(h->device));
    *fault_mask = 0;
    if (!h->d_fault.ptr) return ORB_OK;   // nothing has run
    hipStream_t st = (hipStream_t)stream;
    ORB_HIP_TRY(hipMemcpyAsync(&h->fault_host, h->d_fault.ptr, 4, hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipMemsetAsync(h->d_fault.ptr, 0, 4, st));
    ORB_HIP_TRY(hipStreamSynchronize(st));
    *fault_mask = h->fault_host;
    if (h->fault_host) {
        set_error("device capacity check failed in a batch (fault mask " + std::to_string(h->fault_host) + ")");
        return ORB_EINTERNAL;
    }
    return ORB_OK;
}

int orbx_fault_word_device(orbx_extractor* h, uint32_t** d_fault) {
    ORB_CHECK_ARG(h && d_fault, "null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    ORB_HIP_TRY(hipSetDevice(h->device));
    int rc;
    if (!h->d_fault.ptr) {
        if ((rc = h->d_fault.reserve(16))) return rc;
        ORB_HIP_TRY(hipMemset(h->d_fault.ptr, 0, 16));
    }
    *d_fault = h->d_fault.as<uint32_t>();
    return ORB_OK;
}

int orbx_pyramid_device(const orbx_extractor* h, int frame, int level, const uint8_t** ptr, int* rows, int* cols,
                        size_t* step) {
    ORB_CHECK_ARG(h && ptr && h->last_in, "no extraction has run");
    ORB_CHECK_ARG(frame >= 0 && frame < h->last_frames && level >= 0 && level < h->geom.nlevels, "bad index");
    const LevelDev& L = h->geom.lv[level];
    if (level == 0) {
        *ptr = h->last_in + (long long)frame * h->last_fstride;
        if (step) *step = h->last_step;
    } else {
        *ptr = h->d_pyr.as<uint8_t>() + (long long)frame * h->geom.pyr_frame_bytes + L.off;
        if (step) *step = (size_t)L.stride;
    }
    if (rows) *rows = L.h;
    if (cols) *cols = L.w;
    return ORB_OK;
}

int orbx_pyramid_level(const orbx_extractor* h, int level, uint8_t* dst, size_t dst_step, int* rows, int* cols) {
    const uint8_t* p = nullptr;
    int r = 0, c = 0;
    size_t st = 0;
    int rc = orbx_pyramid_device(h, 0, level, &p, &r, &c, &st);
    if (rc) return rc;
    if (rows) *rows = r;
    if (cols) *cols = c;
    if (!dst) return ORB_OK;
    ORB_CHECK_ARG(dst_step >= (size_t)c, "dst_step too small");
    ORB_HIP_TRY(hipSetDevice(h->device));
    ORB_HIP_TRY(hipStreamSynchronize(h->stream));
    if (dst_step == st) {
        ORB_HIP_TRY(hipMemcpy(dst, p, (size_t)(r - 1) * st + c, hipMemcpyDeviceToHost));
    } else {   // one 1D copy of the level's rows into host staging, then the row repack on the host: a
               // pitched copy into pageable memory may be staged row by row (ms per level)
        std::vector<uint8_t>& tmp = const_cast<orbx_extractor*>(h)->h_stage;
        tmp.resize((size_t)(r - 1) * st + c);
        ORB_HIP_TRY(hipMemcpy(tmp.data(), p, tmp.size(), hipMemcpyDeviceToHost));
        for (int y = 0; y < r; y++) std::memcpy(dst + (size_t)y * dst_step, tmp.data() + (size_t)y * st, (size_t)c);
    }
    return ORB_OK;
}

int orbx_debug_level_candidates(const orbx_extractor* h, int frame, int level, uint32_t* out, int cap, int* n) {
    ORB_CHECK_ARG(h && n && h->last_frames > 0, "no extraction has run");
    ORB_CHECK_ARG(frame >= 0 && frame < h->last_frames && level >= 0 && level < h->geom.nlevels, "bad index");
    ORB_HIP_TRY(hipSetDevice(h->device));
    ORB_HIP_TRY(hipDeviceSynchronize());
    const Geom& g = h->geom;
    const LevelDev& L = g.lv[level];
    std::vector<int> cnt(std::max(1, L.ncells));
    if (L.ncells)
        ORB_HIP_TRY(hipMemcpy(cnt.data(), h->d_cellcnt.as<int>() + (long long)frame * g.ncells_total + L.cell_base,
                              4 * (size_t)L.ncells, hipMemcpyDeviceToHost));
    std::vector<uint32_t> slots((size_t)g.slot_frame);
    ORB_HIP_TRY(hipMemcpy(slots.data(), h->d_slots.as<uint32_t>() + (long long)frame * g.slot_frame,
                          4 * (size_t)g.slot_frame, hipMemcpyDeviceToHost));
    int m = 0;
    for (int c = 0; c < L.ncells; c++) {
        const CellDev& cd = h->cells[L.cell_base + c];
        for (int j = 0; j < (cnt[c] & CELL_CNT_MASK); j++) {
            if (out && m < cap) out[m] = slots[cd.slot + j];
            m++;
        }
    }
    *n = m;
    return ORB_OK;
}

int orbx_debug_level_selected(const orbx_extractor* h, int frame, int level, uint32_t* out, int cap, int* n) {
    ORB_CHECK_ARG(h && n && h->last_frames > 0, "no extraction has run");
    ORB_CHECK_ARG(frame >= 0 && frame < h->last_frames && level >= 0 && level < h->geom.nlevels, "bad index");
    ORB_HIP_TRY(hipSetDevice(h->device));
    ORB_HIP_TRY(hipDeviceSynchronize());
    const Geom& g = h->geom;
    int c = 0;
    ORB_HIP_TRY(hipMemcpy(&c, h->d_selcnt.as<int>() + frame * g.nlevels + level, 4, hipMemcpyDeviceToHost));
    *n = c;
    if (out && c > 0)
        ORB_HIP_TRY(hipMemcpy(out, h->d_sel.as<uint32_t>() + (long long)frame * g.out_frame + g.lv[level].out_base,
                              4 * (size_t)std::min(c, cap), hipMemcpyDeviceToHost));
    return ORB_OK;
}

int orbx_profile_enable(orbx_extractor* h, int enable) {
    ORB_CHECK_ARG(h, "null extractor");
    std::lock_guard<std::mutex> lk(h->mu);
    h->prof = enable > 0 ? 0xf : (-enable) & 0xf;   // > 0: every stage; < 0: the stages of bitmask -enable

    return ORB_OK;
}

int orbx_pack_descriptors(const uint8_t* desc, int32_t cap, const int32_t* counts, const int32_t* incl,
                          int32_t n_frames, uint8_t* out, int32_t out_rows, void* stream) {
    ORB_CHECK_ARG(n_frames >= 0 && cap >= 0 && out_rows >= 0, "negative sizes");
    if (n_frames == 0 || out_rows == 0) return ORB_OK;
    ORB_CHECK_ARG(desc && counts && incl && out, "null argument");
    ORB_CHECK_ARG(((reinterpret_cast<uintptr_t>(desc) | reinterpret_cast<uintptr_t>(out)) & 15) == 0,
                  "desc / out must be 16-byte aligned");
    hipLaunchKernelGGL(orbamd::pack_rows_kernel, dim3((unsigned)n_frames), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint4*>(desc), (int)cap, counts, incl, reinterpret_cast<uint4*>(out),
                       (int)out_rows);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

int orbx_profile_read(orbx_extractor* h, double* ms, int32_t* launches) {
    ORB_CHECK_ARG(h, "null extractor");
    std::lock_guard<std::mutex> lk(h->mu);
    ORB_HIP_TRY(hipSetDevice(h->device));
    for (int k = 0; k < 4; k++) {
        double tot = 0;
        for (auto& pr : h->prof_ev[k]) {
            ORB_HIP_TRY(hipEventSynchronize(pr.second));
            float t = 0;
            ORB_HIP_TRY(hipEventElapsedTime(&t, pr.first, pr.second));
            tot += t;
            h->ev_pool.push_back(pr.first);
            h->ev_pool.push_back(pr.second);
        }
        if (ms) ms[k] = tot;
        if (launches) launches[k] = (int32_t)h->prof_ev[k].size();
        h->prof_ev[k].clear();
    }
    return ORB_OK;
}

int orbx_debug_qt_sort(const int32_t* sizes, int n, int32_t* perm) {
    ORB_CHECK_ARG(n >= 0 && (n == 0 || (sizes && perm)), "bad argument");
    if (n == 0) return ORB_OK;
    std::vector<QtItem> h(n);
    for (int i = 0; i < n; i++) h[i] = QtItem{sizes[i], i};
    DevBuf d;
    int rc;
    if ((rc = d.reserve((size_t)n * sizeof(QtItem) + ((size_t)n * 8 + 16) * sizeof(int) + 64))) return rc;
    QtItem* items = d.as<QtItem>();
    int* scratch = reinterpret_cast<int*>(items + n);
    ORB_HIP_TRY(hipMemcpy(items, h.data(), n * sizeof(QtItem), hipMemcpyHostToDevice));
    // the kernel keeps items in global memory (same code path as LDS: generic pointers)
    hipLaunchKernelGGL(qt_sort_test_kernel, dim3(1), dim3(256), 0, 0, items, n, scratch);
    ORB_HIP_TRY(hipGetLastError());
    ORB_HIP_TRY(hipMemcpy(h.data(), items, n * sizeof(QtItem), hipMemcpyDeviceToHost));
    d.release();
    for (int i = 0; i < n; i++) perm[i] = h[i].node;
    return ORB_OK;
}

static void stereo_side(const orbx_extractor* h, StereoSide& s) {
    std::memset(&s, 0, sizeof(s));
    const Geom& g = h->geom;
    s.nlevels = g.nlevels;
    s.lvl0 = h->last_in;
    s.fstride0 = h->last_fstride;
    s.step0 = (int)h->last_step;
    s.pyr = h->d_pyr.as<uint8_t>();
    s.pyr_frame = g.pyr_frame_bytes;
    for (int l = 0; l < g.nlevels; l++) {
        s.off[l] = g.lv[l].off;
        s.stride[l] = g.lv[l].stride;
        s.rows[l] = g.lv[l].h;
        s.cols[l] = g.lv[l].w;
    }
}

int orbx_stereo_matches_batch_device(orbx_extractor* left, orbx_extractor* right, int n_frames,
                                     const orbx_keypoint* d_kps_l, const uint8_t* d_desc_l,
                                     const int32_t* d_counts_l, const orbx_keypoint* d_kps_r,
                                     const uint8_t* d_desc_r, const int32_t* d_counts_r, int cap, float bf,
                                     float baseline, float* d_uright, float* d_depth, void* stream) {
    ORB_CHECK_ARG(left && right && d_kps_l && d_desc_l && d_counts_l && d_kps_r && d_desc_r && d_counts_r && d_uright &&
                      d_depth, "null argument");
    ORB_CHECK_ARG(n_frames > 0 && cap > 0, "bad sizes");
    ORB_CHECK_ARG(left->last_in && right->last_in && left->last_frames >= n_frames && right->last_frames >= n_frames,
                  "both extractors need a batch of >= n_frames frames first");
    ORB_CHECK_ARG(left->g_rows == right->g_rows && left->g_cols == right->g_cols &&
                      left->p.nlevels == right->p.nlevels && left->p.scaleFactor == right->p.scaleFactor,
                  "left / right extractors differ in image size or pyramid parameters");
    ORB_CHECK_ARG(left->p.nlevels <= ST_MAX_LEVELS, "too many levels");
    std::lock_guard<std::mutex> lk(left->mu);
    ORB_HIP_TRY(hipSetDevice(left->device));
    int rc;
    StereoSide L, R;
    stereo_side(left, L);
    stereo_side(right, R);
    StereoParams sp;
    std::memset(&sp, 0, sizeof(sp));
    for (int l = 0; l < left->p.nlevels; l++) {
        sp.scale[l] = left->scale[l];
        sp.inv_scale[l] = left->inv_scale[l];
    }
    sp.bf = bf;
    sp.baseline = baseline;
    const size_t ints = stereo_scratch_ints(n_frames, cap, L.rows[0], stereo_row_span(sp, left->p.nlevels));
    if ((rc = left->d_stereo_sad.reserve(ints * sizeof(int32_t)))) return rc;
    return launch_stereo(L, R, sp, n_frames, d_kps_l, d_desc_l, d_counts_l, 0, d_kps_r, d_desc_r, d_counts_r, 0, cap,
                         d_uright, d_depth, left->d_stereo_sad.as<int32_t>(), (hipStream_t)stream);
}

int orbx_stereo_matches_last(orbx_extractor* left, orbx_extractor* right, float bf, float baseline, float* uright,
                             float* depth, int n_left) {
    ORB_CHECK_ARG(left && right && left != right && uright && depth, "null argument");
    ORB_CHECK_ARG(left->last_single && right->last_single, "both extractors need a single-frame orbx_extract first");
    ORB_CHECK_ARG(left->g_rows == right->g_rows && left->g_cols == right->g_cols &&
                      left->p.nlevels == right->p.nlevels && left->p.scaleFactor == right->p.scaleFactor &&
                      left->last_kcap == right->last_kcap,
                  "left / right extractors differ in image size or pyramid parameters");
    ORB_CHECK_ARG(left->p.nlevels <= ST_MAX_LEVELS, "too many levels");
    std::unique_lock<std::mutex> la(left->mu, std::defer_lock), lb(right->mu, std::defer_lock);
    std::lock(la, lb);
    ORB_HIP_TRY(hipSetDevice(left->device));
    const int cap = left->last_kcap;
    int32_t nl = 0;
    ORB_HIP_TRY(hipMemcpy(&nl, left->d_counts.ptr, 4, hipMemcpyDeviceToHost));
    ORB_CHECK_ARG(n_left == nl, "n_left differs from the left extractor's keypoint count");
    if (nl == 0) return ORB_OK;
    int rc;
    StereoSide L, R;
    stereo_side(left, L);
    stereo_side(right, R);
    StereoParams sp;
    std::memset(&sp, 0, sizeof(sp));
    for (int l = 0; l < left->p.nlevels; l++) {
        sp.scale[l] = left->scale[l];
        sp.inv_scale[l] = left->inv_scale[l];
    }
    sp.bf = bf;
    sp.baseline = baseline;
    const size_t ints = stereo_scratch_ints(1, cap, L.rows[0], stereo_row_span(sp, left->p.nlevels));
    if ((rc = left->d_stereo_sad.reserve(ints * sizeof(int32_t)))) return rc;
    if ((rc = left->d_stereo_out.reserve(2 * (size_t)cap * sizeof(float)))) return rc;
    float* d_u = left->d_stereo_out.as<float>();
    float* d_d = d_u + cap;
    hipStream_t st = left->stream;
    if ((rc = launch_stereo(L, R, sp, 1, left->d_kps.as<orbx_keypoint>(), left->d_desc.as<uint8_t>(),
                            left->d_counts.as<int32_t>(), 0, right->d_kps.as<orbx_keypoint>(), right->d_desc.as<uint8_t>(),
                            right->d_counts.as<int32_t>(), 0, cap, d_u, d_d, left->d_stereo_sad.as<int32_t>(), st)))
        return rc;
    ORB_HIP_TRY(hipMemcpyAsync(uright, d_u, (size_t)nl * sizeof(float), hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipMemcpyAsync(depth, d_d, (size_t)nl * sizeof(float), hipMemcpyDeviceToHost, st));
    ORB_HIP_TRY(hipStreamSynchronize(st));
    return ORB_OK;
}

int orbx_debug_fast_stamps(unsigned long long* out, int n_words) {
#ifdef ORB_FAST_STAMPS
    ORB_CHECK_ARG(out && n_words > 0 && n_words <= FAST_NSAMP * 8, "bad stamp buffer");
    ORB_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_stamps), (size_t)n_words * 8));
    return ORB_OK;
#else
    (void)out;
    (void)n_words;
    set_error("built without ORB_FAST_STAMPS");
    return ORB_EINVAL;
#endif
}

int orbx_debug_qt_stamps(unsigned long long* out) {
#if defined(ORB_DESC_STAMPS)
    ORB_HIP_TRY(hipDeviceSynchronize());
    ORB_HIP_TRY(hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_desc_stamps), 1024 * 8 * 8));
    return ORB_OK;
#elif defined(ORB_QT_STAMPS)
    ORB_HIP_TRY(hipDeviceSynchronize());
    ORB_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qt_stamps), 64 * 8));
    ORB_HIP_TRY(hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(g_qt_wg), 4096 * 2 * 8));
    return ORB_OK;
#else
    (void)out;
    set_error("built without ORB_QT_STAMPS");
    return ORB_EINVAL;
#endif
}

}  // extern "C"
