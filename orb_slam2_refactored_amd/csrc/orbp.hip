// orbp.hip — FeaturesGrid + ORBmatcher::SearchByProjection(Frame&, const std::vector<MapPoint*>&, th)
// on gfx950, batched over frames.
//
// Reference: src/Frame.cc:71-145 (AssignFeatures / GetFeaturesInArea, Round / RoundUp / RoundDn at
// :32-34), src/ORBmatcher.cc:315-382 (the search) and :53 (RadiusByViewingCos).
//
// The reference loop is sequential in one respect only: a keypoint that an earlier map point has
// claimed (frame.mappoints[idx] with Observations() > 0, :339) is skipped by the later ones.  So
// the work splits into two data-parallel stages and one thin sequential one:
//   pj_grid_kernel   one WG per frame: cell of every keypoint (Round of the scaled offset), a
//                    bitonic sort of (cell << 13 | index) in LDS, the sorted indices and the
//                    3072 + 1 cell starts.  Cell c = cx * 48 + cy, so a window's column cx is one
//                    contiguous range and sorted position = GetFeaturesInArea's scan order.
//   pj_score_kernel  one wavefront per map point: window cells, level / area / entry-claim /
//                    stereo gates, Hamming distance, and the K smallest keys (dist << 13 | scan
//                    position) = the first K of the candidates stably sorted by distance, plus
//                    the candidate count.
//   pj_walk_kernel   one wavefront per frame walks the map points in order with a claim bitmap
//                    in LDS: best / second best = the first two unclaimed of the K (the
//                    reference's strict-< scan keeps exactly the first two of that stable order);
//                    when fewer than two of the K are unclaimed and more candidates exist, the
//                    wavefront rescans that map point's window against the bitmap.  Then the
//                    TH_HIGH / same-level ratio test and the claim.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "common.h"
#include "qt_sort.h"

namespace orbamd {

constexpr int PJ_COLS = ORBM_GRID_COLS, PJ_ROWS = ORBM_GRID_ROWS, PJ_CELLS = PJ_COLS * PJ_ROWS;
constexpr int PJ_MAXKP = ORBM_PROJ_MAX_KP;
constexpr int PJ_IDX_BITS = 13;
static_assert((1 << PJ_IDX_BITS) == PJ_MAXKP, "sort key packs the keypoint index in 13 bits");
constexpr uint32_t PJ_IDX_MASK = (1u << PJ_IDX_BITS) - 1;
#ifndef PJ_K_OVERRIDE
constexpr int PJ_K = 4;          // candidates kept per map point
#else
constexpr int PJ_K = PJ_K_OVERRIDE;   // diagnostic builds: K = 1 forces the rescan path
#endif
constexpr int PJ_TH_HIGH = 100;  // ORBmatcher.cc:41
constexpr int PJ_MAX_LEVELS = 32;
constexpr uint32_t PJ_NONE = 0xffffffffu;

struct PjArgs {
    int n_frames;
    const int32_t* kp_begin;
    const float* kp_xy;
    const int32_t* kp_oct;
    const float* kp_ur;
    const uint8_t* kp_desc;
    const uint8_t* kp_claimed;
    const float* bounds;
    const int32_t* mp_begin;
    const uint8_t* mp_valid;
    const float* mp_proj;
    const float* mp_vcos;
    const int32_t* mp_level;
    const uint8_t* mp_desc;
    const uint8_t* mp_has_obs;
    int n_levels;
    float scale[PJ_MAX_LEVELS];
    float th, nnratio;
    int total_mp;
    // workspace
    int32_t* grid_idx;    // total_kp: frame-relative keypoint index at each sorted position
    int32_t* grid_start;  // n_frames x (PJ_CELLS + 1)
    int32_t* mp_cnt;      // total_mp
    int32_t* mp_frame;    // total_mp: frame of each map point (pj_grid_kernel)
    uint2* mp_top;        // total_mp x PJ_K: (key, index | level << 24)
    // outputs
    int32_t* kp_match;
    int32_t* n_matches;
};

__device__ __forceinline__ int pj_hamming(const uint8_t* a, const uint8_t* b) {
    const uint4* x = reinterpret_cast<const uint4*>(a);
    const uint4* y = reinterpret_cast<const uint4*>(b);
    const uint4 a0 = x[0], a1 = x[1], b0 = y[0], b1 = y[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// reductions over a group of W lanes (W = 64: the wavefront; W = 16: a quarter of it)
template <int W = 64>
__device__ __forceinline__ uint32_t pj_wave_min(uint32_t v) {
#pragma unroll
    for (int m = W / 2; m > 0; m >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, m, W));
    return v;
}

template <int W = 64>
__device__ __forceinline__ int pj_wave_sum(int v) {
#pragma unroll
    for (int m = W / 2; m > 0; m >>= 1) v += __shfl_xor(v, m, W);
    return v;
}

// ---------------------------------------------------------------- FeaturesGrid::AssignFeatures
__global__ __launch_bounds__(256) void pj_grid_kernel(PjArgs a) {
    __shared__ uint32_t keys[PJ_MAXKP];
    const int f = blockIdx.x;
    const int k0 = a.kp_begin[f], n = a.kp_begin[f + 1] - k0;
    int32_t* cs = a.grid_start + (size_t)f * (PJ_CELLS + 1);
    for (int j = a.mp_begin[f] + threadIdx.x; j < a.mp_begin[f + 1]; j += 256) a.mp_frame[j] = f;
    if (n > PJ_MAXKP) return;   // pj_walk_kernel reports the frame
    const float* bd = a.bounds + 4 * (size_t)f;
    const float minx = bd[0], miny = bd[2];
    const float invW = PJ_COLS / (bd[1] - bd[0]);   // COLS / ImageBounds::Width() (Frame.cc:73)
    const float invH = PJ_ROWS / (bd[3] - bd[2]);
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = threadIdx.x; i < P; i += 256) {
        uint32_t key = PJ_NONE;
        if (i < n) {
            const int cx = (int)roundf(invW * (a.kp_xy[2 * (size_t)(k0 + i)] - minx));   // Round (:32, :91)
            const int cy = (int)roundf(invH * (a.kp_xy[2 * (size_t)(k0 + i) + 1] - miny));
            if (cx >= 0 && cx < PJ_COLS && cy >= 0 && cy < PJ_ROWS)
                key = ((uint32_t)(cx * PJ_ROWS + cy) << PJ_IDX_BITS) | (uint32_t)i;
        }
        keys[i] = key;
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)       // bitonic sort; keys are unique (index in the low bits)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t x = keys[i], y = keys[ixj];
                    if ((x > y) == ((i & k) == 0)) { keys[i] = y; keys[ixj] = x; }
                }
            }
            __syncthreads();
        }
    for (int p = threadIdx.x; p < n; p += 256)
        a.grid_idx[k0 + p] = keys[p] == PJ_NONE ? -1 : (int32_t)(keys[p] & PJ_IDX_MASK);
    for (int c = threadIdx.x; c <= PJ_CELLS; c += 256) {   // lower_bound(c << 13)
        const uint32_t want = (uint32_t)c << PJ_IDX_BITS;
        int lo = 0, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (keys[mid] < want) lo = mid + 1; else hi = mid;
        }
        cs[c] = lo;
    }
}

// ---------------------------------------------------------------- GetFeaturesInArea + gates
struct PjPoint {   // one map point's search window (ORBmatcher.cc:322-333, Frame.cc:109-119)
    int mincx, maxcx, mincy, maxcy, lvl;
    float u, v, uR, radius;
    bool any;
};

__device__ __forceinline__ PjPoint pj_point(const PjArgs& a, int f, int mj) {
    PjPoint w;
    w.lvl = a.mp_level[mj];
    const float vcos = a.mp_vcos[mj];
    const float r = (double)vcos > 0.998 ? 2.5f : 4.f;   // RadiusByViewingCos (:53), double compare
    w.radius = a.th * r * a.scale[w.lvl];
    w.u = a.mp_proj[3 * (size_t)mj];
    w.v = a.mp_proj[3 * (size_t)mj + 1];
    w.uR = a.mp_proj[3 * (size_t)mj + 2];
    const float* bd = a.bounds + 4 * (size_t)f;
    const float minx = bd[0], miny = bd[2];
    const float invW = PJ_COLS / (bd[1] - bd[0]), invH = PJ_ROWS / (bd[3] - bd[2]);
    w.mincx = max((int)floorf(invW * (w.u - w.radius - minx)), 0);
    w.maxcx = min((int)ceilf(invW * (w.u + w.radius - minx)), PJ_COLS - 1);
    w.mincy = max((int)floorf(invH * (w.v - w.radius - miny)), 0);
    w.maxcy = min((int)ceilf(invH * (w.v + w.radius - miny)), PJ_ROWS - 1);
    w.any = !(w.mincx >= PJ_COLS || w.maxcx < 0 || w.mincy >= PJ_ROWS || w.maxcy < 0);
    return w;
}

// Calls fn(key, idx, level) for each candidate of this lane that passes every gate; key =
// dist << 13 | sorted position (increasing along GetFeaturesInArea's scan order).
template <bool DYN, int W = 64, class Fn>
__device__ __forceinline__ void pj_scan(const PjArgs& a, int f, int mj, const PjPoint& w, const uint32_t* bits,
                                        int lane, Fn&& fn) {
    if (!w.any) return;
    const int k0 = a.kp_begin[f];
    const int32_t* cs = a.grid_start + (size_t)f * (PJ_CELLS + 1);
    const uint8_t* d1 = a.mp_desc + 32 * (size_t)mj;
    for (int cx = w.mincx; cx <= w.maxcx; cx++) {
        const int p0 = cs[cx * PJ_ROWS + w.mincy], p1 = cs[cx * PJ_ROWS + w.maxcy + 1];
        for (int p = p0 + lane; p < p1; p += W) {
            const int idx = a.grid_idx[k0 + p];
            const int k = k0 + idx;
            const int level = a.kp_oct[k];
            if (level < w.lvl - 1 || level > w.lvl) continue;   // checkLevels (maxLevel >= 0)
            const float distx = a.kp_xy[2 * (size_t)k] - w.u;
            const float disty = a.kp_xy[2 * (size_t)k + 1] - w.v;
            if (!(fabsf(distx) < w.radius && fabsf(disty) < w.radius)) continue;
            if (a.kp_claimed && a.kp_claimed[k]) continue;
            if (DYN && ((bits[idx >> 5] >> (idx & 31)) & 1u)) continue;
            const float ur = a.kp_ur[k];
            if (ur > 0 && fabsf(w.uR - ur) > w.radius) continue;
            const int dist = pj_hamming(d1, a.kp_desc + 32 * (size_t)k);
            fn(((uint32_t)dist << PJ_IDX_BITS) | (uint32_t)p, idx, level);
        }
    }
}

template <int K>
__device__ __forceinline__ void pj_insert(uint32_t (&t)[K], uint32_t key) {
#pragma unroll
    for (int r = 0; r < K; r++) {
        const uint32_t lo = min(t[r], key), hi = max(t[r], key);
        t[r] = lo;
        key = hi;
    }
}

// Pops the wave's K smallest keys (one lane owns each key: positions are unique).
template <int K, int W = 64>
__device__ __forceinline__ void pj_wave_topk(uint32_t (&t)[K], uint32_t (&out)[K]) {
#pragma unroll
    for (int r = 0; r < K; r++) {
        const uint32_t m = pj_wave_min<W>(t[0]);
        out[r] = m;
        if (t[0] == m && m != PJ_NONE) {
#pragma unroll
            for (int q = 0; q + 1 < K; q++) t[q] = t[q + 1];
            t[K - 1] = PJ_NONE;
        }
    }
}

// ---------------------------------------------------------------- per map point: top-K candidates
// A 16-lane group per map point (4 per wavefront; the windows at the search radii hold tens of
// candidates), the frame from pj_grid_kernel's map-point -> frame table.
constexpr int PJ_GW = 16;
__global__ __launch_bounds__(256) void pj_score_kernel(PjArgs a) {
    const int lane = threadIdx.x & (PJ_GW - 1);
    const int mj = blockIdx.x * (256 / PJ_GW) + (threadIdx.x / PJ_GW);
    if (mj >= a.total_mp) return;   // group-uniform (every later reduction stays inside the group)
    const int f = a.mp_frame[mj];
    const int n = a.kp_begin[f + 1] - a.kp_begin[f];
    int cnt = 0;
    uint32_t out[PJ_K];
#pragma unroll
    for (int r = 0; r < PJ_K; r++) out[r] = PJ_NONE;
    const int lvl = a.mp_level[mj];
    if (n <= PJ_MAXKP && a.mp_valid[mj] && lvl >= 0 && lvl < a.n_levels) {
        const PjPoint w = pj_point(a, f, mj);
        uint32_t t[PJ_K];
#pragma unroll
        for (int r = 0; r < PJ_K; r++) t[r] = PJ_NONE;
        int c = 0;
        pj_scan<false, PJ_GW>(a, f, mj, w, nullptr, lane, [&](uint32_t key, int, int) {
            pj_insert(t, key);
            c++;
        });
        cnt = pj_wave_sum<PJ_GW>(c);
        pj_wave_topk<PJ_K, PJ_GW>(t, out);
    }
    if (lane == 0) a.mp_cnt[mj] = cnt;
    if (lane < PJ_K) {
        uint32_t key = out[0];
#pragma unroll
        for (int r = 1; r < PJ_K; r++) key = lane == r ? out[r] : key;
        uint32_t ent = 0;
        if (key != PJ_NONE) {
            const int k0 = a.kp_begin[f];
            const int idx = a.grid_idx[k0 + (int)(key & PJ_IDX_MASK)];
            ent = (uint32_t)idx | ((uint32_t)a.kp_oct[k0 + idx] << 24);
        }
        a.mp_top[(size_t)mj * PJ_K + lane] = make_uint2(key, ent);
    }
}

// ---------------------------------------------------------------- the ordered claim walk
// One wavefront per frame, 64 map points per chunk, one lane per map point.  A map point's outcome
// depends on the earlier ones only through the claim bitmap (keypoints whose map point has
// observations, :339), and only through the claim bits of its K kept candidates while two of them
// remain available (else the window is rescanned).  So every round decides all remaining lanes of
// the chunk at once against the current bitmap, marks each claimed keypoint with the lowest
// claiming lane (LDS atomicMin), and commits the lanes before the first one that either saw an
// available candidate claimed by an earlier lane of the round or needs a rescan.  Claims set bits
// as the reference's loop would, in lane order (a committed lane saw no earlier claim on its
// candidates); kp_match keeps the last map point to match a keypoint (:374) by atomicMax on the map
// point index, which grows with the walk.  The first undecided lane then runs next round, or — when
// it needs the rescan — alone on the wavefront as the sequential walk does.
constexpr int PJ_CHUNK = 64;

__global__ __launch_bounds__(64) void pj_walk_kernel(PjArgs a) {
    __shared__ uint32_t bits[PJ_MAXKP / 32];
    __shared__ int stamp[PJ_MAXKP];   // lowest claiming lane of the round (64: none)
    const int lane = threadIdx.x;
    const int f = blockIdx.x;
    const int k0 = a.kp_begin[f], n = a.kp_begin[f + 1] - k0;
    const int m0 = a.mp_begin[f], nm = a.mp_begin[f + 1] - m0;
    for (int i = lane; i < n; i += 64) a.kp_match[k0 + i] = -1;
    if (n > PJ_MAXKP) {
        if (lane == 0) a.n_matches[f] = -1;
        return;
    }
    for (int w = lane; w < (n + 31) / 32; w += 64) {
        uint32_t v = 0;
        if (a.kp_claimed)
            for (int b = 0; b < 32 && w * 32 + b < n; b++) v |= (uint32_t)(a.kp_claimed[k0 + w * 32 + b] != 0) << b;
        bits[w] = v;
    }
    for (int i = lane; i < n; i += 64) stamp[i] = 64;
    __syncthreads();
    auto bit = [&](int idx) { return (bits[idx >> 5] >> (idx & 31)) & 1u; };
    int nmatches = 0;
    for (int c = 0; c < nm; c += PJ_CHUNK) {
        const int m = min(PJ_CHUNK, nm - c);
        // this lane's map point: validity, candidate count, observations, K kept candidates
        int cnt = 0;
        bool has_obs = false;
        uint2 e[PJ_K];
#pragma unroll
        for (int k = 0; k < PJ_K; k++) e[k] = make_uint2(PJ_NONE, 0);
        if (lane < m) {
            const int mj = m0 + c + lane;
            const int lvl = a.mp_level[mj];
            const bool ok = a.mp_valid[mj] && lvl >= 0 && lvl < a.n_levels;
            cnt = ok ? a.mp_cnt[mj] : 0;
            has_obs = a.mp_has_obs[mj] != 0;
#pragma unroll
            for (int k = 0; k < PJ_K; k++) e[k] = a.mp_top[(size_t)mj * PJ_K + k];
        }
        int start = 0;
        while (start < m) {   // wavefront-uniform
            // decide every lane >= start against the current bitmap
            uint32_t avail = 0;
#pragma unroll
            for (int k = 0; k < PJ_K; k++)
                if (e[k].x != PJ_NONE && !bit((int)(e[k].y & 0xffffffu))) avail |= 1u << k;
            const bool mine = lane >= start && lane < m && cnt > 0;
            const bool rescan = mine && !(__popc(avail) >= 2 || cnt <= PJ_K);
            bool match = false;
            int bidx = -1;
            if (mine && !rescan && avail) {
                const int l0 = __ffs(avail) - 1;
                const uint32_t rest = avail & (avail - 1);
                uint32_t bkey = PJ_NONE, skey = PJ_NONE, be = 0, se = 0;
#pragma unroll
                for (int k = 0; k < PJ_K; k++)
                    if (k == l0) { bkey = e[k].x; be = e[k].y; }
                if (rest) {
                    const int l1 = __ffs(rest) - 1;
#pragma unroll
                    for (int k = 0; k < PJ_K; k++)
                        if (k == l1) { skey = e[k].x; se = e[k].y; }
                }
                const int bestDist = (int)(bkey >> PJ_IDX_BITS);
                const int secondDist = skey == PJ_NONE ? 256 : (int)(skey >> PJ_IDX_BITS);
                const int blev = (int)(be >> 24), slev = skey == PJ_NONE ? -1 : (int)(se >> 24);
                if (bestDist <= PJ_TH_HIGH && !(blev == slev && (float)bestDist > a.nnratio * (float)secondDist)) {   // :367-377
                    match = true;
                    bidx = (int)(be & 0xffffffu);
                }
            }
            const bool claims = match && has_obs;
            if (claims) atomicMin(&stamp[bidx], lane);
            __syncthreads();   // one wavefront: orders its LDS writes before the reads below
            bool conflict = rescan;
            if (mine && !rescan) {
#pragma unroll
                for (int k = 0; k < PJ_K; k++)
                    if (((avail >> k) & 1u) && stamp[(int)(e[k].y & 0xffffffu)] < lane) conflict = true;
            }
            const unsigned long long cb = __ballot(conflict);
            const int stop = cb ? __ffsll((long long)cb) - 1 : m;   // first undecided lane
            // commit [start, stop)
            const bool commit = lane >= start && lane < stop && match;
            if (commit) {
                atomicMax(a.kp_match + k0 + bidx, c + lane);
                if (claims) atomicOr(&bits[bidx >> 5], 1u << (bidx & 31));
            }
            nmatches += (int)__popcll(__ballot(commit));
            if (claims) stamp[bidx] = 64;
            __syncthreads();   // one wavefront: orders its LDS writes before the reads below
            if (stop == start) {
                // lane `start` needs the rescan: the window with the current bitmap, on the wavefront
                const int i = start;
                const int mj = m0 + c + i;
                const PjPoint w = pj_point(a, f, mj);
                uint32_t t[2] = {PJ_NONE, PJ_NONE};
                pj_scan<true>(a, f, mj, w, bits, lane, [&](uint32_t key, int, int) { pj_insert(t, key); });
                uint32_t o[2];
                pj_wave_topk(t, o);
                const uint32_t bkey = o[0], skey = o[1];
                int bi = -1, blev = -1, slev = -1;
                if (bkey != PJ_NONE) {
                    bi = a.grid_idx[k0 + (int)(bkey & PJ_IDX_MASK)];
                    blev = a.kp_oct[k0 + bi];
                }
                if (skey != PJ_NONE) slev = a.kp_oct[k0 + a.grid_idx[k0 + (int)(skey & PJ_IDX_MASK)]];
                const int bestDist = bkey == PJ_NONE ? 256 : (int)(bkey >> PJ_IDX_BITS);
                const int secondDist = skey == PJ_NONE ? 256 : (int)(skey >> PJ_IDX_BITS);
                const bool obs_i = __shfl(has_obs ? 1 : 0, i, 64) != 0;
                if (bestDist <= PJ_TH_HIGH && !(blev == slev && (float)bestDist > a.nnratio * (float)secondDist)) {
                    if (lane == 0) {
                        atomicMax(a.kp_match + k0 + bi, c + i);
                        if (obs_i) bits[bi >> 5] |= 1u << (bi & 31);
                    }
                    nmatches++;
                }
                __syncthreads();   // one wavefront: orders its LDS writes before the reads below
                start = i + 1;
            } else {
                start = stop;
            }
        }
    }
    if (lane == 0) a.n_matches[f] = nmatches;
}

static int launch_projection(PjArgs& a, int total_kp, hipStream_t st) {
    if (a.n_frames == 0) return ORB_OK;
    (void)total_kp;
    hipLaunchKernelGGL(pj_grid_kernel, dim3(a.n_frames), dim3(256), 0, st, a);
    ORB_HIP_TRY(hipGetLastError());
    if (a.total_mp > 0) {
        hipLaunchKernelGGL(pj_score_kernel, dim3((a.total_mp + 256 / PJ_GW - 1) / (256 / PJ_GW)), dim3(256), 0, st, a);
        ORB_HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(pj_walk_kernel, dim3(a.n_frames), dim3(64), 0, st, a);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

// ---------------------------------------------------------------- SearchByProjection(Frame&, const Frame&, th, mono)
// (ORBmatcher.cc:1279-1362, TrackWithMotionModel).  Same grid (pj_grid_kernel) and the same claim
// rule (a keypoint whose current map point has observations is skipped, :1331-1333), but only the
// best distance counts (no ratio), so one wavefront per frame walks the last frame's points in idx1
// order: each point's window is scanned by the lanes against the LDS claim bitmap and the wave
// minimum of (dist << 13 | scan position) is the reference's first-best.  The accepted pair of every
// point is kept (choice) for CheckOrientation, which counts overwritten pairs too (matchIds).
struct PjmExtra {
    const int32_t* motion;
    const float* kp_angle;
    const float* mp_angle;
    int32_t* choice;   // total_mp: accepted idx2 or -1
    int max_dist;      // TH_HIGH (:1347); ORBdist for SearchByProjection(Frame&, KeyFrame*, ...) (:1425)
};

// The window scan of one last-frame point (GetFeaturesInArea + the gates of :1329-1339): each lane's
// smallest (dist << 13 | scan position), against the claim bitmap when `bits` is given.
__device__ __forceinline__ uint32_t pjm_scan(const PjArgs& a, const PjmExtra& e, int f, int j, const uint32_t* bits,
                                             int lane, int nlanes) {
    const int k0 = a.kp_begin[f];
    const int mot = e.motion ? e.motion[f] : 0;
    const float* bd = a.bounds + 4 * (size_t)f;
    const float minx = bd[0], miny = bd[2];
    const float invW = PJ_COLS / (bd[1] - bd[0]), invH = PJ_ROWS / (bd[3] - bd[2]);
    const int32_t* cs = a.grid_start + (size_t)f * (PJ_CELLS + 1);
    const int oct = a.mp_level[j];
    uint32_t best = PJ_NONE;
    if (oct < 0 || oct >= a.n_levels) return best;   // no level to project at: no candidate
    const float r = a.th * a.scale[oct];   // :1316
    // :1318-1319 through GetFeaturesInArea's checkLevels (maxLevel < 0 -> nlevels)
    const int lo = mot == 1 ? oct : (mot == 2 ? 0 : oct - 1);
    const int hi = mot == 1 ? a.n_levels : (mot == 2 ? oct : oct + 1);
    const float u = a.mp_proj[3 * (size_t)j], v = a.mp_proj[3 * (size_t)j + 1];
    const float uR = a.kp_ur ? a.mp_proj[3 * (size_t)j + 2] : 0.f;
    const int mincx = max((int)floorf(invW * (u - r - minx)), 0);
    const int maxcx = min((int)ceilf(invW * (u + r - minx)), PJ_COLS - 1);
    const int mincy = max((int)floorf(invH * (v - r - miny)), 0);
    const int maxcy = min((int)ceilf(invH * (v + r - miny)), PJ_ROWS - 1);
    if (mincx >= PJ_COLS || maxcx < 0 || mincy >= PJ_ROWS || maxcy < 0) return best;
    const uint8_t* d1 = a.mp_desc + 32 * (size_t)j;
    for (int cx = mincx; cx <= maxcx; cx++) {
        const int p0 = cs[cx * PJ_ROWS + mincy], p1 = cs[cx * PJ_ROWS + maxcy + 1];
        for (int p = p0 + lane; p < p1; p += nlanes) {
            const int idx = a.grid_idx[k0 + p];
            const int k = k0 + idx;
            const int level = a.kp_oct[k];
            if (level < lo || level > hi) continue;
            const float distx = a.kp_xy[2 * (size_t)k] - u;
            const float disty = a.kp_xy[2 * (size_t)k + 1] - v;
            if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
            if (a.kp_claimed && a.kp_claimed[k]) continue;
            if (bits && ((bits[idx >> 5] >> (idx & 31)) & 1u)) continue;
            if (a.kp_ur) {   // the stereo gate of :1335 (the relocalisation search has none)
                const float ur = a.kp_ur[k];
                if (ur > 0 && fabsf(uR - ur) > r) continue;
            }
            const int dist = pj_hamming(d1, a.kp_desc + 32 * (size_t)k);
            best = min(best, ((uint32_t)dist << PJ_IDX_BITS) | (uint32_t)p);
        }
    }
    return best;
}

// Data-parallel first pass: every point's best key against the entry claims only (a 16-lane group
// per point).  Claims made during the call only remove candidates, so the walk keeps this key
// whenever its keypoint is still unclaimed and rescans otherwise.
__global__ __launch_bounds__(256) void pjm_score_kernel(PjArgs a, PjmExtra e) {
    const int j = blockIdx.x * (256 / PJ_GW) + (threadIdx.x / PJ_GW), lane = threadIdx.x % PJ_GW;
    if (j >= a.total_mp) return;
    const int f = a.mp_frame[j];
    uint32_t best = PJ_NONE;
    if (a.kp_begin[f + 1] - a.kp_begin[f] <= PJ_MAXKP && a.mp_valid[j]) best = pjm_scan(a, e, f, j, nullptr, lane, PJ_GW);
    best = pj_wave_min<PJ_GW>(best);
    if (lane == 0) a.mp_cnt[j] = (int32_t)best;
}

// The ordered walk: 64 points per chunk with their first-pass keys in registers; a point whose key's
// keypoint was claimed earlier in the call (an earlier point with observations took it) rescans its
// window against the LDS claim bitmap.
__global__ __launch_bounds__(64) void pjm_walk_kernel(PjArgs a, PjmExtra e) {
    __shared__ uint32_t bits[PJ_MAXKP / 32];
    const int f = blockIdx.x, lane = threadIdx.x;
    const int k0 = a.kp_begin[f], n = a.kp_begin[f + 1] - k0;
    const int m0 = a.mp_begin[f], m1 = a.mp_begin[f + 1];
    for (int i = lane; i < n; i += 64) a.kp_match[k0 + i] = -1;   // also for an over-limit frame
    if (n > PJ_MAXKP) {
        for (int j = m0 + lane; j < m1; j += 64) e.choice[j] = -1;
        if (lane == 0) a.n_matches[f] = -1;
        return;
    }
    for (int i = lane; i < PJ_MAXKP / 32; i += 64) bits[i] = 0;
    __syncthreads();
    int nm = 0;
    for (int c = m0; c < m1; c += 64) {
        const int j = c + lane;
        uint32_t key = PJ_NONE;
        int idx = -1, obs = 0;
        if (j < m1) {
            key = (uint32_t)a.mp_cnt[j];
            obs = a.mp_has_obs ? a.mp_has_obs[j] : 1;   // NULL: every accepted point claims (relocalisation)
            if (key != PJ_NONE) idx = a.grid_idx[k0 + (int)(key & PJ_IDX_MASK)];
        }
        int mych = -1;
        const int cnt = min(64, m1 - c);
        for (int i = 0; i < cnt; i++) {
            uint32_t K = (uint32_t)__shfl((int)key, i, 64);
            if (K == PJ_NONE || (int)(K >> PJ_IDX_BITS) > e.max_dist) continue;   // :1347 (a rescan only loses candidates)
            int ch = __shfl(idx, i, 64);
            if ((bits[ch >> 5] >> (ch & 31)) & 1u) {   // taken earlier in this call: rescan
                K = pj_wave_min(pjm_scan(a, e, f, c + i, bits, lane, 64));
                if (K == PJ_NONE || (int)(K >> PJ_IDX_BITS) > e.max_dist) continue;
                ch = a.grid_idx[k0 + (int)(K & PJ_IDX_MASK)];
            }
            const int ob = __shfl(obs, i, 64);   // every lane takes part in the shuffle
            if (lane == 0) {
                a.kp_match[k0 + ch] = c + i - m0;
                if (ob) bits[ch >> 5] |= 1u << (ch & 31);
            }
            if (lane == i) mych = ch;
            nm++;
            __syncthreads();   // one wavefront: the claim bit before the next point
        }
        if (j < m1) e.choice[j] = mych;
    }
    if (lane == 0) a.n_matches[f] = nm;
}

__device__ __forceinline__ int pjm_bin(float ang1, float ang2) {   // diffToBin(keypoint1.angle - keypoint2.angle)
    float diff = ang1 - ang2;
    if (diff < 0) diff += 360.f;
    int bin = __float2int_rn((1.f / 30) * diff);
    if (bin == 30) bin = 0;
    return min(max(bin, 0), 29);
}

// CheckOrientation(lastFrame.keypointsUn, currFrame.keypointsUn, matchIds, currFrame.mappoints)
// (:249-309, :1358-1359): hist of every accepted (idx1, idx2), bins sorted by size with libstdc++'s
// order (qt_sort), mappoints[idx2] erased for every pair outside the kept bins.
__global__ __launch_bounds__(256) void pjm_orient_kernel(PjArgs a, PjmExtra e) {
    __shared__ int hist[30];
    __shared__ uint32_t keep;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int k0 = a.kp_begin[f], n = a.kp_begin[f + 1] - k0;
    const int m0 = a.mp_begin[f], m1 = a.mp_begin[f + 1];
    if (n > PJ_MAXKP) return;
    if (tid < 30) hist[tid] = 0;
    __syncthreads();
    for (int j = m0 + tid; j < m1; j += 256) {
        const int ch = e.choice[j];
        if (ch >= 0) atomicAdd(&hist[pjm_bin(e.mp_angle[j], e.kp_angle[k0 + ch])], 1);
    }
    __syncthreads();
    if (tid == 0) {
        QtItem it[30];
        for (int b = 0; b < 30; b++) it[b] = QtItem{hist[b], b};
        qt_sort(it, it + 30);
        const double max1 = it[0].size, max2 = it[1].size, max3 = it[2].size;
        const int eraseBin = max2 < 0.1 * max1 ? 1 : (max3 < 0.1 * max1 ? 2 : 3);
        uint32_t k = 0;
        int kept = 0;
        for (int r = 0; r < eraseBin; r++) {
            k |= 1u << it[r].node;
            kept += it[r].size;
        }
        keep = k;
        a.n_matches[f] = kept;
    }
    __syncthreads();
    const uint32_t k = keep;
    for (int j = m0 + tid; j < m1; j += 256) {
        const int ch = e.choice[j];
        if (ch >= 0 && !((k >> pjm_bin(e.mp_angle[j], e.kp_angle[k0 + ch])) & 1u)) a.kp_match[k0 + ch] = -1;
    }
}

struct PjScratch {
    DevBuf ws, io;
    int device = -1;
};
thread_local PjScratch g_pj;

static size_t pj_workspace_bytes(int n_frames, int total_kp, int total_mp) {
    return align_up((size_t)std::max(total_kp, 1) * 4, 256) + align_up((size_t)n_frames * (PJ_CELLS + 1) * 4, 256) +
           2 * align_up((size_t)std::max(total_mp, 1) * 4, 256) + align_up((size_t)std::max(total_mp, 1) * PJ_K * 8, 256);
}

static void pj_carve(PjArgs& a, char* ws, int n_frames, int total_kp, int total_mp) {
    size_t o = 0;
    a.grid_idx = (int32_t*)(ws + o);
    o += align_up((size_t)std::max(total_kp, 1) * 4, 256);
    a.grid_start = (int32_t*)(ws + o);
    o += align_up((size_t)n_frames * (PJ_CELLS + 1) * 4, 256);
    a.mp_cnt = (int32_t*)(ws + o);
    o += align_up((size_t)std::max(total_mp, 1) * 4, 256);
    a.mp_frame = (int32_t*)(ws + o);
    o += align_up((size_t)std::max(total_mp, 1) * 4, 256);
    a.mp_top = (uint2*)(ws + o);
}

static int pj_common_args(const orbm_proj_batch* b, PjArgs& a) {
    ORB_CHECK_ARG(b, "null argument");
    ORB_CHECK_ARG(b->n_frames >= 0 && b->total_kp >= 0 && b->total_mp >= 0, "negative sizes");
    ORB_CHECK_ARG(b->n_levels >= 1 && b->n_levels <= PJ_MAX_LEVELS && b->scale_factors, "bad scale pyramid");
    std::memset(&a, 0, sizeof(a));
    a.n_frames = b->n_frames;
    a.n_levels = b->n_levels;
    for (int l = 0; l < b->n_levels; l++) a.scale[l] = b->scale_factors[l];
    a.th = b->th;
    a.nnratio = b->nnratio;
    a.total_mp = b->total_mp;
    return ORB_OK;
}

// ---------------------------------------------------------------- SearchForInitialization
// ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:614-694), batched over pairs (F1, F2).
// The reference walks the octave-0 features of F1 in idx1 order against a state over F2
// (matchedDistance, matches21): a candidate idx2 is skipped when the distance it is held at is <=
// its own, and an accepted query takes idx2 from its earlier holder.  Three stages:
//   pj_grid_kernel   F2's FeaturesGrid (as above; mp_begin = q_begin gives each query its pair)
//   pi_score_kernel  a 16-lane group per query: the octave-0 candidates of its window in
//                    GetFeaturesInArea's scan order with their Hamming distances, up to PI_CAP
//   pi_walk_kernel   one wavefront per pair: the queries in order, lanes over a query's candidates
//                    against the state in LDS (matchedDistance u16, matches21 / matches12 i16),
//                    best = min (dist, scan position), second = the second-smallest distance of the
//                    candidates not skipped; windows with more than PI_CAP candidates are rescanned
//                    from the grid.  Then CheckOrientation over every push (stale ones included),
//                    the output and the prevMatched update.
constexpr int PI_CAP = 128;
constexpr int PI_TH_LOW = 50;    // ORBmatcher.cc:42
constexpr int PI_INF = 0xffff;   // matchedDistance = INT_MAX on entry (:618)

struct PiExtra {
    const int32_t* q_begin;
    const int32_t* q_oct;
    const uint8_t* q_desc;
    const float* q_angle;
    const float* kp_angle;
    float* prev;
    float r, nnratio;
    int check_ori, total_q;
    int32_t* cnt;        // total_q: candidates in the query's window (0: not searched / none)
    uint32_t* cand;      // total_q x PI_CAP: (dist << 13 | idx2) in scan order
    int32_t* matches12;  // total_q
};

struct PiWin {
    int mincx, maxcx, mincy, maxcy, lvl;
    bool chk, any;
    float u, v, r;
};

// GetFeaturesInArea(u, v, windowSize, level1, level1) (Frame.cc:102-145) of query j (octave <= 0).
__device__ __forceinline__ PiWin pi_window(const PjArgs& a, const PiExtra& e, int f, int j) {
    PiWin w;
    w.lvl = e.q_oct[j];
    w.any = w.lvl <= 0;   // :628-630: level1 > 0 continue
    w.chk = w.lvl >= 0;   // checkLevels = minLevel > 0 || maxLevel >= 0
    w.u = e.prev[2 * (size_t)j];
    w.v = e.prev[2 * (size_t)j + 1];
    w.r = e.r;
    const float* bd = a.bounds + 4 * (size_t)f;
    const float minx = bd[0], miny = bd[2];
    const float invW = PJ_COLS / (bd[1] - bd[0]), invH = PJ_ROWS / (bd[3] - bd[2]);
    w.mincx = max((int)floorf(invW * (w.u - w.r - minx)), 0);
    w.maxcx = min((int)ceilf(invW * (w.u + w.r - minx)), PJ_COLS - 1);
    w.mincy = max((int)floorf(invH * (w.v - w.r - miny)), 0);
    w.maxcy = min((int)ceilf(invH * (w.v + w.r - miny)), PJ_ROWS - 1);
    if (w.mincx >= PJ_COLS || w.maxcx < 0 || w.mincy >= PJ_ROWS || w.maxcy < 0) w.any = false;
    return w;
}

// the level / area gates of a keypoint at sorted grid position p of frame f (-1: not a candidate)
__device__ __forceinline__ int pi_gate(const PjArgs& a, const PiWin& w, int k0, int p) {
    const int idx = a.grid_idx[k0 + p];
    const int k = k0 + idx;
    if (w.chk && a.kp_oct[k] != w.lvl) return -1;
    const float distx = a.kp_xy[2 * (size_t)k] - w.u, disty = a.kp_xy[2 * (size_t)k + 1] - w.v;
    return (fabsf(distx) < w.r && fabsf(disty) < w.r) ? idx : -1;
}

__global__ __launch_bounds__(256) void pi_score_kernel(PjArgs a, PiExtra e) {
    const int j = blockIdx.x * 16 + (threadIdx.x >> 4), lane = threadIdx.x & 15;
    if (j >= e.total_q) return;   // whole 16-lane groups
    const int f = a.mp_frame[j];
    const int k0 = a.kp_begin[f], n2 = a.kp_begin[f + 1] - k0;
    int cnt = 0;
    if (n2 <= PJ_MAXKP) {
        const PiWin w = pi_window(a, e, f, j);
        if (w.any) {
            const uint8_t* d1 = e.q_desc + 32 * (size_t)j;
            const int32_t* cs = a.grid_start + (size_t)f * (PJ_CELLS + 1);
            const int gsh = threadIdx.x & 48;   // this group's bit offset in the wave's ballot
            for (int cx = w.mincx; cx <= w.maxcx; cx++) {
                const int p0 = cs[cx * PJ_ROWS + w.mincy], p1 = cs[cx * PJ_ROWS + w.maxcy + 1];
                for (int b = p0; b < p1; b += 16) {
                    const int p = b + lane;
                    const int idx = p < p1 ? pi_gate(a, w, k0, p) : -1;
                    const unsigned long long bm = __ballot(idx >= 0);
                    const uint32_t gm = (uint32_t)(bm >> gsh) & 0xffffu;
                    if (idx >= 0) {
                        const int pos = cnt + __popc(gm & ((1u << lane) - 1u));
                        if (pos < PI_CAP) {
                            const int dist = pj_hamming(d1, a.kp_desc + 32 * (size_t)(k0 + idx));
                            e.cand[(size_t)j * PI_CAP + pos] = ((uint32_t)dist << PJ_IDX_BITS) | (uint32_t)idx;
                        }
                    }
                    cnt += __popc(gm);
                }
            }
        }
    }
    if (lane == 0) e.cnt[j] = cnt;
}

__device__ __forceinline__ unsigned long long pi_wave_min64(unsigned long long v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v, m, 64), hi = (unsigned)__shfl_xor((int)(v >> 32), m, 64);
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

__global__ __launch_bounds__(64) void pi_walk_kernel(PjArgs a, PiExtra e) {
    __shared__ uint16_t mdist[PJ_MAXKP];
    __shared__ int16_t m21[PJ_MAXKP];
    __shared__ int16_t m12[PJ_MAXKP];
    __shared__ int hist[32];
    __shared__ uint32_t keep_s;
    const int f = blockIdx.x, lane = threadIdx.x;
    const int k0 = a.kp_begin[f], n2 = a.kp_begin[f + 1] - k0;
    const int q0 = e.q_begin[f], n1 = e.q_begin[f + 1] - q0;
    if (n1 > PJ_MAXKP || n2 > PJ_MAXKP) {
        for (int i = lane; i < n1; i += 64) e.matches12[q0 + i] = -1;
        if (lane == 0) a.n_matches[f] = -1;
        return;
    }
    for (int i = lane; i < n2; i += 64) { mdist[i] = PI_INF; m21[i] = -1; }
    for (int i = lane; i < n1; i += 64) m12[i] = -1;
    if (lane < 32) hist[lane] = 0;
    __syncthreads();
    const int32_t* cs = a.grid_start + (size_t)f * (PJ_CELLS + 1);
    int nm = 0;
    for (int c = 0; c < n1; c += 64) {
        const int cnt_l = c + lane < n1 ? e.cnt[q0 + c + lane] : 0;
        unsigned long long todo = __ballot(cnt_l > 0);
        while (todo) {
            const int t = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int qi = c + t, j = q0 + qi;
            const int cnt = __shfl(cnt_l, t, 64);
            unsigned long long bkey = ~0ull;   // (dist << 32) | (scan position << 13) | idx2
            int d1 = PI_INF, d2 = PI_INF;      // the lane's two smallest distances not skipped
            auto consider = [&](int dist, int idx2, int pos) {
                if ((int)mdist[idx2] <= dist) return;   // matchedDistance[idx2] <= dist (:650-651)
                const unsigned long long key = ((unsigned long long)dist << 32) | ((unsigned)pos << PJ_IDX_BITS) | (unsigned)idx2;
                bkey = key < bkey ? key : bkey;
                if (dist < d1) { d2 = d1; d1 = dist; } else if (dist < d2) d2 = dist;
            };
            if (cnt <= PI_CAP) {
                for (int k = lane; k < cnt; k += 64) {
                    const uint32_t key = e.cand[(size_t)j * PI_CAP + k];
                    consider((int)(key >> PJ_IDX_BITS), (int)(key & PJ_IDX_MASK), k);
                }
            } else {   // a window with more than PI_CAP candidates: rescan it from the grid
                const PiWin w = pi_window(a, e, f, j);
                const uint8_t* d1p = e.q_desc + 32 * (size_t)j;
                for (int cx = w.mincx; cx <= w.maxcx; cx++) {
                    const int p0 = cs[cx * PJ_ROWS + w.mincy], p1 = cs[cx * PJ_ROWS + w.maxcy + 1];
                    for (int p = p0 + lane; p < p1; p += 64) {
                        const int idx = pi_gate(a, w, k0, p);
                        if (idx >= 0) consider(pj_hamming(d1p, a.kp_desc + 32 * (size_t)(k0 + idx)), idx, p);
                    }
                }
            }
            bkey = pi_wave_min64(bkey);
#pragma unroll
            for (int m = 32; m > 0; m >>= 1) {   // merge the lanes' two smallest: second order statistic
                const int o1 = __shfl_xor(d1, m, 64), o2 = __shfl_xor(d2, m, 64);
                d2 = min(max(d1, o1), min(d2, o2));
                d1 = min(d1, o1);
            }
            if (bkey == ~0ull) continue;
            const int best = (int)(bkey >> 32), b = (int)(bkey & PJ_IDX_MASK);
            // bestDist < secondBestDist * fNNRatio_ in float, INT_MAX when there is no second (:665)
            const float second = d2 >= PI_INF ? 2147483648.0f : (float)d2;
            if (best <= PI_TH_LOW && (float)best < second * e.nnratio) {
                if (lane == 0) {
                    const int old = m21[b];
                    if (old >= 0) { m12[old] = -1; nm--; }   // :667-671
                    m12[qi] = (int16_t)b;
                    m21[b] = (int16_t)qi;
                    mdist[b] = (uint16_t)best;
                    nm++;
                    if (e.check_ori) hist[pjm_bin(e.kp_angle[k0 + b], e.q_angle[j])]++;
                }
                __builtin_amdgcn_wave_barrier();
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
    }
    __syncthreads();
    if (e.check_ori) {   // CheckOrientation(frame2.keypointsUn, frame1.keypointsUn, matchIds, matches12)
        if (lane == 0) {
            QtItem it[30];
            for (int bb = 0; bb < 30; bb++) it[bb] = QtItem{hist[bb], bb};
            qt_sort(it, it + 30);
            const double max1 = it[0].size, max2 = it[1].size, max3 = it[2].size;
            const int eraseBin = max2 < 0.1 * max1 ? 1 : (max3 < 0.1 * max1 ? 2 : 3);
            uint32_t k = 0;
            int kept = 0;
            for (int r = 0; r < eraseBin; r++) {
                k |= 1u << it[r].node;
                kept += it[r].size;
            }
            keep_s = k;
            nm = kept;   // matchIds.size() - reduction
        }
        __syncthreads();
        const uint32_t k = keep_s;
        for (int i = lane; i < n1; i += 64) {
            const int m = m12[i];
            if (m >= 0 && !((k >> pjm_bin(e.kp_angle[k0 + m], e.q_angle[q0 + i])) & 1u)) m12[i] = -1;
        }
        __syncthreads();
    }
    for (int i = lane; i < n1; i += 64) {   // output and the prevMatched update (:686-688)
        const int m = m12[i];
        e.matches12[q0 + i] = m;
        if (m >= 0) {
            e.prev[2 * (size_t)(q0 + i)] = a.kp_xy[2 * (size_t)(k0 + m)];
            e.prev[2 * (size_t)(q0 + i) + 1] = a.kp_xy[2 * (size_t)(k0 + m) + 1];
        }
    }
    if (lane == 0) a.n_matches[f] = nm;
}

static int launch_init(PjArgs& a, PiExtra& e, hipStream_t st) {
    hipLaunchKernelGGL(pj_grid_kernel, dim3(a.n_frames), dim3(256), 0, st, a);
    ORB_HIP_TRY(hipGetLastError());
    if (e.total_q > 0) {
        hipLaunchKernelGGL(pi_score_kernel, dim3((e.total_q + 15) / 16), dim3(256), 0, st, a, e);
        ORB_HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(pi_walk_kernel, dim3(a.n_frames), dim3(64), 0, st, a, e);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

static size_t pi_workspace_bytes(int n_pairs, int total_kp, int total_q) {
    return pj_workspace_bytes(n_pairs, total_kp, total_q) + align_up((size_t)std::max(total_q, 1) * 4, 256) +
           align_up((size_t)std::max(total_q, 1) * PI_CAP * 4, 256);
}

static void pi_carve(PjArgs& a, PiExtra& e, char* ws, int n_pairs, int total_kp, int total_q) {
    pj_carve(a, ws, n_pairs, total_kp, total_q);
    size_t o = pj_workspace_bytes(n_pairs, total_kp, total_q);
    e.cnt = (int32_t*)(ws + o);
    o += align_up((size_t)std::max(total_q, 1) * 4, 256);
    e.cand = (uint32_t*)(ws + o);
}

static int pi_common(const orbm_init_batch* b, PjArgs& a, PiExtra& e) {
    ORB_CHECK_ARG(b, "null argument");
    ORB_CHECK_ARG(b->n_pairs >= 0 && b->total_kp >= 0 && b->total_q >= 0, "negative sizes");
    ORB_CHECK_ARG(b->window >= 0, "negative windowSize");
    std::memset(&a, 0, sizeof(a));
    std::memset(&e, 0, sizeof(e));
    a.n_frames = b->n_pairs;
    a.n_levels = 8;
    a.total_mp = b->total_q;
    e.r = (float)b->window;   // static_cast<float>(windowSize) (:622)
    e.nnratio = b->nnratio;
    e.check_ori = b->check_orientation ? 1 : 0;
    e.total_q = b->total_q;
    return ORB_OK;
}

// ---------------------------------------------------------------- SearchByProjection(Frame&, KeyFrame*, alreadyFound, th, ORBdist)
// (ORBmatcher.cc:1364-1445, Tracking::Relocalization).  reloc_project_kernel turns each keyframe point
// into the motion-model walk's inputs -- validity, projection (u, v) and predicted scale -- with the
// reference's float expressions; the walk then runs as pjm_* with the level window predictedScale +- 1
// (motion 0), no stereo gate, every accepted point claiming and ORBdist as the distance bound.
struct RelocExtra {
    const float* pose;      // n_frames x 12
    const float* camera;    // n_frames x 4
    const uint8_t* valid;   // caller's flag
    const float* xw;
    const float* max_min;
    float log_sf;
    uint8_t* out_valid;
    float* out_proj;        // total_mp x 3 (u, v, 0)
    int32_t* out_level;
};

__global__ __launch_bounds__(256) void reloc_project_kernel(PjArgs a, RelocExtra r) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= a.total_mp) return;
    const int f = a.mp_frame[j];
    bool ok = r.valid[j] != 0;
    float u = 0.f, v = 0.f;
    int ps = 0;
    if (ok) {
        const float* P = r.pose + 12 * (size_t)f;
        const float* K = r.camera + 4 * (size_t)f;
        const float X0 = r.xw[3 * (size_t)j], X1 = r.xw[3 * (size_t)j + 1], X2 = r.xw[3 * (size_t)j + 2];
        // Rcw * Xw + tcw (cv::Matx: s = 0; s += a(i, k) * b(k) for k = 0..2), then CameraToImage
        const float c0 = ((P[0] * X0 + P[1] * X1) + P[2] * X2) + P[9];
        const float c1 = ((P[3] * X0 + P[4] * X1) + P[5] * X2) + P[10];
        const float c2 = ((P[6] * X0 + P[7] * X1) + P[8] * X2) + P[11];
        const float invZ = 1.f / c2;
        u = invZ * K[0] * c0 + K[2];
        v = invZ * K[1] * c1 + K[3];
        const float* bd = a.bounds + 4 * (size_t)f;
        ok = u >= bd[0] && u < bd[1] && v >= bd[2] && v < bd[3];   // ImageBounds::Contains (Frame.cc:51-54)
        if (ok) {
            // Ow = -Rcw^T * tcw (CameraPose::Invt), PO = Xw - Ow, dist3D = (float)cv::norm(PO) (double sum)
            const float o0 = -((P[0] * P[9] + P[3] * P[10]) + P[6] * P[11]);
            const float o1 = -((P[1] * P[9] + P[4] * P[10]) + P[7] * P[11]);
            const float o2 = -((P[2] * P[9] + P[5] * P[10]) + P[8] * P[11]);
            const double d0 = (double)(X0 - o0), d1 = (double)(X1 - o1), d2 = (double)(X2 - o2);
            const float dist3D = (float)sqrt((d0 * d0 + d1 * d1) + d2 * d2);
            const float maxD = r.max_min[2 * (size_t)j], minD = r.max_min[2 * (size_t)j + 1];
            ok = !(dist3D < 0.8f * minD || dist3D > 1.2f * maxD);   // :1399-1401
            if (ok) {   // PredictScale(dist3D, &frame) (MapPoint.cc:405-415)
                const float ratio = maxD / dist3D;
                const int sc = (int)ceil(log((double)ratio) / (double)r.log_sf);
                ps = max(0, min(sc, a.n_levels - 1));
            }
        }
    }
    r.out_valid[j] = ok ? 1 : 0;
    r.out_proj[3 * (size_t)j] = u;
    r.out_proj[3 * (size_t)j + 1] = v;
    r.out_proj[3 * (size_t)j + 2] = 0.f;
    r.out_level[j] = ps;
}

static size_t reloc_workspace_bytes(int n_frames, int total_kp, int total_mp) {
    const size_t M = (size_t)std::max(total_mp, 1);
    return pj_workspace_bytes(n_frames, total_kp, total_mp) + align_up(M * 4, 256) + align_up(M, 256) +
           align_up(M * 12, 256) + align_up(M * 4, 256);
}

static int launch_reloc(PjArgs& a, RelocExtra& r, PjmExtra& e, char* ws, int total_kp, int check_ori, hipStream_t st) {
    pj_carve(a, ws, a.n_frames, total_kp, a.total_mp);
    size_t o = pj_workspace_bytes(a.n_frames, total_kp, a.total_mp);
    const size_t M = (size_t)std::max(a.total_mp, 1);
    e.choice = (int32_t*)(ws + o);
    o += align_up(M * 4, 256);
    r.out_valid = (uint8_t*)(ws + o);
    o += align_up(M, 256);
    r.out_proj = (float*)(ws + o);
    o += align_up(M * 12, 256);
    r.out_level = (int32_t*)(ws + o);
    hipLaunchKernelGGL(pj_grid_kernel, dim3(a.n_frames), dim3(256), 0, st, a);
    ORB_HIP_TRY(hipGetLastError());
    a.mp_valid = r.out_valid;
    a.mp_proj = r.out_proj;
    a.mp_level = r.out_level;
    if (a.total_mp > 0) {
        hipLaunchKernelGGL(reloc_project_kernel, dim3((a.total_mp + 255) / 256), dim3(256), 0, st, a, r);
        ORB_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(pjm_score_kernel, dim3((a.total_mp + 256 / PJ_GW - 1) / (256 / PJ_GW)), dim3(256), 0, st, a, e);
        ORB_HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(pjm_walk_kernel, dim3(a.n_frames), dim3(64), 0, st, a, e);
    ORB_HIP_TRY(hipGetLastError());
    if (check_ori) {
        hipLaunchKernelGGL(pjm_orient_kernel, dim3(a.n_frames), dim3(256), 0, st, a, e);
        ORB_HIP_TRY(hipGetLastError());
    }
    return ORB_OK;
}

static int reloc_common(const orbm_reloc_batch* b, PjArgs& a, RelocExtra& r, PjmExtra& e) {
    ORB_CHECK_ARG(b, "null argument");
    ORB_CHECK_ARG(b->n_frames >= 0 && b->total_kp >= 0 && b->total_mp >= 0, "negative sizes");
    ORB_CHECK_ARG(b->n_levels >= 1 && b->n_levels <= PJ_MAX_LEVELS && b->scale_factors, "bad scale pyramid");
    ORB_CHECK_ARG(b->orb_dist >= 0 && b->orb_dist < 256, "ORBdist must be in [0, 256)");
    std::memset(&a, 0, sizeof(a));
    std::memset(&r, 0, sizeof(r));
    std::memset(&e, 0, sizeof(e));
    a.n_frames = b->n_frames;
    a.n_levels = b->n_levels;
    for (int l = 0; l < b->n_levels; l++) a.scale[l] = b->scale_factors[l];
    a.th = b->th;
    a.total_mp = b->total_mp;
    r.log_sf = b->log_scale_factor;
    e.max_dist = b->orb_dist;
    return ORB_OK;
}

}  // namespace orbamd

using namespace orbamd;

extern "C" int orbm_search_by_projection_device(const orbm_proj_batch* b, int32_t* kp_match, int32_t* n_matches,
                                                void* stream) {
    PjArgs a;
    int rc;
    if ((rc = pj_common_args(b, a))) return rc;
    if (b->n_frames == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->mp_begin && b->bounds && kp_match && n_matches, "null array");
    ORB_CHECK_ARG(b->total_kp == 0 || (b->kp_xy && b->kp_octave && b->kp_uright && b->kp_desc), "null keypoint array");
    ORB_CHECK_ARG(b->total_mp == 0 || (b->mp_valid && b->mp_proj && b->mp_view_cos && b->mp_level && b->mp_desc &&
                                       b->mp_has_obs),
                  "null map point array");
    a.kp_begin = b->kp_begin; a.kp_xy = b->kp_xy; a.kp_oct = b->kp_octave; a.kp_ur = b->kp_uright;
    a.kp_desc = b->kp_desc; a.kp_claimed = b->kp_claimed; a.bounds = b->bounds;
    a.mp_begin = b->mp_begin; a.mp_valid = b->mp_valid; a.mp_proj = b->mp_proj; a.mp_vcos = b->mp_view_cos;
    a.mp_level = b->mp_level; a.mp_desc = b->mp_desc; a.mp_has_obs = b->mp_has_obs;
    a.kp_match = kp_match;
    a.n_matches = n_matches;
    int dev = 0;
    ORB_HIP_TRY(hipGetDevice(&dev));
    if (g_pj.device != dev) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = dev;
    }
    if ((rc = g_pj.ws.reserve(pj_workspace_bytes(b->n_frames, b->total_kp, b->total_mp)))) return rc;
    pj_carve(a, g_pj.ws.as<char>(), b->n_frames, b->total_kp, b->total_mp);
    return launch_projection(a, b->total_kp, (hipStream_t)stream);
}

extern "C" int orbm_search_by_projection(const orbm_proj_batch* b, int32_t* kp_match, int32_t* n_matches,
                                         int device) {
    PjArgs a;
    int rc;
    if ((rc = pj_common_args(b, a))) return rc;
    const int F = b->n_frames;
    if (F == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->mp_begin && b->bounds && kp_match && n_matches, "null array");
    ORB_CHECK_ARG(b->kp_begin[0] == 0 && b->mp_begin[0] == 0 && b->kp_begin[F] == b->total_kp &&
                      b->mp_begin[F] == b->total_mp,
                  "kp_begin / mp_begin must start at 0 and end at total_kp / total_mp");
    for (int f = 0; f < F; f++) {
        ORB_CHECK_ARG(b->kp_begin[f + 1] >= b->kp_begin[f] && b->mp_begin[f + 1] >= b->mp_begin[f],
                      "offsets must be non-decreasing");
        ORB_CHECK_ARG(b->kp_begin[f + 1] - b->kp_begin[f] <= PJ_MAXKP, "frame has more than ORBM_PROJ_MAX_KP keypoints");
    }
    const int K = b->total_kp, M = b->total_mp;
    ORB_CHECK_ARG(K == 0 || (b->kp_xy && b->kp_octave && b->kp_uright && b->kp_desc), "null keypoint array");
    ORB_CHECK_ARG(M == 0 || (b->mp_valid && b->mp_proj && b->mp_view_cos && b->mp_level && b->mp_desc &&
                             b->mp_has_obs),
                  "null map point array");
    for (int j = 0; j < M; j++)
        ORB_CHECK_ARG(!b->mp_valid[j] || (b->mp_level[j] >= 0 && b->mp_level[j] < b->n_levels),
                      "trackScaleLevel out of range (scaleFactors[predictedScale], ORBmatcher.cc:328)");
    ORB_HIP_TRY(hipSetDevice(device));
    if (g_pj.device != device) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = device;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += align_up(std::max<size_t>(bytes, 1), 256); return o; };
    const size_t o_kb = take((size_t)(F + 1) * 4), o_xy = take((size_t)K * 8), o_oc = take((size_t)K * 4),
                 o_ur = take((size_t)K * 4), o_kd = take((size_t)K * 32), o_kc = take(b->kp_claimed ? (size_t)K : 0),
                 o_bd = take((size_t)F * 16), o_mb = take((size_t)(F + 1) * 4), o_mv = take((size_t)M),
                 o_mp = take((size_t)M * 12), o_vc = take((size_t)M * 4), o_ml = take((size_t)M * 4),
                 o_md = take((size_t)M * 32), o_mo = take((size_t)M), o_km = take((size_t)K * 4),
                 o_nm = take((size_t)F * 4);
    if ((rc = g_pj.io.reserve(off))) return rc;
    if ((rc = g_pj.ws.reserve(pj_workspace_bytes(F, K, M)))) return rc;
    char* d = g_pj.io.as<char>();
    auto up = [&](size_t o, const void* src, size_t bytes) -> int {
        if (bytes) ORB_HIP_TRY(hipMemcpy(d + o, src, bytes, hipMemcpyHostToDevice));
        return ORB_OK;
    };
    if ((rc = up(o_kb, b->kp_begin, (size_t)(F + 1) * 4)) || (rc = up(o_xy, b->kp_xy, (size_t)K * 8)) ||
        (rc = up(o_oc, b->kp_octave, (size_t)K * 4)) || (rc = up(o_ur, b->kp_uright, (size_t)K * 4)) ||
        (rc = up(o_kd, b->kp_desc, (size_t)K * 32)) ||
        (b->kp_claimed && (rc = up(o_kc, b->kp_claimed, (size_t)K))) || (rc = up(o_bd, b->bounds, (size_t)F * 16)) ||
        (rc = up(o_mb, b->mp_begin, (size_t)(F + 1) * 4)) || (rc = up(o_mv, b->mp_valid, (size_t)M)) ||
        (rc = up(o_mp, b->mp_proj, (size_t)M * 12)) || (rc = up(o_vc, b->mp_view_cos, (size_t)M * 4)) ||
        (rc = up(o_ml, b->mp_level, (size_t)M * 4)) || (rc = up(o_md, b->mp_desc, (size_t)M * 32)) ||
        (rc = up(o_mo, b->mp_has_obs, (size_t)M)))
        return rc;
    a.kp_begin = (const int32_t*)(d + o_kb); a.kp_xy = (const float*)(d + o_xy); a.kp_oct = (const int32_t*)(d + o_oc);
    a.kp_ur = (const float*)(d + o_ur); a.kp_desc = (const uint8_t*)(d + o_kd);
    a.kp_claimed = b->kp_claimed ? (const uint8_t*)(d + o_kc) : nullptr; a.bounds = (const float*)(d + o_bd);
    a.mp_begin = (const int32_t*)(d + o_mb); a.mp_valid = (const uint8_t*)(d + o_mv);
    a.mp_proj = (const float*)(d + o_mp); a.mp_vcos = (const float*)(d + o_vc); a.mp_level = (const int32_t*)(d + o_ml);
    a.mp_desc = (const uint8_t*)(d + o_md); a.mp_has_obs = (const uint8_t*)(d + o_mo);
    a.kp_match = (int32_t*)(d + o_km);
    a.n_matches = (int32_t*)(d + o_nm);
    pj_carve(a, g_pj.ws.as<char>(), F, K, M);
    if ((rc = launch_projection(a, K, nullptr))) return rc;
    if (K) ORB_HIP_TRY(hipMemcpy(kp_match, d + o_km, (size_t)K * 4, hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(n_matches, d + o_nm, (size_t)F * 4, hipMemcpyDeviceToHost));
    return ORB_OK;
}

extern "C" int orbm_search_by_projection_motion_device(const orbm_motion_batch* b, int32_t* kp_match,
                                                       int32_t* n_matches, void* stream) {
    ORB_CHECK_ARG(b, "null argument");
    ORB_CHECK_ARG(b->n_frames >= 0 && b->total_kp >= 0 && b->total_mp >= 0, "negative sizes");
    ORB_CHECK_ARG(b->n_levels >= 1 && b->n_levels <= PJ_MAX_LEVELS && b->scale_factors, "bad scale pyramid");
    if (b->n_frames == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->mp_begin && b->bounds && kp_match && n_matches, "null array");
    ORB_CHECK_ARG(b->total_kp == 0 || (b->kp_xy && b->kp_octave && b->kp_uright && b->kp_desc), "null keypoint array");
    ORB_CHECK_ARG(b->total_mp == 0 || (b->mp_valid && b->mp_proj && b->mp_octave && b->mp_desc && b->mp_has_obs),
                  "null last-frame point array");
    ORB_CHECK_ARG(!b->check_orientation || (b->kp_angle && (b->total_mp == 0 || b->mp_angle)),
                  "CheckOrientation needs kp_angle / mp_angle");
    PjArgs a;
    std::memset(&a, 0, sizeof(a));
    a.n_frames = b->n_frames;
    a.n_levels = b->n_levels;
    for (int l = 0; l < b->n_levels; l++) a.scale[l] = b->scale_factors[l];
    a.th = b->th;
    a.total_mp = b->total_mp;
    a.kp_begin = b->kp_begin; a.kp_xy = b->kp_xy; a.kp_oct = b->kp_octave; a.kp_ur = b->kp_uright;
    a.kp_desc = b->kp_desc; a.kp_claimed = b->kp_claimed; a.bounds = b->bounds;
    a.mp_begin = b->mp_begin; a.mp_valid = b->mp_valid; a.mp_proj = b->mp_proj; a.mp_level = b->mp_octave;
    a.mp_desc = b->mp_desc; a.mp_has_obs = b->mp_has_obs;
    a.kp_match = kp_match;
    a.n_matches = n_matches;
    int dev = 0, rc;
    ORB_HIP_TRY(hipGetDevice(&dev));
    if (g_pj.device != dev) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = dev;
    }
    const size_t base = pj_workspace_bytes(b->n_frames, b->total_kp, b->total_mp);
    if ((rc = g_pj.ws.reserve(base + align_up((size_t)std::max(b->total_mp, 1) * 4, 256)))) return rc;
    pj_carve(a, g_pj.ws.as<char>(), b->n_frames, b->total_kp, b->total_mp);
    PjmExtra e{b->motion, b->kp_angle, b->mp_angle, reinterpret_cast<int32_t*>(g_pj.ws.as<char>() + base), PJ_TH_HIGH};
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(pj_grid_kernel, dim3(a.n_frames), dim3(256), 0, st, a);
    ORB_HIP_TRY(hipGetLastError());
    if (a.total_mp > 0) {
        hipLaunchKernelGGL(pjm_score_kernel, dim3((a.total_mp + 256 / PJ_GW - 1) / (256 / PJ_GW)), dim3(256), 0, st, a, e);
        ORB_HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(pjm_walk_kernel, dim3(a.n_frames), dim3(64), 0, st, a, e);
    ORB_HIP_TRY(hipGetLastError());
    if (b->check_orientation) {
        hipLaunchKernelGGL(pjm_orient_kernel, dim3(a.n_frames), dim3(256), 0, st, a, e);
        ORB_HIP_TRY(hipGetLastError());
    }
    return ORB_OK;
}


extern "C" int orbm_search_for_initialization_device(const orbm_init_batch* b, int32_t* matches12, int32_t* n_matches,
                                                     void* stream) {
    PjArgs a;
    PiExtra e;
    int rc;
    if ((rc = pi_common(b, a, e))) return rc;
    if (b->n_pairs == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->q_begin && b->bounds && b->prev_matched && matches12 && n_matches, "null array");
    ORB_CHECK_ARG(b->total_kp == 0 || (b->kp_xy && b->kp_octave && b->kp_desc), "null F2 keypoint array");
    ORB_CHECK_ARG(b->total_q == 0 || (b->q_octave && b->q_desc), "null F1 keypoint array");
    ORB_CHECK_ARG(!b->check_orientation || ((b->total_kp == 0 || b->kp_angle) && (b->total_q == 0 || b->q_angle)),
                  "CheckOrientation needs kp_angle / q_angle");
    a.kp_begin = b->kp_begin; a.kp_xy = b->kp_xy; a.kp_oct = b->kp_octave; a.kp_desc = b->kp_desc;
    a.bounds = b->bounds; a.mp_begin = b->q_begin; a.n_matches = n_matches;
    e.q_begin = b->q_begin; e.q_oct = b->q_octave; e.q_desc = b->q_desc; e.q_angle = b->q_angle;
    e.kp_angle = b->kp_angle; e.prev = b->prev_matched; e.matches12 = matches12;
    int dev = 0;
    ORB_HIP_TRY(hipGetDevice(&dev));
    if (g_pj.device != dev) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = dev;
    }
    if ((rc = g_pj.ws.reserve(pi_workspace_bytes(b->n_pairs, b->total_kp, b->total_q)))) return rc;
    pi_carve(a, e, g_pj.ws.as<char>(), b->n_pairs, b->total_kp, b->total_q);
    return launch_init(a, e, (hipStream_t)stream);
}

extern "C" int orbm_search_for_initialization(const orbm_init_batch* b, int32_t* matches12, int32_t* n_matches,
                                              int device) {
    PjArgs a;
    PiExtra e;
    int rc;
    if ((rc = pi_common(b, a, e))) return rc;
    const int P = b->n_pairs;
    if (P == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->q_begin && b->bounds && b->prev_matched && matches12 && n_matches, "null array");
    ORB_CHECK_ARG(b->kp_begin[0] == 0 && b->q_begin[0] == 0 && b->kp_begin[P] == b->total_kp &&
                      b->q_begin[P] == b->total_q,
                  "kp_begin / q_begin must start at 0 and end at total_kp / total_q");
    for (int p = 0; p < P; p++) {
        ORB_CHECK_ARG(b->kp_begin[p + 1] >= b->kp_begin[p] && b->q_begin[p + 1] >= b->q_begin[p],
                      "offsets must be non-decreasing");
        ORB_CHECK_ARG(b->kp_begin[p + 1] - b->kp_begin[p] <= PJ_MAXKP && b->q_begin[p + 1] - b->q_begin[p] <= PJ_MAXKP,
                      "frame has more than ORBM_PROJ_MAX_KP keypoints");
    }
    const int K = b->total_kp, Q = b->total_q;
    ORB_CHECK_ARG(K == 0 || (b->kp_xy && b->kp_octave && b->kp_desc), "null F2 keypoint array");
    ORB_CHECK_ARG(Q == 0 || (b->q_octave && b->q_desc), "null F1 keypoint array");
    ORB_CHECK_ARG(!b->check_orientation || ((K == 0 || b->kp_angle) && (Q == 0 || b->q_angle)),
                  "CheckOrientation needs kp_angle / q_angle");
    if (b->check_orientation) {
        for (int k = 0; k < K; k++)
            ORB_CHECK_ARG(b->kp_angle[k] >= 0.f && b->kp_angle[k] < 360.f, "keypoint angle outside [0, 360) (CV_Assert in CheckOrientation)");
        for (int q = 0; q < Q; q++)
            ORB_CHECK_ARG(b->q_angle[q] >= 0.f && b->q_angle[q] < 360.f, "keypoint angle outside [0, 360) (CV_Assert in CheckOrientation)");
    }
    ORB_HIP_TRY(hipSetDevice(device));
    if (g_pj.device != device) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = device;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += align_up(std::max<size_t>(bytes, 1), 256); return o; };
    const size_t o_kb = take((size_t)(P + 1) * 4), o_xy = take((size_t)K * 8), o_oc = take((size_t)K * 4),
                 o_kd = take((size_t)K * 32), o_ka = take((size_t)K * 4), o_bd = take((size_t)P * 16),
                 o_qb = take((size_t)(P + 1) * 4), o_qo = take((size_t)Q * 4), o_qd = take((size_t)Q * 32),
                 o_qa = take((size_t)Q * 4), o_pm = take((size_t)Q * 8), o_m12 = take((size_t)Q * 4),
                 o_nm = take((size_t)P * 4);
    if ((rc = g_pj.io.reserve(off))) return rc;
    if ((rc = g_pj.ws.reserve(pi_workspace_bytes(P, K, Q)))) return rc;
    char* d = g_pj.io.as<char>();
    auto up = [&](size_t o, const void* src, size_t bytes) -> int {
        if (bytes && src) ORB_HIP_TRY(hipMemcpy(d + o, src, bytes, hipMemcpyHostToDevice));
        return ORB_OK;
    };
    if ((rc = up(o_kb, b->kp_begin, (size_t)(P + 1) * 4)) || (rc = up(o_xy, b->kp_xy, (size_t)K * 8)) ||
        (rc = up(o_oc, b->kp_octave, (size_t)K * 4)) || (rc = up(o_kd, b->kp_desc, (size_t)K * 32)) ||
        (rc = up(o_ka, b->kp_angle, (size_t)K * 4)) || (rc = up(o_bd, b->bounds, (size_t)P * 16)) ||
        (rc = up(o_qb, b->q_begin, (size_t)(P + 1) * 4)) || (rc = up(o_qo, b->q_octave, (size_t)Q * 4)) ||
        (rc = up(o_qd, b->q_desc, (size_t)Q * 32)) || (rc = up(o_qa, b->q_angle, (size_t)Q * 4)) ||
        (rc = up(o_pm, b->prev_matched, (size_t)Q * 8)))
        return rc;
    a.kp_begin = (const int32_t*)(d + o_kb); a.kp_xy = (const float*)(d + o_xy); a.kp_oct = (const int32_t*)(d + o_oc);
    a.kp_desc = (const uint8_t*)(d + o_kd); a.bounds = (const float*)(d + o_bd); a.mp_begin = (const int32_t*)(d + o_qb);
    a.n_matches = (int32_t*)(d + o_nm);
    e.q_begin = (const int32_t*)(d + o_qb); e.q_oct = (const int32_t*)(d + o_qo); e.q_desc = (const uint8_t*)(d + o_qd);
    e.q_angle = (const float*)(d + o_qa); e.kp_angle = (const float*)(d + o_ka); e.prev = (float*)(d + o_pm);
    e.matches12 = (int32_t*)(d + o_m12);
    pi_carve(a, e, g_pj.ws.as<char>(), P, K, Q);
    if ((rc = launch_init(a, e, nullptr))) return rc;
    if (Q) {
        ORB_HIP_TRY(hipMemcpy(matches12, d + o_m12, (size_t)Q * 4, hipMemcpyDeviceToHost));
        ORB_HIP_TRY(hipMemcpy(b->prev_matched, d + o_pm, (size_t)Q * 8, hipMemcpyDeviceToHost));
    }
    ORB_HIP_TRY(hipMemcpy(n_matches, d + o_nm, (size_t)P * 4, hipMemcpyDeviceToHost));
    return ORB_OK;
}


extern "C" int orbm_search_by_projection_reloc_device(const orbm_reloc_batch* b, int32_t* kp_match, int32_t* n_matches,
                                                      void* stream) {
    PjArgs a;
    RelocExtra r;
    PjmExtra e;
    int rc;
    if ((rc = reloc_common(b, a, r, e))) return rc;
    if (b->n_frames == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->mp_begin && b->bounds && b->pose && b->camera && kp_match && n_matches, "null array");
    ORB_CHECK_ARG(b->total_kp == 0 || (b->kp_xy && b->kp_octave && b->kp_desc), "null keypoint array");
    ORB_CHECK_ARG(b->total_mp == 0 || (b->mp_valid && b->mp_xw && b->mp_max_min && b->mp_desc), "null keyframe point array");
    ORB_CHECK_ARG(!b->check_orientation || (b->kp_angle && (b->total_mp == 0 || b->mp_angle)),
                  "CheckOrientation needs kp_angle / mp_angle");
    a.kp_begin = b->kp_begin; a.kp_xy = b->kp_xy; a.kp_oct = b->kp_octave; a.kp_ur = nullptr;
    a.kp_desc = b->kp_desc; a.kp_claimed = b->kp_claimed; a.bounds = b->bounds;
    a.mp_begin = b->mp_begin; a.mp_desc = b->mp_desc; a.mp_has_obs = nullptr;
    a.kp_match = kp_match;
    a.n_matches = n_matches;
    r.pose = b->pose; r.camera = b->camera; r.valid = b->mp_valid; r.xw = b->mp_xw; r.max_min = b->mp_max_min;
    e.kp_angle = b->kp_angle; e.mp_angle = b->mp_angle;
    int dev = 0;
    ORB_HIP_TRY(hipGetDevice(&dev));
    if (g_pj.device != dev) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = dev;
    }
    if ((rc = g_pj.ws.reserve(reloc_workspace_bytes(b->n_frames, b->total_kp, b->total_mp)))) return rc;
    return launch_reloc(a, r, e, g_pj.ws.as<char>(), b->total_kp, b->check_orientation, (hipStream_t)stream);
}

extern "C" int orbm_search_by_projection_reloc(const orbm_reloc_batch* b, int32_t* kp_match, int32_t* n_matches,
                                               int device) {
    PjArgs a;
    RelocExtra r;
    PjmExtra e;
    int rc;
    if ((rc = reloc_common(b, a, r, e))) return rc;
    const int F = b->n_frames;
    if (F == 0) return ORB_OK;
    ORB_CHECK_ARG(b->kp_begin && b->mp_begin && b->bounds && b->pose && b->camera && kp_match && n_matches, "null array");
    ORB_CHECK_ARG(b->kp_begin[0] == 0 && b->mp_begin[0] == 0 && b->kp_begin[F] == b->total_kp &&
                      b->mp_begin[F] == b->total_mp,
                  "kp_begin / mp_begin must start at 0 and end at total_kp / total_mp");
    for (int f = 0; f < F; f++) {
        ORB_CHECK_ARG(b->kp_begin[f + 1] >= b->kp_begin[f] && b->mp_begin[f + 1] >= b->mp_begin[f],
                      "offsets must be non-decreasing");
        ORB_CHECK_ARG(b->kp_begin[f + 1] - b->kp_begin[f] <= PJ_MAXKP, "frame has more than ORBM_PROJ_MAX_KP keypoints");
    }
    const int K = b->total_kp, M = b->total_mp;
    ORB_CHECK_ARG(K == 0 || (b->kp_xy && b->kp_octave && b->kp_desc), "null keypoint array");
    ORB_CHECK_ARG(M == 0 || (b->mp_valid && b->mp_xw && b->mp_max_min && b->mp_desc), "null keyframe point array");
    ORB_CHECK_ARG(!b->check_orientation || (b->kp_angle && (M == 0 || b->mp_angle)),
                  "CheckOrientation needs kp_angle / mp_angle");
    ORB_HIP_TRY(hipSetDevice(device));
    if (g_pj.device != device) {
        g_pj.ws.release();
        g_pj.io.release();
        g_pj.device = device;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += align_up(std::max<size_t>(bytes, 1), 256); return o; };
    const size_t o_kb = take((size_t)(F + 1) * 4), o_xy = take((size_t)K * 8), o_oc = take((size_t)K * 4),
                 o_kd = take((size_t)K * 32), o_ka = take((size_t)K * 4), o_kc = take(b->kp_claimed ? (size_t)K : 0),
                 o_bd = take((size_t)F * 16), o_po = take((size_t)F * 48), o_ca = take((size_t)F * 16),
                 o_mb = take((size_t)(F + 1) * 4), o_mv = take((size_t)M), o_mx = take((size_t)M * 12),
                 o_mm = take((size_t)M * 8), o_md = take((size_t)M * 32), o_ma = take((size_t)M * 4),
                 o_km = take((size_t)K * 4), o_nm = take((size_t)F * 4);
    if ((rc = g_pj.io.reserve(off))) return rc;
    if ((rc = g_pj.ws.reserve(reloc_workspace_bytes(F, K, M)))) return rc;
    char* d = g_pj.io.as<char>();
    auto up = [&](size_t o, const void* src, size_t bytes) -> int {
        if (bytes && src) ORB_HIP_TRY(hipMemcpy(d + o, src, bytes, hipMemcpyHostToDevice));
        return ORB_OK;
    };
    if ((rc = up(o_kb, b->kp_begin, (size_t)(F + 1) * 4)) || (rc = up(o_xy, b->kp_xy, (size_t)K * 8)) ||
        (rc = up(o_oc, b->kp_octave, (size_t)K * 4)) || (rc = up(o_kd, b->kp_desc, (size_t)K * 32)) ||
        (rc = up(o_ka, b->kp_angle, (size_t)K * 4)) || (rc = up(o_kc, b->kp_claimed, (size_t)K)) ||
        (rc = up(o_bd, b->bounds, (size_t)F * 16)) || (rc = up(o_po, b->pose, (size_t)F * 48)) ||
        (rc = up(o_ca, b->camera, (size_t)F * 16)) || (rc = up(o_mb, b->mp_begin, (size_t)(F + 1) * 4)) ||
        (rc = up(o_mv, b->mp_valid, (size_t)M)) || (rc = up(o_mx, b->mp_xw, (size_t)M * 12)) ||
        (rc = up(o_mm, b->mp_max_min, (size_t)M * 8)) || (rc = up(o_md, b->mp_desc, (size_t)M * 32)) ||
        (rc = up(o_ma, b->mp_angle, (size_t)M * 4)))
        return rc;
    a.kp_begin = (const int32_t*)(d + o_kb); a.kp_xy = (const float*)(d + o_xy); a.kp_oct = (const int32_t*)(d + o_oc);
    a.kp_desc = (const uint8_t*)(d + o_kd); a.kp_claimed = b->kp_claimed ? (const uint8_t*)(d + o_kc) : nullptr;
    a.kp_ur = nullptr; a.bounds = (const float*)(d + o_bd); a.mp_begin = (const int32_t*)(d + o_mb);
    a.mp_desc = (const uint8_t*)(d + o_md); a.mp_has_obs = nullptr;
    a.kp_match = (int32_t*)(d + o_km); a.n_matches = (int32_t*)(d + o_nm);
    r.pose = (const float*)(d + o_po); r.camera = (const float*)(d + o_ca); r.valid = (const uint8_t*)(d + o_mv);
    r.xw = (const float*)(d + o_mx); r.max_min = (const float*)(d + o_mm);
    e.kp_angle = b->kp_angle ? (const float*)(d + o_ka) : nullptr;
    e.mp_angle = b->mp_angle ? (const float*)(d + o_ma) : nullptr;
    if ((rc = launch_reloc(a, r, e, g_pj.ws.as<char>(), K, b->check_orientation, nullptr))) return rc;
    if (K) ORB_HIP_TRY(hipMemcpy(kp_match, d + o_km, (size_t)K * 4, hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(n_matches, d + o_nm, (size_t)F * 4, hipMemcpyDeviceToHost));
    return ORB_OK;
}
