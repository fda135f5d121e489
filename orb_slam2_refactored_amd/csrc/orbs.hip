// orbs.hip — ComputeStereoMatches for gfx950 (src/ORBmatcher.cc:72-247,
// PatchDistance :60-68).
//
//  * stereo_match_kernel: one wavefront per left keypoint.  Lanes scan the right keypoints for the
//    row band (the reference's row table: rows floor(y - 2 s_o) .. ceil(y + 2 s_o) of each right
//    keypoint), octave +-1 and disparity window; the first minimum Hamming distance below TH_HIGH
//    is a min-reduction of (distance << 16 | index) keys (lowest index on ties = the ascending
//    row-list scan).  Below (TH_HIGH + TH_LOW) / 2 the 11x11 patch and the 11x21 right window are
//    staged in LDS and the 11 SAD sums (11 rows each) are computed lane-parallel, then the
//    first-minimum shift, parabola refinement and disparity checks run on one lane with the
//    reference's float expression order (-ffp-contract=off).
//  * stereo_filter_kernel: one workgroup per frame: the median of the matched SAD distances
//    (position max(n/2-1, 0) of the descending order) and the 1.5*1.4*median cut (:229-246).
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"
#include "stereo.h"

namespace orbamd {

constexpr int ST_TH_HIGH = 100, ST_TH_LOW = 50, ST_PR = 5, ST_PS = 11, ST_SR = 5;
constexpr int ST_WW = ST_PS + 2 * ST_SR;   // right window width (21)

__device__ __forceinline__ const uint8_t* st_level(const StereoSide& s, int f, int l, int* step) {
    if (l == 0) {
        *step = s.step0;
        return s.lvl0 + (long long)f * s.fstride0;
    }
    *step = s.stride[l];
    return s.pyr + (long long)f * s.pyr_frame + s.off[l];
}

__device__ __forceinline__ int st_hamming(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ void st_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Row table of the right keypoints (ComputeStereoMatches :84-97): keypoint j is listed on every row
// floor(y - r) .. ceil(y + r), r = 2 scale[octave] (clamped to the image; the reference's
// vRowIndices).  One workgroup per frame: LDS counts, an exclusive scan, then the entries.
constexpr int ST_MAX_ROWS = 4096;
__global__ __launch_bounds__(256) void stereo_rows_kernel(StereoSide L, StereoParams sp,
                                                          const orbx_keypoint* __restrict__ kpsR,
                                                          const int32_t* __restrict__ cntR, int nRf, int cap,
                                                          int32_t* __restrict__ roff, int32_t* __restrict__ rlist,
                                                          int span) {
    __shared__ int s_cnt[ST_MAX_ROWS + 1];
    __shared__ int s_part[256];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int nR = cntR ? cntR[f] : nRf;
    const int rows = L.rows[0];
    for (int y = tid; y <= rows; y += 256) s_cnt[y] = 0;
    __syncthreads();
    auto band = [&](int j, int& y0, int& y1) {
        const orbx_keypoint kR = kpsR[(long long)f * cap + j];
        const float r = 2.f * sp.scale[kR.octave];
        y0 = max((int)floorf(kR.y - r), 0);
        y1 = min((int)ceilf(kR.y + r), rows - 1);
    };
    for (int j = tid; j < nR; j += 256) {
        int y0, y1;
        band(j, y0, y1);
        for (int y = y0; y <= y1; y++) atomicAdd(&s_cnt[y], 1);
    }
    __syncthreads();
    // exclusive scan of s_cnt[0..rows): contiguous chunks per thread, then a scan of the chunk sums
    const int per = (rows + 255) / 256, c0 = min(tid * per, rows), c1 = min(c0 + per, rows);
    int sum = 0;
    for (int y = c0; y < c1; y++) sum += s_cnt[y];
    s_part[tid] = sum;
    __syncthreads();
    if (tid < 64) {   // 4 chunk sums per lane, a 64-lane inclusive scan of their totals
        int v[4], acc = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) { v[q] = s_part[4 * tid + q]; acc += v[q]; }
        int inc = acc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(inc, d, 64);
            if (tid >= d) inc += o;
        }
        int run = inc - acc;
#pragma unroll
        for (int q = 0; q < 4; q++) { s_part[4 * tid + q] = run; run += v[q]; }
    }
    __syncthreads();
    int run = s_part[tid];
    int32_t* ro = roff + (long long)f * (rows + 1);
    for (int y = c0; y < c1; y++) {
        const int cnt = s_cnt[y];
        s_cnt[y] = run;   // becomes the fill cursor
        ro[y] = run;
        run += cnt;
    }
    if (tid == 255) ro[rows] = run;   // the last chunk ends at the total (chunks past rows are empty)
    __syncthreads();
    int32_t* rl = rlist + (long long)f * cap * span;
    for (int j = tid; j < nR; j += 256) {
        int y0, y1;
        band(j, y0, y1);
        for (int y = y0; y <= y1; y++) rl[atomicAdd(&s_cnt[y], 1)] = j;
    }
}

__global__ __launch_bounds__(256) void stereo_match_kernel(StereoSide L, StereoSide R, StereoParams sp,
                                                           const orbx_keypoint* __restrict__ kpsL,
                                                           const uint8_t* __restrict__ descL,
                                                           const int32_t* __restrict__ cntL, int nLf,
                                                           const orbx_keypoint* __restrict__ kpsR,
                                                           const uint8_t* __restrict__ descR,
                                                           const int32_t* __restrict__ cntR, int nRf, int cap,
                                                           float* __restrict__ uright, float* __restrict__ depth,
                                                           int32_t* __restrict__ sad, const int32_t* __restrict__ roff,
                                                           const int32_t* __restrict__ rlist, int span) {
    __shared__ uint8_t sIL[4][ST_PS * ST_PS + 7];
    __shared__ uint8_t sW[4][ST_PS * ST_WW + 3];
    __shared__ int sAcc[4][16];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int f = blockIdx.y;
    const int iL = blockIdx.x * 4 + w;
    const int nL = cntL ? cntL[f] : nLf;
    const int nR = cntR ? cntR[f] : nRf;
    if (iL >= nL) return;   // wavefront-uniform; no block barrier below
    const long long o = (long long)f * cap + iL;
    float ur = -1.f, dp = -1.f;
    int sd = -1;
    const orbx_keypoint kL = kpsL[o];
    const int octL = kL.octave;
    const float uL = kL.x, vL = kL.y;
    const int row = (int)vL;
    const float maxd = sp.bf / sp.baseline, mind = 0.f;
    const float minu = uL - maxd, maxu = uL - mind;
    if (row >= 0 && row < L.rows[0] && !(maxu < 0)) {
        const uint4* dl = reinterpret_cast<const uint4*>(descL + o * 32);
        const uint4 a0 = dl[0], a1 = dl[1];
        uint32_t key = 0xffffffffu;
        // the right keypoints whose row band holds this row (stereo_rows_kernel; the reference's
        // vRowIndices[vL], :99): the first minimum is a min of (d << 16 | j), so list order is free
        const int32_t* ro = roff + (long long)f * (L.rows[0] + 1);
        const int32_t* rl = rlist + (long long)f * cap * span;
        const int t0 = ro[row], t1 = ro[row + 1];
        (void)nR;
        for (int t = t0 + lane; t < t1; t += 64) {
            const int j = rl[t];
            const orbx_keypoint kR = kpsR[(long long)f * cap + j];
            if (kR.octave >= octL - 1 && kR.octave <= octL + 1 && kR.x >= minu && kR.x <= maxu) {
                const uint4* dr = reinterpret_cast<const uint4*>(descR + ((long long)f * cap + j) * 32);
                const int d = st_hamming(a0, a1, dr[0], dr[1]);
                if (d < ST_TH_HIGH) key = min(key, ((uint32_t)d << 16) | (uint32_t)j);
            }
        }
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, 64));
        const int TH_ORB_DIST = (ST_TH_HIGH + ST_TH_LOW) / 2;
        if (key != 0xffffffffu && (int)(key >> 16) < TH_ORB_DIST) {
            const int bestIdxR = (int)(key & 0xffffu);
            const float sf = sp.inv_scale[octL];
            const int suL = (int)roundf(sf * kL.x);
            const int svL = (int)roundf(sf * kL.y);
            const int suR = (int)roundf(sf * kpsR[(long long)f * cap + bestIdxR].x);
            if (!(suR + ST_SR - ST_PR < 0 || suR + ST_SR + ST_PR + 1 >= R.cols[octL])) {
                int stepL, stepR;
                const uint8_t* imL = st_level(L, f, octL, &stepL);
                const uint8_t* imR = st_level(R, f, octL, &stepR);
                for (int t = lane; t < ST_PS * ST_PS; t += 64)
                    sIL[w][t] = imL[(long long)(svL - ST_PR + t / ST_PS) * stepL + suL - ST_PR + t % ST_PS];
                for (int t = lane; t < ST_PS * ST_WW; t += 64)
                    sW[w][t] = imR[(long long)(svL - ST_PR + t / ST_WW) * stepR + suR - ST_SR - ST_PR + t % ST_WW];
                if (lane < 16) sAcc[w][lane] = 0;
                st_lds_sync();
                for (int it = lane; it < ST_PS * (2 * ST_SR + 1); it += 64) {
                    const int dxi = it / ST_PS, y = it - dxi * ST_PS;
                    const int sub = (int)sIL[w][ST_PR * ST_PS + ST_PR] - (int)sW[w][ST_PR * ST_WW + ST_PR + dxi];
                    int sum = 0;
#pragma unroll
                    for (int x = 0; x < ST_PS; x++)
                        sum += abs((int)sIL[w][y * ST_PS + x] - (int)sW[w][y * ST_WW + dxi + x] - sub);
                    atomicAdd(&sAcc[w][dxi], sum);
                }
                st_lds_sync();
                if (lane == 0) {
                    int best = INT_MAX, bi = 0;
                    for (int q = 0; q <= 2 * ST_SR; q++)
                        if (sAcc[w][q] < best) { best = sAcc[w][q]; bi = q; }
                    const int bestdx = bi - ST_SR;
                    if (bestdx != -ST_SR && bestdx != ST_SR) {
                        const int d1 = sAcc[w][bi - 1], d2 = sAcc[w][bi], d3 = sAcc[w][bi + 1];
                        const float deltaR = (d1 - d3) / (2.f * (d1 + d3 - 2.f * d2));
                        if (!(deltaR < -1 || deltaR > 1)) {
                            float bestuR = sp.scale[octL] * (suR + bestdx + deltaR);
                            float disparity = uL - bestuR;
                            if (disparity >= mind && disparity < maxd) {
                                if (disparity <= 0) {
                                    disparity = 0.01f;
                                    bestuR = uL - 0.01f;
                                }
                                dp = sp.bf / disparity;
                                ur = bestuR;
                                sd = best;
                            }
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) {
        uright[o] = ur;
        depth[o] = dp;
        sad[o] = sd;
    }
}

// Median-distance filter (:229-246): m = max(n/2 - 1, 0) over the matched SAD distances sorted
// descending; every match with dist >= 1.5f*1.4f*median is dropped.  n == 0: nothing (the
// reference indexes an empty vector there).
__global__ __launch_bounds__(256) void stereo_filter_kernel(const int32_t* __restrict__ cntL, int nLf, int cap,
                                                            float* __restrict__ uright, float* __restrict__ depth,
                                                            const int32_t* __restrict__ sad) {
    extern __shared__ int s_sad[];
    __shared__ int s_n, s_median;
    const int f = blockIdx.x;
    const int nL = cntL ? cntL[f] : nLf;
    if (threadIdx.x == 0) {
        s_n = 0;
        s_median = 0;
    }
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < nL; i += blockDim.x) {
        const int v = sad[(long long)f * cap + i];
        s_sad[i] = v;
        cnt += v >= 0;
    }
    atomicAdd(&s_n, cnt);
    __syncthreads();
    const int n = s_n;
    if (n == 0) return;
    const int m = max(n / 2 - 1, 0);
    for (int i = threadIdx.x; i < nL; i += blockDim.x) {
        const int v = s_sad[i];
        if (v < 0) continue;
        int gt = 0, ge = 0;
        for (int j = 0; j < nL; j++) {
            const int u = s_sad[j];
            gt += u > v;
            ge += u >= v;
        }
        if (gt <= m && m < ge) s_median = v;   // every writer writes the same value
    }
    __syncthreads();
    const float thDist = 1.5f * 1.4f * s_median;
    for (int i = threadIdx.x; i < nL; i += blockDim.x) {
        const int v = s_sad[i];
        if (v >= 0 && !(v < thDist)) {
            uright[(long long)f * cap + i] = -1.f;
            depth[(long long)f * cap + i] = -1.f;
        }
    }
}

int stereo_row_span(const StereoParams& sp, int nlevels) {
    float smax = 1.f;
    for (int l = 0; l < nlevels; l++) smax = std::max(smax, sp.scale[l]);
    return (int)std::ceil(4.f * smax) + 4;   // ceil(y + r) - floor(y - r) + 1 <= 2 r + 3
}

size_t stereo_scratch_ints(int n_frames, int cap, int rows, int span) {
    return (size_t)n_frames * ((size_t)cap + (size_t)(rows + 1) + (size_t)cap * span);
}

int launch_stereo(const StereoSide& L, const StereoSide& R, const StereoParams& sp, int n_frames,
                  const orbx_keypoint* kpsL, const uint8_t* descL, const int32_t* cntL, int nL_fixed,
                  const orbx_keypoint* kpsR, const uint8_t* descR, const int32_t* cntR, int nR_fixed, int cap,
                  float* uright, float* depth, int32_t* scratch, hipStream_t st) {
    if (n_frames <= 0 || cap <= 0) return ORB_OK;
    ORB_CHECK_ARG(cap <= 65535, "stereo: cap too large");
    ORB_CHECK_ARG(L.rows[0] > 0 && L.rows[0] <= ST_MAX_ROWS, "stereo: image rows must be 1..4096");
    const int span = stereo_row_span(sp, L.nlevels);
    int32_t* sad = scratch;
    int32_t* roff = sad + (size_t)n_frames * cap;
    int32_t* rlist = roff + (size_t)n_frames * (L.rows[0] + 1);
    hipLaunchKernelGGL(stereo_rows_kernel, dim3((unsigned)n_frames), dim3(256), 0, st, L, sp, kpsR, cntR, nR_fixed, cap,
                       roff, rlist, span);
    hipLaunchKernelGGL(stereo_match_kernel, dim3((unsigned)((cap + 3) / 4), (unsigned)n_frames), dim3(256), 0, st, L,
                       R, sp, kpsL, descL, cntL, nL_fixed, kpsR, descR, cntR, nR_fixed, cap, uright, depth, sad, roff,
                       rlist, span);
    hipLaunchKernelGGL(stereo_filter_kernel, dim3((unsigned)n_frames), dim3(256), (size_t)cap * sizeof(int), st, cntL,
                       nL_fixed, cap, uright, depth, sad);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

}  // namespace orbamd

using namespace orbamd;

namespace {
struct StereoScratch {
    DevBuf buf;
};
thread_local StereoScratch g_st;
}  // namespace

static int stereo_row_span_host(const float* scale, int nlevels) {
    StereoParams sp;
    std::memset(&sp, 0, sizeof(sp));
    for (int l = 0; l < nlevels && l < ST_MAX_LEVELS; l++) sp.scale[l] = scale[l];
    return stereo_row_span(sp, std::min(nlevels, ST_MAX_LEVELS));
}

extern "C" int orbm_compute_stereo_matches(const orbm_stereo_view* left, const orbm_stereo_view* right,
                                           const float* scale_factors, const float* inv_scale_factors, float bf,
                                           float baseline, float* uright, float* depth) {
    ORB_CHECK_ARG(left && right && scale_factors && inv_scale_factors && uright && depth, "null argument");
    ORB_CHECK_ARG(left->n >= 0 && right->n >= 0, "negative sizes");
    ORB_CHECK_ARG(left->n_levels >= 1 && left->n_levels <= ST_MAX_LEVELS && right->n_levels == left->n_levels,
                  "bad pyramid level count");
    const int nL = left->n, nR = right->n, nl = left->n_levels;
    if (nL == 0) return ORB_OK;
    ORB_CHECK_ARG(left->kps && left->desc && (nR == 0 || (right->kps && right->desc)), "null keypoints");
    for (int i = 0; i < nL; i++)
        ORB_CHECK_ARG(left->kps[i].octave >= 0 && left->kps[i].octave < nl, "left keypoint octave out of range");
    for (int i = 0; i < nR; i++)
        ORB_CHECK_ARG(right->kps[i].octave >= 0 && right->kps[i].octave < nl, "right keypoint octave out of range");
    const int cap = std::max(nL, std::max(nR, 1));
    // one device slab: kpsL kpsR | descL descR | uright depth sad | levels L | levels R
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += align_up(std::max<size_t>(bytes, 1), 256); return o; };
    const size_t o_kL = take((size_t)cap * 28), o_kR = take((size_t)cap * 28), o_dL = take((size_t)cap * 32),
                 o_dR = take((size_t)cap * 32), o_u = take((size_t)cap * 4), o_d = take((size_t)cap * 4),
                 o_s = take(stereo_scratch_ints(1, cap, left->level_rows[0],
                                                stereo_row_span_host(scale_factors, left->n_levels)) * 4);
    size_t o_lv[2][ST_MAX_LEVELS];
    const orbm_stereo_view* views[2] = {left, right};
    for (int v = 0; v < 2; v++)
        for (int l = 0; l < nl; l++) {
            ORB_CHECK_ARG(views[v]->level && views[v]->level[l] && views[v]->level_rows[l] > 0 &&
                              views[v]->level_cols[l] > 0 && views[v]->level_step[l] >= views[v]->level_cols[l],
                          "bad pyramid level");
            o_lv[v][l] = take((size_t)views[v]->level_rows[l] * views[v]->level_cols[l] + 16);
        }
    int rc;
    if ((rc = g_st.buf.reserve(off))) return rc;
    char* base = g_st.buf.as<char>();
    // everything the device reads goes up in two 1D copies from one host staging image of the slab
    // (keypoints + descriptors, then the 2 x nl levels): pitched or per-array copies from pageable
    // memory cost a staging round trip each (a row each, for a pitched level)
    thread_local std::vector<char> stage;
    stage.resize(off);
    std::memcpy(stage.data() + o_kL, left->kps, (size_t)nL * 28);
    if (nR) std::memcpy(stage.data() + o_kR, right->kps, (size_t)nR * 28);
    std::memcpy(stage.data() + o_dL, left->desc, (size_t)nL * 32);
    if (nR) std::memcpy(stage.data() + o_dR, right->desc, (size_t)nR * 32);
    for (int v = 0; v < 2; v++)
        for (int l = 0; l < nl; l++) {
            const int rows = views[v]->level_rows[l], cols = views[v]->level_cols[l];
            const size_t stp = (size_t)views[v]->level_step[l];
            for (int y = 0; y < rows; y++)
                std::memcpy(stage.data() + o_lv[v][l] + (size_t)y * cols, views[v]->level[l] + y * stp, (size_t)cols);
        }
    ORB_HIP_TRY(hipMemcpy(base, stage.data(), o_u, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(base + o_lv[0][0], stage.data() + o_lv[0][0], off - o_lv[0][0], hipMemcpyHostToDevice));
    StereoSide S[2];
    for (int v = 0; v < 2; v++) {
        std::memset(&S[v], 0, sizeof(StereoSide));
        S[v].nlevels = nl;
        for (int l = 0; l < nl; l++) {
            const int rows = views[v]->level_rows[l], cols = views[v]->level_cols[l];
            S[v].off[l] = (long long)o_lv[v][l];
            S[v].stride[l] = cols;
            S[v].rows[l] = rows;
            S[v].cols[l] = cols;
        }
        S[v].lvl0 = reinterpret_cast<const uint8_t*>(base + o_lv[v][0]);
        S[v].fstride0 = 0;
        S[v].step0 = views[v]->level_cols[0];
        S[v].pyr = reinterpret_cast<const uint8_t*>(base);
        S[v].pyr_frame = 0;
    }
    StereoParams sp;
    std::memset(&sp, 0, sizeof(sp));
    for (int l = 0; l < nl; l++) {
        sp.scale[l] = scale_factors[l];
        sp.inv_scale[l] = inv_scale_factors[l];
    }
    sp.bf = bf;
    sp.baseline = baseline;
    if ((rc = launch_stereo(S[0], S[1], sp, 1, reinterpret_cast<const orbx_keypoint*>(base + o_kL),
                            reinterpret_cast<const uint8_t*>(base + o_dL), nullptr, nL,
                            reinterpret_cast<const orbx_keypoint*>(base + o_kR),
                            reinterpret_cast<const uint8_t*>(base + o_dR), nullptr, nR, cap,
                            reinterpret_cast<float*>(base + o_u), reinterpret_cast<float*>(base + o_d),
                            reinterpret_cast<int32_t*>(base + o_s), (hipStream_t)0)))
        return rc;
    ORB_HIP_TRY(hipMemcpy(uright, base + o_u, (size_t)nL * 4, hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(depth, base + o_d, (size_t)nL * 4, hipMemcpyDeviceToHost));
    return ORB_OK;
}
