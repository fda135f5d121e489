// orbm.hip — ORBmatcher Hamming kernels for gfx950.
//
//  * hamming_top2_kernel: brute-force best / second-best over all pairs with the reference's
//    scan semantics (SearchByBoW inner loop, src/ORBmatcher.cc:477-498): one query per lane,
//    query row in VGPRs, candidate rows staged through LDS in 256-row tiles and read as
//    wave-wide broadcasts; distance = 8 x v_bcnt(v_xor) (DescriptorDistance, :1449-1457).
//  * triangulation_kernel: SearchForTriangulation (:768-866) — per query, the last candidate
//    with the minimum distance <= TH_LOW that passes the epipole and epipolar gates
//    (CheckDistEpipolarLine :384-404).  `matched2` is never set by the reference (§0.5), so
//    queries are independent and map one per lane.
#include <cstring>
#include <vector>

#include "common.h"

namespace orbamd {

constexpr int TILE = 256;

__device__ __forceinline__ int hamming32(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ void top2_update(int d, int j, int& bd, int& sd, int& bi) {
    if (d < bd) {
        sd = bd;
        bd = d;
        bi = j;
    } else if (d < sd) {
        sd = d;
    }
}

__global__ __launch_bounds__(256) void hamming_top2_kernel(const uint8_t* __restrict__ A, const int32_t* __restrict__ nA_arr,
                                                           int nA_fixed, int strideA, const uint8_t* __restrict__ B,
                                                           const int32_t* __restrict__ nB_arr, int nB_fixed, int strideB,
                                                           const int32_t* __restrict__ pair_b, float nnratio,
                                                           int th_low, int32_t* __restrict__ best_idx,
                                                           int32_t* __restrict__ best, int32_t* __restrict__ second,
                                                           int32_t* __restrict__ match) {
    __shared__ uint4 tile[TILE * 2];
    const int p = blockIdx.y;
    const int q = pair_b ? pair_b[p] : p;
    const int nA = nA_arr ? nA_arr[p] : nA_fixed;
    const int nB = nB_arr ? nB_arr[q] : nB_fixed;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if ((int)(blockIdx.x * blockDim.x) >= nA) return;   // block-uniform
    const uint8_t* Ap = A + (long long)p * strideA * 32;
    const uint8_t* Bp = B + (long long)q * strideB * 32;
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
    if (i < nA) {
        q0 = reinterpret_cast<const uint4*>(Ap)[2 * i];
        q1 = reinterpret_cast<const uint4*>(Ap)[2 * i + 1];
    }
    int bd = 256, sd = 256, bi = -1;
    for (int t0 = 0; t0 < nB; t0 += TILE) {
        const int nt = min(TILE, nB - t0);
        __syncthreads();
        for (int r = threadIdx.x; r < 2 * nt; r += blockDim.x)
            tile[r] = reinterpret_cast<const uint4*>(Bp)[2 * t0 + r];
        __syncthreads();
        int j = 0;
        for (; j + 4 <= nt; j += 4) {   // four candidates per step: LDS reads issued together
            const uint4 b00 = tile[2 * j], b01 = tile[2 * j + 1], b10 = tile[2 * j + 2], b11 = tile[2 * j + 3];
            const uint4 b20 = tile[2 * j + 4], b21 = tile[2 * j + 5], b30 = tile[2 * j + 6], b31 = tile[2 * j + 7];
            const int d0 = hamming32(q0, q1, b00, b01), d1 = hamming32(q0, q1, b10, b11);
            const int d2 = hamming32(q0, q1, b20, b21), d3 = hamming32(q0, q1, b30, b31);
            top2_update(d0, t0 + j, bd, sd, bi);
            top2_update(d1, t0 + j + 1, bd, sd, bi);
            top2_update(d2, t0 + j + 2, bd, sd, bi);
            top2_update(d3, t0 + j + 3, bd, sd, bi);
        }
        for (; j < nt; j++) top2_update(hamming32(q0, q1, tile[2 * j], tile[2 * j + 1]), t0 + j, bd, sd, bi);
    }
    if (i < nA) {
        const long long o = (long long)p * strideA + i;
        if (best_idx) best_idx[o] = bi;
        if (best) best[o] = bd;
        if (second) second[o] = sd;
        if (match) match[o] = (bd <= th_low && (float)bd < nnratio * (float)sd) ? bi : -1;
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
    hipLaunchKernelGGL(hamming_top2_kernel, dim3((unsigned)((nA + 255) / 256), 1), dim3(256), 0, (hipStream_t)stream,
                       d_A, (const int32_t*)nullptr, nA, nA, d_B, (const int32_t*)nullptr, nB, nB,
                       (const int32_t*)nullptr, 0.6f, 50, d_best_idx, d_best, d_second, (int32_t*)nullptr);
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
    hipLaunchKernelGGL(hamming_top2_kernel, dim3((unsigned)((strideA + 255) / 256), (unsigned)n_pairs), dim3(256), 0,
                       (hipStream_t)stream, d_A, d_nA, 0, strideA, d_B, d_nB, 0, strideB, d_pair_b, nnratio, th_low,
                       d_best_idx, d_best, d_second, d_match);
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
    hipLaunchKernelGGL(hamming_top2_kernel, dim3((unsigned)((nA + 255) / 256), 1), dim3(256), 0, (hipStream_t)0,
                       s.a.as<uint8_t>(), (const int32_t*)nullptr, nA, nA, s.b.as<uint8_t>(), (const int32_t*)nullptr,
                       nB, nB, (const int32_t*)nullptr, nnratio, th_low, o, o + nA, o + 2 * nA, o + 3 * nA);
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
