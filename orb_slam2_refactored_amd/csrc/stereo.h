// Shared between orbs.hip (stereo kernels) and orbx.hip (batched entry point on extractor batches).
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

#include "orbslam2_amd.h"

namespace orbamd {

constexpr int ST_MAX_LEVELS = 16;

// Where one side's unblurred pyramid lives for frame f: level 0 at lvl0 + f*fstride0 (row step
// step0), level l >= 1 at pyr + f*pyr_frame + off[l] (row step stride[l]).
struct StereoSide {
    const uint8_t* lvl0;
    long long fstride0;
    int step0;
    const uint8_t* pyr;
    long long pyr_frame;
    long long off[ST_MAX_LEVELS];
    int stride[ST_MAX_LEVELS], rows[ST_MAX_LEVELS], cols[ST_MAX_LEVELS];
    int nlevels;
};

struct StereoParams {
    float scale[ST_MAX_LEVELS], inv_scale[ST_MAX_LEVELS];
    float bf, baseline;
};

// Rows a right keypoint of any level covers in the row table (floor(y - r) .. ceil(y + r), r = 2 s).
int stereo_row_span(const StereoParams& sp, int nlevels);
// Scratch ints launch_stereo needs: per frame the SAD distances (cap), the row table's offsets
// (rows + 1) and its entries (cap * row span).
size_t stereo_scratch_ints(int n_frames, int cap, int rows, int span);

// Enqueues the row table, the match kernel and the median filter for n_frames frame pairs.
// kps/desc/counts are [n_frames][cap] slot arrays (counts may be NULL with n_fixed keypoints per
// frame).  scratch: stereo_scratch_ints(n_frames, cap, L.rows[0], stereo_row_span(sp, L.nlevels)).
int launch_stereo(const StereoSide& L, const StereoSide& R, const StereoParams& sp, int n_frames,
                  const orbx_keypoint* kpsL, const uint8_t* descL, const int32_t* cntL, int nL_fixed,
                  const orbx_keypoint* kpsR, const uint8_t* descR, const int32_t* cntR, int nR_fixed, int cap,
                  float* uright, float* depth, int32_t* scratch, hipStream_t st);

}  // namespace orbamd
