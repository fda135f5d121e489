/*
 * orbslam2_amd.h — C-ABI of the MI355X (gfx950) ORB front end + local BA.
 *
 * This is the drop-in boundary for the hot path of tiantianxuabc/ORB_SLAM2_Refactored
 * (SURVEY.md §8b).  Every entry point cites the reference interface it replaces.
 * Plain pointers and sizes only; no torch / OpenCV / Eigen types cross it.
 *
 *   status codes: 0 = ok, < 0 = error (orb_last_error() has a thread-local message)
 *   host pointers  : functions without the _device suffix take host memory and are
 *                    synchronous (the reference's calling convention).
 *   device pointers: *_device functions take HBM pointers and a hipStream_t (void*);
 *                    they only enqueue work (no host sync) unless stated.
 */
#ifndef ORBSLAM2_AMD_H
#define ORBSLAM2_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORB_OK          0
#define ORB_EINVAL     -1   /* bad argument (the reference throws cv::Exception via CV_Assert) */
#define ORB_EHIP       -2   /* HIP runtime error */
#define ORB_ENOMEM     -3
#define ORB_ECAP       -4   /* caller's output capacity too small */
#define ORB_EINTERNAL  -5   /* a device-side capacity / consistency check failed */

/* ------------------------------------------------------------------------------------------
 * Extractor.  Replaces ORB_SLAM2::ORBextractor (include/ORBextractor.h:35-81).
 * ---------------------------------------------------------------------------------------- */

/* == ORBextractor::Parameters (include/ORBextractor.h:39-47, defaults src/ORBextractor.cc:830-833) */
typedef struct orbx_params {
    int32_t nfeatures;    /* 2000 */
    float   scaleFactor;  /* 1.2f */
    int32_t nlevels;      /* 8 */
    int32_t iniThFAST;    /* 20 */
    int32_t minThFAST;    /* 7 */
} orbx_params;

/* Byte-compatible with cv::KeyPoint (28 B): pt.x, pt.y, size, angle, response, octave, class_id. */
typedef struct orbx_keypoint {
    float   x, y, size, angle, response;
    int32_t octave, class_id;
} orbx_keypoint;

typedef struct orbx_extractor orbx_extractor;

/* ORBextractor(const Parameters&) + Init() (src/ORBextractor.cc:695-741).  device = HIP ordinal. */
int orbx_create(const orbx_params* params, int device, orbx_extractor** out);
int orbx_destroy(orbx_extractor* h);

/* GetLevels/GetScaleFactors/GetInverseScaleFactors/GetScaleSigmaSquares/
 * GetInverseScaleSigmaSquares (src/ORBextractor.cc:822-827) plus the per-level feature quota
 * (ComputeNumFeaturesPerScale, :472-487).  Each array has nlevels entries; any may be NULL. */
int orbx_scale_tables(const orbx_extractor* h, float* scale, float* inv_scale, float* sigma2,
                      float* inv_sigma2, int32_t* features_per_level);

/* OpenCV-build switches.  Two results of the reference depend on how its OpenCV / C++ headers were
 * built, not on its own source; each is a switch here (default in brackets), restated identically by
 * the CPU oracle (oracle_set_compat).  INTEGRATION.md §1 says how to pick them for a given build.
 *   trig_mode   ComputeOrbDescriptor's `cos(angle)` / `sin(angle)` on a float (src/ORBextractor.cc:107):
 *               [0] ::cos(double) / ::sin(double), the overload visible without `using namespace std`;
 *               1 std::cos(float) / std::sin(float) = glibc cosf / sinf (a `using namespace std`, or a
 *               libstdc++ <math.h> wrapper, before :107).
 *   resize_simd tail mode V of cv::resize INTER_LINEAR 8U's vertical pass (src/ORBextractor.cc:468).
 *               VResizeLinearVec_32s8u rounds via ((S >> 4) * b) >> 16, and OpenCV's uchar
 *               specialisation of VResizeLinear repeats that rounding in its unrolled and scalar tails
 *               [ext, recalled], so [0] (the vector rounding on every column) is every build's result.
 *               8 / 16 / 32 / 64: a FixedPtCast tail (S0*b0 + S1*b1 + 2^21) >> 22 after a V-byte vector
 *               loop; 1: FixedPtCast everywhere.  These are sensitivity switches (parity unpinned).
 * -1 keeps a switch.  Environment defaults at orbx_create: ORBX_TRIG=double|float, ORBX_RESIZE_TAIL=V. */
int orbx_set_opencv_compat(orbx_extractor* h, int trig_mode, int resize_simd);
int orbx_get_opencv_compat(const orbx_extractor* h, int* trig_mode, int* resize_simd);

/* Upper bound on keypoints Extract can return for an image of rows x cols (per-level
 * quadtree output <= max(quota, 4*roots) + 3). */
int orbx_max_keypoints(const orbx_extractor* h, int rows, int cols, int32_t* cap);

/* void ORBextractor::Extract(const cv::Mat& image, KeyPoints& keypoints, cv::Mat& descriptors)
 * (include/ORBextractor.h:55, src/ORBextractor.cc:743-820).  Host memory, synchronous.
 * img: CV_8U rows x cols, row stride `step` bytes.  kps: cap entries; desc: cap x 32 bytes.
 * On return *n = number of keypoints.  Reference quirk kept: when the image yields no keypoint
 * at all *n = 0 and kps/desc are NOT written (Extract returns before keypoints.clear(), :778-782).
 * Returns ORB_ECAP (and *n = required count) if cap is too small. */
int orbx_extract(orbx_extractor* h, const uint8_t* img, int rows, int cols, size_t step,
                 orbx_keypoint* kps, uint8_t* desc, int cap, int* n);

/* GetImagePyramid() (src/ORBextractor.cc:828): copy level `level` of the last extracted image
 * (frame 0 of the last batch) to host memory dst (row stride dst_step; NULL dst = query only). */
int orbx_pyramid_level(const orbx_extractor* h, int level, uint8_t* dst, size_t dst_step,
                       int* rows, int* cols);

/* Batched, HBM-resident Extract over n_frames independent frames of identical size.
 * d_imgs: frame f at d_imgs + f*frame_stride, rows of `step` bytes.
 * Outputs per frame f: d_kps[f*cap .. ], d_desc[(f*cap)*32 .. ], d_counts[f].
 * Keypoint/descriptor order per frame is the reference's (level-major, quadtree list order).
 * Enqueue only (no host sync) on `stream` (a hipStream_t; NULL = the default stream, ordered like
 * any other HIP work on it).  cap must be >= orbx_max_keypoints(). */
int orbx_extract_batch_device(orbx_extractor* h, const uint8_t* d_imgs, int n_frames, int rows,
                              int cols, size_t frame_stride, size_t step, orbx_keypoint* d_kps,
                              uint8_t* d_desc, int32_t* d_counts, int cap, void* stream);

/* Device-side capacity checks of the batched path.  Every kernel of an extraction ORs a fault bit
 * into the handle's fault word when a capacity bound is violated (1 quadtree node array, 2 keypoint
 * outside the root nodes = the reference's CV_Assert :569, 4 FAST cell slot, 8 per-level output,
 * 16 a kernel launched with a block size it is not written for: it exits before touching memory);
 * the batch is then truncated, never written out of bounds.  The word is sticky across batches
 * until read.  orbx_batch_status waits for `stream`, returns the mask in *fault_mask, clears it and
 * returns ORB_EINTERNAL when it was non-zero (the single-frame orbx_extract checks it itself).
 * orbx_fault_word_device returns the word's device address so a pipeline can copy it
 * asynchronously (e.g. into pinned memory) instead of synchronising. */
int orbx_batch_status(orbx_extractor* h, void* stream, uint32_t* fault_mask);
int orbx_fault_word_device(orbx_extractor* h, uint32_t** d_fault);

/* Device pointer to the batch's pyramid (frame f, level s) for downstream consumers
 * (ComputeStereoMatches reads GetImagePyramid(), ORBmatcher.cc:165-166). */
int orbx_pyramid_device(const orbx_extractor* h, int frame, int level, const uint8_t** ptr,
                        int* rows, int* cols, size_t* step);

/* ------------------------------------------------------------------------------------------
 * Matcher.  Replaces the Hamming kernels of ORB_SLAM2::ORBmatcher (src/ORBmatcher.cc).
 * ---------------------------------------------------------------------------------------- */

/* static int ORBmatcher::DescriptorDistance(const cv::Mat&, const cv::Mat&)
 * (include/ORBmatcher.h:54, src/ORBmatcher.cc:1449-1457).  Two 32-byte rows. */
int orbm_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Brute-force best / second-best Hamming search with the reference's loop semantics
 * (SearchByBoW inner loop, src/ORBmatcher.cc:477-498): for each query row i of A scan B in
 * ascending j; best starts at 256 / idx -1, strict '<' updates (lowest j wins ties,
 * second = 2nd order statistic).  Device pointers, enqueue only. */
int orbm_hamming_top2_device(const uint8_t* d_A, int nA, const uint8_t* d_B, int nB,
                             int32_t* d_best_idx, int32_t* d_best, int32_t* d_second, void* stream);

/* Batched pairs: pair p matches A_p (rows d_A + p*strideA*32, count d_nA[p]) against
 * B_q (d_B + q*strideB*32, count d_nB[q]) with q = d_pair_b ? d_pair_b[p] : p (so a batch of
 * frames can be matched against its own predecessors without a copy).  Outputs at p*strideA.
 * Also applies the acceptance test of :500 when d_match != NULL: match = best_idx if
 * best <= th_low and (float)best < nnratio * (float)second, else -1. */
int orbm_bf_match_batch_device(const uint8_t* d_A, const int32_t* d_nA, int strideA,
                               const uint8_t* d_B, const int32_t* d_nB, int strideB,
                               const int32_t* d_pair_b, int n_pairs, float nnratio, int th_low,
                               int32_t* d_best_idx, int32_t* d_best, int32_t* d_second,
                               int32_t* d_match, void* stream);

/* Host-memory convenience form of the two above (synchronous). */
int orbm_bf_match(const uint8_t* A, int nA, const uint8_t* B, int nB, float nnratio, int th_low,
                  int32_t* best_idx, int32_t* best, int32_t* second, int32_t* match);

/* CheckOrientation (src/ORBmatcher.cc:249-309) on a query-indexed match result, applied as
 * SearchForInitialization applies it (:676-686): for every accepted query i (match[i] = j >= 0, in
 * ascending i) the rotation bin is cvRound((angleB[j] - angleA[i] (+360 if < 0)) / 30), 30 bins
 * (bin 30 -> 0); the bins are sorted by size with std::sort's unstable order (libstdc++), the top
 * 1-3 are kept (a 2nd / 3rd bin below 10 % of the largest ends the kept set, :293-298) and every
 * other match is reset to -1.  *nmatches = matches kept.  ORBmatcher(nnratio, checkOri=true)
 * applies it after the brute-force search.  Angles are cv::KeyPoint::angle in [0, 360)
 * (ORB_EINVAL otherwise; the reference CV_Asserts the bin).  Host memory, synchronous. */
int orbm_check_orientation(const float* angleA, int nA, const float* angleB, int nB, int32_t* match,
                           int32_t* nmatches);

/* Batched device form on orbm_bf_match_batch_device's output: pair p's queries have angles
 * d_angA[(p*capA + i)*kstrideA] (kstrideA = 7 with d_angA = &kps[0].angle of an orbx_keypoint
 * array), its targets d_angB[(q*capB + j)*kstrideB] with q = d_pair_b ? d_pair_b[p] : p; d_nA[p]
 * queries; d_match at p*strideM is updated in place; d_nmatches[p] (may be NULL).  One workgroup
 * per pair; enqueue only. */
int orbm_check_orientation_batch_device(const float* d_angA, int kstrideA, int capA, const int32_t* d_nA,
                                        const float* d_angB, int kstrideB, int capB, const int32_t* d_pair_b,
                                        int n_pairs, int32_t* d_match, int strideM, int32_t* d_nmatches,
                                        void* stream);

/* One keyframe's view for SearchForTriangulation (src/ORBmatcher.cc:768-866). */
typedef struct orbm_tri_frame {
    int32_t        n;           /* keyframe->N */
    const float*   kp_xy;       /* keypointsUn pt, n x 2 */
    const int32_t* octave;      /* keypointsUn octave, n */
    const float*   uright;      /* n (< 0: mono) */
    const uint8_t* has_mappoint;/* GetMapPoint(idx) != nullptr, n (0/1) */
    const uint8_t* desc;        /* descriptorsL, n x 32 */
    /* DBoW2 FeatureVector as CSR: node ids ascending, node k owns
     * indices[node_off[k] .. node_off[k+1]) (ascending feature indices). */
    int32_t        n_nodes;
    const uint32_t* node_id;
    const int32_t* node_off;
    const int32_t* indices;
} orbm_tri_frame;

/* int ORBmatcher::SearchForTriangulation(const KeyFrame* kf1, const KeyFrame* kf2,
 *   const cv::Mat& F12, std::vector<std::pair<size_t,size_t>>& matchIds, bool onlyStereo)
 * (include/ORBmatcher.h:84-85).  F12 row-major 3x3 (cv::Mat1f); ep2 = projection of kf1's
 * camera centre in kf2 (:772-773); scale2/sigma2: kf2 pyramid scaleFactors / sigmaSq.
 * Host memory.  match12[idx1] = idx2 or -1 (pairs sorted by idx1 are the non-negative
 * entries); *nmatches = count.  checkOrientation is false at the only caller
 * (LocalMapping.cc:388), so it is not applied. */
int orbm_search_for_triangulation(const orbm_tri_frame* kf1, const orbm_tri_frame* kf2,
                                  const float* F12, const float* ep2, const float* scale2,
                                  const float* sigma2, int n_levels, int only_stereo,
                                  int32_t* match12, int32_t* nmatches);

/* Batched SearchForTriangulation on HBM-resident extractor output (orbx_extract_batch_device slots),
 * e.g. the neighbour-keyframe loop of LocalMapping::CreateNewMapPoints (LocalMapping.cc:380-430)
 * issued as one launch.  Pair p matches keyframe frame1[p] of set 1 (slots at kps1 / desc1 +
 * frame*cap1, counts1[frame]) against frame2[p] of set 2 (NULL index arrays: p).  Sets 1 and 2 may
 * be the same arrays.  Per pair: F12 (9 floats, row-major, from ComputeF12 :55-71) and ep2 (2
 * floats, kf1's camera centre projected by kf2, :772-773; may be non-finite).  uright / has_mappoint
 * per slot (NULL: every keypoint monocular / without a MapPoint).  FeatureVectors in
 * orbv_transform_batch_device's layout (node ids / offsets / indices at frame*fv_cap, offsets at
 * frame*(fv_cap+1), fv_n_nodes[frame]); NULL for both sets = one node holding every keypoint
 * (all-pairs search under the gates, the vocabulary-free C3 setup).  kf2's scale factors / sigma^2
 * are host arrays of n_levels (<= ORBM_TRI_MAX_LEVELS).  Outputs: d_match12[p*cap1 + idx1] = idx2
 * or -1 for idx1 < counts1; d_nmatches[p].  checkOrientation is false at the caller
 * (LocalMapping.cc:388).  Enqueue only on `stream`. */
#define ORBM_TRI_MAX_LEVELS 32
typedef struct orbm_tri_batch {
    int32_t n_pairs;
    int32_t cap1, cap2;
    const orbx_keypoint* kps1; const uint8_t* desc1; const int32_t* counts1;
    const float* uright1; const uint8_t* has_mappoint1;
    const orbx_keypoint* kps2; const uint8_t* desc2; const int32_t* counts2;
    const float* uright2; const uint8_t* has_mappoint2;
    const int32_t* frame1; const int32_t* frame2;
    const float* F12;           /* n_pairs x 9 */
    const float* ep2;           /* n_pairs x 2 */
    const uint32_t* fv_node1; const int32_t* fv_off1; const int32_t* fv_idx1; const int32_t* fv_n_nodes1;
    const uint32_t* fv_node2; const int32_t* fv_off2; const int32_t* fv_idx2; const int32_t* fv_n_nodes2;
    int32_t fv_cap1, fv_cap2;
    int32_t n_levels;
    const float* scale_factors2; /* host, n_levels */
    const float* sigma2;         /* host, n_levels */
    int32_t only_stereo;
} orbm_tri_batch;

int orbm_search_for_triangulation_batch_device(const orbm_tri_batch* b, int32_t* d_match12, int32_t* d_nmatches,
                                               void* stream);

/* int ORBmatcher::SearchByBoW(KeyFrame* keyframe, Frame& frame, std::vector<MapPoint*>& matches)
 * (include/ORBmatcher.h:77, src/ORBmatcher.cc:452-516; callers Tracking.cc TrackReferenceKeyFrame /
 * Relocalization), batched on HBM-resident extractor slots.  Pair p matches keyframe frame1[p] of
 * set 1 (NULL: p) against frame p of set 2.  FeatureVectorIterator (:406-450) joins equal node ids;
 * in a common node every keyframe feature idx1 (ascending, as stored) with mp_valid1 != 0
 * (GetMapPointMatches()[idx1] non-null and not isBad(); NULL = all valid) scans the node's frame
 * features that no earlier idx1 claimed (the reference's `if (matches[idx2]) continue`), keeps the
 * lowest-index best and the second-best distance, and claims bestIdx2 when best <= TH_LOW (50) and
 * (float)best < nnratio * (float)second.  A frame feature sits in one node only, so the claims of
 * different nodes are independent and the result is the reference's.  With check_orientation the
 * rotation-histogram filter (CheckOrientation(keyframe->keypointsUn, frame.keypointsUn, ...),
 * :249-309, :512-513) erases the matches outside the top bins.  FeatureVectors in
 * orbv_transform_batch_device's layout (both sets required).  Outputs: d_match[p*cap2 + idx2] =
 * idx1 (the MapPoint of keyframe feature idx1) or -1 for idx2 < counts2[p]; d_nmatches[p] = the
 * return value.  Enqueue only on `stream`. */
typedef struct orbm_bow_batch {
    int32_t n_pairs;
    int32_t cap1, cap2;
    const orbx_keypoint* kps1; const uint8_t* desc1; const uint8_t* mp_valid1;
    const int32_t* frame1;
    const orbx_keypoint* kps2; const uint8_t* desc2; const int32_t* counts2;
    const uint32_t* fv_node1; const int32_t* fv_off1; const int32_t* fv_idx1; const int32_t* fv_n_nodes1;
    const uint32_t* fv_node2; const int32_t* fv_off2; const int32_t* fv_idx2; const int32_t* fv_n_nodes2;
    int32_t fv_cap1, fv_cap2;
    float nnratio;
    int32_t check_orientation;
    /* KeyFrame-KeyFrame form only (NULL in the Frame form): */
    const int32_t* counts1;      /* kf1 keypoint counts (CheckOrientation) */
    const uint8_t* mp_valid2;    /* kf2 MapPoint valid (NULL: all) */
    const int32_t* frame2;       /* kf2 slot of pair p (NULL: p) */
} orbm_bow_batch;

int orbm_search_by_bow_batch_device(const orbm_bow_batch* b, int32_t* d_match, int32_t* d_nmatches, void* stream);

/* int ORBmatcher::SearchByBoW(KeyFrame* keyframe1, KeyFrame* keyframe2, std::vector<MapPoint*>& matches12)
 * (include/ORBmatcher.h:78, src/ORBmatcher.cc:696-766) on the same batch layout: pair p = (kf1
 * frame1[p] of set 1, kf2 frame2[p] of set 2).  Differences from the Frame form: candidates need a
 * valid kf2 MapPoint (mp_valid2) besides being unclaimed (matched2, :733), acceptance is
 * bestDist < TH_LOW (strict, :750), the result is indexed by idx1 (d_match12[p*cap1 + idx1] = idx2,
 * i.e. matches12[idx1] = mappoints2[idx2]) and CheckOrientation(keypoints2, keypoints1, ...)
 * (:762-763) bins angle2[idx2] - angle1[idx1] and erases matches12[idx1] (needs counts1).
 * Enqueue only on `stream`. */
int orbm_search_by_bow_kf_batch_device(const orbm_bow_batch* b, int32_t* d_match12, int32_t* d_nmatches,
                                       void* stream);

/* Stereo matching.  Replaces ComputeStereoMatches (src/ORBmatcher.cc:72-247, PatchDistance
 * :60-68; called from Frame construction for stereo input, System.cc:458-461): per left keypoint the
 * best right keypoint in the row band (+-2*scale[octave_R] rows), octave +-1 and disparity
 * [0, bf/baseline], Hamming < (TH_HIGH+TH_LOW)/2; then 11x11 SAD over +-5 px on the unblurred
 * level of the left octave, parabola refinement, and the median-distance outlier filter.
 * Outputs uright[i] / depth[i] (-1 = no match), one per left keypoint.
 * A view is one frame: its keypoints (level-0 coordinates, cv::KeyPoint layout), descriptors and
 * unblurred pyramid levels (GetImagePyramid()).  The right keypoints' row table (vRowIndices) is
 * built on the device for images of at most 4096 rows (ORB_EINVAL above); a row band reaching past
 * the image is clipped to it (the reference indexes outside vRowIndices there). */
typedef struct orbm_stereo_view {
    int32_t n;
    const orbx_keypoint* kps;
    const uint8_t* desc;                 /* n x 32 */
    int32_t n_levels;
    const uint8_t* const* level;         /* n_levels level images */
    const int32_t* level_rows;
    const int32_t* level_cols;
    const int32_t* level_step;           /* bytes per row */
} orbm_stereo_view;

int orbm_compute_stereo_matches(const orbm_stereo_view* left, const orbm_stereo_view* right,
                                const float* scale_factors, const float* inv_scale_factors, float bf,
                                float baseline, float* uright, float* depth);

/* Batched device version on the frames of two extractors' last batches (left frame f with right
 * frame f; both extractors with the same Parameters and image size).  Keypoints / descriptors /
 * counts are those batches' outputs.  d_uright / d_depth: n_frames * cap floats, slot f*cap + i.
 * Enqueue only, on `stream` (NULL = default stream). */
int orbx_stereo_matches_batch_device(orbx_extractor* left, orbx_extractor* right, int n_frames,
                                     const orbx_keypoint* d_kps_l, const uint8_t* d_desc_l,
                                     const int32_t* d_counts_l, const orbx_keypoint* d_kps_r,
                                     const uint8_t* d_desc_r, const int32_t* d_counts_r, int cap,
                                     float bf, float baseline, float* d_uright, float* d_depth,
                                     void* stream);

/* ComputeStereoMatches for the reference's own call shape (System.cc:449-461, Frame's stereo
 * constructor: two Extract calls, then ComputeStereoMatches on mvKeys / mvKeysRight and the two
 * extractors' mvImagePyramid): `left` / `right` are the handles whose last call was orbx_extract on
 * the pair's images; their keypoints, descriptors and pyramids are still on the device, so nothing but
 * uright / depth (n_left floats each, -1 = no match) crosses PCIe.  n_left must equal the left
 * Extract's keypoint count.  Synchronous; call after both Extract calls have returned. */
int orbx_stereo_matches_last(orbx_extractor* left, orbx_extractor* right, float bf, float baseline, float* uright,
                             float* depth, int n_left);

/* ------------------------------------------------------------------------------------------
 * Local-map search.  Replaces ORBmatcher::SearchByProjection(Frame&, const std::vector<MapPoint*>&,
 * float th) (include/ORBmatcher.h:58, src/ORBmatcher.cc:315-382) together with the frame's
 * FeaturesGrid (include/Frame.h:62-80; AssignFeatures / GetFeaturesInArea, src/Frame.cc:71-145),
 * batched over frames.  Per frame f: keypoints [kp_begin[f], kp_begin[f+1]) (keypointsUn order)
 * and the local map points [mp_begin[f], mp_begin[f+1]) (vector order) with the fields
 * IsInFrustum filled (Tracking.cc:554-605).
 * ---------------------------------------------------------------------------------------- */
#define ORBM_GRID_COLS 64
#define ORBM_GRID_ROWS 48
#define ORBM_PROJ_MAX_KP 8192   /* keypoints per frame */

typedef struct orbm_proj_batch {
    int32_t        n_frames;
    int32_t        total_kp, total_mp;   /* kp_begin[n_frames], mp_begin[n_frames] (workspace sizing) */
    const int32_t* kp_begin;     /* n_frames + 1 */
    const float*   kp_xy;        /* keypointsUn pt, total_kp x 2 */
    const int32_t* kp_octave;    /* keypointsUn octave */
    const float*   kp_uright;    /* uright */
    const uint8_t* kp_desc;      /* descriptors, total_kp x 32 */
    const uint8_t* kp_claimed;   /* mappoints[i] && mappoints[i]->Observations() > 0 on entry (NULL: none) */
    const float*   bounds;       /* n_frames x 4: imageBounds minx, maxx, miny, maxy */
    const int32_t* mp_begin;     /* n_frames + 1 */
    const uint8_t* mp_valid;     /* trackInView && !isBad() (:320) */
    const float*   mp_proj;      /* total_mp x 3: trackProjX, trackProjY, trackProjXR */
    const float*   mp_view_cos;  /* trackViewCos */
    const int32_t* mp_level;     /* trackScaleLevel (0 .. n_levels-1) */
    const uint8_t* mp_desc;      /* GetDescriptor(), total_mp x 32 */
    const uint8_t* mp_has_obs;   /* Observations() > 0 (a keypoint it claims is then skipped, :339) */
    int32_t        n_levels;
    const float*   scale_factors;/* n_levels (frame.pyramid.scaleFactors), host memory in both entries */
    float          th;           /* SearchLocalPoints: 1, 3 (RGB-D) or 5 after relocalisation (Tracking.cc:1246) */
    float          nnratio;      /* ORBmatcher(0.8f) in SearchLocalPoints (Tracking.cc:646) */
} orbm_proj_batch;

/* kp_match[k]: frame-relative index of the map point the call assigned to keypoint k (the last
 * assignment of frame.mappoints[bestIdx] = mappoint, :376), -1 when the call assigned none.
 * n_matches[f]: SearchByProjection's return value; -1 (device entry) when a frame has more than
 * ORBM_PROJ_MAX_KP keypoints.  Host entry: every pointer is host memory, synchronous. */
int orbm_search_by_projection(const orbm_proj_batch* b, int32_t* kp_match, int32_t* n_matches, int device);
/* Device entry: every array in HBM except scale_factors; enqueue only on `stream`. */
int orbm_search_by_projection_device(const orbm_proj_batch* b, int32_t* kp_match, int32_t* n_matches,
                                     void* stream);

/* int ORBmatcher::SearchByProjection(Frame& currFrame, const Frame& lastFrame, float th, bool monocular)
 * (include/ORBmatcher.h:61, src/ORBmatcher.cc:1279-1362; Tracking::TrackWithMotionModel), batched over
 * frames.  Current frame f: keypoints [kp_begin[f], kp_begin[f+1]) as in orbm_proj_batch, plus
 * kp_angle (keypointsUn angle, for CheckOrientation).  Last frame's points [mp_begin[f], mp_begin[f+1])
 * in idx1 order: mp_valid = mappoints[idx1] && !outlier[idx1] && Xc.z >= 0 && imageBounds.Contains(u, v)
 * (:1295-1311, the caller projects), mp_proj = (u, v, ur = u - DepthToDisparity(Xc.z)), mp_octave =
 * lastFrame.keypoints[idx1].octave, mp_desc = GetDescriptor(), mp_has_obs = Observations() > 0,
 * mp_angle = lastFrame.keypointsUn[idx1].angle.  motion[f]: 0, 1 = forward, 2 = backward (:1286-1288).
 * Window th * scaleFactors[octave] over the levels of :1318-1319, claimed keypoints skipped, the
 * stereo gate with the window radius, best distance <= TH_HIGH; then CheckOrientation(lastFrame,
 * currFrame, ...) (:1358-1359) over every accepted (idx1, bestIdx2) pair in order (overwritten ones
 * included, as the reference's matchIds).  kp_match[k] = frame-relative idx1 the call assigned to
 * keypoint k (-1: none, or erased by the rotation filter); n_matches[f] = the return value (-1 when
 * the frame has more than ORBM_PROJ_MAX_KP keypoints).  Enqueue only on `stream`. */
typedef struct orbm_motion_batch {
    int32_t        n_frames, total_kp, total_mp;
    const int32_t* kp_begin;
    const float*   kp_xy;
    const int32_t* kp_octave;
    const float*   kp_uright;
    const uint8_t* kp_desc;
    const float*   kp_angle;
    const uint8_t* kp_claimed;   /* currFrame.mappoints[i] with Observations() > 0 on entry (NULL: none) */
    const float*   bounds;       /* n_frames x 4 */
    const int32_t* mp_begin;
    const uint8_t* mp_valid;
    const float*   mp_proj;      /* total_mp x 3 */
    const int32_t* mp_octave;
    const uint8_t* mp_desc;
    const uint8_t* mp_has_obs;
    const float*   mp_angle;
    const int32_t* motion;       /* n_frames (NULL: all 0) */
    int32_t        n_levels;
    const float*   scale_factors;/* host, n_levels */
    float          th;
    int32_t        check_orientation;
} orbm_motion_batch;

int orbm_search_by_projection_motion_device(const orbm_motion_batch* b, int32_t* kp_match, int32_t* n_matches,
                                            void* stream);

/* int ORBmatcher::SearchByProjection(Frame& frame, KeyFrame* keyframe, const std::set<MapPoint*>& alreadyFound,
 * float th, int ORBdist) (include/ORBmatcher.h:66, src/ORBmatcher.cc:1364-1445; Tracking::Relocalization
 * calls it with th 10 / ORBdist 100, then th 3 / ORBdist 64, Tracking.cc:403,417), batched over
 * (frame, candidate keyframe) pairs.  Frame f: keypoints [kp_begin[f], kp_begin[f+1]) as in
 * orbm_motion_batch (no uright: the search has no stereo gate), kp_claimed = frame.mappoints[i] != NULL
 * on entry (every non-null entry blocks, :1413-1414), its pose Rcw / tcw and intrinsics.  Keyframe
 * points [mp_begin[f], mp_begin[f+1]) = GetMapPointMatches() in idx1 order: mp_valid = mappoint &&
 * !isBad() && !alreadyFound.count(mappoint), mp_xw = GetWorldPos(), mp_max_min = (maxDistance_,
 * minDistance_) (MapPoint.cc:369-377), mp_angle = keyframe->keypointsUn[idx1].angle.  On the device:
 * the projection and imageBounds.Contains (:1385-1391), the distance-invariance gate with 0.8f /
 * 1.2f (:1393-1401, MapPoint.cc:382-392), PredictScale (MapPoint.cc:405-415: ceil(log(ratio) /
 * logScaleFactor), log taken as ::log(double)), the window th * scaleFactors[predictedScale] over
 * levels predictedScale +- 1, the first-best distance over the keypoints not yet holding a map point,
 * bestDist <= ORBdist (< 256), the claim, then CheckOrientation(keyframe->keypointsUn,
 * frame.keypointsUn, ...) (:1439-1440).  kp_match[k] = idx1 assigned to frame keypoint k (-1: none or
 * erased), n_matches[f] = the return value (-1 when the frame has more than ORBM_PROJ_MAX_KP
 * keypoints). */
typedef struct orbm_reloc_batch {
    int32_t        n_frames, total_kp, total_mp;
    const int32_t* kp_begin;
    const float*   kp_xy;        /* frame keypointsUn pt */
    const int32_t* kp_octave;
    const uint8_t* kp_desc;
    const float*   kp_angle;
    const uint8_t* kp_claimed;   /* frame.mappoints[i] != NULL on entry (NULL: none) */
    const float*   bounds;       /* n_frames x 4: imageBounds minx, maxx, miny, maxy */
    const float*   pose;         /* n_frames x 12: Rcw (row-major 3x3) then tcw */
    const float*   camera;       /* n_frames x 4: fx, fy, cx, cy */
    const int32_t* mp_begin;
    const uint8_t* mp_valid;
    const float*   mp_xw;        /* total_mp x 3 */
    const float*   mp_max_min;   /* total_mp x 2: maxDistance_, minDistance_ */
    const uint8_t* mp_desc;
    const float*   mp_angle;
    int32_t        n_levels;
    const float*   scale_factors;/* host, n_levels */
    float          log_scale_factor; /* pyramid.logScaleFactor */
    float          th;
    int32_t        orb_dist;     /* ORBdist, 0 .. 255 */
    int32_t        check_orientation;
} orbm_reloc_batch;

/* Host entry: every pointer host memory, synchronous. */
int orbm_search_by_projection_reloc(const orbm_reloc_batch* b, int32_t* kp_match, int32_t* n_matches, int device);
/* Device entry: every array in HBM except scale_factors; enqueue only on `stream`. */
int orbm_search_by_projection_reloc_device(const orbm_reloc_batch* b, int32_t* kp_match, int32_t* n_matches,
                                           void* stream);

/* int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
 * std::vector<int>& vnMatches12, int windowSize) (include/ORBmatcher.h:81, src/ORBmatcher.cc:614-694;
 * Tracking::MonocularInitialization, Tracking.cc:1052), batched over initialisation pairs.
 * Pair p: frame F1 (queries idx1) = [q_begin[p], q_begin[p+1]) and frame F2 (searched) =
 * [kp_begin[p], kp_begin[p+1]), both keypointsUn.  Only octave-0 queries search, over the octave-0
 * features of F2 inside FeaturesGrid::GetFeaturesInArea(prevMatched, windowSize) (Frame.cc:102-145,
 * scan order cell by cell); a candidate is skipped when the distance it is already held at
 * (matchedDistance, INT_MAX on entry) is <= its own, so a later query can take a feature from an
 * earlier one (matches12 of the earlier query becomes -1, :669-673).  Accept best <= TH_LOW and
 * best < nnratio * second; then, with check_orientation, CheckOrientation(F2.keypointsUn,
 * F1.keypointsUn, matchIds, matches12) (:249-309) over every accepted (idx2, idx1) in order,
 * replaced ones included, whose count is the return value.  prev_matched[q] (total_q x 2, in/out)
 * becomes F2.keypointsUn[matches12[q]].pt for every surviving match (:690-692).
 * matches12[q] = F2-relative idx2 or -1; n_matches[p] = the return value, -1 (device entry) when a
 * frame of the pair has more than ORBM_PROJ_MAX_KP keypoints. */
typedef struct orbm_init_batch {
    int32_t        n_pairs, total_kp, total_q;
    const int32_t* kp_begin;     /* F2: n_pairs + 1 */
    const float*   kp_xy;        /* F2 keypointsUn pt, total_kp x 2 */
    const int32_t* kp_octave;    /* F2 keypointsUn octave */
    const uint8_t* kp_desc;      /* F2 descriptors, total_kp x 32 */
    const float*   kp_angle;     /* F2 keypointsUn angle (CheckOrientation) */
    const float*   bounds;       /* F2 imageBounds, n_pairs x 4 */
    const int32_t* q_begin;      /* F1: n_pairs + 1 */
    const int32_t* q_octave;     /* F1 keypointsUn octave */
    const uint8_t* q_desc;       /* F1 descriptors, total_q x 32 */
    const float*   q_angle;      /* F1 keypointsUn angle */
    float*         prev_matched; /* total_q x 2, in / out */
    int32_t        window;       /* windowSize (100 in MonocularInitialization) */
    float          nnratio;      /* ORBmatcher(0.9f, true) there */
    int32_t        check_orientation;
} orbm_init_batch;

/* Host entry: every pointer host memory, synchronous. */
int orbm_search_for_initialization(const orbm_init_batch* b, int32_t* matches12, int32_t* n_matches, int device);
/* Device entry: every array in HBM; enqueue only on `stream`. */
int orbm_search_for_initialization_device(const orbm_init_batch* b, int32_t* matches12, int32_t* n_matches,
                                          void* stream);

/* ------------------------------------------------------------------------------------------
 * Bag of words.  Replaces DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> as ORBVocabulary
 * (include/ORBVocabulary.h) for Frame::ComputeBoW / KeyFrame::ComputeBoW (src/Frame.cc:208-214,
 * src/KeyFrame.cc:66-74): loadFromTextFile (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1341-1431)
 * and transform(features, BowVector&, FeatureVector&, levelsup) (:1130-1196, descent :1221-1263).
 * BowVector = std::map<WordId, double> and FeatureVector = std::map<NodeId, vector<unsigned>>
 * (BowVector.h, FeatureVector.h) are returned as ascending arrays / CSR — the FeatureVector CSR is
 * exactly orbm_tri_frame's node_id / node_off / indices.
 * ---------------------------------------------------------------------------------------- */
typedef struct orbv_vocabulary orbv_vocabulary;
#define ORBV_MAX_FEATURES 4096   /* descriptors per transform (2 x nfeatures of the initial extractor) */

/* Text format of saveToTextFile (:1434-1450): "k L scoring weighting", then one line per node
 * 1..N-1 in id order: "parent isLeaf d0 .. d31 weight".  Trailing empty lines are ignored (the
 * reference's eof loop turns a final newline into an extra root child with an uninitialised
 * descriptor and weight 0). */
int orbv_load_text(const char* path, int device, orbv_vocabulary** out);
/* The same content from arrays: node i (1 <= i < n_nodes) has parent[i], is_leaf[i], desc[32 i ..],
 * weight[i]; entries for i = 0 (the root) are ignored. */
int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                orbv_vocabulary** out);
int orbv_destroy(orbv_vocabulary* v);
int orbv_info(const orbv_vocabulary* v, int* k, int* L, int* n_nodes, int* n_words, int* scoring,
              int* weighting);

/* transform(features, BowVector&, FeatureVector&, levelsup) for one descriptor set, host memory.
 * bow_word / bow_weight: capacity n each, *n_words entries, word ids ascending.  fv_node: capacity
 * n, fv_off: n + 1, fv_idx: n; *n_nodes node ids ascending, node t owns fv_idx[fv_off[t] ..
 * fv_off[t+1]) (feature indices ascending).  Stopped words (weight 0) are in neither vector.
 * Where the reference's node id is undefined (a leaf shallower than L - levelsup) the leaf's id
 * is used. */
int orbv_transform(orbv_vocabulary* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word,
                   double* bow_weight, int* n_words, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_idx,
                   int* n_nodes);
/* Batched device form over n_frames descriptor sets (frame f: d_desc + f*cap*32, d_counts[f] rows,
 * cap <= ORBV_MAX_FEATURES) — e.g. an orbx_extract_batch_device output.  Per frame f the outputs
 * use slot f: d_bow_word / d_bow_weight / d_fv_node / d_fv_idx at f*cap, d_fv_off at f*(cap+1),
 * d_n_words[f], d_n_nodes[f].  Enqueue only on `stream`. */
int orbv_transform_batch_device(orbv_vocabulary* v, const uint8_t* d_desc, const int32_t* d_counts, int cap,
                                int n_frames, int levelsup, uint32_t* d_bow_word, double* d_bow_weight,
                                int32_t* d_n_words, uint32_t* d_fv_node, int32_t* d_fv_off, int32_t* d_fv_idx,
                                int32_t* d_n_nodes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Local bundle adjustment.  Replaces Optimizer::LocalBundleAdjustment (include/Optimizer.h:47,
 * src/Optimizer.cc:491-736) from the vertex/edge setup (:540-631) onwards: the caller
 * gathers local / fixed keyframes and map points and flattens them in reference order.
 * ---------------------------------------------------------------------------------------- */
typedef struct orbba_problem {
    int32_t        n_poses;     /* local KFs then fixed KFs (vertex insertion order) */
    const double*  pose_R;      /* n_poses x 9 row-major world->camera rotation (CameraPose R) */
    const double*  pose_t;      /* n_poses x 3 */
    const uint8_t* pose_fixed;  /* n_poses: KF id 0 or a fixed camera */
    int32_t        n_points;
    const double*  points;      /* n_points x 3 world position */
    int32_t        n_edges;     /* observations, in reference insertion order */
    const int32_t* edge_point;  /* n_edges */
    const int32_t* edge_pose;   /* n_edges */
    const double*  edge_obs;    /* n_edges x 3: u, v, ur (ur < 0 => mono edge, :595) */
    const double*  edge_inv_sigma2; /* n_edges: pyramid.invSigmaSq[octave] */
    const double*  edge_cam;    /* n_edges x 5: fx, fy, cx, cy, bf */
} orbba_problem;

typedef struct orbba_result {
    double*   pose_R;       /* n_poses x 9 (optimised; fixed poses unchanged) */
    double*   pose_t;       /* n_poses x 3 */
    double*   pose_q;       /* n_poses x 4 (x,y,z,w), g2o SE3Quat rotation; may be NULL */
    double*   points;       /* n_points x 3 */
    uint8_t*  edge_outlier; /* n_edges: 1 = chi2 > 5.991/7.815 or depth <= 0 at the end (:686-699) */
    double*   edge_chi2;    /* n_edges: final chi2 (may be NULL) */
    int32_t   iterations[2];/* LM iterations run by optimize(5) and optimize(10) */
    double    chi2[2];      /* active robust chi2 after each optimize */
    int32_t   ran;          /* 0: the stop flag was set on entry, nothing was optimised and the caller
                             * must not write anything back (Optimizer.cc:633-634 returns there) */
} orbba_result;

/* Free keyframes per optimize() (the reduced camera system is 6 x that square).  Up to 21 the system
 * is factored in LDS; above that in HBM by a 1024-thread blocked LDL^T (slower per trial, same
 * algorithm).  ORB_EINVAL beyond this limit. */
#define ORBBA_MAX_FREE_KEYFRAMES 512

/* stop_flag: g2o's force-stop flag (sparse_optimizer.h:188, LocalMapping's abortBA_); may be NULL.
 * Polled where g2o polls terminate(): before the call, between optimize(5) and optimize(10), and after
 * every LM trial (the flag is mirrored into device-visible memory while the call waits, and the
 * device's control kernel ends the loop after the trial in which it saw the flag). */
int orbba_local_ba(const orbba_problem* prob, orbba_result* res, const volatile int32_t* stop_flag,
                   int device);

/* ------------------------------------------------------------------------------------------
 * Motion-only bundle adjustment.  Replaces Optimizer::PoseOptimization (include/Optimizer.h:49,
 * src/Optimizer.cc:345-489) for a batch of frames: one SE3 vertex per frame, one unary
 * EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose per matched map point
 * (types_six_dof_expmap.h:143-202), 4 rounds of optimize(10) with chi2 outlier
 * classification (5.991 mono / 7.815 stereo), Huber kernels dropped after round 2, and a
 * single round when a frame has fewer than 10 edges.  The caller flattens, per frame, the
 * keypoints that have a map point in keypoint order (Optimizer.cc:364-410).
 * ---------------------------------------------------------------------------------------- */
#define ORBBA_POSE_MAX_EDGES 16384   /* edges per frame */

typedef struct orbba_pose_batch {
    int32_t        n_frames;
    const int32_t* edge_begin;  /* n_frames + 1: frame f owns edges [edge_begin[f], edge_begin[f+1]) */
    const double*  pose_R;      /* n_frames x 9 row-major Tcw rotation (frame->pose) */
    const double*  pose_t;      /* n_frames x 3 */
    const double*  cam;         /* n_frames x 5: fx, fy, cx, cy, bf (frame->camera) */
    const double*  xw;          /* E x 3: the map point's GetWorldPos() */
    const double*  obs;         /* E x 3: keypointsUn[i].pt.x, .y, uright[i] (ur < 0: monocular, :376) */
    const double*  inv_sigma2;  /* E: pyramid.invSigmaSq[keypointsUn[i].octave] */
} orbba_pose_batch;

typedef struct orbba_pose_result {
    double*  pose_R;     /* n_frames x 9 (frame->SetPose; input pose copied when < 3 edges) */
    double*  pose_t;     /* n_frames x 3 */
    int32_t* n_inliers;  /* n_frames: PoseOptimization's return value (nedges - noutliers, 0 if < 3);
                          * -1 from the device entry when a frame exceeds ORBBA_POSE_MAX_EDGES */
    uint8_t* outlier;    /* E: frame->outlier[i] after the last round */
} orbba_pose_result;

/* Host buffers; synchronous.  ORB_EINVAL if a frame has more than ORBBA_POSE_MAX_EDGES edges. */
int orbba_pose_optimization(const orbba_pose_batch* in, orbba_pose_result* out, int device);
/* Device buffers (every pointer in both structs); enqueue only, on `stream` (NULL = default
 * stream).  One workgroup per frame. */
int orbba_pose_optimization_device(const orbba_pose_batch* in, orbba_pose_result* out, void* stream);

const char* orb_last_error(void);
int orb_device_count(void);

/* Compact descriptor block for the multi-GPU exchange (BASELINE configs[4]: frame i matched to i-1
 * across shard boundaries; no reference counterpart, the reference runs one camera stream): frame f's
 * first counts[f] descriptor rows of desc (n_frames x cap x 32 bytes, the orbx_extract_batch_device
 * layout) go to out rows [incl[f] - counts[f], incl[f]), with incl the inclusive prefix sum of counts.
 * out holds out_rows rows: rows outside [0, out_rows) are not written, and a count outside [0, cap]
 * copies min(max(counts[f], 0), cap) rows (the device-side counts are never trusted to stay inside the
 * buffers).  counts / incl / desc / out are device memory; enqueue only on `stream`.  One launch,
 * 32-byte rows as two 16-byte vector copies. */
int orbx_pack_descriptors(const uint8_t* desc, int32_t cap, const int32_t* counts, const int32_t* incl,
                          int32_t n_frames, uint8_t* out, int32_t out_rows, void* stream);

/* Stage timing with HIP events recorded as part of each kernel's dispatch (hipExtLaunchKernel start /
 * stop events: the kernel's own duration) for the stages 0 pyramid, 1 FAST cells, 2 quadtree,
 * 3 describe.  enable > 0 times every stage, enable < 0 only the stages in the bitmask -enable
 * (e.g. -2: FAST cells only), 0 stops; read synchronises, returns the summed milliseconds and
 * launch count per stage, and resets. */
#define ORBX_NSTAGES 4
int orbx_profile_enable(orbx_extractor* h, int enable);
int orbx_profile_read(orbx_extractor* h, double* ms, int32_t* launches);

/* ------------------------------------------------------------------------------------------
 * Diagnostics (used by the per-stage parity tests; synchronous, host memory).
 * ---------------------------------------------------------------------------------------- */
/* FAST candidates of (frame, level) of the last batch, in DetectFAST's push order (cell raster,
 * row-major inside a cell): packed x | y << 12 | score << 24.  *n = count (cap-limited copy). */
int orbx_debug_level_candidates(const orbx_extractor* h, int frame, int level, uint32_t* out, int cap, int* n);
/* Runs the quadtree's on-device std::sort emulation (one wavefront) on `sizes`: perm[k] = index of
 * the element that std::sort(size-descending, src/ORBextractor.cc:642-643) puts at position k. */
int orbx_debug_qt_sort(const int32_t* sizes, int n, int32_t* perm);
/* PoseOptimization's cross-lane sums on one wavefront: in = 64 lanes x 32 doubles (lane-major);
 * scatter[l] = wave total of value l >> 1 (reduce-scatter butterfly), sum[l] = wave total of
 * in[*][0] (all-reduce).  Checks the permlane / DPP lane mapping against a host sum. */
int orbba_debug_po_wave(const double* in, double* scatter, double* sum);
/* Quadtree output of (frame, level) of the last batch (list order, packed as above). */
int orbx_debug_level_selected(const orbx_extractor* h, int frame, int level, uint32_t* out, int cap, int* n);

#ifdef __cplusplus
}
#endif
#endif /* ORBSLAM2_AMD_H */
