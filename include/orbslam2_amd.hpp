// orbslam2_amd.hpp — C++ drop-in classes over the C-ABI (include/orbslam2_amd.h).
//
// They keep the reference's class / method shapes so Tracking and LocalMapping call them
// unchanged:
//   ORB_SLAM2_AMD::ORBextractor   <- ORB_SLAM2::ORBextractor   (include/ORBextractor.h:35-81)
//   ORB_SLAM2_AMD::ORBmatcher     <- ORB_SLAM2::ORBmatcher Hamming kernels (include/ORBmatcher.h)
//   ORB_SLAM2_AMD::LocalBundleAdjustment <- Optimizer::LocalBundleAdjustment (include/Optimizer.h:47)
//   ORB_SLAM2_AMD::PoseOptimization      <- Optimizer::PoseOptimization (include/Optimizer.h:49)
//   ORB_SLAM2_AMD::SearchByProjection    <- ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)
//   ORB_SLAM2_AMD::ORBVocabulary         <- DBoW2 ORBVocabulary (include/ORBVocabulary.h) transform
// Plain-type overloads are always available; when OpenCV is on the include path the
// cv::Mat / cv::KeyPoint overloads with the reference's exact signatures are added.
// A non-zero C status is turned into an exception, as the reference's CV_Assert does.
#ifndef ORBSLAM2_AMD_HPP
#define ORBSLAM2_AMD_HPP

#include <algorithm>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "orbslam2_amd.h"

#if defined(__has_include)
#if __has_include(<opencv2/core.hpp>)
#include <opencv2/core.hpp>
#define ORBSLAM2_AMD_HAVE_OPENCV 1
#endif
#endif

namespace ORB_SLAM2_AMD {

inline void check(int rc, const char* what) {
    if (rc != ORB_OK) throw std::runtime_error(std::string(what) + ": " + orb_last_error());
}

class ORBextractor {
public:
    struct Parameters {   // include/ORBextractor.h:39-47
        int nfeatures;
        float scaleFactor;
        int nlevels;
        int iniThFAST;
        int minThFAST;
        Parameters(int nfeatures = 2000, float scaleFactor = 1.2f, int nlevels = 8, int iniThFAST = 20,
                   int minThFAST = 7)
            : nfeatures(nfeatures), scaleFactor(scaleFactor), nlevels(nlevels), iniThFAST(iniThFAST),
              minThFAST(minThFAST) {}
    };

    explicit ORBextractor(const Parameters& p, int device = 0) : param_(p) {
        orbx_params c{p.nfeatures, p.scaleFactor, p.nlevels, p.iniThFAST, p.minThFAST};
        check(orbx_create(&c, device, &h_), "orbx_create");
        const int L = p.nlevels;
        scale_.resize(L); inv_.resize(L); s2_.resize(L); is2_.resize(L);
        check(orbx_scale_tables(h_, scale_.data(), inv_.data(), s2_.data(), is2_.data(), nullptr), "orbx_scale_tables");
    }
    ~ORBextractor() { orbx_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // The OpenCV-build switches (orbslam2_amd.h orbx_set_opencv_compat): trig_mode 0
    // ::cos(double) / 1 cosf for src/ORBextractor.cc:107, resize_simd = the cv::resize SIMD width V.
    // -1 keeps a switch.
    void SetOpenCVCompat(int trig_mode, int resize_simd) {
        check(orbx_set_opencv_compat(h_, trig_mode, resize_simd), "orbx_set_opencv_compat");
    }

    // Extract on a raw CV_8U image.  Returns false (outputs untouched) when no keypoint exists —
    // the reference's early return (src/ORBextractor.cc:778-782).
    bool Extract(const uint8_t* img, int rows, int cols, size_t step, std::vector<orbx_keypoint>& keypoints,
                 std::vector<uint8_t>& descriptors) {
        int32_t cap = 0;
        check(orbx_max_keypoints(h_, rows, cols, &cap), "orbx_max_keypoints");
        kbuf_.resize(cap);
        dbuf_.resize((size_t)cap * 32);
        int n = 0;
        check(orbx_extract(h_, img, rows, cols, step, kbuf_.data(), dbuf_.data(), cap, &n), "orbx_extract");
        if (n == 0) {
            descriptors.clear();
            return false;
        }
        keypoints.assign(kbuf_.begin(), kbuf_.begin() + n);
        descriptors.assign(dbuf_.begin(), dbuf_.begin() + (size_t)n * 32);
        return true;
    }

#ifdef ORBSLAM2_AMD_HAVE_OPENCV
    // void Extract(const cv::Mat& image, KeyPoints& keypoints, cv::Mat& descriptors)
    void Extract(const cv::Mat& image, std::vector<cv::KeyPoint>& keypoints, cv::Mat& descriptors) {
        CV_Assert(image.type() == CV_8U);
        std::vector<orbx_keypoint> k;
        std::vector<uint8_t> d;
        if (!Extract(image.data, image.rows, image.cols, image.step, k, d)) {
            descriptors.release();   // keypoints left untouched, as the reference
            return;
        }
        keypoints.resize(k.size());
        for (size_t i = 0; i < k.size(); i++)
            keypoints[i] = cv::KeyPoint(k[i].x, k[i].y, k[i].size, k[i].angle, k[i].response, k[i].octave,
                                        k[i].class_id);
        descriptors.create((int)k.size(), 32, CV_8U);
        std::copy(d.begin(), d.end(), descriptors.data);
    }
#endif

    int GetLevels() const { return param_.nlevels; }
    float GetScaleFactor() const { return param_.scaleFactor; }
    const std::vector<float>& GetScaleFactors() const { return scale_; }
    const std::vector<float>& GetInverseScaleFactors() const { return inv_; }
    const std::vector<float>& GetScaleSigmaSquares() const { return s2_; }
    const std::vector<float>& GetInverseScaleSigmaSquares() const { return is2_; }

    // GetImagePyramid(): level s of the last image, copied to host memory.
    std::vector<uint8_t> GetImagePyramidLevel(int s, int* rows, int* cols) const {
        check(orbx_pyramid_level(h_, s, nullptr, 0, rows, cols), "orbx_pyramid_level");
        std::vector<uint8_t> out((size_t)(*rows) * (*cols));
        check(orbx_pyramid_level(h_, s, out.data(), (size_t)(*cols), rows, cols), "orbx_pyramid_level");
        return out;
    }

    orbx_extractor* handle() const { return h_; }

private:
    Parameters param_;
    orbx_extractor* h_ = nullptr;
    std::vector<float> scale_, inv_, s2_, is2_;
    std::vector<orbx_keypoint> kbuf_;
    std::vector<uint8_t> dbuf_;
};

class ORBmatcher {
public:
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : nnratio_(nnratio), checkOri_(checkOri) {}

    // static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) on 32-byte rows
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbm_descriptor_distance(a, b); }

    // Brute-force best / second-best + ratio test over all rows (reference loop semantics).  With
    // checkOri (the default, as the reference's ORBmatcher(nnratio, checkOri=true)) CheckOrientation
    // (ORBmatcher.cc:249-309) filters `match` as SearchForInitialization applies it (:676-686); the
    // keypoint angles are then required.  Returns the match count.
    int MatchBruteForce(const uint8_t* A, int nA, const uint8_t* B, int nB, std::vector<int>& match, int th_low = 50,
                        const float* angleA = nullptr, const float* angleB = nullptr) const {
        if (checkOri_ && (!angleA || !angleB))
            throw std::invalid_argument("ORBmatcher(checkOri=true)::MatchBruteForce needs the keypoint angles");
        std::vector<int32_t> bi(nA), bd(nA), sd(nA), m(nA);
        check(orbm_bf_match(A, nA, B, nB, nnratio_, th_low, bi.data(), bd.data(), sd.data(), m.data()), "orbm_bf_match");
        int32_t n = 0;
        for (int i = 0; i < nA; i++) n += m[i] >= 0;
        if (checkOri_) check(orbm_check_orientation(angleA, nA, angleB, nB, m.data(), &n), "orbm_check_orientation");
        match.assign(m.begin(), m.end());
        return n;
    }

    // int SearchForTriangulation(kf1, kf2, F12, matchIds, onlyStereo) on flattened keyframes.
    int SearchForTriangulation(const orbm_tri_frame& kf1, const orbm_tri_frame& kf2, const float F12[9],
                               const float ep2[2], const std::vector<float>& scale2, const std::vector<float>& sigma2,
                               std::vector<std::pair<size_t, size_t>>& matchIds, bool onlyStereo) const {
        std::vector<int32_t> m12(kf1.n);
        int32_t n = 0;
        check(orbm_search_for_triangulation(&kf1, &kf2, F12, ep2, scale2.data(), sigma2.data(), (int)scale2.size(),
                                            onlyStereo ? 1 : 0, m12.data(), &n),
              "orbm_search_for_triangulation");
        matchIds.clear();
        matchIds.reserve(n);
        for (int i = 0; i < kf1.n; i++)
            if (m12[i] >= 0) matchIds.emplace_back((size_t)i, (size_t)m12[i]);
        return n;
    }

    // int SearchByBoW(KeyFrame* keyframe, Frame& frame, std::vector<MapPoint*>& matches)
    // (src/ORBmatcher.cc:452-516), batched on HBM-resident slots: the batch's nnratio and
    // check_orientation are taken from this matcher.  Enqueue only; d_match[p*cap2 + idx2] = idx1 or -1
    // (the caller maps idx1 to keyframe->GetMapPointMatches()[idx1]), d_nmatches[p] = the return value.
    void SearchByBoWBatch(orbm_bow_batch b, int32_t* d_match, int32_t* d_nmatches, void* stream = nullptr) const {
        b.nnratio = nnratio_;
        b.check_orientation = checkOri_ ? 1 : 0;
        check(orbm_search_by_bow_batch_device(&b, d_match, d_nmatches, stream), "orbm_search_by_bow_batch_device");
    }

    // int SearchByBoW(KeyFrame* keyframe1, KeyFrame* keyframe2, std::vector<MapPoint*>& matches12)
    // (src/ORBmatcher.cc:696-766), batched: d_match12[p*cap1 + idx1] = idx2 or -1.
    void SearchByBoWKeyFramesBatch(orbm_bow_batch b, int32_t* d_match12, int32_t* d_nmatches,
                                   void* stream = nullptr) const {
        b.nnratio = nnratio_;
        b.check_orientation = checkOri_ ? 1 : 0;
        check(orbm_search_by_bow_kf_batch_device(&b, d_match12, d_nmatches, stream), "orbm_search_by_bow_kf_batch_device");
    }

    // int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& prevMatched,
    //                             std::vector<int>& matches12, int windowSize = 10)
    // (include/ORBmatcher.h:81, src/ORBmatcher.cc:614-694) on the frames' keypointsUn (cv::KeyPoint
    // layout), 32-byte descriptors and F2's image bounds; prevMatched as (x, y) pairs, updated in place.
    // nnratio / checkOri are this matcher's (Tracking.cc:1051 builds ORBmatcher(0.9f, true)).
    int SearchForInitialization(const std::vector<orbx_keypoint>& keypointsUn1, const uint8_t* descriptors1,
                                const std::vector<orbx_keypoint>& keypointsUn2, const uint8_t* descriptors2,
                                const float bounds2[4], std::vector<float>& prevMatched, std::vector<int>& matches12,
                                int windowSize = 10, int device = 0) const {
        const int n1 = (int)keypointsUn1.size(), n2 = (int)keypointsUn2.size();
        if ((int)prevMatched.size() != 2 * n1)
            throw std::invalid_argument("SearchForInitialization: prevMatched must hold 2 floats per F1 keypoint");
        std::vector<float> xy2(2 * (size_t)n2), ang2(n2), ang1(n1);
        std::vector<int32_t> oct2(n2), oct1(n1);
        for (int i = 0; i < n2; i++) {
            xy2[2 * i] = keypointsUn2[i].x; xy2[2 * i + 1] = keypointsUn2[i].y;
            oct2[i] = keypointsUn2[i].octave; ang2[i] = keypointsUn2[i].angle;
        }
        for (int i = 0; i < n1; i++) { oct1[i] = keypointsUn1[i].octave; ang1[i] = keypointsUn1[i].angle; }
        const int32_t kb[2] = {0, n2}, qb[2] = {0, n1};
        orbm_init_batch b;
        b.n_pairs = 1; b.total_kp = n2; b.total_q = n1;
        b.kp_begin = kb; b.kp_xy = xy2.data(); b.kp_octave = oct2.data(); b.kp_desc = descriptors2; b.kp_angle = ang2.data();
        b.bounds = bounds2; b.q_begin = qb; b.q_octave = oct1.data(); b.q_desc = descriptors1; b.q_angle = ang1.data();
        b.prev_matched = prevMatched.data(); b.window = windowSize; b.nnratio = nnratio_;
        b.check_orientation = checkOri_ ? 1 : 0;
        std::vector<int32_t> m(std::max(n1, 1));
        int32_t nm = 0;
        check(orbm_search_for_initialization(&b, m.data(), &nm, device), "orbm_search_for_initialization");
        matches12.assign(m.begin(), m.begin() + n1);
        return nm;
    }

    // The same batched over initialisation pairs on HBM arrays (orbm_init_batch; nnratio / checkOri from
    // this matcher).  Enqueue only.
    void SearchForInitializationBatch(orbm_init_batch b, int32_t* d_matches12, int32_t* d_n_matches,
                                      void* stream = nullptr) const {
        b.nnratio = nnratio_;
        b.check_orientation = checkOri_ ? 1 : 0;
        check(orbm_search_for_initialization_device(&b, d_matches12, d_n_matches, stream),
              "orbm_search_for_initialization_device");
    }

    float nnratio() const { return nnratio_; }
    bool checkOrientation() const { return checkOri_; }

private:
    float nnratio_;
    bool checkOri_;
};

// void ComputeStereoMatches(keypointsL, descriptorsL, pyramidL, keypointsR, descriptorsR, pyramidR,
//                           scaleFactors, invScaleFactors, camera, uright, depth)  (src/ORBmatcher.cc:72-247)
// on raw arrays: keypoints in cv::KeyPoint layout, 32-byte descriptors, pyramid level pointers.
struct PyramidView {
    std::vector<const uint8_t*> level;
    std::vector<int32_t> rows, cols, step;
};

inline void ComputeStereoMatches(const std::vector<orbx_keypoint>& keypointsL, const uint8_t* descriptorsL,
                                 const PyramidView& pyramidL, const std::vector<orbx_keypoint>& keypointsR,
                                 const uint8_t* descriptorsR, const PyramidView& pyramidR,
                                 const std::vector<float>& scaleFactors, const std::vector<float>& invScaleFactors,
                                 float bf, float baseline, std::vector<float>& uright, std::vector<float>& depth) {
    auto view = [](const std::vector<orbx_keypoint>& k, const uint8_t* d, const PyramidView& p) {
        orbm_stereo_view v;
        v.n = (int32_t)k.size();
        v.kps = k.data();
        v.desc = d;
        v.n_levels = (int32_t)p.level.size();
        v.level = p.level.data();
        v.level_rows = p.rows.data();
        v.level_cols = p.cols.data();
        v.level_step = p.step.data();
        return v;
    };
    const orbm_stereo_view l = view(keypointsL, descriptorsL, pyramidL), r = view(keypointsR, descriptorsR, pyramidR);
    uright.assign(keypointsL.size(), -1.f);
    depth.assign(keypointsL.size(), -1.f);
    check(orbm_compute_stereo_matches(&l, &r, scaleFactors.data(), invScaleFactors.data(), bf, baseline, uright.data(),
                                      depth.data()),
          "orbm_compute_stereo_matches");
}

// The same on the two extractors' last Extract (System.cc:449-461): keypoints, descriptors and pyramids stay
// on the device; only uright / depth come back.  nLeft = keypointsLeft.size() of that Extract.
inline void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, size_t nLeft, float bf, float baseline,
                                 std::vector<float>& uright, std::vector<float>& depth) {
    uright.assign(nLeft, -1.f);
    depth.assign(nLeft, -1.f);
    check(orbx_stereo_matches_last(left.handle(), right.handle(), bf, baseline, uright.data(), depth.data(),
                                   (int)nLeft),
          "orbx_stereo_matches_last");
}

// Optimizer::LocalBundleAdjustment from the flattened graph (Optimizer.cc:540-631): the caller
// gathers local / fixed keyframes and local map points exactly as :493-537, calls this, then
// erases the outlier observations and writes poses / points back under the map mutex (:677-735).
// Returns false when the stop flag was already set on entry (the reference returns at
// Optimizer.cc:633-634): nothing was optimised and nothing must be written back.
inline bool LocalBundleAdjustment(const orbba_problem& problem, orbba_result& result, const volatile int32_t* stopFlag,
                                  int device = 0) {
    check(orbba_local_ba(&problem, &result, stopFlag, device), "orbba_local_ba");
    return result.ran != 0;
}

// int Optimizer::PoseOptimization(Frame*) (include/Optimizer.h:49, src/Optimizer.cc:345-489) over a
// batch of frames.  One PoseFrame per frame holds the keypoints that have a map point, in keypoint
// order (:364-410); R / t are frame->pose on entry and the SetPose argument on return, `outlier`
// receives frame->outlier for those keypoints.  Returns each frame's inlier count.
struct PoseFrame {
    double R[9], t[3];
    double fx, fy, cx, cy, bf;
    std::vector<double> xw;         // 3 per edge: MapPoint::GetWorldPos()
    std::vector<double> obs;        // 3 per edge: keypointsUn[i].pt.x, .y, uright[i] (< 0: monocular)
    std::vector<double> invSigma2;  // 1 per edge: pyramid.invSigmaSq[keypointsUn[i].octave]
    std::vector<uint8_t> outlier;   // out
};

inline std::vector<int> PoseOptimization(std::vector<PoseFrame>& frames, int device = 0) {
    const size_t F = frames.size();
    std::vector<int32_t> eb(F + 1, 0);
    for (size_t f = 0; f < F; f++) eb[f + 1] = eb[f] + (int32_t)frames[f].invSigma2.size();
    const size_t E = (size_t)eb[F];
    std::vector<double> R(9 * F), t(3 * F), cam(5 * F), xw(3 * E), obs(3 * E), is2(E);
    for (size_t f = 0; f < F; f++) {
        const PoseFrame& p = frames[f];
        std::copy(p.R, p.R + 9, R.begin() + 9 * f);
        std::copy(p.t, p.t + 3, t.begin() + 3 * f);
        const double c[5] = {p.fx, p.fy, p.cx, p.cy, p.bf};
        std::copy(c, c + 5, cam.begin() + 5 * f);
        std::copy(p.xw.begin(), p.xw.end(), xw.begin() + 3 * (size_t)eb[f]);
        std::copy(p.obs.begin(), p.obs.end(), obs.begin() + 3 * (size_t)eb[f]);
        std::copy(p.invSigma2.begin(), p.invSigma2.end(), is2.begin() + eb[f]);
    }
    std::vector<double> oR(9 * F), ot(3 * F);
    std::vector<int32_t> ninl(F);
    std::vector<uint8_t> outl(E);
    const orbba_pose_batch in{(int32_t)F, eb.data(), R.data(), t.data(), cam.data(), xw.data(), obs.data(), is2.data()};
    orbba_pose_result out{oR.data(), ot.data(), ninl.data(), outl.data()};
    check(orbba_pose_optimization(&in, &out, device), "orbba_pose_optimization");
    std::vector<int> result(F);
    for (size_t f = 0; f < F; f++) {
        PoseFrame& p = frames[f];
        std::copy(oR.begin() + 9 * f, oR.begin() + 9 * f + 9, p.R);
        std::copy(ot.begin() + 3 * f, ot.begin() + 3 * f + 3, p.t);
        p.outlier.assign(outl.begin() + eb[f], outl.begin() + eb[f + 1]);
        result[f] = ninl[f];
    }
    return result;
}

// int ORBmatcher::SearchByProjection(Frame&, const std::vector<MapPoint*>&, float th)
// (include/ORBmatcher.h:58, src/ORBmatcher.cc:315-382) with the frame's FeaturesGrid, for one
// frame.  `keypointsUn` / `descriptors` / `uright` are the frame's, `claimed[i]` is
// frame.mappoints[i] && ->Observations() > 0; per local map point the IsInFrustum fields
// (Tracking.cc:554-605).  Returns the match count; kpMatch[i] = index into the map point arrays
// assigned to keypoint i (frame.mappoints[i] = mappoints[kpMatch[i]]) or -1.
struct ProjectionPoints {
    std::vector<uint8_t> valid;      // trackInView && !isBad()
    std::vector<float> proj;         // 3 per point: trackProjX, trackProjY, trackProjXR
    std::vector<float> viewCos;      // trackViewCos
    std::vector<int32_t> level;      // trackScaleLevel
    std::vector<uint8_t> desc;       // 32 per point: GetDescriptor()
    std::vector<uint8_t> hasObs;     // Observations() > 0
};

inline int SearchByProjection(const std::vector<orbx_keypoint>& keypointsUn, const uint8_t* descriptors,
                              const std::vector<float>& uright, const std::vector<uint8_t>& claimed,
                              const float bounds[4], const std::vector<float>& scaleFactors,
                              const ProjectionPoints& mps, float th, float nnratio, std::vector<int32_t>& kpMatch,
                              int device = 0) {
    const int n = (int)keypointsUn.size(), m = (int)mps.valid.size();
    std::vector<float> xy(2 * (size_t)n);
    std::vector<int32_t> oct(n);
    for (int i = 0; i < n; i++) { xy[2 * i] = keypointsUn[i].x; xy[2 * i + 1] = keypointsUn[i].y; oct[i] = keypointsUn[i].octave; }
    const int32_t kb[2] = {0, n}, mb[2] = {0, m};
    orbm_proj_batch b;
    b.n_frames = 1; b.total_kp = n; b.total_mp = m;
    b.kp_begin = kb; b.kp_xy = xy.data(); b.kp_octave = oct.data(); b.kp_uright = uright.data();
    b.kp_desc = descriptors; b.kp_claimed = claimed.empty() ? nullptr : claimed.data(); b.bounds = bounds;
    b.mp_begin = mb; b.mp_valid = mps.valid.data(); b.mp_proj = mps.proj.data(); b.mp_view_cos = mps.viewCos.data();
    b.mp_level = mps.level.data(); b.mp_desc = mps.desc.data(); b.mp_has_obs = mps.hasObs.data();
    b.n_levels = (int32_t)scaleFactors.size(); b.scale_factors = scaleFactors.data(); b.th = th; b.nnratio = nnratio;
    kpMatch.assign(n, -1);
    int32_t nm = 0;
    check(orbm_search_by_projection(&b, kpMatch.data(), &nm, device), "orbm_search_by_projection");
    return nm;
}

// int ORBmatcher::SearchByProjection(Frame& currFrame, const Frame& lastFrame, float th, bool monocular)
// (src/ORBmatcher.cc:1279-1362), batched on HBM arrays (orbm_motion_batch: the caller projects the
// last frame's points with the motion-model pose and sets motion[f] from tlc / baseline, :1286-1288).
// Enqueue only; kp_match[k] = idx1 assigned to currFrame keypoint k or -1.
inline void SearchByProjectionMotionBatch(const orbm_motion_batch& b, int32_t* d_kp_match, int32_t* d_n_matches,
                                          void* stream = nullptr) {
    check(orbm_search_by_projection_motion_device(&b, d_kp_match, d_n_matches, stream),
          "orbm_search_by_projection_motion_device");
}

// int ORBmatcher::SearchByProjection(Frame& frame, KeyFrame* keyframe, const std::set<MapPoint*>& alreadyFound,
// float th, int ORBdist) (include/ORBmatcher.h:66, src/ORBmatcher.cc:1364-1445), batched over (frame,
// candidate keyframe) pairs on HBM arrays (orbm_reloc_batch: the caller marks mp_valid = mappoint &&
// !isBad() && !alreadyFound.count(mappoint) and kp_claimed = frame.mappoints[i] != nullptr).  Enqueue
// only; kp_match[k] = keyframe idx1 assigned to frame keypoint k (frame.mappoints[k] =
// keyframe->GetMapPointMatches()[idx1]) or -1.
inline void SearchByProjectionRelocBatch(const orbm_reloc_batch& b, int32_t* d_kp_match, int32_t* d_n_matches,
                                         void* stream = nullptr) {
    check(orbm_search_by_projection_reloc_device(&b, d_kp_match, d_n_matches, stream),
          "orbm_search_by_projection_reloc_device");
}
// The same for one (frame, keyframe) pair on host arrays.
inline int SearchByProjectionReloc(const orbm_reloc_batch& b, std::vector<int32_t>& kpMatch, int device = 0) {
    if (b.n_frames != 1) throw std::invalid_argument("SearchByProjectionReloc: one frame per call (use the batch form)");
    kpMatch.assign(std::max(b.total_kp, 1), -1);
    int32_t nm = 0;
    check(orbm_search_by_projection_reloc(&b, kpMatch.data(), &nm, device), "orbm_search_by_projection_reloc");
    kpMatch.resize(b.total_kp);
    return nm;
}

// DBoW2 ORBVocabulary: loadFromTextFile + transform(features, BowVector&, FeatureVector&, levelsup)
// (TemplatedVocabulary.h:1130-1196, :1341-1431) with the reference's container types.
class ORBVocabulary {
public:
    using BowVector = std::map<uint32_t, double>;
    using FeatureVector = std::map<uint32_t, std::vector<unsigned int>>;

    explicit ORBVocabulary(int device = 0) : device_(device) {}
    ~ORBVocabulary() { orbv_destroy(h_); }
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;

    bool loadFromTextFile(const std::string& filename) {
        orbv_destroy(h_);
        h_ = nullptr;
        return orbv_load_text(filename.c_str(), device_, &h_) == ORB_OK;
    }
    bool empty() const {
        int nw = 0;
        return !h_ || orbv_info(h_, nullptr, nullptr, nullptr, &nw, nullptr, nullptr) != ORB_OK || nw == 0;
    }
    // descriptors: n rows of 32 bytes (Converter::toDescriptorVector(descriptors))
    void transform(const uint8_t* descriptors, int n, BowVector& v, FeatureVector& fv, int levelsup) const {
        v.clear();
        fv.clear();
        if (!h_) return;
        const size_t cap = (size_t)std::max(n, 1);
        std::vector<uint32_t> bw(cap), fn(cap);
        std::vector<double> bv(cap);
        std::vector<int32_t> fo(cap + 1), fi(cap);
        int nw = 0, nn = 0;
        check(orbv_transform(h_, descriptors, n, levelsup, bw.data(), bv.data(), &nw, fn.data(), fo.data(), fi.data(),
                             &nn),
              "orbv_transform");
        for (int i = 0; i < nw; i++) v.emplace_hint(v.end(), bw[i], bv[i]);
        for (int t = 0; t < nn; t++)
            fv.emplace_hint(fv.end(), fn[t], std::vector<unsigned int>(fi.begin() + fo[t], fi.begin() + fo[t + 1]));
    }

private:
    int device_;
    orbv_vocabulary* h_ = nullptr;
};

}  // namespace ORB_SLAM2_AMD

#endif  // ORBSLAM2_AMD_HPP
