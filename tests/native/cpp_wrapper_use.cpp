// Compile-only check that the C++ drop-in wrapper builds against the C-ABI header.
#include "orbslam2_amd.hpp"

int use_wrapper() {
    ORB_SLAM2_AMD::ORBextractor::Parameters p(1000);
    (void)p;
    ORB_SLAM2_AMD::ORBmatcher m(0.6f, false);
    uint8_t a[32] = {0}, b[32] = {1};
    return ORB_SLAM2_AMD::ORBmatcher::DescriptorDistance(a, b) + (m.checkOrientation() ? 1 : 0);
}

void use_stereo(const std::vector<orbx_keypoint>& kl, const uint8_t* dl, const std::vector<orbx_keypoint>& kr,
                const uint8_t* dr, const ORB_SLAM2_AMD::PyramidView& pl, const ORB_SLAM2_AMD::PyramidView& pr,
                const std::vector<float>& s, const std::vector<float>& inv) {
    std::vector<float> ur, depth;
    ORB_SLAM2_AMD::ComputeStereoMatches(kl, dl, pl, kr, dr, pr, s, inv, 386.1448f, 0.537f, ur, depth);
}

int use_pose(std::vector<ORB_SLAM2_AMD::PoseFrame>& frames) {
    const std::vector<int> n = ORB_SLAM2_AMD::PoseOptimization(frames);
    return n.empty() ? 0 : n[0];
}

int use_projection(const std::vector<orbx_keypoint>& k, const uint8_t* d, const std::vector<float>& ur,
                   const ORB_SLAM2_AMD::ProjectionPoints& mps, const std::vector<float>& scale) {
    const float bounds[4] = {0.f, 1241.f, 0.f, 376.f};
    std::vector<int32_t> match;
    return ORB_SLAM2_AMD::SearchByProjection(k, d, ur, {}, bounds, scale, mps, 1.f, 0.8f, match);
}

size_t use_vocabulary(const uint8_t* desc, int n) {
    ORB_SLAM2_AMD::ORBVocabulary voc;
    if (!voc.loadFromTextFile("ORBvoc.txt")) return 0;
    ORB_SLAM2_AMD::ORBVocabulary::BowVector v;
    ORB_SLAM2_AMD::ORBVocabulary::FeatureVector fv;
    voc.transform(desc, n, v, fv, 4);
    return v.size() + fv.size();
}
