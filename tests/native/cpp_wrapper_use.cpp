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
