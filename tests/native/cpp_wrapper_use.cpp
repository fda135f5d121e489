// Compile-only check that the C++ drop-in wrapper builds against the C-ABI header.
#include "orbslam2_amd.hpp"

int use_wrapper() {
    ORB_SLAM2_AMD::ORBextractor::Parameters p(1000);
    (void)p;
    ORB_SLAM2_AMD::ORBmatcher m(0.6f, false);
    uint8_t a[32] = {0}, b[32] = {1};
    return ORB_SLAM2_AMD::ORBmatcher::DescriptorDistance(a, b) + (m.checkOrientation() ? 1 : 0);
}
