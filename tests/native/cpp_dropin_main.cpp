// Executes the C++ drop-in classes of include/orbslam2_amd.hpp on the GPU (the boundary the reference
// would link), for tests/test_cpp_dropin_gpu.py.  Raw little-endian binary files in and out:
//
//   cpp_dropin extract  <dir>   image.u8 (rows x cols), meta.i32 {rows, cols, nfeatures}
//                               -> kps.i32 (n x 7, cv::KeyPoint layout), desc.u8 (n x 32), n.i32
//   cpp_dropin match    <dir>   A.u8 (nA x 32), B.u8 (nB x 32), angA.f32, angB.f32, meta.i32 {nA, nB, checkOri}
//                               -> match.i32 (nA), n.i32
//   cpp_dropin localba  <dir>   meta.i32 {P, N, E, stop}, pose_R.f64, pose_t.f64, pose_fixed.u8, points.f64,
//                               edge_point.i32, edge_pose.i32, edge_obs.f64, edge_inv_sigma2.f64, edge_cam.f64
//                               -> out_pose_R.f64, out_pose_t.f64, out_points.f64, out_outlier.u8,
//                                  out_iterations.i32 (2), out_ran.i32
//   cpp_dropin localba_twice <dir>  as localba, twice on the same thread (context reuse)
//   cpp_dropin stereo   <dir>   left.u8, right.u8 (rows x cols), meta.i32 {rows, cols, nfeatures}, cam.f32 {bf, baseline}
//                               -> uright.f32, depth.f32 (nL each), nL.i32: Extract L and R on two std::threads
//                               and ComputeStereoMatches on the two extractors (System.cc:449-461)
#include <cstdio>
#include <thread>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "orbslam2_amd.hpp"

template <class T>
static std::vector<T> load(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot open " + path);
    const std::streamsize n = f.tellg();
    f.seekg(0);
    std::vector<T> v((size_t)n / sizeof(T));
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    return v;
}

template <class T>
static void save(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

static int run_extract(const std::string& d) {
    const auto meta = load<int32_t>(d + "/meta.i32");
    const auto img = load<uint8_t>(d + "/image.u8");
    ORB_SLAM2_AMD::ORBextractor ex{ORB_SLAM2_AMD::ORBextractor::Parameters{meta[2]}};
    std::vector<orbx_keypoint> kps;
    std::vector<uint8_t> desc;
    const bool any = ex.Extract(img.data(), meta[0], meta[1], (size_t)meta[1], kps, desc);
    const int32_t n = any ? (int32_t)kps.size() : 0;
    save(d + "/kps.i32", reinterpret_cast<const int32_t*>(kps.data()), (size_t)n * 7);
    save(d + "/desc.u8", desc.data(), (size_t)n * 32);
    save(d + "/n.i32", &n, 1);
    return 0;
}

static int run_match(const std::string& d) {
    const auto meta = load<int32_t>(d + "/meta.i32");
    const auto A = load<uint8_t>(d + "/A.u8");
    const auto B = load<uint8_t>(d + "/B.u8");
    const auto angA = load<float>(d + "/angA.f32");
    const auto angB = load<float>(d + "/angB.f32");
    ORB_SLAM2_AMD::ORBmatcher m(0.6f, meta[2] != 0);
    std::vector<int> match;
    int32_t n = m.MatchBruteForce(A.data(), meta[0], B.data(), meta[1], match, 50, angA.data(), angB.data());
    // without angles, a checkOri matcher must refuse (the reference would run the filter)
    bool threw = false;
    try {
        std::vector<int> tmp;
        m.MatchBruteForce(A.data(), meta[0], B.data(), meta[1], tmp);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    if (threw != (meta[2] != 0)) {
        std::cerr << "checkOri without angles: unexpected behaviour\n";
        return 3;
    }
    std::vector<int32_t> m32(match.begin(), match.end());
    save(d + "/match.i32", m32.data(), m32.size());
    save(d + "/n.i32", &n, 1);
    return 0;
}

static int run_localba(const std::string& d, int reps) {
    const auto meta = load<int32_t>(d + "/meta.i32");
    const int P = meta[0], N = meta[1], E = meta[2];
    const auto R = load<double>(d + "/pose_R.f64");
    const auto t = load<double>(d + "/pose_t.f64");
    const auto fixed = load<uint8_t>(d + "/pose_fixed.u8");
    const auto X = load<double>(d + "/points.f64");
    const auto ep = load<int32_t>(d + "/edge_point.i32");
    const auto ek = load<int32_t>(d + "/edge_pose.i32");
    const auto obs = load<double>(d + "/edge_obs.f64");
    const auto info = load<double>(d + "/edge_inv_sigma2.f64");
    const auto cam = load<double>(d + "/edge_cam.f64");
    const orbba_problem pr{P, R.data(), t.data(), fixed.data(), N, X.data(), E, ep.data(), ek.data(), obs.data(),
                           info.data(), cam.data()};
    std::vector<double> oR(9 * (size_t)P), ot(3 * (size_t)P), oX(3 * (size_t)N);
    std::vector<uint8_t> outl(E);
    orbba_result res{};
    res.pose_R = oR.data();
    res.pose_t = ot.data();
    res.points = oX.data();
    res.edge_outlier = outl.data();
    volatile int32_t stop = meta[3];
    bool ran = false;
    for (int r = 0; r < reps; r++) ran = ORB_SLAM2_AMD::LocalBundleAdjustment(pr, res, &stop);
    const int32_t ran32 = ran ? 1 : 0;
    save(d + "/out_pose_R.f64", oR.data(), oR.size());
    save(d + "/out_pose_t.f64", ot.data(), ot.size());
    save(d + "/out_points.f64", oX.data(), oX.size());
    save(d + "/out_outlier.u8", outl.data(), outl.size());
    save(d + "/out_iterations.i32", res.iterations, 2);
    save(d + "/out_ran.i32", &ran32, 1);
    return 0;
}

static int run_stereo(const std::string& d) {
    const auto meta = load<int32_t>(d + "/meta.i32");
    const auto L = load<uint8_t>(d + "/left.u8");
    const auto R = load<uint8_t>(d + "/right.u8");
    const auto cam = load<float>(d + "/cam.f32");
    ORB_SLAM2_AMD::ORBextractor exL{ORB_SLAM2_AMD::ORBextractor::Parameters{meta[2]}};
    ORB_SLAM2_AMD::ORBextractor exR{ORB_SLAM2_AMD::ORBextractor::Parameters{meta[2]}};
    std::vector<orbx_keypoint> kL, kR;
    std::vector<uint8_t> dL, dR;
    std::thread tL([&] { exL.Extract(L.data(), meta[0], meta[1], (size_t)meta[1], kL, dL); });
    std::thread tR([&] { exR.Extract(R.data(), meta[0], meta[1], (size_t)meta[1], kR, dR); });
    tL.join();
    tR.join();
    std::vector<float> uright, depth;
    ORB_SLAM2_AMD::ComputeStereoMatches(exL, exR, kL.size(), cam[0], cam[1], uright, depth);
    const int32_t n = (int32_t)kL.size();
    save(d + "/uright.f32", uright.data(), uright.size());
    save(d + "/depth.f32", depth.data(), depth.size());
    save(d + "/nL.i32", &n, 1);
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 3) {
        std::cerr << "usage: cpp_dropin extract|match|localba|localba_twice|stereo <dir>\n";
        return 2;
    }
    const std::string mode = argv[1], dir = argv[2];
    try {
        if (mode == "extract") return run_extract(dir);
        if (mode == "match") return run_match(dir);
        if (mode == "localba") return run_localba(dir, 1);
        if (mode == "localba_twice") return run_localba(dir, 2);
        if (mode == "stereo") return run_stereo(dir);
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
    std::cerr << "unknown mode\n";
    return 2;
}
