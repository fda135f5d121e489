// For every float keypoint angle in [0, 360] (the range of cv::fastAtan2, ORBextractor.cc:100): do the
// two readings of ComputeOrbDescriptor's `cos(angle)` / `sin(angle)` (:105-107) -- ::cos(double) vs
// std::cos(float) = cosf -- give a different sample offset for any of the 512 rBRIEF points
// (:111-113, cvRound(x*b + y*a), cvRound(x*a - y*b), no FMA)?  If no offset differs, the descriptor
// is identical whatever the image.  Build: g++ -O2 -ffp-contract=off -pthread -I<csrc>.
// Prints the number of angles whose (a, b) differ and the number whose offsets differ.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static const float kPattern[1024] = {
#include "orb_pattern31.inc"
};

int main() {
    const float lo = 0.f, hi = 360.f;
    unsigned a0, a1;
    memcpy(&a0, &lo, 4);
    memcpy(&a1, &hi, 4);
    std::atomic<unsigned long long> n_ab{0}, n_off{0}, n_tot{0};
    std::vector<std::thread> th;
    const int nt = 8;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            unsigned long long ab = 0, off = 0, tot = 0;
            for (unsigned u = a0 + t; u <= a1; u += nt) {
                float ang;
                memcpy(&ang, &u, 4);
                const float factorPI = (float)(M_PI / 180.f);
                const float angle = ang * factorPI;
                const float ad = (float)std::cos((double)angle), bd = (float)std::sin((double)angle);
                const float af = std::cos(angle), bf = std::sin(angle);
                tot++;
                if (ad == af && bd == bf) continue;
                ab++;
                for (int i = 0; i < 512; i++) {
                    const float x = kPattern[2 * i], y = kPattern[2 * i + 1];
                    const int r0 = (int)lrintf(x * bd + y * ad), c0 = (int)lrintf(x * ad - y * bd);
                    const int r1 = (int)lrintf(x * bf + y * af), c1 = (int)lrintf(x * af - y * bf);
                    if (r0 != r1 || c0 != c1) {
                        if (off < 3) printf("angle %.9g (0x%08x): point %d offset (%d,%d) vs (%d,%d)\n", ang, u, i, r0, c0, r1, c1);
                        off++;
                        break;
                    }
                }
            }
            n_ab += ab;
            n_off += off;
            n_tot += tot;
        });
    for (auto& x : th) x.join();
    printf("angles %llu, (a,b) differ %llu, some sample offset differs %llu\n", (unsigned long long)n_tot,
           (unsigned long long)n_ab, (unsigned long long)n_off);
    return 0;
}
