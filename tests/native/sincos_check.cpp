// Compares orbamd::sincos_f2d against glibc (float)sin / (float)cos of (double)x (mode d, default) or
// orbamd::sincosf_glibc against glibc sinf / cosf (mode f) for every float x in [lo, hi) (default
// [0, 6.2832]), split over threads.  Build: g++ -O2 -ffp-contract=off -pthread.
// Usage: sincos_check [threads] [step] [d|f|t]   (d: the fdlibm form sincos_f2d that describe uses, t: the
// table form sincos_f2d_tab, both against (float)sin / cos((double)x); f: sincosf_glibc against sinf / cosf)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <atomic>

#include "../../orb_slam2_refactored_amd/csrc/sincos_f.h"

int main(int argc, char** argv) {
    float lo = 0.f, hi = 6.2832f;
    int nt = argc > 1 ? atoi(argv[1]) : 8;
    unsigned step = argc > 2 ? (unsigned)atoi(argv[2]) : 1;   // test every step-th float
    const bool fmode = argc > 3 && argv[3][0] == 'f';
    const bool tmode = argc > 3 && argv[3][0] == 't';
    unsigned a, b;
    memcpy(&a, &lo, 4);
    memcpy(&b, &hi, 4);
    std::atomic<unsigned long long> bad{0}, tested{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            unsigned long long nb = 0, nn = 0;
            for (unsigned u = a + (unsigned)t * step; u < b; u += (unsigned)nt * step) {
                float x;
                memcpy(&x, &u, 4);
                float s, c;
                float rs, rc;
                if (fmode) {
                    orbamd::sincosf_glibc(x, &s, &c);
                    rs = ::sinf(x);
                    rc = ::cosf(x);
                } else {
                    if (tmode) orbamd::sincos_f2d_tab(x, &s, &c);
                    else orbamd::sincos_f2d(x, &s, &c);
                    rs = (float)::sin((double)x);
                    rc = (float)::cos((double)x);
                }
                if (memcmp(&s, &rs, 4) || memcmp(&c, &rc, 4)) {
                    if (nb < 5) printf("mismatch x=%.9g (0x%08x): s %.9g vs %.9g, c %.9g vs %.9g\n", x, u, s, rs, c, rc);
                    nb++;
                }
                nn++;
            }
            bad += nb;
            tested += nn;
        });
    for (auto& x : th) x.join();
    printf("tested %llu floats, %llu mismatches\n", (unsigned long long)tested, (unsigned long long)bad);
    return bad != 0;
}
