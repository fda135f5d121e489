// Compares orbamd::qt_sort (the device emulation) with the real libstdc++ std::sort on the
// quadtree's DivisibleNode comparator (src/ORBextractor.cc:642-643).  Prints "OK <cases>" or the
// first mismatch.  Built and run by tests/test_qt_sort.py.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "qt_sort.h"

struct DivisibleNode { size_t size; const int* ptr; };

int main(int argc, char** argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937 rng(12345);
    static int tags[5000];
    for (int c = 0; c < cases; c++) {
        const int n = std::uniform_int_distribution<int>(0, c % 10 == 0 ? 3000 : 300)(rng);
        const int maxv = std::uniform_int_distribution<int>(1, 40)(rng);
        std::vector<DivisibleNode> ref(n);
        std::vector<orbamd::QtItem> emu(n);
        for (int i = 0; i < n; i++) {
            const int v = std::uniform_int_distribution<int>(2, 1 + maxv)(rng);
            ref[i] = {(size_t)v, &tags[i]};
            emu[i] = {v, i};
        }
        if (c % 7 == 3) {  // adversarial-ish: sorted / reverse sorted inputs
            std::sort(ref.begin(), ref.end(), [](const DivisibleNode& a, const DivisibleNode& b) { return a.size < b.size; });
            for (int i = 0; i < n; i++) emu[i] = {(int)ref[i].size, (int)(ref[i].ptr - tags)};
        }
        std::sort(ref.begin(), ref.end(), [](const DivisibleNode& a, const DivisibleNode& b) { return a.size > b.size; });
        std::vector<orbamd::QtItem> par = emu;
        orbamd::qt_sort(emu.data(), emu.data() + n);
        std::vector<int> Ls(n + 1), Rs(n + 1), sl(n + 1), sn(n + 1);
        std::vector<orbamd::QtItem> tmp(n + 1);
        orbamd::qt_sort_parallel_form(par.data(), n, Ls.data(), Rs.data(), sl.data(), sn.data(), tmp.data());
        for (int i = 0; i < n; i++) {
            if ((int)(ref[i].ptr - tags) != emu[i].node || (int)ref[i].size != emu[i].size) {
                printf("MISMATCH case %d n %d at %d\n", c, n, i);
                return 1;
            }
            if (par[i].node != emu[i].node) {
                printf("PARALLEL-FORM MISMATCH case %d n %d at %d\n", c, n, i);
                return 1;
            }
        }
    }
    // heap-sort fallback == std::partial_sort(first, last, last) (std::__partial_sort)
    for (int c = 0; c < cases / 10; c++) {
        const int n = std::uniform_int_distribution<int>(0, 500)(rng);
        std::vector<DivisibleNode> ref(n);
        std::vector<orbamd::QtItem> emu(n);
        for (int i = 0; i < n; i++) {
            const int v = std::uniform_int_distribution<int>(2, 12)(rng);
            ref[i] = {(size_t)v, &tags[i]};
            emu[i] = {v, i};
        }
        std::partial_sort(ref.begin(), ref.end(), ref.end(), [](const DivisibleNode& a, const DivisibleNode& b) { return a.size > b.size; });
        orbamd::qt_heap_sort(emu.data(), emu.data() + n);
        for (int i = 0; i < n; i++)
            if ((int)(ref[i].ptr - tags) != emu[i].node) { printf("HEAP MISMATCH case %d at %d\n", c, i); return 1; }
    }
    printf("OK %d\n", cases);
    return 0;
}
