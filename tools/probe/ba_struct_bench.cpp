// Host timing of the LocalBA structure build (csrc/ba_structure.h) on a graph dumped by
// tools/probe/ba_struct_dump.py: P, N, E, fixed[P] (u8), ep[E], ek[E] (i32).  Prints µs per build and a
// checksum of the arrays (to compare builds).  g++ -O3 -I orb_slam2_refactored_amd/csrc
#include <chrono>
#include <cstdio>
#include <vector>

#include "ba_structure.h"

int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "/tmp/c4_graph.bin", "rb");
    if (!f) return 1;
    int P, N, E;
    if (fread(&P, 4, 1, f) != 1 || fread(&N, 4, 1, f) != 1 || fread(&E, 4, 1, f) != 1) return 1;
    std::vector<uint8_t> fixed(P);
    std::vector<int> ep(E), ek(E);
    if (fread(fixed.data(), 1, P, f) != (size_t)P || fread(ep.data(), 4, E, f) != (size_t)E ||
        fread(ek.data(), 4, E, f) != (size_t)E)
        return 1;
    fclose(f);
    std::vector<uint8_t> level(E, 0);
    orbamd_host::HostStructure hs;
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    orbamd_host::build_structure(P, N, level, fixed.data(), ep.data(), ek.data(), hs);   // warm
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) orbamd_host::build_structure(P, N, level, fixed.data(), ep.data(), ek.data(), hs);
    auto t1 = std::chrono::steady_clock::now();
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const std::vector<int>& v) { for (int x : v) h = (h ^ (unsigned)x) * 1099511628211ull; };
    mix(hs.act); mix(hs.hp); mix(hs.hl); mix(hs.pt_beg); mix(hs.pt_slot); mix(hs.pt_id); mix(hs.ps_beg); mix(hs.ps_slot);
    mix(hs.ps_id); mix(hs.blk_i1); mix(hs.blk_i2); mix(hs.blk_beg);
    for (auto& p : hs.blk_pair) h = ((h ^ (unsigned)p.x) * 1099511628211ull ^ (unsigned)p.y) * 1099511628211ull;
    printf("build_structure %.1f us (P %d N %d E %d np %d nl %d blocks %zu pairs %zu) checksum %016llx\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / reps, P, N, E, hs.np, hs.nl, hs.blk_i1.size(),
           hs.blk_pair.size(), h);
    // the host half of the device build (the default path)
    orbamd_host::HostStructure hc;
    if (!orbamd_host::build_structure_counts(P, N, fixed.data(), ep.data(), ek.data(), E, hc)) return 2;
    t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) orbamd_host::build_structure_counts(P, N, fixed.data(), ep.data(), ek.data(), E, hc);
    t1 = std::chrono::steady_clock::now();
    h = 1469598103934665603ull;
    mix(hc.hp); mix(hc.hl); mix(hc.pt_beg); mix(hc.pt_id); mix(hc.ps_beg); mix(hc.ps_id); mix(hc.blk_i1); mix(hc.blk_i2);
    mix(hc.blk_beg);
    printf("build_structure_counts %.1f us (blocks %zu pairs %d) checksum %016llx\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / reps, hc.blk_i1.size(), hc.n_pairs, h);
    return 0;
}
