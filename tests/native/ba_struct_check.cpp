// The LocalBA device-side structure build (round 6) against the host build, on the CPU: the host half
// (ba_structure.h build_structure_counts) plus a line-by-line emulation of the two fill kernels
// (orbba.hip ba_struct_slots_kernel: the pose-major slot table; ba_struct_pairs_kernel: each block's
// points ascending, a diagonal block's first members = ps_slot) must give exactly the arrays of
// build_structure (generic and point-sorted), on random point-sorted graphs with fixed poses, points
// without free poses and empty pose pairs.  Graphs that break a precondition (unsorted edges, a point
// seeing a pose twice) must be refused by build_structure_counts.  Prints "N problems, 0 mismatches".
#include <cstdio>
#include <random>
#include <vector>

#include "ba_structure.h"

using namespace orbamd_host;

static bool device_emulation(int P, int N, const std::vector<uint8_t>& fixed, const std::vector<int>& ep,
                             const std::vector<int>& ek, HostStructure& s, std::vector<int>& act,
                             std::vector<int>& pt_slot, std::vector<int>& ps_slot, std::vector<int2h>& pairs) {
    const int E = (int)ep.size();
    if (!build_structure_counts(P, N, fixed.data(), ep.data(), ek.data(), E, s)) return false;
    const int np = s.np, nl = s.nl;
    std::vector<int> slot((size_t)np * nl, -1);
    act.assign(E, 0);
    pt_slot.assign(E, 0);
    for (int e = 0; e < E; e++) {   // ba_struct_slots_kernel
        act[e] = e;
        pt_slot[e] = e;
        const int h = s.hp[ek[e]];
        if (h >= 0) slot[(size_t)h * nl + s.hl[ep[e]]] = e;
    }
    ps_slot.assign(s.n_ps, -7);
    pairs.assign(s.n_pairs, int2h{-7, -7});
    for (size_t b = 0; b < s.blk_i1.size(); b++) {   // ba_struct_pairs_kernel
        const int i1 = s.blk_i1[b], i2 = s.blk_i2[b];
        int pos = s.blk_beg[b];
        const int psd = i1 == i2 ? s.ps_beg[i1] - s.blk_beg[b] : 0;
        for (int l = 0; l < nl; l++) {
            const int a = slot[(size_t)i1 * nl + l], c = slot[(size_t)i2 * nl + l];
            if (a < 0 || c < 0) continue;
            if (pos >= s.blk_beg[b + 1]) return false;
            pairs[pos] = int2h{a, c};
            if (i1 == i2) ps_slot[pos + psd] = a;
            pos++;
        }
        if (pos != s.blk_beg[b + 1]) return false;
    }
    return true;
}

int main(int argc, char** argv) {
    const int nprob = argc > 1 ? atoi(argv[1]) : 400;
    std::mt19937 rng(12345);
    int bad = 0, refused_ok = 0;
    for (int t = 0; t < nprob; t++) {
        const int P = 1 + rng() % 24, N = 1 + rng() % 300;
        std::vector<uint8_t> fixed(P);
        for (int i = 0; i < P; i++) fixed[i] = rng() % 5 == 0;
        std::vector<int> ep, ek;
        const int mode = t % 10;   // 8: unsorted, 9: a repeated pose (both must be refused)
        for (int l = 0; l < N; l++) {
            if (rng() % 7 == 0) continue;   // points with no edge
            std::vector<int> poses;
            for (int i = 0; i < P; i++)
                if (rng() % 3 == 0) poses.push_back(i);
            std::shuffle(poses.begin(), poses.end(), rng);
            for (int i : poses) { ep.push_back(l); ek.push_back(i); }
        }
        if (ep.size() < 2) continue;
        if (mode == 8) {
            if (t % 20 == 8) {   // the ends swapped
                std::swap(ep[0], ep[ep.size() - 1]), std::swap(ek[0], ek[ek.size() - 1]);
            } else {   // the whole edge list shuffled: far more point runs than points (the build's
                       // scratch slots must hold them; the test is also built with ASan)
                std::vector<size_t> ord(ep.size());
                for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
                std::shuffle(ord.begin(), ord.end(), rng);
                std::vector<int> ep2(ep.size()), ek2(ek.size());
                for (size_t i = 0; i < ord.size(); i++) ep2[i] = ep[ord[i]], ek2[i] = ek[ord[i]];
                ep.swap(ep2);
                ek.swap(ek2);
            }
        }
        if (mode == 9) { ep.insert(ep.begin() + 1, ep[0]); ek.insert(ek.begin() + 1, ek[0]); }
        const int E = (int)ep.size();
        HostStructure d;
        std::vector<int> act, pts, pss;
        std::vector<int2h> pairs;
        const bool ok = device_emulation(P, N, fixed, ep, ek, d, act, pts, pss, pairs);
        bool unsorted = false, dup = false;
        for (int e = 1; e < E; e++) unsorted |= ep[e] < ep[e - 1];
        if (mode == 8 || mode == 9) {
            // refused exactly when a precondition fails (a repeated FIXED pose is no duplicate)
            if (mode == 9 && !unsorted) dup = !fixed[ek[0]];
            if (ok == (unsorted || dup)) { bad++; printf("problem %d: precondition handling\n", t); }
            else refused_ok++;
            if (!ok) continue;
        }
        if (!ok) { bad++; printf("problem %d: refused\n", t); continue; }
        std::vector<uint8_t> level(E, 0);
        for (int sorted = 0; sorted < 2; sorted++) {
            HostStructure h;
            build_structure(P, N, level, fixed.data(), ep.data(), ek.data(), h, sorted != 0);
            bool same = h.np == d.np && h.nl == d.nl && h.hp == d.hp && h.hl == d.hl && h.pt_beg == d.pt_beg &&
                        h.pt_id == d.pt_id && h.ps_beg == d.ps_beg && h.ps_id == d.ps_id && h.blk_i1 == d.blk_i1 &&
                        h.blk_i2 == d.blk_i2 && h.blk_beg == d.blk_beg && h.act == act && h.pt_slot == pts &&
                        h.ps_slot == pss && h.blk_pair.size() == pairs.size() && h.n_act == d.n_act &&
                        h.n_ps == d.n_ps && h.n_pairs == d.n_pairs;
            for (size_t k = 0; same && k < pairs.size(); k++)
                same = h.blk_pair[k].x == pairs[k].x && h.blk_pair[k].y == pairs[k].y;
            if (!same) { bad++; printf("problem %d (sorted %d): arrays differ\n", t, sorted); }
        }
    }
    printf("%d problems, %d precondition cases, %d mismatches\n", nprob, refused_ok, bad);
    return bad ? 1 : 0;
}
