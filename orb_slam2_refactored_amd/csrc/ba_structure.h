// LocalBA host-side structure (SparseOptimizer::initializeOptimization + the BlockSolver fill
// pattern), plain C++ so that a CPU probe (tools/probe/ba_struct_bench.cpp) and orbba.hip share it.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace orbamd_host {

struct int2h {
    int x, y;
};

struct HostStructure {
    std::vector<int> act, hp, hl, pt_beg, pt_slot, pt_id, ps_beg, ps_slot, ps_id, blk_i1, blk_i2, blk_beg;
    std::vector<int> last_pt, blk_cur;   // point-sorted path scratch: last point per pose, block cursors
    std::vector<int2h> blk_pair;
    std::vector<int> blk_index, fs_beg, fs_slot, fs_hp, sl, sp, cur;   // scratch (capacity kept across calls)
    std::vector<uint8_t> pa, la;
    std::vector<unsigned long long> col;   // per-pose bitsets over the points (pair blocks)
    std::vector<int> slot_of;              // [pose][point] -> free slot (pair blocks; a block's fill reads
                                           // two rows in point order)
    int np = 0, nl = 0;
    int n_act = 0, n_ps = 0, n_pairs = 0;   // sizes of act / ps_slot / blk_pair (also when the device fills them)
};

// The host half of the device-side build (round 6; orbba.hip ba_struct_slots_kernel +
// ba_struct_pairs_kernel fill act, pt_slot, ps_slot and blk_pair on the GPU).  Under the
// point-sorted preconditions (every edge active, point ids non-decreasing, no point seeing a free
// pose twice -- Optimizer.cc:580-627 adds the edges map point by map point) it computes everything
// but those four arrays: the vertex indices, the point runs, the per-pose counts and the pose-pair
// block list with each block's pair count (popcounts of per-pose point bitsets).  O(E) plus
// np^2/2 x nl/64 popcounts; the arrays the device fills equal build_structure's (the fill walks
// the points of each block in ascending order, as the bitset path does).  Returns false (the
// caller then runs build_structure) when a precondition fails.
inline bool build_structure_counts(int P, int N, const uint8_t* fixed, const int* ep, const int* ek, int E,
                                   HostStructure& s) {
    // One pass over the edges: the sort check, the point runs and the poses that have edges.  Branch-
    // free: every edge stores its index and point into the slot of the run after the current one,
    // which the next run's first edge (or the final pb[nl] = E) overwrites, so only a run's first
    // edge leaves its values (points start every ~4 edges: a branch there mispredicted often).
    s.pa.assign(P, 0);
    s.hl.assign(N, -1);
    s.pt_id.resize((size_t)N + 1);
    s.pt_beg.resize((size_t)N + 1);
    int nl = 0;
    {
        uint8_t* pa = s.pa.data();
        int* hl = s.hl.data();
        int* pid = s.pt_id.data();
        int* pb = s.pt_beg.data();
        int prev = -1;
        bool unsorted = false;
        for (int e = 0; e < E; e++) {
            const int x = ep[e];
            unsorted |= x < prev;
            const int j = nl < N ? nl : N;   // unsorted input can start more than N runs (then refused
            pb[j] = e;                       // below): slot N is scratch, so no store leaves the arrays
            pid[j] = x;
            nl += x != prev;
            hl[x] = (nl < N ? nl : N) - 1;
            prev = x;
            pa[ek[e]] = 1;
        }
        if (unsorted) return false;   // not point-sorted
        pb[nl] = E;
    }
    s.pt_beg.resize((size_t)nl + 1);
    s.pt_id.resize(nl);
    s.hp.resize(P);
    s.ps_id.resize(P);
    int np = 0;
    {
        const uint8_t* pa = s.pa.data();
        int* hp = s.hp.data();
        int* pid = s.ps_id.data();
        for (int i = 0; i < P; i++) {
            hp[i] = (pa[i] && !fixed[i]) ? np : -1;
            if (hp[i] >= 0) pid[np++] = i;
        }
    }
    s.ps_id.resize(np);
    const int W = (nl + 63) >> 6;
    s.col.assign((size_t)np * W, 0ull);
    s.ps_beg.assign((size_t)np + 1, 0);
    {
        const int* hp = s.hp.data();
        const int* pb = s.pt_beg.data();
        unsigned long long* col = s.col.data();
        int* qb = s.ps_beg.data();
        // one flat pass over the edges (the point index follows the runs; no per-point inner loop)
        (void)pb;
        const int* epp = ep;
        int l = -1, prev = -1;
        for (int e = 0; e < E; e++) {
            const int x = epp[e];
            l += x != prev;
            prev = x;
            const int h = hp[ek[e]];
            if (h < 0) continue;
            unsigned long long& w = col[(size_t)h * W + (l >> 6)];
            const unsigned long long bit = 1ull << (l & 63);
            if (w & bit) return false;   // the point sees this free pose twice
            w |= bit;
            qb[h + 1]++;
        }
        for (int i = 0; i < np; i++) qb[i + 1] += qb[i];
    }
    s.blk_i1.clear(); s.blk_i2.clear(); s.blk_beg.assign(1, 0);
    int total = 0;
    {
        const unsigned long long* col = s.col.data();
        for (int i1 = 0; i1 < np; i1++)
            for (int i2 = i1; i2 < np; i2++) {
                const unsigned long long* c1 = col + (size_t)i1 * W;
                const unsigned long long* c2 = col + (size_t)i2 * W;
                int cnt = 0;
                for (int w = 0; w < W; w++) cnt += __builtin_popcountll(c1[w] & c2[w]);
                if (cnt == 0 && i1 != i2) continue;
                s.blk_i1.push_back(i1);
                s.blk_i2.push_back(i2);
                total += cnt;
                s.blk_beg.push_back(total);
            }
    }
    s.np = np; s.nl = nl;
    s.n_act = E; s.n_ps = s.ps_beg[np]; s.n_pairs = total;
    return true;
}

inline void build_structure_generic(int P, int N, const std::vector<uint8_t>& level, const uint8_t* fixed, const int* ep,
                                    const int* ek, HostStructure& s);

// The same arrays when every edge is active (the first optimize()) and the edges come grouped by point
// (point ids non-decreasing): Optimizer.cc:580-627 adds them so, map point by map point, each with its
// observations.  Then the point lists are runs (pt_slot = identity), the pose lists one counting sort,
// and the pose-pair blocks come from each point's free slots directly: pass 1 counts the pairs of
// every block (np x np counters), pass 2 appends each point's pairs to their blocks, points ascending --
// the order the bitset path produces (block (i1, i2): points of col[i1] & col[i2] ascending, pair
// (slot of i1, slot of i2)) without the per-pose bitsets and the (pose, point) slot table.  A point
// that sees a free pose twice (the bitset path's `dup`) or unsorted edges take the generic build.
// Returns false (nothing built) when the preconditions do not hold.
inline bool build_structure_point_sorted(int P, int N, const std::vector<uint8_t>& level, const uint8_t* fixed,
                                         const int* ep, const int* ek, HostStructure& s) {
    const int E = (int)level.size();
    {
        const uint8_t* lv = level.data();
        int bad = 0;
        for (int e = 0; e < E; e++) bad |= lv[e] | (e > 0 && ep[e] < ep[e - 1]);
        if (bad) return false;
    }
    // (raw pointers throughout: a store through a vector's int* may alias another vector's members, so
    // the compiler would reload every data pointer per element)
    s.pa.assign(P, 0);
    s.hp.resize(P);
    s.ps_id.resize(P);
    int np = 0;
    {
        uint8_t* pa = s.pa.data();
        for (int e = 0; e < E; e++) pa[ek[e]] = 1;
        int* hp = s.hp.data();
        int* pid = s.ps_id.data();
        for (int i = 0; i < P; i++) {
            hp[i] = (pa[i] && !fixed[i]) ? np : -1;
            if (hp[i] >= 0) pid[np++] = i;
        }
    }
    s.ps_id.resize(np);
    // per edge its Hessian pose index (sp); a point seeing a free pose twice takes the generic build
    s.sp.resize(E);
    s.last_pt.assign(std::max(np, 1), -1);
    {
        const int* hp = s.hp.data();
        int* sp = s.sp.data();
        int* last = s.last_pt.data();
        for (int e = 0; e < E; e++) {
            const int h = hp[ek[e]];
            sp[e] = h;
            if (h < 0) continue;
            if (last[h] == ep[e]) return false;
            last[h] = ep[e];
        }
    }
    s.act.resize(E);
    s.pt_slot.resize(E);
    s.hl.assign(N, -1);
    s.pt_id.resize(N);
    s.pt_beg.resize((size_t)N + 1);
    int nl = 0;
    {
        int* act = s.act.data();
        int* pts = s.pt_slot.data();
        int* hl = s.hl.data();
        int* pid = s.pt_id.data();
        int* pb = s.pt_beg.data();
        for (int e = 0; e < E; e++) {
            act[e] = e;
            pts[e] = e;
            if (e == 0 || ep[e] != ep[e - 1]) {   // points: runs of the sorted edges
                hl[ep[e]] = nl;
                pid[nl] = ep[e];
                pb[nl++] = e;
            }
        }
        pb[nl] = E;
    }
    s.pt_beg.resize((size_t)nl + 1);
    s.pt_id.resize(nl);
    s.np = np; s.nl = nl;
    // poses: counting sort of the free edges by Hessian pose index (stable: e ascending)
    s.ps_beg.assign((size_t)np + 1, 0);
    {
        const int* sp = s.sp.data();
        int* qb = s.ps_beg.data();
        for (int e = 0; e < E; e++)
            if (sp[e] >= 0) qb[sp[e] + 1]++;
        for (int i = 0; i < np; i++) qb[i + 1] += qb[i];
        s.ps_slot.resize(qb[np]);
        s.cur.assign(s.ps_beg.begin(), s.ps_beg.end() - 1);
        int* cur = s.cur.data();
        int* pss = s.ps_slot.data();
        for (int e = 0; e < E; e++)
            if (sp[e] >= 0) pss[cur[sp[e]]++] = e;
    }
    // pose-pair blocks: pass 1 counts, the block list, pass 2 fills (points ascending)
    s.blk_index.assign((size_t)np * np, 0);
    int* cnt = s.blk_index.data();
    const int* sp = s.sp.data();
    const int* pb = s.pt_beg.data();
    for (int l = 0; l < nl; l++) {
        const int b0 = pb[l], b1 = pb[l + 1];
        for (int a = b0; a < b1; a++) {
            const int ia = sp[a];
            if (ia < 0) continue;
            for (int c = a; c < b1; c++) {
                const int ic = sp[c];
                if (ic >= 0) cnt[ia < ic ? ia * np + ic : ic * np + ia]++;
            }
        }
    }
    s.blk_i1.clear(); s.blk_i2.clear(); s.blk_beg.assign(1, 0);
    int total = 0;
    for (int i1 = 0; i1 < np; i1++)
        for (int i2 = i1; i2 < np; i2++) {
            int& c = cnt[(size_t)i1 * np + i2];
            if (c == 0 && i1 != i2) { c = -1; continue; }
            s.blk_i1.push_back(i1);
            s.blk_i2.push_back(i2);
            const int beg = total;
            total += c;
            c = beg;   // now the block's fill cursor
            s.blk_beg.push_back(total);
        }
    s.blk_pair.resize(total);
    int2h* out = s.blk_pair.data();
    for (int l = 0; l < nl; l++) {
        const int b0 = pb[l], b1 = pb[l + 1];
        for (int a = b0; a < b1; a++) {
            const int ia = sp[a];
            if (ia < 0) continue;
            for (int c = a; c < b1; c++) {
                const int ic = sp[c];
                if (ic < 0) continue;
                if (ia <= ic) out[cnt[ia * np + ic]++] = int2h{a, c};
                else out[cnt[ic * np + ia]++] = int2h{c, a};
            }
        }
    }
    return true;
}

// SparseOptimizer::initializeOptimization(level) (sparse_optimizer.cpp:206-264) and the
// BlockSolver structure (block_solver.hpp:142-295): active edges / vertices, Hessian indices, and
// the Schur fill pattern (pose pairs that share a point).  Flat two-pass build (count, then fill)
// over per-slot (point, pose) Hessian ids, into vectors that keep their capacity across calls: no
// allocation per point or per block.
// Pair order inside a block: points ascending, then (slot a, slot c) in the point's slot order.
// sorted: try the point-sorted path first (ORBBA_STRUCT=sorted; measured, see DESIGN §4 LocalBA round 6)
inline void build_structure(int P, int N, const std::vector<uint8_t>& level, const uint8_t* fixed, const int* ep,
                     const int* ek, HostStructure& s, bool sorted = false) {
    if (!(sorted && build_structure_point_sorted(P, N, level, fixed, ep, ek, s)))
        build_structure_generic(P, N, level, fixed, ep, ek, s);
    s.n_act = (int)s.act.size();
    s.n_ps = (int)s.ps_slot.size();
    s.n_pairs = (int)s.blk_pair.size();
}
inline void build_structure_generic(int P, int N, const std::vector<uint8_t>& level, const uint8_t* fixed, const int* ep,
                                    const int* ek, HostStructure& s) {
    const int E = (int)level.size();
    s.pa.assign(P, 0);
    s.la.assign(N, 0);
    s.act.resize(E);
    int Ea = 0;
    {
        int* act = s.act.data();
        uint8_t* pa = s.pa.data();
        uint8_t* la = s.la.data();
        for (int e = 0; e < E; e++)
            if (level[e] == 0) { act[Ea++] = e; pa[ek[e]] = 1; la[ep[e]] = 1; }
    }
    s.act.resize(Ea);
    s.hp.resize(P); s.hl.resize(N);
    s.ps_id.resize(P); s.pt_id.resize(N);
    int np = 0, nl = 0;
    for (int i = 0; i < P; i++) {
        s.hp[i] = (s.pa[i] && !fixed[i]) ? np : -1;
        if (s.hp[i] >= 0) s.ps_id[np++] = i;
    }
    for (int i = 0; i < N; i++) {
        s.hl[i] = s.la[i] ? nl : -1;
        if (s.la[i]) s.pt_id[nl++] = i;
    }
    s.ps_id.resize(np); s.pt_id.resize(nl);
    s.np = np; s.nl = nl;
    // per active slot k: its point's and pose's Hessian ids
    s.sl.resize(Ea); s.sp.resize(Ea);
    int* sl = s.sl.data();
    int* sp = s.sp.data();
    for (int k = 0; k < Ea; k++) {
        const int e = s.act[k];
        sl[k] = s.hl[ep[e]];
        sp[k] = s.hp[ek[e]];
    }
    s.pt_beg.assign(nl + 1, 0); s.ps_beg.assign(np + 1, 0); s.fs_beg.assign(nl + 1, 0);
    {
        int* pb = s.pt_beg.data();
        int* qb = s.ps_beg.data();
        int* fb = s.fs_beg.data();
        for (int k = 0; k < Ea; k++) {
            pb[sl[k] + 1]++;
            if (sp[k] >= 0) { qb[sp[k] + 1]++; fb[sl[k] + 1]++; }
        }
        for (int i = 0; i < nl; i++) { pb[i + 1] += pb[i]; fb[i + 1] += fb[i]; }
        for (int i = 0; i < np; i++) qb[i + 1] += qb[i];
    }
    s.pt_slot.resize(Ea); s.ps_slot.resize(s.ps_beg[np]);
    s.fs_slot.resize(s.fs_beg[nl]); s.fs_hp.resize(s.fs_beg[nl]);
    {
        // fill cursors (k ascending, so every list is in slot order)
        s.cur.resize(2 * (size_t)nl + np);
        int* fp = s.cur.data();
        int* fr = fp + nl;
        int* fq = fr + nl;
        std::copy(s.pt_beg.begin(), s.pt_beg.end() - 1, fp);
        std::copy(s.fs_beg.begin(), s.fs_beg.end() - 1, fr);
        std::copy(s.ps_beg.begin(), s.ps_beg.end() - 1, fq);
        int* pts = s.pt_slot.data();
        int* pss = s.ps_slot.data();
        int* fss = s.fs_slot.data();
        int* fsh = s.fs_hp.data();
        for (int k = 0; k < Ea; k++) {
            const int l = sl[k], h = sp[k];
            pts[fp[l]++] = k;
            if (h >= 0) {
                pss[fq[h]++] = k;
                fss[fr[l]] = k;
                fsh[fr[l]++] = h;
            }
        }
    }
    // pose-pair blocks (i1 <= i2): pass 1 counts the pairs per block, pass 2 fills them, from each
    // point's free slots (slot order) with their Hessian pose index.  Reference order inside a block:
    // points ascending, then (slot a, slot c) in the point's slot order with pose(a) <= pose(c).
    //
    // Bitset path: a point that sees every free pose at most once (a MapPoint holds one observation
    // per keyframe) has exactly one pair in each block it touches, so block (i1, i2) holds the points
    // of col[i1] & col[i2] (per-pose bitsets over the points) in ascending order: counts are popcounts
    // and the fill walks the set bits, with the same result as the two nested slot loops below, which
    // remain for problems where some point repeats a pose.
    {
        const int W = (nl + 63) >> 6;
        s.col.assign((size_t)np * W, 0ull);
        s.slot_of.resize((size_t)std::max(nl, 1) * std::max(np, 1));   // read only where written
        const int* fh = s.fs_hp.data();
        const int* fb = s.fs_beg.data();
        const int* fsl = s.fs_slot.data();
        unsigned long long* col = s.col.data();
        int* so = s.slot_of.data();
        bool dup = false;
        for (int l = 0; l < nl && !dup; l++)
            for (int a = fb[l]; a < fb[l + 1]; a++) {
                unsigned long long& w = col[(size_t)fh[a] * W + (l >> 6)];
                const unsigned long long bit = 1ull << (l & 63);
                dup |= (w & bit) != 0;
                w |= bit;
                so[(size_t)fh[a] * nl + l] = fsl[a];
            }
        if (!dup) {
            s.blk_i1.clear(); s.blk_i2.clear(); s.blk_beg.assign(1, 0);
            int total = 0;
            for (int i1 = 0; i1 < np; i1++)
                for (int i2 = i1; i2 < np; i2++) {
                    const unsigned long long* c1 = col + (size_t)i1 * W;
                    const unsigned long long* c2 = col + (size_t)i2 * W;
                    int cnt = 0;
                    for (int w = 0; w < W; w++) cnt += __builtin_popcountll(c1[w] & c2[w]);
                    if (cnt == 0 && i1 != i2) continue;
                    s.blk_i1.push_back(i1);
                    s.blk_i2.push_back(i2);
                    total += cnt;
                    s.blk_beg.push_back(total);
                }
            s.blk_pair.resize(total);
            int2h* out = s.blk_pair.data();
            for (size_t k = 0; k < s.blk_i1.size(); k++) {
                const int i1 = s.blk_i1[k], i2 = s.blk_i2[k];
                const unsigned long long* c1 = col + (size_t)i1 * W;
                const unsigned long long* c2 = col + (size_t)i2 * W;
                const int* s1 = so + (size_t)i1 * nl;
                const int* s2 = so + (size_t)i2 * nl;
                for (int w = 0; w < W; w++)
                    for (unsigned long long m = c1[w] & c2[w]; m; m &= m - 1) {
                        const int l = (w << 6) + __builtin_ctzll(m);
                        *out++ = int2h{s1[l], s2[l]};
                    }
            }
            return;
        }
    }
    s.blk_index.assign((size_t)np * np, 0);
    {
        const int* fh = s.fs_hp.data();
        const int* fb = s.fs_beg.data();
        int* cnt = s.blk_index.data();
        for (int l = 0; l < nl; l++) {
            const int b0 = fb[l], b1 = fb[l + 1];
            for (int a = b0; a < b1; a++) {
                const int i1 = fh[a];
                int* row = cnt + (size_t)i1 * np;
                for (int c = b0; c < b1; c++) row[fh[c]] += i1 <= fh[c];
            }
        }
    }
    s.blk_i1.clear(); s.blk_i2.clear(); s.blk_beg.assign(1, 0);
    int total = 0;
    for (int i1 = 0; i1 < np; i1++)
        for (int i2 = i1; i2 < np; i2++) {
            int& cnt = s.blk_index[(size_t)i1 * np + i2];
            if (cnt == 0 && i1 != i2) { cnt = -1; continue; }
            s.blk_i1.push_back(i1);
            s.blk_i2.push_back(i2);
            const int beg = total;
            total += cnt;
            cnt = beg;   // now the block's fill cursor
            s.blk_beg.push_back(total);
        }
    s.blk_pair.resize(total);
    {
        const int* fh = s.fs_hp.data();
        const int* fb = s.fs_beg.data();
        const int* fsl = s.fs_slot.data();
        int* curp = s.blk_index.data();
        int2h* out = s.blk_pair.data();
        for (int l = 0; l < nl; l++) {
            const int b0 = fb[l], b1 = fb[l + 1];
            for (int a = b0; a < b1; a++) {
                const int i1 = fh[a];
                int* row = curp + (size_t)i1 * np;
                for (int c = b0; c < b1; c++)
                    if (i1 <= fh[c]) out[row[fh[c]]++] = int2h{fsl[a], fsl[c]};
            }
        }
    }
}


}  // namespace orbamd_host
