// orbv.hip — DBoW2 ORBVocabulary transform on gfx950.
//
// Reference: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h — loadFromTextFile (:1341-1431),
// transform(features, BowVector&, FeatureVector&, levelsup) (:1130-1196) and the per-descriptor
// descent (:1221-1263); BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84),
// FeatureVector::addFeature (FeatureVector.cpp:31-45), FORB::distance (FORB.cpp:80-100), the
// normalisation each scoring type asks for (ScoringObject.h:74-89).  Called by Frame::ComputeBoW /
// KeyFrame::ComputeBoW with levelsup = 4 (src/Frame.cc:208-214, src/KeyFrame.cc:66-74).
//
// Layout in HBM: node descriptors as one [n_nodes][32] byte array, children as CSR in file order,
// per-node word id (u32) and weight (f64).  ORBvoc-sized trees (k = 10, L = 6, ~1.1 M nodes) take
// ~50 MB.
//   voc_descend_kernel    G lanes per descriptor (G = 16 when every node has <= 16 children): lane c
//                         scores child c, the group takes the minimum key (dist << 16 | c) = the
//                         first closest child as the reference's strict-< scan, one level per step;
//                         records the node at level L - levelsup.
//   voc_aggregate_kernel  one workgroup per frame: bitonic sorts of (word, feature) and (node, feature)
//                         in LDS; per word the weight added in feature order (the map's += sequence),
//                         the L1 / L2 norm summed in word order by one lane, then the division;
//                         FeatureVector as CSR.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

struct orbv_vocabulary {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0;
    int n_nodes = 0, n_words = 0, max_children = 0;
    orbamd::DevBuf buf;   // child_off | orig | desc | word | weight, in breadth-first node order
    int32_t* child_off = nullptr;
    int32_t* orig = nullptr;   // breadth-first id -> the file's node id
    uint8_t* desc = nullptr;
    uint32_t* word = nullptr;
    double* weight = nullptr;
    orbamd::DevBuf ws, io;   // per-feature (word, weight, node); host-entry staging
};

namespace orbamd {

constexpr uint32_t VOC_NONE = 0xffffffffu;
constexpr int VOC_MAXF = ORBV_MAX_FEATURES;

// The tree in breadth-first order (voc_upload relabels it): node u's children are the consecutive ids
// child_off[u] + 1 .. child_off[u + 1], so a child's descriptor address needs no index load; orig maps
// back to the file's node ids (the FeatureVector's node ids).
struct VocDev {
    const int32_t* child_off;
    const int32_t* orig;
    const uint8_t* desc;
    const uint32_t* word;
    const double* weight;
    int nid_level;
};

struct VocFeat {   // per descriptor slot: the descent's result
    uint32_t* word;
    double* weight;
    uint32_t* node;
};

__device__ __forceinline__ int voc_hamming(uint4 a0, uint4 a1, const uint8_t* b) {
    const uint4* y = reinterpret_cast<const uint4*>(b);
    const uint4 b0 = y[0], b1 = y[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

template <int G>
__global__ __launch_bounds__(256) void voc_descend_kernel(VocDev v, const uint8_t* desc, const int32_t* counts,
                                                          int cap, int n_frames, VocFeat out) {
    const int lane = threadIdx.x & (G - 1);
    const long long g = ((long long)blockIdx.x * 256 + threadIdx.x) / G;   // descriptor slot
    if (g >= (long long)n_frames * cap) return;   // group-uniform
    const int f = (int)(g / cap), i = (int)(g % cap);
    if (i >= counts[f]) return;
    const uint4* d = reinterpret_cast<const uint4*>(desc + g * 32);
    const uint4 a0 = d[0], a1 = d[1];
    uint32_t node = 0, nid = v.nid_level <= 0 ? 0u : VOC_NONE;
    int level = 0;
    while (true) {
        const int off = v.child_off[node], cnt = v.child_off[node + 1] - off;
        if (cnt == 0) break;   // leaf (the root of a non-empty vocabulary has children)
        ++level;
        uint32_t key = VOC_NONE;
        for (int c0 = 0; c0 < cnt; c0 += G) {
            const int c = c0 + lane;
            if (c < cnt) {
                const int dist = voc_hamming(a0, a1, v.desc + (size_t)(off + 1 + c) * 32);
                key = min(key, ((uint32_t)dist << 16) | (uint32_t)c);
            }
        }
#pragma unroll
        for (int m = G / 2; m > 0; m >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, G));
        node = (uint32_t)(off + 1 + (int)(key & 0xffffu));
        if (level == v.nid_level) nid = node;
    }
    if (lane == 0) {
        out.word[g] = v.word[node];
        out.weight[g] = v.weight[node];
        out.node[g] = (uint32_t)v.orig[nid == VOC_NONE ? node : nid];   // undefined in the reference: the leaf
    }
}

__device__ __forceinline__ void voc_bitonic(unsigned long long* keys, int P) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = keys[i], y = keys[ixj];
                    if ((x > y) == ((i & k) == 0)) { keys[i] = y; keys[ixj] = x; }
                }
            }
            __syncthreads();
        }
}

// Exclusive block scan of 0/1 flags over P positions (256 threads); returns the total.
__device__ __forceinline__ int voc_scan_flags(int* pos, int P, int* s_part) {
    const int per = (P + 255) / 256;
    const int b = threadIdx.x * per;
    int c = 0;
    for (int t = b; t < min(b + per, P); t++) c += pos[t];
    s_part[threadIdx.x] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int t = 0; t < 256; t++) { const int x = s_part[t]; s_part[t] = run; run += x; }
        s_part[256] = run;
    }
    __syncthreads();
    int run = s_part[threadIdx.x];
    for (int t = b; t < min(b + per, P); t++) { const int x = pos[t]; pos[t] = run; run += x; }
    __syncthreads();
    return s_part[256];
}

struct VocAggOut {
    uint32_t* bow_word;
    double* bow_weight;
    int32_t* n_words;
    uint32_t* fv_node;
    int32_t* fv_off;
    int32_t* fv_idx;
    int32_t* n_nodes;
};

__global__ __launch_bounds__(256) void voc_aggregate_kernel(VocFeat ft, const int32_t* counts, int cap, int scoring,
                                                            int weighting, int empty_voc, VocAggOut o) {
    // LDS: VOC_MAXF sort keys (u64) | VOC_MAXF segment indices (int) | VOC_MAXF word values (f64)
    extern __shared__ unsigned long long s_keys[];
    int* s_pos = reinterpret_cast<int*>(s_keys + VOC_MAXF);
    double* s_val = reinterpret_cast<double*>(s_pos + VOC_MAXF);
    __shared__ int s_part[257];
    __shared__ double s_norm;
    const int f = blockIdx.x;
    const int n = empty_voc ? 0 : counts[f];
    const size_t base = (size_t)f * cap;
    int P = 1;
    while (P < n) P <<= 1;
    const bool tf = weighting == 0 || weighting == 1;   // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    auto is_start = [&](int p) {
        return s_keys[p] != ~0ull && (p == 0 || (s_keys[p] >> 32) != (s_keys[p - 1] >> 32));
    };
    // ---- BowVector: (word, feature) ascending
    for (int i = threadIdx.x; i < P; i += 256)
        s_keys[i] = (i < n && ft.weight[base + i] > 0) ? ((unsigned long long)ft.word[base + i] << 32) | (unsigned)i
                                                       : ~0ull;
    __syncthreads();
    voc_bitonic(s_keys, P);
    for (int p = threadIdx.x; p < P; p += 256) s_pos[p] = is_start(p) ? 1 : 0;
    __syncthreads();
    const int U = voc_scan_flags(s_pos, P, s_part);
    for (int p = threadIdx.x; p < P; p += 256) {
        if (!is_start(p)) continue;
        const uint32_t w = (uint32_t)(s_keys[p] >> 32);
        const double wt = ft.weight[base + (unsigned)(s_keys[p] & 0xffffffffu)];   // the word node's weight
        double val = wt;
        if (tf)   // v[id] += w once per further feature, in feature order
            for (int q = p + 1; q < P && s_keys[q] != ~0ull && (uint32_t)(s_keys[q] >> 32) == w; q++) val += wt;
        s_val[s_pos[p]] = val;
        o.bow_word[base + s_pos[p]] = w;
    }
    __syncthreads();
    const bool must = scoring != 5;   // DotProductScoring does not normalise
    if (threadIdx.x == 0) {
        double norm = 0.0;
        if (must) {   // BowVector::normalize: the sum in ascending word order
            if (scoring != 1) {
                for (int u = 0; u < U; u++) norm += fabs(s_val[u]);
            } else {
                for (int u = 0; u < U; u++) norm += s_val[u] * s_val[u];
                norm = sqrt(norm);
            }
        } else if (tf && U > 0) {
            norm = (double)U;   // v /= v.size() (TemplatedVocabulary.h:1166-1172)
        }
        s_norm = norm;
        o.n_words[f] = U;
    }
    __syncthreads();
    const double norm = s_norm;
    const bool divide = must ? norm > 0.0 : (tf && U > 0);
    for (int u = threadIdx.x; u < U; u += 256) o.bow_weight[base + u] = divide ? s_val[u] / norm : s_val[u];
    __syncthreads();
    // ---- FeatureVector: (node, feature) ascending
    for (int i = threadIdx.x; i < P; i += 256)
        s_keys[i] = (i < n && ft.weight[base + i] > 0) ? ((unsigned long long)ft.node[base + i] << 32) | (unsigned)i
                                                       : ~0ull;
    __syncthreads();
    voc_bitonic(s_keys, P);
    for (int p = threadIdx.x; p < P; p += 256) s_pos[p] = is_start(p) ? 1 : 0;
    __syncthreads();
    const int T = voc_scan_flags(s_pos, P, s_part);
    for (int p = threadIdx.x; p < P; p += 256) {
        if (s_keys[p] == ~0ull) continue;
        o.fv_idx[base + p] = (int32_t)(s_keys[p] & 0xffffffffu);
        if (is_start(p)) {
            o.fv_node[base + s_pos[p]] = (uint32_t)(s_keys[p] >> 32);
            o.fv_off[(size_t)f * (cap + 1) + s_pos[p]] = p;
        }
    }
    if (threadIdx.x == 0) {   // valid keys sort first: their count is the first ~0 position
        int lo = 0, hi = P;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_keys[mid] != ~0ull) lo = mid + 1; else hi = mid;
        }
        o.fv_off[(size_t)f * (cap + 1) + T] = lo;
        o.n_nodes[f] = T;
    }
}

constexpr size_t VOC_AGG_LDS = (size_t)VOC_MAXF * (8 + 4 + 8);

}  // namespace orbamd

using namespace orbamd;

namespace {

// Builds the device tree from parsed nodes (index 1..n-1; parent, leaf flag, descriptor, weight).
int voc_upload(orbv_vocabulary* v, int n, const std::vector<int32_t>& parent, const std::vector<uint8_t>& leaf,
               const uint8_t* desc, const std::vector<double>& weight) {
    std::vector<int32_t> cnt(n + 1, 0), off(n + 1, 0), child(std::max(n - 1, 1), 0);
    for (int i = 1; i < n; i++) {
        ORB_CHECK_ARG(parent[i] >= 0 && parent[i] < n && parent[i] != i, "vocabulary: bad parent id");
        cnt[parent[i]]++;
    }
    for (int i = 0; i < n; i++) off[i + 1] = off[i] + cnt[i];
    std::vector<int32_t> fill(off.begin(), off.end() - 1);
    for (int i = 1; i < n; i++) child[fill[parent[i]]++] = i;   // children in file order (push_back)
    // breadth-first relabelling: new id -> file id (children of a node get consecutive new ids, in
    // file order, so the device needs only the offsets); a node the walk from the root cannot reach
    // (a parent cycle) is an error
    std::vector<int32_t> bfs(1, 0);
    bfs.reserve(n);
    for (size_t h = 0; h < bfs.size() && (int)bfs.size() <= n; h++) {
        const int u = bfs[h];
        for (int q = off[u]; q < off[u + 1]; q++) bfs.push_back(child[q]);
    }
    ORB_CHECK_ARG((int)bfs.size() == n, "vocabulary: nodes unreachable from the root");
    std::vector<int32_t> boff(n + 1, 0);
    for (int u = 0; u < n; u++) boff[u + 1] = boff[u] + cnt[bfs[u]];   // children of new u: boff[u]+1 ..
    std::vector<uint32_t> word(n, 0);
    int nw = 0, maxc = 0;
    for (int i = 1; i < n; i++)
        if (leaf[i]) word[i] = (uint32_t)nw++;
    for (int i = 0; i < n; i++) maxc = std::max(maxc, cnt[i]);
    ORB_CHECK_ARG(maxc < 65536, "vocabulary: more than 65535 children under one node");
    v->n_nodes = n;
    v->n_words = nw;
    v->max_children = maxc;
    ORB_CHECK_ARG(nw == 0 || cnt[0] > 0, "vocabulary: words but an empty root");
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += align_up(std::max<size_t>(bytes, 1), 256); return r; };
    const size_t o_off = take((size_t)(n + 1) * 4), o_or = take((size_t)n * 4), o_d = take((size_t)n * 32),
                 o_w = take((size_t)n * 4), o_wt = take((size_t)n * 8);
    int rc;
    if ((rc = v->buf.reserve(o))) return rc;
    char* b = v->buf.as<char>();
    v->child_off = (int32_t*)(b + o_off);
    v->orig = (int32_t*)(b + o_or);
    v->desc = (uint8_t*)(b + o_d);
    v->word = (uint32_t*)(b + o_w);
    v->weight = (double*)(b + o_wt);
    std::vector<uint8_t> dd((size_t)n * 32, 0);   // the root's descriptor stays zero
    std::vector<uint32_t> bw(n, 0);
    std::vector<double> bwt(n, 0.0);
    for (int u = 1; u < n; u++) {
        const int i = bfs[u];
        std::memcpy(dd.data() + (size_t)u * 32, desc + (size_t)i * 32, 32);
        bw[u] = word[i];
        bwt[u] = weight[i];
    }
    ORB_HIP_TRY(hipMemcpy(v->child_off, boff.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(v->orig, bfs.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(v->desc, dd.data(), (size_t)n * 32, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(v->word, bw.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(v->weight, bwt.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    return ORB_OK;
}

// Whitespace tokenizer with istream >> semantics for the fields we read (failure -> 0).
struct Tok {
    const char* p;
    long next_int() {
        while (*p == ' ' || *p == '\t' || *p == '\r') p++;
        char* e = nullptr;
        const long x = std::strtol(p, &e, 10);
        if (e == p) return 0;
        p = e;
        return x;
    }
    double next_double() {
        while (*p == ' ' || *p == '\t' || *p == '\r') p++;
        char* e = nullptr;
        const double x = std::strtod(p, &e);
        if (e == p) return 0.0;
        p = e;
        return x;
    }
};

int voc_launch(orbv_vocabulary* v, const uint8_t* d_desc, const int32_t* d_counts, int cap, int n_frames, int levelsup,
               VocAggOut o, hipStream_t st) {
    if (n_frames == 0) return ORB_OK;
    int rc;
    const size_t slots = (size_t)n_frames * cap;
    if ((rc = v->ws.reserve(align_up(slots * 4, 256) * 2 + slots * 8))) return rc;
    char* w = v->ws.as<char>();
    VocFeat ft{(uint32_t*)w, (double*)(w + align_up(slots * 4, 256) * 2), (uint32_t*)(w + align_up(slots * 4, 256))};
    if (v->n_words > 0) {
        const VocDev dv{v->child_off, v->orig, v->desc, v->word, v->weight, v->L - levelsup};
        // lanes per descriptor for trees of <= 16 children: 8 (two children per lane at k = 10; more
        // descents in flight per wavefront than 16: 546k -> 583k frames/s); ORBV_LANES = 4 / 16
        static const int lanes = [] { const char* e = getenv("ORBV_LANES"); return e ? atoi(e) : 8; }();
        if (v->max_children <= 16 && lanes == 8) {
            const long long thr = (long long)slots * 8;
            hipLaunchKernelGGL(voc_descend_kernel<8>, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, dv,
                               d_desc, d_counts, cap, n_frames, ft);
        } else if (v->max_children <= 16 && lanes == 4) {
            const long long thr = (long long)slots * 4;
            hipLaunchKernelGGL(voc_descend_kernel<4>, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, dv,
                               d_desc, d_counts, cap, n_frames, ft);
        } else if (v->max_children <= 16) {
            const long long thr = (long long)slots * 16;
            hipLaunchKernelGGL(voc_descend_kernel<16>, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, dv,
                               d_desc, d_counts, cap, n_frames, ft);
        } else {
            const long long thr = (long long)slots * 64;
            hipLaunchKernelGGL(voc_descend_kernel<64>, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, dv,
                               d_desc, d_counts, cap, n_frames, ft);
        }
        ORB_HIP_TRY(hipGetLastError());
    }
    static bool attr = [] {
        return hipFuncSetAttribute((const void*)voc_aggregate_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)VOC_AGG_LDS) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL(voc_aggregate_kernel, dim3(n_frames), dim3(256), VOC_AGG_LDS, st, ft, d_counts, cap, v->scoring,
                       v->weighting, v->n_words == 0 ? 1 : 0, o);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

}  // namespace

extern "C" int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
                           const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                           orbv_vocabulary** out) {
    ORB_CHECK_ARG(out && n_nodes >= 1, "bad argument");
    ORB_CHECK_ARG(k >= 0 && k <= 20 && L >= 1 && L <= 10 && scoring >= 0 && scoring <= 5 && weighting >= 0 &&
                      weighting <= 3,
                  "vocabulary header out of range (TemplatedVocabulary.h:1362-1366)");
    ORB_CHECK_ARG(n_nodes == 1 || (parent && is_leaf && desc && weight), "null node arrays");
    ORB_HIP_TRY(hipSetDevice(device));
    orbv_vocabulary* v = new orbv_vocabulary;
    v->device = device;
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting;
    std::vector<int32_t> par(n_nodes, 0);
    std::vector<uint8_t> lf(n_nodes, 0);
    std::vector<double> wt(n_nodes, 0.0);
    std::vector<uint8_t> ds((size_t)n_nodes * 32, 0);
    for (int i = 1; i < n_nodes; i++) { par[i] = parent[i]; lf[i] = is_leaf[i] ? 1 : 0; wt[i] = weight[i]; }
    if (n_nodes > 1) std::memcpy(ds.data() + 32, desc + 32, (size_t)(n_nodes - 1) * 32);
    const int rc = voc_upload(v, n_nodes, par, lf, ds.data(), wt);
    if (rc) { delete v; return rc; }
    *out = v;
    return ORB_OK;
}

extern "C" int orbv_load_text(const char* path, int device, orbv_vocabulary** out) {
    ORB_CHECK_ARG(path && out, "null argument");
    FILE* fp = std::fopen(path, "rb");
    ORB_CHECK_ARG(fp != nullptr, std::string("cannot open vocabulary ") + path);
    std::string text;
    {
        char buf[1 << 16];
        size_t r;
        while ((r = std::fread(buf, 1, sizeof(buf), fp)) > 0) text.append(buf, r);
        std::fclose(fp);
    }
    size_t pos = 0;
    auto next_line = [&](std::string& line) -> bool {
        if (pos >= text.size()) return false;
        size_t e = text.find('\n', pos);
        if (e == std::string::npos) e = text.size();
        line.assign(text, pos, e - pos);
        pos = e + 1;
        return true;
    };
    std::string line;
    ORB_CHECK_ARG(next_line(line), "empty vocabulary file");
    Tok h{line.c_str()};
    const int k = (int)h.next_int(), L = (int)h.next_int(), n1 = (int)h.next_int(), n2 = (int)h.next_int();
    ORB_CHECK_ARG(!(k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3),
                  "Vocabulary loading failure: This is not a correct text file!");
    std::vector<int32_t> par(1, 0);
    std::vector<uint8_t> lf(1, 0), ds(32, 0);
    std::vector<double> wt(1, 0.0);
    while (next_line(line)) {
        if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
        Tok t{line.c_str()};
        par.push_back((int32_t)t.next_int());
        lf.push_back(t.next_int() > 0 ? 1 : 0);
        for (int i = 0; i < 32; i++) ds.push_back((uint8_t)t.next_int());
        wt.push_back(t.next_double());
    }
    ORB_HIP_TRY(hipSetDevice(device));
    orbv_vocabulary* v = new orbv_vocabulary;
    v->device = device;
    v->k = k; v->L = L; v->scoring = n1; v->weighting = n2;
    const int rc = voc_upload(v, (int)par.size(), par, lf, ds.data(), wt);
    if (rc) { delete v; return rc; }
    *out = v;
    return ORB_OK;
}

extern "C" int orbv_destroy(orbv_vocabulary* v) {
    if (!v) return ORB_OK;
    (void)hipSetDevice(v->device);
    v->buf.release();
    v->ws.release();
    v->io.release();
    delete v;
    return ORB_OK;
}

extern "C" int orbv_info(const orbv_vocabulary* v, int* k, int* L, int* n_nodes, int* n_words, int* scoring,
                         int* weighting) {
    ORB_CHECK_ARG(v, "null vocabulary");
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    return ORB_OK;
}

extern "C" int orbv_transform_batch_device(orbv_vocabulary* v, const uint8_t* d_desc, const int32_t* d_counts, int cap,
                                           int n_frames, int levelsup, uint32_t* d_bow_word, double* d_bow_weight,
                                           int32_t* d_n_words, uint32_t* d_fv_node, int32_t* d_fv_off,
                                           int32_t* d_fv_idx, int32_t* d_n_nodes, void* stream) {
    ORB_CHECK_ARG(v, "null vocabulary");
    ORB_CHECK_ARG(n_frames >= 0 && cap >= 1 && cap <= VOC_MAXF, "cap must be in [1, ORBV_MAX_FEATURES]");
    if (n_frames == 0) return ORB_OK;
    ORB_CHECK_ARG(d_desc && d_counts && d_bow_word && d_bow_weight && d_n_words && d_fv_node && d_fv_off && d_fv_idx &&
                      d_n_nodes,
                  "null device array");
    ORB_HIP_TRY(hipSetDevice(v->device));
    return voc_launch(v, d_desc, d_counts, cap, n_frames, levelsup,
                      VocAggOut{d_bow_word, d_bow_weight, d_n_words, d_fv_node, d_fv_off, d_fv_idx, d_n_nodes},
                      (hipStream_t)stream);
}

extern "C" int orbv_transform(orbv_vocabulary* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word,
                              double* bow_weight, int* n_words, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_idx,
                              int* n_nodes) {
    ORB_CHECK_ARG(v && n_words && n_nodes, "null argument");
    ORB_CHECK_ARG(n >= 0 && n <= VOC_MAXF, "n must be in [0, ORBV_MAX_FEATURES]");
    ORB_CHECK_ARG(n == 0 || (desc && bow_word && bow_weight && fv_node && fv_off && fv_idx), "null array");
    ORB_HIP_TRY(hipSetDevice(v->device));
    const int cap = std::max(n, 1);
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t r = o; o += align_up(std::max<size_t>(bytes, 1), 256); return r; };
    const size_t o_d = take((size_t)cap * 32), o_c = take(4), o_bw = take((size_t)cap * 4), o_bv = take((size_t)cap * 8),
                 o_nw = take(4), o_fn = take((size_t)cap * 4), o_fo = take((size_t)(cap + 1) * 4),
                 o_fi = take((size_t)cap * 4), o_nn = take(4);
    int rc;
    if ((rc = v->io.reserve(o))) return rc;
    char* d = v->io.as<char>();
    if (n) ORB_HIP_TRY(hipMemcpy(d + o_d, desc, (size_t)n * 32, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(d + o_c, &n, 4, hipMemcpyHostToDevice));
    if ((rc = voc_launch(v, (const uint8_t*)(d + o_d), (const int32_t*)(d + o_c), cap, 1, levelsup,
                         VocAggOut{(uint32_t*)(d + o_bw), (double*)(d + o_bv), (int32_t*)(d + o_nw),
                                   (uint32_t*)(d + o_fn), (int32_t*)(d + o_fo), (int32_t*)(d + o_fi),
                                   (int32_t*)(d + o_nn)},
                         nullptr)))
        return rc;
    int32_t nw = 0, nn = 0;
    ORB_HIP_TRY(hipMemcpy(&nw, d + o_nw, 4, hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(&nn, d + o_nn, 4, hipMemcpyDeviceToHost));
    *n_words = nw;
    *n_nodes = nn;
    if (nw) {
        ORB_HIP_TRY(hipMemcpy(bow_word, d + o_bw, (size_t)nw * 4, hipMemcpyDeviceToHost));
        ORB_HIP_TRY(hipMemcpy(bow_weight, d + o_bv, (size_t)nw * 8, hipMemcpyDeviceToHost));
    }
    if (fv_off) ORB_HIP_TRY(hipMemcpy(fv_off, d + o_fo, (size_t)(nn + 1) * 4, hipMemcpyDeviceToHost));
    if (nn) {
        ORB_HIP_TRY(hipMemcpy(fv_node, d + o_fn, (size_t)nn * 4, hipMemcpyDeviceToHost));
        int32_t tot = 0;
        ORB_HIP_TRY(hipMemcpy(&tot, d + o_fo + (size_t)nn * 4, 4, hipMemcpyDeviceToHost));
        if (tot) ORB_HIP_TRY(hipMemcpy(fv_idx, d + o_fi, (size_t)tot * 4, hipMemcpyDeviceToHost));
    }
    return ORB_OK;
}
