// orbpo.hip — Optimizer::PoseOptimization on gfx950.
//
// Motion-only BA of src/Optimizer.cc:345-489: one SE3Expmap vertex per frame and one unary
// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose per matched map point
// (types_six_dof_expmap.h:143-202), solved by g2o's Levenberg-Marquardt with a dense 6x6
// linear solver, 4 rounds of optimize(10) with chi2 outlier classification in between.
//
// One 256-lane workgroup owns one frame for the whole optimisation (a single launch per batch):
//   - the frame's first PO_LDS_EDGES edges are staged once into LDS (structure of arrays, fp64);
//     lane i owns edges i, i+256, ... (at most 64, so a lane's outlier / level flags are one
//     register mask);
//   - a pass over the active edges computes computeError + robust chi2 (and, for the
//     linearisation pass, the Jacobian and the 21 + 6 entries of H and b), reduced across the
//     wavefront by a reduce-scatter butterfly built from v_permlane32_swap / v_permlane16_swap
//     and DPP moves (VALU only, no LDS round trips), then across the 4 wavefronts through LDS
//     in a fixed order, and broadcast back to every lane with v_readlane;
//   - every lane then runs the LM control, the packed 6x6 LDL^T solve and the SE3 exp update
//     redundantly on wave-uniform values — identical inputs, identical results, so the pose stays
//     in registers and no lane has to broadcast it.
// fp64 throughout, like the reference.  Sums run in a fixed order: results are bit-reproducible.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "common.h"
#include "se3.h"

namespace orbamd {

#ifndef PO_THREADS_OVERRIDE
constexpr int PO_THREADS = 256;
#else
constexpr int PO_THREADS = PO_THREADS_OVERRIDE;
#endif
constexpr int PO_WAVES = PO_THREADS / 64;
#ifndef PO_LDS_EDGES_OVERRIDE
constexpr int PO_LDS_EDGES = 1024;   // staged edges per frame: 7 doubles each = 56 KiB (2 frames per CU)
#else
constexpr int PO_LDS_EDGES = PO_LDS_EDGES_OVERRIDE;
#endif
constexpr size_t PO_LDS_BYTES = (size_t)7 * PO_LDS_EDGES * sizeof(double);
static_assert(ORBBA_POSE_MAX_EDGES <= PO_THREADS * 64, "outlier mask is one u64 per lane");

#ifdef ORB_PO_STAMPS
// Diagnostic build only (tools/diag/po_stamps.py): cycles per phase summed over block 0, lane 0.
//   0 linearize pass, 1 28-value reduction, 2 6x6 solve, 3 exp update, 4 chi pass + reduction,
//   5 classification, 6 LM iterations, 7 trials
__device__ unsigned long long g_po_stamps[8];
#define PO_T0() unsigned long long _po_t = __builtin_amdgcn_s_memtime()
#define PO_ACC(k)                                                                               \
    do {                                                                                        \
        const unsigned long long _n = __builtin_amdgcn_s_memtime();                             \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_po_stamps[(k)] += _n - _po_t;                \
        _po_t = _n;                                                                             \
    } while (0)
#define PO_CNT(k) do { if (blockIdx.x == 0 && threadIdx.x == 0) g_po_stamps[(k)] += 1; } while (0)
#else
#define PO_T0() do {} while (0)
#define PO_ACC(k) do {} while (0)
#define PO_CNT(k) do {} while (0)
#endif

struct PoArgs {
    int n_frames;
    const int32_t* edge_begin;
    const double *R, *t, *cam, *xw, *obs, *isig2;
    double *oR, *ot;
    int32_t* n_inliers;
    uint8_t* outlier;
};

struct PoEdge {   // one observation as loaded by a pass
    double X[3], z[3], info;
    bool stereo;
};

// Edge store of one frame: the first nl edges in LDS (SoA), the rest read from HBM.
struct PoEdges {
    const double* lds;   // 7 arrays of PO_LDS_EDGES: X0 X1 X2 u v ur info
    const double *xw, *obs, *isig2;   // frame-relative global arrays
    int nl;
};

__device__ __forceinline__ void po_load(const PoEdges& s, int e, PoEdge& d) {
    if (e < s.nl) {
        const double* L = s.lds + e;
        d.X[0] = L[0]; d.X[1] = L[PO_LDS_EDGES]; d.X[2] = L[2 * PO_LDS_EDGES];
        d.z[0] = L[3 * PO_LDS_EDGES]; d.z[1] = L[4 * PO_LDS_EDGES]; d.z[2] = L[5 * PO_LDS_EDGES];
        d.info = L[6 * PO_LDS_EDGES];
    } else {
        const double* x = s.xw + 3 * (size_t)e;
        const double* o = s.obs + 3 * (size_t)e;
        d.X[0] = x[0]; d.X[1] = x[1]; d.X[2] = x[2];
        d.z[0] = o[0]; d.z[1] = o[1]; d.z[2] = o[2];
        d.info = s.isig2[e];
    }
    d.stereo = !(d.z[2] < 0);   // ur < 0: monocular edge (Optimizer.cc:376)
}

struct PoCam { double fx, fy, cx, cy, bf; };

// computeError (types_six_dof_expmap.h:153-158 / :184-189 with cam_project .cpp:290-306) and
// BaseEdge::chi2 = e . (Omega e); returns chi2, the camera point in Xc.
__device__ __forceinline__ double po_error(const PoEdge& d, const PoCam& c, const double* q, const double* t,
                                           double* Xc, double* err) {
    se3_map(q, t, d.X, Xc);
    if (!d.stereo) {
        err[0] = d.z[0] - (Xc[0] / Xc[2] * c.fx + c.cx);
        err[1] = d.z[1] - (Xc[1] / Xc[2] * c.fy + c.cy);
        err[2] = 0;
    } else {   // invz narrowed to float; bf is a double member of the unary stereo edge
        const float invz = (float)(1.0 / Xc[2]);
        const double u = Xc[0] * invz * c.fx + c.cx;
        const double v = Xc[1] * invz * c.fy + c.cy;
        err[0] = d.z[0] - u;
        err[1] = d.z[1] - v;
        err[2] = d.z[2] - (u - c.bf * invz);
    }
    double s = err[0] * (d.info * err[0]) + err[1] * (d.info * err[1]);
    if (d.stereo) s += err[2] * (d.info * err[2]);
    return s;
}

// RobustKernelHuber::robustify (robust_kernel_impl.cpp:65-91), delta = sqrt(CHI2_*) (Optimizer.cc:46-47)
__device__ __forceinline__ void po_robustify(bool robust, bool stereo, double c, double& r0, double& r1) {
    const double delta = stereo ? sqrt(7.815) : sqrt(5.991), dsqr = delta * delta;
    if (!robust || c <= dsqr) { r0 = c; r1 = 1.0; }
    else { const double s = sqrt(c); r0 = 2 * s * delta - dsqr; r1 = delta / s; }
}

// ---------------------------------------------------------------- cross-lane sums (VALU only)
template <int CTRL>
__device__ __forceinline__ double po_dpp(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_QUAD_XOR1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int DPP_ROR4 = 0x124, DPP_ROR8 = 0x128, DPP_ROR12 = 0x12C;

union PoD2 { double d; int i[2]; };

// (a, b) -> (a', b'): lanes 32..63 of a swapped with lanes 0..31 of b (v_permlane32_swap), or odd
// rows of a with even rows of b (v_permlane16_swap) when ROW16.
template <bool ROW16>
__device__ __forceinline__ void po_swap(double& a, double& b) {
    PoD2 x{a}, y{b};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        if constexpr (ROW16) {
            auto r = __builtin_amdgcn_permlane16_swap(x.i[h], y.i[h], false, false);
            x.i[h] = r[0]; y.i[h] = r[1];
        } else {
            auto r = __builtin_amdgcn_permlane32_swap(x.i[h], y.i[h], false, false);
            x.i[h] = r[0]; y.i[h] = r[1];
        }
    }
    a = x.d; b = y.d;
}

// Partner value across lane bit M (M = 4, 8 via DPP row rotates, 1, 2 via quad perms).
template <int M>
__device__ __forceinline__ double po_xor(double v, int lane) {
    if constexpr (M == 1) return po_dpp<DPP_QUAD_XOR1>(v);
    else if constexpr (M == 2) return po_dpp<DPP_QUAD_XOR2>(v);
    else if constexpr (M == 8) return po_dpp<DPP_ROR8>(v);
    else {
        static_assert(M == 4, "");
        // row_ror:N delivers lane (l - N) mod 16: l + 4 is ror 12, l - 4 is ror 4
        const double up = po_dpp<DPP_ROR12>(v), dn = po_dpp<DPP_ROR4>(v);
        return (lane & 4) ? dn : up;
    }
}

// One butterfly step over H value pairs: a lane keeps index i (bit clear) or i + H (bit set)
// and adds its partner's copy of it.
template <int H>
__device__ __forceinline__ void po_scatter_step(double (&v)[32], int lane) {
#pragma unroll
    for (int i = 0; i < H; i++) {
        if constexpr (H == 16) {          // across lane bit 5
            double a = v[i], b = v[i + H];
            po_swap<false>(a, b);
            v[i] = a + b;
        } else if constexpr (H == 8) {    // across lane bit 4
            double a = v[i], b = v[i + H];
            po_swap<true>(a, b);
            v[i] = a + b;
        } else {                          // across lane bit log2(2H): DPP
            const bool hi = (lane & (2 * H)) != 0;
            const double send = hi ? v[i] : v[i + H];
            const double keep = hi ? v[i + H] : v[i];
            v[i] = keep + po_xor<2 * H>(send, lane);
        }
    }
}

// Wavefront reduce-scatter of 32 doubles: on return lane l holds the wave total of value l >> 1.
__device__ __forceinline__ double po_wave_scatter32(double (&v)[32], int lane) {
    po_scatter_step<16>(v, lane);
    po_scatter_step<8>(v, lane);
    po_scatter_step<4>(v, lane);
    po_scatter_step<2>(v, lane);
    po_scatter_step<1>(v, lane);
    return v[0] + po_xor<1>(v[0], lane);
}

// Wavefront all-reduce of one double (every lane gets the same bits: each step adds the same two
// operands, a + b == b + a).
__device__ __forceinline__ double po_wave_sum(double v, int lane) {
    v += po_xor<1>(v, lane);
    v += po_xor<2>(v, lane);
    v += po_xor<4>(v, lane);
    v += po_xor<8>(v, lane);
    { double a = v, b = v; po_swap<true>(a, b); v = a + b; }
    { double a = v, b = v; po_swap<false>(a, b); v = a + b; }
    return v;
}

__device__ __forceinline__ double po_readlane(double v, int l) {
    PoD2 x{v};
    x.i[0] = __builtin_amdgcn_readlane(x.i[0], l);
    x.i[1] = __builtin_amdgcn_readlane(x.i[1], l);
    return x.d;
}

// LDS partials: the 28-value system has its own slot (read again by every trial of the
// iteration); the 1-value sums alternate between two slots so one barrier each suffices.
struct PoRed {
    double sys[PO_WAVES][32];
    double one[2][PO_WAVES];
};

// H (packed upper, 21) | b (6) | robust chi2 (1), summed over the block, wave-uniform in every lane.
struct PoSys { double v[28]; };

__device__ __forceinline__ void po_block_sum28(double (&acc)[32], PoSys& out, PoRed& R) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double r = po_wave_scatter32(acc, lane);
    if ((lane & 1) == 0) R.sys[w][lane >> 1] = r;
    __syncthreads();
    double s = 0;
    if (lane < 28) {
        s = R.sys[0][lane];
#pragma unroll
        for (int k = 1; k < PO_WAVES; k++) s += R.sys[k][lane];
    }
#pragma unroll
    for (int j = 0; j < 28; j++) out.v[j] = po_readlane(s, j);
}

__device__ __forceinline__ double po_block_sum1(double v, PoRed& R, int& par) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    v = po_wave_sum(v, lane);
    if (lane == 0) R.one[par][w] = v;
    __syncthreads();
    double s = R.one[par][0];
#pragma unroll
    for (int k = 1; k < PO_WAVES; k++) s += R.one[par][k];
    par ^= 1;
    return s;
}

// Linearisation pass: robust chi2 total (acc[27]), H upper triangle (acc[0..20], row-major),
// b (acc[21..26]) over the active edges, at pose (q, t).  linearizeOplus (.cpp:266-288,
// :335-364) and BaseUnaryEdge::constructQuadraticForm with weightedOmega = rho' * Omega.
__device__ __forceinline__ void po_linearize(const PoEdges& S, int E, uint64_t outl, const PoCam& c,
                                             const double* q, const double* t, bool robust, double (&acc)[32]) {
#pragma unroll
    for (int j = 0; j < 32; j++) acc[j] = 0;
    int i = 0;
    for (int e = threadIdx.x; e < E; e += PO_THREADS, i++) {
        if ((outl >> i) & 1) continue;
        PoEdge d;
        po_load(S, e, d);
        double Xc[3], err[3];
        const double chi = po_error(d, c, q, t, Xc, err);
        double r0, r1;
        po_robustify(robust, d.stereo, chi, r0, r1);
        acc[27] += r0;
        const double X = Xc[0], Y = Xc[1], invz = 1.0 / Xc[2], invz2 = invz * invz;
        double J[3][6];
        J[0][0] = X * Y * invz2 * c.fx; J[0][1] = -(1 + (X * X * invz2)) * c.fx; J[0][2] = Y * invz * c.fx;
        J[0][3] = -invz * c.fx;         J[0][4] = 0;                             J[0][5] = X * invz2 * c.fx;
        J[1][0] = (1 + Y * Y * invz2) * c.fy; J[1][1] = -X * Y * invz2 * c.fy; J[1][2] = -X * invz * c.fy;
        J[1][3] = 0;                          J[1][4] = -invz * c.fy;          J[1][5] = Y * invz2 * c.fy;
        J[2][0] = J[0][0] - c.bf * Y * invz2; J[2][1] = J[0][1] + c.bf * X * invz2; J[2][2] = J[0][2];
        J[2][3] = J[0][3];                    J[2][4] = 0;                          J[2][5] = J[0][5] - c.bf * invz2;
        const double w = r1 * d.info;
        const double oe[3] = {d.info * err[0], d.info * err[1], d.info * err[2]};
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; r++) {
            double s = J[0][r] * oe[0] + J[1][r] * oe[1];
            if (d.stereo) s += J[2][r] * oe[2];
            acc[21 + r] -= r1 * s;
#pragma unroll
            for (int cc = r; cc < 6; cc++, k++) {
                double h = J[0][r] * w * J[0][cc] + J[1][r] * w * J[1][cc];
                if (d.stereo) h += J[2][r] * w * J[2][cc];
                acc[k] += h;
            }
        }
    }
}

// Trial pass: robust chi2 of the active edges at (q, t) (computeActiveErrors + activeRobustChi2).
__device__ __forceinline__ double po_chi_pass(const PoEdges& S, int E, uint64_t outl, const PoCam& c,
                                              const double* q, const double* t, bool robust) {
    double s = 0;
    int i = 0;
    for (int e = threadIdx.x; e < E; e += PO_THREADS, i++) {
        if ((outl >> i) & 1) continue;
        PoEdge d;
        po_load(S, e, d);
        double Xc[3], err[3];
        double r0, r1;
        po_robustify(robust, d.stereo, po_error(d, c, q, t, Xc, err), r0, r1);
        s += r0;
    }
    return s;
}

// Packed upper-triangle index of (r, c), r <= c.
__host__ __device__ constexpr int pk(int r, int c) { return r * 6 - r * (r - 1) / 2 + (c - r); }

// LinearSolverDense (linear_solver_dense.h:65-113): LDL^T of H + lambda I, rejected unless
// positive semi-definite.  In place on the packed triangle (L(i,j) overwrites H(j,i), D the
// diagonal); same operation order as the oracle.
__device__ __forceinline__ bool po_solve(const PoSys& S, double lambda, double (&x)[6]) {
    double A[21];
#pragma unroll
    for (int k = 0; k < 21; k++) A[k] = S.v[k];
#pragma unroll
    for (int i = 0; i < 6; i++) A[pk(i, i)] += lambda;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double v = A[pk(j, j)];
#pragma unroll
        for (int k = 0; k < j; k++) v -= A[pk(k, j)] * A[pk(k, j)] * A[pk(k, k)];
        ok = ok && (v >= 0) && isfinite(v);
        A[pk(j, j)] = v;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double s = A[pk(j, i)];
#pragma unroll
            for (int k = 0; k < j; k++) s -= A[pk(k, i)] * A[pk(k, j)] * A[pk(k, k)];
            A[pk(j, i)] = v != 0 ? s / v : 0;
        }
    }
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = S.v[21 + i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= A[pk(k, i)] * y[k];
        y[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = A[pk(i, i)] != 0 ? y[i] / A[pk(i, i)] : 0;
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= A[pk(i, k)] * x[k];
        x[i] = s;
    }
    if (!ok)
#pragma unroll
        for (int i = 0; i < 6; i++) x[i] = 0;
    return ok;
}

__global__ __launch_bounds__(PO_THREADS) void pose_opt_kernel(PoArgs a) {
    extern __shared__ double po_lds[];
    __shared__ PoRed red;
    const int f = blockIdx.x;
    const int e0 = a.edge_begin[f], E = a.edge_begin[f + 1] - e0;
    const double* R0 = a.R + 9 * (size_t)f;
    const double* t0 = a.t + 3 * (size_t)f;
    if (E < 3 || E > ORBBA_POSE_MAX_EDGES) {   // Optimizer.cc:412-414: return 0, pose untouched
        if (threadIdx.x < 9) a.oR[9 * (size_t)f + threadIdx.x] = R0[threadIdx.x];
        if (threadIdx.x < 3) a.ot[3 * (size_t)f + threadIdx.x] = t0[threadIdx.x];
        if (threadIdx.x == 0) a.n_inliers[f] = E > ORBBA_POSE_MAX_EDGES ? -1 : 0;
        for (int e = threadIdx.x; e < E; e += PO_THREADS) a.outlier[e0 + e] = 0;
        return;
    }
    const PoEdges S{po_lds, a.xw + 3 * (size_t)e0, a.obs + 3 * (size_t)e0, a.isig2 + e0, min(E, PO_LDS_EDGES)};
    for (int e = threadIdx.x; e < S.nl; e += PO_THREADS) {   // stage: SoA X0 X1 X2 u v ur info
#pragma unroll
        for (int k = 0; k < 3; k++) po_lds[k * PO_LDS_EDGES + e] = S.xw[3 * e + k];
#pragma unroll
        for (int k = 0; k < 3; k++) po_lds[(3 + k) * PO_LDS_EDGES + e] = S.obs[3 * e + k];
        po_lds[6 * PO_LDS_EDGES + e] = S.isig2[e];
    }
    __syncthreads();
    const double* cp = a.cam + 5 * (size_t)f;
    const PoCam c{cp[0], cp[1], cp[2], cp[3], cp[4]};
    double q0[4], tt0[3];   // ToSE3Quat(frame->pose)
    {
        double Rm[9];
#pragma unroll
        for (int i = 0; i < 9; i++) Rm[i] = R0[i];
        Q4 qq = q_from_R(Rm);
        q_normalize_pos(qq);
        q0[0] = qq.x; q0[1] = qq.y; q0[2] = qq.z; q0[3] = qq.w;
        tt0[0] = t0[0]; tt0[1] = t0[1]; tt0[2] = t0[2];
    }
    double q[4], t[3], qe[4], te[3];   // current estimate, pose of the last computeActiveErrors
    uint64_t outl = 0;                 // this lane's edges at level 1 (frame->outlier)
    int noutliers = 0, par = 0;
    bool robust = true;
    PO_T0();
    const int rounds = E < 10 ? 1 : 4;   // optimizer.edges().size() < 10 -> break after round 0
    for (int k = 0; k < rounds; k++) {   // Optimizer.cc:422-484
#pragma unroll
        for (int i = 0; i < 4; i++) { q[i] = q0[i]; qe[i] = q0[i]; }
#pragma unroll
        for (int i = 0; i < 3; i++) { t[i] = tt0[i]; te[i] = tt0[i]; }
        if (E - noutliers > 0) {   // optimize(10) (sparse_optimizer.cpp:354-419; levenberg.cpp:60-163)
            double lambda = 0, ni = 2;
            int nbad = 0;
            for (int it = 0; it < 10; it++) {
                PoSys sys;
                {
                    double acc[32];
                    PO_CNT(6);
                    PO_ACC(5);
                    po_linearize(S, E, outl, c, q, t, robust, acc);
                    PO_ACC(0);
                    po_block_sum28(acc, sys, red);
                    PO_ACC(1);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) qe[i] = q[i];
#pragma unroll
                for (int i = 0; i < 3; i++) te[i] = t[i];
                double cur = sys.v[27];
                const double ini = cur;
                if (it == 0) {   // computeLambdaInit (levenberg.cpp:166-180), tau = 1e-5
                    double m = 0;
#pragma unroll
                    for (int j = 0; j < 6; j++) m = fmax(m, fabs(sys.v[pk(j, j)]));
                    lambda = 1e-5 * m; ni = 2; nbad = 0;
                }
                double rho = 0;
                int qn = 0;
                do {
                    double sq[4], st[3], x[6];
#pragma unroll
                    for (int i = 0; i < 4; i++) sq[i] = q[i];
#pragma unroll
                    for (int i = 0; i < 3; i++) st[i] = t[i];
                    PO_CNT(7);
                    PO_ACC(5);
                    const bool ok = po_solve(sys, lambda, x);
                    PO_ACC(2);
                    se3_exp_update(x, q, t);   // VertexSE3Expmap::oplusImpl
                    PO_ACC(3);
                    double tmp = po_block_sum1(po_chi_pass(S, E, outl, c, q, t, robust), red, par);
                    PO_ACC(4);
#pragma unroll
                    for (int i = 0; i < 4; i++) qe[i] = q[i];
#pragma unroll
                    for (int i = 0; i < 3; i++) te[i] = t[i];
                    if (!ok) tmp = DBL_MAX;
                    rho = cur - tmp;
                    double sc = 0;   // computeScale (levenberg.cpp:182-190)
#pragma unroll
                    for (int j = 0; j < 6; j++) sc += x[j] * (lambda * x[j] + sys.v[21 + j]);
                    rho /= sc + 1e-3;
                    if (rho > 0 && isfinite(tmp)) {
                        const double u = 2 * rho - 1;   // pow(2 rho - 1, 3) in g2o
                        double alpha = 1. - u * u * u;
                        alpha = fmin(alpha, 2. / 3.);
                        lambda *= fmax(1. / 3., alpha);
                        ni = 2;
                        cur = tmp;
                    } else {
                        lambda *= ni;
                        ni *= 2;
#pragma unroll
                        for (int i = 0; i < 4; i++) q[i] = sq[i];
#pragma unroll
                        for (int i = 0; i < 3; i++) t[i] = st[i];
                    }
                    qn++;
                } while (rho < 0 && qn < 10);
                if (qn == 10 || rho == 0) break;
                if ((ini - cur) * 1e3 < ini) nbad++; else nbad = 0;
                if (nbad >= 3) break;
            }
        }
        // classification (Optimizer.cc:431-481): an edge that was an outlier gets computeError()
        // at the current estimate; the others keep the error of the last computeActiveErrors.
        uint64_t nout_mask = 0;
        int i = 0, cnt = 0;
        for (int e = threadIdx.x; e < E; e += PO_THREADS, i++) {
            const bool was = (outl >> i) & 1;
            PoEdge d;
            po_load(S, e, d);
            double Xc[3], err[3];
            const double chi = was ? po_error(d, c, q, t, Xc, err) : po_error(d, c, qe, te, Xc, err);
            const bool out = chi > (d.stereo ? 7.815 : 5.991);
            nout_mask |= (uint64_t)out << i;
            cnt += out;
        }
        outl = nout_mask;
        noutliers = (int)po_block_sum1((double)cnt, red, par);
        PO_ACC(5);
        if (k == 2) robust = false;   // setRobustKernel(0)
    }
    double Rf[9];
    q_to_R(q, Rf);
    if (threadIdx.x < 9) a.oR[9 * (size_t)f + threadIdx.x] = Rf[threadIdx.x];
    if (threadIdx.x < 3) a.ot[3 * (size_t)f + threadIdx.x] = t[threadIdx.x];
    if (threadIdx.x == 0) a.n_inliers[f] = E - noutliers;
    int i = 0;
    for (int e = threadIdx.x; e < E; e += PO_THREADS, i++) a.outlier[e0 + e] = (uint8_t)((outl >> i) & 1);
}

static int launch_pose_opt(const PoArgs& a, hipStream_t st) {
    if (a.n_frames == 0) return ORB_OK;
    static bool attr = [] {
        return hipFuncSetAttribute((const void*)pose_opt_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)PO_LDS_BYTES) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL(pose_opt_kernel, dim3(a.n_frames), dim3(PO_THREADS), PO_LDS_BYTES, st, a);
    ORB_HIP_TRY(hipGetLastError());
    return ORB_OK;
}

extern "C" int orbba_debug_po_stamps(unsigned long long* out) {
#ifdef ORB_PO_STAMPS
    ORB_HIP_TRY(hipDeviceSynchronize());
    ORB_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_po_stamps), sizeof(g_po_stamps)));
    const unsigned long long z[8] = {0};
    ORB_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_po_stamps), z, sizeof(z)));
    return ORB_OK;
#else
    (void)out;
    set_error("built without ORB_PO_STAMPS");
    return ORB_EINVAL;
#endif
}

// Diagnostic: the wavefront primitives on one wave.  in: 64 lanes x 32 values (lane-major);
// scatter[l] = po_wave_scatter32 result of lane l; sum[l] = po_wave_sum of in[l][0].
__global__ void po_wave_test_kernel(const double* in, double* scatter, double* sum) {
    const int lane = threadIdx.x;
    double v[32];
#pragma unroll
    for (int j = 0; j < 32; j++) v[j] = in[32 * lane + j];
    const double s = po_wave_sum(v[0], lane);
    scatter[lane] = po_wave_scatter32(v, lane);
    sum[lane] = s;
}

extern "C" int orbba_debug_po_wave(const double* in, double* scatter, double* sum) {
    ORB_CHECK_ARG(in && scatter && sum, "null argument");
    DevBuf b;
    int rc;
    if ((rc = b.reserve((64 * 32 + 128) * sizeof(double)))) return rc;
    double* d = b.as<double>();
    ORB_HIP_TRY(hipMemcpy(d, in, 64 * 32 * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(po_wave_test_kernel, dim3(1), dim3(64), 0, nullptr, d, d + 2048, d + 2112);
    ORB_HIP_TRY(hipGetLastError());
    ORB_HIP_TRY(hipMemcpy(scatter, d + 2048, 64 * sizeof(double), hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(sum, d + 2112, 64 * sizeof(double), hipMemcpyDeviceToHost));
    b.release();
    return ORB_OK;
}

struct PoScratch {
    DevBuf buf;
    int device = -1;
};
thread_local PoScratch g_po;

}  // namespace orbamd

using namespace orbamd;

extern "C" int orbba_pose_optimization_device(const orbba_pose_batch* in, orbba_pose_result* out, void* stream) {
    ORB_CHECK_ARG(in && out, "null argument");
    ORB_CHECK_ARG(in->n_frames >= 0, "negative frame count");
    if (in->n_frames == 0) return ORB_OK;
    ORB_CHECK_ARG(in->edge_begin && in->pose_R && in->pose_t && in->cam && in->xw && in->obs && in->inv_sigma2,
                  "null input array");
    ORB_CHECK_ARG(out->pose_R && out->pose_t && out->n_inliers && out->outlier, "null output array");
    PoArgs a{in->n_frames, in->edge_begin, in->pose_R, in->pose_t, in->cam, in->xw, in->obs, in->inv_sigma2,
             out->pose_R, out->pose_t, out->n_inliers, out->outlier};
    return launch_pose_opt(a, (hipStream_t)stream);
}

extern "C" int orbba_pose_optimization(const orbba_pose_batch* in, orbba_pose_result* out, int device) {
    ORB_CHECK_ARG(in && out, "null argument");
    const int n = in->n_frames;
    ORB_CHECK_ARG(n >= 0, "negative frame count");
    if (n == 0) return ORB_OK;
    ORB_CHECK_ARG(in->edge_begin && in->pose_R && in->pose_t && in->cam, "null input array");
    ORB_CHECK_ARG(out->pose_R && out->pose_t && out->n_inliers, "null output array");
    ORB_CHECK_ARG(in->edge_begin[0] == 0, "edge_begin[0] must be 0");
    for (int f = 0; f < n; f++) {
        const int E = in->edge_begin[f + 1] - in->edge_begin[f];
        ORB_CHECK_ARG(E >= 0, "edge_begin must be non-decreasing");
        ORB_CHECK_ARG(E <= ORBBA_POSE_MAX_EDGES, "frame has more than ORBBA_POSE_MAX_EDGES edges");
    }
    const size_t E = (size_t)in->edge_begin[n];
    ORB_CHECK_ARG(E == 0 || (in->xw && in->obs && in->inv_sigma2 && out->outlier), "null edge array");
    ORB_HIP_TRY(hipSetDevice(device));
    if (g_po.device != device) {
        g_po.buf.release();
        g_po.device = device;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += align_up(std::max<size_t>(bytes, 1), 256); return o; };
    const size_t o_eb = take((n + 1) * 4), o_R = take(n * 72), o_t = take(n * 24), o_c = take(n * 40),
                 o_x = take(E * 24), o_o = take(E * 24), o_s = take(E * 8), o_oR = take(n * 72),
                 o_ot = take(n * 24), o_ni = take(n * 4), o_ol = take(E);
    int rc;
    if ((rc = g_po.buf.reserve(off))) return rc;
    char* b = g_po.buf.as<char>();
    ORB_HIP_TRY(hipMemcpy(b + o_eb, in->edge_begin, (n + 1) * 4, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(b + o_R, in->pose_R, n * 72, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(b + o_t, in->pose_t, n * 24, hipMemcpyHostToDevice));
    ORB_HIP_TRY(hipMemcpy(b + o_c, in->cam, n * 40, hipMemcpyHostToDevice));
    if (E) {
        ORB_HIP_TRY(hipMemcpy(b + o_x, in->xw, E * 24, hipMemcpyHostToDevice));
        ORB_HIP_TRY(hipMemcpy(b + o_o, in->obs, E * 24, hipMemcpyHostToDevice));
        ORB_HIP_TRY(hipMemcpy(b + o_s, in->inv_sigma2, E * 8, hipMemcpyHostToDevice));
    }
    PoArgs a{n, (const int32_t*)(b + o_eb), (const double*)(b + o_R), (const double*)(b + o_t),
             (const double*)(b + o_c), (const double*)(b + o_x), (const double*)(b + o_o),
             (const double*)(b + o_s), (double*)(b + o_oR), (double*)(b + o_ot), (int32_t*)(b + o_ni),
             (uint8_t*)(b + o_ol)};
    if ((rc = launch_pose_opt(a, nullptr))) return rc;
    ORB_HIP_TRY(hipMemcpy(out->pose_R, b + o_oR, n * 72, hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(out->pose_t, b + o_ot, n * 24, hipMemcpyDeviceToHost));
    ORB_HIP_TRY(hipMemcpy(out->n_inliers, b + o_ni, n * 4, hipMemcpyDeviceToHost));
    if (E) ORB_HIP_TRY(hipMemcpy(out->outlier, b + o_ol, E, hipMemcpyDeviceToHost));
    return ORB_OK;
}
