// orbba.hip — Optimizer::LocalBundleAdjustment on gfx950.
//
// g2o's Levenberg-Marquardt over SE3Expmap poses and marginalised XYZ points, fp64 throughout.
// Points own their edges (CSR); a point is served by a group of 8 lanes (one edge per lane,
// fixed-order shuffle reductions), so per-point work spreads over ~N/8 wavefronts.
//   per LM trial (OptimizationAlgorithmLevenberg::solve, levenberg.cpp:61-164; the do { ... } while
//   (rho < 0 ...) retries re-run only the lambda-dependent parts), five launches:
//     ba_iter_kernel         on a new iteration: computeActiveErrors + robust chi2 + linearizeOplus +
//                            constructQuadraticForm, Hll / b_l per point, per-edge pose parts; then
//                            (lambda known) D^-1 = (Hll + lambda I)^-1, W = Hpl D^-1, Hpl D^-1 b_l
//     ba_schur_block_kernel  S(i1,i2) = Hpp + lambda I - sum W Hpl^T per block (pair list in parts);
//                            beside them one workgroup per pose: on a new iteration its Hpp / b_p,
//                            then b_schur; and the chi2 total
//     ba_solve_kernel        blocked LDL^T of the (6P)^2 reduced camera system in LDS, triangular
//                            solves, push + SE3 exp-update of the free poses
//     ba_point_update_kernel back-substitution, push, point +=, errors + robust chi2 of its edges
//     ba_decide_kernel       rho, lambda / nu update, accept or pop (restore)
//   The first trial of an optimize() call runs ba_pose_accum_kernel and ba_schur_point_kernel
//   (computeLambdaInit from the diagonal maxima the first two gather, then the Schur point terms)
//   between the first two.
// Every reduction runs in a fixed order, so results are bit-reproducible run to run.  The LM
// control scalars live on the device; the host reads one small status block per trial to decide
// whether to run another (the reference's loop condition), and polls the stop flag like g2o.
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <vector>

#include <chrono>
#include <thread>

#include "ba_structure.h"
#include "common.h"
#include "se3.h"

namespace orbamd {

struct BACtl {
    double lambda, ni, cur, ini, tmp, scale, rho;
    int ok2, accepted;
    double maxdiag;
    unsigned long long maxdiag_bits;   // computeLambdaInit's max |diag H| as the bits of a double >= 0
    // LM loop state, advanced on the device by ba_decide_step (g2o SparseOptimizer::optimize +
    // OptimizationAlgorithmLevenberg::solve): iteration, trial within it, nBad, flags
    int it, q, nbad, done, need_lin, iters_max, iters_done;
    int trials;    // LM trials since the start of the LocalBA call (both optimize() calls; test hook)
    int stopped;   // the force-stop flag ended the loop
    int seq;       // host snapshot sequence id (written last; see ba_decide_step)
    int n_active;  // level-0 edges after the outlier classification between the optimize() calls
    int pad_;
    double chi_out;
};

// Every kernel of an LM step returns at once when the loop has finished (steps are enqueued ahead
// of the host learning that); the linearisation kernels also skip on a retry trial.
#define BA_RETURN_IF_DONE(b) \
    do {                     \
        if ((b).ctl->done) return; \
    } while (0)

// ------------------------------------------------------------------ problem on the device
struct BADev {
    int P, N, E;
    double* q;      // P x 4
    double* t;      // P x 3
    double* q_sv;   // push/pop copies
    double* t_sv;
    double* X;      // N x 3
    double* X_sv;
    const uint8_t* fixed;
    const int* ep;
    const int* ek;
    const uint8_t* stereo;
    int cam_step;         // 5: a camera per edge; 0: one camera for every edge (uploaded once)
    const double* obs;    // E x 3
    const double* info;   // E
    const double* cam;    // E x 5
    uint8_t* robust;      // E
    double* err;          // E x 3 (last computed error, g2o's _error)
    const uint8_t* level; // E: g2o edge level; only level-0 edges take part (initializeOptimization(0))
    // active structure
    int Ea, np, nl, nblk;
    const int* act;       // Ea: edge id per active slot (ascending edge id)
    const int* hp;        // P: hessian index or -1
    const int* hl;        // N: point index or -1
    const int* pt_beg;    // nl+1: CSR of active slots per active point (slot order)
    const int* pt_slot;
    int4* pt_rec;         // Ea, per point-list entry u: {k = pt_slot[u], e = act[k], pose ek[e], hp[ek[e]]}
    const int* pt_id;     // nl: point id of point index
    const int* ps_beg;    // np+1: CSR of active slots per free pose
    const int* ps_slot;
    const int* ps_id;     // np: pose id
    const int* blk_i1;    // nblk
    const int* blk_i2;
    const int* blk_beg;   // nblk+1: CSR of (slot1, slot2) pairs
    const int2* blk_pair;
    // per active slot products
    double* J;            // Ea x 72: Hll(9) bl(3) Hpp(36) bp(6) Hpl(18, pose-major 6x3)
    double* W;            // Ea x 24: W = Hpl Dinv (18) | Hpl Dinv b_l (6)
    // per point / pose system
    double* Hll;          // nl x 9
    double* bl;           // nl x 3
    double* Dinv;         // nl x 9
    double* Hpp;          // np x 36
    double* bp;           // np x 6
    double* S;            // D x D reduced system
    double* Sg;           // Dp x (Dp+1) padded working copy for the global-memory solve (D > 128), else null
    double* bs;           // D
    double* x;            // D + 3 nl
    double* rchi;         // Ea: robust chi2 per active slot
    double* part;         // scale partials: nl + np
    double* Spart;         // the Schur-block parts' partial blocks (+ Hpp): (SB_SPLIT + 1) x nblk x 36 for the
                           // global solve, (SB_SPLIT + 1) row-major D x D matrices (both orientations) for the LDS solve
    unsigned* blk_done;    // nblk: parts of the block finished (the last one forms S)
    const int* blk_diag;   // np: block index of the diagonal block (i, i)
    BACtl* ctl;
    const int32_t* stop;   // device view of the host's force-stop flag (mapped pinned mirror), or null
    int stop_after;        // test hook: stop once this many trials have run (-1: off)
};

__device__ __forceinline__ double edge_chi2(const BADev& b, int e) {
    const int d = b.stereo[e] ? 3 : 2;
    double s = 0;
    for (int i = 0; i < d; i++) s += b.err[3 * e + i] * b.info[e] * b.err[3 * e + i];
    return s;
}
__device__ __forceinline__ void robustify(const BADev& b, int e, double chi, double& r0, double& r1) {
    if (!b.robust[e]) { r0 = chi; r1 = 1.0; return; }
    const double delta = b.stereo[e] ? sqrt(7.815) : sqrt(5.991);   // Optimizer.cc:44-47
    const double dsqr = delta * delta;
    if (chi <= dsqr) { r0 = chi; r1 = 1.0; }
    else { const double s = sqrt(chi); r0 = 2 * s * delta - dsqr; r1 = delta / s; }   // robust_kernel_impl.cpp:78-91
}

// EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::computeError (types_six_dof_expmap.h:90-95,122-127)
// for edge e with camera-frame point Xc; stores g2o's _error and returns the robust chi2 term.
__device__ __forceinline__ double edge_error(const BADev& b, int e, const double* Xc) {
    const double* c = b.cam + b.cam_step * e;
    const double* z = b.obs + 3 * e;
    if (!b.stereo[e]) {
        b.err[3 * e + 0] = z[0] - (Xc[0] / Xc[2] * c[0] + c[2]);
        b.err[3 * e + 1] = z[1] - (Xc[1] / Xc[2] * c[1] + c[3]);
        b.err[3 * e + 2] = 0;
    } else {   // cam_project(..., bf): invz narrowed to float, bf*invz in float (.cpp:148-156)
        const float invz = 1.0f / Xc[2];
        const float bf = (float)c[4];
        const double u = Xc[0] * invz * c[0] + c[2];
        const double v = Xc[1] * invz * c[1] + c[3];
        b.err[3 * e + 0] = z[0] - u;
        b.err[3 * e + 1] = z[1] - v;
        b.err[3 * e + 2] = z[2] - (u - (double)(bf * invz));
    }
    double r0, r1;
    robustify(b, e, edge_chi2(b, e), r0, r1);
    return r0;
}

// fixed-order sum over the 8-lane group of a point
__device__ __forceinline__ double grp_sum(double v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    return v;
}

constexpr int GRP = 8;   // lanes per point

__device__ __forceinline__ bool inv3(const double* m, double* o);

// BlockSolver::solve, landmark part (block_solver.hpp:377-419) for point l: every lane of the point's
// group forms D^-1 = (Hll + lambda I)^-1 (same values), each lane handles its edges'
// W = Hpl D^-1 and Hpl D^-1 b_l.  H / bl are the point's Hll / b_l (identical in every lane).
__device__ __forceinline__ void schur_point_terms(const BADev& b, int l, int sub, const double (&H)[9],
                                                  const double (&bl)[3], double lam) {
    double D[9], Di[9];
#pragma unroll
    for (int i = 0; i < 9; i++) D[i] = H[i];
    D[0] += lam; D[4] += lam; D[8] += lam;
    inv3(D, Di);
    if (sub == 0)
        for (int i = 0; i < 9; i++) b.Dinv[9 * l + i] = Di[i];
    double db[3];
#pragma unroll
    for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
    for (int u = b.pt_beg[l] + sub; u < b.pt_beg[l + 1]; u += GRP) {
        const int4 rc = b.pt_rec[u];
        if (rc.w < 0) continue;
        const int k = rc.x;
        const double* Hpl = b.J + (long long)k * 72 + 54;
        double* W = b.W + (long long)k * 24;
        for (int r = 0; r < 6; r++) {
            for (int c = 0; c < 3; c++)
                W[3 * r + c] = Hpl[3 * r] * Di[c] + Hpl[3 * r + 1] * Di[3 + c] + Hpl[3 * r + 2] * Di[6 + c];
            W[18 + r] = Hpl[3 * r] * db[0] + Hpl[3 * r + 1] * db[1] + Hpl[3 * r + 2] * db[2];
        }
    }
}

// Per LM trial, point side.  On a linearising trial: errors + robust chi2 (computeActiveErrors /
// activeRobustChi2), linearizeOplus and constructQuadraticForm of every active edge
// (types_six_dof_expmap.cpp:103-139,188-234; base_binary_edge.hpp:54-120), Hll / b_l summed per
// point, pose parts stored per edge.  Then, once lambda is known (every trial but the very first of
// an optimize() call, whose lambda comes from computeLambdaInit), the point's Schur terms; a retry
// trial (rho < 0) does only those, with the new lambda.
__global__ __launch_bounds__(64) void ba_iter_kernel(BADev b) {
    if (b.ctl->done) return;
    const bool lin = b.ctl->need_lin != 0;
    const bool schur = !lin || b.ctl->it > 0;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = t / GRP, sub = t % GRP;
    const bool live = l < b.nl;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0}, chi = 0;
    if (!lin) {
        if (live) {
#pragma unroll
            for (int i = 0; i < 9; i++) H[i] = b.Hll[9 * l + i];
#pragma unroll
            for (int i = 0; i < 3; i++) g[i] = b.bl[3 * l + i];
            schur_point_terms(b, l, sub, H, g, b.ctl->lambda);
        }
        return;
    }
    if (live) {
        const double* Xl = b.X + 3 * b.pt_id[l];   // = X + 3 ep[e] for every edge of the point
        for (int u = b.pt_beg[l] + sub; u < b.pt_beg[l + 1]; u += GRP) {
            const int4 rc = b.pt_rec[u];
            const int k = rc.x, e = rc.y;
            if (b.level[e]) {   // a level-1 edge (second optimize()): no error, no terms -- its pose-side
                                // terms are zeros (written here: the call no longer clears J per optimize())
                if (rc.w >= 0) {
                    double* J = b.J + (long long)k * 72;
#pragma unroll
                    for (int i = 12; i < 72; i++) J[i] = 0.0;
                }
                continue;
            }
            const int pi = rc.z;
            const double* q4 = b.q + 4 * pi;
            double Xc[3], R[9];
            se3_map(q4, b.t + 3 * pi, Xl, Xc);
            chi += edge_error(b, e, Xc);
            q_to_R(q4, R);
            // Jacobians with one reciprocal of z (g2o divides by z / z^2 in every term; the
            // difference is rounding-level, within the LocalBA tolerance)
            const double x = Xc[0], y = Xc[1], z = Xc[2];
            const double iz = 1.0 / z, iz2 = iz * iz;
            const double* c = b.cam + b.cam_step * e;
            const double fx = c[0], fy = c[1], bf = c[4];
            const bool st = b.stereo[e];
            const int d = st ? 3 : 2;
            double A[3][3], Bm[3][6];
            if (!st) {
                const double tmp[2][3] = {{fx, 0, -x * iz * fx}, {0, fy, -y * iz * fy}};
                for (int r = 0; r < 2; r++)
                    for (int j = 0; j < 3; j++) {
                        double s = 0;
                        for (int m = 0; m < 3; m++) s += tmp[r][m] * R[3 * m + j];
                        A[r][j] = -iz * s;
                    }
                for (int j = 0; j < 3; j++) A[2][j] = 0;
            } else {
                for (int j = 0; j < 3; j++) {
                    A[0][j] = -fx * R[j] * iz + fx * x * R[6 + j] * iz2;
                    A[1][j] = -fy * R[3 + j] * iz + fy * y * R[6 + j] * iz2;
                    A[2][j] = A[0][j] - bf * R[6 + j] * iz2;
                }
            }
            Bm[0][0] = x * y * iz2 * fx; Bm[0][1] = -(1 + (x * x * iz2)) * fx; Bm[0][2] = y * iz * fx;
            Bm[0][3] = -iz * fx;         Bm[0][4] = 0;                         Bm[0][5] = x * iz2 * fx;
            Bm[1][0] = (1 + y * y * iz2) * fy; Bm[1][1] = -x * y * iz2 * fy; Bm[1][2] = -x * iz * fy;
            Bm[1][3] = 0;                      Bm[1][4] = -iz * fy;          Bm[1][5] = y * iz2 * fy;
            if (st) {
                Bm[2][0] = Bm[0][0] - bf * y * iz2; Bm[2][1] = Bm[0][1] + bf * x * iz2; Bm[2][2] = Bm[0][2];
                Bm[2][3] = Bm[0][3];                Bm[2][4] = 0;                       Bm[2][5] = Bm[0][5] - bf * iz2;
            } else {
                for (int j = 0; j < 6; j++) Bm[2][j] = 0;
            }
            double r0, r1;
            robustify(b, e, edge_chi2(b, e), r0, r1);
            const double w = r1 * b.info[e];
            // row 2 of A / Bm and om_r[2] are zero for a mono edge, so the fixed 3-row sums add exact
            // zeros to the reference's 2-row sums (same values) and every array stays in registers
            double om_r[3];
#pragma unroll
            for (int r = 0; r < 3; r++) om_r[r] = r < d ? -b.info[e] * b.err[3 * e + r] * r1 : 0.0;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                double s = 0;
#pragma unroll
                for (int r = 0; r < 3; r++) s += A[r][i] * om_r[r];
                g[i] += s;
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    double h = 0;
#pragma unroll
                    for (int r = 0; r < 3; r++) h += A[r][i] * w * A[r][j];
                    H[3 * i + j] += h;
                }
            }
            if (rc.w >= 0) {   // free pose
                double* J = b.J + (long long)k * 72;
#pragma unroll
                for (int i = 0; i < 6; i++) {
                    double s = 0;
#pragma unroll
                    for (int r = 0; r < 3; r++) s += Bm[r][i] * om_r[r];
                    J[48 + i] = s;
#pragma unroll
                    for (int j = 0; j < 6; j++) {
                        double h = 0;
#pragma unroll
                        for (int r = 0; r < 3; r++) h += Bm[r][i] * w * Bm[r][j];
                        J[12 + 6 * i + j] = h;
                    }
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        double h = 0;
#pragma unroll
                        for (int r = 0; r < 3; r++) h += Bm[r][i] * w * A[r][j];
                        J[54 + 3 * i + j] = h;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 9; i++) H[i] = grp_sum(H[i]);
#pragma unroll
    for (int i = 0; i < 3; i++) g[i] = grp_sum(g[i]);
    chi = grp_sum(chi);
    if (b.ctl->it == 0) {   // first trial of an optimize(): computeLambdaInit's max over the points' diagonals
        double m = live && sub == 0 ? fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8]))) : 0.0;
        for (int o = 32; o >= GRP; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
        if (threadIdx.x == 0 && m > 0)
            atomicMax(&b.ctl->maxdiag_bits, (unsigned long long)__double_as_longlong(m));
    }
    if (live && sub == 0) {
        for (int i = 0; i < 9; i++) b.Hll[9 * l + i] = H[i];
        for (int i = 0; i < 3; i++) b.bl[3 * l + i] = g[i];
        b.rchi[l] = chi;
    }
    // the lane's own J writes above are visible to its own reads in schur_point_terms
    if (live && schur) schur_point_terms(b, l, sub, H, g, b.ctl->lambda);
}

// Deterministic single-workgroup sum (fixed strided order + fixed tree).
__device__ double block_sum_1024(const double* v, int n, double* sh) {
    double s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += v[i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

// One workgroup (1008 threads) per free pose: 42 sums (Hpp 36 + b 6), 24 partial groups with
// four interleaved accumulators each, combined in a fixed order.  Block np: chi2 total.
constexpr int PA_G = 24;
constexpr int PA_SLOTS = 4096;   // a pose's edge-slot list staged in LDS when it has at most this many
__device__ __forceinline__ void stage_pose_slots(const BADev& b, int i, int* sslot) {
    const int beg = b.ps_beg[i], n = b.ps_beg[i + 1] - beg;
    if (n <= PA_SLOTS)
        for (int u = threadIdx.x; u < n; u += blockDim.x) sslot[u] = b.ps_slot[beg + u];
}
__device__ __forceinline__ void pose_accum(const BADev& b, int i, double* sh, const int* sslot);
__device__ __forceinline__ void chi_total(const BADev& b, double* sh) {
    const double c = block_sum_1024(b.rchi, b.nl, sh);
    if (threadIdx.x == 0) {
        b.ctl->cur = c;
        b.ctl->ini = c;
    }
}
// The first trial of an optimize() call (computeLambdaInit needs Hpp before the Schur step);
// later linearising trials accumulate inside ba_schur_block_kernel.
__global__ __launch_bounds__(1024) void ba_pose_accum_kernel(BADev b) {
    if (b.ctl->done || !b.ctl->need_lin) return;
    __shared__ double sh[1024];
    __shared__ int sslot[PA_SLOTS];
    if ((int)blockIdx.x == b.np) chi_total(b, sh);
    else {
        stage_pose_slots(b, blockIdx.x, sslot);
        __syncthreads();
        pose_accum(b, blockIdx.x, sh, sslot);   // ends with a barrier: Hpp visible to the workgroup
        if (threadIdx.x == 0) {   // computeLambdaInit's max over this pose's diagonal
            double m = 0;
            for (int k = 0; k < 6; k++) m = fmax(m, fabs(b.Hpp[36 * blockIdx.x + 7 * k]));
            if (m > 0) atomicMax(&b.ctl->maxdiag_bits, (unsigned long long)__double_as_longlong(m));
        }
    }
}
// (the caller staged the pose's slots with stage_pose_slots and a barrier; a pose with more than
// PA_SLOTS edges reads them from HBM)
__device__ __forceinline__ void pose_accum(const BADev& b, int i, double* sh, const int* sslot) {
    const int g = threadIdx.x / 42, c = threadIdx.x % 42;
    const int beg = b.ps_beg[i], end = b.ps_beg[i + 1];
    auto sum = [&](auto slot) {   // slot(u), u in [beg, end): LDS-staged or HBM (two instantiations)
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        int u = beg + g;
        for (; u + 3 * PA_G < end; u += 4 * PA_G) {
            s0 += b.J[(long long)slot(u) * 72 + 12 + c];
            s1 += b.J[(long long)slot(u + PA_G) * 72 + 12 + c];
            s2 += b.J[(long long)slot(u + 2 * PA_G) * 72 + 12 + c];
            s3 += b.J[(long long)slot(u + 3 * PA_G) * 72 + 12 + c];
        }
        for (; u < end; u += PA_G) s0 += b.J[(long long)slot(u) * 72 + 12 + c];
        sh[g * 42 + c] = (s0 + s1) + (s2 + s3);
    };
    if (g < PA_G) {
        if (end - beg <= PA_SLOTS) sum([&](int u) { return sslot[u - beg]; });
        else sum([&](int u) { return b.ps_slot[u]; });
    }
    __syncthreads();
    if (threadIdx.x < 42) {
        double s = 0;
        for (int q = 0; q < PA_G; q++) s += sh[q * 42 + threadIdx.x];
        if (threadIdx.x < 36) b.Hpp[36 * i + threadIdx.x] = s;
        else b.bp[6 * i + threadIdx.x - 36] = s;
    }
    __syncthreads();   // sh reused by the caller; Hpp / bp read back by the same workgroup
}

__device__ __forceinline__ bool inv3(const double* m, double* o) {
    const double c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8], c02 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
    if (det == 0) return false;
    const double id = 1.0 / det;
    o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    o[3] = c01 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    o[6] = c02 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
    return true;
}

// The first trial of an optimize() call: computeLambdaInit (levenberg.cpp:166-180: tau * max |diag H|
// over the active vertices, the max gathered by ba_iter_kernel and ba_pose_accum_kernel), then the
// Schur point terms with that lambda.
__global__ __launch_bounds__(64) void ba_schur_point_kernel(BADev b) {
    BA_RETURN_IF_DONE(b);
    const double maxdiag = __longlong_as_double((long long)b.ctl->maxdiag_bits);
    const double lam = 1e-5 * maxdiag;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) {
        b.ctl->maxdiag = maxdiag;
        b.ctl->lambda = lam;
        b.ctl->ni = 2;
    }
    const int l = t / GRP, sub = t % GRP;
    if (l >= b.nl) return;
    double H[9], g[3];
#pragma unroll
    for (int i = 0; i < 9; i++) H[i] = b.Hll[9 * l + i];
#pragma unroll
    for (int i = 0; i < 3; i++) g[i] = b.bl[3 * l + i];
    schur_point_terms(b, l, sub, H, g, lam);
}

// Reduced camera system block (i1, i2): 36 entries x 28 partial groups (two accumulators each),
// fixed-order combine.
// The pair list of a block is split into SB_SPLIT contiguous parts, one workgroup each (blockIdx.y),
// each storing its partial block (device-coherent stores, completed before it counts in); the last
// part of a block to count in adds the partials in part order and writes the block of S.
// Per free pose one more workgroup (blockIdx.x = nblk + 1 + i, part 0): with `accum` (every step but
// an optimize() call's first) on a linearising trial the Hpp / b_p sums of its pose (what
// ba_pose_accum_kernel would do), then b_schur = b_p - sum Hpp D^-1 b_l; it counts in on the pose's
// diagonal block as one more part, so the diagonal block's last arriver finds Hpp published and forms
// part 0 + Hpp + lambda I exactly as part 0 itself used to (same rounding).  Workgroup nblk: the chi2
// total.  (Round 3: the pose sums and b_schur ran inside the diagonal blocks' part 0, after its pair
// loop, on the kernel's critical path.)
constexpr int SB_G = 28;
#ifndef SB_SPLIT_DEF
#define SB_SPLIT_DEF 2
#endif
constexpr int SB_SPLIT = SB_SPLIT_DEF;

// count in on block blk (expect arrivals in all); the last arriver forms the block of S
__device__ __forceinline__ void schur_block_count_in(const BADev& b, int blk, int D, int expect) {
    __shared__ int s_last;
    // Hand-off by the memory model: the partials' stores happen before thread 0's agent-scope
    // release (workgroup barrier), and the last part's agent-scope acquire happens before its loads
    // (the same barrier pattern on the consumer side).  Callers publish the partial from threads of
    // wavefront 0 only (the wavefront of the counting thread).
    __syncthreads();
    if (threadIdx.x == 0) {
#ifndef ORBBA_DIAG_RELAXED_COUNTIN
        s_last = __hip_atomic_fetch_add(&b.blk_done[blk], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)expect - 1;
        if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#else   // timing diagnostic only (no hand-off ordering; results may be wrong): the cost of the release
        s_last = __hip_atomic_fetch_add(&b.blk_done[blk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)expect - 1;
#endif
    }
    __syncthreads();
    if (s_last && threadIdx.x < 36) {
        const int i1 = b.blk_i1[blk], i2 = b.blk_i2[blk];
        const int r = threadIdx.x / 6, cc = threadIdx.x % 6;
        double v = 0;
        for (int k = 0; k < SB_SPLIT; k++) {
            double pk = b.Spart[((long long)k * b.nblk + blk) * 36 + threadIdx.x];
            if (k == 0 && i1 == i2) {   // part 0 + Hpp (the pose workgroup's part) + lambda I, in that order
                pk += b.Spart[((long long)SB_SPLIT * b.nblk + blk) * 36 + threadIdx.x];
                if (r == cc) pk += b.ctl->lambda;
            }
            v += pk;
        }
        b.S[(long long)(6 * i1 + r) * D + 6 * i2 + cc] = v;
        if (i1 != i2) b.S[(long long)(6 * i2 + cc) * D + 6 * i1 + r] = v;
        if (threadIdx.x == 0) __hip_atomic_store(&b.blk_done[blk], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(1024) void ba_schur_block_kernel(BADev b, int D, int accum, int direct) {
    BA_RETURN_IF_DONE(b);
    __shared__ double sh[1024];
    __shared__ int sslot[PA_SLOTS];
    const int blk = blockIdx.x, part = blockIdx.y;
    const bool acc = accum && b.ctl->need_lin;
    if (blk == b.nblk) {
        if (acc && part == 0) chi_total(b, sh);
        return;
    }
    if (blk > b.nblk) {   // pose workgroup
        if (part != 0) return;
        const int i1 = blk - b.nblk - 1;
        stage_pose_slots(b, i1, sslot);   // the pose's edge slots (no dependent HBM loads below)
        __syncthreads();
#ifndef BA_DIAG_NO_PA   // diagnostic timing builds only (wrong results): tools/probe/ba_schur_parts.sh
        if (acc) {
            pose_accum(b, i1, sh, sslot);
            __syncthreads();   // b_p of this trial (global, this workgroup's stores) before b_schur
        }
#endif
        // b_schur for pose i1: 6 entries x 168 partial groups
        const int g2 = threadIdx.x / 6, c2 = threadIdx.x % 6;
        double s = 0;
        {
            const int beg = b.ps_beg[i1], end = b.ps_beg[i1 + 1];
            if (g2 < 168) {
                if (end - beg <= PA_SLOTS)
                    for (int u = beg + g2; u < end; u += 168) s += b.W[(long long)sslot[u - beg] * 24 + 18 + c2];
                else
                    for (int u = beg + g2; u < end; u += 168) s += b.W[(long long)b.ps_slot[u] * 24 + 18 + c2];
            }
        }
        sh[threadIdx.x] = g2 < 168 ? s : 0.0;
        __syncthreads();
        // two-level fixed-order sum of the 168 partials per entry (8 runs of 21, then the 8 run sums)
        // instead of one 168-long dependent chain on 6 threads
        double run = 0;
        if (threadIdx.x < 48) {
            const int e = threadIdx.x % 6, h = threadIdx.x / 6;
            for (int q = 21 * h; q < 21 * h + 21; q++) run += sh[q * 6 + e];
        }
        __syncthreads();
        if (threadIdx.x < 48) sh[threadIdx.x] = run;
        __syncthreads();
        if (threadIdx.x < 6) {
            double tot = 0;
            for (int h = 0; h < 8; h++) tot += sh[6 * h + threadIdx.x];
            b.bs[6 * i1 + threadIdx.x] = b.bp[6 * i1 + threadIdx.x] - tot;
        }
        // Hpp (this trial's or the kept one) as the diagonal block's extra part, republished by
        // wavefront 0 so that the counting wavefront's own release orders it
        if (direct) {   // the LDS solve sums the parts itself (no count-in)
            if (threadIdx.x < 36)
                b.Spart[((long long)SB_SPLIT * D + 6 * i1 + threadIdx.x / 6) * D + 6 * i1 + threadIdx.x % 6] =
                    b.Hpp[36 * i1 + threadIdx.x];
            return;
        }
        const int dblk = b.blk_diag[i1];
        if (threadIdx.x < 36) b.Spart[((long long)SB_SPLIT * b.nblk + dblk) * 36 + threadIdx.x] = b.Hpp[36 * i1 + threadIdx.x];
        schur_block_count_in(b, dblk, D, SB_SPLIT + 1);
        return;
    }
    const int i1 = b.blk_i1[blk], i2 = b.blk_i2[blk];
    const int g = threadIdx.x / 36, c = threadIdx.x % 36;
    const int r = c / 6, cc = c % 6;
    if (g < SB_G) {
        double s0 = 0, s1 = 0;
        const int pb = b.blk_beg[blk], pn = b.blk_beg[blk + 1] - pb;
        const int end = pb + (int)(((long long)pn * (part + 1)) / SB_SPLIT);
        int u = pb + (int)(((long long)pn * part) / SB_SPLIT) + g;
        for (; u + SB_G < end; u += 2 * SB_G) {
            const int2 p0 = b.blk_pair[u], p1 = b.blk_pair[u + SB_G];
            const double* W0 = b.W + (long long)p0.x * 24 + 3 * r;
            const double* H0 = b.J + (long long)p0.y * 72 + 54 + 3 * cc;
            const double* W1 = b.W + (long long)p1.x * 24 + 3 * r;
            const double* H1 = b.J + (long long)p1.y * 72 + 54 + 3 * cc;
            s0 += W0[0] * H0[0] + W0[1] * H0[1] + W0[2] * H0[2];
            s1 += W1[0] * H1[0] + W1[1] * H1[1] + W1[2] * H1[2];
        }
        if (u < end) {
            const int2 p0 = b.blk_pair[u];
            const double* W0 = b.W + (long long)p0.x * 24 + 3 * r;
            const double* H0 = b.J + (long long)p0.y * 72 + 54 + 3 * cc;
            s0 += W0[0] * H0[0] + W0[1] * H0[1] + W0[2] * H0[2];
        }
        sh[g * 36 + c] = s0 + s1;
    }
    __syncthreads();
    if (threadIdx.x < 36) {
        double s = 0;
        for (int q = 0; q < SB_G; q++) s += sh[q * 36 + threadIdx.x];
        if (direct) {   // part matrix `part`, both orientations (as S itself)
            double* Sp = b.Spart + (long long)part * D * D;
            Sp[(long long)(6 * i1 + r) * D + 6 * i2 + cc] = -s;
            if (i1 != i2) Sp[(long long)(6 * i2 + cc) * D + 6 * i1 + r] = -s;
        } else {
            b.Spart[((long long)part * b.nblk + blk) * 36 + threadIdx.x] = -s;
        }
    }
    if (!direct) schur_block_count_in(b, blk, D, i1 == i2 ? SB_SPLIT + 1 : SB_SPLIT);
}


__device__ __forceinline__ double readlane_d(double v, int lane) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffff), lane);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// Reduced camera system solve + pose update: right-looking blocked LDL^T of the (6P)^2 system in
// LDS, padded with identity to Dp = 16*ceil(D/16) so every block is a full 16 columns (the padded
// unknowns solve to 0).  Row stride Dp+1 (odd) keeps column walks bank-conflict free.  The forward
// substitution is carried along; back substitution is blocked.  Per block J:
//   (1) wavefront 0: LDL^T of the 16x16 diagonal block in registers (lane i owns row i, pivot rows
//       broadcast with v_readlane, branch-free), z_J, and Linv_JJ = L_JJ^-1 (kept in the unused upper
//       triangle of the block: Linv[j][k] at (k, j));
//   (2) panel, one thread per row: U_iJ = A_iJ Linv_JJ^T (= L_iJ D_J) as independent dot products;
//       y_i -= L_iJ z_J;
//   (3) trailing A_ik -= U_iJ D_J^-1 U_kJ^T on the lower triangle: thread (ty, tx) of a 16x16 grid
//       owns rows R0+ty+16a, columns R0+tx+16c (c <= a), so a wavefront walks 16 consecutive rows.
constexpr int SB = 16;

#ifdef ORB_BA_STAMPS
__device__ unsigned long long g_ba_stamps[64];
#define BA_STAMP(k)                                                                              \
    do {                                                                                         \
        if (threadIdx.x == 0 && (k) < 64) g_ba_stamps[(k)] = __builtin_amdgcn_s_memtime();       \
    } while (0)
#define BA_STAMPW(k)                                                                             \
    do {                                                                                         \
        if ((threadIdx.x & 63) == 0 && (k) < 64) g_ba_stamps[(k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define BA_STAMP(k) do {} while (0)
#define BA_STAMPW(k) do {} while (0)
#endif

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

typedef double d4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int solve_dp(int D) { return (D + SB - 1) / SB * SB; }
__host__ __device__ constexpr size_t solve_lds_doubles(int D) {
    return (size_t)solve_dp(D) * (solve_dp(D) + 1) + 3 * (size_t)solve_dp(D);
}

#ifndef ORBBA_NEWTON
#define ORBBA_NEWTON 2
#endif
__device__ __forceinline__ double rcp_d(double d) {   // 1/d: v_rcp_f64 + ORBBA_NEWTON Newton steps
    double r = __builtin_amdgcn_rcp(d);
#pragma unroll
    for (int k = 0; k < ORBBA_NEWTON; k++) {
        const double e = fma(-d, r, 1.0);
        r = fma(r, e, r);
    }
    return r;
}

// A_ik -= sum_j U_ij dinv_j U_kj for the NBK x NBK lower block-triangle below block J.
template <int NBK>
__device__ __forceinline__ void trailing_update(double* A, const double* dinv, int ld, int J0, int R0, int tid) {
    const int ty = tid >> 4, tx = tid & 15;
    double acc[NBK][NBK];
#pragma unroll
    for (int a = 0; a < NBK; a++)
#pragma unroll
        for (int c = 0; c < NBK; c++) acc[a][c] = 0;
    const double* wrow = A + (R0 + ty) * ld + J0;
    const double* lrow = A + (R0 + tx) * ld + J0;
#pragma unroll 4
    for (int j = 0; j < SB; j++) {
        const double dj = dinv[J0 + j];
        double wi[NBK], lk[NBK];
#pragma unroll
        for (int a = 0; a < NBK; a++) {
            wi[a] = wrow[SB * a * ld + j];
            lk[a] = lrow[SB * a * ld + j] * dj;
        }
#pragma unroll
        for (int a = 0; a < NBK; a++)
#pragma unroll
            for (int c = 0; c <= a; c++) acc[a][c] = fma(wi[a], lk[c], acc[a][c]);
    }
#pragma unroll
    for (int a = 0; a < NBK; a++)
#pragma unroll
        for (int c = 0; c <= a; c++) A[(R0 + ty + SB * a) * ld + R0 + tx + SB * c] -= acc[a][c];
}

// v_fmac_f64 with src0 = lane J's value of each 16-lane row (DPP row_newbcast): r += bcast_J(r) * nl,
// and the plain broadcast.  The compiler's hazard recognizer does not look inside inline asm, so each
// statement carries the 2 wait states a DPP read needs after a VALU write of its source (s_nop 1);
// the code that uses them has no EXEC writes (no divergent branches), whose DPP hazard is 5 states.
// The statements are not volatile, so the scheduler may interleave independent ones.
template <int J>
__device__ __forceinline__ void fmac_bcast_t(double& r, double nl) {
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(nl), "n"(J));
}
template <int J>
__device__ __forceinline__ double bcast_nop_t(double v) {
    double o;
    asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(o) : "v"(v), "n"(J));
    return o;
}
// j must fold to a constant after unrolling
__device__ __forceinline__ void fmac_bcast(double& r, double nl, int j) {
    switch (j) {
        case 0: fmac_bcast_t<0>(r, nl); break;
        case 1: fmac_bcast_t<1>(r, nl); break;
        case 2: fmac_bcast_t<2>(r, nl); break;
        case 3: fmac_bcast_t<3>(r, nl); break;
        case 4: fmac_bcast_t<4>(r, nl); break;
        case 5: fmac_bcast_t<5>(r, nl); break;
        case 6: fmac_bcast_t<6>(r, nl); break;
        case 7: fmac_bcast_t<7>(r, nl); break;
        case 8: fmac_bcast_t<8>(r, nl); break;
        case 9: fmac_bcast_t<9>(r, nl); break;
        case 10: fmac_bcast_t<10>(r, nl); break;
        case 11: fmac_bcast_t<11>(r, nl); break;
        case 12: fmac_bcast_t<12>(r, nl); break;
        case 13: fmac_bcast_t<13>(r, nl); break;
        case 14: fmac_bcast_t<14>(r, nl); break;
        default: fmac_bcast_t<15>(r, nl); break;
    }
}
__device__ __forceinline__ double bcast_nop(double v, int j) {
    switch (j) {
        case 0: return bcast_nop_t<0>(v);
        case 1: return bcast_nop_t<1>(v);
        case 2: return bcast_nop_t<2>(v);
        case 3: return bcast_nop_t<3>(v);
        case 4: return bcast_nop_t<4>(v);
        case 5: return bcast_nop_t<5>(v);
        case 6: return bcast_nop_t<6>(v);
        case 7: return bcast_nop_t<7>(v);
        case 8: return bcast_nop_t<8>(v);
        case 9: return bcast_nop_t<9>(v);
        case 10: return bcast_nop_t<10>(v);
        case 11: return bcast_nop_t<11>(v);
        case 12: return bcast_nop_t<12>(v);
        case 13: return bcast_nop_t<13>(v);
        case 14: return bcast_nop_t<14>(v);
        default: return bcast_nop_t<15>(v);
    }
}

// Diagonal block J0 of the blocked LDL^T on ONE wavefront, in registers: lane i (of every 16-lane
// row; the four rows hold the same copy of r and y) owns row i of the block (r), of Linv = L_JJ^-1 (x;
// 16-lane row q holds Linv's columns 4m + q, so a pivot updates j / 4 + 1 x registers instead of
// j + 1: 4.5k -> 3.7k ticks per block alone, tools/probe/diag_probe.hip) and the rhs entry y_i.  Pivot j: d_j and 1/d_j by a DPP broadcast + v_rcp_f64 and two Newton steps,
// nl_i = -L_ij (rows below the pivot, else 0), then fused broadcast-FMAs: the trailing columns
// r_k += nl * r_j[k], the forward substitution y_i += nl * z_j and the inverse rows
// x_i[c] += nl * x_j[c] (c <= j: row j of Linv is final after pivot j-1).  The next pivot's column is
// updated first, so its broadcast and reciprocal chain interleave with the rest of the step
// (ordered volatile asm from tools/gen_ba_diag.py: the in-order issue then hides the chain).
// Outputs: dinv_J, z_J (in y), Linv in the block's upper triangle (Linv[i][c] at (c, i), c < i) and
// vz_J = Linv^T D^-1 z_J; the lower triangle is not needed by the later steps.
__device__ __forceinline__ bool solve_diag_block(double* A, double* y, double* dinv, double* vz, int ld, int J0,
                                                 int lane, int nreal) {
    const int i = lane & (SB - 1);
    double r[SB], x[SB / 4];   // x[m]: Linv column 4m + q on the lanes of 16-lane row q
#pragma unroll
    for (int k = 0; k < SB; k++) r[k] = A[(J0 + max(i, k)) * ld + J0 + min(i, k)];
#pragma unroll
    for (int m = 0; m < SB / 4; m++) x[m] = 4 * m + (lane >> 4) == i ? 1.0 : 0.0;
    double yi = y[J0 + i];
    double rci = 1.0;   // 1/d_i (identity padding rows: d = 1)
    bool ok = true;
    double dj = bcast_nop(r[0], 0);
    double rc = rcp_d(dj);
    // 16 pivot steps, unrolled with the next pivot's broadcast + reciprocal interleaved into the
    // current step's broadcast-FMAs (tools/gen_ba_diag.py)
#ifndef ORBBA_DIAG_INC
#define ORBBA_DIAG_INC "orbba_diag.inc"
#endif
#include ORBBA_DIAG_INC
    if (lane < SB) {
        dinv[J0 + i] = rci;
        y[J0 + i] = yi;
    }
#pragma unroll
    for (int m = 0; m < SB / 4; m++) {   // every 16-lane row stores its Linv columns
        const int c = 4 * m + (lane >> 4);
        if (c < i) A[(J0 + c) * ld + J0 + i] = x[m];
    }
    wave_lds_sync();
    // v_c = sum_{j >= c} Linv[j][c] dinv_j z_j
    double v = dinv[J0 + i] * y[J0 + i];
#pragma unroll
    for (int j = 1; j < SB; j++) {
        const double lv = A[(J0 + min(i, j)) * ld + J0 + j];   // Linv[j][i] for j > i
        v = fma(j > i ? lv : 0.0, dinv[J0 + j] * y[J0 + j], v);
    }
    if (lane < SB) vz[J0 + i] = v;
    wave_lds_sync();
    return ok;
}

// One 16x16 tile of the trailing update: A[i0.., k0..] -= U_I D_J^-1 U_K^T (v_mfma_f64_16x16x4).
__device__ __forceinline__ void solve_trailing_tile(double* A, int ld, int J0, int i0, int k0, int col, int kq,
                                                    const double (&dk)[4]) {
    double av[4], bv[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) {
        av[s2] = A[(i0 + col) * ld + J0 + 4 * s2 + kq];
        bv[s2] = A[(k0 + col) * ld + J0 + 4 * s2 + kq] * dk[s2];
    }
    d4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], bv[s2], acc, 0, 0, 0);
    const double u[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int r2 = 0; r2 < 4; r2++) A[(i0 + kq + 4 * r2) * ld + k0 + col] -= u[r2];
}

__device__ __forceinline__ void solve_trailing_tile_g(double* A, int ld, int J0, int i0, int k0, int col, int kq,
                                                      const double (&dk)[4]) {
    double av[4], bv[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) {
        av[s2] = A[(long long)(i0 + col) * ld + J0 + 4 * s2 + kq];
        bv[s2] = A[(long long)(k0 + col) * ld + J0 + 4 * s2 + kq] * dk[s2];
    }
    d4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], bv[s2], acc, 0, 0, 0);
    const double u[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int r2 = 0; r2 < 4; r2++) A[(long long)(i0 + kq + 4 * r2) * ld + k0 + col] -= u[r2];
}

// Schedule per block J (one barrier each after the panel and after the trailing step):
//   panel J (all waves) | wavefront 0: trailing tile (J+1, J+1), then the diagonal block J+1
//   (lookahead), while wavefronts 1-3 update every other trailing tile.
// Back substitution runs on wavefront 0 alone: x_J = Linv_JJ^T t_J, then t_c -= sum_i L_ic x_i for
// all earlier columns c (right-looking), block by block from the last.
// NT threads (round 6: 1024 by default, ORBBA_SOLVE_THREADS=256 the round-5 form): wavefront 0 as
// above; the other NT/64 - 1 wavefronts load S, take the panels and the trailing tiles -- with 15 of
// them instead of 3, the lookahead phase of an early block (up to 28 trailing tiles) no longer
// outlasts wavefront 0's diagonal factorisation.  The trailing tiles go to the wavefronts that do
// not share wavefront 0's SIMD first (waves w with w % 4 != 0; a workgroup's waves are dealt to the
// SIMDs in turn), so the diagonal chain keeps its SIMD's issue slots.
// S's entries (r, c), (r, c + 1) (c even: one pose block) from the Schur-block part matrices, summed
// as schur_block_count_in forms them for the global solve: part 0 (+ the pose's Hpp part + lambda I on a
// diagonal block), then parts 1 .. (round 6: S is no longer assembled in HBM by a last-arriving
// workgroup, whose agent-scope release cost ba_schur_block_kernel ~4.5 us per trial).
__device__ __forceinline__ double2 s_piece(const BADev& b, int D, int r, int c, double lam) {
    const int i1 = r / 6, rr = r - 6 * i1, i2 = c / 6, cc = c - 6 * i2;
    const long long pstride = (long long)D * D;
    const double* p = b.Spart + (long long)r * D + c;
    // Branch-free, so every piece's loads are in flight together: the Hpp matrix is zero off the
    // diagonal pose blocks, and adding +0 there changes nothing (at most -0 -> +0 in pk, which v = 0 + pk
    // turns into +0 anyway).
    const bool dg = i1 == i2;
    const double2 h = *reinterpret_cast<const double2*>(p + SB_SPLIT * pstride);
    double2 v = make_double2(0.0, 0.0);
#pragma unroll
    for (int k = 0; k < SB_SPLIT; k++) {
        double2 pk = *reinterpret_cast<const double2*>(p + k * pstride);
        if (k == 0) {
            pk.x = (pk.x + h.x) + (dg && rr == cc ? lam : 0.0);
            pk.y = (pk.y + h.y) + (dg && rr == cc + 1 ? lam : 0.0);
        }
        v.x += pk.x;
        v.y += pk.y;
    }
    return v;
}

template <int NT>
__global__ __launch_bounds__(NT) void ba_solve_kernel(BADev b, int D, int simd0_helpers) {
    BA_RETURN_IF_DONE(b);
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) double A[];   // Dp x ld
    const int Dp = solve_dp(D), ld = Dp + 1;
    double* y = A + (size_t)Dp * ld;   // rhs -> z -> D^-1 z -> x
    double* dinv = y + Dp;
    double* vz = dinv + Dp;
    __shared__ int s_ok;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int col = lane & 15, kq = lane >> 4;
    BA_STAMP(41);
    // the rhs first: its load is in flight with S's
    const double bs_v = tid < D ? b.bs[tid] : 0.0;   // D <= 128 < blockDim
    const double lam = b.ctl->lambda;
    // S -> LDS, only its lower block triangle (row r: columns up to the end of its 16-column block):
    // the factorisation, the panels, the trailing updates and the back substitution read nothing
    // above the diagonal blocks, and the diagonal blocks' upper triangles receive Linv before they are
    // read.  Wavefront 0 stages block 0 (rows 0-15, with the identity padding of a system smaller
    // than one block) and factors it while wavefronts 1-3 load rows 16.. (the load is latency-bound:
    // 38 rows of 16-byte pieces in flight per lane, lane c = piece c of the row).  D = 6 np is even,
    // so every row of S starts 16-byte aligned.
    if (wv == 0) {
        double2 v[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {   // 16 rows x 8 pieces over 64 lanes
            const int p = lane + 64 * k, r = p >> 3, c = 2 * (p & 7);
            // loads from a clamped (in-bounds) position, unconditionally: no branch around them
            const double2 sv = s_piece(b, D, min(r, D - 1), min(c, D - 2), lam);
            v[k] = r < D && c < D ? sv : make_double2(r == c ? 1.0 : 0.0, r == c + 1 ? 1.0 : 0.0);
        }
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int p = lane + 64 * k, r = p >> 3, c = 2 * (p & 7);
            A[r * ld + c] = v[k].x;
            A[r * ld + c + 1] = v[k].y;
        }
        if (lane < Dp) y[lane] = bs_v;
        if (lane == 0) s_ok = 1;
        wave_lds_sync();
        BA_STAMPW(0);
        if (!solve_diag_block(A, y, dinv, vz, ld, 0, lane, D) && lane == 0) s_ok = 0;
    } else {
        constexpr int RQ = (128 - SB + NW - 2) / (NW - 1);   // rows per wavefront: (NW-1) x RQ >= 128 - 16
        const int r0 = SB + wv - 1;
        double2 v[RQ];
#pragma unroll
        for (int q = 0; q < RQ; q++) {
            const int r = min(r0 + (NW - 1) * q, D - 1);
            const int npr = min(D, (r & ~(SB - 1)) + SB) >> 1;   // pieces up to the block's end
            const double2 sv = s_piece(b, D, r, min(2 * lane, D - 2), lam);   // r is clamped above
            v[q] = r0 + (NW - 1) * q < D && lane < npr ? sv : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int q = 0; q < RQ; q++) {
            const int r = r0 + (NW - 1) * q;
            const int npr = min(D, (r & ~(SB - 1)) + SB) >> 1;
            if (r < D && lane < npr) {
                A[r * ld + 2 * lane] = v[q].x;
                A[r * ld + 2 * lane + 1] = v[q].y;
            }
        }
        // identity padding of rows 16.. (no divisions): columns D..Dp-1 of every row, then rows
        // D..Dp-1; a thread per (row group, column) of each
        const int t = tid - 64, npad = Dp - D;
        for (int r = SB + t / 16; r < Dp; r += (NT - 64) / 16)
            if ((t & 15) < npad) A[r * ld + D + (t & 15)] = r == D + (t & 15) ? 1.0 : 0.0;
        for (int r = max(D, SB) + t / 64; r < Dp; r += NW - 1)
            for (int c = lane; c < D; c += 64) A[r * ld + c] = 0.0;
        if (tid < Dp) y[tid] = bs_v;
    }
    __syncthreads();
    for (int J0 = 0; J0 < Dp && s_ok; J0 += SB) {
        const int R0 = J0 + SB;
        const int nbk = (Dp - R0) / SB;
        BA_STAMP(1 + 3 * (J0 / SB));
        if (nbk == 0) break;
        // (2) panel U_I = A_IJ Linv^T per 16-row tile (MFMA); rhs y_i -= A_iJ v with v = Linv^T D^-1 z_J
        if (wv < nbk) {
            double binv[4], bvz[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) {
                const int k = 4 * s2 + kq;
                const double v = A[(J0 + min(k, col)) * ld + J0 + max(k, col)];
                binv[s2] = col > k ? v : (col == k ? 1.0 : 0.0);
            }
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) bvz[s2] = col == 0 ? vz[J0 + 4 * s2 + kq] : 0.0;   // B = [v | 0]
            for (int t = wv; t < nbk; t += NW) {
                const int i0 = R0 + SB * t;
                double av[4];
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) av[s2] = A[(i0 + col) * ld + J0 + 4 * s2 + kq];
                d4 acc = {0, 0, 0, 0}, accy = {0, 0, 0, 0};
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) {
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], binv[s2], acc, 0, 0, 0);
                    accy = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], bvz[s2], accy, 0, 0, 0);
                }
                const double u[4] = {acc.x, acc.y, acc.z, acc.w};
                const double uy[4] = {accy.x, accy.y, accy.z, accy.w};
#pragma unroll
                for (int r2 = 0; r2 < 4; r2++) {
                    const int row = i0 + kq + 4 * r2;
                    A[row * ld + J0 + col] = u[r2];
                    if (col == 0) y[row] -= uy[r2];
                }
            }
        }
        __syncthreads();
        BA_STAMP(2 + 3 * (J0 / SB));
        // (3) trailing update with lookahead
        {
            double dk[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) dk[s2] = dinv[J0 + 4 * s2 + kq];
            if (wv == 0) {
                solve_trailing_tile(A, ld, J0, R0, R0, col, kq, dk);
                wave_lds_sync();
                if (J0 == 32) BA_STAMPW(44);
                if (!solve_diag_block(A, y, dinv, vz, ld, R0, lane, D - R0) && lane == 0) s_ok = 0;
                if (J0 == 32) BA_STAMPW(45);
            } else {
                const int ntile = nbk * (nbk + 1) / 2;
                // helper h: the waves off wavefront 0's SIMD first (w % 4 != 0), then its SIMD-mates
                // (simd0_helpers = 0: wavefront 0's SIMD-mates take no tiles at all when there are enough
                // other helpers, so the diagonal chain has its SIMD to itself)
                constexpr int NOFF = NW - NW / 4;   // helpers off SIMD 0
                const int NH = (simd0_helpers || NOFF == 0) ? NW - 1 : NOFF;
                const int h = (wv & 3) ? (wv >> 2) * 3 + (wv & 3) - 1 : NOFF + (wv >> 2) - 1;
                for (int t = 1 + h; h < NH && t < ntile; t += NH) {   // tile 0 = (J+1, J+1) belongs to wavefront 0
                    int I = 0;
                    while ((I + 1) * (I + 2) / 2 <= t) I++;
                    const int K = t - I * (I + 1) / 2;
                    solve_trailing_tile(A, ld, J0, R0 + SB * I, R0 + SB * K, col, kq, dk);
                }
                if (J0 == 32) BA_STAMPW(45 + wv);
            }
        }
        __syncthreads();
        BA_STAMP(3 + 3 * (J0 / SB));
    }
    const int ok = s_ok;
    // pose state for the update at the end, loaded now so its latency hides behind the back
    // substitution (loaded at the kernel start, it was live across the factorisation: with S staged
    // from the part matrices that spilled it to scratch, each load then waited for in turn)
    double q_pre[4] = {0, 0, 0, 0}, t_pre[3] = {0, 0, 0}, bp_pre[6] = {0, 0, 0, 0, 0, 0};
    if (tid < b.np) {
        const int id = b.ps_id[tid];
        for (int j = 0; j < 4; j++) q_pre[j] = b.q[4 * id + j];
        for (int j = 0; j < 3; j++) t_pre[j] = b.t[3 * id + j];
        for (int j = 0; j < 6; j++) bp_pre[j] = b.bp[6 * tid + j];
    }
    if (ok) {   // back substitution, block by block from the last: x_J on wavefront 0, then every
                // earlier column's update (one thread per column) on the whole workgroup
        for (int i = tid; i < Dp; i += blockDim.x) y[i] *= dinv[i];   // t = D^-1 z
        __syncthreads();
        for (int J0 = Dp - SB; J0 >= 0; J0 -= SB) {
            if (wv == 0) {
                // x_J = Linv_JJ^T t_J: x_c = t_c + sum_{j>c} Linv[j][c] t_j (four partial sums)
                double xp[4] = {y[J0 + col], 0, 0, 0};
#pragma unroll
                for (int j = 1; j < SB; j++) {
                    const double lv = A[(J0 + min(col, j)) * ld + J0 + j];   // Linv[j][col] for j > col
                    xp[j & 3] = fma(j > col ? lv : 0.0, y[J0 + j], xp[j & 3]);   // select, not a branch
                }
                const double xc = (xp[0] + xp[1]) + (xp[2] + xp[3]);
                wave_lds_sync();
                if (lane < SB) y[J0 + col] = xc;
            }
            __syncthreads();
            // t_c -= sum_{i in J} L_ic x_i, L_ic = U_ic dinv_c, for all earlier columns c < J0
            for (int c = tid; c < J0; c += blockDim.x) {
                double sp[4] = {0, 0, 0, 0};
#pragma unroll
                for (int k = 0; k < SB; k++) sp[k & 3] = fma(A[(J0 + k) * ld + c], y[J0 + k], sp[k & 3]);
                y[c] = fma(-((sp[0] + sp[1]) + (sp[2] + sp[3])), dinv[c], y[c]);
            }
            __syncthreads();
        }
    }
    __syncthreads();
    BA_STAMP(40);
    for (int i = tid; i < D; i += blockDim.x) b.x[i] = ok ? y[i] : 0.0;
    if (tid == 0) b.ctl->ok2 = ok;
    __syncthreads();
    // push() + oplus for the free poses, scale terms x.(lambda x + b) (lam: read at the start)
    if (tid < b.np) {   // np <= 21 < blockDim
        const int i = tid;
        const int id = b.ps_id[i];
        double xi[6], part = 0;
        for (int j = 0; j < 6; j++) {
            xi[j] = ok ? y[6 * i + j] : 0.0;
            part += xi[j] * (lam * xi[j] + bp_pre[j]);
        }
        b.part[b.nl + i] = part;
        for (int j = 0; j < 4; j++) b.q_sv[4 * id + j] = q_pre[j];
        for (int j = 0; j < 3; j++) b.t_sv[3 * id + j] = t_pre[j];
        se3_exp_update(xi, q_pre, t_pre);
        for (int j = 0; j < 4; j++) b.q[4 * id + j] = q_pre[j];
        for (int j = 0; j < 3; j++) b.t[3 * id + j] = t_pre[j];
    }
    BA_STAMP(42);
}

// The point lists' entry records (once per call, after the structure): one 16-byte load per entry in
// the per-trial point kernels instead of the pt_slot -> act -> ek -> hp chain of dependent loads.  The
// host-built structure only; the device build writes them in ba_struct_slots_kernel.
__global__ __launch_bounds__(256) void ba_rec_kernel(BADev b) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= b.Ea) return;
    const int k = b.pt_slot[u], e = b.act[k], pi = b.ek[e];
    b.pt_rec[u] = make_int4(k, e, pi, b.hp[pi]);
}

// ---- Device half of the structure build (round 6; host half: ba_structure.h build_structure_counts).
// The (free pose, point) slot table, pose-major (row i: the edge of pose i at each point, -1 where
// none; memset to -1 first), the identity lists of the point-sorted case and their entry records.
__global__ void ba_struct_slots_kernel(const int* __restrict__ ep, const int* __restrict__ ek,
                                       const int* __restrict__ hp, const int* __restrict__ hl, int E, int nl,
                                       int* __restrict__ act, int* __restrict__ pt_slot, int* __restrict__ slot_of,
                                       int4* __restrict__ rec) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    act[e] = e;
    pt_slot[e] = e;
    const int pi = ek[e], h = hp[pi];
    rec[e] = make_int4(e, e, pi, h);
    if (h >= 0) slot_of[(long long)h * nl + hl[ep[e]]] = e;
}
// One workgroup per pose-pair block (i1, i2): the points with an edge to both, ascending, as (edge of
// i1, edge of i2) pairs -- build_structure's order; a diagonal block's first members are also the
// pose's edge list (ps_slot).  Ordered compaction 1024 points at a time (wave ballots + an LDS scan).
__global__ __launch_bounds__(1024) void ba_struct_pairs_kernel(const int* __restrict__ blk_i1,
                                                                const int* __restrict__ blk_i2,
                                                                const int* __restrict__ blk_beg,
                                                                const int* __restrict__ ps_beg,
                                                                const int* __restrict__ slot_of, int nl,
                                                                int2* __restrict__ blk_pair, int* __restrict__ ps_slot) {
    __shared__ int wsum[16];
    const int blk = blockIdx.x, i1 = blk_i1[blk], i2 = blk_i2[blk];
    const int* r1 = slot_of + (long long)i1 * nl;
    const int* r2 = slot_of + (long long)i2 * nl;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int psd = i1 == i2 ? ps_beg[i1] - blk_beg[blk] : 0;   // ps_slot index - pair index
    int base = blk_beg[blk];
    for (int l0 = 0; l0 < nl; l0 += 1024) {
        const int l = l0 + threadIdx.x;
        int a = -1, c = -1;
        if (l < nl) {
            a = r1[l];
            c = r2[l];
        }
        const bool keep = a >= 0 && c >= 0;
        const unsigned long long bm = __ballot(keep);
        if (lane == 0) wsum[wv] = __popcll(bm);
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            const int v = wsum[w];
            off += w < wv ? v : 0;
            tot += v;
        }
        if (keep) {
            const int pos = base + off + __popcll(bm & below);
            blk_pair[pos] = make_int2(a, c);
            if (i1 == i2) ps_slot[pos + psd] = a;
        }
        base += tot;
        __syncthreads();
    }
}

// The same blocked LDL^T for reduced systems too large for LDS (more than 21 free keyframes, D > 128;
// the reference's window is every covisible keyframe, Optimizer.cc:494-504, with no upper bound).
// The padded system lives in HBM / L2 (b.Sg, row stride Dp+1); y, D^-1 and the forward-substitution
// vector stay in LDS.  One 1024-thread workgroup (16 wavefronts), per block J:
//   (1) wavefronts 0 / 1 factor the 16x16 diagonal block and form its inverse in an LDS copy (the
//       same concurrent pair as the LDS kernel), then the block goes back to HBM (L below, Linv in
//       the upper triangle, as the LDS kernel keeps it);
//   (2) the panel U_iJ = A_iJ Linv^T and y_i -= U_iJ D^-1 z_J over all 16 wavefronts (MFMA);
//   (3) the trailing update A_IK -= U_IJ D_J^-1 U_KJ^T, one 16x16 tile per wavefront step (MFMA).
// Back substitution: x_J on wavefront 0, the updates of earlier rows over the whole workgroup.
// ~D^3/3 flops at a few hundred GFLOP/s (one CU): 0.1-1 ms per trial for 22-100 free keyframes.
__global__ __launch_bounds__(1024) void ba_solve_global_kernel(BADev b, int D) {
    BA_RETURN_IF_DONE(b);
    extern __shared__ __attribute__((aligned(16))) double ysh[];   // y | dinv | vz, Dp each
    __shared__ double Ad[SB * (SB + 1)];
    __shared__ int s_ok;
    const int Dp = solve_dp(D), ld = Dp + 1;
    double* A = b.Sg;
    double* y = ysh;
    double* dinv = y + Dp;
    double* vz = dinv + Dp;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, NW = 16;
    const int col = lane & 15, kq = lane >> 4;
    for (long long u = tid; u < (long long)Dp * Dp; u += blockDim.x) {
        const int r = (int)(u / Dp), c = (int)(u % Dp);
        A[(long long)r * ld + c] = (r < D && c < D) ? b.S[(long long)r * D + c] : (r == c ? 1.0 : 0.0);
    }
    for (int i = tid; i < Dp; i += blockDim.x) y[i] = i < D ? b.bs[i] : 0.0;
    if (tid == 0) s_ok = 1;
    __syncthreads();
    for (int J0 = 0; J0 < Dp; J0 += SB) {
        const int R0 = J0 + SB;
        const int nbk = (Dp - R0) / SB;
        // (1) diagonal block in LDS; Av addresses it with the global (J0, J0) indexing of the helpers
        if (tid < SB * SB) Ad[(tid >> 4) * (SB + 1) + (tid & 15)] = A[(long long)(J0 + (tid >> 4)) * ld + J0 + (tid & 15)];
        __syncthreads();
        double* Av = Ad - ((long long)J0 * (SB + 1) + J0);
        if (wv == 0 && !solve_diag_block(Av, y, dinv, vz, SB + 1, J0, lane, D - J0) && lane == 0) s_ok = 0;
        __syncthreads();
        if (!s_ok) break;
        if (tid < SB * SB) A[(long long)(J0 + (tid >> 4)) * ld + J0 + (tid & 15)] = Ad[(tid >> 4) * (SB + 1) + (tid & 15)];
        if (nbk == 0) break;
        // (2) panel
        {
            double binv[4], bvz[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) {
                const int k = 4 * s2 + kq;
                const double v = Ad[min(k, col) * (SB + 1) + max(k, col)];
                binv[s2] = col > k ? v : (col == k ? 1.0 : 0.0);
                bvz[s2] = col == 0 ? vz[J0 + 4 * s2 + kq] : 0.0;
            }
            for (int t = wv; t < nbk; t += NW) {
                const int i0 = R0 + SB * t;
                double av[4];
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) av[s2] = A[(long long)(i0 + col) * ld + J0 + 4 * s2 + kq];
                d4 acc = {0, 0, 0, 0}, accy = {0, 0, 0, 0};
#pragma unroll
                for (int s2 = 0; s2 < 4; s2++) {
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], binv[s2], acc, 0, 0, 0);
                    accy = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s2], bvz[s2], accy, 0, 0, 0);
                }
                const double u[4] = {acc.x, acc.y, acc.z, acc.w};
                const double uy[4] = {accy.x, accy.y, accy.z, accy.w};
#pragma unroll
                for (int r2 = 0; r2 < 4; r2++) {
                    const int row = i0 + kq + 4 * r2;
                    A[(long long)row * ld + J0 + col] = u[r2];
                    if (col == 0) y[row] -= uy[r2];
                }
            }
        }
        __syncthreads();
        // (3) trailing update over the lower block triangle
        {
            double dk[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) dk[s2] = dinv[J0 + 4 * s2 + kq];
            const int ntile = nbk * (nbk + 1) / 2;
            int I = 0, K = wv;   // tile t = I (I + 1) / 2 + K, walked with a stride of NW
            while (K > I) { K -= I + 1; I++; }
            for (int t = wv; t < ntile; t += NW) {
                solve_trailing_tile_g(A, ld, J0, R0 + SB * I, R0 + SB * K, col, kq, dk);
                K += NW;
                while (K > I) { K -= I + 1; I++; }
            }
        }
        __syncthreads();
    }
    __syncthreads();
    const int ok = s_ok;
    if (ok) {
        for (int i = tid; i < Dp; i += blockDim.x) y[i] *= dinv[i];   // t = D^-1 z
        __syncthreads();
        for (int J0 = Dp - SB; J0 >= 0; J0 -= SB) {
            if (wv == 0) {   // x_J = Linv_JJ^T t_J
                double xp[4] = {y[J0 + col], 0, 0, 0};
#pragma unroll
                for (int j = 1; j < SB; j++) {
                    const double lv = A[(long long)(J0 + min(col, j)) * ld + J0 + j];
                    xp[j & 3] = fma(j > col ? lv : 0.0, y[J0 + j], xp[j & 3]);
                }
                const double xc = (xp[0] + xp[1]) + (xp[2] + xp[3]);
                wave_lds_sync();
                if (lane < SB) y[J0 + col] = xc;
            }
            __syncthreads();
            double xj[SB];
#pragma unroll
            for (int k = 0; k < SB; k++) xj[k] = y[J0 + k];
            for (int c = tid; c < J0; c += blockDim.x) {
                double sp[4] = {0, 0, 0, 0};
#pragma unroll
                for (int k = 0; k < SB; k++) sp[k & 3] = fma(A[(long long)(J0 + k) * ld + c], xj[k], sp[k & 3]);
                y[c] = fma(-((sp[0] + sp[1]) + (sp[2] + sp[3])), dinv[c], y[c]);
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < D; i += blockDim.x) b.x[i] = ok ? y[i] : 0.0;
    if (tid == 0) b.ctl->ok2 = ok;
    const double lam = b.ctl->lambda;
    for (int i = tid; i < b.np; i += blockDim.x) {   // push() + oplus, scale terms x.(lambda x + b)
        const int id = b.ps_id[i];
        double q[4], t[3], xi[6], part = 0;
        for (int j = 0; j < 4; j++) q[j] = b.q[4 * id + j];
        for (int j = 0; j < 3; j++) t[j] = b.t[3 * id + j];
        for (int j = 0; j < 6; j++) {
            xi[j] = ok ? y[6 * i + j] : 0.0;
            part += xi[j] * (lam * xi[j] + b.bp[6 * i + j]);
        }
        b.part[b.nl + i] = part;
        for (int j = 0; j < 4; j++) b.q_sv[4 * id + j] = q[j];
        for (int j = 0; j < 3; j++) b.t_sv[3 * id + j] = t[j];
        se3_exp_update(xi, q, t);
        for (int j = 0; j < 4; j++) b.q[4 * id + j] = q[j];
        for (int j = 0; j < 3; j++) b.t[3 * id + j] = t[j];
    }
}

// A point-update workgroup's chi2 / scale partials: its 8 points (group leaders, lanes 0, 8, .., 56)
// summed in order; ba_decide_kernel sums the workgroups' partials in a fixed order.
__device__ __forceinline__ void ba_point_update_partials(double* wgpart, double chi, double part) {
    double pc = 0, pp = 0;
#pragma unroll
    for (int g = 0; g < 64; g += GRP) {
        pc += readlane_d(chi, g);
        pp += readlane_d(part, g);
    }
    if (threadIdx.x == 0) {
        wgpart[2 * blockIdx.x] = pc;
        wgpart[2 * blockIdx.x + 1] = pp;
    }
}

// Back-substitution xl = Dinv (bl - Hpl^T xp), push(), point +=, scale term, then the errors and
// robust chi2 of the point's edges at the new estimate (computeActiveErrors after update()).
// The workgroups' chi2 / scale partials go to wgpart (ba_decide_kernel sums them).
__global__ __launch_bounds__(64) void ba_point_update_kernel(BADev b, int D, double* wgpart) {
    BA_RETURN_IF_DONE(b);
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = t / GRP, sub = t % GRP;
    const bool live = l < b.nl;
    double cl[3] = {0, 0, 0};
    if (live)
        for (int u = b.pt_beg[l] + sub; u < b.pt_beg[l + 1]; u += GRP) {
            const int4 rc = b.pt_rec[u];
            const int k = rc.x, ip = rc.w;
            if (ip < 0) continue;
            const double* Hpl = b.J + (long long)k * 72 + 54;
            for (int c = 0; c < 3; c++) {
                double s = 0;
                for (int r = 0; r < 6; r++) s += Hpl[3 * r + c] * b.x[6 * ip + r];
                cl[c] += s;
            }
        }
    for (int c = 0; c < 3; c++) cl[c] = grp_sum(cl[c]);
    double chi = 0, part = 0;   // every lane of a group ends with the same part
    if (live) {
        const double lam = b.ctl->lambda;
        double bl[3], xl[3];
        for (int c = 0; c < 3; c++) bl[c] = b.bl[3 * l + c];
        const double* Di = b.Dinv + 9 * l;
        for (int c = 0; c < 3; c++) cl[c] = bl[c] - cl[c];
        const int id = b.pt_id[l];
        double Xn[3];
        for (int i = 0; i < 3; i++) {
            xl[i] = Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1] + Di[3 * i + 2] * cl[2];
            Xn[i] = b.X[3 * id + i] + xl[i];
            part += xl[i] * (lam * xl[i] + bl[i]);
        }
        // every lane of the group read X before lane 0 overwrites it below (same wavefront, in order)
        __builtin_amdgcn_wave_barrier();
        if (sub == 0) {
            for (int i = 0; i < 3; i++) {
                b.x[D + 3 * l + i] = xl[i];
                b.X_sv[3 * id + i] = b.X[3 * id + i];
                b.X[3 * id + i] = Xn[i];
            }
            b.part[l] = part;
        }
        for (int u = b.pt_beg[l] + sub; u < b.pt_beg[l + 1]; u += GRP) {
            const int4 rc = b.pt_rec[u];
            const int e = rc.y;
            if (b.level[e]) continue;   // g2o computes active errors only: a level-1 edge keeps its _error
            const int pi = rc.z;
            double Xc[3];
            se3_map(b.q + 4 * pi, b.t + 3 * pi, Xn, Xc);
            chi += edge_error(b, e, Xc);
        }
    }
    // group partial (lanes of a group are contiguous; sum in fixed order via shuffles)
    chi += __shfl_xor(chi, 1, 64);
    chi += __shfl_xor(chi, 2, 64);
    chi += __shfl_xor(chi, 4, 64);
    if (live && sub == 0) b.rchi[l] = chi;
    ba_point_update_partials(wgpart, chi, part);
}

__device__ bool ba_decide_step(const BADev& b, BACtl* host_snap, int seq, double tmp_sum, double scale_sum);

// The decide step after a trial: fixed-order sums of the point-update workgroups' partials (thread-
// strided, then a fixed tree) + the pose scale terms of the solve, ba_decide_step on one thread, and
// pop() (restore the pushed estimates) on a rejected step.
__global__ __launch_bounds__(256) void ba_decide_kernel(BADev b, BACtl* host_snap, int seq, const double* wgpart,
                                                        int G) {
    BA_RETURN_IF_DONE(b);
    __shared__ double sc[256], sp[256];
    __shared__ int s_acc;
    const int tid = threadIdx.x;
    double c0 = 0, p0 = 0;
    for (int w = tid; w < G; w += 256) {
        c0 += wgpart[2 * w];
        p0 += wgpart[2 * w + 1];
    }
    for (int i = tid; i < b.np; i += 256) p0 += b.part[b.nl + i];
    sc[tid] = c0;
    sp[tid] = p0;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) {
            sc[tid] += sc[tid + o];
            sp[tid] += sp[tid + o];
        }
        __syncthreads();
    }
    if (tid == 0) s_acc = ba_decide_step(b, host_snap, seq, sc[0], sp[0]);
    __syncthreads();
    if (s_acc) return;
    for (int t = tid; t < b.nl + b.np; t += 256) {   // pop(): restore the pushed estimates
        if (t < b.nl) {
            const int id = b.pt_id[t];
            for (int i = 0; i < 3; i++) b.X[3 * id + i] = b.X_sv[3 * id + i];
        } else {
            const int id = b.ps_id[t - b.nl];
            for (int j = 0; j < 4; j++) b.q[4 * id + j] = b.q_sv[4 * id + j];
            for (int j = 0; j < 3; j++) b.t[3 * id + j] = b.t_sv[3 * id + j];
        }
    }
}

__device__ __forceinline__ void snapshot_to_host(const BACtl& snap, int seq, BACtl* host_snap);

// levenberg.cpp:120-147 — accept / reject, lambda / nu update, then the trial / iteration bookkeeping
// of g2o's solve() / optimize(); one thread.  Returns whether the step was accepted.
__device__ bool ba_decide_step(const BADev& b, BACtl* host_snap, int seq, double tmp_sum, double scale_sum) {
    BACtl* c = b.ctl;
    c->tmp = tmp_sum;
    c->scale = scale_sum;
    double tmp = tmp_sum;
    if (!c->ok2) tmp = 1.7976931348623157e308;   // std::numeric_limits<double>::max()
    double rho = c->cur - tmp;
    rho /= (scale_sum + 1e-3);
    c->rho = rho;
    if (rho > 0 && isfinite(tmp)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        c->lambda *= fmax(1. / 3., alpha);
        c->ni = 2;
        c->cur = tmp;
        c->accepted = 1;
    } else {
        c->lambda *= c->ni;
        c->ni *= 2;
        c->accepted = 0;
    }
    // trial / iteration bookkeeping (host loop of levenberg solve + SparseOptimizer::optimize)
    c->q += 1;
    c->trials += 1;
    // g2o polls terminate() after every trial (levenberg.cpp:149) and before every iteration
    // (sparse_optimizer.cpp:376): a raised flag ends the loop once this trial is done
    const bool stop = (b.stop && __atomic_load_n(b.stop, __ATOMIC_RELAXED) != 0) ||
                      (b.stop_after >= 0 && c->trials >= b.stop_after);
    if (rho < 0 && c->q < 10 && !stop) {
        c->need_lin = 0;   // retry with the new lambda
    } else {
        c->iters_done += 1;
        c->chi_out = c->cur;
        bool term = c->q == 10 || rho == 0;
        if (!term) {
            if ((c->ini - c->cur) * 1e3 < c->ini) c->nbad++;
            else c->nbad = 0;
            term = c->nbad >= 3;
        }
        c->it += 1;
        if (c->it >= c->iters_max) term = true;
        if (stop) {
            term = true;
            c->stopped = 1;
        }
        if (term) c->done = 1;
        else {
            c->need_lin = 1;
            c->q = 0;
        }
    }
    // control snapshot straight into pinned host memory (no copy on the stream, no event).  (A
    // forwarder kernel on a side stream, so the decide kernel would not wait for the PCIe writes,
    // was slower: 1.73 -> 1.92 ms per C4 call.)
    BACtl snap = *c;
    snap.seq = -1;
    snapshot_to_host(snap, seq, host_snap);
    return c->accepted != 0;
}

// The control snapshot into pinned host memory: the body as relaxed system-scope stores (write-through
// to the host), then the sequence id the host polls for as a system-scope RELEASE store, so the host's
// acquire load of `seq` (the host ring poll in orbba_local_ba) orders every body word before it by the
// memory model, not by the gfx9 rule that vmcnt(0) retires earlier stores (What's weak 8).
// Cost: on gfx950 the release compiles to `buffer_wbl2 sc0 sc1; s_waitcnt vmcnt(0)` before the seq store,
// i.e. a write-back of the whole L2 on every snapshot (once per LM trial, from one thread).  Measured
// against the relaxed form (ORBBA_SNAP_RELEASE=0, tools/ab_build.sh), alternating on one box, 40 calls
// each: 9.27-9.33k vs 8.98-9.31k LM iterations/s -- no cost above the noise, since the L2 holds little
// dirty data between the solve kernels.  ORBBA_SNAP_RELEASE=0 builds the round-3 form for A/B only.
#ifndef ORBBA_SNAP_RELEASE
#define ORBBA_SNAP_RELEASE 1
#endif
__device__ __forceinline__ void snapshot_to_host(const BACtl& snap, int seq, BACtl* host_snap) {
    static_assert(sizeof(BACtl) % 8 == 0, "snapshot copied as 8-byte words");
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&snap);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(host_snap);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(BACtl) / 8); k++)
        __hip_atomic_store(dst + k, src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#if ORBBA_SNAP_RELEASE
    __hip_atomic_store(&host_snap->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&host_snap->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
}


// final outlier classification (Optimizer.cc:644-670, :686-699) + chi2 out
// check_active (the second optimize()): with no level-0 edge left, g2o's optimize() has nothing to do
// (initializeOptimization(0) finds no active edge); the loop ends here and the snapshot the host waits
// for as step 0's (`seq` in ring slot `host_snap`) is written by this kernel, so the host never needs the
// classification on its side.
// only_if_done: enqueued speculatively behind the first loop (after its guarded classification); it
// starts the second loop only if the first has ended by then.
__global__ void ba_ctl_start_kernel(BADev b, int iters, int check_active, BACtl* host_snap, int seq, int only_if_done) {
    BACtl* c = b.ctl;
    if (only_if_done && !c->done) return;
    c->it = 0;
    c->q = 0;
    c->nbad = 0;
    const bool idle = check_active && c->n_active == 0;
    c->done = (iters <= 0 || idle) ? 1 : 0;
    c->maxdiag_bits = 0;
    c->need_lin = 1;
    c->iters_max = iters;
    c->iters_done = 0;
    c->chi_out = 0;
    c->rho = 0;
    if (idle) {
        BACtl snap = *c;
        snap.seq = -1;
        snapshot_to_host(snap, seq, host_snap);
    }
}

__global__ void ba_ctl_stop_kernel(BADev b) { b.ctl->done = 1; }

// With rq / rt / rX (the final call) it also gathers the poses and points into the result region,
// so the results come back in one copy.
// only_if_done: the final gather enqueued speculatively behind the LM step the host expects to be the
// last; it does nothing unless the loop has ended by then (the host then enqueues another).
__global__ void ba_classify_kernel(BADev b, uint8_t* outlier, double* chi2o, uint8_t* level, int set_level,
                                   double* rq, double* rt, double* rX, int only_if_done) {
    if (only_if_done && !b.ctl->done) return;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (rq && e < b.P) {
        for (int j = 0; j < 4; j++) rq[4 * e + j] = b.q[4 * e + j];
        for (int j = 0; j < 3; j++) rt[3 * e + j] = b.t[3 * e + j];
    }
    if (rX && e < b.N)
        for (int j = 0; j < 3; j++) rX[3 * e + j] = b.X[3 * e + j];
    uint8_t bad = 1;
    if (e < b.E) {
        const double maxc = b.stereo[e] ? 7.815 : 5.991;
        const double c = edge_chi2(b, e);
        double Xc[3];
        const int pi = b.ek[e];
        se3_map(b.q + 4 * pi, b.t + 3 * pi, b.X + 3 * b.ep[e], Xc);
        bad = (c > maxc || !(Xc[2] > 0.0)) ? 1 : 0;
        if (outlier) outlier[e] = bad;
        if (chi2o) chi2o[e] = c;
        if (set_level) {
            if (bad) level[e] = 1;
            b.robust[e] = 0;
        }
    }
    if (set_level) {   // the edges left at level 0 (the set_level launch covers E only: no early return above)
        const int n = __syncthreads_count(!bad);
        if (threadIdx.x == 0 && n) atomicAdd(&b.ctl->n_active, n);
    }
}

}  // namespace orbamd

using namespace orbamd;

namespace {

// Grow-only pinned host buffer.  Only grown when no copy from it is in flight.
struct PinnedBuf {
    char* ptr = nullptr;
    char* dptr = nullptr;   // the device's view (mapped buffers)
    size_t cap = 0;
    int ensure(size_t bytes, bool mapped = false) {
        if (bytes <= cap) return ORB_OK;
        if (ptr) (void)hipHostFree(ptr);
        ptr = dptr = nullptr;
        cap = 0;
        const size_t c = align_up(bytes + bytes / 4, 1 << 16);
        ORB_HIP_TRY(hipHostMalloc((void**)&ptr, c, mapped ? hipHostMallocMapped : hipHostMallocDefault));
        if (mapped) ORB_HIP_TRY(hipHostGetDevicePointer((void**)&dptr, ptr, 0));
        cap = c;
        return ORB_OK;
    }
    ~PinnedBuf() {
        if (ptr) (void)hipHostFree(ptr);
    }
};

// A helper thread per calling thread (round 6): it runs the host half of the structure build (the
// counts, ~50 us at C4) while the calling thread stages and enqueues the problem upload, instead of
// after it.  Started on first use; a process that forked after that (the thread does not exist in the
// child) runs the job on the calling thread.
class HostHelper {
public:
    void post(std::function<void()> f) {
        if (!start()) {   // no helper in this process: run it here
            f();
            done_.store(true, std::memory_order_release);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = std::move(f);
            has_ = true;
            done_.store(false, std::memory_order_relaxed);
        }
        cv_.notify_one();
    }
    void wait() const {   // the job is short: spin (yielding) rather than sleep
        while (!done_.load(std::memory_order_acquire)) std::this_thread::yield();
    }
    ~HostHelper() {
        if (th_.joinable()) {
            if (pid_ != getpid()) {   // forked child: the thread object has no thread behind it
                th_.detach();
                return;
            }
            {
                std::lock_guard<std::mutex> lk(m_);
                quit_ = true;
            }
            cv_.notify_one();
            th_.join();
        }
    }

private:
    bool start() {
        if (th_.joinable()) return pid_ == getpid();
        pid_ = getpid();
        th_ = std::thread([this] { run(); });
        return true;
    }
    void run() {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_.wait(lk, [&] { return has_ || quit_; });
            if (quit_) return;
            std::function<void()> f = std::move(job_);
            has_ = false;
            lk.unlock();
            f();
            done_.store(true, std::memory_order_release);
            lk.lock();
        }
    }
    std::thread th_;
    pid_t pid_ = 0;
    std::mutex m_;
    std::condition_variable cv_;
    std::function<void()> job_;
    bool has_ = false, quit_ = false;
    std::atomic<bool> done_{true};
};

// Device-resident LocalBA workspace (one per thread: LocalMapping runs one LocalBA at a time).
struct BAContext {
    HostHelper helper;   // destroyed last (declared first): no job is in flight after a call returns
    int device = -1;
    hipStream_t st = nullptr;
    DevBuf prob, state, structure, sys, ctlbuf;
    BACtl* h_ctl = nullptr;   // pinned
    BACtl* h_ring = nullptr;  // pinned, device-mapped control snapshots, one per step in flight
    BACtl* d_ring = nullptr;
    int step_seq = 0;         // id of the last enqueued LM step (snapshot sequence)
    int32_t* h_stop = nullptr;   // pinned, device-mapped mirror of the caller's stop flag
    int32_t* d_stop = nullptr;
    PinnedBuf h_prob, h_struct, h_res;   // pinned staging images (one copy each way)
    // Everything device-bound belongs to `device`: a call on another device from the same thread
    // releases it all (buffers, stream, events) before building the new device's set.
    void reset_device() {
        if (device >= 0) (void)hipSetDevice(device);
        if (st) (void)hipStreamSynchronize(st);
        prob.release(); state.release(); structure.release(); sys.release(); ctlbuf.release();
        if (st) { (void)hipStreamDestroy(st); st = nullptr; }
        if (h_ring) { (void)hipHostFree(h_ring); h_ring = nullptr; d_ring = nullptr; }
        if (h_stop) { (void)hipHostFree(h_stop); h_stop = nullptr; d_stop = nullptr; }
        if (h_ctl) { (void)hipHostFree(h_ctl); h_ctl = nullptr; }
        device = -1;
    }
    ~BAContext() {
        if (h_stop) (void)hipHostFree(h_stop);
        if (h_ring) (void)hipHostFree(h_ring);
        prob.release(); state.release(); structure.release(); sys.release(); ctlbuf.release();
        if (h_ctl) (void)hipHostFree(h_ctl);
        if (st) (void)hipStreamDestroy(st);
    }
};
thread_local BAContext g_ba;

// The call's buffer initialisations as ONE launch per batch instead of a hipMemsetAsync each (round 6:
// 11 memsets per call ran as 16 fill kernels of ~4.4 us, ~70 us of the call's GPU time in rocprofv3).
// Segments start 16-byte aligned (carve offsets are multiples of 256); a byte value replicated.
constexpr int BA_FILL_MAX = 8;
struct BAFill {
    void* p[BA_FILL_MAX];
    unsigned long long n[BA_FILL_MAX];
    unsigned v[BA_FILL_MAX];
    int cnt;
    BACtl* ctl;       // when set: the first optimize()'s control block, written whole (ba_ctl_start_kernel's
    BACtl ctl_init;   // job for that call, one launch earlier)
};
__global__ __launch_bounds__(256) void ba_fill_kernel(BAFill f) {
    const unsigned long long gt = blockIdx.x * 256ull + threadIdx.x, gs = gridDim.x * 256ull;
    if (f.ctl && gt < sizeof(BACtl) / 8)
        reinterpret_cast<unsigned long long*>(f.ctl)[gt] = reinterpret_cast<const unsigned long long*>(&f.ctl_init)[gt];
    for (int s = 0; s < f.cnt; s++) {
        uint8_t* p = static_cast<uint8_t*>(f.p[s]);
        const unsigned b = f.v[s] & 0xffu, w = b * 0x01010101u;
        const uint4 v4 = make_uint4(w, w, w, w);
        const unsigned long long nv = f.n[s] >> 4;
        for (unsigned long long i = gt; i < nv; i += gs) reinterpret_cast<uint4*>(p)[i] = v4;
        for (unsigned long long i = (nv << 4) + gt; i < f.n[s]; i += gs) p[i] = (uint8_t)b;
    }
}
struct FillQueue {
    BAFill f{};
    unsigned long long bytes = 0;
    int add(void* p, size_t n, int v, hipStream_t st) {
        if (!n) return ORB_OK;
        if (f.cnt == BA_FILL_MAX) {
            if (int rc = flush(st)) return rc;
        }
        f.p[f.cnt] = p;
        f.n[f.cnt] = n;
        f.v[f.cnt] = (unsigned)v;
        f.cnt++;
        bytes += n;
        return ORB_OK;
    }
    void set_ctl(BACtl* c, const BACtl& init) {
        f.ctl = c;
        f.ctl_init = init;
    }
    int flush(hipStream_t st) {
        if (!f.cnt && !f.ctl) return ORB_OK;
        const unsigned nb = (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>(1024, bytes / (16 * 256 * 2)));
        hipLaunchKernelGGL(ba_fill_kernel, dim3(nb), dim3(256), 0, st, f);
        f.cnt = 0;
        f.ctl = nullptr;
        bytes = 0;
        ORB_HIP_TRY(hipGetLastError());
        return ORB_OK;
    }
};

struct Carve {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(size_t n) {
        T* p = reinterpret_cast<T*>(base + off);
        off += align_up(std::max<size_t>(n, 1) * sizeof(T), 256);
        return p;
    }
};
template <class T>
size_t carve_size(size_t n) { return align_up(std::max<size_t>(n, 1) * sizeof(T), 256); }

using orbamd_host::HostStructure;
using orbamd_host::build_structure;

}  // namespace

extern "C" int orbba_local_ba(const orbba_problem* pr, orbba_result* res, const volatile int32_t* stop_flag,
                              int device) {
    ORB_CHECK_ARG(pr && res, "null argument");
    const int P = pr->n_poses, N = pr->n_points, E = pr->n_edges;
    ORB_CHECK_ARG(P >= 0 && N >= 0 && E >= 0, "negative sizes");
    ORB_CHECK_ARG(res->pose_R && res->pose_t && res->points && res->edge_outlier, "null result buffers");
    // host-side phase timing (ORBBA_DEBUG_TIMING=1: printed to stderr at the end of the call)
    static const bool tdbg = getenv("ORBBA_DEBUG_TIMING") != nullptr;
    std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> marks;
    auto mark = [&](const char* n) {
        if (tdbg) marks.emplace_back(n, std::chrono::steady_clock::now());
    };
    mark("entry");
    for (int e = 0; e < E; e++)
        ORB_CHECK_ARG(pr->edge_point[e] >= 0 && pr->edge_point[e] < N && pr->edge_pose[e] >= 0 &&
                          pr->edge_pose[e] < P, "edge references a missing vertex");
    mark("edge checks");
    BAContext& C = g_ba;
    if (C.device != device) {
        int ndev = 0;
        ORB_HIP_TRY(hipGetDeviceCount(&ndev));
        ORB_CHECK_ARG(device >= 0 && device < ndev, "no such HIP device");
        C.reset_device();
        ORB_HIP_TRY(hipSetDevice(device));
        ORB_HIP_TRY(hipStreamCreateWithFlags(&C.st, hipStreamNonBlocking));
        ORB_HIP_TRY(hipHostMalloc((void**)&C.h_ctl, sizeof(BACtl), hipHostMallocDefault));
        ORB_HIP_TRY(hipHostMalloc((void**)&C.h_ring, 2 * sizeof(BACtl), hipHostMallocMapped));
        ORB_HIP_TRY(hipHostGetDevicePointer((void**)&C.d_ring, C.h_ring, 0));
        ORB_HIP_TRY(hipHostMalloc((void**)&C.h_stop, 64, hipHostMallocMapped));
        ORB_HIP_TRY(hipHostGetDevicePointer((void**)&C.d_stop, C.h_stop, 0));
        for (int k = 0; k < 2; k++) C.h_ring[k].seq = -1;
        C.device = device;
    }
    ORB_HIP_TRY(hipSetDevice(device));
    hipStream_t st = C.st;
    auto stopped = [&]() { return stop_flag && *stop_flag; };
    int stop_after = -1;   // test hook (ORBBA_DEBUG_STOP_AFTER_TRIALS): tests/test_ba_gpu.py
    if (const char* e = getenv("ORBBA_DEBUG_STOP_AFTER_TRIALS")) stop_after = atoi(e);
    *C.h_stop = stopped() ? 1 : 0;

    mark("context");
    // The host half of the structure build: on the helper thread, in parallel with the staging below
    // (default path).  ORBBA_STRUCT: "host" = the whole build on the host (generic), "sorted" = the
    // host's point-sorted variant; default: counts on the host, lists on the device when the edges are
    // point-sorted (read per call: tests compare the forms in one process).
    thread_local HostStructure hs;   // capacity kept across calls
    const char* smode_env = getenv("ORBBA_STRUCT");
    const std::string smode = smode_env ? smode_env : "";
    const bool try_counts = smode != "host" && smode != "sorted" && smode != "generic";
    bool counts_ok = false;
    struct HelperWait {   // every return path waits for a posted job (it writes hs and counts_ok)
        HostHelper& h;
        bool on;
        ~HelperWait() {
            if (on) h.wait();
        }
    } helper_wait{C.helper, false};
    if (try_counts && E >= 1024) {
        HostStructure* hsp = &hs;   // (the helper's own thread_local hs is another object)
        C.helper.post([hsp, &counts_ok, P, N, E, pr] {
            try {   // (an exception must not leave the helper thread: the calling thread's build takes over)
                counts_ok = build_structure_counts(P, N, pr->pose_fixed, pr->edge_point, pr->edge_pose, E, *hsp);
            } catch (...) {
                counts_ok = false;
            }
        });
        helper_wait.on = true;
    }
    // initial estimates: SE3Quat(R, t) -> Quaterniond(R) normalised (Optimizer.cc:145-150)
    std::vector<double> q0(4 * (size_t)P);
    for (int i = 0; i < P; i++) {
        const double* m = pr->pose_R + 9 * i;
        double x, y, z, w;
        const double tr = m[0] + m[4] + m[8];
        if (tr > 0) {
            double s = std::sqrt(tr + 1.0);
            w = 0.5 * s; s = 0.5 / s;
            x = (m[7] - m[5]) * s; y = (m[2] - m[6]) * s; z = (m[3] - m[1]) * s;
        } else {
            int a = 0;
            if (m[4] > m[0]) a = 1;
            if (m[8] > m[3 * a + a]) a = 2;
            const int bb = (a + 1) % 3, c = (bb + 1) % 3;
            double s = std::sqrt(m[3 * a + a] - m[3 * bb + bb] - m[3 * c + c] + 1.0);
            double qv[3];
            qv[a] = 0.5 * s; s = 0.5 / s;
            w = (m[3 * c + bb] - m[3 * bb + c]) * s;
            qv[bb] = (m[3 * bb + a] + m[3 * a + bb]) * s;
            qv[c] = (m[3 * c + a] + m[3 * a + c]) * s;
            x = qv[0]; y = qv[1]; z = qv[2];
        }
        if (w < 0) { x = -x; y = -y; z = -z; w = -w; }
        const double n = std::sqrt(x * x + y * y + z * z + w * w);
        if (n > 0) { x /= n; y /= n; z /= n; w /= n; }
        q0[4 * i] = x; q0[4 * i + 1] = y; q0[4 * i + 2] = z; q0[4 * i + 3] = w;
    }

    // ---- device problem + state.  Everything the host provides is laid out in one region, built
    // in pinned staging with the same offsets and uploaded with a single copy.
    // One camera for the whole window (every keyframe of a map shares the calibration: the usual case)
    // goes up once instead of 40 B per edge: half the staging copy and the upload (round 6)
    bool one_cam = E > 0;
    for (int e = 1; e < E && one_cam; e++) one_cam = std::memcmp(pr->edge_cam + 5 * (size_t)e, pr->edge_cam, 40) == 0;
    const size_t ncam = one_cam ? 5 : 5 * (size_t)E;
    const size_t up_bytes = carve_size<uint8_t>(P) + carve_size<int>(E) * 2 + carve_size<uint8_t>(E) +
                            carve_size<double>(3 * (size_t)E) + carve_size<double>(E) +
                            carve_size<double>(ncam) + carve_size<double>(4 * (size_t)P) +
                            carve_size<double>(3 * (size_t)P) + carve_size<double>(3 * (size_t)N);
    const size_t state_bytes = carve_size<double>(4 * (size_t)P) + carve_size<double>(3 * (size_t)P) +
                               carve_size<double>(3 * (size_t)N) + carve_size<uint8_t>(E) * 2 +
                               carve_size<double>(3 * (size_t)E);
    const size_t res_bytes = carve_size<double>(4 * (size_t)P) + carve_size<double>(3 * (size_t)P) +
                             carve_size<double>(3 * (size_t)N) + carve_size<uint8_t>(E) + carve_size<double>(E);
    int rc;
    if ((rc = C.prob.reserve(up_bytes))) return rc;
    if ((rc = C.state.reserve(state_bytes))) return rc;
    if ((rc = C.ctlbuf.reserve(sizeof(BACtl) + 64))) return rc;
    if ((rc = C.h_prob.ensure(up_bytes))) return rc;
    if ((rc = C.h_res.ensure(res_bytes, true))) return rc;   // mapped: the final gather writes it directly
    Carve cp{C.prob.as<char>()}, hp{C.h_prob.ptr}, cs{C.state.as<char>()};
    BADev b;
    std::memset(&b, 0, sizeof(b));
    b.P = P; b.N = N; b.E = E;
    uint8_t* d_fixed = cp.take<uint8_t>(P);
    int* d_ep = cp.take<int>(E);
    int* d_ek = cp.take<int>(E);
    uint8_t* d_st = cp.take<uint8_t>(E);
    double* d_obs = cp.take<double>(3 * (size_t)E);
    double* d_info = cp.take<double>(E);
    double* d_cam = cp.take<double>(ncam);
    b.q = cp.take<double>(4 * (size_t)P);
    b.t = cp.take<double>(3 * (size_t)P);
    b.X = cp.take<double>(3 * (size_t)N);
    {
        std::memcpy(hp.take<uint8_t>(P), pr->pose_fixed, P);
        std::memcpy(hp.take<int>(E), pr->edge_point, 4 * (size_t)E);
        std::memcpy(hp.take<int>(E), pr->edge_pose, 4 * (size_t)E);
        uint8_t* hst = hp.take<uint8_t>(E);
        for (int e = 0; e < E; e++) hst[e] = pr->edge_obs[3 * e + 2] < 0 ? 0 : 1;   // ur < 0 => mono (:595)
        std::memcpy(hp.take<double>(3 * (size_t)E), pr->edge_obs, 24 * (size_t)E);
        std::memcpy(hp.take<double>(E), pr->edge_inv_sigma2, 8 * (size_t)E);
        std::memcpy(hp.take<double>(ncam), pr->edge_cam, 8 * ncam);
        std::memcpy(hp.take<double>(4 * (size_t)P), q0.data(), 32 * (size_t)P);
        std::memcpy(hp.take<double>(3 * (size_t)P), pr->pose_t, 24 * (size_t)P);
        std::memcpy(hp.take<double>(3 * (size_t)N), pr->points, 24 * (size_t)N);
    }
    b.q_sv = cs.take<double>(4 * (size_t)P);
    b.t_sv = cs.take<double>(3 * (size_t)P);
    b.X_sv = cs.take<double>(3 * (size_t)N);
    b.robust = cs.take<uint8_t>(E);
    uint8_t* d_level = cs.take<uint8_t>(E);
    b.err = cs.take<double>(3 * (size_t)E);
    b.fixed = d_fixed; b.ep = d_ep; b.ek = d_ek; b.stereo = d_st; b.obs = d_obs; b.info = d_info; b.cam = d_cam;
    b.cam_step = one_cam ? 0 : 5;
    b.level = d_level;
    b.ctl = C.ctlbuf.as<BACtl>();
    b.stop = stop_flag ? C.d_stop : nullptr;
    b.stop_after = stop_after;
    FillQueue fills;   // flushed (one launch) before the first kernel that reads them
    // (the control block is written whole by the first optimize()'s fill: trials / stopped count from 0
    // over the whole call)
    ORB_HIP_TRY(hipMemcpyAsync(C.prob.ptr, C.h_prob.ptr, cp.off, hipMemcpyHostToDevice, st));
    if ((rc = fills.add(b.robust, E, 1, st)) || (rc = fills.add(d_level, E, 0, st)) ||
        (rc = fills.add(b.err, 24 * (size_t)E, 0, st)))
        return rc;
    res->iterations[0] = res->iterations[1] = 0;
    res->chi2[0] = res->chi2[1] = 0;

    mark("staging + upload enqueued");
    std::vector<uint8_t> level(E, 0);
    bool hook_stopped = false;   // the device ended a loop on the stop flag (or the test hook)
    // the final classification + poses / points, gathered straight into the mapped pinned result region
    // (round 6: no device-to-host copy behind the kernel); `gather` enqueues it
    Carve dres{C.h_res.dptr};
    double* rq = dres.take<double>(4 * (size_t)P);
    double* rt = dres.take<double>(3 * (size_t)P);
    double* rX = dres.take<double>(3 * (size_t)N);
    uint8_t* ro = dres.take<uint8_t>(E);
    double* rch = dres.take<double>(E);
    const int n_gather = std::max(E, std::max(N, P));
    auto gather = [&](int only_if_done) {
        hipLaunchKernelGGL(ba_classify_kernel, dim3((n_gather + 255) / 256), dim3(256), 0, st, b, ro,
                           res->edge_chi2 ? rch : (double*)nullptr, (uint8_t*)nullptr, 0, rq, rt, rX, only_if_done);
    };
    bool gathered = false;   // a speculative gather ran behind the step that ended the last loop
    // the outlier classification between the loops (Optimizer.cc:644-670): levels + robust kernels off
    auto classify_levels = [&](int only_if_done) {
        hipLaunchKernelGGL(ba_classify_kernel, dim3((E + 255) / 256), dim3(256), 0, st, b, (uint8_t*)nullptr,
                           (double*)nullptr, d_level, 1, (double*)nullptr, (double*)nullptr, (double*)nullptr,
                           only_if_done);
    };
    bool leveled = false;   // likewise for the classification after the first loop
    bool started_ahead = false;   // ... and the second loop's ctl_start
    int spec_launched[2] = {0, 0};   // speculative loop ends enqueued per loop (ORBBA_DEBUG_TIMING report)
    // test hook (ORBBA_DEBUG_SPEC_EARLY=1, tests/test_ba_gpu.py): enqueue the loop ends one step too
    // early, so that each loop's first guesses miss and the fallback paths run
    const int spec_slack = [] {
        const char* e = getenv("ORBBA_DEBUG_SPEC_EARLY");
        return e && atoi(e) != 0 ? 1 : 0;
    }();
    constexpr int next_iters = 10;   // the second optimize()'s iterations (Optimizer.cc:672)
    // ------------------------------------------------------------------ one optimize(iters)
    // The structure is built once, for the first optimize() (every edge at level 0).  The second
    // optimize() (initializeOptimization(0) after the outliers went to level 1) reuses it: its active
    // edges are a subset, the kernels skip level-1 edges (their J / W stay 0, so every sum, Schur block
    // and dense factorisation sees exact zeros in their place), and a vertex left without active edges
    // keeps a zero Hessian block (+ lambda), i.e. a zero update, as if it were not in the problem.
    bool have_structure = false;
    bool have_classified = false;   // the outlier classification ran (second optimize())
    auto optimize = [&](int iters, int32_t* iters_out, double* chi_out, bool last_loop) -> int {
        bool dev_build = false;   // act / pt_slot / ps_slot / blk_pair filled on the device
        const bool fresh = !have_structure;   // the first optimize() of the call
        if (!have_structure) {
            if (helper_wait.on) {   // the counts posted at entry
                C.helper.wait();
                helper_wait.on = false;
                dev_build = counts_ok;
            } else {
                dev_build = try_counts && build_structure_counts(P, N, pr->pose_fixed, pr->edge_point, pr->edge_pose, E, hs);
            }
            if (!dev_build)
                build_structure(P, N, level, pr->pose_fixed, pr->edge_point, pr->edge_pose, hs, smode == "sorted");
            mark(dev_build ? "build_structure (counts)" : "build_structure");
        }
        const int Ea = hs.n_act, np = hs.np, nl = hs.nl, D = 6 * np;
        const int nblk = (int)hs.blk_i1.size();
        *iters_out = 0;
        *chi_out = 0;
        // (the second optimize()'s level-0 edge count is on the device: ba_ctl_start_kernel ends the
        // loop at once when the classification left none)
        if (Ea == 0 || np + nl == 0) return ORB_OK;
        // reduced system: in LDS up to 21 free keyframes (D <= 128), else in HBM (ba_solve_global_kernel)
        const bool glob = D > 128 || solve_lds_doubles(D) * 8 + 4096 > 160 * 1024;
        // the LDS solve's workgroup: 1024 threads, or the round-5 256 (ORBBA_SOLVE_THREADS=256; read per call)
        const bool solve256 = [] {
            const char* e = getenv("ORBBA_SOLVE_THREADS");
            return e && atoi(e) == 256;
        }();
        const int simd0_helpers = [] {   // ORBBA_SOLVE_SIMD0=1: wavefront 0's SIMD-mates take trailing tiles too
            const char* e = getenv("ORBBA_SOLVE_SIMD0");
            return e && atoi(e) != 0 ? 1 : 0;
        }();
        const void* solve_fn = glob ? (const void*)ba_solve_global_kernel
                               : solve256 ? (const void*)ba_solve_kernel<256> : (const void*)ba_solve_kernel<1024>;

        if (glob && np > ORBBA_MAX_FREE_KEYFRAMES) {
            set_error("LocalBA: more than ORBBA_MAX_FREE_KEYFRAMES free keyframes in the local window");
            return ORB_EINVAL;
        }
        const int Dp = solve_dp(D);
        // structure upload
        const size_t nps = (size_t)hs.n_ps, npairs = (size_t)hs.n_pairs;
        const size_t sbytes = carve_size<int>(P) + carve_size<int>(N) + carve_size<int>(nl + 1) + carve_size<int>(nl) +
                              carve_size<int>(np + 1) + carve_size<int>(np) + carve_size<int>(nblk) * 2 +
                              carve_size<int>(nblk + 1) + carve_size<int>(np) + carve_size<int>(Ea) * 2 +
                              carve_size<int>(nps) + carve_size<int2>(npairs) + carve_size<int4>(Ea) +
                              (dev_build ? carve_size<int>((size_t)np * nl) : 0);
        int rc2;
        // system buffers (carved before the structure upload, so that their clears and the control
        // block ride on the structure's fill launch)
        const size_t spart_n = (size_t)(SB_SPLIT + 1) * (glob ? 36 * (size_t)nblk : (size_t)D * D);   // + Hpp part
        const size_t ybytes = carve_size<double>(72 * (size_t)Ea) + carve_size<double>(24 * (size_t)Ea) +
                              carve_size<double>(9 * (size_t)nl) * 2 + carve_size<double>(3 * (size_t)nl) +
                              carve_size<double>(36 * (size_t)np) + carve_size<double>(6 * (size_t)np) +
                              carve_size<double>((size_t)D * D) + carve_size<double>(spart_n) +
                              carve_size<unsigned>((size_t)nblk) + carve_size<double>(D) +
                              carve_size<double>(D + 3 * (size_t)nl) + carve_size<double>(std::max(Ea, nl)) +
                              carve_size<double>(nl + np) + (glob ? carve_size<double>((size_t)Dp * (Dp + 1)) : 0) +
                              carve_size<double>(2 * (size_t)((nl * 8 + 63) / 64)) +
                              64;
        if ((rc2 = C.sys.reserve(ybytes))) return rc2;
        Carve cy{C.sys.as<char>()};
        b.J = cy.take<double>(72 * (size_t)Ea);
        b.W = cy.take<double>(24 * (size_t)Ea);
        b.Hll = cy.take<double>(9 * (size_t)nl);
        b.Dinv = cy.take<double>(9 * (size_t)nl);
        b.bl = cy.take<double>(3 * (size_t)nl);
        b.Hpp = cy.take<double>(36 * (size_t)np);
        b.bp = cy.take<double>(6 * (size_t)np);
        b.S = cy.take<double>((size_t)D * D);
        b.Spart = cy.take<double>(spart_n);
        b.blk_done = cy.take<unsigned>((size_t)nblk);
        b.bs = cy.take<double>(D);
        b.x = cy.take<double>(D + 3 * (size_t)nl);
        b.rchi = cy.take<double>(std::max(Ea, nl));
        b.part = cy.take<double>(nl + np);
        b.Sg = glob ? cy.take<double>((size_t)Dp * (Dp + 1)) : nullptr;
        double* d_wgpart = cy.take<double>(2 * (size_t)((nl * 8 + 63) / 64));   // point-update workgroup partials
        // (J needs no clearing: every linearising trial writes the entries that are read -- those of the
        // edges to free poses, zeros for a level-1 edge.  S / the part matrices are zero where no pose
        // pair block is, and the second optimize() keeps the structure, so they are cleared once.)
        if (fresh && ((rc2 = glob ? fills.add(b.S, (size_t)D * D * 8, 0, st) : fills.add(b.Spart, spart_n * 8, 0, st)) ||
                      (rc2 = fills.add(b.blk_done, (size_t)nblk * 4, 0, st))))
            return rc2;
        if (fresh) {   // the first optimize()'s control block (ba_ctl_start_kernel(iters, 0) on a zeroed block)
            BACtl init{};
            init.done = iters <= 0 ? 1 : 0;
            init.need_lin = 1;
            init.iters_max = iters;
            fills.set_ctl(b.ctl, init);
        }
        if (!have_structure) {
        if ((rc2 = C.structure.reserve(sbytes))) return rc2;
        if ((rc2 = C.h_struct.ensure(sbytes))) return rc2;
        Carve cr{C.structure.as<char>()}, hr{C.h_struct.ptr};
        auto put = [&](const void* src, size_t n, char* hdst) {
            if (n) std::memcpy(hdst, src, n);
        };
        // the host-built arrays first (the device build uploads only these), then the four lists
        int* d_hp = cr.take<int>(P);
        int* d_hl = cr.take<int>(N);
        int* d_ptb = cr.take<int>(nl + 1);
        int* d_pti = cr.take<int>(nl);
        int* d_psb = cr.take<int>(np + 1);
        int* d_psi = cr.take<int>(np);
        int* d_b1 = cr.take<int>(nblk);
        int* d_b2 = cr.take<int>(nblk);
        int* d_bb = cr.take<int>(nblk + 1);
        int* d_bd = cr.take<int>(np);
        const size_t small_bytes = cr.off;
        int* d_act = cr.take<int>(Ea);
        int* d_pts = cr.take<int>(Ea);
        int* d_pss = cr.take<int>(nps);
        int2* d_bp = cr.take<int2>(npairs);
        const size_t list_bytes = cr.off;   // the host build uploads up to here
        int4* d_rec = cr.take<int4>(Ea);
        put(hs.hp.data(), 4 * (size_t)P, (char*)hr.take<int>(P));
        put(hs.hl.data(), 4 * (size_t)N, (char*)hr.take<int>(N));
        put(hs.pt_beg.data(), 4 * (size_t)(nl + 1), (char*)hr.take<int>(nl + 1));
        put(hs.pt_id.data(), 4 * (size_t)nl, (char*)hr.take<int>(nl));
        put(hs.ps_beg.data(), 4 * (size_t)(np + 1), (char*)hr.take<int>(np + 1));
        put(hs.ps_id.data(), 4 * (size_t)np, (char*)hr.take<int>(np));
        put(hs.blk_i1.data(), 4 * (size_t)nblk, (char*)hr.take<int>(nblk));
        put(hs.blk_i2.data(), 4 * (size_t)nblk, (char*)hr.take<int>(nblk));
        put(hs.blk_beg.data(), 4 * (size_t)(nblk + 1), (char*)hr.take<int>(nblk + 1));
        {
            int* bd = hr.take<int>(np);
            for (int k = 0; k < nblk; k++)
                if (hs.blk_i1[k] == hs.blk_i2[k]) bd[hs.blk_i1[k]] = k;
        }
        if (dev_build) {
            int* d_slot = cr.take<int>((size_t)np * nl);
            ORB_HIP_TRY(hipMemcpyAsync(C.structure.ptr, C.h_struct.ptr, small_bytes, hipMemcpyHostToDevice, st));
            if ((rc2 = fills.add(d_slot, 4 * (size_t)np * nl, 0xff, st)) || (rc2 = fills.flush(st))) return rc2;
            if (Ea)
                hipLaunchKernelGGL(ba_struct_slots_kernel, dim3((Ea + 255) / 256), dim3(256), 0, st, d_ep, d_ek, d_hp, d_hl,
                                   Ea, nl, d_act, d_pts, d_slot, d_rec);
            if (nblk && nl)
                hipLaunchKernelGGL(ba_struct_pairs_kernel, dim3(nblk), dim3(1024), 0, st, d_b1, d_b2, d_bb, d_psb, d_slot, nl,
                                   d_bp, d_pss);
            ORB_HIP_TRY(hipGetLastError());
        } else {
            put(hs.act.data(), 4 * (size_t)Ea, (char*)hr.take<int>(Ea));
            put(hs.pt_slot.data(), 4 * (size_t)Ea, (char*)hr.take<int>(Ea));
            put(hs.ps_slot.data(), 4 * nps, (char*)hr.take<int>(nps));
            put(hs.blk_pair.data(), 8 * npairs, (char*)hr.take<int2>(npairs));
            ORB_HIP_TRY(hipMemcpyAsync(C.structure.ptr, C.h_struct.ptr, list_bytes, hipMemcpyHostToDevice, st));
        }
        b.Ea = Ea; b.np = np; b.nl = nl; b.nblk = nblk;
        b.act = d_act; b.hp = d_hp; b.hl = d_hl; b.pt_beg = d_ptb; b.pt_slot = d_pts; b.pt_id = d_pti;
        b.ps_beg = d_psb; b.ps_slot = d_pss; b.ps_id = d_psi; b.blk_i1 = d_b1; b.blk_i2 = d_b2; b.blk_beg = d_bb;
        b.blk_pair = d_bp;
        b.blk_diag = d_bd;
        b.pt_rec = d_rec;
        if (Ea && !dev_build) hipLaunchKernelGGL(ba_rec_kernel, dim3((Ea + 255) / 256), dim3(256), 0, st, b);
        ORB_HIP_TRY(hipGetLastError());
        have_structure = true;
        }
        if ((rc2 = fills.flush(st))) return rc2;
        const size_t ldlt_lds = glob ? (size_t)3 * Dp * 8 : std::max<size_t>(solve_lds_doubles(D) * 8, 16);
        {   // the dynamic LDS limit is a process-wide attribute of the kernel: raised (a host call) only
            // when a call needs more than any call before it on this device, never lowered
            static std::mutex mu;
            static size_t lim[64][3] = {};
            const size_t need = std::max<size_t>(ldlt_lds, 1024);
            std::lock_guard<std::mutex> lk(mu);
            size_t& cur = lim[device & 63][glob ? 1 : solve256 ? 2 : 0];
            if (need > cur) {
                ORB_HIP_TRY(hipFuncSetAttribute(solve_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need));
                cur = need;
            }
        }
        const dim3 gg((nl * 8 + 63) / 64);   // 8 lanes per point
        // The LM loop runs on the device (ba_decide_step advances it); the host keeps LOOKAHEAD
        // steps enqueued and reads each step's control snapshot from a pinned ring, so no trial
        // waits for a host round trip.  Steps enqueued past the end return immediately.
        mark("structure upload enqueued");
        constexpr int LOOKAHEAD = 2;
        const int first_seq = C.step_seq == 0x7fffffff ? 1 : C.step_seq + 1;   // step 0's id (slot 0)
        if (!fresh && !started_ahead)   // (the first optimize()'s control block came with the fill launch; the
                                         // second's ctl_start may have been enqueued behind the first loop)
            hipLaunchKernelGGL(ba_ctl_start_kernel, dim3(1), dim3(1), 0, st, b, iters, have_classified ? 1 : 0,
                               C.d_ring + 0, first_seq, 0);
        const int max_steps = iters * 10;
        int enq = 0, seen = 0;
        int spec_at = 0;   // steps enqueued ahead of the latest speculative gather / classification
        bool trans_spec = false;   // the second loop's ctl_start is enqueued behind the first loop's steps
        int ids[LOOKAHEAD] = {0, 0};
        bool fin = false, stop_sent = false;
        BACtl last{};
        while (!fin) {
            // no trial past the ones that can still be needed: each completes at most one iteration, so
            // with as many in flight as iterations remain (the latest snapshot's), the next is enqueued
            // only if one of those turns out a retry (round 6: the call used to end behind up to
            // LOOKAHEAD no-op trials of 5 launches each)
            const int remaining = seen ? last.iters_max - last.it : iters;
            while (enq < max_steps && enq - seen < LOOKAHEAD && enq - seen < remaining && !(trans_spec && seen < spec_at)) {
                hipLaunchKernelGGL(ba_iter_kernel, gg, dim3(64), 0, st, b);
                if (enq == 0) {   // first trial: computeLambdaInit needs Hpp before the Schur step
                    hipLaunchKernelGGL(ba_pose_accum_kernel, dim3(np + 1), dim3(1024), 0, st, b);
                    hipLaunchKernelGGL(ba_schur_point_kernel, gg, dim3(64), 0, st, b);
                }
                hipLaunchKernelGGL(ba_schur_block_kernel, dim3(nblk + 1 + np, SB_SPLIT), dim3(1024), 0, st, b, D, enq == 0 ? 0 : 1,
                                   glob ? 0 : 1);
                if (glob) hipLaunchKernelGGL(ba_solve_global_kernel, dim3(1), dim3(1024), ldlt_lds, st, b, D);
                else if (solve256) hipLaunchKernelGGL(ba_solve_kernel<256>, dim3(1), dim3(256), ldlt_lds, st, b, D, 1);
                else hipLaunchKernelGGL(ba_solve_kernel<1024>, dim3(1), dim3(1024), ldlt_lds, st, b, D, simd0_helpers);
                const int slot = enq % LOOKAHEAD;
                C.step_seq = C.step_seq == 0x7fffffff ? 1 : C.step_seq + 1;
                ids[slot] = C.step_seq;
                hipLaunchKernelGGL(ba_point_update_kernel, gg, dim3(64), 0, st, b, D, d_wgpart);
                hipLaunchKernelGGL(ba_decide_kernel, dim3(1), dim3(256), 0, st, b, C.d_ring + slot, ids[slot],
                                   (const double*)d_wgpart, (int)gg.x);
                ORB_HIP_TRY(hipGetLastError());
                enq++;
            }
            // the call's last loop: once the steps in flight are all that can be needed (no retry),
            // the final gather goes right behind them, guarded on `done` -- the GPU need not wait for
            // the host to see the last snapshot (round 6: ~15 us per call)
            // (the first loop: the classification, which leaves the control block as it is, so steps
            // enqueued after it still run as the first loop's; loop 2's ctl_start stays host-driven)
            // Without a stop flag or test hook, the first loop also gets the second's ctl_start behind
            // its classification: then no step of the first loop is enqueued after them until every
            // step before them has reported (trans_spec), since a step run after a ctl_start that did
            // start the second loop would be taken for the second loop's.
            if ((last_loop ? n_gather : E) && enq > spec_at && !stop_sent &&
                enq - seen >= (seen ? last.iters_max - last.it : iters) - spec_slack) {
                spec_launched[last_loop ? 1 : 0]++;
                if (last_loop) {
                    gather(1);
                } else {
                    classify_levels(1);
                    if (!stop_flag && stop_after < 0) {
                        const int seq2 = C.step_seq == 0x7fffffff ? 1 : C.step_seq + 1;   // the second loop's step 0
                        hipLaunchKernelGGL(ba_ctl_start_kernel, dim3(1), dim3(1), 0, st, b, next_iters, 1, C.d_ring + 0,
                                           seq2, 1);
                        trans_spec = true;
                    }
                }
                spec_at = enq;
            }
            if (seen == enq || stop_sent) break;
            const int slot = seen % LOOKAHEAD;
            // wait for the step's snapshot (a step that runs always writes one), mirroring the
            // caller's stop flag into the device-visible word the decide kernel polls after every
            // trial; the stream is queried now and then so a failed launch cannot hang the host
            auto t_q = std::chrono::steady_clock::now();
            while (__atomic_load_n(&C.h_ring[slot].seq, __ATOMIC_ACQUIRE) != ids[slot]) {
                if (stop_flag) __atomic_store_n(C.h_stop, *stop_flag ? 1 : 0, __ATOMIC_RELEASE);
                const auto now = std::chrono::steady_clock::now();
                if (now - t_q > std::chrono::microseconds(200)) {
                    t_q = now;
                    const hipError_t q = hipStreamQuery(st);
                    if (q != hipSuccess && q != hipErrorNotReady) ORB_HIP_TRY(q);
                    if (q == hipSuccess && __atomic_load_n(&C.h_ring[slot].seq, __ATOMIC_ACQUIRE) != ids[slot]) {
                        set_error("LocalBA: LM step finished without a control snapshot");
                        return ORB_EHIP;
                    }
                }
            }
            last = C.h_ring[slot];
            seen++;
            fin = last.done != 0;
            if (trans_spec && !fin && seen == spec_at) trans_spec = false;   // it did nothing: go on
            if (!fin && stopped() && !stop_sent) {   // force stop: end the loop after the steps in flight
                hipLaunchKernelGGL(ba_ctl_stop_kernel, dim3(1), dim3(1), 0, st, b);
                stop_sent = true;
            }
        }
        mark("LM loop done");
        if (!fin) {   // loop cut short (step cap or force stop): the device state is authoritative
            ORB_HIP_TRY(hipStreamSynchronize(st));
            ORB_HIP_TRY(hipMemcpy(&last, b.ctl, sizeof(BACtl), hipMemcpyDeviceToHost));
        }
        // else: `last` is the final snapshot; the steps still queued return at once, stream-ordered
        // before anything the caller enqueues next.  The step that ended the loop is step `seen` - 1:
        // a speculative gather enqueued after it ran on the final state.
        if (fin && seen <= spec_at) {
            (last_loop ? gathered : leveled) = true;
            if (trans_spec) started_ahead = true;
        }
        *iters_out = last.iters_done;
        *chi_out = last.chi_out;
        hook_stopped = hook_stopped || last.stopped;
        return ORB_OK;
    };

    const bool run = !stopped() && stop_after != 0;   // Optimizer.cc:633-634: stop before optimising => nothing done
    res->ran = run ? 1 : 0;
    if (run) {
        if ((rc = optimize(5, &res->iterations[0], &res->chi2[0], false))) return rc;
        if (!stopped() && !hook_stopped) {   // doMore (:639-642)
            // tag outliers (level 1) and drop the robust kernels (:644-670)
            // (no host copy of the levels: the structure is not rebuilt and the device counts the
            // level-0 edges for ba_ctl_start_kernel)
            if (E) {
                if (!leveled) classify_levels(0);
                ORB_HIP_TRY(hipGetLastError());
                have_classified = true;
            }
            mark("classify enqueued");
            if ((rc = optimize(next_iters, &res->iterations[1], &res->chi2[1], true))) return rc;
        }
    }
    Carve hres{C.h_res.ptr};
    double* hq = hres.take<double>(4 * (size_t)P);
    double* ht = hres.take<double>(3 * (size_t)P);
    double* hX = hres.take<double>(3 * (size_t)N);
    uint8_t* ho = hres.take<uint8_t>(E);
    double* hc = hres.take<double>(E);
    if ((rc = fills.flush(st))) return rc;   // (a call that optimised nothing still classifies)
    if (n_gather && !gathered) {
        gather(0);
        ORB_HIP_TRY(hipGetLastError());
    }
    ORB_HIP_TRY(hipStreamSynchronize(st));
    mark("results copied");
    std::memcpy(res->pose_t, ht, 24 * (size_t)P);
    std::memcpy(res->points, hX, 24 * (size_t)N);
    if (run) std::memcpy(res->edge_outlier, ho, E);
    else std::memset(res->edge_outlier, 0, E);
    if (res->edge_chi2) std::memcpy(res->edge_chi2, hc, 8 * (size_t)E);
    for (int i = 0; i < P; i++) {
        q_to_R(&hq[4 * i], res->pose_R + 9 * i);
        if (res->pose_q) std::memcpy(res->pose_q + 4 * i, &hq[4 * i], 32);
    }
    if (helper_wait.on) {   // (a call that optimised nothing never waited for the counts)
        C.helper.wait();
        helper_wait.on = false;
    }
    // the dense pair-block scratch (slot_of: nl x np ints, col: np x nl/64 words) of a very large window
    // is released rather than kept with the thread (C4 keeps its 0.3 MB)
    if (hs.slot_of.capacity() * sizeof(int) + hs.col.capacity() * sizeof(unsigned long long) > (8u << 20)) {
        std::vector<int>().swap(hs.slot_of);
        std::vector<unsigned long long>().swap(hs.col);
    }
    mark("end");
    if (tdbg)
        fprintf(stderr, "orbba loop ends enqueued ahead: first loop %d (used %d, ctl_start %d), second %d (used %d)\n",
                spec_launched[0], leveled ? 1 : 0, started_ahead ? 1 : 0, spec_launched[1], gathered ? 1 : 0);
    if (tdbg)
        for (size_t i = 1; i < marks.size(); i++)
            fprintf(stderr, "orbba %-28s %8.1f us\n", marks[i].first,
                    std::chrono::duration<double, std::micro>(marks[i].second - marks[i - 1].second).count());
    return ORB_OK;
}

extern "C" int orbba_debug_stamps(unsigned long long* out) {
#ifdef ORB_BA_STAMPS
    ORB_HIP_TRY(hipDeviceSynchronize());
    ORB_HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ba_stamps), 64 * 8));
    return ORB_OK;
#else
    (void)out;
    set_error("built without ORB_BA_STAMPS");
    return ORB_EINVAL;
#endif
}
