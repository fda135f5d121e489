// Probe: ticks of orbba.hip's solve_diag_block (one 16x16 diagonal block of the LocalBA solve) on one
// wavefront alone, repeated; the rest of the workgroup idle.  Build: see tools/probe/README.
#include "orbba.hip"
#include <cstring>
using namespace orbamd;
__global__ __launch_bounds__(64) void diag_probe(unsigned long long* out, int reps) {
    __shared__ double A[17 * 17 + 3 * 16];
    double* y = A + 17 * 17;
    double* dinv = y + 16;
    double* vz = dinv + 16;
    const int lane = threadIdx.x;
    unsigned long long acc = 0;
    for (int r = 0; r < reps; r++) {
        for (int i = lane; i < 16 * 16; i += 64) {
            const int a = i / 16, c = i % 16;
            A[a * 17 + c] = a == c ? 20.0 + a : 1.0 / (1 + a + c);
        }
        if (lane < 16) y[lane] = 1.0 + lane;
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        const bool ok = solve_diag_block(A, y, dinv, vz, 17, 0, lane, 16);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        acc += t1 - t0;
        if (!ok) acc += 1ull << 40;
        __syncthreads();
    }
    if (lane == 0) out[0] = acc;
    // results of the last call: Linv (upper triangle, (c, i) = Linv[i][c]), dinv, y (= z)
    for (int i = lane; i < 16 * 16; i += 64) out[1 + i] = __double_as_longlong(A[(i / 16) * 17 + i % 16]);
    if (lane < 16) {
        out[1 + 256 + lane] = __double_as_longlong(dinv[lane]);
        out[1 + 272 + lane] = __double_as_longlong(y[lane]);
    }
}
int main() {
    unsigned long long* o;
    (void)hipMalloc(&o, 8 * 300);
    unsigned long long h[300] = {0};
    for (int k = 0; k < 2; k++) {
        hipLaunchKernelGGL(diag_probe, dim3(1), dim3(64), 0, 0, o, 100);
        (void)hipMemcpy(h, o, 8 * 300, hipMemcpyDeviceToHost);
    }
    printf("solve_diag_block alone: %.0f ticks per call (16 pivots)\n", (double)(h[0] & ((1ull << 40) - 1)) / 100);
    // CPU LDL^T of the same block: Linv, dinv, z
    double A[16][16], L[16][16] = {}, d[16], z[16], Li[16][16] = {};
    for (int a = 0; a < 16; a++)
        for (int c = 0; c < 16; c++) A[a][c] = a == c ? 20.0 + a : 1.0 / (1 + a + c);
    for (int j = 0; j < 16; j++) {
        double s = A[j][j];
        for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k] * d[k];
        d[j] = s;
        L[j][j] = 1;
        for (int i = j + 1; i < 16; i++) {
            double t = A[i][j];
            for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k] * d[k];
            L[i][j] = t / d[j];
        }
    }
    for (int i = 0; i < 16; i++) {
        double t = 1.0 + i;
        for (int k = 0; k < i; k++) t -= L[i][k] * z[k];
        z[i] = t;
    }
    for (int c = 0; c < 16; c++) {
        Li[c][c] = 1;
        for (int i = c + 1; i < 16; i++) {
            double t = 0;
            for (int k = c; k < i; k++) t -= L[i][k] * Li[k][c];
            Li[i][c] = t;
        }
    }
    double eL = 0, eD = 0, eZ = 0;
    for (int i = 0; i < 16; i++)
        for (int c = 0; c < i; c++) {
            double g;
            unsigned long long u = h[1 + c * 16 + i];
            memcpy(&g, &u, 8);
            eL = fmax(eL, fabs(g - Li[i][c]));
        }
    for (int i = 0; i < 16; i++) {
        double g1, g2;
        memcpy(&g1, &h[257 + i], 8);
        memcpy(&g2, &h[273 + i], 8);
        eD = fmax(eD, fabs(g1 - 1.0 / d[i]));
        eZ = fmax(eZ, fabs(g2 - z[i]));
    }
    printf("max |err|: Linv %.3g  dinv %.3g  z %.3g\n", eL, eD, eZ);
    if (eL > 1e-12) {   // wrong Linv entries (row i: columns c < i marked)
        for (int i = 1; i < 16; i++) {
            printf("  row %2d: ", i);
            for (int c = 0; c < i; c++) {
                double g;
                unsigned long long u = h[1 + c * 16 + i];
                memcpy(&g, &u, 8);
                printf("%c", fabs(g - Li[i][c]) > 1e-12 ? 'X' : '.');
            }
            printf("\n");
        }
    }
    return 0;
}
