// Probe: ticks of orbba.hip's solve_diag_block (one 16x16 diagonal block of the LocalBA solve) on one
// wavefront alone, repeated; the rest of the workgroup idle.  Build: see tools/probe/README.
#include "orbba.hip"
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
}
int main() {
    unsigned long long* o;
    (void)hipMalloc(&o, 8);
    unsigned long long h = 0;
    for (int k = 0; k < 2; k++) {
        hipLaunchKernelGGL(diag_probe, dim3(1), dim3(64), 0, 0, o, 100);
        (void)hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost);
    }
    printf("solve_diag_block alone: %.0f ticks per call (16 pivots)\n", (double)(h & ((1ull << 40) - 1)) / 100);
    return 0;
}
