// Dependent-launch floor on one stream: N launches of a trivial kernel, wall time per launch, for
// (a) an empty kernel with a 16-byte argument, (b) a 512-byte argument struct, (c) (b) plus one
// global flag load, (d) (c) at 94 x 256 threads, (e) (c) with 128 KiB of dynamic LDS.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { void* p[64]; };
__global__ void k_small(int* f) { if (f[0] == 12345) f[1] = 1; }
__global__ void k_big(Big b) { if (threadIdx.x == 1000) ((int*)b.p[0])[0] = 1; }
__global__ void k_big_flag(Big b) {
    if (*(volatile int*)b.p[0] == 12345) return;
    if (threadIdx.x == 1000) ((int*)b.p[1])[0] = 1;
}
__global__ void k_lds(Big b) {
    extern __shared__ int sm[];
    if (*(volatile int*)b.p[0] == 12345) return;
    if (threadIdx.x == 1000) sm[0] = 1, ((int*)b.p[1])[0] = sm[1];
}

template <typename F>
static double run(const char* name, F launch, hipStream_t s, int n) {
    for (int i = 0; i < 50; i++) launch();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < n; i++) launch();
    hipStreamSynchronize(s);
    auto t1 = std::chrono::high_resolution_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
    printf("%-28s %.2f us per launch\n", name, us);
    return us;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* d;
    hipMalloc(&d, 4096);
    hipMemset(d, 0, 4096);
    Big b{};
    for (int i = 0; i < 64; i++) b.p[i] = d;
    hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    const int n = 2000;
    for (int rep = 0; rep < 2; rep++) {
        run("empty, 8 B arg, 1x64", [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d); }, s, n);
        run("512 B arg, 1x256", [&] { hipLaunchKernelGGL(k_big, dim3(1), dim3(256), 0, s, b); }, s, n);
        run("512 B arg + flag, 1x256", [&] { hipLaunchKernelGGL(k_big_flag, dim3(1), dim3(256), 0, s, b); }, s, n);
        run("512 B arg + flag, 94x256", [&] { hipLaunchKernelGGL(k_big_flag, dim3(94), dim3(256), 0, s, b); }, s, n);
        run("512 B arg + flag, 380x1024", [&] { hipLaunchKernelGGL(k_big_flag, dim3(380), dim3(1024), 0, s, b); }, s, n);
        run("+ 128 KiB LDS, 1x256", [&] { hipLaunchKernelGGL(k_lds, dim3(1), dim3(256), 131072, s, b); }, s, n);
    }
    // the same chains captured in a graph (no host launch cost): the dependent-boundary floor
    auto graph = [&](const char* name, auto launch) {
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < 200; i++) launch();
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int i = 0; i < 3; i++) hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        auto t0 = std::chrono::high_resolution_clock::now();
        for (int i = 0; i < 10; i++) hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        auto t1 = std::chrono::high_resolution_clock::now();
        printf("graph %-22s %.2f us per kernel\n", name, std::chrono::duration<double, std::micro>(t1 - t0).count() / 2000);
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
    };
    for (int rep = 0; rep < 2; rep++) {
        graph("empty 1x64", [&] { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d); });
        graph("512 B + flag 94x256", [&] { hipLaunchKernelGGL(k_big_flag, dim3(94), dim3(256), 0, s, b); });
        graph("512 B + flag 380x1024", [&] { hipLaunchKernelGGL(k_big_flag, dim3(380), dim3(1024), 0, s, b); });
        graph("128 KiB LDS 1x256", [&] { hipLaunchKernelGGL(k_lds, dim3(1), dim3(256), 131072, s, b); });
    }
    printf("done\n");
    return 0;
}
