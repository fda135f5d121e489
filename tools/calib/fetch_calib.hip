// PMC calibration: FETCH_SIZE / WRITE_SIZE per dispatch for known byte counts with the access
// widths the extractor kernels use (global_load_dword, _dwordx2, _dwordx4; global_store_dword).
// MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B/lane streaming reads; other widths
// must be calibrated on a known byte count.  Run under rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__global__ void read_kernel(const T* __restrict__ src, size_t n, unsigned* sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = src[i];
        const unsigned* w = reinterpret_cast<const unsigned*>(&v);
        for (unsigned k = 0; k < sizeof(T) / 4; k++) acc ^= w[k];
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;   // practically never: keeps the loads alive
}

__global__ void write_kernel(unsigned* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = (unsigned)i;
}

int main() {
    const size_t bytes = (size_t)1 << 30;   // 1 GiB: past the 256 MiB Infinity Cache
    void* buf = nullptr;
    unsigned* sink = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    (void)hipDeviceSynchronize();
    const dim3 grid(256 * 8), block(256);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(read_kernel<unsigned>, grid, block, 0, 0, (const unsigned*)buf, bytes / 4, sink);
        hipLaunchKernelGGL(read_kernel<uint2>, grid, block, 0, 0, (const uint2*)buf, bytes / 8, sink);
        hipLaunchKernelGGL(read_kernel<uint4>, grid, block, 0, 0, (const uint4*)buf, bytes / 16, sink);
        hipLaunchKernelGGL(write_kernel, grid, block, 0, 0, (unsigned*)buf, bytes / 4);
    }
    (void)hipDeviceSynchronize();
    printf("calibration buffer %zu bytes per dispatch\n", bytes);
    (void)hipFree(buf);
    (void)hipFree(sink);
    return 0;
}
