// FETCH_SIZE calibration (rocprofv3 --pmc FETCH_SIZE): streaming reads of a 256 MiB buffer with
// 4-, 8- and 16-byte loads per lane; the known byte count calibrates the counter for the access
// widths of the loss kernels (MI355X_MICROARCH.md: only 16-B reads are calibrated there).
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void k_read(const T* __restrict__ src, size_t n, float* out) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = src[i];
        acc += reinterpret_cast<const float*>(&v)[0];
    }
    if (acc == 12345.0f) out[0] = acc;  // keeps the loads
}

template <typename T>
__global__ void k_write(T* __restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        reinterpret_cast<float*>(&v)[0] = (float)i;
        for (int j = 1; j < (int)(sizeof(T) / 4); ++j) reinterpret_cast<float*>(&v)[j] = 0.0f;
        dst[i] = v;
    }
}

int main() {
    const size_t bytes = 256ull << 20;
    void* buf;
    float* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
    const dim3 grid(4096), block(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read<float>, grid, block, 0, 0, (const float*)buf, bytes / 4, out);
        hipLaunchKernelGGL(k_read<float2>, grid, block, 0, 0, (const float2*)buf, bytes / 8, out);
        hipLaunchKernelGGL(k_read<float4>, grid, block, 0, 0, (const float4*)buf, bytes / 16, out);
        hipLaunchKernelGGL(k_write<float>, grid, block, 0, 0, (float*)buf, bytes / 4);
        hipLaunchKernelGGL(k_write<float4>, grid, block, 0, 0, (float4*)buf, bytes / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("bytes per kernel %zu\n", bytes);
    return 0;
}
