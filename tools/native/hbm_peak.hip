// Achievable HBM bandwidth: a streaming read kernel (dwordx4
// loads, grid-stride, one partial sum per thread written at the end) and a
// dwordx4 copy kernel, timed with HIP events.  Measurement tool only.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(256) void read_kernel(const float4* __restrict__ a, size_t n4, float* __restrict__ out) {
    float s = 0.0f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 4 * stride) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i + u * stride < n4 ? a[i + u * stride] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void copy_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) b[i] = a[i];
}

extern "C" int hbm_peak(const void* a, void* b, size_t bytes, int reps, float* read_ms, float* copy_ms) {
    const size_t n4 = bytes / 16;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1;
    const int grid = cus * 8;
    float* part = nullptr;
    if (hipMalloc(&part, (size_t)grid * 256 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](bool copy) {
        if (copy) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0, (const float4*)a, (float4*)b, n4);
        else hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, (const float4*)a, n4, part);
    };
    for (int c = 0; c < 2; ++c) {
        run(c == 1);
        hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) run(c == 1);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        (c == 1 ? *copy_ms : *read_ms) = ms / reps;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipFree(part);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
