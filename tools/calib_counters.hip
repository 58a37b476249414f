// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the decoder
// kernels use: coalesced 4-byte-per-lane and 16-byte-per-lane reads and writes of a 1 GiB
// buffer (well past the 256 MiB Infinity Cache).  Run under rocprofv3 --pmc and divide the
// counter (KB) by the known byte count.
//
//   hipcc --offload-arch=gfx950 -O3 tools/calib_counters.hip -o build/calib_counters
//   rocprofv3 --pmc FETCH_SIZE -d ... -o run --output-format csv -- build/calib_counters
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void read4(const float *__restrict__ p, size_t n, float *out) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 12345.678f) out[0] = acc;  // keeps the loads alive
}

__global__ void read16(const float4 *__restrict__ p, size_t n, float *out) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.678f) out[0] = acc;
}

__global__ void write4(float *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = 1.0f;
}

__global__ void write16(float4 *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    float *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 0, bytes);
    const dim3 grid(4096), block(256);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(read4, grid, block, 0, 0, buf, bytes / 4, out);
        hipLaunchKernelGGL(read16, grid, block, 0, 0, (const float4 *)buf, bytes / 16, out);
        hipLaunchKernelGGL(write4, grid, block, 0, 0, buf, bytes / 4);
        hipLaunchKernelGGL(write16, grid, block, 0, 0, (float4 *)buf, bytes / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("calib: %zu bytes per kernel\n", bytes);
    hipFree(buf);
    hipFree(out);
    return 0;
}
