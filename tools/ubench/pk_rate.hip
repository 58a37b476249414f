// Throughput of scalar f32 VALU (v_fma_f32 / v_mul_f32) vs packed (v_pk_fma_f32 / v_pk_mul_f32)
// on gfx950: 8 independent chains per lane, many waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIt = 4096;
__global__ __launch_bounds__(256) void k_scalar(float *out, float a, float b) {
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = threadIdx.x + i;
    for (int it = 0; it < kIt; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) x[i] = __builtin_fmaf(x[i], a, b);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_packed(float *out, float a, float b) {
    f2 x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = f2{(float)threadIdx.x + i, (float)threadIdx.x - i};
    const f2 A = {a, a}, B = {b, b};
    for (int it = 0; it < kIt; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_elementwise_fma(x[i], A, B);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pmul(float *out, float a, float b) {
    f2 x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = f2{(float)threadIdx.x + i, (float)threadIdx.x - i};
    const f2 A = {a, a};
    for (int it = 0; it < kIt; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = x[i] * A;
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    float *d;
    const int blocks = 256 * 8 * 4;
    hipMalloc(&d, blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int k = 0; k < 3; k++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            if (k == 0) k_scalar<<<blocks, 256>>>(d, 0.999f, 0.001f);
            if (k == 1) k_packed<<<blocks, 256>>>(d, 0.999f, 0.001f);
            if (k == 2) k_pmul<<<blocks, 256>>>(d, 0.999f, 0.001f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)blocks * 256 * kIt * 16;  // f32 element-ops
            printf("%s: %.3f ms, %.1f Gop/s (element ops)\n", k == 0 ? "scalar fma" : k == 1 ? "pk_fma" : "pk_mul", ms, ops / ms / 1e6);
        }
    }
    return 0;
}
