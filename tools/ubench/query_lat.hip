// Microbenchmark: cycles per flat_query (the seed loop's set-A query, grow.hip) and per
// connection evaluation (forward + reverse query) for one wave alone on the GPU, over a
// synthetic 128-column set held in registers as eval_ahead holds it, with 1 / 4 / 16 / 64
// columns inside the query box.  Tells the query's own latency apart from what the seed
// loop's neighbours add (stamps).  Build + run on the box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//       tools/ubench/query_lat.hip -L openpifpaf_amd -lpifpaf_amd -o query_lat &&
//   LD_LIBRARY_PATH=openpifpaf_amd ./query_lat
#include "../../openpifpaf_amd/csrc/grow.hip"

#include <stdio.h>

using namespace pp;

__global__ __launch_bounds__(64) void query_lat(const float *cols, int n, float spread, int reps,
                                                 uint64_t *cycles, float *sink) {
    float v[kFlatPer][kColRows];
    flat_load(cols, 128, n, v);
    float acc = 0.0f, dep = 0.0f;  // dep: each query waits for the previous one's result
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < reps; i++) {
        float nx[4];
        const float x = 100.0f + spread * (float)(i & 7) * 1e-3f + dep;
        flat_query<false>(v, n, x, 100.0f, 4.0f, 0, nx);
        acc += nx[0] + nx[3];
        dep = 0.0f * nx[3];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < reps; i++) {  // connection evaluation: forward, then reverse
        float nx[4], rv[4];
        const float x = 100.0f + spread * (float)(i & 7) * 1e-3f + dep;
        flat_query<false>(v, n, x, 100.0f, 4.0f, 0, nx);
        flat_query<false>(v, n, nx[0], nx[1], max0(nx[2]), 0, rv);
        acc += rv[0] + rv[3];
        dep = 0.0f * rv[3];
    }
    const uint64_t t2 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        cycles[0] = t1 - t0;
        cycles[1] = t2 - t1;
    }
    sink[threadIdx.x] = acc;
}

int main() {
    const int n = 128;
    float h[kColRows * 128];
    for (int inbox : {1, 4, 16, 64}) {
        // columns: rows 0 score, 1-2 source x / y, 3-4 target x / y, 5 target scale, 6 index
        for (int k = 0; k < n; k++) {
            const bool in = k < inbox;
            h[0 * 128 + k] = 0.5f + 0.001f * k;
            h[1 * 128 + k] = in ? 100.0f + 0.1f * k : 500.0f + k;
            h[2 * 128 + k] = in ? 100.0f - 0.05f * k : 500.0f;
            h[3 * 128 + k] = 110.0f + 0.01f * k;
            h[4 * 128 + k] = 101.0f;
            h[5 * 128 + k] = 4.0f;
            h[6 * 128 + k] = __builtin_bit_cast(float, k);
        }
        float *d;
        uint64_t *cy;
        float *sink;
        (void)hipMalloc(&d, sizeof(h));
        (void)hipMalloc(&cy, 16);
        (void)hipMalloc(&sink, 256);
        (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
        const int reps = 2000;
        hipLaunchKernelGGL(query_lat, dim3(1), dim3(64), 0, 0, d, n, 1.0f, reps, cy, sink);
        uint64_t c[2];
        (void)hipMemcpy(c, cy, 16, hipMemcpyDeviceToHost);
        printf("columns in box %2d: %.0f cycles per query, %.0f per forward + reverse evaluation "
               "(s_memtime, one wave alone)\n", inbox, (double)c[0] / reps, (double)c[1] / reps);
        (void)hipFree(d);
        (void)hipFree(cy);
        (void)hipFree(sink);
    }
    return 0;
}
