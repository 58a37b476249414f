// div_check.hip — div_refined (pp_common.hpp) vs the compiler's IEEE f32 division, bit for
// bit, over the domain the CifHr fold uses it on: divisors d = sigma^2 in [1, 2^100],
// numerators n = -0.5 * (dx^2 + dy^2) with sum in [0.25, d] (plus NaN numerators).
// Exhaustive over d's float grid in [1, 64) x sampled numerators, random elsewhere.
// Build + run: tests/test_gpu_divcheck.py.  Prints the mismatch count; exit 1 if any.
#include "../../openpifpaf_amd/csrc/pp_common.hpp"

#include <stdio.h>

using namespace pp;

__global__ void check(unsigned long long *bad, unsigned long long *done, uint32_t d_lo, uint32_t d_n,
                      int n_per_d, uint32_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= d_n) return;
    const float d = __uint_as_float(d_lo + (uint32_t)t);  // consecutive floats
    volatile float dv = d;
    const Recip R = recip_of(d);
    uint32_t x = seed ^ (uint32_t)(t * 2654435761u);
    unsigned long long nb = 0, nd = 0;
    for (int k = 0; k < n_per_d; k++) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        // sum uniform in [0.25, d] by bits: random mantissa / exponent in range
        const float u = (float)(x >> 8) * 0x1p-24f;
        float sum = 0.25f + u * (d - 0.25f);
        if (k == 0) sum = d;          // circle edge
        if (k == 1) sum = 0.25f;
        const float num = -0.5f * sum;
        const float a = num / dv;    // the compiler's IEEE division
        const float b = div_refined(num, R);
        nb += __float_as_uint(a) != __float_as_uint(b);
        nd++;
    }
    if (nb) atomicAdd(bad, nb);
    atomicAdd(done, nd);
}

int main() {
    unsigned long long *bad, *done;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&done, 8);
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(done, 0, 8);
    // every float in [1, 64): 6 * 2^23 divisors, 64 numerators each
    const uint32_t lo = __builtin_bit_cast(uint32_t, 1.0f), hi = __builtin_bit_cast(uint32_t, 64.0f);
    const uint32_t n = hi - lo;
    hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, bad, done, lo, n, 64, 12345u);
    // sampled divisors up to 2^100: 2^20 consecutive floats at several exponents
    const float starts[] = {64.0f, 1000.0f, 3.3e5f, 1e9f, 1e15f, 1e22f, 1e29f};
    for (float st : starts) {
        const uint32_t l = __builtin_bit_cast(uint32_t, st);
        hipLaunchKernelGGL(check, dim3((1u << 20) / 256), dim3(256), 0, 0, bad, done, l, 1u << 20, 64, 777u);
    }
    unsigned long long hb = 0, hd = 0;
    (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hd, done, 8, hipMemcpyDeviceToHost);
    printf("checked %llu divisions, mismatches %llu\n", hd, hb);
    return hb == 0 && hd > 0 ? 0 : 1;
}
