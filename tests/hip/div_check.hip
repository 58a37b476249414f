// div_check.hip — div_refined (pp_common.hpp) vs the compiler's IEEE f32 division, bit for
// bit, over the domains it is used on:
//  - the CifHr fold: divisors d = sigma^2 in [1, 2^100], numerators n = -0.5 * (dx^2 + dy^2)
//    with sum in [0.25, d] (plus NaN numerators);
//  - the CAF score (grow.hip score_arg): d = sigma^2 in [1, 2^90], n = -0.5 d^2 with
//    d^2 in [0, 128 sigma^2], log-uniform down to the subnormals, and exact zeros: the
//    quotient bit for bit where |n| >= 2^-60, np.exp of it below (both quotients round
//    np.exp to 1 there);
//  - NumPy's exp (pp_common.hpp np_exp_f32): (2 num) / (2 den) with den in [0.9, 1.1] and
//    num in [0.7, 1.5].
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

// numerators log-uniform over [2^-149, hi] (and 0), negated: the CAF score's domain
__global__ void check_wide(unsigned long long *bad, unsigned long long *done, uint32_t d_lo,
                           uint32_t d_n, int n_per_d, uint32_t seed, float hi_scale) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= d_n) return;
    const float d = __uint_as_float(d_lo + (uint32_t)t);
    volatile float dv = d;
    const Recip R = recip_of(d);
    uint32_t x = seed ^ (uint32_t)(t * 2654435761u);
    unsigned long long nb = 0, nd = 0;
    const float hi = hi_scale * d;
    float worst = 0.0f;
    for (int k = 0; k < n_per_d; k++) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const uint32_t hb = __float_as_uint(hi);
        // a random float bit pattern in [1 (subnormal), hi]
        const uint32_t u = 1u + (uint32_t)(((uint64_t)x * (uint64_t)(hb - 1u)) >> 32);
        float sum = __uint_as_float(u);
        if (k == 0) sum = 0.0f;
        if (k == 1) sum = hi;
        const float num = -0.5f * sum;
        const float a = num / dv;
        const float b = div_refined(num, R);
        // the quotient itself where |num| >= 2^-60; below, the score only needs the same
        // np.exp (both quotients are < 2^-59 in magnitude, where exp rounds to 1)
        const bool miss = sum >= 0x1p-59f ? __float_as_uint(a) != __float_as_uint(b)
                                          : __float_as_uint(np_exp_f32(a)) != __float_as_uint(np_exp_f32(b));
        nb += miss;
        if (miss) worst = fmaxf(worst, sum);
        nd++;
    }
    if (nb) {
        atomicAdd(bad, nb);
        atomicMax((unsigned int *)(bad + 1), __float_as_uint(worst));  // largest failing sum
    }
    atomicAdd(done, nd);
}

// np_exp_f32's (2 num) / (2 den): den in [0.9, 1.1] (every float), num random in [0.7, 1.5]
__global__ void check_exp(unsigned long long *bad, unsigned long long *done, uint32_t d_lo,
                          uint32_t d_n, int n_per_d, uint32_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= d_n) return;
    const float den = __uint_as_float(d_lo + (uint32_t)t);
    volatile float dv = den;
    const Recip R = recip_of(2.0f * den);
    uint32_t x = seed ^ (uint32_t)(t * 2654435761u);
    unsigned long long nb = 0, nd = 0;
    for (int k = 0; k < n_per_d; k++) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const float num = 0.7f + (float)(x >> 8) * 0x1p-24f * 0.8f;
        const float a = num / dv;
        const float b = div_refined(2.0f * num, R);
        nb += __float_as_uint(a) != __float_as_uint(b);
        nd++;
    }
    if (nb) atomicAdd(bad, nb);
    atomicAdd(done, nd);
}

int main() {
    unsigned long long *bad, *done, *bad_w, *bad_e;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&done, 8);
    (void)hipMalloc(&bad_w, 16);
    (void)hipMalloc(&bad_e, 8);
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(done, 0, 8);
    (void)hipMemset(bad_w, 0, 16);
    (void)hipMemset(bad_e, 0, 8);
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
    // the CAF score: every float in [1, 16), and sampled divisors up to 2^90
    {
        const uint32_t l1 = __builtin_bit_cast(uint32_t, 1.0f), h1 = __builtin_bit_cast(uint32_t, 16.0f);
        hipLaunchKernelGGL(check_wide, dim3((h1 - l1 + 255) / 256), dim3(256), 0, 0, bad_w, done, l1,
                           h1 - l1, 32, 4242u, 64.0f);
        const float wide[] = {16.0f, 777.0f, 1e6f, 1e12f, 1e20f, 1e26f};
        for (float st : wide) {
            const uint32_t l = __builtin_bit_cast(uint32_t, st);
            hipLaunchKernelGGL(check_wide, dim3((1u << 20) / 256), dim3(256), 0, 0, bad_w, done, l,
                               1u << 20, 32, 99u, 64.0f);
        }
        // np_exp_f32's quotients: every den in [0.9, 1.1]
        const uint32_t le = __builtin_bit_cast(uint32_t, 0.9f), he = __builtin_bit_cast(uint32_t, 1.1f);
        hipLaunchKernelGGL(check_exp, dim3((he - le + 255) / 256), dim3(256), 0, 0, bad_e, done, le,
                           he - le, 32, 31337u);
    }
    unsigned long long hb = 0, hd = 0, hw[2] = {0, 0}, he = 0;
    (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hd, done, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hw, bad_w, 16, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&he, bad_e, 8, hipMemcpyDeviceToHost);
    const uint32_t ws = (uint32_t)hw[1];
    printf("fold domain mismatches %llu; score domain mismatches %llu (largest failing sum %a); "
           "exp quotient mismatches %llu\n", hb, hw[0], __builtin_bit_cast(float, ws), he);
    hb += hw[0] + he;
    printf("checked %llu divisions, mismatches %llu\n", hd, hb);
    return hb == 0 && hd > 0 ? 0 : 1;
}
