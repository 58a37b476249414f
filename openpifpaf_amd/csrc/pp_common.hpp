// pp_common.hpp — shared device helpers for the gfx950 CIF/CAF decoder kernels.
//
// Numerics contract: every kernel is compiled with
// -ffp-contract=off and IEEE-correct f32 division/sqrt (hipcc's default), so each float
// op below rounds exactly like the reference's compiled Cython / NumPy float32 op.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "pifpaf_amd.h"

namespace pp {

constexpr int kWave = 64;

// -------------------------------------------------------------------------------------
// host-side error plumbing (thread-local message, pp_status codes)
// -------------------------------------------------------------------------------------
void set_error(const std::string &msg);
// Annotation.score() of a host record (stages_cpu.hip): zero_j >= 0 suppress_score_index,
// w the record's own score_weights (NULL: the default weights)
double ann_score_cpu(const pp_ann &a, int K, int zero_j = -1, const double *w = nullptr);
int fail(int status, const std::string &msg);
int check_launch(const char *what);

inline int64_t hr_dim(int64_t n, int stride) { return (n - 1) * stride + 1; }
// CifHr maps must stay below this many pixels per side: the fold packs a pixel's (x, y)
// into two signed 16-bit halves for its box test
constexpr int kMaxHrSide = 32768;

// -------------------------------------------------------------------------------------
// device helpers
// -------------------------------------------------------------------------------------

// functional.pyx:67-68 clip(): fmax(minv, fmin(maxv, v)); the double round trip of the
// generated C is exact for float inputs, and NaN behaves the same (fmin/fmax drop NaN).
__host__ __device__ __forceinline__ float clip_ref(float v, float minv, float maxv) {
    return fmaxf(minv, fminf(maxv, v));
}

// functional.pyx:57-64 approx_exp.  (float)(1.0 + (double)x / 8.0) == fl32(1 + x*0.125f):
// x/8 is exact and double rounding of a single add is innocuous (53 >= 2*24+2).
__host__ __device__ __forceinline__ float approx_exp_ref(float x) {
    if (x > 2.0f || x < -2.0f) return 0.0f;
    x = 1.0f + x * 0.125f;
    x = x * x;
    x = x * x;
    x = x * x;
    return x;
}

// Correctly rounded n / d with a reciprocal refined once per divisor: the compiler's IEEE
// f32 division (v_div_scale, v_rcp, Newton step, two fma corrections, v_div_fmas,
// v_div_fixup) minus the scaling and special-case steps, which are the identity when
// d is in [1, 2^100] and n is finite or NaN with |n| <= 2^100 (no operand scaling is
// needed there; vcc = 0 makes v_div_fmas a plain fma).  Bit-identical to `n / d` on that
// domain (tests/hip/div_check.hip checks it exhaustively over sampled ranges); callers
// keep `n / d` for divisors outside it.
struct Recip {
    float d, r;
};
__device__ __forceinline__ Recip recip_of(float d) {
    float r = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    return {d, r};
}
__device__ __forceinline__ bool recip_ok(float d) { return d >= 1.0f && d <= 0x1p100f; }
__device__ __forceinline__ float div_refined(float n, const Recip &R) {
    float q = n * R.r;
    float rem = __builtin_fmaf(-R.d, q, n);
    q = __builtin_fmaf(rem, R.r, q);
    rem = __builtin_fmaf(-R.d, q, n);
    return __builtin_fmaf(rem, R.r, q);
}

// np.exp of a float32 (cifcaf.py:139) as NumPy computes it on x86-64 with FMA3 or AVX512F:
// NumPy 2.2's simd_exp_f32 (numpy/_core/src/umath/loops_exponent_log.dispatch.c.src, the
// constants of npy_simd_data.h).  The quadrant q = rint(x * log2 e) by the 1.5 * 2^23 trick,
// Cody-Waite reduction with two fused multiply-adds, a rational approximation (degree 5
// over degree 2, Horner with fused multiply-adds), one IEEE division, times 2^q (exact, or
// correctly rounded to a subnormal, as scalef / ldexp).  Bit-exact against np.exp over every
// float32 in [-104, 0] (tests/test_np_exp.py, host and device); it differs from a correctly
// rounded exp in about a third of its results (by one ulp).
__host__ __device__ __forceinline__ float np_exp_f32(float x) {
    if (x != x) return x;
    if (x >= 88.72283935546875f) return __builtin_inff();
    if (x <= -103.97208404541015625f) return 0.0f;
    float q = x * 1.442695040888963407359924681001892137f;
    q = q + 0x1.800000p+23f;
    q = q - 0x1.800000p+23f;
    float r = fmaf(q, -6.93145752e-1f, x);
    r = fmaf(q, -1.42860677e-6f, r);
    r = fmaf(q, 0.0f, r);
    float num = fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    num = fmaf(num, r, 5.114512081637298353406e-02f);
    num = fmaf(num, r, 2.473615434895520810817e-01f);
    num = fmaf(num, r, 7.257664613233124478488e-01f);
    num = fmaf(num, r, 9.999999999980870924916e-01f);
    float den = fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    den = fmaf(den, r, 1.0f);
#ifdef __HIP_DEVICE_COMPILE__
    // num / den correctly rounded through the refined reciprocal: |r| <= ln 2 / 2 puts den
    // in [0.9, 1.1], so 2 den lies in div_refined's divisor domain [1, 2^100] and 2 num
    // (< 3) in its dividend domain; (2 num) / (2 den) is the same quotient, and the
    // reciprocal (v_rcp + two fma) runs beside num's Horner steps
    const float quo = div_refined(2.0f * num, recip_of(2.0f * den));
#else
    const float quo = num / den;
#endif
    return ldexpf(quo, (int)q);
}

// np.float32 ** 2 (cifcaf.py:139 `sigma**2`, sigma a NumPy float32 scalar): NumPy's scalar
// power calls the C library's powf(x, 2.0f), here glibc 2.35's (sysdeps/ieee754/flt-32/
// e_powf.c, the FMA3 build the x86-64 ifunc selects on any CPU with FMA), which is NOT
// x * x: it rounds a double approximation of 2 log2|x| -> exp2, whose relative error is
// below 2^-33.03 over every normal result, and so differs from the correctly rounded square
// in about 0.07 % of inputs (tests/test_np_exp.py: bit-exact over every float32 x >= 0).
// Fast path: when every value within 2^-32 of the exact square x * x (a double, exact)
// rounds to the same float, that float is powf's result; otherwise the routine itself: a
// 16-entry log2 table (1/c, log2 c) with a degree-5 polynomial in r = z/c - 1, then a
// 32-entry exp2 table and a degree-3 polynomial, every multiply-add fused as the FMA build
// has it.  The table and coefficient values are glibc's (__powf_log2_data, __exp2f_data).
// bit casts usable on the host and on the device
__host__ __device__ __forceinline__ uint32_t u32_of(float f) { return __builtin_bit_cast(uint32_t, f); }
__host__ __device__ __forceinline__ float f32_of(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ __forceinline__ uint64_t u64_of(double d) { return __builtin_bit_cast(uint64_t, d); }
__host__ __device__ __forceinline__ double f64_of(uint64_t u) { return __builtin_bit_cast(double, u); }

// (not inlined: the slow path is rare, and inlined at every query it cost the grow kernels
// registers -- the seed loop's spills 61 -> 90, force-complete 128 -> 140 VGPRs)
inline __host__ __device__ __noinline__ double glibc_powf2_double(uint32_t ix, double *ylogx_out) {
    static constexpr double kInvc[16] = {
        0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0, 0x1.3c995b0b80385p+0,
        0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
        0x1.0953f419900a7p+0, 0x1.0000000000000p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1,
        0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
    static constexpr double kLogc[16] = {
        -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
        -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7af0p-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
        -0x1.a6f9db6475fcep-5, 0.0, 0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3,
        0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2, 0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2};
    static constexpr uint64_t kExp2[32] = {
        0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
        0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
        0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
        0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
        0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
        0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
        0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
        0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
    // log2_inline: x = 2^k z, z in [0x3f330000, 2 * 0x3f330000), c near the subinterval's centre
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const uint32_t top = tmp & 0xff800000u;
    const int k = (int32_t)top >> 23;
    const double z = (double)f32_of(ix - top);
    const double r = fma(z, kInvc[i], -1.0);
    const double y0 = kLogc[i] + (double)k;
    double y = fma(r, 0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2);
    const double p = fma(r, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1);
    const double r2 = r * r;
    double q = fma(r, 0x1.71547652ab82bp+0, y0);
    const double r4 = r2 * r2;
    q = fma(r2, p, q);
    y = fma(y, r4, q);
    const double ylogx = 2.0 * y;  // y * log2|x| with y = 2
    *ylogx_out = ylogx;
    // exp2_inline: ylogx = k/32 + r, 2^(k/32) from the table (exponent bits added)
    double kd = ylogx + 0x1.8p+47;
    const uint64_t ki = u64_of(kd);
    kd -= 0x1.8p+47;
    const double rr = ylogx - kd;
    const double s = f64_of(kExp2[ki & 31u] + (ki << 47));
    const double zz = fma(rr, 0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3);
    const double rr2 = rr * rr;
    double yy = fma(rr, 0x1.62e42ff0c52d6p-1, 1.0);
    yy = fma(zz, rr2, yy);
    return yy * s;
}

__host__ __device__ inline float np_pow2_f32(float x) {
    const double xd = (double)x;
    const double sq = xd * xd;  // exact (48 significant bits)
    if (sq >= 0x1p-126 && sq <= 0x1p+127) {
        const float lo = (float)(sq * (1.0 - 0x1p-32)), hi = (float)(sq * (1.0 + 0x1p-32));
        if (lo == hi) return lo;
    }
    uint32_t ix = u32_of(x) & 0x7fffffffu;  // y = 2 is even: the sign drops out
    if (ix == 0u || ix >= 0x7f800000u) return fabsf(x) * fabsf(x);  // 0, inf, NaN
    if (ix < 0x800000u) {  // subnormal: normalised (x 2^23, exponent -23)
        ix = u32_of(f32_of(ix) * 0x1p23f) & 0x7fffffffu;
        ix -= 23u << 23;
    }
    double ylogx;
    const double yd = glibc_powf2_double(ix, &ylogx);
    if (((u64_of(ylogx) >> 47) & 0xffffu) >= 0x80bfu) {  // |ylogx| >= 126
        if (ylogx > 0x1.fffffffd1d571p+6) return __builtin_inff();  // overflow
        if (ylogx <= -150.0) return 0.0f;                            // underflow
        if (ylogx < -149.0) return 0x1p-149f;                        // may underflow
    }
    return (float)yd;
}

// correctly rounded float32 exp through f64 (not inlined: exp_mode 1 is the rare mode)
inline __host__ __device__ __noinline__ float exp_cr_f32(float q) { return (float)exp((double)q); }

// the CAF score's np.exp under pp_config.exp_mode: 0 NumPy's SIMD routine, 1 correctly
// rounded (through f64; NumPy's scalar loop on CPUs without FMA3)
__host__ __device__ __forceinline__ float caf_exp(float q, int mode) {
    return mode ? exp_cr_f32(q) : np_exp_f32(q);
}

// functional.pyx:231-244 scalar_values for one point (bounds inclusive of W'-1, truncation)
__host__ __device__ __forceinline__ float hr_lookup(const float *field, int hh, int ww,
                                                    int64_t pitch, float x, float y, float dflt) {
    const float maxx = (float)ww - 1.0f, maxy = (float)hh - 1.0f;
    if (x < 0.0f || y < 0.0f || x > maxx || y > maxy) return dflt;
    if (x != x || y != y) return dflt;  // NaN: the reference indexes with (Py_ssize_t)NaN (UB)
    return field[(int64_t)(int)y * pitch + (int)x];
}

// The functional.pyx primitives' per-element bodies, shared by the gfx950 kernels
// (functional.hip) and their host twins (functional_cpu.hip).

// functional.pyx:247-286 point lookup i into out[i]; mode: 0 scalar_value, 1
// scalar_value_clipped (float field), 2 scalar_nonzero, 3 scalar_nonzero_clipped,
// 4 scalar_nonzero_clipped_with_reduction (u8 field)
__host__ __device__ __forceinline__ void lookup_at(const void *field, int h, int w, int64_t pitch,
                                                   int mode, float x, float y, float dflt, float r,
                                                   void *out, int64_t i) {
    const float maxx = (float)(w - 1), maxy = (float)(h - 1);
    if (mode == 0 || mode == 2) {
        const bool oob = x < 0.0f || y < 0.0f || x > maxx || y > maxy || x != x || y != y;
        if (mode == 0)
            ((float *)out)[i] = oob ? dflt : ((const float *)field)[(int64_t)(int)y * pitch + (int)x];
        else
            ((uint8_t *)out)[i] =
                oob ? (uint8_t)(int)dflt : ((const uint8_t *)field)[(int64_t)(int)y * pitch + (int)x];
        return;
    }
    if (mode == 4) {
        x = x / r;
        y = y / r;
    }
    x = clip_ref(x, 0.0f, maxx);
    y = clip_ref(y, 0.0f, maxy);
    const int64_t at = (int64_t)(int)y * pitch + (int)x;
    if (mode == 1)
        ((float *)out)[i] = ((const float *)field)[at];
    else
        ((uint8_t *)out)[i] = ((const uint8_t *)field)[at];
}

// column i of a (rows, n) field passes the filter (functional.pyx:214-228 paf_mask_center
// (3), 289-310 paf_center_b (2), 313-335 paf_center (1), 338-359 caf_center_s (0))
__host__ __device__ __forceinline__ bool center_take(const float *f, int64_t pitch, int64_t i,
                                                     int mode, float x, float y, float sigma) {
    const float r1 = f[pitch + i], r2 = f[2 * pitch + i];
    if (mode == 0 || mode == 1)
        return !(r1 < x - sigma) && !(r1 > x + sigma) && !(r2 < y - sigma) && !(r2 > y + sigma);
    const float r3 = f[3 * pitch + i];
    return r1 > x - sigma * r3 && r1 < x + sigma * r3 && r2 > y - sigma * r3 &&
           r2 < y + sigma * r3;
}

// functional.pyx:172-211, sequential sums in the reference's order; returns the steps run
__host__ __device__ inline int64_t weiszfeld_run(const float *x, int64_t n, int64_t xp, float *y,
                                                 const float *wts, float eps, int64_t max_steps,
                                                 float *denom) {
    for (int64_t s = 0; s < max_steps; s++) {
        const float prev0 = y[0], prev1 = y[1];
        for (int64_t i = 0; i < n; i++) {
            const float ax = x[i * xp] - prev0, ay = x[i * xp + 1] - prev1;
            denom[i] = (float)(sqrt((double)(ax * ax + ay * ay)) + (double)eps);
        }
        float top0 = 0.0f, top1 = 0.0f, bottom = 0.0f;
        for (int64_t j = 0; j < n; j++) {
            const float w = wts[j];
            top0 += (w * x[j * xp + 0]) / denom[j];  // weights_x[j, 0] / denom[j]
            top1 += (w * x[j * xp + 1]) / denom[j];
            bottom = bottom + w / denom[j];
        }
        y[0] = top0 / bottom;
        y[1] = top1 / bottom;
        if (fabs((double)(y[0] - prev0)) + fabs((double)(y[1] - prev1)) < 1e-2) return s + 1;
    }
    return max_steps > 0 ? max_steps : 0;
}

// Occupancy.set (occupancy.py:36-44) + scalar_square_add_single (decoder/utils.py:61-66):
// the box [x0, x1) x [y0, y1) of one mark, false when the reference marks nothing.
// round(x / reduction) etc.: float32 scalar division (NEP 50), half-to-even rounding;
// Python's max(min_scale_reduced, s) keeps the first argument unless s is larger
__host__ __device__ __forceinline__ bool occupancy_mark_box(int f, int n_planes, int64_t h,
                                                            int64_t w, float x, float y, float s,
                                                            float r, float msr, int64_t &x0,
                                                            int64_t &x1, int64_t &y0,
                                                            int64_t &y1) {
    const float xr = x / r, yr = y / r, sr = s / r;
    const float sm = sr > msr ? sr : msr;
    const bool ok = f >= 0 && f < n_planes && fabsf(xr) < 0x1p60f && fabsf(yr) < 0x1p60f &&
                    fabsf(sm) < 0x1p60f;  // NaN / inf: the reference's round() raises
    if (!ok) return false;
    const int64_t xi = (int64_t)rintf(xr), yi = (int64_t)rintf(yr), si = (int64_t)rintf(sm);
    x0 = xi - si > 0 ? xi - si : 0;
    y0 = yi - si > 0 ? yi - si : 0;
    const int64_t hx = xi + si + 1 < w ? xi + si + 1 : w, hy = yi + si + 1 < h ? yi + si + 1 : h;
    x1 = x0 + 1 > hx ? x0 + 1 : hx;
    y1 = y0 + 1 > hy ? y0 + 1 : hy;
    x1 = x1 < w ? x1 : w;
    y1 = y1 < h ? y1 : h;
    return x1 > x0 && y1 > y0;
}

// The CifHr map as the decode stages read it: dense row-major (n_img * K, hh, pitch) — the
// caller-visible layout — or, for the decoder's scratch map, block-sparse: 64x64 tiles of
// 8x8 blocks, (n_img * K, tiles, 64 blocks, 64 px) block-major, with one u64 per tile whose
// bit b says block b (= 8 * by + bx) was written.  The sparse kernel writes only blocks
// some splat box touches; an unwritten block reads as its true value 0.
constexpr int kHrTile = 64;

struct HrMap {
    const float *base;
    const uint64_t *masks; // block-sparse: (n_img * K, tiles) written-block masks; NULL: dense
    int hh, ww;
    int64_t pitch;         // dense row pitch
    int tiles_x, tiles;    // tile grid (tiles_x = pitch / 64 rounded up)
    // functional.pyx:231-244 scalar_values on plane `plane` (= image * K + field)
    __device__ __forceinline__ float at(int64_t plane, float x, float y, float dflt) const {
        const float maxx = (float)ww - 1.0f, maxy = (float)hh - 1.0f;
        if (x < 0.0f || y < 0.0f || x > maxx || y > maxy) return dflt;
        if (x != x || y != y) return dflt;
        const int ix = (int)x, iy = (int)y;
        if (!masks) return base[(plane * hh + iy) * pitch + ix];
        const int64_t t = plane * tiles + (iy >> 6) * tiles_x + (ix >> 6);
        const int b = ((iy >> 3) & 7) * 8 + ((ix >> 3) & 7);
        // a block's slot is fixed, so the value is loaded together with the mask (one
        // memory round trip) and dropped when the block was not written this launch
        const uint64_t m = masks[t];
        const float v = base[(t * 64 + b) * 64 + (iy & 7) * 8 + (ix & 7)];
        return ((m >> b) & 1ull) ? v : 0.0f;
    }
};

// dense map view of a caller's (n_img * K, hh, pitch) buffer
inline HrMap dense_hr(const float *base, int hh, int ww) {
    HrMap m{};
    m.base = base;
    m.hh = hh;
    m.ww = ww;
    m.pitch = (ww + 31) / 32 * 32;  // pp_cifhr_pitch
    m.tiles_x = (int)((m.pitch + kHrTile - 1) / kHrTile);
    m.tiles = m.tiles_x * ((hh + kHrTile - 1) / kHrTile);
    return m;
}

// Orders this wave's LDS / global accesses the way __syncthreads() does (workgroup-scope
// fence: outstanding stores complete before later loads) without the s_barrier, so code
// can run in ONE wave of a multi-wave workgroup (the seed loop's committer, a CifHr tile
// stripe) as well as in single-wave workgroups.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// count of set bits of `mask` below this lane (v_mbcnt)
__device__ __forceinline__ int lane_prefix(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Order-preserving block compaction: returns this thread's slot among the flagged threads
// of the block (threads in threadIdx order) and the block total.  `s_tmp` holds NW ints.
template <int NW>
__device__ __forceinline__ int block_compact(bool flag, int *s_tmp, int &total) {
    const uint64_t m = __ballot(flag);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s_tmp[wave] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const int c = s_tmp[w];
        off += (w < wave) ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + lane_prefix(m);
}

// XCD-aware remap: blocks b and b+8 land on one XCD (round-robin dispatch, speed only),
// so consecutive work items of one XCD share its L2.  nblocks must be a multiple of 8.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nblocks) {
    const int64_t per = nblocks >> 3;
    return (b & 7) * per + (b >> 3);
}

// rows of one column of the decoder's bucketed CAF sets (caf_bucketed_kernel): score,
// source x, y, target x, y, target scale, row-major index (as float bits)
constexpr int kColRows = 7;
// force-complete sets (caf_bucketed_kernel<true, ...>) of at most this many cells per
// (image, field) store u16 cell indices (the LDS-stash build), larger ones int32
constexpr int kSetBIdx16Max = 8192;

// The CIF and CAF heads of one decode (a FieldConfig, field_config.py:7-13); a
// single-scale decode is one CIF and one CAF head.  Concatenated cell index of CAF head m =
// caf_off[m] + row-major cell: the order of the reference's concatenated column sets
// (caf_scored.py:70, 81); seeds concatenate the CIF heads the same way (cif_off).
constexpr int kMaxHeads = PP_MAX_SCALES;

struct Heads {
    // CIF heads (cif_indices order)
    const float *cif[kMaxHeads];  // (n_img, K, 5, H, W)
    int cH[kMaxHeads], cW[kMaxHeads], cstride[kMaxHeads];
    int64_t cif_off[kMaxHeads + 1];
    float ms_th[kMaxHeads];       // fl32(cif_min_scale / stride)  (p[4] > ms_th)
    uint32_t ms_on;               // heads whose min scale is set (truthy in the reference)
    int n_cif;
    // CifHr groups (cif_hr.py:42-73 fill_multiple): gsize heads per group, member i of group
    // g is head g + i * n_groups (gsize 2: the hflip pairs g, g + n/2; gsize n: one group)
    int gsize;
    int n_groups;
    // the CifHr map's size: from a PP_ROLE_HRMAP entry, else CIF head 0's (H-1)*stride+1
    int hr_hh, hr_ww;
    // CAF heads (caf_indices order)
    const float *caf[kMaxHeads];  // (n_img, C, 9, H, W)
    int aH[kMaxHeads], aW[kMaxHeads], astride[kMaxHeads];
    int64_t caf_off[kMaxHeads + 1];
    float dmin_th[kMaxHeads];     // fl32(caf_min_distance / stride) (dist > dmin_th)
    float dmax_th[kMaxHeads];     // fl32(caf_max_distance / stride) (dist < dmax_th)
    uint32_t dmin_on, dmax_on;
    int n_caf;
    __host__ __device__ __forceinline__ int64_t cif_hw(int m) const { return (int64_t)cH[m] * cW[m]; }
    __host__ __device__ __forceinline__ int64_t caf_hw(int m) const { return (int64_t)aH[m] * aW[m]; }
    __host__ __device__ __forceinline__ int64_t cif_cells() const { return cif_off[n_cif]; }
    __host__ __device__ __forceinline__ int64_t caf_cells() const { return caf_off[n_caf]; }
    // CifHr group g: its members; the group uses head g's stride and min scale
    __host__ __device__ __forceinline__ int group_size() const { return gsize; }
    __host__ __device__ __forceinline__ int member(int g, int i) const { return g + i * n_groups; }
    // CAF head of a concatenated cell index (n <= 16: a short scalar scan)
    __host__ __device__ __forceinline__ int caf_head_of(int64_t idx) const {
        int m = 0;
        while (m + 1 < n_caf && idx >= caf_off[m + 1]) m++;
        return m;
    }
};

// validates a pp_scale list into Heads (need: PP_ROLE_* lists that must be non-empty);
// returns PP_OK or a pp_status
int make_heads(const pp_scale *sc, int n, int pairs, int need, Heads *h, const char *who);
// one CIF and one CAF head from the single-scale arguments
Heads single_head(const float *cif, const float *caf, int H, int W, int stride);

// stage launchers over heads (splat.hip, stages.hip)
size_t cifhr_heads_workspace_size(const Heads &h, int n_img, int K);
// dense (n_img * K, hh, pitch) map, every pixel written
template <bool DET>
int cifhr_heads_launch(const Heads &h, int32_t n_img, int32_t K, const pp_config *cfg,
                       float *d_cifhr, void *d_workspace, size_t workspace_bytes, hipStream_t s,
                       const char *who);
// the decoder's block-sparse scratch map (HrMap with masks): d_map (n_img * K, tiles, 64, 64),
// d_masks (n_img * K, tiles); d_aux (same size as d_map) only when h.n_groups > 1
size_t cifhr_sparse_workspace_size(const Heads &h, int n_img, int K);

// Seed emission fused into the decoder's CifHr kernel (cif_seeds.py:28-47 run by the
// workgroup that has just written the field's map): the per-(image, field) segments
// seeds_emit_kernel writes, in its layout (SeedArgs in stages.hip), for seeds_sort_kernel.
struct SeedSink {
    float *g_keys;   // (n_img, 4, cap): v, x, y, s planes; field f's segment at f * H * W
    int *g_f;        // (n_img, cap) field of each slot
    int *f_counts;   // (n_img, K) seeds per field
    int64_t cap;     // K * H * W
    int K;
    float th, score_scale;
    uint32_t skip;   // pp_config.seed_skip_mask
};
// the seeds scratch of launch_seeds as a SeedSink (stages.hip)
SeedSink seed_sink(int n_img, int K, const pp_config *cfg, int cap, void *scratch);
// whether the decoder emits the seeds inside its CifHr kernels for this batch: one CIF head,
// one workgroup per field or split fields with a prebuilt list (the fold's last workgroup
// per field emits them), seed threshold >= CifHr threshold (every seed cell is then a
// splat of the field's list); launch_seeds then only sorts
bool cifhr_fuses_seeds(const Heads &h, int n_img, int K, const pp_config *cfg);

// `sink` (NULL: none): emit the seeds too (cifhr_fuses_seeds must hold)
int cifhr_sparse_launch(const Heads &h, int32_t n_img, int32_t K, const pp_config *cfg,
                        float *d_map, float *d_aux, uint64_t *d_masks, void *d_workspace,
                        size_t workspace_bytes, hipStream_t s, const char *who,
                        const SeedSink *sink = nullptr);

}  // namespace pp
