// functional_cpu.hip — host twins of the openpifpaf.functional primitives (pp_*_cpu).
//
// every functional.pyx entry point has a `_hip` form (the gfx950 kernels
// in splat.hip / functional.hip, device pointers, a stream) and a `_cpu` form (this file:
// host pointers, run on the calling thread).  The twins exist for callers that hold host
// buffers and want the reference's arithmetic without a device round trip (the reference's
// own Cython module is CPU-only, functional.pyx:1-359).  No product path reaches them by
// fallback: the decoder and openpifpaf_amd.functional compute on the device and raise
// without one; openpifpaf_amd.functional_cpu is the explicit host API.
//
// The arithmetic is the kernels': the shared per-element helpers of pp_common.hpp
// (clip_ref, approx_exp_ref, hr_lookup, lookup_at, center_take, weiszfeld_run,
// occupancy_mark_box) are __host__ __device__, and the splats run the reference's own
// scatter loops (points in order, box columns then rows) with its double temporaries.
#include <cmath>

#include "pp_common.hpp"

namespace {

using pp::approx_exp_ref;
using pp::clip_ref;

// functional.pyx:105-141 / 71-102 / 144-169: the three Gaussian splats share the box and
// the value; MODE 0 with max (+1 on the high bounds, circle test, clamp), 1 add, 2 max.
template <int MODE>
void gauss_cpu(float *field, int64_t h, int64_t w, int64_t pitch, const float *x, const float *y,
               const float *sigma, const float *v, int64_t n, float truncate, float max_value) {
    const float truncate2 = truncate * truncate;
    for (int64_t i = 0; i < n; i++) {
        const float csigma = sigma[i], csigma2 = csigma * csigma;
        const float cx = x[i], cy = y[i], cv = v[i];
        float hx = cx + truncate * csigma, hy = cy + truncate * csigma;
        if (MODE == 0) {  // `... + 1` evaluated in double by the generated C
            hx = (float)((double)hx + 1.0);
            hy = (float)((double)hy + 1.0);
        }
        const int64_t minx = (int64_t)clip_ref(cx - truncate * csigma, 0.0f, (float)(w - 1));
        const int64_t maxx = (int64_t)clip_ref(hx, (float)(minx + 1), (float)w);
        const int64_t miny = (int64_t)clip_ref(cy - truncate * csigma, 0.0f, (float)(h - 1));
        const int64_t maxy = (int64_t)clip_ref(hy, (float)(miny + 1), (float)h);
        for (int64_t xx = minx; xx < maxx; xx++) {
            const float dx = (float)xx - cx, deltax2 = dx * dx;
            for (int64_t yy = miny; yy < maxy; yy++) {
                const float dy = (float)yy - cy, deltay2 = dy * dy;
                if (MODE == 0 && deltax2 + deltay2 > truncate2 * csigma2) continue;
                const float e = approx_exp_ref(
                    (float)((-0.5 * (double)(deltax2 + deltay2)) / (double)csigma2));
                float &f = field[yy * pitch + xx];
                if (MODE == 2) {
                    f = (float)std::fmax((double)f, (double)(cv * e));
                    continue;
                }
                const float vv = (deltax2 < 0.25 && deltay2 < 0.25) ? cv : cv * e;
                f += vv;
                if (MODE == 0) f = (f < max_value) ? f : max_value;
            }
        }
    }
}

// the (minx, maxx, miny, maxy) box of functional.pyx:15-18 / 40-43 (no +1)
struct Box {
    int64_t x0, x1, y0, y1;
};
inline Box width_box(float cx, float cy, float cwidth, int64_t h, int64_t w) {
    Box b;
    b.x0 = (int64_t)clip_ref(cx - cwidth, 0.0f, (float)(w - 1));
    b.x1 = (int64_t)clip_ref(cx + cwidth, (float)(b.x0 + 1), (float)w);
    b.y0 = (int64_t)clip_ref(cy - cwidth, 0.0f, (float)(h - 1));
    b.y1 = (int64_t)clip_ref(cy + cwidth, (float)(b.y0 + 1), (float)h);
    return b;
}

bool bad_field(const void *f, int64_t h, int64_t w, int64_t pitch) {
    return !f || h < 0 || w < 0 || pitch < w;
}

}  // namespace

extern "C" {

int pp_scalar_square_add_gauss_with_max_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                            const float *x, const float *y, const float *sigma,
                                            const float *v, int64_t n, float truncate,
                                            float max_value) {
    if (bad_field(field, h, w, pitch) || n < 0 || (n > 0 && (!x || !y || !sigma || !v)))
        return pp::fail(PP_EINVAL, "pp_scalar_square_add_gauss_with_max_cpu: bad argument");
    gauss_cpu<0>(field, h, w, pitch, x, y, sigma, v, n, truncate, max_value);
    return PP_OK;
}

int pp_scalar_square_add_gauss_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                   const float *x, const float *y, const float *sigma,
                                   const float *v, int64_t n, float truncate) {
    if (bad_field(field, h, w, pitch) || n < 0 || (n > 0 && (!x || !y || !sigma || !v)))
        return pp::fail(PP_EINVAL, "pp_scalar_square_add_gauss_cpu: bad argument");
    gauss_cpu<1>(field, h, w, pitch, x, y, sigma, v, n, truncate, 0.0f);
    return PP_OK;
}

int pp_scalar_square_max_gauss_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                   const float *x, const float *y, const float *sigma,
                                   const float *v, int64_t n, float truncate) {
    if (bad_field(field, h, w, pitch) || n < 0 || (n > 0 && (!x || !y || !sigma || !v)))
        return pp::fail(PP_EINVAL, "pp_scalar_square_max_gauss_cpu: bad argument");
    gauss_cpu<2>(field, h, w, pitch, x, y, sigma, v, n, truncate, 0.0f);
    return PP_OK;
}

// functional.pyx:7-26
int pp_scalar_square_add_constant_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                      const float *x, const float *y, const float *width,
                                      const float *v, int64_t n) {
    if (bad_field(field, h, w, pitch) || n < 0 || (n > 0 && (!x || !y || !width || !v)))
        return pp::fail(PP_EINVAL, "pp_scalar_square_add_constant_cpu: bad argument");
    for (int64_t i = 0; i < n; i++) {
        const Box b = width_box(x[i], y[i], width[i], h, w);
        for (int64_t xx = b.x0; xx < b.x1; xx++)
            for (int64_t yy = b.y0; yy < b.y1; yy++) field[yy * pitch + xx] += v[i];
    }
    return PP_OK;
}

// functional.pyx:29-54 (cdivision: f32 quotient; points with w <= 0 skipped)
int pp_cumulative_average_cpu(float *cuma, float *cumw, int64_t h, int64_t w, int64_t pitch,
                              const float *x, const float *y, const float *width,
                              const float *v, const float *wt, int64_t n) {
    if (bad_field(cuma, h, w, pitch) || !cumw || n < 0 ||
        (n > 0 && (!x || !y || !width || !v || !wt)))
        return pp::fail(PP_EINVAL, "pp_cumulative_average_cpu: bad argument");
    for (int64_t i = 0; i < n; i++) {
        const float cw = wt[i], cv = v[i];
        if (cw <= 0.0f) continue;
        const Box b = width_box(x[i], y[i], width[i], h, w);
        for (int64_t xx = b.x0; xx < b.x1; xx++)
            for (int64_t yy = b.y0; yy < b.y1; yy++) {
                float &a = cuma[yy * pitch + xx], &s = cumw[yy * pitch + xx];
                a = (cw * cv + s * a) / (s + cw);
                s += cw;
            }
    }
    return PP_OK;
}

// functional.pyx:172-211; *out_steps (optional) = iterations run
int pp_weiszfeld_nd_cpu(const float *x, int64_t n, int64_t d, int64_t x_pitch, float *y,
                        const float *weights, float epsilon, int64_t max_steps, float *denom,
                        int64_t *out_steps) {
    if (!x || !y || !weights || !denom) return pp::fail(PP_EINVAL, "pp_weiszfeld_nd_cpu: NULL argument");
    if (n < 0 || d < 2 || x_pitch < d) return pp::fail(PP_ESHAPE, "pp_weiszfeld_nd_cpu: bad shape");
    const int64_t s = pp::weiszfeld_run(x, n, x_pitch, y, weights, epsilon, max_steps, denom);
    if (out_steps) *out_steps = s;
    return PP_OK;
}

// functional.pyx:231-244
int pp_scalar_values_cpu(const float *field, int64_t h, int64_t w, int64_t pitch, const float *x,
                         const float *y, int64_t n, float default_value, float *out) {
    if (bad_field(field, h, w, pitch) || (n > 0 && (!x || !y || !out)))
        return pp::fail(PP_EINVAL, "pp_scalar_values_cpu: bad argument");
    for (int64_t i = 0; i < n; i++)
        out[i] = pp::hr_lookup(field, (int)h, (int)w, pitch, x[i], y[i], default_value);
    return PP_OK;
}

// functional.pyx:247-286, mode as pp_scalar_lookup
int pp_scalar_lookup_cpu(const void *field, int64_t h, int64_t w, int64_t pitch, int32_t mode,
                         const float *x, const float *y, int64_t n, float default_value,
                         float reduction, void *out) {
    if (!field || (n > 0 && (!x || !y || !out))) return pp::fail(PP_EINVAL, "pp_scalar_lookup_cpu: NULL argument");
    if (mode < 0 || mode > 4) return pp::fail(PP_EINVAL, "pp_scalar_lookup_cpu: bad mode");
    if (h <= 0 || w <= 0 || pitch < w) return pp::fail(PP_ESHAPE, "pp_scalar_lookup_cpu: bad field shape");
    for (int64_t i = 0; i < n; i++)
        pp::lookup_at(field, (int)h, (int)w, pitch, mode, x[i], y[i], default_value, reduction, out, i);
    return PP_OK;
}

// Occupancy.set + scalar_square_add_single (occupancy.py:36-44, decoder/utils.py:61-66)
int pp_occupancy_set_cpu(uint8_t *occ, int32_t n_planes, int64_t h, int64_t w, int64_t pitch,
                         const int32_t *f, const float *x, const float *y, const float *sigma,
                         int64_t n, float reduction, float min_scale_reduced) {
    if (!occ || (n > 0 && (!f || !x || !y || !sigma))) return pp::fail(PP_EINVAL, "pp_occupancy_set_cpu: NULL argument");
    if (n_planes < 0 || h < 0 || w < 0 || pitch < w || n < 0 || !(reduction > 0.0f))
        return pp::fail(PP_ESHAPE, "pp_occupancy_set_cpu: bad shape");
    for (int64_t i = 0; i < n; i++) {
        int64_t x0, x1, y0, y1;
        if (!pp::occupancy_mark_box(f[i], n_planes, h, w, x[i], y[i], sigma[i], reduction,
                                    min_scale_reduced, x0, x1, y0, y1))
            continue;
        uint8_t *plane = occ + (int64_t)f[i] * h * pitch;
        for (int64_t yy = y0; yy < y1; yy++)
            for (int64_t xx = x0; xx < x1; xx++) plane[yy * pitch + xx] = (uint8_t)(plane[yy * pitch + xx] + 1);
    }
    return PP_OK;
}

int pp_np_exp_cpu(const float *x, float *y, int64_t n, int32_t exp_mode) {
    if (!x || !y) return pp::fail(PP_EINVAL, "pp_np_exp_cpu: NULL argument");
    if (n < 0) return pp::fail(PP_ESHAPE, "pp_np_exp_cpu: bad length");
    if (exp_mode != 0 && exp_mode != 1) return pp::fail(PP_EINVAL, "pp_np_exp_cpu: bad exp_mode");
    for (int64_t i = 0; i < n; i++) y[i] = pp::caf_exp(x[i], exp_mode);
    return PP_OK;
}

int pp_np_square_cpu(const float *x, float *y, int64_t n) {
    if (!x || !y) return pp::fail(PP_EINVAL, "pp_np_square_cpu: NULL argument");
    if (n < 0) return pp::fail(PP_ESHAPE, "pp_np_square_cpu: bad length");
    for (int64_t i = 0; i < n; i++) y[i] = pp::np_pow2_f32(x[i]);
    return PP_OK;
}

// functional.pyx:214-228, 289-359 (mode as pp_center_filter); *count = kept columns
int pp_center_filter_cpu(const float *field, int64_t rows, int64_t n, int64_t pitch, int32_t mode,
                         float x, float y, float sigma, void *out, int64_t out_pitch,
                         int32_t *count) {
    if (!field || !out) return pp::fail(PP_EINVAL, "pp_center_filter_cpu: NULL argument");
    if (mode < 0 || mode > 3) return pp::fail(PP_EINVAL, "pp_center_filter_cpu: bad mode");
    if (rows < (mode >= 2 ? 4 : 3) || n < 0 || pitch < n)
        return pp::fail(PP_ESHAPE, "pp_center_filter_cpu: bad field shape");
    int64_t k = 0;
    for (int64_t i = 0; i < n; i++) {
        const bool take = pp::center_take(field, pitch, i, mode, x, y, sigma);
        if (mode == 3) {
            ((uint8_t *)out)[i] = take ? 1 : 0;
            continue;
        }
        if (!take) continue;
        for (int64_t r = 0; r < rows; r++) ((float *)out)[r * out_pitch + k] = field[r * pitch + i];
        k++;
    }
    if (count) *count = (int32_t)(mode == 3 ? n : k);
    return PP_OK;
}

}  // extern "C"
