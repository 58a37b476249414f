// functional.hip — the remaining openpifpaf.functional primitives on gfx950:
// point lookups (functional.pyx:231-286), the order-preserving column filters
// caf_center_s / paf_center / paf_center_b / paf_mask_center (functional.pyx:214-228,
// 289-359) and weiszfeld_nd (functional.pyx:172-211).  None of these is on the timed
// decoder path in v0.11.6 except through the batched kernels; they exist so the
// `functional` API is complete and bit-exact on device data.
#include "pp_common.hpp"

namespace pp {

__global__ __launch_bounds__(256) void scalar_values_kernel(const float *__restrict__ f, int h,
                                                            int w, int64_t pitch,
                                                            const float *__restrict__ x,
                                                            const float *__restrict__ y, int64_t n,
                                                            float dflt, float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out[i] = hr_lookup(f, h, w, pitch, x[i], y[i], dflt);
}

// mode: 0 scalar_value, 1 scalar_value_clipped, 2 scalar_nonzero, 3 scalar_nonzero_clipped,
//       4 scalar_nonzero_clipped_with_reduction (lookup_at, pp_common.hpp)
__global__ __launch_bounds__(256) void scalar_lookup_kernel(const void *field, int h, int w,
                                                            int64_t pitch, int mode,
                                                            const float *__restrict__ xs,
                                                            const float *__restrict__ ys,
                                                            int64_t n, float dflt, float r,
                                                            void *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    lookup_at(field, h, w, pitch, mode, xs[i], ys[i], dflt, r, out, i);
}

// one workgroup, 1024 threads: order-preserving compaction of the kept columns
__global__ __launch_bounds__(1024) void center_filter_kernel(const float *__restrict__ f, int rows,
                                                             int64_t n, int64_t pitch, int mode,
                                                             float x, float y, float sigma,
                                                             void *out, int64_t out_pitch,
                                                             int *count) {
    __shared__ int s_tmp[16];
    int64_t running = 0;
    for (int64_t base = 0; base < n; base += 1024) {
        const int64_t i = base + threadIdx.x;
        bool take = false;
        if (i < n) {
            take = center_take(f, pitch, i, mode, x, y, sigma);
            if (mode == 3) ((uint8_t *)out)[i] = take ? 1 : 0;
        }
        int total;
        const int slot = block_compact<16>(take, s_tmp, total);
        if (mode != 3 && take) {
            float *o = (float *)out;
            for (int r = 0; r < rows; r++) o[r * out_pitch + running + slot] = f[r * pitch + i];
        }
        running += total;
    }
    if (threadIdx.x == 0 && count) *count = (int)(mode == 3 ? n : running);
}

// the decoder's CAF-score exp (caf_exp; mode 2: its sigma**2, np_pow2_f32) over an array
__global__ void np_exp_kernel(const float *__restrict__ x, float *__restrict__ y, int64_t n,
                              int mode) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = mode == 2 ? np_pow2_f32(x[i]) : caf_exp(x[i], mode);
}

// functional.pyx:172-211, sequential sums in the reference's order (one lane)
__global__ void weiszfeld_kernel(const float *__restrict__ x, int64_t n, int64_t d, int64_t xp,
                                 float *y, const float *__restrict__ wts, float eps,
                                 int64_t max_steps, float *denom) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    weiszfeld_run(x, n, xp, y, wts, eps, max_steps, denom);
}

}  // namespace pp

using namespace pp;

// Occupancy.set (occupancy.py:36-44) + scalar_square_add_single (decoder/utils.py:61-66),
// marks applied in order by one workgroup: lanes cover one mark's box, a barrier between
// marks.  u8 += 1 wraps as NumPy's in-place add.
__global__ __launch_bounds__(256) void occupancy_set_kernel(uint8_t *occ, int n_planes, int64_t h,
                                                            int64_t w, int64_t pitch,
                                                            const int *fs, const float *xs,
                                                            const float *ys, const float *sig,
                                                            int64_t n, float r, float msr) {
    for (int64_t i = 0; i < n; i++) {
        int64_t x0, x1, y0, y1;
        if (occupancy_mark_box(fs[i], n_planes, h, w, xs[i], ys[i], sig[i], r, msr, x0, x1, y0, y1)) {
            const int64_t bw = x1 - x0, cells = bw * (y1 - y0);
            uint8_t *plane = occ + (int64_t)fs[i] * h * pitch;
            for (int64_t c = threadIdx.x; c < cells; c += 256) {
                uint8_t *p = plane + (y0 + c / bw) * pitch + x0 + c % bw;
                *p = (uint8_t)(*p + 1);
            }
        }
        __syncthreads();
    }
}

extern "C" {

int pp_occupancy_set(uint8_t *d_occ, int32_t n_planes, int64_t h, int64_t w, int64_t pitch,
                     const int32_t *d_f, const float *d_x, const float *d_y, const float *d_sigma,
                     int64_t n, float reduction, float min_scale_reduced, void *stream) {
    if (!d_occ || (n > 0 && (!d_f || !d_x || !d_y || !d_sigma)))
        return fail(PP_EINVAL, "pp_occupancy_set: NULL argument");
    if (n_planes < 0 || h < 0 || w < 0 || pitch < w || n < 0 || !(reduction > 0.0f))
        return fail(PP_ESHAPE, "pp_occupancy_set: bad shape");
    if (n == 0 || h == 0 || w == 0) return PP_OK;
    hipLaunchKernelGGL(occupancy_set_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, d_occ,
                       n_planes, h, w, pitch, d_f, d_x, d_y, d_sigma, n, reduction,
                       min_scale_reduced);
    return check_launch("pp_occupancy_set");
}

int pp_scalar_values(const float *d_field, int64_t h, int64_t w, int64_t pitch, const float *d_x,
                     const float *d_y, int64_t n, float default_value, float *d_out, void *stream) {
    if (!d_field || (n > 0 && (!d_x || !d_y || !d_out))) return fail(PP_EINVAL, "pp_scalar_values: NULL argument");
    if (h < 0 || w < 0 || pitch < w) return fail(PP_ESHAPE, "pp_scalar_values: bad field shape");
    if (n <= 0) return PP_OK;
    hipLaunchKernelGGL(scalar_values_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_field, (int)h, (int)w, pitch, d_x, d_y, n,
                       default_value, d_out);
    return check_launch("pp_scalar_values");
}

int pp_scalar_lookup(const void *d_field, int64_t h, int64_t w, int64_t pitch, int32_t mode,
                     const float *d_x, const float *d_y, int64_t n, float default_value,
                     float reduction, void *d_out, void *stream) {
    if (!d_field || (n > 0 && (!d_x || !d_y || !d_out))) return fail(PP_EINVAL, "pp_scalar_lookup: NULL argument");
    if (mode < 0 || mode > 4) return fail(PP_EINVAL, "pp_scalar_lookup: bad mode");
    if (h <= 0 || w <= 0 || pitch < w) return fail(PP_ESHAPE, "pp_scalar_lookup: bad field shape");
    if (n <= 0) return PP_OK;
    hipLaunchKernelGGL(scalar_lookup_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_field, (int)h, (int)w, pitch, mode, d_x, d_y, n,
                       default_value, reduction, d_out);
    return check_launch("pp_scalar_lookup");
}

int pp_center_filter(const float *d_field, int64_t rows, int64_t n, int64_t pitch, int32_t mode,
                     float x, float y, float sigma, void *d_out, int64_t out_pitch,
                     int32_t *d_count, void *stream) {
    if (!d_field || !d_out) return fail(PP_EINVAL, "pp_center_filter: NULL argument");
    if (mode < 0 || mode > 3) return fail(PP_EINVAL, "pp_center_filter: bad mode");
    if (rows < (mode >= 2 ? 4 : 3) || n < 0 || pitch < n)
        return fail(PP_ESHAPE, "pp_center_filter: bad field shape");
    hipLaunchKernelGGL(center_filter_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_field,
                       (int)rows, n, pitch, mode, x, y, sigma, d_out, out_pitch, d_count);
    return check_launch("pp_center_filter");
}

int pp_np_exp(const float *d_x, float *d_y, int64_t n, int32_t exp_mode, void *stream) {
    if (!d_x || !d_y) return fail(PP_EINVAL, "pp_np_exp: NULL argument");
    if (n < 0 || n > ((int64_t)1 << 38)) return fail(PP_ESHAPE, "pp_np_exp: bad length");
    if (exp_mode != 0 && exp_mode != 1) return fail(PP_EINVAL, "pp_np_exp: bad exp_mode");
    if (n == 0) return PP_OK;
    hipLaunchKernelGGL(np_exp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_x, d_y, n, exp_mode);
    return check_launch("pp_np_exp");
}

int pp_np_square(const float *d_x, float *d_y, int64_t n, void *stream) {
    if (!d_x || !d_y) return fail(PP_EINVAL, "pp_np_square: NULL argument");
    if (n < 0 || n > ((int64_t)1 << 38)) return fail(PP_ESHAPE, "pp_np_square: bad length");
    if (n == 0) return PP_OK;
    hipLaunchKernelGGL(np_exp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_x, d_y, n, 2);
    return check_launch("pp_np_square");
}

int pp_weiszfeld_nd(const float *d_x, int64_t n, int64_t d, int64_t x_pitch, float *d_y,
                    const float *d_weights, float epsilon, int64_t max_steps, float *d_denom,
                    void *stream) {
    if (!d_x || !d_y || !d_weights || !d_denom) return fail(PP_EINVAL, "pp_weiszfeld_nd: NULL argument");
    if (n < 0 || d < 2 || x_pitch < d) return fail(PP_ESHAPE, "pp_weiszfeld_nd: bad shape");
    hipLaunchKernelGGL(weiszfeld_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_x, n, d,
                       x_pitch, d_y, d_weights, epsilon, max_steps, d_denom);
    return check_launch("pp_weiszfeld_nd");
}

}  // extern "C"
