/*
 * pp_oracle.c — CPU restatement of the openpifpaf v0.11.6 CIF/CAF decoder hot path.
 *
 * TEST INFRASTRUCTURE.  This is the parity checker, not the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it (through
 * oracle/oracle.py).  The product (openpifpaf_amd + libpifpaf_amd.so) never links or
 * calls it.
 *
 * Parity pinned: tests/golden/ holds vectors produced by the reference itself (the
 * Cython functional.pyx compiled by oracle/build_ref.sh + the reference's Python decoder,
 * see tests/golden/gen_golden.py); tests/test_oracle_golden.py checks this file against
 * them.
 *
 * Arithmetic follows the reference operation by operation:
 *   - functional.pyx is compiled C: float ops, with the double temporaries Cython emits
 *     (e.g. functional.c `-0.5 * (dx2 + dy2) / (double)csigma2`, `1.0 + (double)x / 8.0`,
 *     clip() through fmax/fmin on doubles).  Built with -ffp-contract=off.
 *   - the Python decoder runs NumPy float32 arithmetic; under NumPy 2 (NEP 50) Python
 *     float scalars are cast to float32, so each expression below is one f32 op per
 *     NumPy op, in the reference's evaluation order.
 *   - np.exp(float32): NumPy's SIMD float32 exp (np_exp_f32 below, the AVX2 / AVX512F
 *     routine NumPy dispatches to on any x86-64 with FMA3, which is what produced the
 *     fixtures: tests/golden/meta.json records AVX512_SKX), bit-exact against np.exp over
 *     every float32 in [-104, 0] (tests/test_np_exp.py); pp_config.exp_mode 1 selects a
 *     correctly rounded exp instead (NumPy's scalar path on CPUs without FMA3).
 *   - `sigma**2` of a float32 scalar is the C library's powf(sigma, 2) (np_scalar_square),
 *     as NumPy's scalar power computes it.  With both, every decode fixture matches the
 *     reference bit for bit.
 *   - Annotation.score(): float64, NumPy pairwise summation replicated (pw_sum below).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pifpaf_amd.h"

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------ */
/* functional.pyx primitives                                                        */
/* ------------------------------------------------------------------------------ */

/* functional.pyx:67-68  clip() = fmax(minv, fmin(maxv, v)) on doubles, float result */
static inline float clip_ref(float v, float minv, float maxv) {
    return (float)fmax((double)minv, fmin((double)maxv, (double)v));
}

/* functional.pyx:57-64  (functional.c: x = 1.0 + (double)x / 8.0) */
static inline float approx_exp_ref(float x) {
    if (x > 2.0 || x < -2.0) return 0.0f;
    x = (float)(1.0 + ((double)x) / 8.0);
    x *= x;
    x *= x;
    x *= x;
    return x;
}

#define AT(f, yy, xx, sh, sw) ((f)[(yy) * (sh) + (xx) * (sw)])

/* functional.pyx:7-26 */
EXPORT void orc_scalar_square_add_constant(float *field, long h, long w, long sh, long sw,
                                           const float *x, const float *y, const float *width,
                                           const float *v, long n) {
    for (long i = 0; i < n; i++) {
        float cx = x[i], cy = y[i], cv = v[i], cwidth = width[i];
        long minx = (long)clip_ref(cx - cwidth, 0.0f, (float)(w - 1));
        long maxx = (long)clip_ref(cx + cwidth, (float)(minx + 1), (float)w);
        long miny = (long)clip_ref(cy - cwidth, 0.0f, (float)(h - 1));
        long maxy = (long)clip_ref(cy + cwidth, (float)(miny + 1), (float)h);
        for (long xx = minx; xx < maxx; xx++)
            for (long yy = miny; yy < maxy; yy++) AT(field, yy, xx, sh, sw) += cv;
    }
}

/* functional.pyx:29-54 (cdivision) */
EXPORT void orc_cumulative_average(float *cuma, float *cumw, long h, long w, long sh, long sw,
                                   const float *x, const float *y, const float *width,
                                   const float *v, const float *wt, long n) {
    for (long i = 0; i < n; i++) {
        float cw = wt[i];
        if (cw <= 0.0f) continue;
        float cv = v[i], cx = x[i], cy = y[i], cwidth = width[i];
        long minx = (long)clip_ref(cx - cwidth, 0.0f, (float)(w - 1));
        long maxx = (long)clip_ref(cx + cwidth, (float)(minx + 1), (float)w);
        long miny = (long)clip_ref(cy - cwidth, 0.0f, (float)(h - 1));
        long maxy = (long)clip_ref(cy + cwidth, (float)(miny + 1), (float)h);
        for (long xx = minx; xx < maxx; xx++)
            for (long yy = miny; yy < maxy; yy++) {
                float *a = &AT(cuma, yy, xx, sh, sw);
                float *b = &AT(cumw, yy, xx, sh, sw);
                *a = (cw * cv + *b * *a) / (*b + cw);
                *b += cw;
            }
    }
}

/* functional.pyx:71-102 (no +1 on the box, no circle test, no clamp) */
EXPORT void orc_scalar_square_add_gauss(float *field, long h, long w, long sh, long sw,
                                        const float *x, const float *y, const float *sigma,
                                        const float *v, long n, float truncate) {
    for (long i = 0; i < n; i++) {
        float csigma = sigma[i];
        float csigma2 = csigma * csigma;
        float cx = x[i], cy = y[i], cv = v[i];
        long minx = (long)clip_ref(cx - truncate * csigma, 0.0f, (float)(w - 1));
        long maxx = (long)clip_ref(cx + truncate * csigma, (float)(minx + 1), (float)w);
        long miny = (long)clip_ref(cy - truncate * csigma, 0.0f, (float)(h - 1));
        long maxy = (long)clip_ref(cy + truncate * csigma, (float)(miny + 1), (float)h);
        for (long xx = minx; xx < maxx; xx++) {
            float dx = (float)xx - cx;
            float deltax2 = dx * dx; /* powf(d, 2.0) == d*d */
            for (long yy = miny; yy < maxy; yy++) {
                float dy = (float)yy - cy;
                float deltay2 = dy * dy;
                float vv;
                if (deltax2 < 0.25 && deltay2 < 0.25)
                    vv = cv;
                else
                    vv = cv * approx_exp_ref(
                                  (float)((-0.5 * (double)(deltax2 + deltay2)) / (double)csigma2));
                AT(field, yy, xx, sh, sw) += vv;
            }
        }
    }
}

/* functional.pyx:105-141 — the CifHr splat */
EXPORT void orc_scalar_square_add_gauss_with_max(float *field, long h, long w, long sh, long sw,
                                                 const float *x, const float *y,
                                                 const float *sigma, const float *v, long n,
                                                 float truncate, float max_value) {
    float truncate2 = truncate * truncate;
    for (long i = 0; i < n; i++) {
        float csigma = sigma[i];
        float csigma2 = csigma * csigma;
        float cx = x[i], cy = y[i], cv = v[i];
        long minx = (long)clip_ref(cx - truncate * csigma, 0.0f, (float)(w - 1));
        long maxx = (long)clip_ref((float)((double)(cx + truncate * csigma) + 1.0),
                                   (float)(minx + 1), (float)w);
        long miny = (long)clip_ref(cy - truncate * csigma, 0.0f, (float)(h - 1));
        long maxy = (long)clip_ref((float)((double)(cy + truncate * csigma) + 1.0),
                                   (float)(miny + 1), (float)h);
        for (long xx = minx; xx < maxx; xx++) {
            float dx = (float)xx - cx;
            float deltax2 = dx * dx;
            for (long yy = miny; yy < maxy; yy++) {
                float dy = (float)yy - cy;
                float deltay2 = dy * dy;
                if (deltax2 + deltay2 > truncate2 * csigma2) continue;
                float vv;
                if (deltax2 < 0.25 && deltay2 < 0.25)
                    vv = cv;
                else
                    vv = cv * approx_exp_ref(
                                  (float)((-0.5 * (double)(deltax2 + deltay2)) / (double)csigma2));
                float *f = &AT(field, yy, xx, sh, sw);
                *f += vv;
                *f = (*f < max_value) ? *f : max_value; /* min(max_value, f) as emitted */
            }
        }
    }
}

/* functional.pyx:144-169 */
EXPORT void orc_scalar_square_max_gauss(float *field, long h, long w, long sh, long sw,
                                        const float *x, const float *y, const float *sigma,
                                        const float *v, long n, float truncate) {
    for (long i = 0; i < n; i++) {
        float csigma = sigma[i];
        float csigma2 = csigma * csigma;
        float cx = x[i], cy = y[i], cv = v[i];
        long minx = (long)clip_ref(cx - truncate * csigma, 0.0f, (float)(w - 1));
        long maxx = (long)clip_ref(cx + truncate * csigma, (float)(minx + 1), (float)w);
        long miny = (long)clip_ref(cy - truncate * csigma, 0.0f, (float)(h - 1));
        long maxy = (long)clip_ref(cy + truncate * csigma, (float)(miny + 1), (float)h);
        for (long xx = minx; xx < maxx; xx++) {
            float dx = (float)xx - cx;
            float deltax2 = dx * dx;
            for (long yy = miny; yy < maxy; yy++) {
                float dy = (float)yy - cy;
                float deltay2 = dy * dy;
                float vv = cv * approx_exp_ref(
                                    (float)((-0.5 * (double)(deltax2 + deltay2)) / (double)csigma2));
                float *f = &AT(field, yy, xx, sh, sw);
                *f = (float)fmax((double)*f, (double)vv);
            }
        }
    }
}

/* functional.pyx:172-211.  Returns the number of steps run. */
EXPORT long orc_weiszfeld_nd(const float *x, long n, long d, long xs0, long xs1, float *y,
                             const float *weights, float epsilon, long max_steps, float *denom) {
    float *wx = (float *)calloc((size_t)(n * d > 0 ? n * d : 1), sizeof(float));
    for (long i = 0; i < n; i++)
        for (long j = 0; j < d; j++) wx[i * d + j] = weights[i] * x[i * xs0 + j * xs1];
    float prev[2], top[2];
    long s;
    for (s = 0; s < max_steps; s++) {
        prev[0] = y[0];
        prev[1] = y[1];
        for (long i = 0; i < n; i++) {
            float ax = x[i * xs0] - prev[0];
            float ay = x[i * xs0 + xs1] - prev[1];
            denom[i] = (float)(sqrt((double)(ax * ax + ay * ay)) + (double)epsilon);
        }
        top[0] = 0.0f;
        top[1] = 0.0f;
        float bottom = 0.0f;
        for (long j = 0; j < n; j++) {
            top[0] += wx[j * d + 0] / denom[j];
            top[1] += wx[j * d + 1] / denom[j];
            bottom = bottom + weights[j] / denom[j];
        }
        y[0] = top[0] / bottom;
        y[1] = top[1] / bottom;
        if (fabs((double)(y[0] - prev[0])) + fabs((double)(y[1] - prev[1])) < 1e-2) {
            s++;
            break;
        }
    }
    free(wx);
    return s;
}

/* functional.pyx:231-244 */
EXPORT void orc_scalar_values(const float *field, long h, long w, long sh, long sw, const float *x,
                              const float *y, long n, float dflt, float *out) {
    float maxx = (float)w - 1, maxy = (float)h - 1;
    for (long i = 0; i < n; i++) {
        out[i] = dflt;
        if (x[i] < 0.0 || y[i] < 0.0 || x[i] > maxx || y[i] > maxy) continue;
        out[i] = AT(field, (long)y[i], (long)x[i], sh, sw);
    }
}

/* functional.pyx:247-286; mode as pp_scalar_lookup */
EXPORT void orc_scalar_lookup(const void *field, long h, long w, long sh, long sw, int mode,
                              const float *xs, const float *ys, long n, float dflt, float r,
                              void *out) {
    for (long i = 0; i < n; i++) {
        float x = xs[i], y = ys[i];
        if (mode == 0) {
            const float *f = (const float *)field;
            float res = dflt;
            if (!(x < 0.0 || y < 0.0 || x > w - 1 || y > h - 1)) res = AT(f, (long)y, (long)x, sh, sw);
            ((float *)out)[i] = res;
        } else if (mode == 1) {
            const float *f = (const float *)field;
            x = clip_ref(x, 0.0f, (float)(w - 1));
            y = clip_ref(y, 0.0f, (float)(h - 1));
            ((float *)out)[i] = AT(f, (long)y, (long)x, sh, sw);
        } else {
            const uint8_t *f = (const uint8_t *)field;
            uint8_t res;
            if (mode == 2) {
                res = (uint8_t)dflt;
                if (!(x < 0.0 || y < 0.0 || x > w - 1 || y > h - 1)) res = AT(f, (long)y, (long)x, sh, sw);
            } else if (mode == 3) {
                x = clip_ref(x, 0.0f, (float)(w - 1));
                y = clip_ref(y, 0.0f, (float)(h - 1));
                res = AT(f, (long)y, (long)x, sh, sw);
            } else {
                x = clip_ref(x / r, 0.0f, (float)(w - 1));
                y = clip_ref(y / r, 0.0f, (float)(h - 1));
                res = AT(f, (long)y, (long)x, sh, sw);
            }
            ((uint8_t *)out)[i] = res;
        }
    }
}

/* functional.pyx:214-228 (mode 3), 289-310 (2), 313-335 (1), 338-359 (0).
 * field (rows, n) with strides (s0, s1); out (rows, n) contiguous; returns kept count. */
EXPORT long orc_center_filter(const float *f, long rows, long n, long s0, long s1, int mode,
                              float x, float y, float sigma, void *out) {
    long k = 0;
    for (long i = 0; i < n; i++) {
        float r1 = f[1 * s0 + i * s1], r2 = f[2 * s0 + i * s1];
        int take;
        if (mode == 0 || mode == 1) {
            take = !(r1 < x - sigma) && !(r1 > x + sigma) && !(r2 < y - sigma) && !(r2 > y + sigma);
        } else {
            float r3 = f[3 * s0 + i * s1];
            take = r1 > x - sigma * r3 && r1 < x + sigma * r3 && r2 > y - sigma * r3 &&
                   r2 < y + sigma * r3;
        }
        if (mode == 3) {
            ((uint8_t *)out)[i] = (uint8_t)take;
            continue;
        }
        if (!take) continue;
        for (long r = 0; r < rows; r++) ((float *)out)[r * n + k] = f[r * s0 + i * s1];
        k++;
    }
    return mode == 3 ? n : k;
}

/* ------------------------------------------------------------------------------ */
/* decoder stages                                                                   */
/* ------------------------------------------------------------------------------ */

static inline long hr_dim(long n, int stride) { return (n - 1) * stride + 1; }

/* cif_hr.py:26-40, 42-65, 67-81 — out (K, H', W') contiguous, zero-initialised here */
EXPORT void orc_cifhr(const float *cif, int K, int H, int W, const pp_config *cfg, float *out) {
    long hh = hr_dim(H, cfg->stride), ww = hr_dim(W, cfg->stride);
    long hw = (long)H * W;
    float *xs = (float *)malloc(sizeof(float) * 4 * (size_t)hw);
    float *ys = xs + hw, *ss = ys + hw, *vs = ss + hw;
    memset(out, 0, sizeof(float) * (size_t)K * hh * ww);
    float stride = (float)cfg->stride;
    for (int f = 0; f < K; f++) {
        const float *p = cif + (size_t)f * 5 * hw;
        long n = 0;
        for (long c = 0; c < hw; c++) {
            if (!(p[c] > cfg->cif_threshold)) continue; /* p[:, p[0] > v_threshold] */
            xs[n] = p[1 * hw + c] * stride;
            ys[n] = p[2 * hw + c] * stride;
            float sg = (0.5f * p[4 * hw + c]) * stride;
            ss[n] = fmaxf(1.0f, sg); /* np.maximum(1.0, 0.5*scale*stride) */
            if (sg != sg) ss[n] = sg; /* np.maximum propagates NaN */
            vs[n] = (p[c] / (float)cfg->cif_neighbors) / 1.0f; /* v / neighbors / len_cifs */
            n++;
        }
        orc_scalar_square_add_gauss_with_max(out + (size_t)f * hh * ww, hh, ww, ww, 1, xs, ys, ss,
                                             vs, n, 1.0f, 1.0f);
    }
    free(xs);
}

static int seed_cmp_desc(const void *pa, const void *pb) {
    /* sorted(seeds, reverse=True) on (v, f, x, y, s); stable -> emission index ascending */
    const float *a = (const float *)pa, *b = (const float *)pb; /* v f x y s idx */
    for (int i = 0; i < 5; i++) {
        if (a[i] == b[i]) continue;
        return (a[i] > b[i]) ? -1 : 1;
    }
    return (a[5] < b[5]) ? -1 : (a[5] > b[5]);
}

/* cif_seeds.py:23-64.  hr (K, H', pitch).  Returns the number of seeds (all written if
 * <= cap). */
EXPORT long orc_seeds(const float *cif, const float *hr, long hr_pitch, int K, int H, int W,
                      const pp_config *cfg, pp_seed *out, long cap) {
    long hh = hr_dim(H, cfg->stride), ww = hr_dim(W, cfg->stride);
    long hw = (long)H * W;
    float stride = (float)cfg->stride;
    float *tmp = (float *)malloc(sizeof(float) * 6 * (size_t)(K * hw + 1));
    long n = 0;
    for (int f = 0; f < K; f++) {
        if ((cfg->seed_skip_mask >> f) & 1u) continue; /* cif_seeds.py:28-29 seed_mask */
        const float *p = cif + (size_t)f * 5 * hw;
        const float *t = hr + (size_t)f * hh * hr_pitch;
        for (long c = 0; c < hw; c++) {
            float conf = p[c];
            if (!(conf > cfg->seed_threshold)) continue;
            float x = p[1 * hw + c] * stride, y = p[2 * hw + c] * stride;
            float v;
            orc_scalar_values(t, hh, ww, hr_pitch, 1, &x, &y, 1, 0.0f, &v);
            v = 0.9f * v + 0.1f * conf;
            if (cfg->seed_score_scale != 1.0f) v = v * cfg->seed_score_scale;
            if (!(v > cfg->seed_threshold)) continue;
            float *r = tmp + 6 * n;
            r[0] = v;
            r[1] = (float)f;
            r[2] = x;
            r[3] = y;
            r[4] = p[4 * hw + c] * stride;
            r[5] = (float)n;
            n++;
        }
    }
    qsort(tmp, (size_t)n, sizeof(float) * 6, seed_cmp_desc);
    for (long i = 0; i < n && i < cap; i++) {
        float *r = tmp + 6 * i;
        out[i].v = r[0];
        out[i].field = (int32_t)r[1];
        out[i].x = r[2];
        out[i].y = r[3];
        out[i].s = r[4];
    }
    free(tmp);
    return n;
}

/* caf_scored.py:32-98.  cols (C, 2, 9, H*W): dir 0 backward, 1 forward; counts (C, 2). */
EXPORT void orc_caf_scored(const float *caf, const float *hr, long hr_pitch, int K, int C, int H,
                           int W, const int32_t *skel, float score_th, const pp_config *cfg,
                           float *cols, int32_t *counts) {
    long hh = hr_dim(H, cfg->stride), ww = hr_dim(W, cfg->stride);
    long hw = (long)H * W;
    float stride = (float)cfg->stride;
    float floor_ = cfg->cif_floor;
    float one_minus = (float)(1.0 - (double)cfg->cif_floor);
    for (int i = 0; i < C; i++) {
        const float *p = caf + (size_t)i * 9 * hw;
        float *bwd = cols + ((size_t)i * 2 + 0) * 9 * hw;
        float *fwd = cols + ((size_t)i * 2 + 1) * 9 * hw;
        int j1i = skel[2 * i] - 1, j2i = skel[2 * i + 1] - 1;
        long nb = 0, nf = 0;
        for (long c = 0; c < hw; c++) {
            float nine[9];
            nine[0] = p[c];
            if (!(nine[0] > score_th)) continue;
            for (int r = 1; r < 9; r++) nine[r] = p[r * hw + c] * stride;
            float score = nine[0];
            float sb = score, sf = score;
            if (floor_ < 1.0f && j1i < K) {
                float h1;
                orc_scalar_values(hr + (size_t)j1i * hh * hr_pitch, hh, ww, hr_pitch, 1, &nine[1],
                                  &nine[2], 1, 0.0f, &h1);
                sb = score * (floor_ + one_minus * h1);
            }
            if (sb > score_th) {
                static const int order_b[9] = {0, 5, 6, 7, 8, 1, 2, 3, 4};
                for (int r = 0; r < 9; r++) bwd[r * hw + nb] = nine[order_b[r]];
                bwd[nb] = sb;
                nb++;
            }
            if (floor_ < 1.0f && j2i < K) {
                float h2;
                orc_scalar_values(hr + (size_t)j2i * hh * hr_pitch, hh, ww, hr_pitch, 1, &nine[5],
                                  &nine[6], 1, 0.0f, &h2);
                sf = score * (floor_ + one_minus * h2);
            }
            if (sf > score_th) {
                for (int r = 0; r < 9; r++) fwd[r * hw + nf] = nine[r];
                fwd[nf] = sf;
                nf++;
            }
        }
        counts[2 * i + 0] = (int32_t)nb;
        counts[2 * i + 1] = (int32_t)nf;
    }
}

/* ------------------------------------------------------------------------------ */
/* CifCaf greedy decoder (generator/cifcaf.py)                                       */
/* ------------------------------------------------------------------------------ */

typedef struct {
    int n;
    int k[PP_MAX_EDGES * 2];
    int caf[PP_MAX_EDGES * 2];
    int fwd[PP_MAX_EDGES * 2];
} by_source_t;

typedef struct {
    int K, C, H, W;
    long hw;
    const pp_config *cfg;
    by_source_t bs[PP_MAX_KP];
    /* CafScored column sets: cols (C, 2, 9, hw), counts (C, 2) */
    const float *cols;
    const int32_t *counts;
} dec_t;

/* cifcaf.py:62-65 — defaultdict(dict) with insertion order, later keys overwrite values */
static void build_by_source(dec_t *d, const int32_t *skel) {
    memset(d->bs, 0, sizeof(d->bs));
    for (int ci = 0; ci < d->C; ci++) {
        int j1 = skel[2 * ci] - 1, j2 = skel[2 * ci + 1] - 1;
        int ins[2][3] = {{j1, j2, 1}, {j2, j1, 0}};
        for (int t = 0; t < 2; t++) {
            by_source_t *b = &d->bs[ins[t][0]];
            int pos = -1;
            for (int e = 0; e < b->n; e++)
                if (b->k[e] == ins[t][1]) pos = e;
            if (pos < 0) pos = b->n++;
            b->k[pos] = ins[t][1];
            b->caf[pos] = ci;
            b->fwd[pos] = ins[t][2];
        }
    }
}

static int by_source_find(const dec_t *d, int j, int k) {
    const by_source_t *b = &d->bs[j];
    for (int e = 0; e < b->n; e++)
        if (b->k[e] == k) return e;
    return -1;
}

/* NumPy 2.2's float32 exp for x86 SIMD (numpy/_core/src/umath/
 * loops_exponent_log.dispatch.c.src, simd_exp_f32 for FMA3 / AVX512F, with the constants of
 * npy_simd_data.h): x * log2(e) rounded to an integer quadrant by the 1.5 * 2^23 trick,
 * Cody-Waite reduction r = x + q * (-ln2 hi) + q * (-ln2 lo) (fused), the rational
 * approximation p5..p0 / q2..q0 in Horner form with fused multiply-adds, one correctly
 * rounded division, times 2^q (scalef / ldexp: exact, or correctly rounded to a subnormal).
 * x >= 88.72283935546875 -> inf, x <= -103.97208404541015625 -> 0, NaN -> NaN. */
static float np_exp_f32(float x) {
    if (x != x) return x;
    if (x >= 88.72283935546875f) return INFINITY;
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
    return ldexpf(num / den, (int)q);
}

/* exported for tests/test_np_exp.py (exhaustive check against np.exp) */
EXPORT void orc_np_exp(const float *x, float *y, long n) {
    for (long i = 0; i < n; i++) y[i] = np_exp_f32(x[i]);
}

/* `sigma**2` of a NumPy float32 scalar (cifcaf.py:139): NumPy's scalar power calls the C
 * library's powf (numpy/_core/src/umath/scalarmath.c.src, npy_powf), glibc 2.35's here,
 * which is not always x * x.  Called through a volatile pointer: the compiler would
 * otherwise fold powf(x, 2) into x * x. */
static float np_scalar_square(float x) {
    float (*volatile powf_p)(float, float) = powf;
    return powf_p(x, 2.0f);
}

/* exported for tests/test_np_exp.py */
EXPORT void orc_np_square(const float *x, float *y, long n) {
    float (*volatile powf_p)(float, float) = powf;
    for (long i = 0; i < n; i++) y[i] = powf_p(x[i], 2.0f);
}

/* np.exp of the decoder's scores (cifcaf.py:139) under pp_config.exp_mode */
static inline float exp_cr(float q, int mode) {
    return mode ? (float)exp((double)q) : np_exp_f32(q);
}

/* cifcaf.py:124-192: _grow_connection + _target_with_blend / _target_with_maxscore.
 * caf_field = (9, n) column set with row stride hw.  Returns x, y, s, score. */
static void grow_connection(const dec_t *d, float x, float y, float xy_scale, const float *cf,
                            long n, float out[4]) {
    long hw = d->hw;
    float sigma_box = 2.0f * xy_scale;
    float lo_x = x - sigma_box, hi_x = x + sigma_box, lo_y = y - sigma_box, hi_y = y + sigma_box;
    float sigma = 0.5f * xy_scale;
    float sigma2 = np_scalar_square(sigma);
    long m = 0, i1 = -1, i2 = -1;
    float s1 = 0.0f, s2 = 0.0f;
    int method_max = d->cfg->connection_method == 1;
    for (long i = 0; i < n; i++) {
        float c1 = cf[1 * hw + i], c2 = cf[2 * hw + i];
        if (c1 < lo_x || c1 > hi_x || c2 < lo_y || c2 > hi_y) continue; /* caf_center_s */
        float dx = x - c1, dy = y - c2;
        float dd = sqrtf(dx * dx + dy * dy);
        float score = exp_cr((-0.5f * (dd * dd)) / sigma2, d->cfg->exp_mode) * cf[i];
        m++;
        if (method_max) {
            if (i1 < 0 || score > s1) { /* np.argmax: first maximum */
                i1 = i;
                s1 = score;
            }
            continue;
        }
        /* top-2 of a stable ascending argsort: ties -> higher column index ranks higher */
        if (i1 < 0 || score >= s1) {
            i2 = i1;
            s2 = s1;
            i1 = i;
            s1 = score;
        } else if (i2 < 0 || score >= s2) {
            i2 = i;
            s2 = score;
        }
    }
    if (m == 0) {
        out[0] = out[1] = out[2] = out[3] = 0.0f;
        return;
    }
    const float *t0 = cf + 5 * hw, *t1 = cf + 6 * hw, *t3 = cf + 8 * hw;
    if (method_max) {
        out[0] = t0[i1];
        out[1] = t1[i1];
        out[2] = t3[i1];
        out[3] = s1;
        return;
    }
    if (m == 1) {
        out[0] = t0[i1];
        out[1] = t1[i1];
        out[2] = t3[i1];
        out[3] = s1 * 0.5f;
        return;
    }
    if (s2 < 0.01f || s2 < 0.5f * s1) {
        out[0] = t0[i1];
        out[1] = t1[i1];
        out[2] = t3[i1];
        out[3] = s1 * 0.5f;
        return;
    }
    float ex = t0[i1] - t0[i2], ey = t1[i1] - t1[i2];
    float dist = sqrtf(ex * ex + ey * ey);
    if (dist > t3[i1] / 2.0f) {
        out[0] = t0[i1];
        out[1] = t1[i1];
        out[2] = t3[i1];
        out[3] = s1 * 0.5f;
        return;
    }
    float ssum = s1 + s2;
    out[0] = (s1 * t0[i1] + s2 * t0[i2]) / ssum;
    out[1] = (s1 * t1[i1] + s2 * t1[i2]) / ssum;
    out[2] = (s1 * t3[i1] + s2 * t3[i2]) / ssum;
    out[3] = 0.5f * (s1 + s2);
}

static inline float max0(float v) { return (v > 0.0f) ? v : 0.0f; } /* max(0.0, v) */

/* cifcaf.py:194-217 */
static void connection_value(const dec_t *d, const pp_ann *a, int start_i, int end_i,
                             int reverse_match, float out[4]) {
    int e = by_source_find(d, start_i, end_i);
    int caf_i = d->bs[start_i].caf[e], forward = d->bs[start_i].fwd[e];
    long hw = d->hw;
    const float *cols_f = d->cols + ((size_t)caf_i * 2 + (forward ? 1 : 0)) * 9 * hw;
    const float *cols_b = d->cols + ((size_t)caf_i * 2 + (forward ? 0 : 1)) * 9 * hw;
    long n_f = d->counts[2 * caf_i + (forward ? 1 : 0)];
    long n_b = d->counts[2 * caf_i + (forward ? 0 : 1)];
    const float *xyv = a->data[start_i];
    float xy_scale_s = max0(a->joint_scales[start_i]);
    float nx[4];
    grow_connection(d, xyv[0], xyv[1], xy_scale_s, cols_f, n_f, nx);
    float ks = sqrtf(nx[3] * xyv[2]);
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    if (ks < d->cfg->keypoint_threshold) return;
    if (nx[3] == 0.0f) return;
    float xy_scale_t = max0(nx[2]);
    if (reverse_match) {
        float rv[4];
        grow_connection(d, nx[0], nx[1], xy_scale_t, cols_b, n_b, rv);
        if (rv[2] == 0.0f) return;
        if (fabsf(xyv[0] - rv[0]) + fabsf(xyv[1] - rv[1]) > xy_scale_s) return;
    }
    out[0] = nx[0];
    out[1] = nx[1];
    out[2] = nx[2];
    out[3] = ks;
}

/* frontier entry: (-score, None | xysv, j, k) (cifcaf.py:261,281,285) */
typedef struct {
    float neg;
    int eval;
    float xysv[4];
    int j, k;
} fentry;

static int fentry_less(const fentry *a, const fentry *b) {
    if (a->neg != b->neg) return a->neg < b->neg;
    if (a->eval != b->eval) return a->eval < b->eval; /* reference would raise TypeError */
    if (a->eval)
        for (int t = 0; t < 4; t++)
            if (a->xysv[t] != b->xysv[t]) return a->xysv[t] < b->xysv[t];
    if (a->j != b->j) return a->j < b->j;
    return a->k < b->k;
}

typedef struct {
    fentry e[4 * PP_MAX_EDGES + 8];
    int n;
} fheap;

static void fheap_push(fheap *h, fentry x) {
    int i = h->n++;
    h->e[i] = x;
    while (i > 0) {
        int p = (i - 1) / 2;
        if (!fentry_less(&h->e[i], &h->e[p])) break;
        fentry t = h->e[i];
        h->e[i] = h->e[p];
        h->e[p] = t;
        i = p;
    }
}

static fentry fheap_pop(fheap *h) {
    fentry top = h->e[0];
    h->e[0] = h->e[--h->n];
    int i = 0;
    for (;;) {
        int l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && fentry_less(&h->e[l], &h->e[m])) m = l;
        if (r < h->n && fentry_less(&h->e[r], &h->e[m])) m = r;
        if (m == i) break;
        fentry t = h->e[i];
        h->e[i] = h->e[m];
        h->e[m] = t;
        i = m;
    }
    return top;
}

/* cifcaf.py:247-307 */
static void grow(const dec_t *d, pp_ann *a, int reverse_match) {
    static _Thread_local fheap h; /* per thread: bench.py times the oracle on every core */
    h.n = 0;
    uint8_t in_frontier[PP_MAX_KP][PP_MAX_KP];
    memset(in_frontier, 0, sizeof(in_frontier));
    int K = d->K;

#define ADD_TO_FRONTIER(start_i)                                                              \
    do {                                                                                      \
        const by_source_t *b_ = &d->bs[(start_i)];                                            \
        for (int e_ = 0; e_ < b_->n; e_++) {                                                  \
            int end_ = b_->k[e_];                                                             \
            if (a->data[end_][2] > 0.0f) continue;                                            \
            if (in_frontier[(start_i)][end_]) continue;                                       \
            fentry x_;                                                                        \
            /* max_possible_score *= confidence_scales[caf_i] (cifcaf.py:258-260) */         \
            x_.neg = d->cfg->confidence_scales                                                \
                         ? -(sqrtf(a->data[(start_i)][2]) * d->cfg->confidence_scales[b_->caf[e_]]) \
                         : -sqrtf(a->data[(start_i)][2]);                                     \
            x_.eval = 0;                                                                      \
            x_.j = (start_i);                                                                 \
            x_.k = end_;                                                                      \
            fheap_push(&h, x_);                                                               \
            in_frontier[(start_i)][end_] = 1;                                                 \
            if (a->n_frontier < PP_MAX_FRONTIER) {                                            \
                a->frontier_pairs[a->n_frontier][0] = (uint8_t)(start_i);                     \
                a->frontier_pairs[a->n_frontier][1] = (uint8_t)end_;                          \
            }                                                                                 \
            a->n_frontier++;                                                                  \
        }                                                                                     \
    } while (0)

    for (int j = 0; j < K; j++) {
        if (a->data[j][2] == 0.0f) continue;
        ADD_TO_FRONTIER(j);
    }
    for (;;) {
        /* frontier_get (cifcaf.py:265-285) */
        fentry got;
        int have = 0;
        while (h.n) {
            fentry en = fheap_pop(&h);
            if (en.eval) {
                got = en;
                have = 1;
                break;
            }
            if (a->data[en.k][2] > 0.0f) continue;
            float nx[4];
            connection_value(d, a, en.j, en.k, reverse_match, nx);
            if (nx[3] == 0.0f) continue;
            fentry ev;
            ev.neg = -nx[3];
            if (d->cfg->confidence_scales && !d->cfg->greedy) { /* cifcaf.py:282-284 */
                const by_source_t *b = &d->bs[en.j];
                int caf = 0;
                for (int e = 0; e < b->n; e++)
                    if (b->k[e] == en.k) caf = b->caf[e];
                ev.neg = -(nx[3] * d->cfg->confidence_scales[caf]);
            }
            ev.eval = 1;
            memcpy(ev.xysv, nx, sizeof(nx));
            ev.j = en.j;
            ev.k = en.k;
            if (d->cfg->greedy) {
                got = ev;
                have = 1;
                break;
            }
            fheap_push(&h, ev);
        }
        if (!have) break;
        int jsi = got.j, jti = got.k;
        if (a->data[jti][2] > 0.0f) continue;
        a->data[jti][0] = got.xysv[0];
        a->data[jti][1] = got.xysv[1];
        a->data[jti][2] = got.xysv[3];
        a->joint_scales[jti] = got.xysv[2];
        if (a->n_decoding < PP_MAX_KP) {
            int t = a->n_decoding;
            a->decoding_pairs[t][0] = (uint8_t)jsi;
            a->decoding_pairs[t][1] = (uint8_t)jti;
            memcpy(&a->decoding_xyv[t][0], a->data[jsi], 3 * sizeof(float));
            memcpy(&a->decoding_xyv[t][3], a->data[jti], 3 * sizeof(float));
        }
        a->n_decoding++;
        ADD_TO_FRONTIER(jti);
    }
#undef ADD_TO_FRONTIER
}

/* flood-fill entry (-v, end_i, start_xyv, s) (cifcaf.py:317) */
typedef struct {
    float neg;
    int end;
    float sxyv[3];
    float s;
} ffentry;

static int ffentry_less(const ffentry *a, const ffentry *b) {
    if (a->neg != b->neg) return a->neg < b->neg;
    if (a->end != b->end) return a->end < b->end;
    for (int t = 0; t < 3; t++)
        if (a->sxyv[t] != b->sxyv[t]) return a->sxyv[t] < b->sxyv[t];
    return a->s < b->s;
}

/* cifcaf.py:309-331 (binary heap over at most K*K entries) */
static void flood_fill(const dec_t *d, pp_ann *a) {
    ffentry h[PP_MAX_KP * PP_MAX_KP + 4];
    int n = 0;
    int K = d->K;
#define FF_PUSH(x_)                                                                           \
    do {                                                                                      \
        int i_ = n++;                                                                         \
        h[i_] = (x_);                                                                         \
        while (i_ > 0) {                                                                      \
            int p_ = (i_ - 1) / 2;                                                            \
            if (!ffentry_less(&h[i_], &h[p_])) break;                                         \
            ffentry t_ = h[i_];                                                               \
            h[i_] = h[p_];                                                                    \
            h[p_] = t_;                                                                       \
            i_ = p_;                                                                          \
        }                                                                                     \
    } while (0)
    /* add_to_frontier keys on the ENCLOSING xyv (App. D item 5): passed as key_v */
#define FF_ADD(start_i, key_v)                                                                \
    do {                                                                                      \
        const by_source_t *b_ = &d->bs[(start_i)];                                            \
        for (int e_ = 0; e_ < b_->n; e_++) {                                                  \
            int end_ = b_->k[e_];                                                             \
            if (a->data[end_][2] > 0.0f) continue;                                            \
            ffentry x_;                                                                       \
            x_.neg = -(key_v);                                                                \
            x_.end = end_;                                                                    \
            memcpy(x_.sxyv, a->data[(start_i)], 3 * sizeof(float));                           \
            x_.s = a->joint_scales[(start_i)];                                                \
            if (n < PP_MAX_KP * PP_MAX_KP + 4) FF_PUSH(x_);                                   \
        }                                                                                     \
    } while (0)

    for (int j = 0; j < K; j++) {
        if (a->data[j][2] == 0.0f) continue;
        FF_ADD(j, a->data[j][2]);
    }
    while (n) {
        ffentry top = h[0];
        h[0] = h[--n];
        int i = 0;
        for (;;) {
            int l = 2 * i + 1, r = l + 1, m = i;
            if (l < n && ffentry_less(&h[l], &h[m])) m = l;
            if (r < n && ffentry_less(&h[r], &h[m])) m = r;
            if (m == i) break;
            ffentry t = h[i];
            h[i] = h[m];
            h[m] = t;
            i = m;
        }
        int end_i = top.end;
        if (a->data[end_i][2] > 0.0f) continue;
        a->data[end_i][0] = top.sxyv[0];
        a->data[end_i][1] = top.sxyv[1];
        a->data[end_i][2] = 0.00001f;
        a->joint_scales[end_i] = top.s;
        FF_ADD(end_i, top.sxyv[2]);
    }
#undef FF_ADD
#undef FF_PUSH
}

/* NumPy pairwise summation of a float64 array (umath loops, PW_BLOCKSIZE 128) */
static double pw_sum(const double *a, long n) {
    if (n < 8) {
        double res = 0.0;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        long i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return pw_sum(a, n2) + pw_sum(a + n2, n - n2);
}

static int float_cmp_asc(const void *pa, const void *pb) {
    float a = *(const float *)pa, b = *(const float *)pb;
    return (a < b) ? -1 : (a > b);
}

/* annotation.py:24-28, 60-71 */
EXPORT double orc_ann_score(const float *v, int K) {
    double w[PP_MAX_KP] = {0}, prod[PP_MAX_KP] = {0};
    float vs[PP_MAX_KP];
    for (int i = 0; i < K; i++) w[i] = 1.0;
    for (int i = 0; i < K && i < 3; i++) w[i] = 3.0;
    double ws = pw_sum(w, K);
    for (int i = 0; i < K; i++) w[i] /= ws;
    for (int i = 0; i < K; i++) vs[i] = v[3 * i];
    qsort(vs, (size_t)K, sizeof(float), float_cmp_asc);
    for (int i = 0; i < K; i++) prod[i] = w[i] * (double)vs[K - 1 - i];
    return pw_sum(prod, K);
}

static double ann_score(const pp_ann *a, int K) { return orc_ann_score(&a->data[0][2], K); }

/* occupancy.py:10-47 + decoder/utils.py:61-66 */
typedef struct {
    uint8_t *occ;
    long f, h, w;
    float reduction;
    float min_scale_reduced;
} occ_t;

static void occ_init(occ_t *o, long f, long h, long w, int reduction, int min_scale) {
    o->f = f;
    o->h = (long)((double)h / reduction);
    o->w = (long)((double)w / reduction);
    if (o->h < 0) o->h = 0;
    if (o->w < 0) o->w = 0;
    o->reduction = (float)reduction;
    o->min_scale_reduced = (float)((double)min_scale / reduction);
    o->occ = (uint8_t *)calloc((size_t)(f * o->h * o->w + 1), 1);
}

static long round_half_even(float x) { return (long)nearbyintf(x); }

static void occ_set(occ_t *o, int f, float x, float y, float sigma) {
    if (f >= o->f) return;
    long xi = round_half_even(x / o->reduction);
    long yi = round_half_even(y / o->reduction);
    float sr = sigma / o->reduction;
    /* max(min_scale_reduced, sigma / reduction): Python max keeps the first on ties */
    float sm = (sr > o->min_scale_reduced) ? sr : o->min_scale_reduced;
    long si = round_half_even(sm);
    long minx = xi - si > 0 ? xi - si : 0;
    long miny = yi - si > 0 ? yi - si : 0;
    long mx = xi + si + 1 < o->w ? xi + si + 1 : o->w;
    long my = yi + si + 1 < o->h ? yi + si + 1 : o->h;
    long maxx = minx + 1 > mx ? minx + 1 : mx;
    long maxy = miny + 1 > my ? miny + 1 : my;
    if (maxx > o->w) maxx = o->w; /* numpy slice clipping */
    if (maxy > o->h) maxy = o->h;
    uint8_t *p = o->occ + (size_t)f * o->h * o->w;
    for (long yy = miny; yy < maxy; yy++)
        for (long xx = minx; xx < maxx; xx++) p[yy * o->w + xx] += 1;
}

static int occ_get(const occ_t *o, int f, float x, float y) {
    if (f >= o->f) return 1;
    if (o->h <= 0 || o->w <= 0) return 0; /* reference reads out of bounds here */
    uint8_t v;
    orc_scalar_lookup(o->occ + (size_t)f * o->h * o->w, o->h, o->w, o->w, 1, 4, &x, &y, 1, 0.0f,
                      o->reduction, &v);
    return v != 0;
}

static void mark_occupied(occ_t *o, const pp_ann *a, int K) {
    for (int j = 0; j < K; j++) {
        if (a->data[j][2] == 0.0f) continue;
        occ_set(o, j, a->data[j][0], a->data[j][1], a->joint_scales[j]);
    }
}

typedef struct {
    double score;
    int idx;
} score_idx;

static int score_idx_cmp(const void *pa, const void *pb) {
    const score_idx *a = (const score_idx *)pa, *b = (const score_idx *)pb;
    double ka = -a->score, kb = -b->score;
    if (ka < kb) return -1;
    if (ka > kb) return 1;
    return (a->idx < b->idx) ? -1 : (a->idx > b->idx); /* stable */
}

/* nms.py:17-57 — in place on anns[0..n); returns the new count (order rewritten) */
static int nms_keypoints(const dec_t *d, pp_ann *anns, int n) {
    const pp_config *cfg = d->cfg;
    int K = d->K;
    pp_ann *tmp = (pp_ann *)malloc(sizeof(pp_ann) * (size_t)(n + 1));
    score_idx *si = (score_idx *)malloc(sizeof(score_idx) * (size_t)(n + 1));
    for (int i = 0; i < n; i++)
        for (int j = 0; j < K; j++)
            if (anns[i].data[j][2] < cfg->nms_keypoint_threshold)
                anns[i].data[j][0] = anns[i].data[j][1] = anns[i].data[j][2] = 0.0f;
    int m = 0;
    for (int i = 0; i < n; i++)
        if (ann_score(&anns[i], K) >= (double)cfg->nms_instance_threshold) tmp[m++] = anns[i];
    if (m == 0) {
        free(tmp);
        free(si);
        return 0;
    }
    float mx = -INFINITY, my = -INFINITY;
    for (int i = 0; i < m; i++) {
        float ax = tmp[i].data[0][0], ay = tmp[i].data[0][1];
        for (int j = 1; j < K; j++) {
            if (tmp[i].data[j][0] > ax) ax = tmp[i].data[j][0];
            if (tmp[i].data[j][1] > ay) ay = tmp[i].data[j][1];
        }
        if (i == 0 || ax > mx) mx = ax;
        if (i == 0 || ay > my) my = ay;
    }
    occ_t o;
    occ_init(&o, K, (long)(my + 1.0f), (long)(mx + 1.0f), cfg->occupancy_reduction,
             cfg->occupancy_min_scale);
    for (int i = 0; i < m; i++) {
        si[i].score = ann_score(&tmp[i], K);
        si[i].idx = i;
    }
    qsort(si, (size_t)m, sizeof(score_idx), score_idx_cmp);
    for (int r = 0; r < m; r++) {
        pp_ann *a = &tmp[si[r].idx];
        for (int f = 0; f < K; f++) {
            float v = a->data[f][2];
            if (v == 0.0f) continue;
            if (occ_get(&o, f, a->data[f][0], a->data[f][1]))
                a->data[f][2] *= cfg->nms_suppression;
            else
                occ_set(&o, f, a->data[f][0], a->data[f][1], a->joint_scales[f]);
        }
    }
    free(o.occ);
    /* anns = sorted order; filter again; sort again */
    int k = 0;
    for (int r = 0; r < m; r++) {
        pp_ann *a = &tmp[si[r].idx];
        for (int j = 0; j < K; j++)
            if (a->data[j][2] < cfg->nms_keypoint_threshold)
                a->data[j][0] = a->data[j][1] = a->data[j][2] = 0.0f;
        if (ann_score(a, K) >= (double)cfg->nms_instance_threshold) anns[k++] = *a;
    }
    for (int i = 0; i < k; i++) {
        si[i].score = ann_score(&anns[i], K);
        si[i].idx = i;
    }
    qsort(si, (size_t)k, sizeof(score_idx), score_idx_cmp);
    for (int i = 0; i < k; i++) tmp[i] = anns[si[i].idx];
    memcpy(anns, tmp, sizeof(pp_ann) * (size_t)k);
    free(tmp);
    free(si);
    return k;
}

/* nms.Keypoints().annotations (nms.py:17-57) on caller records; survivors written to
 * anns[0..k) in output order (carry an input index in pp_ann.image to track them) */
EXPORT long orc_nms_keypoints(pp_ann *anns, long n, int K, const pp_config *cfg) {
    if (K <= 0 || K > PP_MAX_KP || n < 0) return -1;
    if (n == 0) return 0;
    dec_t d;
    memset(&d, 0, sizeof(d));
    d.K = K;
    d.cfg = cfg;
    return nms_keypoints(&d, anns, (int)n);
}

EXPORT long orc_decode_multi(const pp_scale *sc, int n, int pairs, int K, int C,
                             const int32_t *skel, const pp_config *cfg, pp_ann *out, long cap);

static void ann_init(pp_ann *a, int K) {
    memset(a, 0, sizeof(*a));
    a->n_keypoints = K;
}

/* cifcaf.py:67-122 for one image.  Returns the number of annotations (written when
 * <= cap). */
EXPORT long orc_decode(const float *cif, const float *caf, int K, int C, int H, int W,
                       const int32_t *skel, const pp_config *cfg, pp_ann *out, long cap) {
    pp_scale sc;
    memset(&sc, 0, sizeof(sc));
    sc.cif = cif;
    sc.caf = caf;
    sc.H = H;
    sc.W = W;
    sc.stride = cfg->stride;
    return orc_decode_multi(&sc, 1, 0, K, C, skel, cfg, out, cap);
}

/* ---- multi-scale (cif_hr.py:42-73, cif_seeds.py:56-64, caf_scored.py:32-98) ----------- */

/* the CIF (role bit 1) or CAF (role bit 2) heads of a pp_scale list, in order */
static int role_list(const pp_scale *sc, int n, int bit, const pp_scale **out) {
    int k = 0;
    for (int i = 0; i < n; i++)
        if ((sc[i].role ? sc[i].role : 3) & bit) out[k++] = &sc[i];
    return k;
}

/* the CifHr map's geometry: a PP_ROLE_HRMAP (4) entry's, else CIF head 0's */
static void hr_geometry(const pp_scale *all, int n_all, long *hh, long *ww) {
    for (int i = 0; i < n_all; i++)
        if (all[i].role == 4) {
            *hh = hr_dim(all[i].H, all[i].stride);
            *ww = hr_dim(all[i].W, all[i].stride);
            return;
        }
    const pp_scale *cl[2 * PP_MAX_SCALES];
    role_list(all, n_all, 1, cl);
    *hh = hr_dim(cl[0]->H, cl[0]->stride);
    *ww = hr_dim(cl[0]->W, cl[0]->stride);
}

/* CifHr.fill / fill_multiple (cif_hr.py:42-73): groups of len heads (pairs 0: len 1, every
 * head on its own; 1: hflip pairs, heads i and i + n/2; m >= 2: len m, member t of group i =
 * head i + t * n/m) accumulate into one map with len_cifs = len at head i's stride / min
 * scale.  Maps combine by np.maximum in order.  out (K, H', W') (hr_geometry). */
EXPORT void orc_cifhr_multi(const pp_scale *all, int n_all, int pairs, int K, const pp_config *cfg,
                            float *out) {
    const pp_scale *cl[2 * PP_MAX_SCALES];
    int n = role_list(all, n_all, 1, cl);
    long hh, ww;
    hr_geometry(all, n_all, &hh, &ww);
    size_t plane = (size_t)hh * ww;
    float *ta = (float *)malloc(sizeof(float) * K * plane);
    int len = pairs <= 0 ? 1 : (pairs == 1 ? 2 : pairs);
    int n_groups = n / len;
    for (int gi = 0; gi < n_groups; gi++) {
        float stride = (float)cl[gi]->stride;
        float min_scale = cl[gi]->cif_min_scale;
        memset(ta, 0, sizeof(float) * K * plane);
        for (int mi = 0; mi < len; mi++) {
            const pp_scale *m = cl[gi + mi * n_groups];
            long hw = (long)m->H * m->W;
            float *xs = (float *)malloc(sizeof(float) * 4 * (size_t)(hw + 1));
            float *ys = xs + hw, *ss = ys + hw, *vs = ss + hw;
            for (int f = 0; f < K; f++) {
                const float *p = m->cif + (size_t)f * 5 * hw;
                long k = 0;
                for (long c = 0; c < hw; c++) {
                    if (!(p[c] > cfg->cif_threshold)) continue;
                    if (min_scale != 0.0f && !(p[4 * hw + c] > (float)((double)min_scale / stride)))
                        continue;
                    xs[k] = p[1 * hw + c] * stride;
                    ys[k] = p[2 * hw + c] * stride;
                    float sg = (0.5f * p[4 * hw + c]) * stride;
                    ss[k] = (sg != sg) ? sg : fmaxf(1.0f, sg);
                    vs[k] = (p[c] / (float)cfg->cif_neighbors) / (float)len;
                    k++;
                }
                orc_scalar_square_add_gauss_with_max(ta + f * plane, hh, ww, ww, 1, xs, ys, ss,
                                                     vs, k, 1.0f, 1.0f);
            }
            free(xs);
        }
        if (gi == 0) {
            memcpy(out, ta, sizeof(float) * K * plane);
        } else {
            for (size_t i = 0; i < K * plane; i++) { /* np.maximum(ta, accumulated) */
                float a = ta[i], b = out[i];
                out[i] = (a != a || b != b) ? NAN : (a > b ? a : b);
            }
        }
    }
    free(ta);
}

/* CifSeeds.fill over every CIF head in order; sorted as get() */
EXPORT long orc_seeds_multi(const pp_scale *all, int n_all, int K, const float *hr, long hh,
                            long ww, const pp_config *cfg, pp_seed *out, long cap) {
    const pp_scale *cl[2 * PP_MAX_SCALES];
    int n = role_list(all, n_all, 1, cl);
    long total = 0;
    for (int m = 0; m < n; m++) total += (long)K * cl[m]->H * cl[m]->W;
    float *tmp = (float *)malloc(sizeof(float) * 6 * (size_t)(total + 1));
    long k = 0;
    for (int m = 0; m < n; m++) {
        long hw = (long)cl[m]->H * cl[m]->W;
        float stride = (float)cl[m]->stride;
        for (int f = 0; f < K; f++) {
            if ((cfg->seed_skip_mask >> f) & 1u) continue; /* cif_seeds.py:28-29 seed_mask */
            const float *p = cl[m]->cif + (size_t)f * 5 * hw;
            const float *t = hr + (size_t)f * hh * ww;
            for (long c = 0; c < hw; c++) {
                float conf = p[c];
                if (!(conf > cfg->seed_threshold)) continue;
                if (cl[m]->cif_min_scale != 0.0f &&
                    !(p[4 * hw + c] > (float)((double)cl[m]->cif_min_scale / cl[m]->stride)))
                    continue;
                float x = p[1 * hw + c] * stride, y = p[2 * hw + c] * stride, v;
                orc_scalar_values(t, hh, ww, ww, 1, &x, &y, 1, 0.0f, &v);
                v = 0.9f * v + 0.1f * conf;
                if (cfg->seed_score_scale != 1.0f) v = v * cfg->seed_score_scale;
                if (!(v > cfg->seed_threshold)) continue;
                float *r = tmp + 6 * k;
                r[0] = v;
                r[1] = (float)f;
                r[2] = x;
                r[3] = y;
                r[4] = p[4 * hw + c] * stride;
                r[5] = (float)k;
                k++;
            }
        }
    }
    qsort(tmp, (size_t)k, sizeof(float) * 6, seed_cmp_desc);
    for (long i = 0; i < k && i < cap; i++) {
        float *r = tmp + 6 * i;
        out[i].v = r[0];
        out[i].field = (int32_t)r[1];
        out[i].x = r[2];
        out[i].y = r[3];
        out[i].s = r[4];
    }
    free(tmp);
    return k;
}

/* CafScored.fill over every CAF head in order: per field the heads' columns concatenated.
 * cols (C, 2, 9, cap) with cap >= sum of H*W over the heads */
EXPORT void orc_caf_scored_multi(const pp_scale *all, int n_all, int K, int C, const float *hr,
                                 long hh, long ww, const int32_t *skel, float score_th,
                                 const pp_config *cfg, float *cols, long cap, int32_t *counts) {
    const pp_scale *al[2 * PP_MAX_SCALES];
    int n = role_list(all, n_all, 2, al);
    float floor_ = cfg->cif_floor;
    float one_minus = (float)(1.0 - (double)cfg->cif_floor);
    for (int i = 0; i < C; i++) {
        float *bwd = cols + ((size_t)i * 2 + 0) * 9 * cap;
        float *fwd = cols + ((size_t)i * 2 + 1) * 9 * cap;
        int j1i = skel[2 * i] - 1, j2i = skel[2 * i + 1] - 1;
        long nb = 0, nf = 0;
        for (int m = 0; m < n; m++) {
            long hw = (long)al[m]->H * al[m]->W;
            float stride = (float)al[m]->stride;
            const float *p = al[m]->caf + (size_t)i * 9 * hw;
            float dmin = al[m]->caf_min_distance, dmax = al[m]->caf_max_distance;
            float tmin = (float)((double)dmin / al[m]->stride), tmax = (float)((double)dmax / al[m]->stride);
            for (long c = 0; c < hw; c++) {
                float nine[9];
                nine[0] = p[c];
                if (!(nine[0] > score_th)) continue;
                if (dmin != 0.0f || dmax != 0.0f) { /* np.linalg.norm(nine[1:3] - nine[5:7]) */
                    float dx = p[1 * hw + c] - p[5 * hw + c], dy = p[2 * hw + c] - p[6 * hw + c];
                    float dist = sqrtf(dx * dx + dy * dy);
                    if (dmin != 0.0f && !(dist > tmin)) continue;
                    if (dmax != 0.0f && !(dist < tmax)) continue;
                }
                for (int r = 1; r < 9; r++) nine[r] = p[r * hw + c] * stride;
                float score = nine[0], sb = score, sf = score;
                if (floor_ < 1.0f && j1i < K) {
                    float h1;
                    orc_scalar_values(hr + (size_t)j1i * hh * ww, hh, ww, ww, 1, &nine[1], &nine[2],
                                      1, 0.0f, &h1);
                    sb = score * (floor_ + one_minus * h1);
                }
                if (sb > score_th) {
                    static const int order_b[9] = {0, 5, 6, 7, 8, 1, 2, 3, 4};
                    for (int r = 0; r < 9; r++) bwd[r * cap + nb] = nine[order_b[r]];
                    bwd[nb] = sb;
                    nb++;
                }
                if (floor_ < 1.0f && j2i < K) {
                    float h2;
                    orc_scalar_values(hr + (size_t)j2i * hh * ww, hh, ww, ww, 1, &nine[5], &nine[6],
                                      1, 0.0f, &h2);
                    sf = score * (floor_ + one_minus * h2);
                }
                if (sf > score_th) {
                    for (int r = 0; r < 9; r++) fwd[r * cap + nf] = nine[r];
                    fwd[nf] = sf;
                    nf++;
                }
            }
        }
        counts[2 * i + 0] = (int32_t)nb;
        counts[2 * i + 1] = (int32_t)nf;
    }
}

/* cifcaf.py:67-122 over a FieldConfig of n CIF / CAF heads (one image): CifHr, CifSeeds and
 * CafScored fill from every head (the functions above), the rest as one scale.  `init`
 * (n_init records, may be NULL): initial_annotations, grown, appended and marked occupied
 * before the seed loop (cifcaf.py:95-98).  out_index (optional, cap entries): each output
 * annotation's position in the list before NMS. */
EXPORT long orc_decode_initial(const pp_scale *sc, int n, int pairs, int K, int C,
                               const int32_t *skel, const pp_config *cfg, const pp_ann *init,
                               long n_init, pp_ann *out, long cap, int32_t *out_index) {
    if (K > PP_MAX_KP || C > PP_MAX_EDGES || K <= 0 || C <= 0 || n <= 0 || n_init < 0) return -1;
    const pp_scale *cl[2 * PP_MAX_SCALES], *al[2 * PP_MAX_SCALES];
    int n_cif = role_list(sc, n, 1, cl), n_caf = role_list(sc, n, 2, al);
    int gsize = pairs <= 0 ? 1 : (pairs == 1 ? 2 : pairs);
    if (n_cif == 0 || n_caf == 0 || (n_cif % gsize)) return -1;
    long total_hw = 0, cif_hw = 0;
    for (int m = 0; m < n; m++)
        if (sc[m].H <= 0 || sc[m].W <= 0 || sc[m].stride <= 0) return -1;
    for (int m = 0; m < n_cif; m++) cif_hw += (long)cl[m]->H * cl[m]->W;
    for (int m = 0; m < n_caf; m++) total_hw += (long)al[m]->H * al[m]->W;
    long hh, ww;
    hr_geometry(sc, n, &hh, &ww);
    float *hr = (float *)malloc(sizeof(float) * (size_t)K * hh * ww);
    orc_cifhr_multi(sc, n, pairs, K, cfg, hr);
    pp_seed *seeds = (pp_seed *)malloc(sizeof(pp_seed) * (size_t)(K * cif_hw + 1));
    long n_seeds = orc_seeds_multi(sc, n, K, hr, hh, ww, cfg, seeds, K * cif_hw);

    dec_t d;
    d.K = K;
    d.C = C;
    d.H = cl[0]->H;
    d.W = cl[0]->W;
    d.hw = total_hw; /* column capacity of every (connection, direction) set */
    d.cfg = cfg;
    build_by_source(&d, skel);
    float *cols = (float *)malloc(sizeof(float) * (size_t)C * 2 * 9 * total_hw);
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * (size_t)C * 2);
    orc_caf_scored_multi(sc, n, K, C, hr, hh, ww, skel, cfg->caf_threshold, cfg, cols, total_hw,
                         counts);
    d.cols = cols;
    d.counts = counts;

    occ_t o;
    occ_init(&o, K, hh, ww, cfg->occupancy_reduction, cfg->occupancy_min_scale);
    long acap = 64 + n_init, na = 0;
    pp_ann *anns = (pp_ann *)malloc(sizeof(pp_ann) * (size_t)acap);
    for (long i = 0; i < n_init; i++) { /* cifcaf.py:95-98 */
        pp_ann *a = &anns[na++];
        *a = init[i];
        a->n_keypoints = K;
        a->image = 0;
        grow(&d, a, 1);
        mark_occupied(&o, a, K);
    }
    for (long s = 0; s < n_seeds; s++) {
        const pp_seed *sd = &seeds[s];
        if (occ_get(&o, sd->field, sd->x, sd->y)) continue;
        if (na == acap) {
            acap *= 2;
            anns = (pp_ann *)realloc(anns, sizeof(pp_ann) * (size_t)acap);
        }
        pp_ann *a = &anns[na++];
        ann_init(a, K);
        a->data[sd->field][0] = sd->x;
        a->data[sd->field][1] = sd->y;
        a->data[sd->field][2] = sd->v;
        a->joint_scales[sd->field] = sd->s;
        grow(&d, a, 1);
        mark_occupied(&o, a, K);
    }
    free(o.occ);

    if (cfg->force_complete) {
        /* cifcaf.py:333-351 */
        orc_caf_scored_multi(sc, n, K, C, hr, hh, ww, skel, cfg->complete_caf_threshold, cfg, cols,
                             total_hw, counts);
        for (long i = 0; i < na; i++) {
            pp_ann *a = &anns[i];
            int unfilled[PP_MAX_KP];
            for (int j = 0; j < K; j++) unfilled[j] = a->data[j][2] == 0.0f;
            grow(&d, a, 0);
            for (int j = 0; j < K; j++)
                if (unfilled[j] && a->data[j][2] > 0.0f)
                    a->data[j][2] = (0.001f < a->data[j][2]) ? 0.001f : a->data[j][2];
            int any0 = 0;
            for (int j = 0; j < K; j++) any0 |= a->data[j][2] == 0.0f;
            if (any0) flood_fill(&d, a);
        }
    }
    for (long i = 0; i < na; i++) anns[i].image = (int32_t)i; /* tracks positions through NMS */
    if (cfg->apply_nms) na = nms_keypoints(&d, anns, (int)na);
    for (long i = 0; i < na; i++) {
        anns[i].score = ann_score(&anns[i], K);
        if (out_index && i < cap) out_index[i] = anns[i].image;
        anns[i].image = 0;
        if (i < cap) out[i] = anns[i];
    }
    free(anns);
    free(cols);
    free(counts);
    free(seeds);
    free(hr);
    return na;
}

EXPORT long orc_decode_multi(const pp_scale *sc, int n, int pairs, int K, int C,
                             const int32_t *skel, const pp_config *cfg, pp_ann *out, long cap) {
    return orc_decode_initial(sc, n, pairs, K, C, skel, cfg, NULL, 0, out, cap, NULL);
}

/* ---- CifDet (decoder/generator/cifdet.py:27-52) ---------------------------------------- */

/* cif_hr.py:84-100 on (K, 7, H, W) fields [c, x, y, b, w, h, b2]; out (K, H', W') */
EXPORT void orc_cifdet_hr(const float *det, int K, int H, int W, const pp_config *cfg, float *out) {
    long hh = hr_dim(H, cfg->stride), ww = hr_dim(W, cfg->stride);
    long hw = (long)H * W;
    float *xs = (float *)malloc(sizeof(float) * 4 * (size_t)hw);
    float *ys = xs + hw, *ss = ys + hw, *vs = ss + hw;
    memset(out, 0, sizeof(float) * (size_t)K * hh * ww);
    float stride = (float)cfg->stride;
    for (int f = 0; f < K; f++) {
        const float *p = det + (size_t)f * 7 * hw;
        long n = 0;
        for (long c = 0; c < hw; c++) {
            if (!(p[c] > cfg->cif_threshold)) continue;
            xs[n] = p[1 * hw + c] * stride;
            ys[n] = p[2 * hw + c] * stride;
            float w = p[4 * hw + c], h = p[5 * hw + c];
            float m = (w != w) ? w : ((h != h) ? h : (h < w ? h : w)); /* np.minimum */
            float sg = (0.1f * m) * stride;
            ss[n] = (sg != sg) ? sg : fmaxf(1.0f, sg); /* np.maximum(1.0, .) */
            vs[n] = (p[c] / (float)cfg->cif_neighbors) / 1.0f;
            n++;
        }
        orc_scalar_square_add_gauss_with_max(out + (size_t)f * hh * ww, hh, ww, ww, 1, xs, ys, ss,
                                             vs, n, 1.0f, 1.0f);
    }
    free(xs);
}

static int det_seed_cmp_desc(const void *pa, const void *pb) {
    /* sorted(seeds, reverse=True) on (v, f, x, y, w, h); stable -> emission ascending */
    const float *a = (const float *)pa, *b = (const float *)pb; /* v f x y w h idx */
    for (int i = 0; i < 6; i++) {
        if (a[i] == b[i]) continue;
        return (a[i] > b[i]) ? -1 : 1;
    }
    return (a[6] < b[6]) ? -1 : (a[6] > b[6]);
}

/* cif_seeds.py:67-90.  out (cap, 7): v, f, x, y, w, h, emission index */
EXPORT long orc_cifdet_seeds(const float *det, const float *hr, long hr_pitch, int K, int H, int W,
                             const pp_config *cfg, float *out, long cap) {
    long hh = hr_dim(H, cfg->stride), ww = hr_dim(W, cfg->stride);
    long hw = (long)H * W;
    float stride = (float)cfg->stride;
    float *tmp = (float *)malloc(sizeof(float) * 7 * (size_t)(K * hw + 1));
    long n = 0;
    for (int f = 0; f < K; f++) {
        if ((cfg->seed_skip_mask >> f) & 1u) continue; /* cif_seeds.py:70-71 seed_mask */
        const float *p = det + (size_t)f * 7 * hw;
        const float *t = hr + (size_t)f * hh * hr_pitch;
        for (long c = 0; c < hw; c++) {
            float conf = p[c];
            if (!(conf > cfg->seed_threshold)) continue;
            float x = p[1 * hw + c], y = p[2 * hw + c];
            float xs = x * stride, ys = y * stride, v;
            orc_scalar_values(t, hh, ww, hr_pitch, 1, &xs, &ys, 1, 0.0f, &v);
            v = 0.9f * v + 0.1f * conf;
            if (cfg->seed_score_scale != 1.0f) v = v * cfg->seed_score_scale;
            if (!(v > cfg->seed_threshold)) continue;
            float *r = tmp + 7 * n;
            r[0] = v;
            r[1] = (float)f;
            r[2] = xs;
            r[3] = ys;
            r[4] = p[4 * hw + c] * stride;
            r[5] = p[5 * hw + c] * stride;
            r[6] = (float)n;
            n++;
        }
    }
    qsort(tmp, (size_t)n, sizeof(float) * 7, det_seed_cmp_desc);
    for (long i = 0; i < n && i < cap; i++) memcpy(out + 7 * i, tmp + 7 * i, sizeof(float) * 7);
    free(tmp);
    return n;
}

static inline float np_max(float a, float b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }
static inline float np_min(float a, float b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }

/* nms.Detection.bbox_iou (nms.py:67-77) for one pair, float32 as NumPy evaluates it */
static float det_iou(const float *b, const float *o) {
    float x1 = np_max(b[0], o[0]), y1 = np_max(b[1], o[1]);
    float x2 = np_min(b[0] + b[2], o[0] + o[2]), y2 = np_min(b[1] + b[3], o[1] + o[3]);
    float inter = np_max(0.0f, x2 - x1) * np_max(0.0f, y2 - y1);
    float ba = b[2] * b[3], oa = o[2] * o[3];
    return inter / (((ba + oa) - inter) + 1e-5f);
}

typedef struct {
    float score;
    int idx;
} det_si;

static int det_si_cmp(const void *pa, const void *pb) { /* sorted(key=-score), stable */
    const det_si *a = (const det_si *)pa, *b = (const det_si *)pb;
    float ka = -a->score, kb = -b->score;
    if (ka < kb) return -1;
    if (ka > kb) return 1;
    return (a->idx < b->idx) ? -1 : (a->idx > b->idx);
}

/* nms.py:79-102 in place on d[0..n); returns the new count */
static long det_nms(pp_det *d, long n, const pp_det_nms *p) {
    det_si *si = (det_si *)malloc(sizeof(det_si) * (size_t)(n + 1));
    pp_det *tmp = (pp_det *)malloc(sizeof(pp_det) * (size_t)(n + 1));
    long m = 0;
    for (long i = 0; i < n; i++)
        if (d[i].score >= p->instance_threshold) tmp[m++] = d[i];
    if (m == 0) {
        free(si);
        free(tmp);
        return 0;
    }
    for (long i = 0; i < m; i++) {
        si[i].score = tmp[i].score;
        si[i].idx = (int)i;
    }
    qsort(si, (size_t)m, sizeof(det_si), det_si_cmp);
    for (long i = 0; i < m; i++) d[i] = tmp[si[i].idx];
    for (long i = 1; i < m; i++) {
        float mx = -INFINITY; /* np.max over the masked IoUs: NaN if any is NaN */
        int nan = 0;
        for (long j = 0; j < i; j++) {
            if (!(d[j].score >= p->instance_threshold)) continue;
            float iou = det_iou(d[i].bbox, d[j].bbox);
            if (iou != iou)
                nan = 1;
            else if (iou > mx)
                mx = iou;
        }
        if (nan) mx = NAN;
        if (mx > p->iou_threshold)
            d[i].score *= p->suppression;
        else if (mx > p->iou_threshold_soft)
            d[i].score *= p->suppression_soft;
    }
    long k = 0;
    for (long i = 0; i < m; i++)
        if (d[i].score >= p->instance_threshold) tmp[k++] = d[i];
    for (long i = 0; i < k; i++) {
        si[i].score = tmp[i].score;
        si[i].idx = (int)i;
    }
    qsort(si, (size_t)k, sizeof(det_si), det_si_cmp);
    for (long i = 0; i < k; i++) d[i] = tmp[si[i].idx];
    free(si);
    free(tmp);
    return k;
}

/* CifDet.__call__ for one image; returns the number of detections (written when <= cap) */
EXPORT long orc_cifdet_decode(const float *det, int K, int H, int W, const pp_config *cfg,
                              const pp_det_nms *nms, pp_det *out, long cap) {
    long hh = hr_dim(H, cfg->stride), ww = hr_dim(W, cfg->stride);
    float *hr = (float *)malloc(sizeof(float) * (size_t)K * hh * ww);
    orc_cifdet_hr(det, K, H, W, cfg, hr);
    long hw = (long)H * W;
    float *seeds = (float *)malloc(sizeof(float) * 7 * (size_t)(K * hw + 1));
    long ns = orc_cifdet_seeds(det, hr, ww, K, H, W, cfg, seeds, K * hw);
    occ_t o;
    occ_init(&o, K, hh, ww, 2, 2); /* Occupancy(cifhr.shape, 2, min_scale=2.0) */
    pp_det *d = (pp_det *)calloc((size_t)(ns + 1), sizeof(pp_det));
    long n = 0;
    for (long i = 0; i < ns; i++) {
        const float *r = seeds + 7 * i;
        int f = (int)r[1];
        float x = r[2], y = r[3], w = r[4], h = r[5];
        if (occ_get(&o, f, x, y)) continue;
        d[n].field = f;
        d[n].score = r[0];
        d[n].bbox[0] = x - w / 2.0f;
        d[n].bbox[1] = y - h / 2.0f;
        d[n].bbox[2] = w;
        d[n].bbox[3] = h;
        n++;
        float mwh = (h < w) ? h : w; /* builtin min(w, h) */
        occ_set(&o, f, x, y, 0.1f * mwh);
    }
    if (nms->apply) n = det_nms(d, n, nms);
    for (long i = 0; i < n && i < cap; i++) out[i] = d[i];
    free(o.occ);
    free(d);
    free(seeds);
    free(hr);
    return n;
}

EXPORT int orc_sizeof_ann(void) { return (int)sizeof(pp_ann); }
