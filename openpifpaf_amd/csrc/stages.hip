// stages.hip — CifSeeds and CafScored on gfx950.
//
//   seeds_kernel       one workgroup per image: threshold + CifHr rescore + order-preserving
//                      ballot compaction (cif_seeds.py:23-50), then a bitonic sort that
//                      reproduces sorted(seeds, reverse=True) (cif_seeds.py:54) including
//                      its stability (ties broken by emission order).  LDS-resident up to
//                      kSortLds seeds, global-memory network beyond.
//   caf_scored_kernel  one workgroup per (image, CAF field): threshold, x stride, CifHr
//                      lookups at both ends, forward/backward column sets in row-major
//                      cell order (caf_scored.py:32-87), one or two thresholds per pass.
//
// There is deliberately NO spatial NMS before the sort: v0.11.6 suppresses duplicate
// seeds only through the occupancy test in the seed loop (cifcaf.py:100-102).
#include "pp_common.hpp"

namespace pp {

constexpr int kSortLds = 4096;

struct SeedKeys {
    const float *v, *x, *y, *s;
    const int *f;
    int n;
    // true when seed a must come before seed b in sorted(..., reverse=True) order
    __device__ __forceinline__ bool before(int a, int b) const {
        if (a >= n) return false;  // padding sorts last
        if (b >= n) return true;
        if (v[a] != v[b]) return v[a] > v[b];
        if (f[a] != f[b]) return f[a] > f[b];
        if (x[a] != x[b]) return x[a] > x[b];
        if (y[a] != y[b]) return y[a] > y[b];
        if (s[a] != s[b]) return s[a] > s[b];
        return a < b;  // stable
    }
};

template <typename Perm>
__device__ void bitonic_sort(Perm *p, int np, const SeedKeys &keys) {
    for (int k = 2; k <= np; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int a = p[i], b = p[ixj];
                    const bool asc = (i & k) == 0;
                    const bool sw = asc ? keys.before(b, a) : keys.before(a, b);
                    if (sw) {
                        p[i] = b;
                        p[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

struct SeedArgs {
    const float *cif, *hr;
    int K, H, W, hh, ww;
    int64_t pitch;
    float stride, th, score_scale;
    pp_seed *seeds;     // (n_img, cap) sorted output
    int cap;
    int *counts;
    float *g_keys;      // (n_img, 4, cap) global sort scratch (v, x, y, s)
    int *g_f;           // (n_img, cap)
    int *g_perm;        // (n_img, np_cap)
    int np_cap;
};

__global__ __launch_bounds__(256) void seeds_kernel(SeedArgs a) {
    __shared__ int s_tmp[4];
    __shared__ float s_v[kSortLds], s_x[kSortLds], s_y[kSortLds], s_s[kSortLds];
    __shared__ int s_f[kSortLds];
    __shared__ uint16_t s_perm[kSortLds];
    const int img = blockIdx.x;
    const int hw = a.H * a.W;
    const int64_t cap = a.cap;
    float *gv = a.g_keys + (int64_t)img * 4 * cap, *gx = gv + cap, *gy = gx + cap, *gs = gy + cap;
    int *gf = a.g_f + (int64_t)img * cap;
    int running = 0;
    for (int f = 0; f < a.K; f++) {
        const float *p = a.cif + ((int64_t)img * a.K + f) * 5 * hw;
        const float *t = a.hr + ((int64_t)img * a.K + f) * a.hh * a.pitch;
        for (int base = 0; base < hw; base += 256) {
            const int cell = base + threadIdx.x;
            bool keep = false;
            float v = 0.0f, x = 0.0f, y = 0.0f, sc = 0.0f;
            if (cell < hw) {
                const float c = p[cell];
                if (c > a.th) {  // p[:, p[0] > threshold]
                    x = p[hw + cell] * a.stride;
                    y = p[2 * hw + cell] * a.stride;
                    const float h = hr_lookup(t, a.hh, a.ww, a.pitch, x, y, 0.0f);
                    v = 0.9f * h + 0.1f * c;
                    if (a.score_scale != 1.0f) v = v * a.score_scale;
                    keep = v > a.th;
                    sc = p[4 * hw + cell] * a.stride;
                }
            }
            int total;
            const int slot = block_compact<4>(keep, s_tmp, total);
            const int pos = running + slot;
            if (keep && pos < a.cap) {
                if (pos < kSortLds) {
                    s_v[pos] = v;
                    s_x[pos] = x;
                    s_y[pos] = y;
                    s_s[pos] = sc;
                    s_f[pos] = f;
                }
                gv[pos] = v;
                gx[pos] = x;
                gy[pos] = y;
                gs[pos] = sc;
                gf[pos] = f;
            }
            running += total;
        }
    }
    if (threadIdx.x == 0) a.counts[img] = running;
    if (running > a.cap) return;  // overflow: host re-runs with a larger capacity
    const int n = running;
    int np = 1;
    while (np < n) np <<= 1;
    pp_seed *out = a.seeds + (int64_t)img * cap;
    __syncthreads();
    if (n <= kSortLds) {
        for (int i = threadIdx.x; i < np; i += blockDim.x) s_perm[i] = (uint16_t)i;
        __syncthreads();
        SeedKeys keys{s_v, s_x, s_y, s_s, s_f, n};
        bitonic_sort(s_perm, np, keys);
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int k = s_perm[i];
            pp_seed r;
            r.v = s_v[k];
            r.field = s_f[k];
            r.x = s_x[k];
            r.y = s_y[k];
            r.s = s_s[k];
            out[i] = r;
        }
    } else {
        int *perm = a.g_perm + (int64_t)img * a.np_cap;
        for (int i = threadIdx.x; i < np; i += blockDim.x) perm[i] = i;
        __syncthreads();
        SeedKeys keys{gv, gx, gy, gs, gf, n};
        bitonic_sort(perm, np, keys);
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int k = perm[i];
            pp_seed r;
            r.v = gv[k];
            r.field = gf[k];
            r.x = gx[k];
            r.y = gy[k];
            r.s = gs[k];
            out[i] = r;
        }
    }
}

// ------------------------------------------------------------------------------------
constexpr int kMaxCaf = PP_MAX_EDGES;

struct CafArgs {
    const float *caf, *hr;
    int K, C, H, W, hh, ww;
    int64_t pitch;
    float stride, cif_floor, one_minus_floor;
    int nt;             // number of thresholds (1 or 2)
    float th[2];
    float *cols[2];     // (n_img, C, 2, 9, H*W): dir 0 backward, 1 forward
    int *counts[2];     // (n_img, C, 2)
    int j1[kMaxCaf], j2[kMaxCaf];
};

__global__ __launch_bounds__(256) void caf_scored_kernel(CafArgs a) {
    __shared__ int s_tmp[4];
    const int64_t fld = blockIdx.x;  // image * C + caf field
    const int img = (int)(fld / a.C), ci = (int)(fld % a.C);
    const int hw = a.H * a.W;
    const float *p = a.caf + fld * 9 * hw;
    const int j1i = a.j1[ci], j2i = a.j2[ci];
    const bool use1 = a.cif_floor < 1.0f && j1i < a.K;
    const bool use2 = a.cif_floor < 1.0f && j2i < a.K;
    const float *t1 = a.hr + ((int64_t)img * a.K + (use1 ? j1i : 0)) * a.hh * a.pitch;
    const float *t2 = a.hr + ((int64_t)img * a.K + (use2 ? j2i : 0)) * a.hh * a.pitch;
    int run_b[2] = {0, 0}, run_f[2] = {0, 0};
    const float th_min = a.nt == 2 ? fminf(a.th[0], a.th[1]) : a.th[0];
    for (int base = 0; base < hw; base += 256) {
        const int cell = base + threadIdx.x;
        float nine[9];
        float sb = 0.0f, sf = 0.0f;
        bool any = false;
        if (cell < hw) {
            nine[0] = p[cell];
            any = nine[0] > th_min;
            if (any) {
#pragma unroll
                for (int r = 1; r < 9; r++) nine[r] = p[r * hw + cell] * a.stride;
                const float score = nine[0];
                sb = score;
                sf = score;
                if (use1)
                    sb = score * (a.cif_floor +
                                  a.one_minus_floor *
                                      hr_lookup(t1, a.hh, a.ww, a.pitch, nine[1], nine[2], 0.0f));
                if (use2)
                    sf = score * (a.cif_floor +
                                  a.one_minus_floor *
                                      hr_lookup(t2, a.hh, a.ww, a.pitch, nine[5], nine[6], 0.0f));
            }
        }
        for (int t = 0; t < a.nt; t++) {
            const float th = a.th[t];
            const bool pass = any && nine[0] > th;  // mask = nine[0] > score_th
            const bool kb = pass && sb > th, kf = pass && sf > th;
            int tot_b, tot_f;
            const int slot_b = block_compact<4>(kb, s_tmp, tot_b);
            const int slot_f = block_compact<4>(kf, s_tmp, tot_f);
            float *bwd = a.cols[t] + (fld * 2 + 0) * 9 * (int64_t)hw;
            float *fwd = a.cols[t] + (fld * 2 + 1) * 9 * (int64_t)hw;
            if (kb) {
                // backward rows (0, 5, 6, 7, 8, 1, 2, 3, 4) with row 0 = scores_b
                const int c = run_b[t] + slot_b;
                bwd[c] = sb;
                bwd[1 * hw + c] = nine[5];
                bwd[2 * hw + c] = nine[6];
                bwd[3 * hw + c] = nine[7];
                bwd[4 * hw + c] = nine[8];
                bwd[5 * hw + c] = nine[1];
                bwd[6 * hw + c] = nine[2];
                bwd[7 * hw + c] = nine[3];
                bwd[8 * hw + c] = nine[4];
            }
            if (kf) {
                const int c = run_f[t] + slot_f;
                fwd[c] = sf;
#pragma unroll
                for (int r = 1; r < 9; r++) fwd[r * hw + c] = nine[r];
            }
            run_b[t] += tot_b;
            run_f[t] += tot_f;
        }
    }
    if (threadIdx.x == 0) {
        for (int t = 0; t < a.nt; t++) {
            a.counts[t][fld * 2 + 0] = run_b[t];
            a.counts[t][fld * 2 + 1] = run_f[t];
        }
    }
}

static inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

int launch_seeds(const float *cif, const float *hr, int n_img, int K, int H, int W,
                 const pp_config *cfg, pp_seed *seeds, int cap, int *counts, void *scratch,
                 hipStream_t s) {
    SeedArgs a{};
    a.cif = cif;
    a.hr = hr;
    a.K = K;
    a.H = H;
    a.W = W;
    a.hh = (int)hr_dim(H, cfg->stride);
    a.ww = (int)hr_dim(W, cfg->stride);
    a.pitch = pp_cifhr_pitch(a.ww);
    a.stride = (float)cfg->stride;
    a.th = cfg->seed_threshold;
    a.score_scale = cfg->seed_score_scale;
    a.seeds = seeds;
    a.cap = cap;
    a.counts = counts;
    int np = 1;
    while (np < cap) np <<= 1;
    a.np_cap = np;
    char *w = (char *)scratch;
    a.g_keys = (float *)w;
    w += round_up((int64_t)n_img * 4 * cap * sizeof(float), 256);
    a.g_f = (int *)w;
    w += round_up((int64_t)n_img * cap * sizeof(int), 256);
    a.g_perm = (int *)w;
    hipLaunchKernelGGL(seeds_kernel, dim3(n_img), dim3(256), 0, s, a);
    return check_launch("pp_seeds");
}

size_t seeds_scratch_size(int n_img, int cap) {
    int64_t np = 1;
    while (np < cap) np <<= 1;
    return round_up((int64_t)n_img * 4 * cap * sizeof(float), 256) +
           round_up((int64_t)n_img * cap * sizeof(int), 256) +
           round_up((int64_t)n_img * np * sizeof(int), 256);
}

int launch_caf_scored(const float *caf, const float *hr, int n_img, int K, int C, int H, int W,
                      const int32_t *skeleton, const pp_config *cfg, int nt, const float *th,
                      float *const *cols, int *const *counts, hipStream_t s) {
    if (C > kMaxCaf) return fail(PP_ESHAPE, "caf_scored: more than PP_MAX_EDGES CAF fields");
    CafArgs a{};
    a.caf = caf;
    a.hr = hr;
    a.K = K;
    a.C = C;
    a.H = H;
    a.W = W;
    a.hh = (int)hr_dim(H, cfg->stride);
    a.ww = (int)hr_dim(W, cfg->stride);
    a.pitch = pp_cifhr_pitch(a.ww);
    a.stride = (float)cfg->stride;
    a.cif_floor = cfg->cif_floor;
    a.one_minus_floor = (float)(1.0 - (double)cfg->cif_floor);  // (1.0 - self.cif_floor)
    a.nt = nt;
    for (int t = 0; t < nt; t++) {
        a.th[t] = th[t];
        a.cols[t] = cols[t];
        a.counts[t] = counts[t];
    }
    for (int i = 0; i < C; i++) {
        a.j1[i] = skeleton[2 * i] - 1;
        a.j2[i] = skeleton[2 * i + 1] - 1;
        if (a.j1[i] < 0 || a.j2[i] < 0) return fail(PP_EINVAL, "caf_scored: skeleton is 1-based");
    }
    hipLaunchKernelGGL(caf_scored_kernel, dim3((unsigned)((int64_t)n_img * C)), dim3(256), 0, s, a);
    return check_launch("pp_caf_scored");
}

}  // namespace pp

using namespace pp;

extern "C" {

int pp_seeds(const float *d_cif, const float *d_cifhr, int32_t n_img, int32_t K, int32_t H,
             int32_t W, const pp_config *cfg, pp_seed *d_seeds, int32_t seed_capacity,
             int32_t *d_counts, void *stream) {
    if (!d_cif || !d_cifhr || !cfg || !d_seeds || !d_counts) return fail(PP_EINVAL, "pp_seeds: NULL argument");
    if (n_img < 0 || K <= 0 || H <= 0 || W <= 0 || seed_capacity <= 0)
        return fail(PP_ESHAPE, "pp_seeds: bad shape");
    if (n_img == 0) return PP_OK;
    void *scratch = nullptr;
    hipStream_t s = (hipStream_t)stream;
    if (hipMallocAsync(&scratch, seeds_scratch_size(n_img, seed_capacity), s) != hipSuccess)
        return fail(PP_EHIP, "pp_seeds: scratch allocation failed");
    int rc = launch_seeds(d_cif, d_cifhr, n_img, K, H, W, cfg, d_seeds, seed_capacity, d_counts,
                          scratch, s);
    hipFreeAsync(scratch, s);
    return rc;
}

int pp_caf_scored(const float *d_caf, const float *d_cifhr, int32_t n_img, int32_t K, int32_t C,
                  int32_t H, int32_t W, const int32_t *skeleton, float score_th,
                  const pp_config *cfg, float *d_cols, int32_t *d_counts, void *stream) {
    if (!d_caf || !d_cifhr || !skeleton || !cfg || !d_cols || !d_counts)
        return fail(PP_EINVAL, "pp_caf_scored: NULL argument");
    if (n_img < 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0) return fail(PP_ESHAPE, "pp_caf_scored: bad shape");
    if (n_img == 0) return PP_OK;
    float *cols[1] = {d_cols};
    int *counts[1] = {d_counts};
    return launch_caf_scored(d_caf, d_cifhr, n_img, K, C, H, W, skeleton, cfg, 1, &score_th, cols,
                             counts, (hipStream_t)stream);
}

}  // extern "C"
