// det.hip — the CifDet detection decoder (decoder/generator/cifdet.py:27-52) on gfx950.
//
//   pp_cifdet_hr (splat.hip)   CifDetHr: the CifHr gather-fold with detection sigmas
//   det_seeds_emit_kernel      CifDetSeeds.fill_cif (cif_seeds.py:67-90) per (image, field)
//   det_select_kernel          per (image, field): the field's seeds sorted as the reference
//                              orders them, then the occupancy loop of cifdet.py:38-45.
//                              Occupancy planes are per field, so each field is independent;
//                              marks are kept as a list of boxes and a seed is occupied iff
//                              the number of boxes covering its cell is non-zero mod 256
//                              (the reference's u8 grid wraps)
//   det_output_kernel          per image: kept seeds merged into the global seed order,
//                              AnnotationDet boxes, nms.Detection (nms.py:79-102) in float32
//                              as NumPy evaluates it, output records
#include "pp_common.hpp"

#include <math.h>

namespace pp {

constexpr int kDetSortLds = 4096;  // seeds of one field sorted in LDS (global beyond)
constexpr int kDetBoxLds = 1024;   // marked boxes of one field kept in LDS (global beyond)

struct DetArgs {
    Heads hd;              // the detection heads (CIF role, (n_img, K, 7, H, W) each), in
                           // cif_indices order
    const float *hr;       // (n_img, K, hh, pitch): the CifDetHr map (head 0's size)
    int K, hh, ww;
    int cells;             // segment plane size: the heads' H * W summed
    int64_t pitch;
    float th, score_scale;
    uint32_t skip;         // pp_config.seed_skip_mask (cif_seeds.py:70-71 seed_mask)
    // per (image, field) segments: v, x, y, w, h (each `cells`) and counts
    float *seg;
    int *seg_n;
    uint64_t *gkeys;       // (n_img * K, cells) global sort keys beyond kDetSortLds
    int2 *gbox;            // (n_img * K, cells) boxes beyond kDetBoxLds
    int *kept;             // (n_img * K, cells) kept seeds (emission indices), in sorted order
    int *kept_n;
    int oh, ow;            // occupancy grid (cifhr.shape / 2)
    // per image
    int cap;               // detections per image
    float *cand;           // (n_img, cap, kCand)
    int *perm;             // (n_img, 3 * np_cap)
    int np_cap;
    pp_det_nms nms;
    pp_det *out;
    int *counts;
    int *status;
};

__device__ __forceinline__ int64_t seg_base(const DetArgs &a, int64_t fld) {
    return fld * 5 * (int64_t)a.cells;
}

// CifDetSeeds.fill (cif_seeds.py:56-64 over the heads, 67-90 per head) for one field: the
// heads in order, each one's cells in row-major order, appended to the field's segment
__global__ __launch_bounds__(256) void det_seeds_emit_kernel(DetArgs a) {
    __shared__ int s_tmp[4];
    const int64_t fld = blockIdx.x;
    const int img = (int)(fld / a.K), f = (int)(fld % a.K);
    const int64_t cells = a.cells;
    const float *t = a.hr + ((int64_t)img * a.K + f) * a.hh * a.pitch;
    float *sv = a.seg + seg_base(a, fld), *sx = sv + cells, *sy = sx + cells, *sw = sy + cells,
          *sh = sw + cells;
    int running = 0;
    const int n_heads = ((a.skip >> f) & 1u) ? 0 : a.hd.n_cif;  // a masked field emits nothing
    for (int m = 0; m < n_heads; m++) {
        const int hw = a.hd.cH[m] * a.hd.cW[m];
        const float *p = a.hd.cif[m] + fld * 7 * (int64_t)hw;
        const float stride = (float)a.hd.cstride[m];
        // `if min_scale:` p[4] > min_scale / stride, then p[5] (cif_seeds.py:75-77)
        const bool ms_on = (a.hd.ms_on >> m) & 1u;
        const float ms_th = a.hd.ms_th[m];
        for (int base = 0; base < hw; base += 256) {
            const int cell = base + threadIdx.x;
            bool keep = false;
            float v = 0.0f, x = 0.0f, y = 0.0f, w = 0.0f, h = 0.0f;
            if (cell < hw) {
                const float c = p[cell];
                // p[:, p[0] > threshold] (and the min-scale masks)
                if (c > a.th && (!ms_on || (p[4 * hw + cell] > ms_th && p[5 * hw + cell] > ms_th))) {
                    x = p[hw + cell] * stride;
                    y = p[2 * hw + cell] * stride;
                    const float hv = hr_lookup(t, a.hh, a.ww, a.pitch, x, y, 0.0f);
                    v = 0.9f * hv + 0.1f * c;
                    if (a.score_scale != 1.0f) v = v * a.score_scale;
                    keep = v > a.th;
                    w = p[4 * hw + cell] * stride;
                    h = p[5 * hw + cell] * stride;
                }
            }
            int total;
            const int slot = block_compact<4>(keep, s_tmp, total);
            if (keep) {
                const int q = running + slot;
                sv[q] = v;
                sx[q] = x;
                sy[q] = y;
                sw[q] = w;
                sh[q] = h;
            }
            running += total;
        }
    }
    if (threadIdx.x == 0) a.seg_n[fld] = running;
}

// Occupancy.set box (occupancy.py:31-39, utils.py:61-66) with reduction 2, min_scale 2.0
__device__ __forceinline__ bool det_box(int ow, int oh, float x, float y, float sigma, int2 &box) {
    const long xi = (long)rintf(x / 2.0f), yi = (long)rintf(y / 2.0f);  // round(): half to even
    const float sr = sigma / 2.0f;
    const long si = (long)rintf(sr > 1.0f ? sr : 1.0f);  // max(min_scale_reduced, sigma / r)
    const long minx = xi - si > 0 ? xi - si : 0;
    const long miny = yi - si > 0 ? yi - si : 0;
    const long mx = xi + si + 1 < ow ? xi + si + 1 : ow;
    const long my = yi + si + 1 < oh ? yi + si + 1 : oh;
    long maxx = minx + 1 > mx ? minx + 1 : mx;
    long maxy = miny + 1 > my ? miny + 1 : my;
    if (maxx > ow) maxx = ow;  // numpy slice clipping
    if (maxy > oh) maxy = oh;
    if (minx >= maxx || miny >= maxy) return false;
    box = make_int2((int)minx | ((int)maxx << 16), (int)miny | ((int)maxy << 16));
    return true;
}

__device__ __forceinline__ bool box_covers(int2 b, int xi, int yi) {
    return xi >= (b.x & 0xFFFF) && xi < (b.x >> 16) && yi >= (b.y & 0xFFFF) && yi < (b.y >> 16);
}

constexpr uint32_t kDetEmitMask = 0xFFFFFFFFu;

// one field: sort (v desc, then x, y, w, h desc, then emission) and run the occupancy loop
__global__ __launch_bounds__(256) void det_select_kernel(DetArgs a) {
    __shared__ uint64_t s_key[kDetSortLds];
    __shared__ int2 s_box[kDetBoxLds];
    const int64_t fld = blockIdx.x;
    const int hw = a.cells;
    const int n = a.seg_n[fld];
    const float *sv = a.seg + seg_base(a, fld), *sx = sv + hw, *sy = sx + hw, *sw = sy + hw,
                *sh = sw + hw;
    int np = 1;
    while (np < n) np <<= 1;
    uint64_t *key = np <= kDetSortLds ? s_key : a.gkeys + fld * (int64_t)hw;
    // seeds have v > threshold >= 0: float order == integer order of the bits
    for (int i = threadIdx.x; i < np; i += 256)
        key[i] = i < n ? ((uint64_t)__float_as_uint(sv[i]) << 32) | (kDetEmitMask - (uint32_t)i) : 0;
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t ka = key[i], kb = key[ixj];
                    const bool desc = (i & k) == 0;
                    if (desc ? ka < kb : ka > kb) {
                        key[i] = kb;
                        key[ixj] = ka;
                    }
                }
            }
            __syncthreads();
        }
    }
    // equal v: the reference's tuple order goes on to x, y, w, h (descending), then the
    // emission order (stable)
    for (int i = threadIdx.x; i < n; i += 256) {
        const uint32_t vi = (uint32_t)(key[i] >> 32);
        const bool tie_prev = i > 0 && (uint32_t)(key[i - 1] >> 32) == vi;
        const bool tie_next = i + 1 < n && (uint32_t)(key[i + 1] >> 32) == vi;
        if (tie_prev || !tie_next) continue;
        int end = i + 1;
        while (end < n && (uint32_t)(key[end] >> 32) == vi) end++;
        auto before = [&](uint64_t p, uint64_t q) {
            const int ep = (int)(kDetEmitMask - (uint32_t)p), eq = (int)(kDetEmitMask - (uint32_t)q);
            if (sx[ep] != sx[eq]) return sx[ep] > sx[eq];
            if (sy[ep] != sy[eq]) return sy[ep] > sy[eq];
            if (sw[ep] != sw[eq]) return sw[ep] > sw[eq];
            if (sh[ep] != sh[eq]) return sh[ep] > sh[eq];
            return ep < eq;
        };
        for (int u = i + 1; u < end; u++) {
            const uint64_t cur = key[u];
            int w = u;
            while (w > i && before(cur, key[w - 1])) {
                key[w] = key[w - 1];
                w--;
            }
            key[w] = cur;
        }
    }
    __syncthreads();
    if (threadIdx.x >= 64) return;
    // cifdet.py:38-45 on this field's plane, one wave: 64 seeds per step
    const int lane = threadIdx.x;
    int2 *boxes = n <= kDetBoxLds ? s_box : a.gbox + fld * (int64_t)hw;
    int *kept = a.kept + fld * (int64_t)hw;
    int nbox = 0, nk = 0;
    for (int base = 0; base < n; base += 64) {
        const int pos = base + lane;
        const bool valid = pos < n;
        int e = 0, xi = 0, yi = 0;
        float x = 0.0f, y = 0.0f, w = 0.0f, h = 0.0f;
        if (valid) {
            e = (int)(kDetEmitMask - (uint32_t)key[pos]);
            x = sx[e];
            y = sy[e];
            w = sw[e];
            h = sh[e];
        }
        bool fixed_free = a.oh <= 0 || a.ow <= 0;  // the reference reads out of bounds here
        if (!fixed_free) {
            xi = (int)clip_ref(x / 2.0f, 0.0f, (float)(a.ow - 1));
            yi = (int)clip_ref(y / 2.0f, 0.0f, (float)(a.oh - 1));
        }
        int cnt = 0;
        for (int q = 0; q < nbox; q++) cnt += box_covers(boxes[q], xi, yi);
        int last = -1;
        for (;;) {
            const bool free_ = valid && (fixed_free || (cnt & 255) == 0) && lane > last;
            const uint64_t m = __ballot(free_);
            if (!m) break;
            const int l = __ffsll((unsigned long long)m) - 1;
            const float bx = __shfl(x, l), by = __shfl(y, l), bw = __shfl(w, l), bh = __shfl(h, l);
            const int ke = __shfl(e, l);  // full exec: never shuffle under a branch
            if (lane == 0) kept[nk] = ke;  // the seed's emission index in the segment
            nk++;
            const float mwh = bh < bw ? bh : bw;  // builtin min(w, h)
            int2 b;
            if (!fixed_free && det_box(a.ow, a.oh, bx, by, 0.1f * mwh, b)) {
                if (lane == 0) boxes[nbox] = b;
                nbox++;
                cnt += box_covers(b, xi, yi);
            }
            last = l;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) a.kept_n[fld] = nk;
}

// NumPy's float32 np.maximum / np.minimum (NaN propagates)
__device__ __forceinline__ float npmax(float p, float q) { return (p != p || q != q) ? NAN : (p > q ? p : q); }
__device__ __forceinline__ float npmin(float p, float q) { return (p != p || q != q) ? NAN : (p < q ? p : q); }

// nms.Detection.bbox_iou for one pair (nms.py:67-77)
__device__ __forceinline__ float det_iou(float b0, float b1, float b2, float b3, float o0, float o1,
                                         float o2, float o3) {
    const float x1 = npmax(b0, o0), y1 = npmax(b1, o1);
    const float x2 = npmin(b0 + b2, o0 + o2), y2 = npmin(b1 + b3, o1 + o3);
    const float inter = npmax(0.0f, x2 - x1) * npmax(0.0f, y2 - y1);
    const float ba = b2 * b3, oa = o2 * o3;
    return inter / (((ba + oa) - inter) + 1e-5f);
}

// block-wide stable bitonic on perm[0..np) (entries >= n sort last) with less(p, q)
template <typename Less>
__device__ void block_sort(int *perm, int np, int n, Less less) {
    for (int i = threadIdx.x; i < np; i += blockDim.x) perm[i] = i;
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int p = perm[i], q = perm[ixj];
                    auto before = [&](int u, int v) {
                        if (u >= n) return false;
                        if (v >= n) return true;
                        if (less(u, v)) return true;
                        if (less(v, u)) return false;
                        return u < v;  // stable
                    };
                    const bool asc = (i & k) == 0;
                    if (asc ? before(q, p) : before(p, q)) {
                        perm[i] = q;
                        perm[ixj] = p;
                    }
                }
            }
            __syncthreads();
        }
    }
}

constexpr int kCand = 10;  // candidate: v f x y w h e score bx by (bbox = bx, by, w, h)

// nms.Detection.annotations (nms.py:79-102) on cand[order[0..n)] (the list order), then the
// records: out[r] for r < returned count, out_index[r] = the candidate's e.  Block-wide.
__device__ int det_nms_output(const DetArgs &a, int img, float *cand, int *perm, int *perm2,
                              const int *order, int n, pp_det *out, int *out_index) {
    __shared__ int s_m;
    const pp_det_nms &z = a.nms;
    int m = n;
    if (threadIdx.x == 0) {  // list order, or the kept subset in list order
        int k = 0;
        for (int r = 0; r < n; r++)
            if (!z.apply || cand[kCand * order[r] + 7] >= z.instance_threshold) perm2[k++] = order[r];
        s_m = k;
    }
    __syncthreads();
    m = s_m;
    int *rank = perm2 + a.np_cap / 2;  // scratch (np_cap >= 2 * cap)
    if (z.apply) {
        int npm = 1;
        while (npm < m) npm <<= 1;
        block_sort(rank, npm, m, [&](int p, int q) {  // sorted(key=-score), stable
            return -cand[kCand * perm2[p] + 7] < -cand[kCand * perm2[q] + 7];
        });
        for (int i = threadIdx.x; i < m; i += blockDim.x) perm[i] = perm2[rank[i]];
        __syncthreads();
        // nms.py:86-95: sequential over the sorted detections, IoU against the earlier ones
        // still above the threshold (with their current scores)
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            for (int i = 1; i < m; i++) {
                const float *ci = cand + kCand * perm[i];
                float mx = -INFINITY;
                bool nan = false;
                for (int j = lane; j < i; j += 64) {
                    const float *cj = cand + kCand * perm[j];
                    if (!(cj[7] >= z.instance_threshold)) continue;
                    const float iou = det_iou(ci[8], ci[9], ci[4], ci[5], cj[8], cj[9], cj[4], cj[5]);
                    if (iou != iou)
                        nan = true;
                    else
                        mx = iou > mx ? iou : mx;
                }
                for (int off = 32; off > 0; off >>= 1) {  // wave max; np.max is NaN if any is
                    const float o = __shfl_xor(mx, off);
                    mx = o > mx ? o : mx;
                }
                const float mi = __ballot(nan) ? NAN : mx;
                if (lane == 0) {
                    float sc = ci[7];
                    if (mi > z.iou_threshold)
                        sc = sc * z.suppression;
                    else if (mi > z.iou_threshold_soft)
                        sc = sc * z.suppression_soft;
                    cand[kCand * perm[i] + 7] = sc;
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // nms.py:97-98: filter again, sort again
            int k = 0;
            for (int r = 0; r < m; r++)
                if (cand[kCand * perm[r] + 7] >= z.instance_threshold) perm2[k++] = perm[r];
            s_m = k;
        }
        __syncthreads();
        m = s_m;
        npm = 1;
        while (npm < m) npm <<= 1;
        block_sort(rank, npm, m, [&](int p, int q) {
            return -cand[kCand * perm2[p] + 7] < -cand[kCand * perm2[q] + 7];
        });
        for (int i = threadIdx.x; i < m; i += blockDim.x) rank[i] = perm2[rank[i]];
        __syncthreads();
    } else {
        for (int i = threadIdx.x; i < m; i += blockDim.x) rank[i] = perm2[i];
        __syncthreads();
    }
    for (int r = threadIdx.x; r < m; r += blockDim.x) {
        const float *c = cand + kCand * rank[r];
        pp_det d;
        d.field = (int)c[1];
        d.score = c[7];
        d.bbox[0] = c[8];
        d.bbox[1] = c[9];
        d.bbox[2] = c[4];
        d.bbox[3] = c[5];
        d.image = img;
        d.pad_ = 0;
        out[r] = d;
        if (out_index) out_index[r] = (int)c[6];
    }
    __syncthreads();
    return m;
}

// kept seeds -> AnnotationDet in the global seed order -> nms.Detection -> records
__global__ __launch_bounds__(256) void det_output_kernel(DetArgs a) {
    __shared__ int s_n, s_status;
    const int img = blockIdx.x;
    const int hw = a.cells;
    float *cand = a.cand + (int64_t)img * a.cap * kCand;
    int *perm = a.perm + (int64_t)img * 3 * a.np_cap, *perm2 = perm + a.np_cap,
        *order = perm2 + a.np_cap;
    if (threadIdx.x == 0) {
        int n = 0, st = 0;
        for (int f = 0; f < a.K; f++) {
            const int64_t fld = (int64_t)img * a.K + f;
            const int nk = a.kept_n[fld];
            const float *sv = a.seg + seg_base(a, fld), *sx = sv + hw, *sy = sx + hw,
                        *sw = sy + hw, *sh = sw + hw;
            const int *kept = a.kept + fld * (int64_t)hw;
            for (int k = 0; k < nk; k++) {
                if (n >= a.cap) {
                    st |= PP_ST_ANN_OVERFLOW;
                    break;
                }
                const int e = kept[k];
                float *c = cand + kCand * n;
                c[0] = sv[e];
                c[1] = (float)f;
                c[2] = sx[e];
                c[3] = sy[e];
                c[4] = sw[e];
                c[5] = sh[e];
                c[6] = (float)e;
                c[7] = sv[e];
                c[8] = sx[e] - sw[e] / 2.0f;  // AnnotationDet bbox (x - w / 2.0, y - h / 2.0, w, h)
                c[9] = sy[e] - sh[e] / 2.0f;
                n++;
            }
        }
        s_n = n;
        s_status = st;
    }
    __syncthreads();
    const int n = s_n;
    int np = 1;
    while (np < n) np <<= 1;
    // the global seed order: sorted(seeds, reverse=True) on (v, f, x, y, w, h), stable
    block_sort(order, np, n, [&](int p, int q) {
        const float *cp = cand + kCand * p, *cq = cand + kCand * q;
        for (int t = 0; t < 6; t++)
            if (cp[t] != cq[t]) return cp[t] > cq[t];
        return cp[6] < cq[6];  // same field: emission (cell) order
    });
    const int m = det_nms_output(a, img, cand, perm, perm2, order, n,
                                 a.out + (int64_t)img * a.cap, nullptr);
    if (threadIdx.x == 0) {
        a.counts[img] = m;
        a.status[img] = s_status;
    }
}

// standalone nms.Detection over caller records (input order = list order)
__global__ __launch_bounds__(256) void det_nms_kernel(DetArgs a, const pp_det *in, const int *in_n,
                                                      int *out_index, float *scores_out) {
    const int img = blockIdx.x;
    const int n = min(max(in_n[img], 0), a.cap);
    float *cand = a.cand + (int64_t)img * a.cap * kCand;
    int *perm = a.perm + (int64_t)img * 3 * a.np_cap, *perm2 = perm + a.np_cap,
        *order = perm2 + a.np_cap;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const pp_det d = in[(int64_t)img * a.cap + i];
        float *c = cand + kCand * i;
        c[0] = d.score;
        c[1] = (float)d.field;
        c[2] = c[3] = 0.0f;
        c[4] = d.bbox[2];
        c[5] = d.bbox[3];
        c[6] = (float)i;
        c[7] = d.score;
        c[8] = d.bbox[0];
        c[9] = d.bbox[1];
        order[i] = i;
    }
    __syncthreads();
    const int m = det_nms_output(a, img, cand, perm, perm2, order, n, a.out + (int64_t)img * a.cap,
                                 out_index ? out_index + (int64_t)img * a.cap : nullptr);
    if (threadIdx.x == 0) a.counts[img] = m;
    if (scores_out) {  // every input's score after the in-place edits (nms.py:90-99)
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x)
            scores_out[(int64_t)img * a.cap + i] = cand[kCand * i + 7];
    }
}

static inline size_t align_up(size_t v) { return (v + 255) / 256 * 256; }

struct DetLayout {
    size_t off_hr, off_hr_ws, off_seg, off_seg_n, off_keys, off_box, off_kept, off_kept_n,
        off_cand, off_perm, total;
    int64_t pitch;
    size_t hr_ws;
    int np_cap;
};

static DetLayout det_layout(const Heads &h, int n_img, int K, int cap) {
    DetLayout d{};
    const int hh = h.hr_hh, ww = h.hr_ww;
    d.pitch = pp_cifhr_pitch(ww);
    d.hr_ws = cifhr_heads_workspace_size(h, n_img, K);
    d.np_cap = 1;
    while (d.np_cap < 2 * cap) d.np_cap <<= 1;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += align_up(bytes);
        return at;
    };
    const size_t nf = (size_t)n_img * K, cells = (size_t)h.cif_cells();
    d.off_hr = take((size_t)n_img * K * hh * d.pitch * sizeof(float));
    d.off_hr_ws = take(d.hr_ws);
    d.off_seg = take(nf * 5 * cells * sizeof(float));
    d.off_seg_n = take(nf * sizeof(int));
    d.off_keys = take(nf * cells * sizeof(uint64_t));
    d.off_box = take(nf * cells * sizeof(int2));
    d.off_kept = take(nf * cells * sizeof(int));
    d.off_kept_n = take(nf * sizeof(int));
    d.off_cand = take((size_t)n_img * cap * 10 * sizeof(float));
    d.off_perm = take((size_t)n_img * 3 * d.np_cap * sizeof(int));
    d.total = o;
    return d;
}

// the seeds' arguments over a head list (pp_cifdet_seeds*, pp_cifdet_decode*)
static DetArgs det_seed_args(const Heads &h, const float *hr, int K, const pp_config *cfg,
                             float *seg, int *seg_n) {
    DetArgs a{};
    a.hd = h;
    a.hr = hr;
    a.K = K;
    a.hh = h.hr_hh;
    a.ww = h.hr_ww;
    a.cells = (int)h.cif_cells();
    a.pitch = pp_cifhr_pitch(a.ww);
    a.th = cfg->seed_threshold;
    a.skip = cfg->seed_skip_mask;
    a.score_scale = cfg->seed_score_scale;
    a.seg = seg;
    a.seg_n = seg_n;
    return a;
}

static int det_seeds_launch(const Heads &h, const float *d_cifhr, int32_t n_img, int32_t K,
                            const pp_config *cfg, float *d_seg, int32_t *d_seg_counts,
                            hipStream_t s, const char *who) {
    if (!d_cifhr || !cfg || !d_seg || !d_seg_counts)
        return fail(PP_EINVAL, std::string(who) + ": NULL argument");
    for (int m = 0; m < h.n_cif; m++)
        if (!h.cif[m]) return fail(PP_EINVAL, std::string(who) + ": NULL field");
    if (n_img < 0 || K <= 0) return fail(PP_ESHAPE, std::string(who) + ": bad shape");
    if (h.cif_cells() >= (int64_t)1 << 31) return fail(PP_ESHAPE, std::string(who) + ": too many cells");
    if (n_img == 0) return PP_OK;
    const DetArgs a = det_seed_args(h, d_cifhr, K, cfg, d_seg, d_seg_counts);
    hipLaunchKernelGGL(det_seeds_emit_kernel, dim3((unsigned)((int64_t)n_img * K)), dim3(256), 0,
                       s, a);
    return check_launch(who);
}

static int det_decode_launch(const Heads &h, int32_t n_img, int32_t K, const pp_config *cfg,
                             const pp_det_nms *nms, float *d_cifhr, pp_det *d_out,
                             int32_t det_capacity, int32_t *d_counts, int32_t *d_status,
                             void *d_workspace, size_t workspace_bytes, hipStream_t s,
                             const char *who) {
    if (!cfg || !nms || !d_out || !d_counts || !d_status || !d_workspace)
        return fail(PP_EINVAL, std::string(who) + ": NULL argument");
    for (int m = 0; m < h.n_cif; m++)
        if (!h.cif[m]) return fail(PP_EINVAL, std::string(who) + ": NULL field");
    if (n_img < 0 || K <= 0 || K > 4096 || det_capacity <= 0)
        return fail(PP_ESHAPE, std::string(who) + ": bad shape");
    if (h.cif_cells() >= (int64_t)1 << 31) return fail(PP_ESHAPE, std::string(who) + ": too many cells");
    if (!(cfg->seed_threshold >= 0.0f))
        return fail(PP_EINVAL, std::string(who) + ": seed_threshold must be >= 0");
    if (n_img == 0) return PP_OK;
    const DetLayout d = det_layout(h, n_img, K, det_capacity);
    if (workspace_bytes < d.total) return fail(PP_ENOMEM, std::string(who) + ": workspace too small");
    const int hh = h.hr_hh, ww = h.hr_ww;
    if (hh >= 65535 || ww >= 65535) return fail(PP_ESHAPE, std::string(who) + ": field too large");
    char *ws = (char *)d_workspace;
    float *hr = d_cifhr ? d_cifhr : (float *)(ws + d.off_hr);
    int rc = cifhr_heads_launch<true>(h, n_img, K, cfg, hr, ws + d.off_hr_ws, d.hr_ws, s, who);
    if (rc) return rc;
    DetArgs a = det_seed_args(h, hr, K, cfg, (float *)(ws + d.off_seg), (int *)(ws + d.off_seg_n));
    a.gkeys = (uint64_t *)(ws + d.off_keys);
    a.gbox = (int2 *)(ws + d.off_box);
    a.kept = (int *)(ws + d.off_kept);
    a.kept_n = (int *)(ws + d.off_kept_n);
    a.oh = (int)((double)hh / 2.0);  // Occupancy(cifhr.shape, 2, min_scale=2.0)
    a.ow = (int)((double)ww / 2.0);
    a.cap = det_capacity;
    a.cand = (float *)(ws + d.off_cand);
    a.perm = (int *)(ws + d.off_perm);
    a.np_cap = d.np_cap;
    a.nms = *nms;
    a.out = d_out;
    a.counts = d_counts;
    a.status = d_status;
    const unsigned nf = (unsigned)((int64_t)n_img * K);
    hipLaunchKernelGGL(det_seeds_emit_kernel, dim3(nf), dim3(256), 0, s, a);
    hipLaunchKernelGGL(det_select_kernel, dim3(nf), dim3(256), 0, s, a);
    hipLaunchKernelGGL(det_output_kernel, dim3((unsigned)n_img), dim3(256), 0, s, a);
    return check_launch(who);
}

}  // namespace pp

using namespace pp;

extern "C" {

void pp_default_det_nms(pp_det_nms *z) {
    if (!z) return;
    z->suppression = 0.1f;
    z->suppression_soft = 0.3f;
    z->instance_threshold = 0.1f;
    z->iou_threshold = 0.7f;
    z->iou_threshold_soft = 0.5f;
    z->apply = 1;
}

int pp_cifdet_seeds(const float *d_det, const float *d_cifhr, int32_t n_img, int32_t K, int32_t H,
                    int32_t W, const pp_config *cfg, float *d_seg, int32_t *d_seg_counts,
                    void *stream) {
    if (!d_det || !cfg) return fail(PP_EINVAL, "pp_cifdet_seeds: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_cifdet_seeds: bad shape");
    return det_seeds_launch(single_head(d_det, nullptr, H, W, cfg->stride), d_cifhr, n_img, K, cfg,
                            d_seg, d_seg_counts, (hipStream_t)stream, "pp_cifdet_seeds");
}

int pp_cifdet_seeds_multi(const pp_scale *scales, int32_t n_scales, const float *d_cifhr,
                          int32_t n_img, int32_t K, const pp_config *cfg, float *d_seg,
                          int32_t *d_seg_counts, void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, 0, PP_ROLE_CIF, &h, "pp_cifdet_seeds_multi");
    if (rc) return rc;
    return det_seeds_launch(h, d_cifhr, n_img, K, cfg, d_seg, d_seg_counts, (hipStream_t)stream,
                            "pp_cifdet_seeds_multi");
}

size_t pp_nms_detection_workspace_size(int32_t n_img, int32_t capacity) {
    if (n_img < 0 || capacity <= 0) return 0;
    int np = 1;
    while (np < 2 * capacity) np <<= 1;
    return align_up((size_t)n_img * capacity * 10 * sizeof(float)) +
           align_up((size_t)n_img * 3 * np * sizeof(int));
}

int pp_nms_detection(const pp_det *d_in, const int32_t *d_counts, int32_t n_img, int32_t capacity,
                     const pp_det_nms *nms, pp_det *d_out, int32_t *d_out_counts,
                     int32_t *d_out_index, float *d_scores_out, void *d_workspace,
                     size_t workspace_bytes, void *stream) {
    if (!d_in || !d_counts || !nms || !d_out || !d_out_counts || !d_workspace)
        return fail(PP_EINVAL, "pp_nms_detection: NULL argument");
    if (n_img < 0 || capacity <= 0) return fail(PP_ESHAPE, "pp_nms_detection: bad shape");
    if (n_img == 0) return PP_OK;
    if (workspace_bytes < pp_nms_detection_workspace_size(n_img, capacity))
        return fail(PP_ENOMEM, "pp_nms_detection: workspace too small");
    DetArgs a{};
    a.cap = capacity;
    a.np_cap = 1;
    while (a.np_cap < 2 * capacity) a.np_cap <<= 1;
    a.cand = (float *)d_workspace;
    a.perm = (int *)((char *)d_workspace + align_up((size_t)n_img * capacity * 10 * sizeof(float)));
    a.nms = *nms;
    a.out = d_out;
    a.counts = d_out_counts;
    hipLaunchKernelGGL(det_nms_kernel, dim3((unsigned)n_img), dim3(256), 0, (hipStream_t)stream, a,
                       d_in, d_counts, d_out_index, d_scores_out);
    return check_launch("pp_nms_detection");
}

size_t pp_cifdet_workspace_size(int32_t n_img, int32_t K, int32_t H, int32_t W,
                                const pp_config *cfg, int32_t det_capacity) {
    if (!cfg || n_img < 0 || K <= 0 || H <= 0 || W <= 0 || det_capacity <= 0 || cfg->stride <= 0)
        return 0;
    return det_layout(single_head(nullptr, nullptr, H, W, cfg->stride), n_img, K, det_capacity).total;
}

int pp_cifdet_decode(const float *d_det, int32_t n_img, int32_t K, int32_t H, int32_t W,
                     const pp_config *cfg, const pp_det_nms *nms, float *d_cifhr, pp_det *d_out,
                     int32_t det_capacity, int32_t *d_counts, int32_t *d_status,
                     void *d_workspace, size_t workspace_bytes, void *stream) {
    if (!d_det || !cfg) return fail(PP_EINVAL, "pp_cifdet_decode: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_cifdet_decode: bad shape");
    return det_decode_launch(single_head(d_det, nullptr, H, W, cfg->stride), n_img, K, cfg, nms,
                             d_cifhr, d_out, det_capacity, d_counts, d_status, d_workspace,
                             workspace_bytes, (hipStream_t)stream, "pp_cifdet_decode");
}

size_t pp_cifdet_multi_workspace_size(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                      int32_t n_img, int32_t K, int32_t det_capacity) {
    Heads h;
    if (make_heads(scales, n_scales, cif_pairs, PP_ROLE_CIF, &h, "pp_cifdet_multi_workspace_size") ||
        n_img < 0 || K <= 0 || det_capacity <= 0)
        return 0;
    return det_layout(h, n_img, K, det_capacity).total;
}

int pp_cifdet_decode_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                           int32_t n_img, int32_t K, const pp_config *cfg, const pp_det_nms *nms,
                           float *d_cifhr, pp_det *d_out, int32_t det_capacity, int32_t *d_counts,
                           int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                           void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, cif_pairs, PP_ROLE_CIF, &h, "pp_cifdet_decode_multi");
    if (rc) return rc;
    return det_decode_launch(h, n_img, K, cfg, nms, d_cifhr, d_out, det_capacity, d_counts,
                             d_status, d_workspace, workspace_bytes, (hipStream_t)stream,
                             "pp_cifdet_decode_multi");
}

}  // extern "C"
