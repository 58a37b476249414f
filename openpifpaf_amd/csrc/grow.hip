// grow.hip — the CifCaf greedy decoder (generator/cifcaf.py) as one gfx950 workgroup per image.
//
// The seed loop is sequential by construction (each annotation's occupancy marks decide
// whether later seeds start annotations, cifcaf.py:100-108), so an image is one wave64
// workgroup and a batch fills the chip with one workgroup per image.  Inside an image:
//
//   * the serial control (seed loop, lazy best-first frontier, force-complete, flood fill,
//     keypoint NMS) runs wave-uniformly with its state in LDS: the current annotation, the
//     frontier binary heap (cifcaf.py:248 PriorityQueue, same tuple order), the
//     by_source table (cifcaf.py:62-65, dict insertion order);
//   * caf_center_s + scoring (functional.pyx:338-359, cifcaf.py:124-145) is the parallel
//     part: 64 lanes stride the CAF column set with coalesced loads, each lane keeps its
//     top-2 (score, column) and a 6-step xor-shuffle merge yields the argsort top-2 that
//     _target_with_blend (cifcaf.py:157-192) needs;
//   * occupancy grids (occupancy.py, u8 += 1 with wrap) live in a per-image workspace that
//     every launch leaves zeroed: each box a launch marks is logged and cleared again.
//
// Float arithmetic is f32 op-for-op as NumPy evaluates it (NEP 50); np.exp is computed
// correctly rounded through f64.
#include "pp_common.hpp"

#include <stdio.h>
#include <stdlib.h>

// Diagnostic build only (-DPP_STAMPS, libpifpaf_amd_stamps.so): per-section shader-cycle
// sums of the decode kernel, dumped to $PP_STAMPS_OUT.  The product build compiles these
// to nothing.
#ifdef PP_STAMPS
#define STAMP_DECL                                                                          \
    uint64_t st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};                              \
    uint64_t st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                                            \
    do {                                                                                    \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                   \
        st_acc[i] += t_ - st_t;                                                             \
        st_t = t_;                                                                          \
    } while (0)
#define STAMP_FLUSH(ph)                                                                     \
    if (lane == 0 && g.stamps)                                                              \
        for (int q_ = 0; q_ < 12; q_++) g.stamps[((int64_t)img * 2 + (ph)-1) * 12 + q_] = st_acc[q_];
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH(ph)
#endif

namespace pp {

constexpr int kKP = PP_MAX_KP;
constexpr int kBS = 2 * PP_MAX_EDGES;       // by_source entries per joint (upper bound)
constexpr int kHeap = 4 * PP_MAX_EDGES + 8; // frontier entries per _grow call
constexpr int kOccMargin = 64;              // NMS occupancy slack beyond the main grid

struct HeapEntry {
    float neg;   // -score
    int eval;    // 0: (.., None, j, k)   1: (.., xysv, j, k)
    float xysv[4];
    int j, k;
};

struct FFEntry {  // _flood_fill frontier entry (-v, end_i, start_xyv, s)
    float neg;
    int end;
    float sxyv[3];
    float s;
};

struct OccLog {
    int f;
    int16_t x0, x1, y0, y1;
};

struct GrowArgs {
    const pp_seed *seeds;
    const int *seed_counts;
    int seed_cap;
    const float *cols[2];     // bucketed column sets (n_img, C, 2, 10, H*W): set A at
                              // caf_threshold, set B at complete_caf_threshold
    const int *offs[2];       // bucket boundaries (n_img, C, 2, nb + 1)
    int bw, bh, nb;           // bucket grid (see caf_bucketed_kernel)
    float inv_e;
    int K, C, H, W, hh, ww;
    int64_t hw;
    pp_config cfg;
    int skel[2 * PP_MAX_EDGES];
    // workspace (per image regions)
    uint8_t *occ;
    int64_t occ_cap;          // bytes per image
    OccLog *log;
    int log_cap;              // entries per image
    pp_ann *work;             // working annotations
    double *nms_score;        // (n_img, ann_cap)
    int *nms_idx;             // (n_img, 2 * ann_cap + ann_np)
    int ann_np;               // next pow2 >= ann_cap
    int ann_cap;
    uint64_t *stamps;         // diagnostic build: (n_img, 2, 12) cycle sums, else NULL
    int *n_work;              // (n_img) annotations after the seed loop (phase 1 -> 2)
    int *need_complete;       // (n_img) 1 if force-complete has work (gates the B columns)
    // outputs
    pp_ann *out;
    int *counts;
    int *status;
};

struct GrowLDS {
    pp_ann a;                  // current annotation
    HeapEntry heap[kHeap];
    FFEntry ff[kHeap];
    uint32_t in_frontier[kKP];
    int bs_n[kKP];
    uint8_t bs_k[kKP][kBS], bs_caf[kKP][kBS], bs_fwd[kKP][kBS];
    int seg_st[64], seg_pre[64];  // flattened bucket segments of one caf_center_s scan
    int mark_pre[kKP + 1];        // occupancy boxes of one annotation: area prefix
    int mark_box[kKP][4];
    double prod[kKP];             // Annotation.score() terms
    double score_bc;
    int heap_n;
    int ff_n;
    int log_n;
    int status;
};

// ---------------------------------------------------------------------------------------
// frontier heap (tuple order of cifcaf.py:261,281,285)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool heap_less(const HeapEntry &a, const HeapEntry &b) {
    if (a.neg != b.neg) return a.neg < b.neg;
    if (a.eval != b.eval) return a.eval < b.eval;  // reference raises TypeError here
    if (a.eval) {
        for (int t = 0; t < 4; t++)
            if (a.xysv[t] != b.xysv[t]) return a.xysv[t] < b.xysv[t];
    }
    if (a.j != b.j) return a.j < b.j;
    return a.k < b.k;
}

__device__ void heap_push(GrowLDS &L, const HeapEntry &x) {
    int i = L.heap_n;
    if (i >= kHeap) {
        L.status |= PP_ST_DEC_OVERFLOW;
        return;
    }
    L.heap_n = i + 1;
    while (i > 0) {
        const int p = (i - 1) >> 1;
        if (!heap_less(x, L.heap[p])) break;
        L.heap[i] = L.heap[p];
        i = p;
    }
    L.heap[i] = x;
}

__device__ HeapEntry heap_pop(GrowLDS &L) {
    const HeapEntry top = L.heap[0];
    const int n = L.heap_n - 1;
    L.heap_n = n;
    if (n > 0) {
        const HeapEntry x = L.heap[n];
        int i = 0;
        for (;;) {
            const int l = 2 * i + 1, r = l + 1;
            int m = i;
            const HeapEntry *mv = &x;
            if (l < n && heap_less(L.heap[l], *mv)) {
                m = l;
                mv = &L.heap[l];
            }
            if (r < n && heap_less(L.heap[r], *mv)) m = r;
            if (m == i) break;
            L.heap[i] = L.heap[m];
            i = m;
        }
        L.heap[i] = x;
    }
    return top;
}

__device__ __forceinline__ bool ff_less(const FFEntry &a, const FFEntry &b) {
    if (a.neg != b.neg) return a.neg < b.neg;
    if (a.end != b.end) return a.end < b.end;
    for (int t = 0; t < 3; t++)
        if (a.sxyv[t] != b.sxyv[t]) return a.sxyv[t] < b.sxyv[t];
    return a.s < b.s;
}

__device__ void ff_push(GrowLDS &L, const FFEntry &x) {
    int i = L.ff_n;
    if (i >= kHeap) {
        L.status |= PP_ST_DEC_OVERFLOW;
        return;
    }
    L.ff_n = i + 1;
    while (i > 0) {
        const int p = (i - 1) >> 1;
        if (!ff_less(x, L.ff[p])) break;
        L.ff[i] = L.ff[p];
        i = p;
    }
    L.ff[i] = x;
}

__device__ FFEntry ff_pop(GrowLDS &L) {
    const FFEntry top = L.ff[0];
    const int n = L.ff_n - 1;
    L.ff_n = n;
    if (n > 0) {
        const FFEntry x = L.ff[n];
        int i = 0;
        for (;;) {
            const int l = 2 * i + 1, r = l + 1;
            int m = i;
            const FFEntry *mv = &x;
            if (l < n && ff_less(L.ff[l], *mv)) {
                m = l;
                mv = &L.ff[l];
            }
            if (r < n && ff_less(L.ff[r], *mv)) m = r;
            if (m == i) break;
            L.ff[i] = L.ff[m];
            i = m;
        }
        L.ff[i] = x;
    }
    return top;
}

// ---------------------------------------------------------------------------------------
// _grow_connection: caf_center_s + scores + blend / max (cifcaf.py:124-192)
// ---------------------------------------------------------------------------------------
struct Top2 {
    float s1, s2;
    int o1, o2;  // column index in the reference's row-major order (tie-breaks)
    int k1, k2;  // storage slot (where the column's rows are)
};

// blend: top-2 of a stable ascending argsort (ties -> higher column ranks higher)
// max:   np.argmax (ties -> lower column)
template <bool MAXM>
__device__ __forceinline__ bool better(float sa, int ia, float sb, int ib) {
    if (ia < 0) return false;
    if (ib < 0) return true;
    if (sa != sb) return sa > sb;
    return MAXM ? ia < ib : ia > ib;
}

template <bool MAXM>
__device__ __forceinline__ void top2_insert(Top2 &t, float s, int o, int k) {
    if (better<MAXM>(s, o, t.s1, t.o1)) {
        t.s2 = t.s1;
        t.o2 = t.o1;
        t.k2 = t.k1;
        t.s1 = s;
        t.o1 = o;
        t.k1 = k;
    } else if (better<MAXM>(s, o, t.s2, t.o2)) {
        t.s2 = s;
        t.o2 = o;
        t.k2 = k;
    }
}

template <bool MAXM>
__device__ __forceinline__ void top2_wave_merge(Top2 &t) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float os1 = __shfl_xor(t.s1, off), os2 = __shfl_xor(t.s2, off);
        const int oo1 = __shfl_xor(t.o1, off), oo2 = __shfl_xor(t.o2, off);
        const int ok1 = __shfl_xor(t.k1, off), ok2 = __shfl_xor(t.k2, off);
        top2_insert<MAXM>(t, os1, oo1, ok1);
        top2_insert<MAXM>(t, os2, oo2, ok2);
    }
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(v, off);
        if (lane >= off) v += o;
    }
    return v;
}

struct ColQuery {
    float x, y, lo_x, hi_x, lo_y, hi_y, sigma2;
};

__device__ __forceinline__ ColQuery make_query(float x, float y, float xy_scale) {
    ColQuery q;
    const float sbox = 2.0f * xy_scale;  // caf_center_s(..., sigma=2.0 * xy_scale)
    q.x = x;
    q.y = y;
    q.lo_x = x - sbox;
    q.hi_x = x + sbox;
    q.lo_y = y - sbox;
    q.hi_y = y + sbox;
    const float sigma = 0.5f * xy_scale;
    q.sigma2 = sigma * sigma;
    return q;
}

// one column: caf_center_s test, then the score (cifcaf.py:134-139)
template <bool MAXM>
__device__ __forceinline__ void consider(const float *__restrict__ cf, int64_t hw, const ColQuery &q,
                                         int k, int o, Top2 &t, int &m) {
    const float c1 = cf[hw + k], c2 = cf[2 * hw + k];
    if (c1 < q.lo_x || c1 > q.hi_x || c2 < q.lo_y || c2 > q.hi_y) return;
    const float dx = q.x - c1, dy = q.y - c2;
    const float dd = sqrtf(dx * dx + dy * dy);  // np.linalg.norm(axis=0)
    const float qq = (-0.5f * (dd * dd)) / q.sigma2;
    const float score = (float)exp((double)qq) * cf[k];  // np.exp, correctly rounded
    m++;
    top2_insert<MAXM>(t, score, o, k);
}

// _target_with_blend / _target_with_maxscore (cifcaf.py:147-192) on the merged top-2
template <bool MAXM>
__device__ void finish_connection(const float *__restrict__ cf, int64_t hw, Top2 t, int m,
                                  float out[4]) {
    m = wave_sum(m);
    if (m == 0) {
        out[0] = out[1] = out[2] = out[3] = 0.0f;
        return;
    }
    top2_wave_merge<MAXM>(t);
    const float *t0 = cf + 5 * hw, *t1 = cf + 6 * hw, *t3 = cf + 8 * hw;
    const float x1 = t0[t.k1], y1 = t1[t.k1], sc1 = t3[t.k1];
    if (MAXM) {
        out[0] = x1;
        out[1] = y1;
        out[2] = sc1;
        out[3] = t.s1;
        return;
    }
    if (m == 1 || t.s2 < 0.01f || t.s2 < 0.5f * t.s1) {
        out[0] = x1;
        out[1] = y1;
        out[2] = sc1;
        out[3] = t.s1 * 0.5f;
        return;
    }
    const float x2 = t0[t.k2], y2 = t1[t.k2], sc2 = t3[t.k2];
    const float ex = x1 - x2, ey = y1 - y2;
    const float dist = sqrtf(ex * ex + ey * ey);
    if (dist > sc1 / 2.0f) {
        out[0] = x1;
        out[1] = y1;
        out[2] = sc1;
        out[3] = t.s1 * 0.5f;
        return;
    }
    const float ssum = t.s1 + t.s2;
    out[0] = (t.s1 * x1 + t.s2 * x2) / ssum;
    out[1] = (t.s1 * y1 + t.s2 * y2) / ssum;
    out[2] = (t.s1 * sc1 + t.s2 * sc2) / ssum;
    out[3] = 0.5f * (t.s1 + t.s2);
}

// column set in the reference's order, n columns (the functional API entry point)
template <bool MAXM>
__device__ void grow_connection_flat(const float *__restrict__ cf, int n, int64_t hw, float x,
                                     float y, float xy_scale, float out[4]) {
    const int lane = threadIdx.x & 63;
    const ColQuery q = make_query(x, y, xy_scale);
    Top2 t{0.0f, 0.0f, -1, -1, -1, -1};
    int m = 0;
    for (int i = lane; i < n; i += 64) consider<MAXM>(cf, hw, q, i, i, t, m);
    finish_connection<MAXM>(cf, hw, t, m, out);
}

// bucketed column set (caf_bucketed_kernel): visit only the buckets the 2*scale box
// overlaps (+ the NaN-source bucket), flattened over the 64 lanes
template <bool MAXM>
__device__ void grow_connection(const GrowArgs &g, GrowLDS &L, const float *__restrict__ cf,
                                const int *__restrict__ off, float x, float y, float xy_scale,
                                float out[4]) {
    const int lane = threadIdx.x & 63;
    const int64_t hw = g.hw;
    const ColQuery q = make_query(x, y, xy_scale);
    Top2 t{0.0f, 0.0f, -1, -1, -1, -1};
    int m = 0;
    int bx0, bx1, by0, by1;
    if (q.lo_x != q.lo_x || q.hi_x != q.hi_x || q.lo_y != q.lo_y || q.hi_y != q.hi_y) {
        bx0 = 0;  // NaN bounds pass every column (every comparison is false): scan all
        bx1 = g.bw - 1;
        by0 = 0;
        by1 = g.bh - 1;
    } else {
        bx0 = (int)fminf(fmaxf(floorf(q.lo_x * g.inv_e), 0.0f), (float)(g.bw - 1));
        bx1 = (int)fminf(fmaxf(floorf(q.hi_x * g.inv_e), 0.0f), (float)(g.bw - 1));
        by0 = (int)fminf(fmaxf(floorf(q.lo_y * g.inv_e), 0.0f), (float)(g.bh - 1));
        by1 = (int)fminf(fmaxf(floorf(q.hi_y * g.inv_e), 0.0f), (float)(g.bh - 1));
    }
    const int nseg = (by1 - by0 + 1) + 1;  // bucket rows + the NaN bucket
    for (int sb = 0; sb < nseg; sb += 64) {
        const int r = sb + lane;
        int st = 0, len = 0;
        if (r < nseg) {
            int lo, hi;
            if (r == nseg - 1) {
                lo = g.nb - 1;
                hi = g.nb;
            } else {
                const int row = by0 + r;
                lo = row * g.bw + bx0;
                hi = row * g.bw + bx1 + 1;
            }
            st = off[lo];
            len = off[hi] - st;
        }
        const int incl = wave_incl_scan(len);
        const int total = __shfl(incl, 63);
        L.seg_st[lane] = st;
        L.seg_pre[lane] = incl - len;
        __syncthreads();
        const int ng = min(64, nseg - sb);
        for (int tt = lane; tt < total; tt += 64) {
            int lo = 0, hi = ng - 1;  // largest segment whose start prefix <= tt
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (L.seg_pre[mid] <= tt)
                    lo = mid;
                else
                    hi = mid - 1;
            }
            const int k = L.seg_st[lo] + tt - L.seg_pre[lo];
            consider<MAXM>(cf, hw, q, k, __float_as_int(cf[9 * hw + k]), t, m);
        }
        __syncthreads();
    }
    finish_connection<MAXM>(cf, hw, t, m, out);
}

__device__ __forceinline__ float max0(float v) { return (v > 0.0f) ? v : 0.0f; }

__device__ __forceinline__ const float *col_set(const GrowArgs &g, int set, int img, int caf_i,
                                                int dir) {
    return g.cols[set] + (((int64_t)img * g.C + caf_i) * 2 + dir) * 10 * g.hw;
}

__device__ __forceinline__ const int *col_offs(const GrowArgs &g, int set, int img, int caf_i,
                                               int dir) {
    return g.offs[set] + (((int64_t)img * g.C + caf_i) * 2 + dir) * (int64_t)(g.nb + 1);
}

// cifcaf.py:194-217
__device__ void connection_value(const GrowArgs &g, GrowLDS &L, int img, int set, int start_i,
                                 int end_i, bool reverse_match, float out[4]) {
    int e = 0;
    for (int t = 0; t < L.bs_n[start_i]; t++)
        if (L.bs_k[start_i][t] == end_i) e = t;
    const int caf_i = L.bs_caf[start_i][e];
    const int fwd = L.bs_fwd[start_i][e];
    const int df = fwd ? 1 : 0, db = fwd ? 0 : 1;
    const float xv0 = L.a.data[start_i][0], xv1 = L.a.data[start_i][1], xv2 = L.a.data[start_i][2];
    const float xy_scale_s = max0(L.a.joint_scales[start_i]);
    const bool maxm = g.cfg.connection_method == 1;
    float nx[4];
    if (maxm)
        grow_connection<true>(g, L, col_set(g, set, img, caf_i, df), col_offs(g, set, img, caf_i, df),
                              xv0, xv1, xy_scale_s, nx);
    else
        grow_connection<false>(g, L, col_set(g, set, img, caf_i, df),
                               col_offs(g, set, img, caf_i, df), xv0, xv1, xy_scale_s, nx);
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    const float ks = sqrtf(nx[3] * xv2);  // geometric mean
    if (ks < g.cfg.keypoint_threshold) return;
    if (nx[3] == 0.0f) return;
    const float xy_scale_t = max0(nx[2]);
    if (reverse_match) {
        float rv[4];
        if (maxm)
            grow_connection<true>(g, L, col_set(g, set, img, caf_i, db),
                                  col_offs(g, set, img, caf_i, db), nx[0], nx[1], xy_scale_t, rv);
        else
            grow_connection<false>(g, L, col_set(g, set, img, caf_i, db),
                                   col_offs(g, set, img, caf_i, db), nx[0], nx[1], xy_scale_t, rv);
        if (rv[2] == 0.0f) return;  // tests the SCALE (cifcaf.py:212)
        if (fabsf(xv0 - rv[0]) + fabsf(xv1 - rv[1]) > xy_scale_s) return;
    }
    out[0] = nx[0];
    out[1] = nx[1];
    out[2] = nx[2];
    out[3] = ks;
}

__device__ void add_to_frontier(GrowLDS &L, int start_i) {
    for (int e = 0; e < L.bs_n[start_i]; e++) {
        const int end_i = L.bs_k[start_i][e];
        if (L.a.data[end_i][2] > 0.0f) continue;
        if (L.in_frontier[start_i] & (1u << end_i)) continue;
        HeapEntry x;
        x.neg = -sqrtf(L.a.data[start_i][2]);
        x.eval = 0;
        x.xysv[0] = x.xysv[1] = x.xysv[2] = x.xysv[3] = 0.0f;
        x.j = start_i;
        x.k = end_i;
        heap_push(L, x);
        L.in_frontier[start_i] |= 1u << end_i;
        const int t = L.a.n_frontier;
        if (t < PP_MAX_FRONTIER) {
            L.a.frontier_pairs[t][0] = (uint8_t)start_i;
            L.a.frontier_pairs[t][1] = (uint8_t)end_i;
        } else {
            L.status |= PP_ST_DEC_OVERFLOW;
        }
        L.a.n_frontier = t + 1;
    }
}

// cifcaf.py:247-307
__device__ void grow(const GrowArgs &g, GrowLDS &L, int img, int set, bool reverse_match) {
    L.heap_n = 0;
    for (int j = 0; j < kKP; j++) L.in_frontier[j] = 0u;
    for (int j = 0; j < g.K; j++) {
        if (L.a.data[j][2] == 0.0f) continue;
        add_to_frontier(L, j);
    }
    for (;;) {
        HeapEntry got;
        bool have = false;
        while (L.heap_n > 0) {
            const HeapEntry en = heap_pop(L);
            if (en.eval) {
                got = en;
                have = true;
                break;
            }
            if (L.a.data[en.k][2] > 0.0f) continue;
            float nx[4];
            connection_value(g, L, img, set, en.j, en.k, reverse_match, nx);
            if (nx[3] == 0.0f) continue;
            HeapEntry ev;
            ev.neg = -nx[3];
            ev.eval = 1;
            ev.xysv[0] = nx[0];
            ev.xysv[1] = nx[1];
            ev.xysv[2] = nx[2];
            ev.xysv[3] = nx[3];
            ev.j = en.j;
            ev.k = en.k;
            if (g.cfg.greedy) {
                got = ev;
                have = true;
                break;
            }
            heap_push(L, ev);
        }
        if (!have) break;
        const int jsi = got.j, jti = got.k;
        if (L.a.data[jti][2] > 0.0f) continue;
        L.a.data[jti][0] = got.xysv[0];
        L.a.data[jti][1] = got.xysv[1];
        L.a.data[jti][2] = got.xysv[3];
        L.a.joint_scales[jti] = got.xysv[2];
        const int t = L.a.n_decoding;
        if (t < kKP) {
            L.a.decoding_pairs[t][0] = (uint8_t)jsi;
            L.a.decoding_pairs[t][1] = (uint8_t)jti;
            for (int c = 0; c < 3; c++) {
                L.a.decoding_xyv[t][c] = L.a.data[jsi][c];
                L.a.decoding_xyv[t][3 + c] = L.a.data[jti][c];
            }
        } else {
            L.status |= PP_ST_DEC_OVERFLOW;
        }
        L.a.n_decoding = t + 1;
        add_to_frontier(L, jti);
    }
}

// cifcaf.py:309-331 (the key is the ENCLOSING xyv, App. D item 5)
__device__ void flood_fill(const GrowArgs &g, GrowLDS &L) {
    L.ff_n = 0;
    auto add = [&](int start_i, float key_v) {
        for (int e = 0; e < L.bs_n[start_i]; e++) {
            const int end_i = L.bs_k[start_i][e];
            if (L.a.data[end_i][2] > 0.0f) continue;
            FFEntry x;
            x.neg = -key_v;
            x.end = end_i;
            x.sxyv[0] = L.a.data[start_i][0];
            x.sxyv[1] = L.a.data[start_i][1];
            x.sxyv[2] = L.a.data[start_i][2];
            x.s = L.a.joint_scales[start_i];
            ff_push(L, x);
        }
    };
    for (int j = 0; j < g.K; j++) {
        if (L.a.data[j][2] == 0.0f) continue;
        add(j, L.a.data[j][2]);
    }
    while (L.ff_n > 0) {
        const FFEntry top = ff_pop(L);
        const int end_i = top.end;
        if (L.a.data[end_i][2] > 0.0f) continue;
        L.a.data[end_i][0] = top.sxyv[0];
        L.a.data[end_i][1] = top.sxyv[1];
        L.a.data[end_i][2] = 0.00001f;
        L.a.joint_scales[end_i] = top.s;
        add(end_i, top.sxyv[2]);
    }
}

// ---------------------------------------------------------------------------------------
// occupancy (occupancy.py:10-47, decoder/utils.py:61-66)
// ---------------------------------------------------------------------------------------
struct OccGrid {
    uint8_t *p;
    int f, h, w;
};

__device__ __forceinline__ long round_half_even(float x) { return (long)rintf(x); }

// Occupancy.get (occupancy.py:41-47): nonzero at floor((x, y) / reduction), clipped
__device__ bool occ_get(const OccGrid &o, int f, float x, float y, float red) {
    if (f >= o.f) return true;
    if (o.h <= 0 || o.w <= 0) return false;  // the reference reads out of bounds here
    x = clip_ref(x / red, 0.0f, (float)(o.w - 1));
    y = clip_ref(y / red, 0.0f, (float)(o.h - 1));
    const int xi = (int)x, yi = (int)y;
    return o.p[((int64_t)f * o.h + yi) * o.w + xi] != 0;
}

// Occupancy.set box (occupancy.py:31-39 + utils.py:61-66) of joint f; false when empty
__device__ bool occ_box(const GrowArgs &g, const OccGrid &o, int f, float x, float y, float sigma,
                        int box[4]) {
    if (f >= o.f) return false;
    const float red = (float)g.cfg.occupancy_reduction;
    const float msr = (float)((double)g.cfg.occupancy_min_scale / g.cfg.occupancy_reduction);
    const long xi = (long)rintf(x / red);  // round(): half to even
    const long yi = (long)rintf(y / red);
    const float sr = sigma / red;
    const long si = (long)rintf((sr > msr) ? sr : msr);  // max(min_scale_reduced, sigma / r)
    const long minx = xi - si > 0 ? xi - si : 0;
    const long miny = yi - si > 0 ? yi - si : 0;
    const long mx = xi + si + 1 < o.w ? xi + si + 1 : o.w;
    const long my = yi + si + 1 < o.h ? yi + si + 1 : o.h;
    long maxx = minx + 1 > mx ? minx + 1 : mx;
    long maxy = miny + 1 > my ? miny + 1 : my;
    if (maxx > o.w) maxx = o.w;  // numpy slice clipping
    if (maxy > o.h) maxy = o.h;
    if (minx >= maxx || miny >= maxy) return false;
    box[0] = (int)minx;
    box[1] = (int)maxx;
    box[2] = (int)miny;
    box[3] = (int)maxy;
    return true;
}

// Mark the boxes of every joint j with mark(j) in one pass: joints live on different
// occupancy planes, so the per-joint `+= 1` boxes are independent and spread over the 64
// lanes.  Each marked box is logged for occ_clear.  Collective (all 64 lanes).
template <typename MarkFn>
__device__ void occ_mark(const GrowArgs &g, GrowLDS &L, OccLog *log, const OccGrid &o,
                         const float (*xy)[3], const float *scales, int K, MarkFn mark) {
    const int lane = threadIdx.x & 63;
    int box[4] = {0, 0, 0, 0};
    bool has = false;
    if (lane < K && mark(lane)) has = occ_box(g, o, lane, xy[lane][0], xy[lane][1], scales[lane], box);
    const int area = has ? (box[1] - box[0]) * (box[3] - box[2]) : 0;
    const int incl = wave_incl_scan(area);
    const int total = __shfl(incl, 63);
    const uint64_t hm = __ballot(has);
    if (lane < K) {
        L.mark_pre[lane] = incl - area;
        L.mark_box[lane][0] = box[0];
        L.mark_box[lane][1] = box[1];
        L.mark_box[lane][2] = box[2];
        L.mark_box[lane][3] = box[3];
        if (has) {
            const int li = L.log_n + lane_prefix(hm);
            if (li < g.log_cap) {
                OccLog e;
                e.f = lane;
                e.x0 = (int16_t)box[0];
                e.x1 = (int16_t)box[1];
                e.y0 = (int16_t)box[2];
                e.y1 = (int16_t)box[3];
                log[li] = e;
            }
        }
    }
    __syncthreads();
    for (int t = lane; t < total; t += 64) {
        int lo = 0, hi = K - 1;  // largest joint whose area prefix <= t
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (L.mark_pre[mid] <= t)
                lo = mid;
            else
                hi = mid - 1;
        }
        const int u = t - L.mark_pre[lo];
        const int bw = L.mark_box[lo][1] - L.mark_box[lo][0];
        const int yy = L.mark_box[lo][2] + u / bw, xx = L.mark_box[lo][0] + u % bw;
        uint8_t *c = &o.p[((int64_t)lo * o.h + yy) * o.w + xx];
        *c = (uint8_t)(*c + 1);
    }
    const int nm = __popcll(hm);
    if (L.log_n + nm > g.log_cap) L.status |= PP_ST_NMS_OVERFLOW;
    __syncthreads();
    L.log_n = L.log_n + nm;
    __syncthreads();
}

// zero every box the launch marked, so the next launch starts from a clean grid
__device__ void occ_clear(const GrowArgs &g, GrowLDS &L, OccLog *log, const OccGrid &o) {
    __syncthreads();
    const int n = L.log_n < g.log_cap ? L.log_n : g.log_cap;
    const int lane = threadIdx.x & 63;
    for (int e0 = 0; e0 < n; e0 += 64) {  // 64 boxes per round, one per lane
        const int e = e0 + lane;
        OccLog l{0, 0, 0, 0, 0};
        if (e < n) l = log[e];
        const int area = (e < n) ? (l.x1 - l.x0) * (l.y1 - l.y0) : 0;
        for (int t = 0; t < area; t++) {
            const int bw = l.x1 - l.x0;
            o.p[((int64_t)l.f * o.h + l.y0 + t / bw) * o.w + l.x0 + t % bw] = 0;
        }
    }
    L.log_n = 0;
    __syncthreads();
}

// Annotation.score() (annotation.py:24-28, 60-71) in float64, collective over the wave:
// lane j finds the rank of v_j in descending order, the rank-ordered products go to LDS
// and NumPy's pairwise summation (n <= 128 path) adds them in its fixed order.
__device__ double ann_score(GrowLDS &L, const float (*data)[3], int K) {
    const int lane = threadIdx.x & 63;
    const double ws = (double)(3 * min(K, 3) + (K - min(K, 3)));  // np.sum(weights): exact
    if (lane < K) {
        const float vj = data[lane][2];
        int rank = 0;
        for (int i = 0; i < K; i++) {
            const float vi = data[i][2];
            rank += (vi > vj) || (vi == vj && i < lane);
        }
        const double w = (rank < 3 ? 3.0 : 1.0) / ws;
        L.prod[rank] = w * (double)vj;
    }
    __syncthreads();
    if (lane == 0) {
        const double *a = L.prod;
        double res;
        if (K < 8) {
            res = 0.0;
            for (int i = 0; i < K; i++) res += a[i];
        } else {
            double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6],
                   r7 = a[7];
            int i;
            for (i = 8; i < K - (K % 8); i += 8) {
                r0 += a[i];
                r1 += a[i + 1];
                r2 += a[i + 2];
                r3 += a[i + 3];
                r4 += a[i + 4];
                r5 += a[i + 5];
                r6 += a[i + 6];
                r7 += a[i + 7];
            }
            res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
            for (; i < K; i++) res += a[i];
        }
        L.score_bc = res;
    }
    __syncthreads();
    const double res = L.score_bc;
    __syncthreads();
    return res;
}

__device__ void copy_ann(pp_ann *dst, const pp_ann *src) {
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    constexpr int nw = sizeof(pp_ann) / 4;
    for (int t = threadIdx.x & 63; t < nw; t += 64) d[t] = s[t];
    __syncthreads();
}

// stable sort of idx[0..n) by descending score (sorted(anns, key=lambda a: -a.score()))
__device__ void sort_by_score(int *perm, int np, int n, const double *score) {
    for (int i = threadIdx.x & 63; i < np; i += 64) perm[i] = i;
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x & 63; i < np; i += 64) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const int a = perm[i], b = perm[ixj];
                    auto before = [&](int p, int q) {
                        if (p >= n) return false;
                        if (q >= n) return true;
                        const double kp = -score[p], kq = -score[q];
                        if (kp != kq) return kp < kq;
                        return p < q;
                    };
                    const bool asc = (i & k) == 0;
                    if (asc ? before(b, a) : before(a, b)) {
                        perm[i] = b;
                        perm[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------------------
// the per-image decode kernel
// ---------------------------------------------------------------------------------------
template <int PHASE>
__global__ __launch_bounds__(64) void grow_kernel(GrowArgs g) {
    __shared__ GrowLDS L;
    const int img = blockIdx.x;
    const int K = g.K;
    const int lane = threadIdx.x & 63;

    // by_source (cifcaf.py:62-65): dict insertion order, later duplicate keys overwrite
    if (lane == 0) {
        for (int j = 0; j < kKP; j++) L.bs_n[j] = 0;
        for (int ci = 0; ci < g.C; ci++) {
            const int j1 = g.skel[2 * ci] - 1, j2 = g.skel[2 * ci + 1] - 1;
            const int ins[2][3] = {{j1, j2, 1}, {j2, j1, 0}};
            for (int t = 0; t < 2; t++) {
                const int s = ins[t][0];
                int pos = -1;
                for (int e = 0; e < L.bs_n[s]; e++)
                    if (L.bs_k[s][e] == ins[t][1]) pos = e;
                if (pos < 0) pos = L.bs_n[s]++;
                L.bs_k[s][pos] = (uint8_t)ins[t][1];
                L.bs_caf[s][pos] = (uint8_t)ci;
                L.bs_fwd[s][pos] = (uint8_t)ins[t][2];
            }
        }
        L.status = PHASE == 1 ? 0 : g.status[img];
        L.log_n = 0;
    }
    __syncthreads();

    STAMP_DECL
    uint8_t *occ_base = g.occ + (int64_t)img * g.occ_cap;
    OccLog *log = g.log + (int64_t)img * g.log_cap;
    pp_ann *work = g.work + (int64_t)img * g.ann_cap;
    const float red = (float)g.cfg.occupancy_reduction;

    if (PHASE == 1) {
        // ---- seed loop (cifcaf.py:84-108) ----
        // The occupancy grid only changes when an annotation is created, so the occupancy
        // test of the next 64 seeds runs in parallel (one lane each) and the first free seed
        // starts the next annotation; the occupied ones before it are skipped exactly as the
        // sequential loop skips them.
        OccGrid occ{occ_base, K, (int)((double)g.hh / g.cfg.occupancy_reduction),
                    (int)((double)g.ww / g.cfg.occupancy_reduction)};
        const int n_seeds = min(g.seed_counts[img], g.seed_cap);
        const pp_seed *seeds = g.seeds + (int64_t)img * g.seed_cap;
        int n_anns = 0;
        bool need_complete = false;
        int s = 0;
        while (s < n_seeds) {
            const int idx = s + lane;
            bool is_free = false;
            if (idx < n_seeds) {
                const pp_seed c = seeds[idx];
                is_free = !occ_get(occ, c.field, c.x, c.y, red);
            }
            const uint64_t m = __ballot(is_free);
            STAMP(0);
            if (m == 0) {
                s += 64;
                continue;
            }
            const int si = s + __ffsll((unsigned long long)m) - 1;
            s = si + 1;
            const pp_seed sd = seeds[si];
            if (n_anns >= g.ann_cap) {
                L.status |= PP_ST_ANN_OVERFLOW;
                break;
            }
            // Annotation(keypoints, out_skeleton).add(f, (x, y, v)); joint_scales[f] = s
            {
                uint32_t *z = reinterpret_cast<uint32_t *>(&L.a);
                for (int t = lane; t < (int)(sizeof(pp_ann) / 4); t += 64) z[t] = 0u;
                __syncthreads();
            }
            if (lane == 0) {
                L.a.n_keypoints = K;
                L.a.image = img;
                L.a.data[sd.field][0] = sd.x;
                L.a.data[sd.field][1] = sd.y;
                L.a.data[sd.field][2] = sd.v;
                L.a.joint_scales[sd.field] = sd.s;
            }
            __syncthreads();
            STAMP(1);
            grow(g, L, img, 0, true);
            __syncthreads();
            STAMP(2);
            copy_ann(&work[n_anns], &L.a);
            n_anns++;
            STAMP(3);
            // mark_occupied (cifcaf.py:87-93): every joint with v != 0, in one pass
            for (int j = 0; j < K; j++) need_complete = need_complete || L.a.data[j][2] == 0.0f;
            occ_mark(g, L, log, occ, L.a.data, L.a.joint_scales, K,
                     [&](int j) { return L.a.data[j][2] != 0.0f; });
            STAMP(4);
        }
        occ_clear(g, L, log, occ);
        __syncthreads();
        STAMP(5);
        STAMP_FLUSH(1);
        if (lane == 0) {
            g.n_work[img] = n_anns;
            g.need_complete[img] = (g.cfg.force_complete && need_complete) ? 1 : 0;
            g.status[img] = L.status;
        }
        return;
    }
    const int n_anns = g.n_work[img];
    STAMP(0);

    // ---- complete_annotations (cifcaf.py:333-351) ----
    // Annotations with every joint set are unchanged by it (their frontier is empty), so
    // only images flagged by phase 1 run it, and only on annotations with a zero joint.
    if (g.cfg.force_complete && g.need_complete[img]) {
        for (int i = 0; i < n_anns; i++) {
            bool has0 = false;
            for (int j = 0; j < K; j++) has0 = has0 || work[i].data[j][2] == 0.0f;
            if (!has0) continue;
            copy_ann(&L.a, &work[i]);
            bool unfilled[kKP];
            for (int j = 0; j < K; j++) unfilled[j] = L.a.data[j][2] == 0.0f;
            grow(g, L, img, 1, false);
            bool any0 = false;
            for (int j = 0; j < K; j++) {
                float &v = L.a.data[j][2];
                if (unfilled[j] && v > 0.0f) v = (0.001f < v) ? 0.001f : v;  // np.minimum
                any0 = any0 || v == 0.0f;
            }
            if (any0) flood_fill(g, L);
            __syncthreads();
            copy_ann(&work[i], &L.a);
        }
    }

    STAMP(1);
    int n_out = n_anns;
    int *keep = g.nms_idx + (int64_t)img * (2 * g.ann_cap + g.ann_np);  // kept work indices
    int *surv = keep + g.ann_cap;                                          // survivors
    int *perm = surv + g.ann_cap;                                          // sort permutation
    double *score = g.nms_score + (int64_t)img * g.ann_cap;
    pp_ann *out = g.out + (int64_t)img * g.ann_cap;
    if (g.cfg.apply_nms && n_anns > 0) {
        // ---- nms.Keypoints.annotations (nms.py:17-57) ----
        const float kt = g.cfg.nms_keypoint_threshold;
        const double it = (double)g.cfg.nms_instance_threshold;
        int m = 0;
        float mx = 0.0f, my = 0.0f;
        for (int i = 0; i < n_anns; i++) {  // nms.py:20-22
            pp_ann &a = work[i];
            if (lane < K && a.data[lane][2] < kt) {
                a.data[lane][0] = 0.0f;
                a.data[lane][1] = 0.0f;
                a.data[lane][2] = 0.0f;
            }
            __syncthreads();
            const double sc = ann_score(L, a.data, K);
            if (sc >= it) {
                float ax = a.data[0][0], ay = a.data[0][1];
                for (int j = 1; j < K; j++) {
                    ax = a.data[j][0] > ax ? a.data[j][0] : ax;
                    ay = a.data[j][1] > ay ? a.data[j][1] : ay;
                }
                if (m == 0 || ax > mx) mx = ax;
                if (m == 0 || ay > my) my = ay;
                if (lane == 0) {
                    keep[m] = i;
                    score[m] = sc;
                }
                m++;
            }
        }
        __syncthreads();
        STAMP(2);
        n_out = 0;
        if (m > 0) {
            // Occupancy((K, int(max y + 1), int(max x + 1)), 2, min_scale=4)  (nms.py:27-31)
            const long oh = (long)((double)(long)(my + 1.0f) / g.cfg.occupancy_reduction);
            const long ow = (long)((double)(long)(mx + 1.0f) / g.cfg.occupancy_reduction);
            OccGrid no{occ_base, K, (int)(oh > 0 ? oh : 0), (int)(ow > 0 ? ow : 0)};
            if ((int64_t)K * no.h * no.w > g.occ_cap) {
                L.status |= PP_ST_NMS_OVERFLOW;
            } else {
                int np = 1;
                while (np < m) np <<= 1;
                sort_by_score(perm, np, m, score);  // nms.py:33 (stable)
                STAMP(3);
                for (int r = 0; r < m; r++) {  // nms.py:34-45
                    pp_ann &a = work[keep[perm[r]]];
                    // joints sit on separate occupancy planes: test all in parallel, then
                    // suppress the occupied ones and mark the free ones
                    bool occd = false;
                    if (lane < K && a.data[lane][2] != 0.0f)
                        occd = occ_get(no, lane, a.data[lane][0], a.data[lane][1], red);
                    const uint64_t om = __ballot(occd);
                    __syncthreads();
                    if (occd) a.data[lane][2] = a.data[lane][2] * g.cfg.nms_suppression;
                    occ_mark(g, L, log, no, a.data, a.joint_scales, K, [&](int j) {
                        return !((om >> j) & 1ull) && a.data[j][2] != 0.0f;
                    });
                }
                STAMP(4);
                occ_clear(g, L, log, no);
                STAMP(5);
                int m2 = 0;
                for (int r = 0; r < m; r++) {  // nms.py:51-53, in sorted order
                    const int wi = keep[perm[r]];
                    pp_ann &a = work[wi];
                    if (lane < K && a.data[lane][2] < kt) {
                        a.data[lane][0] = 0.0f;
                        a.data[lane][1] = 0.0f;
                        a.data[lane][2] = 0.0f;
                    }
                    __syncthreads();
                    const double sc = ann_score(L, a.data, K);
                    if (sc >= it) {
                        if (lane == 0) {
                            surv[m2] = wi;
                            score[m2] = sc;
                        }
                        m2++;
                    }
                }
                __syncthreads();
                STAMP(6);
                int np2 = 1;
                while (np2 < m2) np2 <<= 1;
                if (m2 > 0) sort_by_score(perm, np2, m2, score);  // nms.py:54
                STAMP(7);
                for (int r = 0; r < m2; r++) {
                    copy_ann(&out[r], &work[surv[perm[r]]]);
                    if (lane == 0) out[r].score = score[perm[r]];
                }
                n_out = m2;
            }
        }
    } else {
        for (int i = 0; i < n_anns; i++) {
            copy_ann(&out[i], &work[i]);
            const double sc = ann_score(L, work[i].data, K);
            if (lane == 0) out[i].score = sc;
        }
    }
    __syncthreads();
    STAMP(8);
    STAMP_FLUSH(2);
    if (lane == 0) {
        g.counts[img] = n_out;
        g.status[img] = L.status;
    }
}

}  // namespace pp

// ---------------------------------------------------------------------------------------
// host: workspace layout + pp_decode_batch
// ---------------------------------------------------------------------------------------
namespace pp {

int launch_seeds(const float *cif, const float *hr, int n_img, int K, int H, int W,
                 const pp_config *cfg, pp_seed *seeds, int cap, int *counts, void *scratch,
                 hipStream_t s);
size_t seeds_scratch_size(int n_img, int cap);
int launch_caf_bucketed(const float *caf, const float *hr, int n_img, int K, int C, int H, int W,
                        const int32_t *skeleton, const pp_config *cfg, float th, float *cols,
                        int *offs, const int *gate, hipStream_t s);
void caf_bucket_grid(int H, int W, int stride, int *bw, int *bh, int *nb, float *inv_e);

static inline size_t align_up(size_t a) { return (a + 255) / 256 * 256; }

struct DecodeLayout {
    int hh, ww;
    int64_t pitch, hw;
    int seed_cap, ann_cap, ann_np, log_cap;
    int bw, bh, nb;
    float inv_e;
    int64_t occ_cap;
    size_t off_cifhr, off_cifhr_ws, off_seeds, off_seed_counts, off_seed_ws, off_cols[2],
        off_offs[2], off_n_work, off_need, off_occ, off_log, off_work, off_nms_score,
        off_nms_idx, total;
    size_t cifhr_ws_bytes;
};

static DecodeLayout make_layout(int n_img, int K, int C, int H, int W, const pp_config *cfg,
                                int ann_cap) {
    DecodeLayout d{};
    d.hh = (int)hr_dim(H, cfg->stride);
    d.ww = (int)hr_dim(W, cfg->stride);
    d.pitch = pp_cifhr_pitch(d.ww);
    d.hw = (int64_t)H * W;
    d.seed_cap = (int)(K * d.hw);  // every cell of every field: no seed overflow possible
    d.ann_cap = ann_cap;
    d.ann_np = 1;
    while (d.ann_np < ann_cap) d.ann_np <<= 1;
    d.log_cap = K * ann_cap;
    const int64_t oh = (int64_t)((double)d.hh / cfg->occupancy_reduction);
    const int64_t ow = (int64_t)((double)d.ww / cfg->occupancy_reduction);
    d.occ_cap = (int64_t)align_up((size_t)(K * (oh + kOccMargin) * (ow + kOccMargin)));
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += align_up(bytes);
        return at;
    };
    const size_t n = (size_t)n_img;
    d.off_cifhr = take(n * K * d.hh * d.pitch * sizeof(float));
    d.cifhr_ws_bytes = pp_cifhr_workspace_size(n_img, K, H, W);
    d.off_cifhr_ws = take(d.cifhr_ws_bytes);
    d.off_seeds = take(n * d.seed_cap * sizeof(pp_seed));
    d.off_seed_counts = take(n * sizeof(int));
    d.off_seed_ws = take(seeds_scratch_size(n_img, d.seed_cap));
    caf_bucket_grid(H, W, cfg->stride, &d.bw, &d.bh, &d.nb, &d.inv_e);
    for (int t = 0; t < 2; t++) {
        const bool used = t == 0 || cfg->force_complete;
        d.off_cols[t] = take(used ? n * C * 2 * 10 * d.hw * sizeof(float) : 0);
        d.off_offs[t] = take(used ? n * C * 2 * (d.nb + 1) * sizeof(int) : 0);
    }
    d.off_n_work = take(n * sizeof(int));
    d.off_need = take(n * sizeof(int));
    d.off_occ = take(n * d.occ_cap);
    d.off_log = take(n * d.log_cap * sizeof(OccLog));
    d.off_work = take(n * ann_cap * sizeof(pp_ann));
    d.off_nms_score = take(n * ann_cap * sizeof(double));
    d.off_nms_idx = take(n * (2 * ann_cap + d.ann_np) * sizeof(int));
    d.total = o;
    return d;
}

}  // namespace pp

using namespace pp;

extern "C" {

size_t pp_decode_workspace_size(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                                const pp_config *cfg, int32_t ann_capacity) {
    if (!cfg || n_img < 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0 || ann_capacity <= 0) return 0;
    return make_layout(n_img, K, C, H, W, cfg, ann_capacity).total;
}

size_t pp_decode_workspace_zero_offset(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                                       const pp_config *cfg, int32_t ann_capacity) {
    if (!cfg || n_img <= 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0 || ann_capacity <= 0) return 0;
    return make_layout(n_img, K, C, H, W, cfg, ann_capacity).off_occ;
}

int pp_decode_stages(const float *d_cif, const float *d_caf, int32_t n_img, int32_t K, int32_t C,
                     int32_t H, int32_t W, const int32_t *skeleton, const pp_config *cfg,
                     float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                     int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                     uint32_t stages, void *stream) {
    if (!d_cif || !d_caf || !skeleton || !cfg || !d_anns || !d_counts || !d_status || !d_workspace)
        return fail(PP_EINVAL, "pp_decode_batch: NULL argument");
    if (n_img < 0 || K <= 0 || K > PP_MAX_KP || C <= 0 || C > PP_MAX_EDGES || H <= 0 || W <= 0 ||
        ann_capacity <= 0 || cfg->stride <= 0 || cfg->occupancy_reduction <= 0)
        return fail(PP_ESHAPE, "pp_decode_batch: shape outside the supported envelope "
                               "(K <= PP_MAX_KP, C <= PP_MAX_EDGES)");
    if (cfg->connection_method != 0 && cfg->connection_method != 1)
        return fail(PP_EINVAL, "connection method not known");
    for (int i = 0; i < 2 * C; i++)
        if (skeleton[i] < 1 || skeleton[i] > K)
            return fail(PP_EINVAL, "pp_decode_batch: skeleton joint index out of 1..K");
    if (n_img == 0) return PP_OK;
    const DecodeLayout d = make_layout(n_img, K, C, H, W, cfg, ann_capacity);
    if (workspace_bytes < d.total) return fail(PP_ENOMEM, "pp_decode_batch: workspace too small");
    if ((int64_t)d.hh >= 32767 * 2 || (int64_t)d.ww >= 32767 * 2)
        return fail(PP_ESHAPE, "pp_decode_batch: field too large");
    char *ws = (char *)d_workspace;
    hipStream_t s = (hipStream_t)stream;
    float *hr = d_cifhr ? d_cifhr : (float *)(ws + d.off_cifhr);
    pp_seed *seeds = (pp_seed *)(ws + d.off_seeds);
    int *seed_counts = (int *)(ws + d.off_seed_counts);
    float *cols[2] = {(float *)(ws + d.off_cols[0]), (float *)(ws + d.off_cols[1])};
    int *offs[2] = {(int *)(ws + d.off_offs[0]), (int *)(ws + d.off_offs[1])};
    int rc = PP_OK;
    if (stages & 1u) {
        rc = pp_cifhr(d_cif, n_img, K, H, W, cfg, hr, ws + d.off_cifhr_ws, d.cifhr_ws_bytes, s);
        if (rc) return rc;
    }
    if (stages & 2u) {
        rc = launch_seeds(d_cif, hr, n_img, K, H, W, cfg, seeds, d.seed_cap, seed_counts,
                          ws + d.off_seed_ws, s);
        if (rc) return rc;
    }
    if (stages & 4u) {  // CafScored at caf_threshold; the force-complete set is lazy
        rc = launch_caf_bucketed(d_caf, hr, n_img, K, C, H, W, skeleton, cfg, cfg->caf_threshold,
                                 cols[0], offs[0], nullptr, s);
        if (rc) return rc;
    }
    if (stages & 8u) {
        GrowArgs g{};
        g.seeds = seeds;
        g.seed_counts = seed_counts;
        g.seed_cap = d.seed_cap;
        g.cols[0] = cols[0];
        g.cols[1] = cols[1];
        g.offs[0] = offs[0];
        g.offs[1] = offs[1];
        g.bw = d.bw;
        g.bh = d.bh;
        g.nb = d.nb;
        g.inv_e = d.inv_e;
        g.K = K;
        g.C = C;
        g.H = H;
        g.W = W;
        g.hh = d.hh;
        g.ww = d.ww;
        g.hw = d.hw;
        g.cfg = *cfg;
        for (int i = 0; i < 2 * C; i++) g.skel[i] = skeleton[i];
        g.occ = (uint8_t *)(ws + d.off_occ);
        g.occ_cap = d.occ_cap;
        g.log = (OccLog *)(ws + d.off_log);
        g.log_cap = d.log_cap;
        g.work = (pp_ann *)(ws + d.off_work);
        g.nms_score = (double *)(ws + d.off_nms_score);
        g.nms_idx = (int *)(ws + d.off_nms_idx);
        g.ann_np = d.ann_np;
        g.ann_cap = ann_capacity;
        g.stamps = nullptr;
#ifdef PP_STAMPS
        hipMalloc((void **)&g.stamps, (size_t)n_img * 2 * 12 * sizeof(uint64_t));
        hipMemsetAsync(g.stamps, 0, (size_t)n_img * 2 * 12 * sizeof(uint64_t), s);
#endif
        g.n_work = (int *)(ws + d.off_n_work);
        g.need_complete = (int *)(ws + d.off_need);
        g.out = d_anns;
        g.counts = d_counts;
        g.status = d_status;
        hipLaunchKernelGGL(grow_kernel<1>, dim3(n_img), dim3(64), 0, s, g);
        rc = check_launch("pp_decode_batch(seed loop)");
        if (rc) return rc;
        if (cfg->force_complete) {
            // complete_annotations' CafScored(score_th=0.0001) only where phase 1 left work
            rc = launch_caf_bucketed(d_caf, hr, n_img, K, C, H, W, skeleton, cfg,
                                     cfg->complete_caf_threshold, cols[1], offs[1],
                                     g.need_complete, s);
            if (rc) return rc;
        }
        hipLaunchKernelGGL(grow_kernel<2>, dim3(n_img), dim3(64), 0, s, g);
        rc = check_launch("pp_decode_batch(complete + nms)");
#ifdef PP_STAMPS
        hipStreamSynchronize(s);
        const size_t nst = (size_t)n_img * 2 * 12;
        uint64_t *h = (uint64_t *)malloc(nst * sizeof(uint64_t));
        hipMemcpy(h, g.stamps, nst * sizeof(uint64_t), hipMemcpyDeviceToHost);
        const char *path = getenv("PP_STAMPS_OUT");
        FILE *fo = fopen(path ? path : "pp_stamps.bin", "ab");
        if (fo) {
            fwrite(h, sizeof(uint64_t), nst, fo);
            fclose(fo);
        }
        free(h);
        hipFree(g.stamps);
#endif
    }
    return rc;
}

int pp_decode_batch(const float *d_cif, const float *d_caf, int32_t n_img, int32_t K, int32_t C,
                    int32_t H, int32_t W, const int32_t *skeleton, const pp_config *cfg,
                    float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                    int32_t *d_status, void *d_workspace, size_t workspace_bytes, void *stream) {
    return pp_decode_stages(d_cif, d_caf, n_img, K, C, H, W, skeleton, cfg, d_cifhr, d_anns,
                            ann_capacity, d_counts, d_status, d_workspace, workspace_bytes, 15u,
                            stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// one _grow_connection (+ blend / max) on a device column set, for the functional API
// ---------------------------------------------------------------------------------------
namespace pp {
template <bool MAXM>
__global__ __launch_bounds__(64) void grow_connection_kernel(const float *cf, int n, int64_t pitch,
                                                             float x, float y, float xy_scale,
                                                             float *out) {
    float r[4];
    grow_connection_flat<MAXM>(cf, n, pitch, x, y, xy_scale, r);
    if (threadIdx.x < 4) out[threadIdx.x] = r[threadIdx.x];
}
}  // namespace pp

extern "C" int pp_grow_connection(const float *d_cols, int64_t n, int64_t pitch, float x, float y,
                                  float xy_scale, int32_t method, float *d_out, void *stream) {
    if (!d_cols || !d_out) return fail(PP_EINVAL, "pp_grow_connection: NULL argument");
    if (n < 0 || pitch < n || n > INT32_MAX) return fail(PP_ESHAPE, "pp_grow_connection: bad shape");
    if (method != 0 && method != 1) return fail(PP_EINVAL, "connection method not known");
    hipStream_t s = (hipStream_t)stream;
    if (method == 1)
        hipLaunchKernelGGL(grow_connection_kernel<true>, dim3(1), dim3(64), 0, s, d_cols, (int)n,
                           pitch, x, y, xy_scale, d_out);
    else
        hipLaunchKernelGGL(grow_connection_kernel<false>, dim3(1), dim3(64), 0, s, d_cols, (int)n,
                           pitch, x, y, xy_scale, d_out);
    return check_launch("pp_grow_connection");
}
