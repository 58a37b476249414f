// grow.hip — the CifCaf greedy decoder (generator/cifcaf.py) on gfx950.
//
// The seed loop is sequential by construction (each annotation's occupancy marks decide
// whether later seeds start annotations, cifcaf.py:100-108), so an image is one workgroup
// and a batch fills the chip with one workgroup per image.  Inside it, wave 0 commits in
// the reference order while seven helper waves grow seeds it is likely to reach (a grow is
// a pure function of the seed and the CAF columns); each wave's serial state lives in
// REGISTERS, not memory:
//
//   * the annotation being grown: lane j holds joint j's (x, y, v, scale);
//   * the frontier (cifcaf.py:248 PriorityQueue): at most one entry per directed skeleton
//     edge is ever live (in_frontier admits (j, k) once; its evaluated re-push replaces
//     the popped unevaluated entry), so lane d holds the entry of directed edge d (by_source
//     order, cifcaf.py:62-65) and pop-min is a wave reduction with the reference's tuple
//     order (-score, None|xysv, j, k);
//   * caf_center_s + scoring (functional.pyx:338-359, cifcaf.py:124-145): the lanes scan
//     the CAF columns (the image's small set-A sets from LDS, else the buckets the 2*scale
//     box overlaps, caf_bucketed_kernel) and merge the argsort top-2 _target_with_blend
//     (cifcaf.py:157-192) needs, targets included;
//   * occupancy grids (occupancy.py, u8 += 1 with wrap) live in a per-image workspace that
//     every launch leaves zeroed: each box a launch marks is logged and cleared again.
//
// Force-complete (cifcaf.py:333-351) spreads an image's annotations over 64 workgroups;
// NMS (nms.py:17-57) is one 8-wave workgroup per image.  Float arithmetic is f32
// op-for-op as NumPy evaluates it (NEP 50); np.exp is computed correctly rounded through
// f64.
#include "pp_common.hpp"

#include <stdio.h>
#include <stdlib.h>

#include <mutex>

// Diagnostic build only (-DPP_STAMPS, libpifpaf_amd_stamps.so): per-section shader-cycle
// sums of the decode kernel, dumped to $PP_STAMPS_OUT.  The product build compiles these
// to nothing.
#ifdef PP_STAMPS
#define STAMP_DECL                                                                          \
    uint64_t st_acc[kStampSlots] = {};                                                     \
    uint64_t st_t = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                                                            \
    do {                                                                                    \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                   \
        st_acc[i] += t_ - st_t;                                                             \
        st_t = t_;                                                                          \
    } while (0)
#define STAMP_FLUSH(ph)                                                                     \
    if (lane == 0 && g.stamps) {                                                            \
        st_acc[9] = L.fst[0];                                                               \
        st_acc[10] = L.fst[1];                                                              \
        st_acc[11] = L.fst[2];                                                              \
        st_acc[8] = L.fst[3];                                                               \
        st_acc[12] = L.fst[6];                                                              \
        st_acc[13] = L.fst[7];                                                              \
        for (int q_ = 0; q_ < kStampSlots; q_++)                                            \
            atomicAdd((unsigned long long *)&g.stamps[((int64_t)img * 3 + (ph)-1) * kStampSlots + q_], \
                      (unsigned long long)st_acc[q_]);                                      \
    }
#define FSTAMP_BEGIN const uint64_t fst_t0 = __builtin_amdgcn_s_memtime();
// eval_ahead's sections on wave 0 (fst[6]: from the column loads to their data, fst[7]: the
// forward query), with a vmcnt / lgkmcnt drain after the loads so the wait is attributed
#define ESTAMP(L, i, t)                                                                     \
    do {                                                                                    \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                   \
        if ((threadIdx.x & 63) == 0) (L).fst[i] += t_ - (t);                                \
        (t) = t_;                                                                           \
    } while (0)
#define FSTAMP_END(L, i)                                                                    \
    if ((threadIdx.x & 63) == 0) (L).fst[i] += __builtin_amdgcn_s_memtime() - fst_t0;
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_FLUSH(ph)
#define FSTAMP_BEGIN
#define FSTAMP_END(L, i)
#define ESTAMP(L, i, t)
#endif
constexpr int kStampSlots = 16;  // per (image, phase) in the diagnostic build

namespace pp {

constexpr int kKP = PP_MAX_KP;
constexpr int kSlots = 2 * PP_MAX_EDGES;   // directed edges (two lanes' worth of slots)
// flood-fill heap capacity: every joint is expanded at most once, pushing its by_source
// entries, so a fill pushes at most 2C <= 2 * PP_MAX_EDGES entries
constexpr int kHeap = 2 * PP_MAX_EDGES + 8;
constexpr int kOccMargin = 64;              // NMS occupancy slack beyond the main grid
constexpr int kCompleteWays = 64;           // force-complete workgroups per image

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

struct SeedExt;  // the seed loop's external-helper words (below)

struct GrowArgs {
    const pp_seed *seeds;
    const int *seed_counts;
    int seed_cap;
    const float *cols[2];     // bucketed column sets (n_img, C, 2, kColRows, col_cap): set A
                              // at caf_threshold, set B at complete_caf_threshold
    const int *offs[2];       // bucket boundaries (n_img, C, 2, nb + 1)
    int64_t col_cap;          // columns per set: the cells of all heads
    // set B (force-complete, complete_caf_threshold) holds only concatenated cell indices
    // (n_img, C, 2, col_cap); its queries read the heads' raw CAF and rescore with CifHr
    // (consider_raw)
    Heads heads;
    HrMap hr;                 // CifHr (dense, or the tile-major scratch layout)
    float cif_floor, one_minus_floor, th_b;
    uint8_t caf_j1[PP_MAX_EDGES], caf_j2[PP_MAX_EDGES];  // 0-based joints of each CAF
    int bw, bh, nb;           // bucket grid (see caf_bucketed_kernel)
    float inv_e;
    int K, C, hh, ww;
    pp_config cfg;
    // directed edges ("slots") in by_source order (cifcaf.py:62-65): joint j's entries
    // are slots j_off[j] .. j_off[j+1]-1 in dict insertion order
    int nd;
    uint8_t j_off[kKP + 1];
    uint8_t d_j[kSlots], d_k[kSlots], d_caf[kSlots], d_fwd[kSlots];
    // CifCaf(confidence_scales=...) (cifcaf.py:259-260, 282-284): the slot's CAF weight on
    // its frontier priorities when has_cs (pp_config.confidence_scales), else unused
    int has_cs;
    float slot_cs[kSlots];
    // workspace (per image regions)
    uint8_t *occ;
    int64_t occ_cap;          // bytes per image
    OccLog *log;
    int log_cap;              // entries per image
    pp_ann *work;             // working annotations
    pp_ann *spec;             // (n_img, kSpecCache) speculatively grown annotations
    float spec_far;           // seed-loop speculation distance, in joint scales
    int n_ext;                // external helper workgroups per image (seed loop)
    SeedExt *xext;            // (n_img) their hand-off words (zero at launch; the loop's last
                              // workgroup out re-zeroes them, ext_exit)
    pp_ann *xrec;             // (n_img, kExtCache) their published annotations
    double *nms_score;        // (n_img, 2 * ann_cap)
    // standalone NMS over caller annotations (pp_nms_keypoints_scored), else NULL: per
    // (image, record) -2 fixed_score, -1 none, j >= 0 suppress_score_index; the record's
    // score_weights (K each) and fixed scores (annotation.py:60-71)
    const int32_t *nms_spec;
    const double *nms_sw;
    const double *nms_fixed;
    double nms_it;            // nms.Keypoints.instance_threshold as the float64 it compares in
    int *nms_idx;             // (n_img, 4 * ann_cap + ann_np)
    float *nms_f;             // (n_img, 2 * ann_cap) per-annotation max x, max y
    int2 *nms_box;            // (n_img, kNmsBoxLists, ann_cap) plane box lists beyond registers
    int ann_np;               // next pow2 >= ann_cap
    int ann_cap;
    uint64_t *stamps;         // diagnostic build: (n_img, 3, kStampSlots) cycle sums, else NULL
    int *n_work;              // (n_img) annotations after the seed loop (phase 1 -> 2)
    int *complete_next;       // (n_img) force-complete work counters (zero region; the NMS
                              // kernel, ordered after completion, resets them)
    int *need_complete;       // (n_img) bitmask of joints left unset by the seed loop in any
                              // annotation (force-complete has work iff != 0; gates the B sets)
    // initial annotations (cifcaf.py:95-98), optional: (n_img, init_cap) records, the
    // first init_counts[img] of an image grown and committed before its seed loop
    const pp_ann *init;
    const int *init_counts;
    int init_cap;
    // outputs
    int *out_idx;             // optional (n_img, ann_cap): input index of each output record
    pp_ann *out;
    int *counts;
    int *status;
};

// per-wave LDS of the grow kernels; HEAP: the flood-fill heap (force-complete only)
template <bool HEAP>
struct GrowLDST {
    pp_ann a;                     // record being built (lists; data synced from registers)
    FFEntry ff[HEAP ? kHeap : 1];
    int mark_pre[kKP + 1];        // occupancy boxes of one annotation: area prefix
    int mark_box[kKP][4];
    int ff_n;
    int log_n;
    int status;
#ifdef PP_STAMPS
    uint64_t fst[10];  // inside-grow section sums (diagnostic build); [8], [9]: seed loop
#endif
};
using GrowLDS = GrowLDST<true>;
using SeedLDS = GrowLDST<false>;  // the seed loop's waves (no flood fill)


__device__ __forceinline__ float rl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int rl_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Wave reductions on DPP (row-level VALU data movement, no LDS round trip): quad xor 1,
// quad xor 2, row half-mirror, row mirror, then row_bcast15 / row_bcast31 fold the rows
// into lane 63.  Each step pairs lanes holding disjoint lane sets, so any associative,
// commutative merge (sum, min, exact top-2) is correct; lanes outside a step's row mask
// receive `old` (the identity).
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;
constexpr int kDppMirror = 0x140;
constexpr int kDppBcast15 = 0x142;
constexpr int kDppBcast31 = 0x143;

template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_f(float old, float v) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROWS, 0xF, false));
}

// sum over the wave, uniform result
__device__ __forceinline__ int wave_total(int v) {
    v += dpp_i<kDppXor1, 0xF>(0, v);
    v += dpp_i<kDppXor2, 0xF>(0, v);
    v += dpp_i<kDppHalfMirror, 0xF>(0, v);
    v += dpp_i<kDppMirror, 0xF>(0, v);
    v += dpp_i<kDppBcast15, 0xA>(0, v);
    v += dpp_i<kDppBcast31, 0xC>(0, v);
    return __builtin_amdgcn_readlane(v, 63);
}

// min over the wave (fminf: NaN ignored), uniform result
__device__ __forceinline__ float wave_fmin(float v) {
    v = fminf(v, dpp_f<kDppXor1, 0xF>(INFINITY, v));
    v = fminf(v, dpp_f<kDppXor2, 0xF>(INFINITY, v));
    v = fminf(v, dpp_f<kDppHalfMirror, 0xF>(INFINITY, v));
    v = fminf(v, dpp_f<kDppMirror, 0xF>(INFINITY, v));
    v = fminf(v, dpp_f<kDppBcast15, 0xA>(INFINITY, v));
    v = fminf(v, dpp_f<kDppBcast31, 0xC>(INFINITY, v));
    return rl_f(v, 63);
}

__device__ __forceinline__ bool ff_less(const FFEntry &a, const FFEntry &b) {
    if (a.neg != b.neg) return a.neg < b.neg;
    if (a.end != b.end) return a.end < b.end;
    for (int t = 0; t < 3; t++)
        if (a.sxyv[t] != b.sxyv[t]) return a.sxyv[t] < b.sxyv[t];
    return a.s < b.s;
}

__device__ __forceinline__ void ff_push(GrowLDS &L, const FFEntry &x) {
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

__device__ __forceinline__ FFEntry ff_pop(GrowLDS &L) {
    const FFEntry top = L.ff[0];
    const int n = L.ff_n - 1;
    L.ff_n = n;
    if (n > 0) {
        const FFEntry x = L.ff[n];
        int i = 0;
        for (;;) {
            const int l = 2 * i + 1, r = l + 1;
            int m = i;
            if (l < n && ff_less(L.ff[l], x)) m = l;
            if (r < n && ff_less(L.ff[r], m == i ? x : L.ff[l])) m = r;
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
// Candidate columns are ranked by a 64-bit key, larger = better: high word = the score's
// bits (scores are >= 0, so float order == unsigned order; NaN sorts last in np.argsort,
// i.e. largest, and its bits are above every finite score), low word = the column's
// row-major index, so ties follow the reference: blend (stable argsort, last wins) ->
// higher index; max (np.argmax, first wins) -> lower index.  0 = no candidate.
template <bool MAXM>
__device__ __forceinline__ uint64_t cand_key(float score, int o) {
    const uint32_t hi = (score != score) ? 0xFFFFFFFFu : __float_as_uint(score);
    const uint32_t lo = MAXM ? (uint32_t)(0x7FFFFFFF - o) : (uint32_t)(o + 1);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ float key_score(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }

struct Top2 {
    uint64_t k1, k2;   // best and second-best keys of this lane (0 = none)
    float x1, y1, c1;  // target (x2, y2, s2) rows of the best column
    float x2, y2, c2;  // ... and of the second best
};

// branch-free on purpose: values feed DPP reductions, which must not run under a
// partial exec mask
__device__ __forceinline__ void top2_insert(Top2 &t, uint64_t k, float x, float y, float c) {
    const bool b1 = k > t.k1;
    const bool b2 = !b1 & (k > t.k2);
    t.k2 = b1 ? t.k1 : (b2 ? k : t.k2);
    t.x2 = b1 ? t.x1 : (b2 ? x : t.x2);
    t.y2 = b1 ? t.y1 : (b2 ? y : t.y2);
    t.c2 = b1 ? t.c1 : (b2 ? c : t.c2);
    t.k1 = b1 ? k : t.k1;
    t.x1 = b1 ? x : t.x1;
    t.y1 = b1 ? y : t.y1;
    t.c1 = b1 ? c : t.c1;
}

template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)dpp_i<CTRL, ROWS>(0, (int)(uint32_t)v);
    const uint32_t hi = (uint32_t)dpp_i<CTRL, ROWS>(0, (int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// max of a 64-bit key over the wave, uniform result
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    uint64_t o;
    o = dpp_u64<kDppXor1, 0xF>(v);
    v = o > v ? o : v;
    o = dpp_u64<kDppXor2, 0xF>(v);
    v = o > v ? o : v;
    o = dpp_u64<kDppHalfMirror, 0xF>(v);
    v = o > v ? o : v;
    o = dpp_u64<kDppMirror, 0xF>(v);
    v = o > v ? o : v;
    o = dpp_u64<kDppBcast15, 0xA>(v);
    v = o > v ? o : v;
    o = dpp_u64<kDppBcast31, 0xC>(v);
    v = o > v ? o : v;
    const uint32_t lo = (uint32_t)rl_i((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)rl_i((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

// exact top-2 over the wave (uniform): the global best K1 by a max reduction, then the
// best key other than K1 (keys are unique per column); targets from the holding lane
struct Best2 {
    uint64_t k1, k2;
    float x1, y1, c1, x2, y2, c2;
};

__device__ __forceinline__ uint64_t rl_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)rl_i((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)rl_i((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// at most two lanes hold candidates (the usual case: the 2*scale box passes a handful of
// columns): merge them with scalar reads instead of the two DPP reductions
__device__ __forceinline__ Best2 top2_wave(const Top2 &t) {
    Best2 b;
    const uint64_t cm = __ballot(t.k1 != 0);
    if (__popcll(cm) <= 2) {
        const uint64_t cm2 = cm & (cm - 1);
        const int la = cm ? __ffsll((unsigned long long)cm) - 1 : 0;
        const int lb = cm2 ? __ffsll((unsigned long long)cm2) - 1 : la;
        const uint64_t ka1 = rl_u64(t.k1, la), ka2 = rl_u64(t.k2, la);
        const uint64_t kb1 = cm2 ? rl_u64(t.k1, lb) : 0, kb2 = cm2 ? rl_u64(t.k2, lb) : 0;
        const bool a_first = ka1 > kb1;  // equal only when both are 0
        const int l1 = a_first ? la : lb, lo = a_first ? lb : la;
        const uint64_t own2 = a_first ? ka2 : kb2, oth1 = a_first ? kb1 : ka1;
        const bool own_second = own2 > oth1;  // the best lane's runner-up beats the other's best
        b.k1 = a_first ? ka1 : kb1;
        b.k2 = own_second ? own2 : oth1;
        b.x1 = rl_f(t.x1, l1);
        b.y1 = rl_f(t.y1, l1);
        b.c1 = rl_f(t.c1, l1);
        const int l2 = own_second ? l1 : lo;
        b.x2 = own_second ? rl_f(t.x2, l2) : rl_f(t.x1, l2);
        b.y2 = own_second ? rl_f(t.y2, l2) : rl_f(t.y1, l2);
        b.c2 = own_second ? rl_f(t.c2, l2) : rl_f(t.c1, l2);
        return b;
    }
    b.k1 = wave_max_u64(t.k1);
    b.k2 = wave_max_u64(t.k1 == b.k1 ? t.k2 : t.k1);
    const uint64_t m1 = __ballot(t.k1 == b.k1 && b.k1 != 0);
    const int l1 = m1 ? __ffsll((unsigned long long)m1) - 1 : 0;
    b.x1 = rl_f(t.x1, l1);
    b.y1 = rl_f(t.y1, l1);
    b.c1 = rl_f(t.c1, l1);
    const uint64_t m2a = __ballot(t.k1 == b.k2 && b.k2 != 0);
    const uint64_t m2b = __ballot(t.k2 == b.k2 && b.k2 != 0);
    const int l2a = m2a ? __ffsll((unsigned long long)m2a) - 1 : 0;
    const int l2b = m2b ? __ffsll((unsigned long long)m2b) - 1 : 0;
    b.x2 = m2a ? rl_f(t.x1, l2a) : rl_f(t.x2, l2b);
    b.y2 = m2a ? rl_f(t.y1, l2a) : rl_f(t.y2, l2b);
    b.c2 = m2a ? rl_f(t.c1, l2a) : rl_f(t.c2, l2b);
    return b;
}

struct ColQuery {
    float x, y, lo_x, hi_x, lo_y, hi_y, sigma2;
    int exp_mode;  // pp_config.exp_mode (caf_exp)
    // sigma2's refined reciprocal (div_refined) for every column's -0.5 d^2 / sigma2, when
    // the query is in its domain: sigma2 in [1, 2^90] and finite box bounds (a column that
    // passes the box test then has |-0.5 d^2| <= 16 sigma2 <= 2^94); else IEEE division
    Recip sr;
    bool fast;
};

__device__ __forceinline__ ColQuery make_query(float x, float y, float xy_scale, int exp_mode) {
    ColQuery q;
    q.exp_mode = exp_mode;
    const float sbox = 2.0f * xy_scale;  // caf_center_s(..., sigma=2.0 * xy_scale)
    q.x = x;
    q.y = y;
    q.lo_x = x - sbox;
    q.hi_x = x + sbox;
    q.lo_y = y - sbox;
    q.hi_y = y + sbox;
    const float sigma = 0.5f * xy_scale;
    q.sigma2 = np_pow2_f32(sigma);  // `sigma**2` of a NumPy float32 scalar: libm powf
    q.sr = recip_of(q.sigma2);
    q.fast = q.sigma2 >= 1.0f && q.sigma2 <= 0x1p90f && fabsf(q.lo_x) <= 0x1p100f &&
             fabsf(q.hi_x) <= 0x1p100f && fabsf(q.lo_y) <= 0x1p100f && fabsf(q.hi_y) <= 0x1p100f;
    return q;
}

// -0.5 d^2 / sigma^2 of a column inside the query's box (cifcaf.py:139), IEEE-rounded
__device__ __forceinline__ float score_arg(const ColQuery &q, float dd) {
    const float n = -0.5f * (dd * dd);
    return q.fast ? div_refined(n, q.sr) : n / q.sigma2;
}

// column k (all rows loaded in one round): caf_center_s test, score (cifcaf.py:134-139).
// PACKED: the decoder's kColRows layout (index in row 6); else the reference's 9 rows
// with the column's position k as its index.
template <bool MAXM>
__device__ __forceinline__ void consider_vals(const ColQuery &q, float c0, float c1, float c2, float tx,
                                              float ty, float tc, int o, Top2 &t) {
    if (c1 < q.lo_x || c1 > q.hi_x || c2 < q.lo_y || c2 > q.hi_y) return;
    const float dx = q.x - c1, dy = q.y - c2;
    const float dd = sqrtf(dx * dx + dy * dy);  // np.linalg.norm(axis=0)
    const float score = caf_exp(score_arg(q, dd), q.exp_mode) * c0;  // np.exp
    top2_insert(t, cand_key<MAXM>(score, o), tx, ty, tc);
}

template <bool MAXM, bool PACKED>
__device__ __forceinline__ void consider(const float *__restrict__ cf, int64_t hw, const ColQuery &q,
                                         int k, Top2 &t) {
    const float c1 = cf[hw + k], c2 = cf[2 * hw + k], c0 = cf[k];
    const float tx = cf[(PACKED ? 3 : 5) * hw + k], ty = cf[(PACKED ? 4 : 6) * hw + k];
    const float tc = cf[(PACKED ? 5 : 8) * hw + k];
    const int o = PACKED ? __float_as_int(cf[6 * hw + k]) : k;
    consider_vals<MAXM>(q, c0, c1, c2, tx, ty, tc, o, t);
}

// a set-B column: concatenated cell index -> the head's raw CAF values (caf_scored.py:58-81
// for this one column: rows * stride, CifHr rescoring at the target, the second
// threshold), then as consider
struct RawSet {
    const int *idx;      // bucketed concatenated cell indices (int32), or
    const uint16_t *idx16;  // u16 ones (sets of at most kSetBIdx16Max cells)
    int64_t fld;         // image * C + CAF field
    int64_t hrt;         // CifHr plane of the direction's target joint (rescore), or -1
    int src, tgt, tsc;   // raw rows of source x, target x, target scale (y = x + 1)
};

template <bool MAXM>
__device__ __forceinline__ void consider_raw(const GrowArgs &g, const RawSet &r, const ColQuery &q,
                                             int k, Top2 &t) {
    const int key = r.idx16 ? (int)r.idx16[k] : r.idx[k];
    const Heads &h = g.heads;
    int hm = 0, cell = key;
    if (h.n_caf > 1) {
        hm = h.caf_head_of(key);
        cell = key - (int)h.caf_off[hm];
    }
    const int64_t hw = (int64_t)h.aH[hm] * h.aW[hm];
    const float stride = (float)h.astride[hm];
    const float *caf9 = h.caf[hm] + r.fld * 9 * hw;
    const float c = caf9[cell];
    const float c1 = caf9[r.src * hw + cell] * stride;
    const float c2 = caf9[(r.src + 1) * hw + cell] * stride;
    const float tx = caf9[r.tgt * hw + cell] * stride;
    const float ty = caf9[(r.tgt + 1) * hw + cell] * stride;
    const float tc = caf9[r.tsc * hw + cell] * stride;
    if (c1 < q.lo_x || c1 > q.hi_x || c2 < q.lo_y || c2 > q.hi_y) return;
    float c0 = c;
    if (r.hrt >= 0) c0 = c * (g.cif_floor + g.one_minus_floor * g.hr.at(r.hrt, tx, ty, 0.0f));
    if (!(c0 > g.th_b)) return;
    const float dx = q.x - c1, dy = q.y - c2;
    const float dd = sqrtf(dx * dx + dy * dy);
    const float score = caf_exp(score_arg(q, dd), q.exp_mode) * c0;
    top2_insert(t, cand_key<MAXM>(score, key), tx, ty, tc);
}

// _target_with_blend / _target_with_maxscore (cifcaf.py:147-192) on the merged top-2
template <bool MAXM>
__device__ __forceinline__ void finish_connection(const Top2 &t, float out[4]) {
    const Best2 b = top2_wave(t);
    if (b.k1 == 0) {  // no candidate (every candidate's key is nonzero)
        out[0] = out[1] = out[2] = out[3] = 0.0f;
        return;
    }
    const float s1 = key_score(b.k1), s2 = key_score(b.k2);
    if (MAXM) {
        out[0] = b.x1;
        out[1] = b.y1;
        out[2] = b.c1;
        out[3] = s1;
        return;
    }
    // one candidate (len(scores) == 1): k2 = 0, s2 = 0.0 takes this branch with the same
    // result
    if (s2 < 0.01f || s2 < 0.5f * s1) {
        out[0] = b.x1;
        out[1] = b.y1;
        out[2] = b.c1;
        out[3] = s1 * 0.5f;
        return;
    }
    const float ex = b.x1 - b.x2, ey = b.y1 - b.y2;
    const float dist = sqrtf(ex * ex + ey * ey);
    if (dist > b.c1 / 2.0f) {
        out[0] = b.x1;
        out[1] = b.y1;
        out[2] = b.c1;
        out[3] = s1 * 0.5f;
        return;
    }
    const float ssum = s1 + s2;
    out[0] = (s1 * b.x1 + s2 * b.x2) / ssum;
    out[1] = (s1 * b.y1 + s2 * b.y2) / ssum;
    out[2] = (s1 * b.c1 + s2 * b.c2) / ssum;
    out[3] = 0.5f * (s1 + s2);
}

__device__ __forceinline__ Top2 top2_empty() {
    Top2 t;
    t.k1 = t.k2 = 0;
    t.x1 = t.y1 = t.c1 = t.x2 = t.y2 = t.c2 = 0.0f;
    return t;
}

// column set in the reference's order, n columns (the functional API entry point)
template <bool MAXM>
__device__ void grow_connection_flat(const float *__restrict__ cf, int n, int64_t hw, float x,
                                     float y, float xy_scale, int exp_mode, float out[4]) {
    const int lane = threadIdx.x & 63;
    const ColQuery q = make_query(x, y, xy_scale, exp_mode);
    Top2 t = top2_empty();
    for (int i = lane; i < n; i += 64) consider<MAXM, false>(cf, hw, q, i, t);
    finish_connection<MAXM>(t, out);
}

#ifdef PP_STAMPS
__device__ uint64_t *g_gc_stamps;  // diagnostic: [img][4] section sums of grow_connection
#define GSTAMP(i)                                                                           \
    do {                                                                                    \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                   \
        if (lane == 0 && g_gc_stamps) atomicAdd((unsigned long long *)&g_gc_stamps[blockIdx.x * 4 + (i)], (unsigned long long)(t_ - gs_t));        \
        gs_t = t_;                                                                          \
    } while (0)
#else
#define GSTAMP(i)
#endif

// bucketed column set (caf_bucketed_kernel): visit only the buckets the 2*scale box
// overlaps (+ the NaN-source bucket); segments flattened over the 64 lanes
template <bool MAXM, bool RAW>
__device__ __forceinline__ void grow_connection(const GrowArgs &g, const float *__restrict__ cf, const RawSet &raw,
                                const int *__restrict__ off, float x, float y, float xy_scale,
                                float out[4]) {
    const int lane = threadIdx.x & 63;
#ifdef PP_STAMPS
    uint64_t gs_t = __builtin_amdgcn_s_memtime();
#endif
    const int64_t hw = g.col_cap;
    const ColQuery q = make_query(x, y, xy_scale, g.cfg.exp_mode);
    Top2 t = top2_empty();
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
        const int ng = min(64, nseg - sb);
        int total = 0;
        for (int rr = 0; rr < ng; rr++) total += rl_i(len, rr);  // scalar
        GSTAMP(0);
        for (int base = 0; base < total; base += 64) {
            const int tt = base + lane;
            int k = -1, run = 0;
            for (int rr = 0; rr < ng; rr++) {  // the segment holding tt (uniform loop)
                const int l = rl_i(len, rr);
                if (tt >= run && tt < run + l) k = rl_i(st, rr) + (tt - run);
                run += l;
            }
            if (k >= 0) {
                if (RAW)
                    consider_raw<MAXM>(g, raw, q, k, t);
                else
                    consider<MAXM, true>(cf, hw, q, k, t);
            }
        }
        GSTAMP(1);
    }
    finish_connection<MAXM>(t, out);
    GSTAMP(2);
}

__device__ __forceinline__ float max0(float v) { return (v > 0.0f) ? v : 0.0f; }

__device__ __forceinline__ const float *col_set(const GrowArgs &g, int set, int img, int caf_i,
                                                int dir) {
    return g.cols[set] + (((int64_t)img * g.C + caf_i) * 2 + dir) * (set ? 1 : kColRows) * g.col_cap;
}

// set B of (image, CAF, direction): dir 1 forward (x1, y1) -> (x2, y2, s2), rescored at
// joint j2; dir 0 backward (x2, y2) -> (x1, y1, s1), rescored at j1 (caf_scored.py:58-81)
__device__ __forceinline__ RawSet raw_set(const GrowArgs &g, int img, int caf_i, int dir) {
    RawSet r;
    const float *cs = col_set(g, 1, img, caf_i, dir);
    const bool i16 = g.col_cap <= kSetBIdx16Max;  // caf_bucketed_kernel<true, true>
    r.idx = i16 ? nullptr : reinterpret_cast<const int *>(cs);
    r.idx16 = i16 ? reinterpret_cast<const uint16_t *>(cs) : nullptr;
    r.fld = (int64_t)img * g.C + caf_i;
    const int tj = dir ? g.caf_j2[caf_i] : g.caf_j1[caf_i];
    r.hrt = (g.cif_floor < 1.0f && tj < g.K) ? (int64_t)img * g.K + tj : -1;
    r.src = dir ? 1 : 5;
    r.tgt = dir ? 5 : 1;
    r.tsc = dir ? 8 : 4;
    return r;
}

__device__ __forceinline__ const int *col_offs(const GrowArgs &g, int set, int img, int caf_i,
                                               int dir) {
    return g.offs[set] + (((int64_t)img * g.C + caf_i) * 2 + dir) * (int64_t)(g.nb + 1);
}

// cifcaf.py:194-217 for start joint (jx, jy, jv, js) along CAF caf_i in direction fwd
__device__ __forceinline__ void connection_value(const GrowArgs &g, int img, int set, int caf_i, int fwd,
                                 float jx, float jy, float jv, float js, bool reverse_match,
                                 float out[4]) {
    const int df = fwd ? 1 : 0, db = fwd ? 0 : 1;
    const float xy_scale_s = max0(js);
    const bool maxm = g.cfg.connection_method == 1;
    // one query along direction `dir` from (qx, qy, qs)
    auto query = [&](int dir, float qx, float qy, float qs, float r[4]) {
        const float *cf = col_set(g, set, img, caf_i, dir);
        const int *off = col_offs(g, set, img, caf_i, dir);
        if (set) {
            const RawSet raw = raw_set(g, img, caf_i, dir);
            if (maxm)
                grow_connection<true, true>(g, cf, raw, off, qx, qy, qs, r);
            else
                grow_connection<false, true>(g, cf, raw, off, qx, qy, qs, r);
        } else {
            const RawSet none{};
            if (maxm)
                grow_connection<true, false>(g, cf, none, off, qx, qy, qs, r);
            else
                grow_connection<false, false>(g, cf, none, off, qx, qy, qs, r);
        }
    };
    float nx[4];
    query(df, jx, jy, xy_scale_s, nx);

    out[0] = out[1] = out[2] = out[3] = 0.0f;
    const float ks = sqrtf(nx[3] * jv);  // geometric mean
    if (ks < g.cfg.keypoint_threshold) return;
    if (nx[3] == 0.0f) return;
    const float xy_scale_t = max0(nx[2]);
    if (reverse_match) {
        float rv[4];
        query(db, nx[0], nx[1], xy_scale_t, rv);
        if (rv[2] == 0.0f) return;  // tests the SCALE (cifcaf.py:212)
        if (fabsf(jx - rv[0]) + fabsf(jy - rv[1]) > xy_scale_s) return;
    }
    out[0] = nx[0];
    out[1] = nx[1];
    out[2] = nx[2];
    out[3] = ks;
}

// ---------------------------------------------------------------------------------------
// the frontier in registers: lane l holds directed-edge slots l and l + 64
// ---------------------------------------------------------------------------------------
struct Frontier {
    int st[2];         // 0 empty, 1 (-max_possible, None, j, k), 2 (-score, xysv, j, k)
    float neg[2];
    float x[2], y[2], s[2], v[2];
    int added[2];      // in_frontier (cifcaf.py:249)
    int sj[2], sk[2], scaf[2], sfwd[2];  // slot constants
    // connection_value of an unevaluated entry computed ahead of its pop (eval_ahead)
    int pc[2];
    float px[2], py[2], ps[2], pv[2];
};

struct Entry {
    int slot, eval, j, k, caf, fwd, pc;
    float neg, x, y, s, v;
    float px, py, ps, pv;
};

// tuple order of (neg, None | (x, y, s, v), j, k); a None/tuple tie would raise TypeError
// in the reference (never happens in a successful run): unevaluated first here
__device__ __forceinline__ bool entry_less(float na, int ea, float xa, float ya, float sa,
                                           float va, int ja, int ka, float nb, int eb, float xb,
                                           float yb, float sb, float vb, int jb, int kb) {
    if (na != nb) return na < nb;
    if (ea != eb) return ea < eb;
    if (ea) {
        if (xa != xb) return xa < xb;
        if (ya != yb) return ya < yb;
        if (sa != sb) return sa < sb;
        if (va != vb) return va < vb;
    }
    if (ja != jb) return ja < jb;
    return ka < kb;
}

__device__ __forceinline__ bool slot_less(const Frontier &F, int a, int b) {
    return entry_less(F.neg[a], F.st[a] == 2, F.x[a], F.y[a], F.s[a], F.v[a], F.sj[a], F.sk[a],
                      F.neg[b], F.st[b] == 2, F.x[b], F.y[b], F.s[b], F.v[b], F.sj[b], F.sk[b]);
}

// PriorityQueue.get(): remove and return the smallest live entry (false when empty)
__device__ __forceinline__ bool frontier_pop(Frontier &F, Entry &e) {
    const int lane = threadIdx.x & 63;
    int lb = -1;
    if (F.st[0]) lb = 0;
    if (F.st[1] && (lb < 0 || slot_less(F, 1, 0))) lb = 1;
    const uint64_t live = __ballot(lb >= 0);
    if (live == 0) return false;
    const bool w1 = lb == 1;  // selects, not F.x[w]: a dynamic index sends F to scratch
    const float myneg = lb >= 0 ? (w1 ? F.neg[1] : F.neg[0]) : INFINITY;
    const float mn = wave_fmin(myneg);
    uint64_t cand = __ballot(lb >= 0 && myneg == mn);
    if (cand == 0) cand = live;  // only NaN scores left
    int win = __ffsll((unsigned long long)cand) - 1;
    const float my_x = w1 ? F.x[1] : F.x[0], my_y = w1 ? F.y[1] : F.y[0];
    const float my_s = w1 ? F.s[1] : F.s[0], my_v = w1 ? F.v[1] : F.v[0];
    const int my_e = (w1 ? F.st[1] : F.st[0]) == 2, my_j = w1 ? F.sj[1] : F.sj[0];
    const int my_k = w1 ? F.sk[1] : F.sk[0];
    if (__popcll(cand) > 1) {  // exact score tie: full tuple comparison (rare)
        uint64_t rest = cand & (cand - 1);
        while (rest) {
            const int c = __ffsll((unsigned long long)rest) - 1;
            rest &= rest - 1;
            if (entry_less(rl_f(myneg, c), rl_i(my_e, c), rl_f(my_x, c), rl_f(my_y, c),
                           rl_f(my_s, c), rl_f(my_v, c), rl_i(my_j, c), rl_i(my_k, c),
                           rl_f(myneg, win), rl_i(my_e, win), rl_f(my_x, win), rl_f(my_y, win),
                           rl_f(my_s, win), rl_f(my_v, win), rl_i(my_j, win), rl_i(my_k, win)))
                win = c;
        }
    }
    const int wr = rl_i(w1 ? 1 : 0, win);
    e.slot = win + 64 * wr;
    e.neg = rl_f(myneg, win);
    e.eval = rl_i(my_e, win);
    e.x = rl_f(my_x, win);
    e.y = rl_f(my_y, win);
    e.s = rl_f(my_s, win);
    e.v = rl_f(my_v, win);
    e.j = rl_i(my_j, win);
    e.k = rl_i(my_k, win);
    e.caf = rl_i(wr ? F.scaf[1] : F.scaf[0], win);
    e.fwd = rl_i(wr ? F.sfwd[1] : F.sfwd[0], win);
    e.pc = rl_i(wr ? F.pc[1] : F.pc[0], win);
    e.px = rl_f(wr ? F.px[1] : F.px[0], win);
    e.py = rl_f(wr ? F.py[1] : F.py[0], win);
    e.ps = rl_f(wr ? F.ps[1] : F.ps[0], win);
    e.pv = rl_f(wr ? F.pv[1] : F.pv[0], win);
    if (lane == win) {
        if (wr)
            F.st[1] = 0;
        else
            F.st[0] = 0;
    }
    return true;
}

// add_to_frontier (cifcaf.py:251-263): the start joint's slots in dict order, one pass
template <bool CS, typename LDS>
__device__ __forceinline__ void add_to_frontier(const GrowArgs &g, LDS &L, Frontier &F, float av, int start,
                                float start_v, int &nfr, uint64_t added[2]) {
    const int lane = threadIdx.x & 63;
    const int lo = g.j_off[start], hi = g.j_off[start + 1];
    const float neg = -sqrtf(start_v);
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int d = lane + 64 * r;
        const float tv = __shfl(av, F.sk[r]);  // target joint's v (all lanes shuffle)
        const bool elig = d >= lo && d < hi && !(tv > 0.0f) && !F.added[r];
        const uint64_t m = __ballot(elig);
        if (elig) {
            F.st[r] = 1;
            // max_possible_score *= confidence_scales[caf_i] (cifcaf.py:258-261)
            F.neg[r] = CS ? -(sqrtf(start_v) * g.slot_cs[d]) : neg;
            F.added[r] = 1;
            const int t = nfr + lane_prefix(m);
            if (t < PP_MAX_FRONTIER) {
                L.a.frontier_pairs[t][0] = (uint8_t)start;
                L.a.frontier_pairs[t][1] = (uint8_t)F.sk[r];
            }
        }
        nfr += __popcll(m);
        added[r] = m;
    }
}

// ---------------------------------------------------------------------------------------
// connection_value ahead of the pop, several edges per memory round trip (seed loop)
// ---------------------------------------------------------------------------------------
// An unevaluated frontier entry (j, k) is evaluated when popped (cifcaf.py:275-279), but
// its connection_value depends only on the CAF columns and on joint j, which never changes
// once set.  So when joint j enters the frontier, the connections of all its new entries
// are computed at once: up to kAhead edges, the column rows of both directions of all of
// them loaded in ONE round trip (flat scan of small set-A column sets, <= kFlatCols
// columns, count from LDS), instead of two dependent round trips (bucket offsets, then
// columns) per edge and direction.  The pop then takes the stored result; the frontier order, the
// evaluation results and everything the reference observes are unchanged.  Edges whose
// sets are larger stay lazy (grow_connection over the buckets).
// edges per batch: 1 since the sets come from LDS (2 batched the HBM round trips; with
// LDS the extra registers only added spills: 1.006 -> 0.979 ms per overlapped step)
constexpr int kAhead = 1;
constexpr int kFlatPer = 2;
constexpr int kFlatCols = 64 * kFlatPer;

__device__ __forceinline__ void flat_load(const float *__restrict__ cf, int64_t hw, int n,
                                          float v[kFlatPer][kColRows]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int p = 0; p < kFlatPer; p++) {
        const int k = p * 64 + lane;
#pragma unroll
        for (int r = 0; r < kColRows; r++) v[p][r] = (k < n) ? cf[r * hw + k] : 0.0f;
    }
}

// Set-A column sets staged in LDS by the seed loop: every small set (<= kFlatCols columns)
// that fits kColLds floats, in (CAF, direction) order, column-major (kColPad floats per
// column: two 16-byte reads).  cofs[q] = its offset, -1 = global.
constexpr int kColPad = 8;
// 74.5 KB (64 KB: 1-2% slower per planted cfg3 step).  With the seed loop's static LDS this
// leaves 39 KB of the CU's 160 KB for the next batch's kernels (DecodePipeline): CafScored
// (caf_bucketed_kernel, 37 KB) must fit beside it (3 KB less: uniform cfg3 4% slower).
constexpr int kColLds = 19072;
// the external-helper kernel (seed_loop_ext_kernel: images with helpers on other CUs, e.g.
// cfg5) stages 48 KB: the LDS it leaves lets the other batch's kernels share its CUs (cfg5
// uniform 1452-1473 -> 1583-1585 images/s, planted 41.3k -> 43.1k-43.7k; 80 KB for the
// one-CU kernel, where 48 / 64 KB measured 1 % slower, A/B on one box)
constexpr int kColLdsExt = 12288;
struct ColStage {
    const int *ncol;   // set-A column counts per (CAF, direction)
    const int *cofs;
    const float *lds;
};

// the same from the LDS copy of the set (offset `lo`, -1 = not staged)
__device__ __forceinline__ void flat_load_set(const float *__restrict__ cf, int64_t hw, int n,
                                              const float *lds, int lo,
                                              float v[kFlatPer][kColRows]) {
    if (lo < 0) {
        flat_load(cf, hw, n, v);
        return;
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int p = 0; p < kFlatPer; p++) {
        const int k = p * 64 + lane;
        float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = a;
        if (k < n) {
            const float4 *c = reinterpret_cast<const float4 *>(lds + lo + k * kColPad);
            a = c[0];
            b = c[1];
        }
        v[p][0] = a.x;
        v[p][1] = a.y;
        v[p][2] = a.z;
        v[p][3] = a.w;
        v[p][4] = b.x;
        v[p][5] = b.y;
        v[p][6] = b.z;
    }
}

// per directed-edge slot (one per lane and half, like the Frontier): both directions' set
// sizes and LDS offsets packed as (count << 16) | (offset + 1), and whether both are small
struct SlotSets {
    int f[2], b[2];
    uint64_t small[2];
};

__device__ __forceinline__ SlotSets slot_sets(const GrowArgs &g, const ColStage &cs) {
    const int lane = threadIdx.x & 63;
    SlotSets t;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int d = lane + 64 * r;
        int f = 0, b = 0;
        bool small = false;
        if (d < g.nd) {
            const int caf = g.d_caf[d], df = g.d_fwd[d] ? 1 : 0;
            const int qf = caf * 2 + df, qb = caf * 2 + 1 - df;
            const int nf = cs.ncol[qf], nb = cs.ncol[qb];
            small = nf <= kFlatCols && nb <= kFlatCols;
            f = (nf << 16) | (cs.cofs[qf] + 1);
            b = (nb << 16) | (cs.cofs[qb] + 1);
        }
        t.f[r] = f;
        t.b[r] = b;
        t.small[r] = __ballot(small);
    }
    return t;
}

// grow_connection over every column of a flat-loaded set (same columns pass caf_center_s
// as through the buckets; the merge is independent of visiting order: unique keys)
template <bool MAXM>
__device__ __forceinline__ void flat_query(const float v[kFlatPer][kColRows], int n, float x, float y,
                                           float xy_scale, int exp_mode, float out[4]) {
    const int lane = threadIdx.x & 63;
    const ColQuery q = make_query(x, y, xy_scale, exp_mode);
    Top2 t = top2_empty();
#pragma unroll
    for (int p = 0; p < kFlatPer; p++)
        if (p * 64 + lane < n)
            consider_vals<MAXM>(q, v[p][0], v[p][1], v[p][2], v[p][3], v[p][4], v[p][5],
                                __float_as_int(v[p][6]), t);
    finish_connection<MAXM>(t, out);
}

// the new entries `added` (slot masks, add_to_frontier) of a start joint: connection_value
// with reverse_match (cifcaf.py:194-217) for those whose two column sets are small
template <bool MAXM, typename LDS>
__device__ __forceinline__ void eval_ahead(const GrowArgs &g, Frontier &F, int img, const ColStage &cs,
                                           const SlotSets &ss, uint64_t r0, uint64_t r1, float ax,
                                           float ay, float av, float as, LDS &L) {
    const int lane = threadIdx.x & 63;
    const int64_t hw = g.col_cap;
    r0 &= ss.small[0];  // the others stay lazy
    r1 &= ss.small[1];
    while (r0 | r1) {
#ifdef PP_STAMPS
        uint64_t et = __builtin_amdgcn_s_memtime();
#endif
        int sl[kAhead];
#pragma unroll
        for (int b = 0; b < kAhead; b++) {  // the next kAhead slots
            sl[b] = -1;
            if (r0) {
                sl[b] = __ffsll((unsigned long long)r0) - 1;
                r0 &= r0 - 1;
            } else if (r1) {
                sl[b] = 64 + __ffsll((unsigned long long)r1) - 1;
                r1 &= r1 - 1;
            }
        }
        // both directions' columns of every edge at once: the reverse query's set is known
        // before the forward result (only its start point is not)
        float vf[kAhead][kFlatPer][kColRows], vb[kAhead][kFlatPer][kColRows];
        int nf[kAhead], nb[kAhead], jj[kAhead];
#pragma unroll
        for (int b = 0; b < kAhead; b++) {
            if (sl[b] < 0) continue;
            const int d = sl[b], l = d & 63;
            const bool h = d >= 64;
            const int pf = rl_i(h ? ss.f[1] : ss.f[0], l), pb = rl_i(h ? ss.b[1] : ss.b[0], l);
            const int caf = rl_i(h ? F.scaf[1] : F.scaf[0], l);
            const int df = rl_i(h ? F.sfwd[1] : F.sfwd[0], l) ? 1 : 0;
            jj[b] = rl_i(h ? F.sj[1] : F.sj[0], l);
            nf[b] = pf >> 16;
            nb[b] = pb >> 16;
            flat_load_set(col_set(g, 0, img, caf, df), hw, nf[b], cs.lds, (pf & 0xFFFF) - 1, vf[b]);
            flat_load_set(col_set(g, 0, img, caf, 1 - df), hw, nb[b], cs.lds, (pb & 0xFFFF) - 1,
                          vb[b]);
        }
#ifdef PP_STAMPS
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        ESTAMP(L, 6, et);
#endif
#pragma unroll
        for (int b = 0; b < kAhead; b++) {
            if (sl[b] < 0) continue;
            const int d = sl[b], j = jj[b];
            const float jx = rl_f(ax, j), jy = rl_f(ay, j), jv = rl_f(av, j), js = rl_f(as, j);
            float nx[4];
            flat_query<MAXM>(vf[b], nf[b], jx, jy, max0(js), g.cfg.exp_mode, nx);
#ifdef PP_STAMPS
            ESTAMP(L, 7, et);
#endif
            float res[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            const float ks = sqrtf(nx[3] * jv);
            if (!(ks < g.cfg.keypoint_threshold) && nx[3] != 0.0f) {
                // reverse query from the new point (cifcaf.py:210-214)
                float rv[4];
                flat_query<MAXM>(vb[b], nb[b], nx[0], nx[1], max0(nx[2]), g.cfg.exp_mode, rv);
                if (rv[2] != 0.0f && !(fabsf(jx - rv[0]) + fabsf(jy - rv[1]) > max0(js))) {
                    res[0] = nx[0];
                    res[1] = nx[1];
                    res[2] = nx[2];
                    res[3] = ks;
                }
            }
            if (lane == (d & 63)) {
                if (d < 64) {
                    F.pc[0] = 1;
                    F.px[0] = res[0];
                    F.py[0] = res[1];
                    F.ps[0] = res[2];
                    F.pv[0] = res[3];
                } else {
                    F.pc[1] = 1;
                    F.px[1] = res[0];
                    F.py[1] = res[1];
                    F.ps[1] = res[2];
                    F.pv[1] = res[3];
                }
            }
        }
    }
}

// _grow (cifcaf.py:247-307) on the record in L.a (joint data mirrored into registers).
// AHEAD (seed loop: set A, reverse_match): new entries' connections via eval_ahead from
// the image's set-A column counts and LDS-staged sets.  Force-complete (set B, no reverse
// matching) evaluates each entry when it is popped: evaluating set-B connections ahead, a
// few edges per memory round trip, needed 224 VGPRs (2 waves per SIMD instead of 4) and
// measured slower (planted cfg3 323k vs 331k, uniform 12.4k vs 15.1k-15.7k images/s, round 4).
// `abort` (a seed-loop helper's speculative grow): stop at the next pop once *abort is set
// (wave 0 is done: the result would never be read)
template <bool AHEAD, bool CS, typename LDS>
__device__ __forceinline__ void grow(const GrowArgs &g, LDS &L, int img, int set, bool reverse_match,
                                     const ColStage &cs = ColStage{}, int *abort = nullptr,
                                     float4 *pub = nullptr, uint32_t *pub_mask = nullptr) {
    const int lane = threadIdx.x & 63;
    const int K = g.K;
    float ax = 0.0f, ay = 0.0f, av = 0.0f, as = 0.0f;
    if (lane < K) {
        ax = L.a.data[lane][0];
        ay = L.a.data[lane][1];
        av = L.a.data[lane][2];
        as = L.a.joint_scales[lane];
    }
    int nfr = L.a.n_frontier, ndec = L.a.n_decoding;
    Frontier F;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int d = lane + 64 * r;
        const bool ok = d < g.nd;
        F.st[r] = 0;
        F.added[r] = 0;
        F.neg[r] = 0.0f;
        F.x[r] = F.y[r] = F.s[r] = F.v[r] = 0.0f;
        F.sj[r] = ok ? g.d_j[d] : 0;
        F.sk[r] = ok ? g.d_k[d] : 0;
        F.scaf[r] = ok ? g.d_caf[d] : 0;
        F.sfwd[r] = ok ? g.d_fwd[d] : 0;
        F.pc[r] = 0;
        F.px[r] = F.py[r] = F.ps[r] = F.pv[r] = 0.0f;
    }
    const bool maxm = g.cfg.connection_method == 1;
    SlotSets ss{};
    if (AHEAD) ss = slot_sets(g, cs);
    auto ahead = [&](const uint64_t added[2]) {
        if (!AHEAD || !(added[0] | added[1])) return;
        FSTAMP_BEGIN
        if (maxm)
            eval_ahead<true>(g, F, img, cs, ss, added[0], added[1], ax, ay, av, as, L);
        else
            eval_ahead<false>(g, F, img, cs, ss, added[0], added[1], ax, ay, av, as, L);
        FSTAMP_END(L, 1)
    };
    // `pub` (the seed loop): every joint the annotation holds, as (x, y, v, scale) in LDS as
    // soon as it is set, and its bit in *pub_mask -- a grow in flight shows the helpers'
    // plans which seeds its person's occupancy will cover (joints never change once set)
    if (pub) {
        if (lane < K && av > 0.0f) pub[lane] = make_float4(ax, ay, av, as);
        const uint32_t m0 = (uint32_t)__ballot(lane < K && av > 0.0f);
        if (lane == 0) __hip_atomic_store(pub_mask, m0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    for (int j = 0; j < K; j++) {  // seeding the frontier (cifcaf.py:288-291)
        const float vj = rl_f(av, j);
        if (vj == 0.0f) continue;
        uint64_t added[2];
        add_to_frontier<CS>(g, L, F, av, j, vj, nfr, added);
        ahead(added);
    }
    for (;;) {
        if (abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            break;
        // frontier_get (cifcaf.py:265-285)
        Entry got;
        bool have = false;
        Entry e;
        for (;;) {
            bool popped;
            {
                FSTAMP_BEGIN
                popped = frontier_pop(F, e);
                FSTAMP_END(L, 0)
            }
            if (!popped) break;
            if (e.eval) {
                got = e;
                have = true;
                break;
            }
            if (rl_f(av, e.k) > 0.0f) continue;
            float nx[4];
            if (AHEAD && e.pc) {  // computed ahead when joint e.j entered
                nx[0] = e.px;
                nx[1] = e.py;
                nx[2] = e.ps;
                nx[3] = e.pv;
            } else {
#ifdef PP_STAMPS
                if (lane == 0) L.fst[3] += 1;
#endif
                FSTAMP_BEGIN
                connection_value(g, img, set, e.caf, e.fwd, rl_f(ax, e.j), rl_f(ay, e.j),
                                 rl_f(av, e.j), rl_f(as, e.j), reverse_match, nx);
                FSTAMP_END(L, 1)
            }
            if (nx[3] == 0.0f) continue;
            e.eval = 1;
            // score *= confidence_scales[caf_i] (cifcaf.py:282-284; not on the greedy return)
            e.neg = CS ? -(nx[3] * g.slot_cs[e.slot]) : -nx[3];
            e.x = nx[0];
            e.y = nx[1];
            e.s = nx[2];
            e.v = nx[3];
            if (g.cfg.greedy) {
                got = e;
                have = true;
                break;
            }
            const int sl = e.slot & 63, sr = e.slot >> 6;  // re-push into the edge's slot
            if (lane == sl) {
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    if (r != sr) continue;
                    F.st[r] = 2;
                    F.neg[r] = e.neg;
                    F.x[r] = e.x;
                    F.y[r] = e.y;
                    F.s[r] = e.s;
                    F.v[r] = e.v;
                }
            }
        }
        if (!have) break;
        const int jsi = got.j, jti = got.k;
        if (rl_f(av, jti) > 0.0f) continue;
        if (lane == jti) {  // ann.data[jti] = (x, y, score); joint_scales[jti] = s
            ax = got.x;
            ay = got.y;
            av = got.v;
            as = got.s;
            if (pub) pub[jti] = make_float4(got.x, got.y, got.v, got.s);
        }
        if (pub && lane == 0)
            __hip_atomic_fetch_or(pub_mask, 1u << jti, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane == 0) {
            if (ndec < kKP) {
                L.a.decoding_pairs[ndec][0] = (uint8_t)jsi;
                L.a.decoding_pairs[ndec][1] = (uint8_t)jti;
                L.a.decoding_xyv[ndec][0] = rl_f(ax, jsi);
                L.a.decoding_xyv[ndec][1] = rl_f(ay, jsi);
                L.a.decoding_xyv[ndec][2] = rl_f(av, jsi);
                L.a.decoding_xyv[ndec][3] = got.x;
                L.a.decoding_xyv[ndec][4] = got.y;
                L.a.decoding_xyv[ndec][5] = got.v;
            } else {
                L.status |= PP_ST_DEC_OVERFLOW;
            }
        }
        ndec++;
        uint64_t added[2];
        {
            FSTAMP_BEGIN
            add_to_frontier<CS>(g, L, F, av, jti, got.v, nfr, added);
            FSTAMP_END(L, 2)
        }
        ahead(added);
    }
    if (nfr > PP_MAX_FRONTIER && lane == 0) L.status |= PP_ST_DEC_OVERFLOW;
    if (lane < K) {
        L.a.data[lane][0] = ax;
        L.a.data[lane][1] = ay;
        L.a.data[lane][2] = av;
        L.a.joint_scales[lane] = as;
    }
    if (lane == 0) {
        L.a.n_frontier = nfr;
        L.a.n_decoding = ndec;
    }
    wave_sync();
}

// cifcaf.py:309-331 (the key is the ENCLOSING xyv, App. D item 5)
__device__ __forceinline__ void flood_fill(const GrowArgs &g, GrowLDS &L) {  // (inlined: a call would copy GrowArgs to scratch)
    L.ff_n = 0;
    auto add = [&](int start_i, float key_v) {
        for (int e = g.j_off[start_i]; e < g.j_off[start_i + 1]; e++) {
            const int end_i = g.d_k[e];
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
// u8 planes (f, h, w) stored with a row pitch of round_up(w, 16) bytes, so that no two
// rows (and no two planes) share a 16-byte chunk: marking updates whole chunks.
struct OccGrid {
    uint8_t *p;
    int f, h, w, pitch;
};

__device__ __forceinline__ OccGrid occ_grid(uint8_t *p, int f, int h, int w) {
    return OccGrid{p, f, h, w, (w + 15) & ~15};
}

__device__ __forceinline__ long round_half_even(float x) { return (long)rintf(x); }

// Occupancy.get (occupancy.py:41-47): nonzero at floor((x, y) / reduction), clipped
__device__ __forceinline__ bool occ_get(const OccGrid &o, int f, float x, float y, float red) {
    if (f >= o.f) return true;
    if (o.h <= 0 || o.w <= 0) return false;  // the reference reads out of bounds here
    x = clip_ref(x / red, 0.0f, (float)(o.w - 1));
    y = clip_ref(y / red, 0.0f, (float)(o.h - 1));
    const int xi = (int)x, yi = (int)y;
    return o.p[((int64_t)f * o.h + yi) * o.pitch + xi] != 0;
}

// Occupancy.set box (occupancy.py:31-39 + utils.py:61-66) of joint f; false when empty.
// red = reduction, msr = min_scale / reduction (occ_box below takes them from the config)
__device__ __forceinline__ bool occ_box_r(float red, float msr, const OccGrid &o, int f, float x,
                                          float y, float sigma, int box[4]) {
    if (f >= o.f) return false;
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

__device__ __forceinline__ float occ_msr(const GrowArgs &g) {
    return (float)((double)g.cfg.occupancy_min_scale / g.cfg.occupancy_reduction);
}

__device__ __forceinline__ bool occ_box(const GrowArgs &g, const OccGrid &o, int f, float x, float y, float sigma,
                        int box[4]) {
    return occ_box_r((float)g.cfg.occupancy_reduction, occ_msr(g), o, f, x, y, sigma, box);
}

// Mark the boxes of every joint j with mark(j) in one pass: joints live on different
// occupancy planes, so the per-joint `+= 1` boxes are independent and spread over the 64
// lanes.  Each marked box is logged for occ_clear.  Collective (all 64 lanes).
// lane j < K holds joint j: (jx, jy), scale js, `on` = mark it
template <typename LDS>
__device__ __forceinline__ void occ_mark(const GrowArgs &g, LDS &L, OccLog *log, const OccGrid &o,
                                         float jx, float jy, float js, bool on, int K) {
    const int lane = threadIdx.x & 63;
    int box[4] = {0, 0, 0, 0};
    bool has = false;
    if (lane < K && on) has = occ_box(g, o, lane, jx, jy, js, box);
    // work items: (row, 16-byte chunk) pairs of the box
    const int area = has ? (box[3] - box[2]) * (((box[1] - 1) >> 4) - (box[0] >> 4) + 1) : 0;
    int pre = 0, total = 0;
    for (int i = 0; i < K; i++) {  // exclusive prefix of the box areas (uniform loop)
        const int ai = rl_i(area, i);
        pre += (i < lane) ? ai : 0;
        total += ai;
    }
    const uint64_t hm = __ballot(has);
    if (lane < K) {
        L.mark_pre[lane] = pre;
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
    wave_sync();
    // Within one call every chunk is updated by one lane only (one box per joint plane,
    // rows padded to whole chunks), so a batch of chunks is loaded before any is stored.
    // u8 += 1 with wrap on the bytes inside the box: ((v & 0x7f..) + inc) ^ (v & 0x80..).
    constexpr int kB = 4;
    for (int t0 = 0; t0 < total; t0 += 64 * kB) {
        uint4 *cell[kB];
        uint4 inc[kB], val[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int t = t0 + u * 64 + lane;
            cell[u] = nullptr;
            inc[u] = make_uint4(0, 0, 0, 0);
            if (t < total) {
                int lo = 0, hi = K - 1;  // largest joint whose item prefix <= t
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (L.mark_pre[mid] <= t)
                        lo = mid;
                    else
                        hi = mid - 1;
                }
                const int r = t - L.mark_pre[lo];
                const int x0 = L.mark_box[lo][0], x1 = L.mark_box[lo][1];
                const int c0 = x0 >> 4, nch = ((x1 - 1) >> 4) - c0 + 1;
                const int yy = L.mark_box[lo][2] + r / nch, cx = (c0 + r % nch) << 4;
                cell[u] = reinterpret_cast<uint4 *>(&o.p[((int64_t)lo * o.h + yy) * o.pitch + cx]);
                uint32_t w4[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    uint32_t m = 0;
#pragma unroll
                    for (int bq = 0; bq < 4; bq++) {
                        const int x = cx + 4 * q + bq;
                        m |= (x >= x0 && x < x1) ? (1u << (8 * bq)) : 0u;
                    }
                    w4[q] = m;
                }
                inc[u] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < kB; u++) val[u] = cell[u] ? *cell[u] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < kB; u++) {
            if (!cell[u]) continue;
            const uint4 v = val[u], m = inc[u];
            *cell[u] = make_uint4(((v.x & 0x7F7F7F7Fu) + m.x) ^ (v.x & 0x80808080u),
                                  ((v.y & 0x7F7F7F7Fu) + m.y) ^ (v.y & 0x80808080u),
                                  ((v.z & 0x7F7F7F7Fu) + m.z) ^ (v.z & 0x80808080u),
                                  ((v.w & 0x7F7F7F7Fu) + m.w) ^ (v.w & 0x80808080u));
        }
    }
    const int nm = __popcll(hm);
    if (L.log_n + nm > g.log_cap) L.status |= PP_ST_NMS_OVERFLOW;
    wave_sync();
    L.log_n = L.log_n + nm;
    wave_sync();
}

// zero every box the launch marked, so the next launch starts from a clean grid
// ---- the seed loop's occupancy as per-seed counters in LDS ----
// The seed loop reads its occupancy grid only at seed positions (cifcaf.py:100-102: the
// free-seed test; the helpers' plans), so for an image with at most kOccSeeds seeds the
// grid is replaced by one u8 counter per seed: a mark adds 1 (wrapping, as the grid's
// `+= 1`, utils.py:66) to every seed of the joint's field whose grid cell lies in the
// joint's box, and a seed is occupied iff its counter is nonzero -- exactly the grid's
// cell value there.  Marks and tests stay in LDS: no global read-modify-write, no clearing.
constexpr int kOccSeeds = 2560;
// Counters, cells and fields are stored by the seeds' position p in field-grouped order (pos:
// seed index -> p), so that a mark reads one seed's cell, field and counter in one LDS round
// trip, four seeds per lane at once, over all the marked joints' fields in one sweep.
struct SeedOcc {
    uint8_t cnt[kOccSeeds];     // counter per position
    uint8_t fld[kOccSeeds];     // field per position
    uint32_t cell[kOccSeeds];   // grid cell (yi << 16 | xi) per position
    uint16_t pos[kOccSeeds];    // position of each seed index
    int foff[kKP + 1];          // field f's positions: foff[f] .. foff[f + 1]
    int fcur[kKP];
    int n;
};

__device__ __forceinline__ bool seed_occupied(const SeedOcc &O, int idx) { return O.cnt[O.pos[idx]] != 0; }

// collective over the workgroup (ends with a barrier): the counters and field groups of
// the image's n <= kOccSeeds seeds
__device__ __forceinline__ void seed_occ_init(SeedOcc &O, const pp_seed *seeds, int n, int K,
                                              const OccGrid &o, float red) {
    if (threadIdx.x < kKP) O.fcur[threadIdx.x] = 0;
    if (threadIdx.x == 0) O.n = n;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&O.fcur[seeds[i].field], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = 0;
        for (int f = 0; f < K; f++) {
            O.foff[f] = a;
            a += O.fcur[f];
            O.fcur[f] = 0;
        }
        O.foff[K] = a;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const pp_seed c = seeds[i];
        const int xi = (int)clip_ref(c.x / red, 0.0f, (float)(o.w - 1));  // occ_get's cell
        const int yi = (int)clip_ref(c.y / red, 0.0f, (float)(o.h - 1));
        const int p = O.foff[c.field] + atomicAdd(&O.fcur[c.field], 1);
        O.pos[i] = (uint16_t)p;
        O.cell[p] = ((uint32_t)yi << 16) | (uint32_t)xi;
        O.fld[p] = (uint8_t)c.field;
        O.cnt[p] = 0;
    }
    __syncthreads();
}

// occ_mark on the counters (one wave): lane j < K holds joint j (x, y, scale, `on`).  Each
// position is one seed of one field, so a sweep touches every counter at most once (no
// races between lanes); a seed whose field's joint is marked gets +1 if its cell is in the
// joint's box (the box from lane `field`, ds_bpermute).
__device__ __forceinline__ void seed_occ_mark(const GrowArgs &g, SeedOcc &O, const OccGrid &o,
                                              float jx, float jy, float js, bool on, int K) {
    const int lane = threadIdx.x & 63;
    int box[4] = {0, 0, 0, 0};
    const bool has = lane < K && on && occ_box(g, o, lane, jx, jy, js, box);
    const uint64_t hm = __ballot(has);
    if (hm) {
        const int n = O.n;
        constexpr int kU = 4;
        for (int p0 = 0; p0 < n; p0 += 64 * kU) {
            uint32_t c[kU];
            int f[kU], v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int p = p0 + u * 64 + lane;
                const bool in = p < n;
                c[u] = in ? O.cell[p] : 0u;
                f[u] = in ? (int)O.fld[p] : 0;
                v[u] = in ? (int)O.cnt[p] : 0;
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const int p = p0 + u * 64 + lane;
                const int x0 = __shfl(box[0], f[u]), x1 = __shfl(box[1], f[u]);
                const int y0 = __shfl(box[2], f[u]), y1 = __shfl(box[3], f[u]);
                const int xi = (int)(c[u] & 0xFFFFu), yi = (int)(c[u] >> 16);
                if (p < n && ((hm >> f[u]) & 1ull) && xi >= x0 && xi < x1 && yi >= y0 && yi < y1)
                    O.cnt[p] = (uint8_t)(v[u] + 1);
            }
        }
    }
    wave_sync();
}

template <typename LDS>
__device__ __forceinline__ void occ_clear(const GrowArgs &g, LDS &L, OccLog *log, const OccGrid &o) {
    wave_sync();
    const int n = L.log_n < g.log_cap ? L.log_n : g.log_cap;
    const int lane = threadIdx.x & 63;
    for (int e0 = 0; e0 < n; e0 += 64) {  // 64 boxes per round, one per lane
        const int e = e0 + lane;
        OccLog l{0, 0, 0, 0, 0};
        if (e < n) l = log[e];
        // bytes outside the marked boxes are zero already: clear whole chunks
        const int c0 = l.x0 >> 4, nch = (e < n) ? ((l.x1 - 1) >> 4) - c0 + 1 : 0;
        const int items = (e < n) ? nch * (l.y1 - l.y0) : 0;
        for (int t = 0; t < items; t++) {
            uint8_t *c = &o.p[((int64_t)l.f * o.h + l.y0 + t / nch) * o.pitch + ((c0 + t % nch) << 4)];
            *reinterpret_cast<uint4 *>(c) = make_uint4(0, 0, 0, 0);
        }
    }
    L.log_n = 0;
    wave_sync();
}

// np.sum of K float64 terms in NumPy's pairwise order (n <= 128: eight accumulators over
// blocks of 8, combined as ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the tail)
__device__ double pw_sum(const double *a, int K) {
    if (K < 8) {
        double res = 0.0;
        for (int i = 0; i < K; i++) res += a[i];
        return res;
    }
    double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
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
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < K; i++) res += a[i];
    return res;
}

// all loads first, then all stores: one round trip (the two records may alias as far as the
// compiler knows, so a plain copy loop waits for every load in turn)
// a record copy in two halves, so that other work overlaps the loads' latency: the loads
// into registers (per lane kAnnWords words), then the stores
constexpr int kAnnWords = (int)((sizeof(pp_ann) / 4 + 63) / 64);
struct AnnRegs {
    uint32_t v[kAnnWords];
};
__device__ __forceinline__ AnnRegs ann_load(const pp_ann *src) {
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    constexpr int nw = sizeof(pp_ann) / 4;
    const int lane = threadIdx.x & 63;
    AnnRegs r;
#pragma unroll
    for (int u = 0; u < kAnnWords; u++) r.v[u] = (u * 64 + lane < nw) ? s[u * 64 + lane] : 0u;
    return r;
}
__device__ __forceinline__ void ann_store(pp_ann *dst, const AnnRegs &r) {
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    constexpr int nw = sizeof(pp_ann) / 4;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < kAnnWords; u++)
        if (u * 64 + lane < nw) d[u * 64 + lane] = r.v[u];
    wave_sync();
}

__device__ __forceinline__ void copy_ann(pp_ann *dst, const pp_ann *src) {
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    constexpr int nw = sizeof(pp_ann) / 4;
    constexpr int per = (nw + 63) / 64;
    const int lane = threadIdx.x & 63;
    uint32_t v[per];
#pragma unroll
    for (int u = 0; u < per; u++) v[u] = (u * 64 + lane < nw) ? s[u * 64 + lane] : 0u;
#pragma unroll
    for (int u = 0; u < per; u++)
        if (u * 64 + lane < nw) d[u * 64 + lane] = v[u];
    wave_sync();
}

// stable sort of idx[0..n) by descending score (sorted(anns, key=lambda a: -a.score()))
__device__ void sort_by_score(int *perm, int np, int n, const double *score) {
    for (int i = threadIdx.x & 63; i < np; i += 64) perm[i] = i;
    wave_sync();
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
            wave_sync();
        }
    }
}

// ---------------------------------------------------------------------------------------
// seed loop (cifcaf.py:84-108): one workgroup of kSeedWaves waves per image
// ---------------------------------------------------------------------------------------
// The loop is sequential: whether a seed starts an annotation depends on the occupancy
// marks of every annotation before it.  But _grow from a seed is a pure function of the
// seed and the CAF columns, so helper waves grow seeds the loop is LIKELY to reach next
// while wave 0 grows the one it needs now; wave 0 then commits strictly in the reference
// order (the next free seed, cifcaf.py:100-104) and takes a seed's annotation from the
// cache when a helper grew it already.  Speculation only changes WHEN an annotation is
// computed, never which seeds start one or what they contain.
//
// Helpers pick free seeds after the committed one that lie far (kSpecFar joint scales,
// Chebyshev) from it, from each other and from the cached ones, since seeds near an
// annotation's joints are the ones its occupancy marks will cover.
//
// Nothing waits for the slowest wave: wave 0 hands a seed to each IDLE helper when it has
// to grow one itself, and a helper publishes its annotation (cache slot state 2) whenever
// it finishes.  Wave 0 waits on a helper only for the seed it needs next, if that helper
// is still growing it.  The handshake is LDS flags with workgroup-scope acquire/release.
// 8 waves; 16 (cache 32, scan 256): 1.79 vs 1.28 ms per cfg3 step; 4 / 6: no better
constexpr int kSeedWaves = 8;
constexpr int kSpecCache = 16;     // speculative annotations of this CU's helpers
constexpr int kSpecScan = 128;     // seeds after the committed one examined per round
// distance (joint scales) a helper's seed keeps from the committed one and from the
// round's other picks; cached annotations are excluded by their exact occupancy boxes.
// Throughput is flat for 0-4 (both generators) and drops beyond 8.
constexpr float kSpecFar = 4.0f;
constexpr int kSelfScan = 256;     // seeds after the decided ones a finished helper examines
// seeds after the committed one that wave 0 of seed_loop_ext_kernel examines per plan round
// (cfg5 planted 42.9k-43.7k -> 45.8k-47.0k images/s with 512 instead of 128, round 6)
constexpr int kExtScan = 512;
// the external-helper plan's speculation distance (joint scales): 1 instead of kSpecFar's 4
// (cfg5 planted 45.5k-46.9k -> 50.3k-50.4k images/s, uniform 1513-1517 vs 1518-1527; with 1
// for the one-CU kernel too, planted cfg3 was 415k vs 415k-420k and uniform 16.1k-16.3k vs
// 16.0k; round 6, r06z_ab_spec_far.txt)
constexpr float kExtSpecFar = 1.0f;
// Wave 0 of seed_loop_ext_kernel plans the idle helpers when it has to grow a seed itself (a
// miss), and, on images of kExtRefillAnns annotations or more, also after a cached commit that
// leaves fewer than kExtRefill speculated seeds ahead: a dense image otherwise ran its helpers
// dry between misses (~77 of ~1370 seeds per cfg5 uniform image grown by wave 0 itself, each a
// whole grow on the critical path, r06h stamps).  cfg5 uniform 1510-1545 -> 1562-1737 images/s
// with 12 (8: 1616-1661, 16: no gain, 20: 1558-1576; planted unchanged from 32 annotations on,
// -2 % when refilling on every image; r06z_ab_refill.txt).
constexpr int kExtRefillAnns = 32;
constexpr int kExtRefill = 12;
// Both plans exclude a seed only for annotations that come BEFORE it in seed order: near a
// seed in flight, inside the occupancy boxes of a grown annotation or of the joints an
// in-flight grow has set so far, when that annotation's seed precedes it (wave 0 commits it
// first, and its boxes then cover the seed).  An annotation whose seed comes after cannot
// cover it at its turn, so excluding it there only made wave 0 grow it itself (cfg5 planted
// 39.4k-40.2k -> 42.9k-43.7k, planted cfg3 406k-413k -> 415k-416k; round 6).
// Who plans the idle helpers when wave 0 has to grow a seed itself: an idle helper, so that
// wave 0 starts its grow at once and the plan (a scan of kSpecScan seeds against the cache,
// about 50k cycles, stamps) is off the committer's path (wave 0 planning before its grow
// measured no faster, round 5).  Wave 0 publishes its seed without the plan lock: a plan
// that misses it only grows a seed twice, which never changes a result.  A helper that
// finishes plans its own next grow (the external helpers of seed_loop_ext_kernel do not:
// cfg5 uniform 725 vs 1080 images/s with it, round 4), and a helper whose plan found
// nothing plans again once wave 0 has committed or passed a seed (idle_dec): a wave 0 that
// only takes cached annotations never misses, so never requests a plan.  Uniform cfg3
// (round 6, A/B on one box): the slot-register plan alone 15.2-15.3k images/s, with the
// re-plan 16.3-16.5k, the round-5 plan 15.7-15.9k.
// Grows in flight publish their joints as they are set (grow's `pub`), and the plans keep
// seeds their occupancy boxes will cover away from the helpers.  Planted cfg3 (stamps,
// serial): at kernel start about 4 of the 7 first picks are seeds the loop commits
// (tools/spec_sim.py).  (Helper waves at issue priority 2 measured no faster, round 5.)

// External helpers.  A batch of fewer images than CUs leaves CUs without a seed loop, so
// each image may get n_ext (<= kExtWgMax) more workgroups whose waves are all helpers.
// They take seeds from wave 0 through per-image global words (SeedExt) and publish into
// kExtCache more cache slots, whose records live in global memory, across CUs and XCDs
// with the agent-scope publish / consume form of cdna_hip_programming.md Guideline 16: the
// record is stored write-through (sc1) and drained (s_waitcnt vmcnt(0)) before one lane
// stores the slot's tag (seed + 1); wave 0 polls tags relaxed and reads records and joints
// with sc1 loads.  A helper announces itself (task word 1 = idle) before wave 0 may hand
// it a seed (CAS 1 -> assigned), so a workgroup that is not resident never holds one; an
// idle helper leaves when wave 0 finishes (fin) or after kExtIdleTicks without work (CAS
// 1 -> 3; losing that CAS to an assignment means: grow it).  The image's workgroups count
// themselves out (SeedExt.exited) after their last access to these words, and the last one
// out zeroes them, so every launch finds them zero whatever runs between two seed loops.
constexpr int kExtWgMax = 3;
constexpr int kExtHelpers = kExtWgMax * kSeedWaves;
constexpr int kExtCache = 32;
constexpr int kCacheSlots = kSpecCache + kExtCache;  // one lane per slot
static_assert(kCacheSlots <= 64 && kSeedWaves + kExtHelpers <= 64, "one lane per slot / helper");
// Policy (s_memrealtime ticks, 100 MHz).  Wave 0 waits for an external slot it needs next
// only if that grow is at least half done by the running mean of external grows (at most
// 2 s: a helper always finishes); otherwise it grows the seed itself and the slot is a
// zombie (state 4) until its tag arrives.  An idle helper leaves after 300 us, so that on
// images with few annotations its CU goes back to the other stages' kernels; once an image
// has kExtHeavyAnns annotations wave 0 flags it heavy (SeedExt.heavy) and helpers stay up
// to 1 s idle.  cfg5 (64 images, 160x160; 16 / 1370 annotations per image), images/s,
// planted / uniform: no helpers 26.4k / 795; this 27.7k / 969; helpers that stay 1 ms idle
// 22.7k / 1024; wave 0 always waiting 22.5k / 1027; also handing out seeds after every 4th
// cached commit 21.7k / 986; a 100 us light idle and no wait before 32 annotations 27.0k / 907.
constexpr int kExtHeavyAnns = 8;
constexpr uint64_t kExtIdleLight = 30000ull, kExtIdleHeavy = 100000000ull;
constexpr uint64_t kExtWaitMax = 200000000ull;
// (Wave 0 planning the idle helpers while it waits for one, once per wait, when that grow is
// expected to run 40 us longer on images of 32+ annotations: cfg5 uniform 1445-1724 vs
// 1670 images/s without, planted 39.8-41.2k vs 40.4-43.5k, round 6.)

struct SeedExt {  // per image; zero at every launch (workspace zero region; the launch's
                  // last workgroup out re-zeroes it, ext_exit)
    unsigned long long task[kExtHelpers];  // 0 absent, 1 idle, 3 left; assigned: 2 |
                                           // slot << 8 | seed << 32
    unsigned int tag[kExtCache];           // seed + 1 of the record published in the slot
    unsigned int fin;                      // wave 0 is done
    unsigned int heavy;                    // wave 0 switched to the heavy regime
    unsigned int exited;                   // workgroups of the image done with these words
    unsigned int pad;
};
static_assert(sizeof(SeedExt) % 16 == 0, "memset block of whole 16-byte units");

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ unsigned int ld_agent(const unsigned int *p) {
    return __hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p) {
    return __hip_atomic_load((gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned int *p, unsigned int v) {
    __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool cas_agent(unsigned long long *p, unsigned long long expect,
                                          unsigned long long v) {
    return __hip_atomic_compare_exchange_strong((gu64 *)p, &expect, v, __ATOMIC_RELAXED,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0's CAS, its result on every lane
__device__ __forceinline__ bool cas_agent_wave(unsigned long long *p, unsigned long long expect,
                                               unsigned long long v) {
    int ok = 0;
    if ((threadIdx.x & 63) == 0) ok = cas_agent(p, expect, v) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(ok) != 0;
}

// One of an image's 1 + n_ext workgroups is done with its SeedExt words (called by every
// thread after a __syncthreads that follows the workgroup's last access to them): it counts
// itself out, and the last one out zeroes the words for the workspace's next seed loop.
// Every workgroup of the image runs (a helper that was not resident before wave 0 finished
// starts later, sees fin and leaves), so exactly one sees the count reach n_ext, after
// every other workgroup's last access.  The workspace contract (zero at each launch) then
// holds after any stage split (PP_STAGE_SEED_LOOP_ONLY with or without the NMS call).
__device__ __forceinline__ void ext_exit(SeedExt *X, int n_ext) {
    if (!X || threadIdx.x != 0) return;
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const unsigned int before = __hip_atomic_fetch_add((gu32 *)&X->exited, 1u, __ATOMIC_ACQ_REL,
                                                       __HIP_MEMORY_SCOPE_AGENT);
    if (before != (unsigned int)n_ext) return;
    unsigned int *w = reinterpret_cast<unsigned int *>(X);
    for (int t = 0; t < (int)(sizeof(SeedExt) / 4); t++) st_agent(w + t, 0u);
}

// an LDS record to global memory, write-through (sc1), drained
__device__ __forceinline__ void publish_ann(pp_ann *dst, const pp_ann *src) {
    const unsigned long long *s = reinterpret_cast<const unsigned long long *>(src);
    unsigned long long *d = reinterpret_cast<unsigned long long *>(dst);
    constexpr int nw = sizeof(pp_ann) / 8;
    for (int t = threadIdx.x & 63; t < nw; t += 64) st_agent(d + t, s[t]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// copy_ann from another CU's published record (sc1 loads)
__device__ __forceinline__ void copy_ann_agent(pp_ann *dst, const pp_ann *src) {
    const unsigned long long *s = reinterpret_cast<const unsigned long long *>(src);
    unsigned long long *d = reinterpret_cast<unsigned long long *>(dst);
    constexpr int nw = sizeof(pp_ann) / 8;
    constexpr int per = (nw + 63) / 64;
    const int lane = threadIdx.x & 63;
    unsigned long long v[per];
#pragma unroll
    for (int u = 0; u < per; u++) v[u] = (u * 64 + lane < nw) ? ld_agent(s + u * 64 + lane) : 0ull;
#pragma unroll
    for (int u = 0; u < per; u++)
        if (u * 64 + lane < nw) d[u * 64 + lane] = v[u];
    wave_sync();
}

template <int NSLOT>
struct SeedLoopSharedT {
    int task[kSeedWaves];          // seed a helper is to grow (-1 idle), set by wave 0
    int task_slot[kSeedWaves];     // cache slot its annotation goes to
    int cache_seed[NSLOT];         // seed index held by a cache slot (< current: dead)
    float cache_x[NSLOT], cache_y[NSLOT], cache_s[NSLOT];  // seed position
    // 0 free, 1 being grown, 2 grown (joints below valid), 4 zombie (external slot whose
    // seed wave 0 grew itself; free once its tag arrives); external slots' 1 -> 2 and
    // 4 -> 0 are wave 0's, on seeing the slot's tag
    int cache_state[NSLOT];
    float4 cache_j[kSpecCache][kKP];  // its joints (x, y, v, scale); the external slots'
                                      // after the column stage in dynamic LDS (cache_joints)
    // seed_loop_kernel: joints of a slot still being grown that are set already (bit j:
    // cache_j[q][j] holds joint j; grow's `pub`), and the same for wave 0's own grow
    uint32_t cache_pm[kSpecCache];
    float4 own_j[kKP];
    uint32_t own_pm;
    int done;
    // seed_loop_kernel's helper self-planning (spec_plan): the plan lock, the first seed not
    // yet decided by wave 0 (seeds before it were committed or skipped), and the seed wave 0
    // grows itself now (own_on)
    int plan_lock, decided, own_on;
    float own_x, own_y, own_s;
    // seed_loop_kernel: wave 0 started a grow of its own; an idle helper plans the others
    int plan_req;
};
struct SeedLoopShared : SeedLoopSharedT<kSpecCache> {
    uint2 cache_box[kSpecCache][kKP];  // the grown slots' occupancy boxes (plan_box)
};
// (kColLds above keeps the one-CU seed loop's LDS at 124,608 bytes with these and SeedOcc)
struct SeedLoopSharedX : SeedLoopSharedT<kCacheSlots> {
    uint32_t cache_t[kCacheSlots];  // external slots: s_memrealtime (low bits) at hand-over
    uint32_t ext_ticks;             // running mean of hand-over -> tag seen (0: none yet)
};

// joints of cache slot q (LDS): this CU's slots in SeedLoopShared, the external ones in the
// dynamic LDS after the kColLdsExt column floats (launched only when n_ext > 0)
__device__ __forceinline__ float4 *cache_joints(SeedLoopSharedX &S, float *s_cols, int q) {
    return q < kSpecCache ? S.cache_j[q]
                          : reinterpret_cast<float4 *>(s_cols + kColLdsExt) + (q - kSpecCache) * kKP;
}
// The occupancy boxes a grown slot's joints will mark once committed (occ_box_r), for the
// plan of seed_loop_ext_kernel: written with the joints, before the slot's state 2, so a
// plan tests a seed against a slot with one LDS read.  Packed x0 | x1 << 16, y0 | y1 << 16;
// an empty box is 0, 0.  (An occupancy grid of 2^16 cells or more per side, reduction < 1,
// garbles them: that only changes which seeds the helpers grow ahead, never a result.)
// After the external joints in the dynamic LDS, one row of kKP per slot (all kCacheSlots).
constexpr size_t kExtDynLds = kColLdsExt * sizeof(float) + (size_t)kExtCache * kKP * sizeof(float4) +
                              (size_t)kCacheSlots * kKP * sizeof(uint2);
__device__ __forceinline__ uint2 *cache_boxes(float *s_cols, int q) {
    return reinterpret_cast<uint2 *>(reinterpret_cast<float4 *>(s_cols + kColLdsExt) + kExtCache * kKP) +
           q * kKP;
}
__device__ __forceinline__ uint2 plan_box(float red, float msr, const OccGrid &o, int f, float4 j) {
    int box[4];
    if (j.z == 0.0f || !occ_box_r(red, msr, o, f, j.x, j.y, j.w, box)) return make_uint2(0u, 0u);
    return make_uint2((uint32_t)box[0] | ((uint32_t)box[1] << 16),
                      (uint32_t)box[2] | ((uint32_t)box[3] << 16));
}
__device__ __forceinline__ bool in_plan_box(uint2 b, int cx, int cy) {
    return cx >= (int)(b.x & 0xFFFFu) && cx < (int)(b.x >> 16) && cy >= (int)(b.y & 0xFFFFu) &&
           cy < (int)(b.y >> 16);
}

__device__ __forceinline__ int lds_acquire(int *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_acquire_u(uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ bool spec_far(float far, float xa, float ya, float sa, float xb,
                                         float yb, float sb) {
    const float r = far * fmaxf(fmaxf(sa, sb), 1.0f);
    return fabsf(xa - xb) > r || fabsf(ya - yb) > r;
}

// Annotation(keypoints, out_skeleton).add(f, (x, y, v)); joint_scales[f] = s
template <typename LDS>
__device__ __forceinline__ void ann_from_seed(LDS &L, const pp_seed &sd, int K, int img) {
    const int lane = threadIdx.x & 63;
    uint32_t *z = reinterpret_cast<uint32_t *>(&L.a);
    for (int t = lane; t < (int)(sizeof(pp_ann) / 4); t += 64) z[t] = 0u;
    wave_sync();
    if (lane == 0) {
        L.a.n_keypoints = K;
        L.a.image = img;
        L.a.data[sd.field][0] = sd.x;
        L.a.data[sd.field][1] = sd.y;
        L.a.data[sd.field][2] = sd.v;
        L.a.joint_scales[sd.field] = sd.s;
    }
    wave_sync();
}

// wave 0: external slots being grown whose tag has arrived become grown (joints into LDS);
// `only` >= 0 restricts the check to that slot
__device__ __forceinline__ void ext_refresh(SeedLoopSharedX &S, float *s_cols, const SeedExt *X,
                                            const pp_ann *xrec, int only, float red, float msr,
                                            const OccGrid &occ) {
    const int lane = threadIdx.x & 63;
    const int q = kSpecCache + lane;
    bool ready = false;
    const int st = lane < kExtCache ? S.cache_state[q] : 0;
    if (lane < kExtCache && (only < 0 || only == q) && (st == 1 || st == 4))
        ready = ld_agent(&X->tag[lane]) == (unsigned int)S.cache_seed[q] + 1u;
    if (ready && st == 4) {  // the zombie's helper is done: free
        S.cache_state[q] = 0;
        ready = false;
    }
    wave_sync();
    const uint64_t rm = __ballot(ready);
    if (rm) {
        const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime();
        const uint32_t dur = ready ? now - S.cache_t[q] : 0u;
        uint32_t mt = S.ext_ticks;
        for (uint64_t b = rm; b; b &= b - 1) {
            const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)dur, __ffsll((unsigned long long)b) - 1);
            mt = mt ? 3u * (mt >> 2) + (d >> 2) : d;
        }
        wave_sync();
        if (lane == 0) S.ext_ticks = mt;
    }
    for (uint64_t m = rm; m; m &= m - 1) {
        const int e = __ffsll((unsigned long long)m) - 1;
        const pp_ann *r = xrec + e;
        if (lane < kKP) {
            const unsigned int *d = reinterpret_cast<const unsigned int *>(&r->data[lane][0]);
            const float4 j = make_float4(
                __uint_as_float(ld_agent(d)), __uint_as_float(ld_agent(d + 1)),
                __uint_as_float(ld_agent(d + 2)),
                __uint_as_float(ld_agent(reinterpret_cast<const unsigned int *>(&r->joint_scales[lane]))));
            cache_joints(S, s_cols, kSpecCache + e)[lane] = j;
            cache_boxes(s_cols, kSpecCache + e)[lane] = plan_box(red, msr, occ, lane, j);
        }
        wave_sync();
        if (lane == 0) S.cache_state[kSpecCache + e] = 2;
        wave_sync();
    }
}

// Speculation plan of seed_loop_kernel, collective over one wave, with S.plan_lock held:
// free seeds in [decided, decided + scan) that the committed occupancy and the cached
// annotations' occupancy boxes do not cover (the grown ones' boxes, S.cache_box, and the
// joints set so far of those in flight, cache_pm / own_pm), kSpecFar joint scales from
// every seed in flight (and from wave 0's own seed when S.own_on), each into a free cache
// slot (never used, or holding a seed before `decided`), for the helper waves in `idle`
// (bit w = wave w), which get their seeds through S.task.  Returns the helpers left idle.
// A slot is claimed state first, seed second (both released): wave 0 reads the seed without
// the lock and, seeing its seed there, waits for state 2.
// The slots are read once, a lane each (only the plan, under the lock, claims slots; a
// helper turning 1 into 2 meanwhile at most keeps this plan from reusing that slot), and
// kept current for the plan's own picks; per seed the slots are tested with SGPR operands
// (readlane), the grown ones' boxes four per LDS round trip.
// Not inlined: it runs outside the grow and takes no GrowArgs (a non-inlined reference to
// the kernarg struct makes the compiler copy it to scratch), so the kernel's registers stay
// the grow's.
__device__ __noinline__ uint64_t spec_plan(SeedLoopShared &S, const pp_seed *seeds, int n_seeds,
                                           int decided, int scan, OccGrid occ, float red,
                                           float msr, float far_k, uint64_t idle,
                                           const SeedOcc *socc) {
    constexpr int NS = kSpecCache;
    const int lane = threadIdx.x & 63;
    const bool sl = lane < NS;
    int r_st = sl ? lds_acquire(&S.cache_state[lane]) : 0;
    int r_seed = sl ? S.cache_seed[lane] : -1;
    float r_x = sl ? S.cache_x[lane] : 0.0f, r_y = sl ? S.cache_y[lane] : 0.0f,
          r_s = sl ? S.cache_s[lane] : 0.0f;
    uint64_t fly = __ballot(sl && r_st == 1);
    const bool own = lds_acquire(&S.own_on) != 0;
    const float ox = S.own_x, oy = S.own_y, osc = S.own_s;
    const int scan_end = min(n_seeds, decided + scan);
    for (int base = decided; base < scan_end && idle; base += 64) {
        const int idx = base + lane;
        bool ok = idx < scan_end;
        pp_seed c{};
        if (ok) {
            c = seeds[idx];
            ok = (!own || spec_far(far_k, c.x, c.y, c.s, ox, oy, osc)) &&
                 !(socc ? seed_occupied(*socc, idx) : occ_get(occ, c.field, c.x, c.y, red));
        }
        const int cxi = (int)clip_ref(c.x / red, 0.0f, (float)(occ.w - 1));
        const int cyi = (int)clip_ref(c.y / red, 0.0f, (float)(occ.h - 1));
        const int cf = c.field;
        // inside the occupancy box joint jq of an annotation will mark (occupancy.py:31-39)
        auto covered = [&](const float4 &jq) {
            int box[4];
            return jq.z != 0.0f && occ_box_r(red, msr, occ, cf, jq.x, jq.y, jq.w, box) &&
                   cxi >= box[0] && cxi < box[1] && cyi >= box[2] && cyi < box[3];
        };
        if (ok && own && ((lds_acquire_u(&S.own_pm) >> cf) & 1u) && covered(S.own_j[cf]))
            ok = false;  // wave 0's own annotation in flight covers it
        // the slots holding a seed from `decided` on, not zombies (the others are free)
        const uint64_t live = __ballot(sl && r_seed >= decided && r_st != 0 && r_st != 4);
        // skip the seeds they hold
        for (uint64_t hq = live & __ballot(sl && r_seed >= base && r_seed < base + 64); hq; hq &= hq - 1)
            if (idx == __builtin_amdgcn_readlane(r_seed, __ffsll((unsigned long long)hq) - 1)) ok = false;
        // seeds near one still being grown, or covered by the joints its grow has set so far
        const uint32_t r_pm = sl ? lds_acquire_u(&S.cache_pm[lane]) : 0u;
        for (uint64_t fq = live & fly; fq; fq &= fq - 1) {
            const int q = __ffsll((unsigned long long)fq) - 1;
            ok = ok && (__builtin_amdgcn_readlane(r_seed, q) > idx ||
                         spec_far(far_k, c.x, c.y, c.s, rl_f(r_x, q), rl_f(r_y, q), rl_f(r_s, q)));
            const uint32_t pm = (uint32_t)__builtin_amdgcn_readlane((int)r_pm, q);
            if (ok && ((pm >> cf) & 1u) && __builtin_amdgcn_readlane(r_seed, q) < idx &&
                covered(S.cache_j[q][cf]))
                ok = false;
        }
        // seeds a grown annotation's occupancy boxes will cover once committed
        const int bf = ok ? cf : 0;
        uint64_t gq = live & ~fly & __ballot(sl && r_st == 2);
        while (gq) {  // four slots' boxes per LDS round trip
            int qs[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                qs[u] = gq ? __ffsll((unsigned long long)gq) - 1 : -1;
                gq &= gq ? gq - 1 : 0ull;
            }
            uint2 bx[4];
#pragma unroll
            for (int u = 0; u < 4; u++) bx[u] = qs[u] >= 0 ? S.cache_box[qs[u]][bf] : make_uint2(0u, 0u);
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (qs[u] >= 0 && __builtin_amdgcn_readlane(r_seed, qs[u]) < idx &&
                    in_plan_box(bx[u], cxi, cyi))
                    ok = false;
        }
        uint64_t m = __ballot(ok);
        while (m && idle) {
            const int l = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const float cx = rl_f(c.x, l), cy = rl_f(c.y, l), csc = rl_f(c.s, l);
            // far from this plan's earlier picks and every other seed in flight (a lane per slot)
            if (__ballot(((fly >> lane) & 1ull) && r_seed < base + l &&
                         !spec_far(far_k, cx, cy, csc, r_x, r_y, r_s)))
                continue;
            // a free slot: never grown into, or grown for a seed already decided
            const uint64_t freeq = __ballot(sl && (r_st == 0 || (r_st == 2 && r_seed < decided)));
            if (!freeq) return idle;  // no slot: nobody else can be planned either
            const int q = __ffsll((unsigned long long)freeq) - 1;
            const int w = __ffsll((unsigned long long)idle) - 1;
            idle &= idle - 1;
            fly |= 1ull << q;
            if (lane == q) {
                r_st = 1;
                r_seed = base + l;
                r_x = cx;
                r_y = cy;
                r_s = csc;
            }
            if (lane == 0) {
                S.cache_x[q] = cx;
                S.cache_y[q] = cy;
                S.cache_s[q] = csc;
                S.cache_pm[q] = 0u;  // no joints of the new grow yet
                lds_release(&S.cache_state[q], 1);
                lds_release(&S.cache_seed[q], base + l);
                S.task_slot[w] = q;
                lds_release(&S.task[w], base + l);
            }
            wave_sync();
        }
    }
    return idle;
}

template <int NS>
__device__ __forceinline__ void plan_lock(SeedLoopSharedT<NS> &S) {
    if ((threadIdx.x & 63) == 0) {
        int expect = 0;
        while (!__hip_atomic_compare_exchange_strong(&S.plan_lock, &expect, 1, __ATOMIC_ACQUIRE,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            expect = 0;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    wave_sync();
}

template <int NS>
__device__ __forceinline__ void plan_unlock(SeedLoopSharedT<NS> &S) {
    wave_sync();
    if ((threadIdx.x & 63) == 0) lds_release(&S.plan_lock, 0);
}

// ---- pieces both seed-loop kernels share (force-inlined: each takes GrowArgs by
// reference, which a real call would copy to scratch) ----

// The image's small set-A column sets (<= kFlatCols columns, in (CAF, direction) order
// while they fit kColLds floats) into LDS, column-major, kColPad floats per column: their
// counts into s_ncol, LDS offsets into s_cofs (-1: read from global memory).  Every wave of
// the workgroup takes part; no barrier after the copy (the caller's init barrier follows).
__device__ __forceinline__ ColStage stage_small_sets(const GrowArgs &g, int img, int *s_ncol,
                                                     int *s_cofs, float *s_cols, int cap) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int q = threadIdx.x; q < 2 * g.C; q += blockDim.x) s_ncol[q] = col_offs(g, 0, img, q >> 1, q & 1)[g.nb];
    __syncthreads();
    if (threadIdx.x == 0) {  // LDS placement of the small sets, in order while they fit
        int o = 0;
        for (int q = 0; q < 2 * g.C; q++) {
            const int sz = kColPad * s_ncol[q];
            const bool fit = s_ncol[q] <= kFlatCols && o + sz <= cap;
            s_cofs[q] = fit ? o : -1;
            o += fit ? sz : 0;
        }
    }
    __syncthreads();
    for (int q = wave; q < 2 * g.C; q += kSeedWaves) {  // one set per wave
        const int n = s_ncol[q];
        if (s_cofs[q] < 0 || n == 0) continue;
        const float *cf = col_set(g, 0, img, q >> 1, q & 1);
        float *dst = s_cols + s_cofs[q];
        for (int k = lane; k < n; k += 64) {
            float c[kColRows];
#pragma unroll
            for (int r = 0; r < kColRows; r++) c[r] = cf[r * g.col_cap + k];
            float4 *o = reinterpret_cast<float4 *>(dst + k * kColPad);
            o[0] = make_float4(c[0], c[1], c[2], c[3]);
            o[1] = make_float4(c[4], c[5], c[6], 0.0f);
        }
    }
    return ColStage{s_ncol, s_cofs, s_cols};
}

// The next free seed from index s on (cifcaf.py:100-104), 64 occupancy tests per step (the
// per-seed LDS counters `socc`, or the global grid); -1 when none is left.  s advances past
// the all-occupied steps.  Wave 0.
__device__ __forceinline__ int next_free_seed(int &s, int n_seeds, const SeedOcc *socc,
                                              const pp_seed *seeds, const OccGrid &occ,
                                              float red) {
    const int lane = threadIdx.x & 63;
    while (s < n_seeds) {
        const int idx = s + lane;
        bool is_free = false;
        if (idx < n_seeds) {
            if (socc) {
                is_free = !seed_occupied(*socc, idx);
            } else {
                const pp_seed c = seeds[idx];
                is_free = !occ_get(occ, c.field, c.x, c.y, red);
            }
        }
        const uint64_t m = __ballot(is_free);
        if (m) return s + __ffsll((unsigned long long)m) - 1;
        s += 64;
    }
    return -1;
}

// Initial annotations (cifcaf.py:95-98): each is grown with set A and reverse matching from
// all its set joints (its decoding / frontier orders are appended to), then committed
// (appended and marked occupied, `commit(record)`), in order, before any seed is looked
// at.  Wave 0.
template <bool CS, typename Commit>
__device__ __forceinline__ void grow_initial(const GrowArgs &g, SeedLDS &L, int img,
                                             const ColStage &cstage, const int &n_anns,
                                             Commit commit) {
    const int lane = threadIdx.x & 63;
    const int n_init = g.init ? min(g.init_counts[img], g.init_cap) : 0;
    for (int i = 0; i < n_init; i++) {
        if (n_anns >= g.ann_cap) {
            if (lane == 0) L.status |= PP_ST_ANN_OVERFLOW;
            break;
        }
        copy_ann(&L.a, &g.init[(int64_t)img * g.init_cap + i]);
        if (lane == 0) {
            L.a.image = img;
            L.a.n_keypoints = g.K;
        }
        wave_sync();
        grow<true, CS>(g, L, img, 0, true, cstage);
        commit(&L.a);
    }
}

// A helper wave's finished grow into this CU's cache slot q: the record (global memory),
// its joints (LDS), then the slot's state 2 (grown).  The record's global stores complete
// before the flag (the workgroup-scope release alone does not wait for them).
template <int NS>
__device__ __forceinline__ void publish_cached(SeedLoopSharedT<NS> &S, pp_ann *cache, int q,
                                               const SeedLDS &L) {
    const int lane = threadIdx.x & 63;
    copy_ann(&cache[q], &L.a);
    if (lane < kKP)
        S.cache_j[q][lane] = make_float4(L.a.data[lane][0], L.a.data[lane][1],
                                         L.a.data[lane][2], L.a.joint_scales[lane]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    if (lane == 0) lds_release(&S.cache_state[q], 2);
    wave_sync();
}

// The end of a seed loop (wave 0, after the barrier that drains the helpers): the image's
// occupancy marks cleared (the grid stays zero between launches), then its annotation
// count, the joints force-complete must fill, and the waves' status bits.
__device__ __forceinline__ void seed_loop_outputs(const GrowArgs &g, const SeedLDS *Ls, int img,
                                                  int n_anns, uint32_t unset_mask) {
    if ((threadIdx.x & 63) == 0) {
        int st = 0;
        for (int w = 0; w < kSeedWaves; w++) st |= Ls[w].status;
        g.n_work[img] = n_anns;
        g.need_complete[img] = g.cfg.force_complete ? (int)unset_mask : 0;
        g.status[img] = st;
    }
}

// <= 168 VGPRs (3 waves per SIMD; a few spills) and the column stage in dynamic LDS: the
// image's workgroup leaves room on its CU for the next batch's CifHr / seeds / CafScored
// workgroups (DecodePipeline).  Planted 1.031 -> 1.013 ms, uniform 21.7 -> 20.4 ms per
// overlapped step; 4 waves per SIMD (128 VGPRs, 532 spills): 1.37 ms.
// Grid: n_img image workgroups, then n_ext * n_img external helper workgroups (helper
// workgroup x of image i is block n_img * (1 + x) + i, on image i's XCD when n_img % 8 == 0).
template <bool CS>
__global__ __launch_bounds__(64 * kSeedWaves) __attribute__((amdgpu_waves_per_eu(3)))
void seed_loop_kernel(GrowArgs g) {
    __shared__ SeedLDS Ls[kSeedWaves];
    __shared__ SeedLoopShared S;
    __shared__ int s_ncol[2 * PP_MAX_EDGES];  // set-A column counts per (CAF, direction)
    __shared__ int s_cofs[2 * PP_MAX_EDGES];  // their LDS offsets in s_cols (-1: global)
    __shared__ SeedOcc s_occ;  // per-seed occupancy (images of at most kOccSeeds seeds)
    extern __shared__ float s_cols[];  // kColLds floats (dynamic: the launch sizes it)
    const int img = blockIdx.x;
    const int K = g.K;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    SeedLDS &L = Ls[wave];
    const ColStage cstage = stage_small_sets(g, img, s_ncol, s_cofs, s_cols, kColLds);
    if (lane == 0) {
        L.status = 0;
        L.log_n = 0;
#ifdef PP_STAMPS
        for (int q = 0; q < 10; q++) L.fst[q] = 0;
#endif
    }
    if (threadIdx.x < kSpecCache) {
        S.cache_seed[threadIdx.x] = -1;
        S.cache_state[threadIdx.x] = 0;
        S.cache_pm[threadIdx.x] = 0u;
    }
    if (threadIdx.x < kSeedWaves) S.task[threadIdx.x] = -1;
    if (threadIdx.x == 0) {
        S.done = 0;
        S.plan_lock = 0;
        S.decided = 0;
        S.own_on = 0;
        S.plan_req = 0;
        S.own_pm = 0u;
    }
    __syncthreads();

    STAMP_DECL
    uint8_t *occ_base = g.occ + (int64_t)img * g.occ_cap;
    OccLog *log = g.log + (int64_t)img * g.log_cap;
    pp_ann *work = g.work + (int64_t)img * g.ann_cap;
    pp_ann *cache = g.spec + (int64_t)img * kSpecCache;
    const float red = (float)g.cfg.occupancy_reduction;
    const float msr = occ_msr(g);
    const OccGrid occ = occ_grid(occ_base, K, (int)((double)g.hh / g.cfg.occupancy_reduction),
                                 (int)((double)g.ww / g.cfg.occupancy_reduction));
    const int n_seeds = min(g.seed_counts[img], g.seed_cap);
    const pp_seed *seeds = g.seeds + (int64_t)img * g.seed_cap;
    // the occupancy at the seeds in LDS (seed_occ_*), or the global grid for more seeds
    const bool socc_on = n_seeds <= kOccSeeds;
    if (socc_on) seed_occ_init(s_occ, seeds, n_seeds, K, occ, red);
    const SeedOcc *socc = socc_on ? &s_occ : nullptr;
    // the plans' speculation distance: kSpecFar, but none on images with more seeds than
    // kOccSeeds (dense fields, where nearly every seed lies near one in flight): uniform
    // cfg3 15.6k-16.1k -> 16.1k-16.2k images/s, planted unchanged (r06z_ab_dense_far.txt)
    const float far_img = socc_on ? g.spec_far : 0.0f;

    // committer state (wave 0)
    int n_anns = 0, s = 0;
    uint32_t unset_mask = 0;
#ifdef PP_STAMPS
    int n_rounds = 0, n_hits = 0;
#endif

    // append one finished annotation and mark_occupied (cifcaf.py:87-93): wave 0 only
    // (lane j < K holds joint j of the record: x, y, v, scale, from LDS)
    // (the record's loads are issued first and stored after the marks: the marks hide
    // their latency)
    auto commit = [&](const pp_ann *src, float jx, float jy, float jv, float js) {
#ifdef PP_STAMPS
        uint64_t ct0 = __builtin_amdgcn_s_memtime();
#endif
        const AnnRegs rec = ann_load(src);
        const uint32_t set = (uint32_t)__ballot(lane < K && jv > 0.0f);
        unset_mask |= ~set & (K >= 32 ? 0xFFFFFFFFu : ((1u << K) - 1u));
        if (socc_on)
            seed_occ_mark(g, s_occ, occ, jx, jy, js, jv != 0.0f, K);
        else
            occ_mark(g, L, log, occ, jx, jy, js, jv != 0.0f, K);
#ifdef PP_STAMPS
        ESTAMP(L, 5, ct0);  // (wave 0) the occupancy marks
#endif
        ann_store(&work[n_anns], rec);
        n_anns++;
#ifdef PP_STAMPS
        ESTAMP(L, 4, ct0);  // (wave 0) the record's stores (after the marks)
#endif
    };

    if (wave > 0) {  // helper: grow the seeds wave 0 hands over until it is done
        // `decided` when this helper's last plan found it nothing to grow (-1: none): once
        // wave 0 has moved on (commits free slots, passes seeds), an idle helper plans itself
        // again instead of waiting for wave 0's next miss (which a wave 0 that only takes
        // cached annotations never has)
        int idle_dec = -1;
        for (;;) {
            int my;
            for (;;) {
                my = lds_acquire(&S.task[wave]);
                if (my >= 0 || lds_acquire(&S.done)) break;
                if (idle_dec >= 0 && lds_acquire(&S.decided) != idle_dec) {
#ifdef PP_STAMPS
                    const uint64_t hp2 = __builtin_amdgcn_s_memtime();
#endif
                    plan_lock(S);
                    uint64_t left = 1ull << wave;
                    const int dec = lds_acquire(&S.decided);
                    if (!lds_acquire(&S.done) && lds_acquire(&S.task[wave]) < 0)
                        left = spec_plan(S, seeds, n_seeds, dec, kSelfScan, occ, red, msr, far_img,
                                         left, socc);
                    plan_unlock(S);
                    idle_dec = left ? dec : -1;
#ifdef PP_STAMPS
                    if (lane == 0) L.fst[8] += __builtin_amdgcn_s_memtime() - hp2;
#endif
                    continue;
                }
                if (lds_acquire(&S.plan_req)) {
                    // wave 0 is growing a seed of its own: plan every idle helper (this one
                    // included) around it
#ifdef PP_STAMPS
                    const uint64_t hp0 = __builtin_amdgcn_s_memtime();
#endif
                    plan_lock(S);
                    if (lds_acquire(&S.plan_req) && !lds_acquire(&S.done)) {
                        if (lane == 0) lds_release(&S.plan_req, 0);
                        const int tk = lane > 0 && lane < kSeedWaves ? lds_acquire(&S.task[lane]) : 0;
                        const uint64_t idle = __ballot(lane > 0 && lane < kSeedWaves && tk < 0);
                        const int dec = lds_acquire(&S.decided);
                        if (idle)
                            spec_plan(S, seeds, n_seeds, dec, kSpecScan, occ, red, msr, far_img,
                                      idle, socc);
                    }
                    plan_unlock(S);
                    if (lds_acquire(&S.task[wave]) < 0) idle_dec = lds_acquire(&S.decided);
#ifdef PP_STAMPS
                    if (lane == 0) L.fst[8] += __builtin_amdgcn_s_memtime() - hp0;
#endif
                    continue;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (my < 0) break;
            const int q = S.task_slot[wave];
#ifdef PP_STAMPS
            const uint64_t hg0 = __builtin_amdgcn_s_memtime();
#endif
            ann_from_seed(L, seeds[my], K, img);
            grow<true, CS>(g, L, img, 0, true, cstage, &S.done, S.cache_j[q], &S.cache_pm[q]);
#ifdef PP_STAMPS
            if (lane == 0) {  // helper grows and their cycles (phase-1 slots 8 and 5)
                L.fst[4] += 1;
                L.fst[5] += __builtin_amdgcn_s_memtime() - hg0;
            }
#endif
            if (lds_acquire(&S.done)) break;  // nobody reads the cache any more
            if (lane < kKP)
                S.cache_box[q][lane] = plan_box(
                    red, msr, occ, lane,
                    make_float4(L.a.data[lane][0], L.a.data[lane][1], L.a.data[lane][2], L.a.joint_scales[lane]));
            publish_cached(S, cache, q, L);  // (its release orders the boxes too)
#ifdef PP_STAMPS
            const uint64_t hp1 = __builtin_amdgcn_s_memtime();
#endif
            // plan this wave's next grow itself, with its own annotation now in the cache (its
            // occupancy boxes rule out the other seeds of the same person); wave 0 plans only
            // when it has to grow a seed itself
            plan_lock(S);
            uint64_t left = 1ull << wave;
            if (!lds_acquire(&S.done)) {
                const int dec = lds_acquire(&S.decided);
                left = spec_plan(S, seeds, n_seeds, dec, kSelfScan, occ, red, msr, far_img, left,
                                 socc);
            }
            if (left && lane == 0) lds_release(&S.task[wave], -1);
            plan_unlock(S);
            idle_dec = left ? lds_acquire(&S.decided) : -1;
#ifdef PP_STAMPS
            if (lane == 0) {
                L.fst[8] += __builtin_amdgcn_s_memtime() - hp1;
                L.fst[9] += 1;
            }
#endif
        }
    } else {
        __builtin_amdgcn_s_setprio(3);  // the committer is the critical path: issue first
        grow_initial<CS>(g, L, img, cstage, n_anns, [&](const pp_ann *a) {
            commit(a, lane < K ? a->data[lane][0] : 0.0f, lane < K ? a->data[lane][1] : 0.0f,
                   lane < K ? a->data[lane][2] : 0.0f, lane < K ? a->joint_scales[lane] : 0.0f);
        });
        for (;;) {
            const int t = next_free_seed(s, n_seeds, socc_on ? &s_occ : nullptr, seeds, occ, red);
            STAMP(0);
            if (t < 0 || n_anns >= g.ann_cap) {
                if (lane == 0 && t >= 0) L.status |= PP_ST_ANN_OVERFLOW;
                break;
            }
            const int cs = lane < kSpecCache ? S.cache_seed[lane] : -1;
            const uint64_t hit = __ballot(lane < kSpecCache && cs == t);
            if (hit) {  // a helper grew it, or is growing it
                const int slot = __ffsll((unsigned long long)hit) - 1;
#ifdef PP_STAMPS
                const uint64_t hw0 = __builtin_amdgcn_s_memtime();
#endif
                while (lds_acquire(&S.cache_state[slot]) != 2) __builtin_amdgcn_s_sleep(1);
#ifdef PP_STAMPS
                if (lane == 0) L.fst[8] += __builtin_amdgcn_s_memtime() - hw0;
#endif
                const float4 jq = lane < kKP ? S.cache_j[slot][lane] : make_float4(0.f, 0.f, 0.f, 0.f);
                commit(&cache[slot], jq.x, jq.y, jq.z, jq.w);
                s = t + 1;
                if (lane == 0) lds_release(&S.decided, s);  // the slot is free again
#ifdef PP_STAMPS
                n_hits++;
#endif
                STAMP(4);
                continue;
            }
            // hand far-away free seeds to the idle helpers (an idle helper plans them), then
            // grow t here
            const pp_seed st = seeds[t];
            if (lane == 0) {
                S.own_pm = 0u;  // (grow publishes the seed joint first)
                S.own_x = st.x;
                S.own_y = st.y;
                S.own_s = st.s;
                lds_release(&S.own_on, 1);
                lds_release(&S.decided, t);
                lds_release(&S.plan_req, 1);
            }
            wave_sync();
#ifdef PP_STAMPS
            n_rounds++;
#endif
            STAMP(1);
            ann_from_seed(L, st, K, img);
            grow<true, CS>(g, L, img, 0, true, cstage, nullptr, S.own_j, &S.own_pm);
            STAMP(2);
            commit(&L.a, lane < K ? L.a.data[lane][0] : 0.0f, lane < K ? L.a.data[lane][1] : 0.0f,
                   lane < K ? L.a.data[lane][2] : 0.0f, lane < K ? L.a.joint_scales[lane] : 0.0f);
            s = t + 1;
            if (lane == 0) {
                lds_release(&S.own_on, 0);
                lds_release(&S.decided, s);
            }
            STAMP(3);
        }
        if (lane == 0) lds_release(&S.done, 1);
    }
    __syncthreads();  // helpers drained: no wave is still growing into the cache
    if (wave == 0) {
        occ_clear(g, L, log, occ);
        STAMP(5);
#ifdef PP_STAMPS
        st_acc[6] = n_rounds;
        st_acc[7] = n_hits;
        {  // helpers' grows (count into slot 8, cycles into slot 5 in place of occ_clear)
            uint64_t hn = 0, hc = 0, hp = 0, hpn = 0;
            for (int w = 1; w < kSeedWaves; w++) {
                hn += Ls[w].fst[4];
                hc += Ls[w].fst[5];
                hp += Ls[w].fst[8];
                hpn += Ls[w].fst[9];
            }
            L.fst[3] = hn;
            st_acc[5] = hc;
            st_acc[14] = hp;  // the helpers' plans (self plans and wave 0's requests)
            st_acc[15] = L.fst[8] | (hpn << 40);  // wave 0's hit waits; self plans << 40
            L.fst[6] = L.fst[4];  // (diagnostic: wave 0's copy / mark cycles in slots 12 / 13)
            L.fst[7] = L.fst[5];
        }
#endif
        STAMP_FLUSH(1);
        seed_loop_outputs(g, Ls, img, n_anns, unset_mask);
    }
}


// The same loop with external helpers (n_ext > 0).  A separate kernel: the big-batch one
// above carries none of the hand-off state, whose registers cost it 4% per planted cfg3
// step when merged into it (spills inside the grow).
template <bool CS>
__global__ __launch_bounds__(64 * kSeedWaves) __attribute__((amdgpu_waves_per_eu(3)))
void seed_loop_ext_kernel(GrowArgs g) {
    constexpr int NS = kCacheSlots;
    __shared__ SeedLDS Ls[kSeedWaves];
    __shared__ SeedLoopSharedX S;
    __shared__ int s_ncol[2 * PP_MAX_EDGES];  // set-A column counts per (CAF, direction)
    __shared__ int s_cofs[2 * PP_MAX_EDGES];  // their LDS offsets in s_cols (-1: global)
    __shared__ SeedOcc s_occ;  // per-seed occupancy (the image's own workgroup)
    // kColLdsExt floats (dynamic: the launch sizes it), then the external slots' joints
    // (cache_joints)
    extern __shared__ float s_cols[];
    const int n_img = (int)gridDim.x / (1 + g.n_ext);
    const bool external = (int)blockIdx.x >= n_img;
    const int img = (int)blockIdx.x % n_img;
    const int K = g.K;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    SeedLDS &L = Ls[wave];
    const ColStage cstage = stage_small_sets(g, img, s_ncol, s_cofs, s_cols, kColLdsExt);
    if (lane == 0) {
        L.status = 0;
        L.log_n = 0;
#ifdef PP_STAMPS
        for (int q = 0; q < 10; q++) L.fst[q] = 0;
#endif
    }
    if (threadIdx.x < NS) {
        S.cache_seed[threadIdx.x] = -1;
        S.cache_state[threadIdx.x] = 0;
    }
    if (threadIdx.x < kSeedWaves) S.task[threadIdx.x] = -1;
    if (threadIdx.x == 0) {
        S.done = 0;
        S.ext_ticks = 0u;
        S.plan_lock = 0;
        S.decided = 0;
        S.own_on = 0;
    }
    __syncthreads();

    const int n_seeds = min(g.seed_counts[img], g.seed_cap);
    bool heavy = false;  // wave 0's regime (see kExtHeavyAnns)
    const pp_seed *seeds = g.seeds + (int64_t)img * g.seed_cap;
    SeedExt *X = g.xext + img;
    pp_ann *xrec = g.xrec + (int64_t)img * kExtCache;

    STAMP_DECL
    uint8_t *occ_base = g.occ + (int64_t)img * g.occ_cap;
    OccLog *log = g.log + (int64_t)img * g.log_cap;
    pp_ann *work = g.work + (int64_t)img * g.ann_cap;
    pp_ann *cache = g.spec + (int64_t)img * kSpecCache;
    const float red = (float)g.cfg.occupancy_reduction;
    const float msr = occ_msr(g);
    const OccGrid occ = occ_grid(occ_base, K, (int)((double)g.hh / g.cfg.occupancy_reduction),
                                 (int)((double)g.ww / g.cfg.occupancy_reduction));
    const int n_help = kSeedWaves + (X ? g.n_ext * kSeedWaves : 0);  // helper lanes 1 .. n_help-1
    // the occupancy at the seeds in LDS (seed_occ_*), or the global grid for more seeds
    const bool socc_on = !external && n_seeds <= kOccSeeds;  // block-uniform
    if (socc_on) seed_occ_init(s_occ, seeds, n_seeds, K, occ, red);

    // committer state (wave 0)
    int n_anns = 0, s = 0;
    uint32_t unset_mask = 0;
#ifdef PP_STAMPS
    int n_rounds = 0, n_hits = 0;
#endif

    // append one finished annotation and mark_occupied (cifcaf.py:87-93): wave 0 only
    // (lane j < K holds joint j of the record: x, y, v, scale, from LDS)
    auto commit = [&](const pp_ann *src, bool other_cu, float jx, float jy, float jv, float js) {
        if (other_cu)
            copy_ann_agent(&work[n_anns], src);
        else
            copy_ann(&work[n_anns], src);
        n_anns++;
        const uint32_t set = (uint32_t)__ballot(lane < K && jv > 0.0f);
        unset_mask |= ~set & (K >= 32 ? 0xFFFFFFFFu : ((1u << K) - 1u));
        if (socc_on)
            seed_occ_mark(g, s_occ, occ, jx, jy, js, jv != 0.0f, K);
        else
            occ_mark(g, L, log, occ, jx, jy, js, jv != 0.0f, K);
    };

    if (external || wave > 0) {
        // helper: grow the seeds wave 0 hands over until it is done.  This CU's helpers
        // take them from LDS words and publish into LDS-flagged slots; external ones poll
        // their global word and publish write-through (see SeedExt)
        unsigned long long *tw =
            external ? &X->task[((int)blockIdx.x / n_img - 1) * kSeedWaves + wave] : nullptr;
        if (external && lane == 0) st_agent(tw, 1ull);
        uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            int my = -1, q = 0;
            if (!external) {
                for (;;) {
                    my = lds_acquire(&S.task[wave]);
                    if (my >= 0 || lds_acquire(&S.done)) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                if (my < 0) break;
                q = S.task_slot[wave];
            } else {
                const unsigned long long v = ld_agent(tw);
                if ((v & 0xFFull) != 2ull) {
                    const bool quit = ld_agent(&X->fin) != 0u ||
                                      __builtin_amdgcn_s_memrealtime() - t0 >
                                          (ld_agent(&X->heavy) ? kExtIdleHeavy : kExtIdleLight);
                    if (quit && cas_agent_wave(tw, 1ull, 3ull)) break;
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
                q = (int)((v >> 8) & 0xFFFFull);
                my = (int)(v >> 32);
            }
            ann_from_seed(L, seeds[my], K, img);
            grow<true, CS>(g, L, img, 0, true, cstage, external ? nullptr : &S.done);
            if (!external && lds_acquire(&S.done)) break;  // nobody reads the cache any more
            if (external) {
                publish_ann(&xrec[q], &L.a);
                if (lane == 0) {
                    st_agent(&X->tag[q], (unsigned int)my + 1u);
                    st_agent(tw, 1ull);
                }
                wave_sync();
                t0 = __builtin_amdgcn_s_memrealtime();
                continue;
            }
            if (lane < kKP)
                cache_boxes(s_cols, q)[lane] = plan_box(
                    red, msr, occ, lane,
                    make_float4(L.a.data[lane][0], L.a.data[lane][1], L.a.data[lane][2], L.a.joint_scales[lane]));
            publish_cached(S, cache, q, L);  // (its release orders the boxes too)
            // idle again: wave 0 plans this CU's helpers (no self-planning here, above)
            plan_lock(S);
            if (lane == 0) lds_release(&S.task[wave], -1);
            plan_unlock(S);
        }
        if (external) {  // every wave of an external workgroup is a helper
            __syncthreads();
            ext_exit(X, g.n_ext);
            return;
        }
    } else {
        __builtin_amdgcn_s_setprio(3);  // the committer is the critical path: issue first
        grow_initial<CS>(g, L, img, cstage, n_anns, [&](const pp_ann *a) {
            commit(a, false, lane < K ? a->data[lane][0] : 0.0f,
                   lane < K ? a->data[lane][1] : 0.0f, lane < K ? a->data[lane][2] : 0.0f,
                   lane < K ? a->joint_scales[lane] : 0.0f);
        });
        // Hand far-away free seeds after t to the idle helpers (this CU's and the external
        // ones), with S.plan_lock held; `own`: wave 0 grows seed st itself next (the picks
        // keep kSpecFar from it too)
        auto plan_round = [&](const int t, const bool own, const pp_seed &st) {
#ifdef PP_STAMPS
            const uint64_t xr0 = __builtin_amdgcn_s_memtime();
#endif
            ext_refresh(S, s_cols, X, xrec, -1, red, msr, occ);
#ifdef PP_STAMPS
            st_acc[14] += __builtin_amdgcn_s_memtime() - xr0;  // plan: the external slots' refresh
#endif
            int tk = 0;
            if (lane > 0 && lane < kSeedWaves)
                tk = lds_acquire(&S.task[lane]) < 0 ? 1 : 0;
            else if (lane >= kSeedWaves && lane < n_help)
                tk = ld_agent(&X->task[lane - kSeedWaves]) == 1ull ? 1 : 0;
            uint64_t idle = __ballot(tk != 0);
            // The slots, one lane each: a snapshot (only wave 0 claims slots; a helper turning
            // 1 into 2 meanwhile at most keeps this plan from reusing or testing that slot),
            // kept current for this plan's own picks.
            const bool sl = lane < NS;
            int r_st = sl ? lds_acquire(&S.cache_state[lane]) : 0;
            int r_seed = sl ? S.cache_seed[lane] : -1;
            float r_x = sl ? S.cache_x[lane] : 0.0f, r_y = sl ? S.cache_y[lane] : 0.0f,
                  r_s = sl ? S.cache_s[lane] : 0.0f;
            // the seeds in flight: later picks keep kSpecFar from them
            uint64_t fly = __ballot(sl && r_st == 1);
            const int scan_end = min(n_seeds, t + 1 + kExtScan);
#ifdef PP_STAMPS
            uint64_t pf0 = __builtin_amdgcn_s_memtime();
#endif
            for (int base = t + 1; base < scan_end && idle; base += 64) {
                const int idx = base + lane;
                bool ok = idx < scan_end;
                pp_seed c{};
                if (ok) {
                    c = seeds[idx];
                    ok = (!own || spec_far(kExtSpecFar, c.x, c.y, c.s, st.x, st.y, st.s)) &&
                         !(socc_on ? seed_occupied(s_occ, idx) : occ_get(occ, c.field, c.x, c.y, red));
                }
                // the slots holding seeds after t (the others are free or passed): skip the
                // seeds they hold, seeds near one still being grown, and seeds that a grown
                // annotation's occupancy boxes will cover once committed
                const uint64_t ahead = __ballot(sl && r_seed > t);
                const uint64_t held = __ballot(sl && r_seed >= base && r_seed < base + 64) & ahead;
                for (uint64_t hq = held; hq; hq &= hq - 1)
                    if (idx == __builtin_amdgcn_readlane(r_seed, __ffsll((unsigned long long)hq) - 1)) ok = false;
                for (uint64_t fq = ahead & fly; fq; fq &= fq - 1) {
                    const int q = __ffsll((unsigned long long)fq) - 1;
                    ok = ok && (__builtin_amdgcn_readlane(r_seed, q) > idx ||
                                 spec_far(kExtSpecFar, c.x, c.y, c.s, rl_f(r_x, q), rl_f(r_y, q), rl_f(r_s, q)));
                }
                const int cxi = (int)clip_ref(c.x / red, 0.0f, (float)(occ.w - 1));
                const int cyi = (int)clip_ref(c.y / red, 0.0f, (float)(occ.h - 1));
                const int cf = ok ? c.field : 0;
                uint64_t gq = ahead & __ballot(sl && r_st == 2);
                while (gq) {  // four slots' boxes per LDS round trip
                    int qs[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        qs[u] = gq ? __ffsll((unsigned long long)gq) - 1 : -1;
                        gq &= gq ? gq - 1 : 0ull;
                    }
                    uint2 b[4];
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        b[u] = qs[u] >= 0 ? cache_boxes(s_cols, qs[u])[cf] : make_uint2(0u, 0u);
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (qs[u] >= 0 && __builtin_amdgcn_readlane(r_seed, qs[u]) < idx &&
                            in_plan_box(b[u], cxi, cyi))
                            ok = false;
                }
                uint64_t m = __ballot(ok);
#ifdef PP_STAMPS
                ESTAMP(L, 6, pf0);  // plan: the seed filter
#endif
                while (m && idle) {
                    const int l = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    const float cx = rl_f(c.x, l), cy = rl_f(c.y, l), csc = rl_f(c.s, l);
                    // far from every seed in flight, this plan's earlier picks included (a
                    // lane per slot)
                    if (__ballot(((fly >> lane) & 1ull) && r_seed < base + l &&
                                 !spec_far(kExtSpecFar, cx, cy, csc, r_x, r_y, r_s)))
                        continue;
                    // a free slot of the helper's kind (this CU's: 0 .. kSpecCache-1; the
                    // external ones after): never grown into, or grown for a seed passed
                    const uint64_t freeq = __ballot(sl && (r_st == 0 || (r_st == 2 && r_seed < t)));
                    const uint64_t free_l = freeq & ((1ull << kSpecCache) - 1ull);
                    const uint64_t free_x = freeq & ~((1ull << kSpecCache) - 1ull);
                    const uint64_t idle_l = idle & ((1ull << kSeedWaves) - 1ull);
                    const uint64_t idle_x = idle & ~((1ull << kSeedWaves) - 1ull);
                    const bool use_l = idle_l && free_l;
                    if (!use_l && !(idle_x && free_x)) {
                        m = 0;
                        idle = 0;
                        break;
                    }
                    const int q = __ffsll((unsigned long long)(use_l ? free_l : free_x)) - 1;
                    const int w = __ffsll((unsigned long long)(use_l ? idle_l : idle_x)) - 1;
                    idle &= ~(1ull << w);
                    const int sd = base + l;
                    if (!use_l) {  // the helper may have just left: then skip it
                        const unsigned long long job = 2ull | ((unsigned long long)(q - kSpecCache) << 8) |
                                                       ((unsigned long long)sd << 32);
#ifdef PP_STAMPS
                        const uint64_t xc0 = __builtin_amdgcn_s_memtime();
#endif
                        const bool got = cas_agent_wave(&X->task[w - kSeedWaves], 1ull, job);
#ifdef PP_STAMPS
                        st_acc[15] += __builtin_amdgcn_s_memtime() - xc0;  // plan: hand-off CAS
#endif
                        if (!got) {
                            m |= 1ull << l;  // the seed is still unassigned
                            continue;
                        }
                    }
                    fly |= 1ull << q;
                    if (lane == q) {
                        r_st = 1;
                        r_seed = sd;
                        r_x = cx;
                        r_y = cy;
                        r_s = csc;
                    }
                    if (lane == 0) {
                        S.cache_x[q] = cx;
                        S.cache_y[q] = cy;
                        S.cache_s[q] = csc;
                        lds_release(&S.cache_state[q], 1);  // state first (spec_plan)
                        lds_release(&S.cache_seed[q], sd);
                        S.cache_t[q] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                        if (use_l) {
                            S.task_slot[w] = q;
                            lds_release(&S.task[w], sd);
                        }
                    }
                    wave_sync();
                }
#ifdef PP_STAMPS
                ESTAMP(L, 6, pf0);  // plan: the picks
#endif
            }
        };
        for (;;) {
            const int t = next_free_seed(s, n_seeds, socc_on ? &s_occ : nullptr, seeds, occ, red);
            STAMP(0);
            if (t < 0 || n_anns >= g.ann_cap) {
                if (lane == 0 && t >= 0) L.status |= PP_ST_ANN_OVERFLOW;
                break;
            }
            if (!heavy && n_anns >= kExtHeavyAnns) {  // helpers stay (kExtIdleHeavy)
                heavy = true;
                if (lane == 0) st_agent(&X->heavy, 1u);
            }
            const int cs = lane < NS ? S.cache_seed[lane] : -1;
            const int cst0 = lane < NS ? S.cache_state[lane] : 0;
            const uint64_t hit = __ballot(lane < NS && cs == t && cst0 != 4);
            bool taken = false;
            int hslot = -1;
            if (hit) {  // a helper grew it, or is growing it
                const int slot = __ffsll((unsigned long long)hit) - 1;
#ifdef PP_STAMPS
                uint64_t hw0 = __builtin_amdgcn_s_memtime();
#endif
                if (slot < kSpecCache) {
                    while (lds_acquire(&S.cache_state[slot]) != 2) __builtin_amdgcn_s_sleep(1);
                } else {
                    // another CU's: wait for its tag (bounded; a helper always finishes), or
                    // on a light image grow the seed here and leave the slot a zombie
                    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
                    const uint32_t el = (uint32_t)w0 - S.cache_t[slot];
                    const uint64_t limit =
                        (S.ext_ticks == 0u || el >= S.ext_ticks / 2u) ? kExtWaitMax : 0ull;
                    for (;;) {
                        ext_refresh(S, s_cols, X, xrec, slot, red, msr, occ);
                        if (S.cache_state[slot] == 2) break;
                        if (__builtin_amdgcn_s_memrealtime() - w0 >= limit) {
                            if (lane == 0) S.cache_state[slot] = 4;  // grow it here instead
                            wave_sync();
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
                taken = S.cache_state[slot] == 2;
                hslot = slot;
#ifdef PP_STAMPS
                ESTAMP(L, 7, hw0);  // a hit: waiting for the helper
#endif
            }
            if (taken) {
                const float4 jq = lane < kKP ? cache_joints(S, s_cols, hslot)[lane]
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
                if (hslot < kSpecCache)
                    commit(&cache[hslot], false, jq.x, jq.y, jq.z, jq.w);
                else
                    commit(&xrec[hslot - kSpecCache], true, jq.x, jq.y, jq.z, jq.w);
                s = t + 1;
                if (lane == 0) lds_release(&S.decided, s);  // the slot is free again
#ifdef PP_STAMPS
                n_hits++;
#endif
                if (n_anns >= kExtRefillAnns) {
                    // few speculated seeds left ahead: plan a round now, not at the next miss
                    const uint64_t aq = __ballot(lane < NS && S.cache_seed[lane] > t &&
                                                 (S.cache_state[lane] == 1 || S.cache_state[lane] == 2));
                    if (__popcll(aq) < kExtRefill) {
                        plan_lock(S);
                        plan_round(t, false, seeds[t]);
                        plan_unlock(S);
                    }
                }
                STAMP(4);
                continue;
            }
            // a miss: hand far-away free seeds to the idle helpers, then grow t here
            const pp_seed st = seeds[t];
            plan_lock(S);  // wave 0 plans every idle helper, this CU's and the external ones
            if (lane == 0) {
                S.own_x = st.x;
                S.own_y = st.y;
                S.own_s = st.s;
                lds_release(&S.own_on, 1);
                lds_release(&S.decided, t);
            }
            wave_sync();
            // (own = false: picks need not keep kExtSpecFar from seed t, which wave 0 grows
            // itself: cfg5 uniform 1517-1798 -> 1742-1787 images/s, planted unchanged;
            // r06z_ab_refill.txt)
            plan_round(t, false, st);
            plan_unlock(S);
#ifdef PP_STAMPS
            n_rounds++;
#endif
            STAMP(1);
            ann_from_seed(L, st, K, img);
            grow<true, CS>(g, L, img, 0, true, cstage);
            STAMP(2);
            commit(&L.a, false, lane < K ? L.a.data[lane][0] : 0.0f,
                   lane < K ? L.a.data[lane][1] : 0.0f, lane < K ? L.a.data[lane][2] : 0.0f,
                   lane < K ? L.a.joint_scales[lane] : 0.0f);
            s = t + 1;
            if (lane == 0) {
                lds_release(&S.own_on, 0);
                lds_release(&S.decided, s);
            }
            STAMP(3);
        }
        if (lane == 0) {
            lds_release(&S.done, 1);
            if (X) st_agent(&X->fin, 1u);
        }
    }
    __syncthreads();  // helpers drained: no wave of this CU is still growing into the cache
    ext_exit(X, g.n_ext);
    if (wave == 0) {
        occ_clear(g, L, log, occ);
        STAMP(5);
#ifdef PP_STAMPS
        st_acc[6] = n_rounds;
        st_acc[7] = n_hits;
#endif
        STAMP_FLUSH(1);
        seed_loop_outputs(g, Ls, img, n_anns, unset_mask);
    }
}

// ---------------------------------------------------------------------------------------
// the per-image decode kernel
// ---------------------------------------------------------------------------------------
// ---- complete_annotations (cifcaf.py:333-351) ----
// Each annotation is completed from its own joints and the read-only set-B columns, so the
// annotations of an image are spread over kCompleteWays workgroups.  Ones with every joint
// set are unchanged by it (their frontier is empty) and are skipped, and images the seed
// loop did not flag return at once.
// (5 or 6 waves per SIMD via amdgpu_waves_per_eu: 21 / 46 spills, slower)
template <bool CS>
__global__ __launch_bounds__(64) void complete_kernel(GrowArgs g) {
    __shared__ GrowLDS L;
    const int img = blockIdx.x;
    const int K = g.K;
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        L.status = 0;
        L.log_n = 0;
#ifdef PP_STAMPS
        for (int q = 0; q < 8; q++) L.fst[q] = 0;
#endif
    }
    wave_sync();
    STAMP_DECL
    pp_ann *work = g.work + (int64_t)img * g.ann_cap;
    const int n_anns = g.n_work[img];
    STAMP(0);
    if (!g.need_complete[img]) return;
    // annotations are handed out one at a time (their completion costs differ widely)
    for (;;) {
        int i = 0;
        if (lane == 0) i = atomicAdd(&g.complete_next[img], 1);
        i = __builtin_amdgcn_readfirstlane(i);
        if (i >= n_anns) break;
        // one vector load for the K visibilities (a short-circuit loop over them would wait
        // for each in turn)
        const float vj = lane < K ? work[i].data[lane][2] : 1.0f;
        if (!__ballot(lane < K && vj == 0.0f)) continue;
        copy_ann(&L.a, &work[i]);
        uint32_t unfilled = 0;
        for (int j = 0; j < K; j++) unfilled |= (L.a.data[j][2] == 0.0f) ? (1u << j) : 0u;
        grow<false, CS, GrowLDS>(g, L, img, 1, false);
        bool any0 = false;
        for (int j = 0; j < K; j++) {
            float &v = L.a.data[j][2];
            if (((unfilled >> j) & 1u) && v > 0.0f) v = (0.001f < v) ? 0.001f : v;  // np.minimum
            any0 = any0 || v == 0.0f;
        }
        if (any0) flood_fill(g, L);
        wave_sync();
        copy_ann(&work[i], &L.a);
    }
    STAMP(1);
    STAMP_FLUSH(2);
    if (lane == 0 && L.status) atomicOr(&g.status[img], L.status);
}

// ---- nms.Keypoints.annotations (nms.py:17-57) + output, one workgroup per image ----
// The score filters are per annotation: spread over the waves.  The suppression pass
// (nms.py:34-45) is sequential over the sorted annotations, but each joint lives on its
// own occupancy plane, so the planes are independent: wave w walks planes w, w + 8, ...
// and keeps the plane's marked boxes in a list instead of a u8 grid.  A joint is
// "occupied" iff the number of earlier marked boxes covering its cell is non-zero mod 256
// (the grid's u8 += 1 wraps), which is exactly what the grid lookup returns.
// Workgroups of kNmsWaves (8) waves for dense batches on the one-CU seed loop
// (PP_STAGE_NMS_WIDE), else kNmsNarrow (4): at 155 VGPRs a 4-wave workgroup (one wave per
// SIMD) fits on a CU beside a seed-loop workgroup (two waves per SIMD at 168), an 8-wave one
// does not, so in the overlapped pipeline the narrow NMS of batch i runs beside batch i + 1's
// seed loop instead of waiting for its CUs.  A/B on one box: planted cfg3 370-375k ->
// 385-394k images/s, cfg5 uniform 1356-1365 -> 1434-1443; uniform cfg3 (400 annotations per
// image, 17 planes on 4 waves) 15.1-15.3k -> 14.4-14.5k, hence the wide form there.
constexpr int kNmsWaves = 8;
constexpr int kNmsNarrow = 4;
// box-list scratch per image: one list per wave of nms_kernel, or per plane of
// nms_planes_kernel's fallback
constexpr int kNmsBoxLists = PP_MAX_KP;
static_assert(kNmsBoxLists >= kNmsWaves, "one box list per NMS wave");
// boxes per plane kept in REGISTERS, kNmsRegBoxes per lane (box i: lane i % 64, slot
// i / 64), global scratch beyond: a check is ALU over the lane's slots plus one wave sum,
// and the kernel needs no LDS for them (it fits beside the seed loop's 104 KB).  With the
// list in LDS (448 per plane) and global memory beyond, uniform cfg5 (1370 annotations per
// image) spent 20M cycles per image in the suppression pass on global-list loads.
constexpr int kNmsRegBoxes = 24;

struct ScoreLDS {
    double prod[kKP];
    double score_bc;
#ifdef PP_STAMPS
    uint64_t fst[8];  // unused here; keeps STAMP_FLUSH uniform
#endif
};

// Annotation.score() (annotation.py:24-28, 60-71) in float64, collective over one wave:
// lane j finds the rank of v_j in descending order, the rank-ordered products go to LDS
// and lane 0 adds them in NumPy's pairwise order.  `zero_j` (suppress_score_index, >= 0)
// reads as v = 0; `w` (the record's own score_weights) replaces the default weights.
__device__ double ann_score_w(ScoreLDS &L, const float (*data)[3], int K, int zero_j = -1,
                              const double *w = nullptr) {
    const int lane = threadIdx.x & 63;
    const double ws = (double)(3 * min(K, 3) + (K - min(K, 3)));
    if (lane < K) {
        const float vj = lane == zero_j ? 0.0f : data[lane][2];
        int rank = 0;
        for (int i = 0; i < K; i++) {
            const float vi = i == zero_j ? 0.0f : data[i][2];
            rank += (vi > vj) || (vi == vj && i < lane);
        }
        L.prod[rank] = (w ? w[rank] : (rank < 3 ? 3.0 : 1.0) / ws) * (double)vj;
    }
    wave_sync();
    if (lane == 0) L.score_bc = pw_sum(L.prod, K);
    wave_sync();
    const double res = L.score_bc;
    wave_sync();
    return res;
}

// the score nms.Keypoints sorts and filters record i of image img by: the default
// Annotation.score(), or with the caller's per-record fixed_score / suppress_score_index /
// score_weights (standalone NMS)
__device__ double nms_ann_score(const GrowArgs &g, ScoreLDS &L, int img, int i,
                                const float (*data)[3], int K) {
    if (!g.nms_spec) return ann_score_w(L, data, K);
    const int64_t gi = (int64_t)img * g.ann_cap + i;
    const int spec = g.nms_spec[gi];
    if (spec == -2) return g.nms_fixed[gi];
    return ann_score_w(L, data, K, spec, g.nms_sw + gi * K);
}

// the grid cell occ_get reads: 1 = occupied whatever the grid holds (f beyond the planes),
// 0 = free whatever it holds (empty grid), -1 = look at (xi, yi)
__device__ __forceinline__ int occ_cell(const OccGrid &o, int f, float x, float y, float red,
                                        int &xi, int &yi) {
    if (f >= o.f) return 1;
    if (o.h <= 0 || o.w <= 0) return 0;
    xi = (int)clip_ref(x / red, 0.0f, (float)(o.w - 1));
    yi = (int)clip_ref(y / red, 0.0f, (float)(o.h - 1));
    return -1;
}

// nms.py:34-45 for plane f: the m kept annotations in sorted order, whose joint f
// `load(r0, wi, x, y, v, s)` gives per lane (annotation r0 + lane: work index, joint f; v = 0
// beyond m).  The plane's marked boxes are kept in a list instead of a u8 grid: kNmsRegBoxes
// per lane in registers, `gbox` beyond.  A joint is "occupied" iff the number of earlier
// marked boxes covering its cell is non-zero mod 256 (the grid's u8 += 1 wraps).  Suppressed
// joints are written (v * suppression) as they are found.
template <typename Load>
__device__ __forceinline__ void nms_plane_boxes(const GrowArgs &g, pp_ann *work, int m, int f,
                                                const OccGrid &no, float red, int2 *gbox,
                                                Load load) {
    const int lane = threadIdx.x & 63;
    int nbox = 0;
    int2 rb[kNmsRegBoxes];  // (x0 | x1 << 16, y0 | y1 << 16); zero: covers nothing
#pragma unroll
    for (int q = 0; q < kNmsRegBoxes; q++) rb[q] = make_int2(0, 0);
    for (int r0 = 0; r0 < m; r0 += 64) {
        int wi = 0;
        float jx = 0.0f, jy = 0.0f, jv = 0.0f, js = 0.0f;
        load(r0, wi, jx, jy, jv, js);
        const int nr = min(64, m - r0);
        for (int l = 0; l < nr; l++) {
            const float v = rl_f(jv, l);
            if (v == 0.0f) continue;
            const float x = rl_f(jx, l), y = rl_f(jy, l);
            int xi = 0, yi = 0;
            const int fixed = occ_cell(no, f, x, y, red, xi, yi);
            int cnt = 0;
            if (fixed < 0) {
#pragma unroll
                for (int q = 0; q < kNmsRegBoxes; q += 4) {  // unused slots are zero
                    if (q * 64 >= nbox) continue;  // uniform: skip empty groups
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int2 b = rb[q + u];
                        cnt += (xi >= (b.x & 0xFFFF) && xi < (b.x >> 16) &&
                                yi >= (b.y & 0xFFFF) && yi < (b.y >> 16));
                    }
                }
                for (int q = kNmsRegBoxes * 64 + lane; q < nbox; q += 64) {
                    const int2 b = gbox[q];
                    cnt += (xi >= (b.x & 0xFFFF) && xi < (b.x >> 16) &&
                            yi >= (b.y & 0xFFFF) && yi < (b.y >> 16));
                }
                cnt = wave_total(cnt);
            }
            const bool occupied = fixed < 0 ? (cnt & 255) != 0 : fixed == 1;
            if (occupied) {
                if (lane == 0) work[rl_i(wi, l)].data[f][2] = v * g.cfg.nms_suppression;
            } else {
                int box[4];
                if (occ_box(g, no, f, x, y, rl_f(js, l), box)) {
                    const int2 nb = make_int2(box[0] | (box[1] << 16), box[2] | (box[3] << 16));
                    if (nbox < kNmsRegBoxes * 64) {
#pragma unroll
                        for (int q = 0; q < kNmsRegBoxes; q++)
                            if (q == (nbox >> 6) && lane == (nbox & 63)) rb[q] = nb;
                    } else if (lane == 0) {
                        gbox[nbox] = nb;
                    }
                    nbox++;
                    // only a box in global memory needs the fence (a fence here waits
                    // for every outstanding store, e.g. the suppressed v above)
                    if (nbox > kNmsRegBoxes * 64) wave_sync();
                }
            }
        }
    }
}

// PHASE 0: the whole of nms.Keypoints.annotations in one launch (suppression planes by
// nms_plane_boxes); 1: up to the sorted keep list, whose count and occupancy-grid shape go
// to the meta words (nms_planes_kernel runs the planes); 3: from the suppressed planes on.
template <int W, int PHASE = 0>
__global__ __launch_bounds__(64 * W) void nms_kernel(GrowArgs g) {
    __shared__ ScoreLDS Ls[W];
    __shared__ int s_m, s_m2, s_status;
    __shared__ float s_mx, s_my;
    const int img = blockIdx.x;
    const int K = g.K;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    ScoreLDS &L = Ls[wave];
    pp_ann *work = g.work + (int64_t)img * g.ann_cap;
    pp_ann *out = g.out + (int64_t)img * g.ann_cap;
    const int n_anns = max(0, min(g.n_work[img], g.ann_cap));
    const int cap = g.ann_cap;
    int *keep = g.nms_idx + (int64_t)img * (4 * cap + g.ann_np);  // kept work indices
    int *surv = keep + cap;                                           // survivors
    int *flag = surv + cap;                                           // per-index pass flags
    int *perm2 = flag + cap;                                          // meta: m, grid h, w
    int *perm = perm2 + cap;                                          // sort permutation
    double *score = g.nms_score + (int64_t)img * 2 * cap;             // by work index
    double *kscore = score + cap;                                     // by kept / survivor rank
    float *amax = g.nms_f + (int64_t)img * 2 * cap;                   // per-ann max x, max y
    int2 *gbox = g.nms_box + ((int64_t)img * kNmsBoxLists + wave) * cap;
    const float red = (float)g.cfg.occupancy_reduction;
    const float kt = g.cfg.nms_keypoint_threshold;
    const double it = g.nms_it;
    if (threadIdx.x == 0) {
        s_status = g.status[img];
        g.complete_next[img] = 0;  // workspace contract: left zero
    }
#ifdef PP_STAMPS
    if (lane == 0)
        for (int q = 0; q < 8; q++) L.fst[q] = 0;
#endif
    __syncthreads();
    STAMP_DECL

    if (PHASE == 0 && !g.cfg.apply_nms) {
        for (int i = wave; i < n_anns; i += W) {
            copy_ann(&out[i], &work[i]);
            const double sc = nms_ann_score(g, L, img, i, work[i].data, K);
            if (lane == 0) {
                out[i].score = sc;
                if (g.out_idx) g.out_idx[(int64_t)img * cap + i] = i;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            g.counts[img] = n_anns;
            g.status[img] = s_status;
        }
        return;
    }

    int m = 0;
    if constexpr (PHASE != 3) {
    // nms.py:20-22: zero joints below keypoint_threshold, drop low scores (per annotation)
    for (int i = wave; i < n_anns; i += W) {
        pp_ann &a = work[i];
        if (lane < K && a.data[lane][2] < kt) {
            a.data[lane][0] = 0.0f;
            a.data[lane][1] = 0.0f;
            a.data[lane][2] = 0.0f;
        }
        wave_sync();
        const double sc = nms_ann_score(g, L, img, i, a.data, K);
        if (lane == 0) {
            float ax = a.data[0][0], ay = a.data[0][1];
            for (int j = 1; j < K; j++) {
                ax = a.data[j][0] > ax ? a.data[j][0] : ax;
                ay = a.data[j][1] > ay ? a.data[j][1] : ay;
            }
            score[i] = sc;
            flag[i] = sc >= it;
            amax[i] = ax;
            amax[cap + i] = ay;
        }
    }
    __syncthreads();
    STAMP(2);
    // keep list in work order + the occupancy shape (nms.py:27-31), then the stable sort
    if (wave == 0) {
        int m = 0;
        float mx = 0.0f, my = 0.0f;
        for (int i0 = 0; i0 < n_anns; i0 += 64) {
            const int i = i0 + lane;
            const bool k = i < n_anns && flag[i];
            float ax = 0.0f, ay = 0.0f;
            double sc = 0.0;
            if (k) {
                ax = amax[i];
                ay = amax[cap + i];
                sc = score[i];
            }
            const uint64_t km = __ballot(k);
            if (k) {
                const int r = m + lane_prefix(km);
                keep[r] = i;
                kscore[r] = sc;
            }
            uint64_t rest = km;
            while (rest) {  // max over the kept annotations, in order (NaN behaviour)
                const int l = __ffsll((unsigned long long)rest) - 1;
                rest &= rest - 1;
                const float lx = rl_f(ax, l), ly = rl_f(ay, l);
                if (m == 0 || lx > mx) mx = lx;
                if (m == 0 || ly > my) my = ly;
                m++;
            }
        }
        wave_sync();
        if (m > 0) {
            int np = 1;
            while (np < m) np <<= 1;
            sort_by_score(perm, np, m, kscore);  // nms.py:33 (stable)
        }
        if (lane == 0) {
            s_m = m;
            s_mx = mx;
            s_my = my;
        }
    }
    __syncthreads();
    STAMP(3);
    m = s_m;
    } else {
        m = perm2[0];
    }
    if constexpr (PHASE == 1) {
        if (threadIdx.x == 0) {
            perm2[0] = m;
            perm2[1] = perm2[2] = 0;
            if (m > 0) {  // Occupancy((K, int(max y + 1), int(max x + 1)), 2, min_scale=4)
                const long oh = (long)((double)(long)(s_my + 1.0f) / g.cfg.occupancy_reduction);
                const long ow = (long)((double)(long)(s_mx + 1.0f) / g.cfg.occupancy_reduction);
                perm2[1] = (int)(oh > 0 ? oh : 0);
                perm2[2] = (int)(ow > 0 ? ow : 0);
            }
        }
        return;
    }
    int n_out = 0;
    if (m > 0) {
        if constexpr (PHASE == 0) {
        // Occupancy((K, int(max y + 1), int(max x + 1)), 2, min_scale=4)
        const long oh = (long)((double)(long)(s_my + 1.0f) / g.cfg.occupancy_reduction);
        const long ow = (long)((double)(long)(s_mx + 1.0f) / g.cfg.occupancy_reduction);
        const OccGrid no = occ_grid(nullptr, K, (int)(oh > 0 ? oh : 0), (int)(ow > 0 ? ow : 0));
        // the first 64 sorted annotations' joints of every plane this wave walks, loaded in
        // one round trip (their work indices in one more) instead of three per plane
        constexpr int kNmsPre = 4;  // planes per wave prefetched (K <= 32)
        int wi0 = 0;
        float pre[kNmsPre][4];
        if (lane < m) wi0 = keep[perm[lane]];
#pragma unroll
        for (int u = 0; u < kNmsPre; u++) {
            const int f = wave + u * W;
            pre[u][0] = pre[u][1] = pre[u][2] = pre[u][3] = 0.0f;
            if (f < K && lane < m) {
                pre[u][0] = work[wi0].data[f][0];
                pre[u][1] = work[wi0].data[f][1];
                pre[u][2] = work[wi0].data[f][2];
                pre[u][3] = work[wi0].joint_scales[f];
            }
        }
        for (int f = wave, u = 0; f < K; f += W, u++) {  // nms.py:34-45, one plane per pass
            nms_plane_boxes(g, work, m, f, no, red, gbox, [&](int r0, int &wi, float &jx, float &jy,
                                                                float &jv, float &js) {
                const int r = r0 + lane;
                if (r0 == 0 && u < kNmsPre) {  // prefetched (selects: no dynamic index)
                    wi = wi0;
#pragma unroll
                    for (int w = 0; w < kNmsPre; w++)
                        if (w == u) {
                            jx = pre[w][0];
                            jy = pre[w][1];
                            jv = pre[w][2];
                            js = pre[w][3];
                        }
                } else if (r < m) {
                    wi = keep[perm[r]];
                    jx = work[wi].data[f][0];
                    jy = work[wi].data[f][1];
                    jv = work[wi].data[f][2];
                    js = work[wi].joint_scales[f];
                }
            });
        }
        __syncthreads();
        STAMP(4);
        }
        // nms.py:51-53 in sorted order: zero low joints, drop low scores
        for (int r = wave; r < m; r += W) {
            const int wi = keep[perm[r]];
            pp_ann &a = work[wi];
            if (lane < K && a.data[lane][2] < kt) {
                a.data[lane][0] = 0.0f;
                a.data[lane][1] = 0.0f;
                a.data[lane][2] = 0.0f;
            }
            wave_sync();
            const double sc = nms_ann_score(g, L, img, wi, a.data, K);
            if (lane == 0) {
                flag[r] = sc >= it;
                score[r] = sc;  // by sorted rank now (the work-index scores are consumed)
            }
        }
        __syncthreads();
        STAMP(6);
        if (wave == 0) {
            int m2 = 0;
            for (int r0 = 0; r0 < m; r0 += 64) {
                const int r = r0 + lane;
                const bool k = r < m && flag[r];
                int wi = 0;
                double sc = 0.0;
                if (k) {
                    wi = keep[perm[r]];
                    sc = score[r];
                }
                const uint64_t km = __ballot(k);
                if (k) {
                    const int q = m2 + lane_prefix(km);
                    surv[q] = wi;
                    kscore[q] = sc;
                }
                m2 += __popcll(km);
            }
            wave_sync();
            if (m2 > 0) {
                int np2 = 1;
                while (np2 < m2) np2 <<= 1;
                sort_by_score(perm, np2, m2, kscore);  // nms.py:54
            }
            if (lane == 0) s_m2 = m2;
        }
        __syncthreads();
        STAMP(7);
        n_out = s_m2;
        for (int r = wave; r < n_out; r += W) {
            copy_ann(&out[r], &work[surv[perm[r]]]);
            if (lane == 0) {
                out[r].score = kscore[perm[r]];
                if (g.out_idx) g.out_idx[(int64_t)img * cap + r] = surv[perm[r]];
            }
        }
    }
    __syncthreads();
    STAMP(8);
    if (wave == 0) {
        STAMP_FLUSH(3);
    }
    if (threadIdx.x == 0) {
        g.counts[img] = n_out;
        g.status[img] = s_status;
    }
}

}  // namespace pp

namespace pp {

// ---- nms.py:34-45 per (image, plane), the plane's occupancy as a bitmap in LDS ----
// Between nms_kernel<W, 1> (the sorted keep list, its count and grid shape in the meta words)
// and nms_kernel<W, 3> (the refilter and output): one wave per (image, joint plane), walking
// the image's kept annotations in sorted order.  The reference's grid holds u8 counts and a
// joint is occupied iff its cell's count is non-zero (mod 256: += 1 wraps).  Here a cell is
// one bit, set when a marked box covers it: the same answer while no cell is covered by 256
// boxes or more.  Counts of the boxes meeting each 32 x 32-cell block (never below any of
// its cells' counts) guard that: a plane where a block reaches 256 boxes is decided again by
// nms_plane_boxes (the exact counting form), which also takes grids larger than the LDS
// bitmap (keypoints far outside the field).  Suppressed joints are written only after the
// plane is decided.  A check is one LDS word, a mark one OR per (box row, word): O(m) per
// plane instead of nms_plane_boxes' O(m * marked boxes / 64).
constexpr int kNmsBlk = 32;

struct NmsBitmapGeo {  // the LDS bitmap's capacity (the launch's dynamic LDS)
    int cap_h, cap_w;  // grid rows and columns it holds
    __host__ __device__ int wpr() const { return (cap_w + 31) >> 5; }
    __host__ __device__ int blocks() const {
        return ((cap_h + kNmsBlk - 1) / kNmsBlk) * ((cap_w + kNmsBlk - 1) / kNmsBlk);
    }
    __host__ __device__ size_t bytes(int ann_cap) const {
        return sizeof(uint32_t) * ((size_t)cap_h * wpr() + blocks() + (ann_cap + 31) / 32);
    }
};

__global__ __launch_bounds__(64) void nms_planes_kernel(GrowArgs g, NmsBitmapGeo geo) {
    extern __shared__ uint32_t s_bm[];
    const int img = blockIdx.x, f = blockIdx.y;
    const int lane = threadIdx.x;
    const int K = g.K, cap = g.ann_cap;
    pp_ann *work = g.work + (int64_t)img * cap;
    const int *keep = g.nms_idx + (int64_t)img * (4 * cap + g.ann_np);
    const int *meta = keep + 3 * cap;  // nms_kernel<W, 1>: m, grid h, grid w
    const int *perm = meta + cap;
    const int m = meta[0], oh = meta[1], ow = meta[2];
    if (m <= 0 || f >= K) return;
    const float red = (float)g.cfg.occupancy_reduction;
    const OccGrid no = occ_grid(nullptr, K, oh, ow);
    auto load = [&](int r0, int &wi, float &jx, float &jy, float &jv, float &js) {
        const int r = r0 + lane;
        if (r < m) {
            wi = keep[perm[r]];
            jx = work[wi].data[f][0];
            jy = work[wi].data[f][1];
            jv = work[wi].data[f][2];
            js = work[wi].joint_scales[f];
        }
    };
    int2 *gbox = g.nms_box + ((int64_t)img * kNmsBoxLists + f) * cap;
    if (oh <= 0 || ow <= 0 || oh > geo.cap_h || ow > geo.cap_w) {
        nms_plane_boxes(g, work, m, f, no, red, gbox, load);
        return;
    }
    const int wpr = (ow + 31) >> 5;
    const int bcols = (ow + kNmsBlk - 1) / kNmsBlk;
    uint32_t *bits = s_bm;                                // oh rows of wpr words
    uint32_t *bcnt = s_bm + (size_t)geo.cap_h * geo.wpr();  // boxes per block
    uint32_t *supp = bcnt + geo.blocks();                   // suppressed ranks
    const int nbits = oh * wpr, nblk = ((oh + kNmsBlk - 1) / kNmsBlk) * bcols;
    for (int i = lane; i < nbits; i += 64) bits[i] = 0u;
    for (int i = lane; i < nblk; i += 64) bcnt[i] = 0u;
    for (int i = lane; i < (m + 31) / 32; i += 64) supp[i] = 0u;
    wave_sync();
    bool over = false;
    for (int r0 = 0; r0 < m; r0 += 64) {
        int wi = 0;
        float jx = 0.0f, jy = 0.0f, jv = 0.0f, js = 0.0f;
        load(r0, wi, jx, jy, jv, js);
        // per lane: its joint's cell, and the box it marks when free (0: none)
        int xi = 0, yi = 0;
        (void)occ_cell(no, f, jx, jy, red, xi, yi);  // -1: f < K and a non-empty grid
        int box[4] = {0, 0, 0, 0};
        const bool hb = r0 + lane < m && jv != 0.0f && occ_box(g, no, f, jx, jy, js, box);
        const int cellp = xi | (yi << 16);
        const int bxp = hb ? box[0] | (box[1] << 16) : 0;  // x1 >= 1 when hb: nonzero
        const int byp = box[2] | (box[3] << 16);
        const int nr = min(64, m - r0);
        for (int l = 0; l < nr; l++) {
            if (rl_f(jv, l) == 0.0f) continue;
            const int cp = rl_i(cellp, l);
            const int cx = cp & 0xFFFF, cy = cp >> 16;
            if ((bits[cy * wpr + (cx >> 5)] >> (cx & 31)) & 1u) {  // occupied
                if (lane == 0) atomicOr(&supp[(r0 + l) >> 5], 1u << ((r0 + l) & 31));
                continue;
            }
            const int bx = rl_i(bxp, l);
            if (bx == 0) continue;  // no box (empty after clipping)
            const int by = rl_i(byp, l);
            const int x0 = bx & 0xFFFF, x1 = bx >> 16, y0 = by & 0xFFFF, y1 = by >> 16;
            const int w0 = x0 >> 5, nw = ((x1 - 1) >> 5) - w0 + 1;
            const int items = (y1 - y0) * nw;
            for (int t = lane; t < items; t += 64) {  // (box row, word) pairs
                const int ry = y0 + t / nw, wq = w0 + t % nw;
                const int lo = max(x0 - 32 * wq, 0), hi = min(x1 - 32 * wq, 32);
                const uint32_t mk = (hi - lo >= 32) ? ~0u : (((1u << (hi - lo)) - 1u) << lo);
                atomicOr(&bits[ry * wpr + wq], mk);
            }
            const int bx0 = x0 / kNmsBlk, bx1 = (x1 - 1) / kNmsBlk;
            const int by0 = y0 / kNmsBlk, by1 = (y1 - 1) / kNmsBlk;
            const int nbk = (bx1 - bx0 + 1) * (by1 - by0 + 1);
            for (int t = lane; t < nbk; t += 64) {  // the guard: boxes per block
                const int bq = (by0 + t / (bx1 - bx0 + 1)) * bcols + bx0 + t % (bx1 - bx0 + 1);
                over |= atomicAdd(&bcnt[bq], 1u) >= 255u;
            }
            wave_sync();  // the marks before the next check
        }
    }
    if (__ballot(over)) {  // a cell may have wrapped: decide the plane by counting
        nms_plane_boxes(g, work, m, f, no, red, gbox, load);
        return;
    }
    for (int r = lane; r < m; r += 64)  // nms.py:43: data[f, 2] *= suppression
        if ((supp[r >> 5] >> (r & 31)) & 1u) {
            float *v = &work[keep[perm[r]]].data[f][2];
            *v = *v * g.cfg.nms_suppression;
        }
}

}  // namespace pp

// ---------------------------------------------------------------------------------------
// host: workspace layout + pp_decode_batch
// ---------------------------------------------------------------------------------------
namespace pp {

int launch_seeds(const Heads &h, const HrMap &hr, int n_img, int K, const pp_config *cfg,
                 pp_seed *seeds, int cap, int *counts, void *scratch, hipStream_t s,
                 bool emitted);
size_t seeds_scratch_size(int n_img, int cap);
int launch_caf_bucketed(const Heads &h, const HrMap &hr, int n_img, int K, int C,
                        const int32_t *skeleton, const pp_config *cfg, float th, float *cols,
                        int *offs, const int *gate, bool index_only, hipStream_t s);
void caf_bucket_grid(int H, int W, int stride, int *bw, int *bh, int *nb, float *inv_e);

static inline size_t align_up(size_t a) { return (a + 255) / 256 * 256; }

struct DecodeLayout {
    int hh, ww;
    int64_t pitch, hw;
    int seed_cap, ann_cap, ann_np, log_cap;
    int bw, bh, nb;
    float inv_e;
    int64_t occ_cap;
    size_t off_cifhr, off_hr_aux, off_hr_masks, off_cifhr_ws, off_seeds, off_seed_counts, off_seed_ws, off_cols[2],
        off_offs[2], off_n_work, off_need, off_occ, off_wq, off_log, off_work, off_spec, off_xext, off_xrec, off_nms_score,
        off_nms_idx, off_nms_f, off_nms_box, total;
    size_t cifhr_ws_bytes;
};

// CifHr map from head 0 (cif_hr.py:46-51); column sets and seeds over the cells of all heads
static DecodeLayout make_layout(int n_img, int K, int C, const Heads &h, const pp_config *cfg,
                                int ann_cap) {
    DecodeLayout d{};
    d.hh = h.hr_hh;
    d.ww = h.hr_ww;
    d.pitch = pp_cifhr_pitch(d.ww);
    d.hw = h.caf_cells();
    d.seed_cap = (int)(K * h.cif_cells());  // every cell of every field: no seed overflow
    d.ann_cap = ann_cap;
    d.ann_np = 1;
    while (d.ann_np < ann_cap) d.ann_np <<= 1;
    d.log_cap = K * ann_cap;
    const int64_t oh = (int64_t)((double)d.hh / cfg->occupancy_reduction);
    const int64_t ow = (int64_t)((double)d.ww / cfg->occupancy_reduction);
    d.occ_cap = (int64_t)align_up((size_t)(K * (oh + kOccMargin) * ((ow + kOccMargin + 15) & ~15)));
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += align_up(bytes);
        return at;
    };
    const size_t n = (size_t)n_img;
    // scratch CifHr, block-sparse (HrMap with masks): 64x64 tiles of 8x8 blocks
    const HrMap geo = dense_hr(nullptr, d.hh, d.ww);
    d.off_cifhr = take(n * K * (size_t)geo.tiles * kHrTile * kHrTile * sizeof(float));
    d.off_hr_aux = take(h.n_groups > 1 ? n * K * (size_t)geo.tiles * kHrTile * kHrTile * sizeof(float) : 0);
    d.off_hr_masks = take(n * K * (size_t)geo.tiles * sizeof(uint64_t));
    d.cifhr_ws_bytes = std::max(cifhr_heads_workspace_size(h, n_img, K),
                                cifhr_sparse_workspace_size(h, n_img, K));
    d.off_cifhr_ws = take(d.cifhr_ws_bytes);
    d.off_seeds = take(n * d.seed_cap * sizeof(pp_seed));
    d.off_seed_counts = take(n * sizeof(int));
    d.off_seed_ws = take(seeds_scratch_size(n_img, d.seed_cap));
    caf_bucket_grid(h.cH[0], h.cW[0], h.cstride[0], &d.bw, &d.bh, &d.nb, &d.inv_e);
    for (int t = 0; t < 2; t++) {
        const bool used = t == 0 || cfg->force_complete;
        d.off_cols[t] = take(used ? n * C * 2 * (t ? 1 : kColRows) * d.hw * sizeof(float) : 0);
        d.off_offs[t] = take(used ? n * C * 2 * (d.nb + 1) * sizeof(int) : 0);
    }
    d.off_n_work = take(n * sizeof(int));
    d.off_need = take(n * sizeof(int));
    d.off_occ = take(n * d.occ_cap);  // zero region from here (pp_decode_workspace_zero_offset)
    d.off_wq = take(n * sizeof(int));
    d.off_log = take(n * d.log_cap * sizeof(OccLog));
    d.off_work = take(n * ann_cap * sizeof(pp_ann));
    d.off_spec = take(n * kSpecCache * sizeof(pp_ann));
    d.off_xext = take(n * sizeof(SeedExt));
    d.off_xrec = take(n * kExtCache * sizeof(pp_ann));
    d.off_nms_score = take(n * 2 * ann_cap * sizeof(double));
    d.off_nms_idx = take(n * (4 * ann_cap + d.ann_np) * sizeof(int));
    d.off_nms_f = take(n * 2 * ann_cap * sizeof(float));
    d.off_nms_box = take(n * kNmsBoxLists * ann_cap * sizeof(int2));
    d.total = o;
    return d;
}

}  // namespace pp

using namespace pp;

extern "C" {

size_t pp_decode_workspace_size(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                                const pp_config *cfg, int32_t ann_capacity) {
    if (!cfg || n_img < 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0 || ann_capacity <= 0 ||
        cfg->stride <= 0)
        return 0;
    return make_layout(n_img, K, C, single_head(nullptr, nullptr, H, W, cfg->stride), cfg,
                       ann_capacity).total;
}

size_t pp_decode_workspace_zero_offset(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                                       const pp_config *cfg, int32_t ann_capacity) {
    if (!cfg || n_img <= 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0 || ann_capacity <= 0 ||
        cfg->stride <= 0)
        return 0;
    return make_layout(n_img, K, C, single_head(nullptr, nullptr, H, W, cfg->stride), cfg,
                       ann_capacity).off_occ;
}

size_t pp_decode_work_offset(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                             const pp_config *cfg, int32_t ann_capacity) {
    if (!cfg || n_img <= 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0 || ann_capacity <= 0 ||
        cfg->stride <= 0)
        return 0;
    return make_layout(n_img, K, C, single_head(nullptr, nullptr, H, W, cfg->stride), cfg,
                       ann_capacity).off_work;
}

size_t pp_decode_multi_work_offset(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                   int32_t n_img, int32_t K, int32_t C, const pp_config *cfg,
                                   int32_t ann_capacity) {
    Heads h;
    if (!cfg || make_heads(scales, n_scales, cif_pairs, 3, &h, "pp_decode_multi_work_offset") ||
        n_img <= 0 || K <= 0 || C <= 0 || ann_capacity <= 0)
        return 0;
    return make_layout(n_img, K, C, h, cfg, ann_capacity).off_work;
}

size_t pp_decode_multi_workspace_size(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                      int32_t n_img, int32_t K, int32_t C, const pp_config *cfg,
                                      int32_t ann_capacity) {
    Heads h;
    if (!cfg || make_heads(scales, n_scales, cif_pairs, 3, &h, "pp_decode_multi_workspace_size") ||
        n_img < 0 || K <= 0 || C <= 0 || ann_capacity <= 0)
        return 0;
    return make_layout(n_img, K, C, h, cfg, ann_capacity).total;
}

size_t pp_decode_multi_workspace_zero_offset(const pp_scale *scales, int32_t n_scales,
                                             int32_t cif_pairs, int32_t n_img, int32_t K,
                                             int32_t C, const pp_config *cfg,
                                             int32_t ann_capacity) {
    Heads h;
    if (!cfg || make_heads(scales, n_scales, cif_pairs, 3, &h, "pp_decode_multi_workspace_zero_offset") ||
        n_img <= 0 || K <= 0 || C <= 0 || ann_capacity <= 0)
        return 0;
    return make_layout(n_img, K, C, h, cfg, ann_capacity).off_occ;
}

}  // extern "C"

namespace pp {

// One non-blocking side stream (+ fork / join events) per device, created on first use;
// the mutex keeps concurrent host threads' fork / join pairs from interleaving.
struct SideStream {
    hipStream_t stream;
    hipEvent_t fork, join;
    mutable std::mutex mu;
};

static const SideStream *side_stream() {
    static std::mutex create_mu;
    static SideStream *per_dev[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lock(create_mu);
    if (!per_dev[dev]) {
        SideStream *ss = new SideStream();
        if (hipStreamCreateWithFlags(&ss->stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ss->fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ss->join, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            delete ss;
            return nullptr;
        }
        per_dev[dev] = ss;
    }
    return per_dev[dev];
}

// External helper workgroups per image for the seed loop: enough to give every CU a seed
// loop workgroup when the batch has fewer images than CUs (at most kExtWgMax).
static int seed_ext_per_image(int n_img) {
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (cus[dev] <= 0 &&
        hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        cus[dev] = 0;
    }
    if (n_img <= 0 || cus[dev] <= 0) return 0;
    return std::max(0, std::min(kExtWgMax, cus[dev] / n_img - 1));
}

// Force-complete workgroups per image.  The workgroups pull annotations from a per-image
// counter, so any count gives the same result; 8 or 16 for sparse batches measured no
// better than 64 (round 5).
static int complete_ways(uint32_t) { return kCompleteWays; }

// nms.Keypoints (nms.py:17-57) of a decode: nms_kernel<W> in one launch, or with `bitmap`
// (PP_STAGE_NMS_BITMAP) nms_kernel<W, 1>, the planes as
// bitmaps (nms_planes_kernel, one wave per (image, plane)), nms_kernel<W, 3> -- unless NMS
// is off or the bitmap would not fit kNmsBitmapLds.  `wide`: 8-wave workgroups
// (PP_STAGE_NMS_WIDE).  The bitmap holds the nominal grid (CifHr map / reduction) plus
// kNmsMargin cells; an image whose keypoints reach further takes nms_plane_boxes in the
// plane kernel.  Measured (round 5, one box): the three launches take 60 vs 76 us per planted
// cfg3 step and 1.48 vs 2.51 ms per uniform one, one step at a time; but in the overlapped
// pipeline planted 397k-402k vs 405k-410k and uniform 14.7k vs 15.5k-15.8k images/s (the
// 4352 one-wave workgroups of the plane kernel beside the next batch's seed loop), so the
// single launch stays the default.
constexpr int kNmsMargin = 16;
constexpr size_t kNmsBitmapLds = 64 * 1024;

static int launch_nms(const GrowArgs &g, int n_img, bool wide, bool bitmap, hipStream_t s) {
    NmsBitmapGeo geo{};
    geo.cap_h = (int)((double)g.hh / g.cfg.occupancy_reduction) + kNmsMargin;
    geo.cap_w = (int)((double)g.ww / g.cfg.occupancy_reduction) + kNmsMargin;
    const size_t lds = geo.bytes(g.ann_cap);
    if (bitmap && g.cfg.apply_nms && lds <= kNmsBitmapLds) {
        if (wide)
            hipLaunchKernelGGL((nms_kernel<kNmsWaves, 1>), dim3(n_img), dim3(64 * kNmsWaves), 0, s, g);
        else
            hipLaunchKernelGGL((nms_kernel<kNmsNarrow, 1>), dim3(n_img), dim3(64 * kNmsNarrow), 0, s, g);
        hipLaunchKernelGGL(nms_planes_kernel, dim3(n_img, g.K), dim3(64), lds, s, g, geo);
        if (wide)
            hipLaunchKernelGGL((nms_kernel<kNmsWaves, 3>), dim3(n_img), dim3(64 * kNmsWaves), 0, s, g);
        else
            hipLaunchKernelGGL((nms_kernel<kNmsNarrow, 3>), dim3(n_img), dim3(64 * kNmsNarrow), 0, s, g);
        return check_launch("pp_decode_batch(nms)");
    }
    if (wide)
        hipLaunchKernelGGL(nms_kernel<kNmsWaves>, dim3(n_img), dim3(64 * kNmsWaves), 0, s, g);
    else
        hipLaunchKernelGGL(nms_kernel<kNmsNarrow>, dim3(n_img), dim3(64 * kNmsNarrow), 0, s, g);
    return check_launch("pp_decode_batch(nms)");
}

// optional inputs of pp_decode_initial
struct DecodeInit {
    const pp_ann *anns = nullptr;
    const int32_t *counts = nullptr;
    int32_t cap = 0;
    int32_t *out_index = nullptr;
};

static int decode_heads(const Heads &h, int32_t n_img, int32_t K, int32_t C,
                        const int32_t *skeleton, const pp_config *cfg, float *d_cifhr,
                        pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                        int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                        uint32_t stages, void *stream, const DecodeInit &init = DecodeInit{}) {
    if (!skeleton || !cfg || !d_anns || !d_counts || !d_status || !d_workspace)
        return fail(PP_EINVAL, "pp_decode_batch: NULL argument");
    for (int m = 0; m < h.n_cif; m++)
        if (!h.cif[m]) return fail(PP_EINVAL, "pp_decode_batch: NULL CIF field");
    for (int m = 0; m < h.n_caf; m++)
        if (!h.caf[m]) return fail(PP_EINVAL, "pp_decode_batch: NULL CAF field");
    if (n_img < 0 || K <= 0 || K > PP_MAX_KP || C <= 0 || C > PP_MAX_EDGES ||
        ann_capacity <= 0 || cfg->occupancy_reduction <= 0)
        return fail(PP_ESHAPE, "pp_decode_batch: shape outside the supported envelope "
                               "(K <= PP_MAX_KP, C <= PP_MAX_EDGES)");
    if (cfg->connection_method != 0 && cfg->connection_method != 1)
        return fail(PP_EINVAL, "connection method not known");
    for (int i = 0; i < 2 * C; i++)
        if (skeleton[i] < 1 || skeleton[i] > K)
            return fail(PP_EINVAL, "pp_decode_batch: skeleton joint index out of 1..K");
    if ((int64_t)K * h.cif_cells() > INT32_MAX || h.caf_cells() > INT32_MAX)
        return fail(PP_ESHAPE, "pp_decode_batch: fields too large");
    if (n_img == 0) return PP_OK;
    const DecodeLayout d = make_layout(n_img, K, C, h, cfg, ann_capacity);
    if (workspace_bytes < d.total) return fail(PP_ENOMEM, "pp_decode_batch: workspace too small");
    if ((int64_t)d.hh >= kMaxHrSide || (int64_t)d.ww >= kMaxHrSide)
        return fail(PP_ESHAPE, "pp_decode_batch: field too large (CifHr map of 32768 px or "
                               "more per side)");
    char *ws = (char *)d_workspace;
    hipStream_t s = (hipStream_t)stream;
    // the caller's d_cifhr gets the dense map; otherwise the decoder keeps the block-sparse
    // scratch map, written only where splat boxes land
    float *hr_base = d_cifhr ? d_cifhr : (float *)(ws + d.off_cifhr);
    uint64_t *hr_masks = d_cifhr ? nullptr : (uint64_t *)(ws + d.off_hr_masks);
    HrMap hr = dense_hr(hr_base, d.hh, d.ww);
    hr.masks = hr_masks;
    pp_seed *seeds = (pp_seed *)(ws + d.off_seeds);
    int *seed_counts = (int *)(ws + d.off_seed_counts);
    float *cols[2] = {(float *)(ws + d.off_cols[0]), (float *)(ws + d.off_cols[1])};
    int *offs[2] = {(int *)(ws + d.off_offs[0]), (int *)(ws + d.off_offs[1])};
    int rc = PP_OK;
    // PP_STAGE_COMPLETE_SETS_EARLY with stage 1 (and without 8): the force-complete sets read
    // only the CAF fields, so they start on the side stream before the CifHr map, and a later
    // call's side-stream join (stages 2 | 4) covers them
    const bool b_first = (stages & PP_STAGE_COMPLETE_SETS_EARLY) && (stages & 1u) &&
                         !(stages & 8u) && cfg->force_complete;
    if (b_first) {
        const SideStream *side = side_stream();
        if (!side) return fail(PP_EHIP, "pp_decode_stages: no side stream for stage 16");
        std::lock_guard<std::mutex> lock(side->mu);
        if (hipEventRecord(side->fork, s) != hipSuccess ||
            hipStreamWaitEvent(side->stream, side->fork, 0) != hipSuccess)
            return fail(PP_EHIP, "pp_decode_batch: side-stream fork failed");
        rc = launch_caf_bucketed(h, hr, n_img, K, C, skeleton, cfg, cfg->complete_caf_threshold,
                                 cols[1], offs[1], nullptr, true, side->stream);
        if (rc) {
            (void)hipEventRecord(side->join, side->stream);
            (void)hipStreamWaitEvent(s, side->join, 0);
            return rc;
        }
    }
    // the block-sparse map's kernel emits the seeds too when it can (stage 1 then writes
    // what seeds_emit_kernel would; stage 2 sorts them): the same test in both stages
    const bool fused_seeds = !d_cifhr && cifhr_fuses_seeds(h, n_img, K, cfg);
    if (stages & 1u) {
        if (d_cifhr) {
            rc = cifhr_heads_launch<false>(h, n_img, K, cfg, d_cifhr, ws + d.off_cifhr_ws,
                                           d.cifhr_ws_bytes, s, "pp_decode_batch(cifhr)");
        } else {
            const SeedSink sink = seed_sink(n_img, K, cfg, d.seed_cap, ws + d.off_seed_ws);
            rc = cifhr_sparse_launch(h, n_img, K, cfg, hr_base, (float *)(ws + d.off_hr_aux),
                                     hr_masks, ws + d.off_cifhr_ws, d.cifhr_ws_bytes, s,
                                     "pp_decode_batch(cifhr)", fused_seeds ? &sink : nullptr);
        }
        if (rc) return rc;
    }
    // CifSeeds and CafScored both read only the fields and the CifHr map: with both stages
    // requested, CafScored runs on a side stream beside the seeds (fork / join events)
    // PP_STAGE_COMPLETE_SETS_EARLY: the force-complete sets (every field and direction) with
    // CafScored instead of gated after the seed loop
    const bool early_b = (stages & PP_STAGE_COMPLETE_SETS_EARLY) && (stages & 4u) &&
                         !(stages & 1u) && cfg->force_complete;
    const SideStream *side = (stages & 6u) == 6u ? side_stream() : nullptr;
    if (side) {
        std::lock_guard<std::mutex> lock(side->mu);
        if (hipEventRecord(side->fork, s) != hipSuccess ||
            hipStreamWaitEvent(side->stream, side->fork, 0) != hipSuccess)
            return fail(PP_EHIP, "pp_decode_batch: side-stream fork failed");
        rc = launch_caf_bucketed(h, hr, n_img, K, C, skeleton, cfg, cfg->caf_threshold, cols[0],
                                 offs[0], nullptr, false, side->stream);
        if (!rc && early_b)
            rc = launch_caf_bucketed(h, hr, n_img, K, C, skeleton, cfg,
                                     cfg->complete_caf_threshold, cols[1], offs[1], nullptr, true,
                                     side->stream);
        if (!rc)
            rc = launch_seeds(h, hr, n_img, K, cfg, seeds, d.seed_cap, seed_counts,
                              ws + d.off_seed_ws, s, fused_seeds);
        // join even after a failed launch, so the caller's stream never runs ahead
        if (hipEventRecord(side->join, side->stream) != hipSuccess ||
            hipStreamWaitEvent(s, side->join, 0) != hipSuccess)
            return fail(PP_EHIP, "pp_decode_batch: side-stream join failed");
        if (rc) return rc;
    } else {
        if (stages & 2u) {
            rc = launch_seeds(h, hr, n_img, K, cfg, seeds, d.seed_cap, seed_counts,
                              ws + d.off_seed_ws, s, fused_seeds);
            if (rc) return rc;
        }
        if (stages & 4u) {  // CafScored at caf_threshold; the force-complete set is lazy
            rc = launch_caf_bucketed(h, hr, n_img, K, C, skeleton, cfg, cfg->caf_threshold,
                                     cols[0], offs[0], nullptr, false, s);
            if (!rc && early_b)
                rc = launch_caf_bucketed(h, hr, n_img, K, C, skeleton, cfg,
                                         cfg->complete_caf_threshold, cols[1], offs[1], nullptr,
                                         true, s);
            if (rc) return rc;
        }
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
        g.hh = d.hh;
        g.ww = d.ww;
        g.col_cap = d.hw;
        g.cfg = *cfg;
        g.nms_it = (double)cfg->nms_instance_threshold;
        g.heads = h;
        g.hr = hr;
        g.cif_floor = cfg->cif_floor;
        g.one_minus_floor = (float)(1.0 - (double)cfg->cif_floor);  // (1.0 - self.cif_floor)
        g.th_b = cfg->complete_caf_threshold;
        for (int ci = 0; ci < C; ci++) {
            g.caf_j1[ci] = (uint8_t)(skeleton[2 * ci] - 1);
            g.caf_j2[ci] = (uint8_t)(skeleton[2 * ci + 1] - 1);
        }
        // by_source (cifcaf.py:62-65): dict insertion order, later duplicate keys
        // overwrite the value in place; flattened into directed-edge slots per start joint
        {
            int nbs[kKP] = {0};
            int bk[kKP][kKP], bc[kKP][kKP], bf[kKP][kKP];
            for (int ci = 0; ci < C; ci++) {
                const int j1 = skeleton[2 * ci] - 1, j2 = skeleton[2 * ci + 1] - 1;
                const int ins[2][3] = {{j1, j2, 1}, {j2, j1, 0}};
                for (int t = 0; t < 2; t++) {
                    const int st = ins[t][0];
                    int pos = -1;
                    for (int e = 0; e < nbs[st]; e++)
                        if (bk[st][e] == ins[t][1]) pos = e;
                    if (pos < 0) pos = nbs[st]++;
                    bk[st][pos] = ins[t][1];
                    bc[st][pos] = ci;
                    bf[st][pos] = ins[t][2];
                }
            }
            int d = 0;
            for (int j = 0; j < K; j++) {
                g.j_off[j] = (uint8_t)d;
                for (int e = 0; e < nbs[j]; e++, d++) {
                    g.d_j[d] = (uint8_t)j;
                    g.d_k[d] = (uint8_t)bk[j][e];
                    g.d_caf[d] = (uint8_t)bc[j][e];
                    g.d_fwd[d] = (uint8_t)bf[j][e];
                }
            }
            g.j_off[K] = (uint8_t)d;
            g.nd = d;
            g.has_cs = cfg->confidence_scales != nullptr;
            for (int e = 0; e < kSlots; e++)
                g.slot_cs[e] = (g.has_cs && e < d) ? cfg->confidence_scales[g.d_caf[e]] : 1.0f;
        }
        g.occ = (uint8_t *)(ws + d.off_occ);
        g.occ_cap = d.occ_cap;
        g.log = (OccLog *)(ws + d.off_log);
        g.log_cap = d.log_cap;
        g.work = (pp_ann *)(ws + d.off_work);
        g.spec = (pp_ann *)(ws + d.off_spec);
        g.spec_far = kSpecFar;
        g.n_ext = seed_ext_per_image(n_img);
        g.xext = (SeedExt *)(ws + d.off_xext);
        g.xrec = (pp_ann *)(ws + d.off_xrec);
        g.nms_score = (double *)(ws + d.off_nms_score);
        g.nms_idx = (int *)(ws + d.off_nms_idx);
        g.nms_f = (float *)(ws + d.off_nms_f);
        g.nms_box = (int2 *)(ws + d.off_nms_box);
        g.ann_np = d.ann_np;
        g.ann_cap = ann_capacity;
        g.stamps = nullptr;
#ifdef PP_STAMPS
        hipMalloc((void **)&g.stamps, (size_t)n_img * 3 * kStampSlots * sizeof(uint64_t));
        hipMemsetAsync(g.stamps, 0, (size_t)n_img * 3 * kStampSlots * sizeof(uint64_t), s);
        uint64_t *gcs = nullptr;
        hipMalloc((void **)&gcs, (size_t)n_img * 4 * sizeof(uint64_t));
        hipMemsetAsync(gcs, 0, (size_t)n_img * 4 * sizeof(uint64_t), s);
        hipMemcpyToSymbolAsync(HIP_SYMBOL(g_gc_stamps), &gcs, sizeof(gcs), 0,
                               hipMemcpyHostToDevice, s);
#endif
        g.n_work = (int *)(ws + d.off_n_work);
        g.need_complete = (int *)(ws + d.off_need);
        g.complete_next = (int *)(ws + d.off_wq);
        g.init = init.anns;
        g.init_counts = init.counts;
        g.init_cap = init.cap;
        g.out_idx = init.out_index;
        g.out = d_anns;
        g.counts = d_counts;
        g.status = d_status;
        // PP_STAGE_SEED_LOOP_ONLY / PP_STAGE_AFTER_SEED_LOOP split stage 8 in two calls
        const bool run_rest = !(stages & PP_STAGE_SEED_LOOP_ONLY);
        if (!(stages & PP_STAGE_AFTER_SEED_LOOP)) {
            // g.xext is zero: the workspace's zero region, which every external-helper seed
            // loop leaves zero (ext_exit)
            const size_t dyn = g.n_ext > 0 ? kExtDynLds : kColLds * sizeof(float);
            // confidence_scales: their own kernel instances (the default ones carry no
            // registers for them: complete_kernel stays at 128 VGPRs, 4 waves per SIMD)
            const dim3 blk(64 * kSeedWaves);
            if (g.n_ext > 0) {
                const dim3 grid(n_img * (1 + g.n_ext));
                if (g.has_cs)
                    hipLaunchKernelGGL(seed_loop_ext_kernel<true>, grid, blk, dyn, s, g);
                else
                    hipLaunchKernelGGL(seed_loop_ext_kernel<false>, grid, blk, dyn, s, g);
            } else if (g.has_cs) {
                hipLaunchKernelGGL(seed_loop_kernel<true>, dim3(n_img), blk, dyn, s, g);
            } else {
                hipLaunchKernelGGL(seed_loop_kernel<false>, dim3(n_img), blk, dyn, s, g);
            }
            rc = check_launch("pp_decode_batch(seed loop)");
            if (rc) return rc;
        }
        // PP_STAGE_COMPLETE_ONLY / PP_STAGE_NMS_ONLY split the rest once more
        const bool run_complete = run_rest && !(stages & PP_STAGE_NMS_ONLY);
        const bool run_nms = run_rest && !(stages & PP_STAGE_COMPLETE_ONLY);
        if (run_complete && cfg->force_complete && !(stages & PP_STAGE_COMPLETE_SETS_EARLY)) {
            // complete_annotations' CafScored(score_th=0.0001) only where phase 1 left work
            rc = launch_caf_bucketed(h, hr, n_img, K, C, skeleton, cfg, cfg->complete_caf_threshold,
                                     cols[1], offs[1], g.need_complete, true, s);
            if (rc) return rc;
        }
        if (run_complete && cfg->force_complete) {
            const dim3 grid(n_img, complete_ways(stages));
            if (g.has_cs)
                hipLaunchKernelGGL(complete_kernel<true>, grid, dim3(64), 0, s, g);
            else
                hipLaunchKernelGGL(complete_kernel<false>, grid, dim3(64), 0, s, g);
            rc = check_launch("pp_decode_batch(force complete)");
            if (rc) return rc;
        }
        if (run_nms)
            rc = launch_nms(g, n_img, (stages & PP_STAGE_NMS_WIDE) && g.n_ext == 0,
                            (stages & PP_STAGE_NMS_BITMAP) != 0, s);
#ifdef PP_STAMPS
        hipStreamSynchronize(s);
        const size_t nst = (size_t)n_img * 3 * kStampSlots;
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
        uint64_t *hg = (uint64_t *)malloc((size_t)n_img * 4 * sizeof(uint64_t));
        hipMemcpy(hg, gcs, (size_t)n_img * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost);
        double a0 = 0, a1 = 0, a2 = 0;
        for (int i = 0; i < n_img; i++) {
            a0 += hg[4 * i];
            a1 += hg[4 * i + 1];
            a2 += hg[4 * i + 2];
        }
        fprintf(stderr, "grow_connection sections per image: offsets+scan-setup %.0f  columns %.0f  merge %.0f\n",
                a0 / n_img, a1 / n_img, a2 / n_img);
        free(hg);
        hipFree(gcs);
#endif
    }
    return rc;
}

}  // namespace pp

extern "C" {

int pp_decode_stages(const float *d_cif, const float *d_caf, int32_t n_img, int32_t K, int32_t C,
                     int32_t H, int32_t W, const int32_t *skeleton, const pp_config *cfg,
                     float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                     int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                     uint32_t stages, void *stream) {
    if (!d_cif || !d_caf || !cfg) return fail(PP_EINVAL, "pp_decode_batch: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_decode_batch: bad shape");
    return decode_heads(single_head(d_cif, d_caf, H, W, cfg->stride), n_img, K, C, skeleton, cfg,
                        d_cifhr, d_anns, ann_capacity, d_counts, d_status, d_workspace,
                        workspace_bytes, stages, stream);
}

int pp_decode_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                    int32_t K, int32_t C, const int32_t *skeleton, const pp_config *cfg,
                    float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                    int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                    uint32_t stages, void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, cif_pairs, 3, &h, "pp_decode_multi");
    if (rc) return rc;
    return decode_heads(h, n_img, K, C, skeleton, cfg, d_cifhr, d_anns, ann_capacity, d_counts,
                        d_status, d_workspace, workspace_bytes, stages, stream);
}

int pp_decode_initial(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                      int32_t K, int32_t C, const int32_t *skeleton, const pp_config *cfg,
                      float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                      int32_t *d_status, const pp_ann *d_initial, const int32_t *d_initial_counts,
                      int32_t initial_capacity, int32_t *d_out_index, void *d_workspace,
                      size_t workspace_bytes, uint32_t stages, void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, cif_pairs, 3, &h, "pp_decode_initial");
    if (rc) return rc;
    if ((d_initial == nullptr) != (d_initial_counts == nullptr))
        return fail(PP_EINVAL, "pp_decode_initial: d_initial and d_initial_counts go together");
    if (d_initial && initial_capacity <= 0)
        return fail(PP_ESHAPE, "pp_decode_initial: bad initial_capacity");
    DecodeInit init;
    init.anns = d_initial;
    init.counts = d_initial_counts;
    init.cap = d_initial ? initial_capacity : 0;
    init.out_index = d_out_index;
    return decode_heads(h, n_img, K, C, skeleton, cfg, d_cifhr, d_anns, ann_capacity, d_counts,
                        d_status, d_workspace, workspace_bytes, stages, stream, init);
}

// ---- standalone nms.Keypoints.annotations (nms.py:17-57) over caller records ----------
namespace {
struct NmsLayout {
    size_t off_status, off_wq, off_score, off_idx, off_f, off_box, total;
    int ann_np;
};
NmsLayout nms_layout(int n_img, int cap) {
    NmsLayout l{};
    l.ann_np = 1;
    while (l.ann_np < cap) l.ann_np <<= 1;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += align_up(bytes);
        return at;
    };
    const size_t n = (size_t)n_img;
    l.off_status = take(n * sizeof(int));
    l.off_wq = take(n * sizeof(int));
    l.off_score = take(n * 2 * cap * sizeof(double));
    l.off_idx = take(n * (4 * (size_t)cap + l.ann_np) * sizeof(int));
    l.off_f = take(n * 2 * cap * sizeof(float));
    l.off_box = take(n * kNmsWaves * (size_t)cap * sizeof(int2));
    l.total = o;
    return l;
}
}  // namespace

size_t pp_nms_workspace_size(int32_t n_img, int32_t ann_capacity) {
    if (n_img < 0 || ann_capacity <= 0) return 0;
    return nms_layout(n_img, ann_capacity).total;
}

int pp_nms_keypoints(pp_ann *d_anns, const int32_t *d_counts, int32_t n_img, int32_t K,
                     int32_t ann_capacity, const pp_config *cfg, pp_ann *d_out,
                     int32_t *d_out_counts, int32_t *d_out_index, void *d_workspace,
                     size_t workspace_bytes, void *stream) {
    if (!cfg) return fail(PP_EINVAL, "pp_nms_keypoints: NULL argument");
    return pp_nms_keypoints_scored(d_anns, d_counts, n_img, K, ann_capacity, cfg,
                                   (double)cfg->nms_instance_threshold, nullptr, nullptr,
                                   nullptr, d_out, d_out_counts, d_out_index, d_workspace,
                                   workspace_bytes, stream);
}

int pp_nms_keypoints_scored(pp_ann *d_anns, const int32_t *d_counts, int32_t n_img, int32_t K,
                            int32_t ann_capacity, const pp_config *cfg,
                            double instance_threshold, const int32_t *d_score_spec, const double *d_score_weights,
                            const double *d_fixed_score, pp_ann *d_out, int32_t *d_out_counts,
                            int32_t *d_out_index, void *d_workspace, size_t workspace_bytes,
                            void *stream) {
    if (!d_anns || !d_counts || !cfg || !d_out || !d_out_counts || !d_workspace)
        return fail(PP_EINVAL, "pp_nms_keypoints: NULL argument");
    if (d_score_spec && (!d_score_weights || !d_fixed_score))
        return fail(PP_EINVAL, "pp_nms_keypoints_scored: d_score_spec needs the weights and "
                               "fixed scores");
    if (n_img < 0 || K <= 0 || K > PP_MAX_KP || ann_capacity <= 0 || cfg->occupancy_reduction <= 0)
        return fail(PP_ESHAPE, "pp_nms_keypoints: shape outside the supported envelope");
    if (n_img == 0) return PP_OK;
    const NmsLayout l = nms_layout(n_img, ann_capacity);
    if (workspace_bytes < l.total) return fail(PP_ENOMEM, "pp_nms_keypoints: workspace too small");
    char *ws = (char *)d_workspace;
    hipStream_t s = (hipStream_t)stream;
    GrowArgs g{};
    g.K = K;
    g.cfg = *cfg;
    g.cfg.apply_nms = 1;
    g.work = d_anns;
    g.n_work = const_cast<int *>(d_counts);
    g.ann_cap = ann_capacity;
    g.ann_np = l.ann_np;
    g.status = (int *)(ws + l.off_status);
    g.complete_next = (int *)(ws + l.off_wq);
    g.nms_score = (double *)(ws + l.off_score);
    g.nms_idx = (int *)(ws + l.off_idx);
    g.nms_f = (float *)(ws + l.off_f);
    g.nms_box = (int2 *)(ws + l.off_box);
    g.nms_spec = d_score_spec;
    g.nms_sw = d_score_weights;
    g.nms_fixed = d_fixed_score;
    g.nms_it = instance_threshold;
    g.out = d_out;
    g.counts = d_out_counts;
    g.out_idx = d_out_index;
    if (hipMemsetAsync(g.status, 0, (size_t)n_img * sizeof(int), s) != hipSuccess)
        return fail(PP_EHIP, "pp_nms_keypoints: memset failed");
    hipLaunchKernelGGL(nms_kernel<kNmsWaves>, dim3(n_img), dim3(64 * kNmsWaves), 0, s, g);
    return check_launch("pp_nms_keypoints");
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
                                                             int exp_mode, float *out) {
    float r[4];
    grow_connection_flat<MAXM>(cf, n, pitch, x, y, xy_scale, exp_mode, r);
    if (threadIdx.x < 4) out[threadIdx.x] = r[threadIdx.x];
}
}  // namespace pp

extern "C" int pp_grow_connection(const float *d_cols, int64_t n, int64_t pitch, float x, float y,
                                  float xy_scale, int32_t method, float *d_out, void *stream) {
    if (!d_cols || !d_out) return fail(PP_EINVAL, "pp_grow_connection: NULL argument");
    if (n < 0 || pitch < n || n > INT32_MAX) return fail(PP_ESHAPE, "pp_grow_connection: bad shape");
    // bit 0: connection method (0 blend, 1 max); bit 1: pp_config.exp_mode 1 (correctly
    // rounded np.exp instead of NumPy's SIMD one)
    if (method < 0 || method > 3) return fail(PP_EINVAL, "connection method not known");
    hipStream_t s = (hipStream_t)stream;
    const int exp_mode = (method >> 1) & 1;
    if (method & 1)
        hipLaunchKernelGGL(grow_connection_kernel<true>, dim3(1), dim3(64), 0, s, d_cols, (int)n,
                           pitch, x, y, xy_scale, exp_mode, d_out);
    else
        hipLaunchKernelGGL(grow_connection_kernel<false>, dim3(1), dim3(64), 0, s, d_cols, (int)n,
                           pitch, x, y, xy_scale, exp_mode, d_out);
    return check_launch("pp_grow_connection");
}

