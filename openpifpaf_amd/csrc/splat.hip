// splat.hip — CifHr accumulation and the square-splat primitives of functional.pyx on gfx950.
//
// Reference semantics: splats are folded into each pixel in
// ascending splat order with a clamp after every add (functional.pyx:140-141), so float
// atomics cannot be bit-exact.  The kernels here are a deterministic GATHER:
//
//   cifhr_splats_kernel  one workgroup per (image, CIF field): order-preserving ballot
//                        compaction of the cells with c > v_threshold (cif_hr.py:27) into
//                        splat records {box, cx, cy, v, sigma^2} (cif_hr.py:31-40).
//   splat_tile_kernel    one workgroup per 64x64 output tile: gathers the splats whose box
//                        intersects the tile into LDS (ballot compaction keeps splat
//                        order), then every lane folds its 16 pixels over the candidate
//                        list in ascending order in registers, and the tile is written
//                        ONCE (fused zero-fill) with 16-B stores staged through LDS.
//
// Workgroups of one field run on one XCD (xcd_remap) so the field's splat list is served
// from that XCD's L2.  Template MODE selects the functional.pyx primitive.
#include "pp_common.hpp"

#include <stdlib.h>

#include <algorithm>

// cifhr_fused_kernel<SEEDS>'s last-workgroup hand-off relies on gfx9's store accounting
// (stores count under vmcnt); this library is built for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "splat.hip: device code assumes gfx950 (see cifhr_fused_kernel's completion counter)"
#endif

#ifdef PP_STAMPS
#include <stdio.h>

#include <vector>
#endif

namespace pp {

struct Splat {
    int4 box;    // minx, maxx, miny, maxy (functional.pyx:122-125 bounds, end-exclusive)
    float4 par;  // cx, cy, v, sigma^2   (CUMAVG: cx, cy, v, w)
};

enum SplatMode { M_GAUSS_MAX = 0, M_GAUSS = 1, M_MAXG = 2, M_CONST = 3, M_CUMAVG = 4 };

constexpr int kTile = 64;     // output tile edge (pixels)
constexpr int kSpCand = 64;   // CifHr candidates per wave pass (lane = candidate)
constexpr int kCand = 512;    // LDS candidate capacity per pass (>= 256 for progress)
constexpr int kOutPad = 72;   // LDS staging row pitch (conflict-free ds_write_b32 columns)

// Box of one splat.  ext = truncate*sigma (gauss modes) or width (const / cumavg).
template <int MODE>
__device__ __forceinline__ int4 splat_box(float cx, float cy, float ext, int h, int w) {
    int4 b;
    b.x = (int)clip_ref(cx - ext, 0.0f, (float)(w - 1));
    float hx = cx + ext;
    if (MODE == M_GAUSS_MAX) hx = hx + 1.0f;  // functional.pyx:123 `... + 1`
    b.y = (int)clip_ref(hx, (float)(b.x + 1), (float)w);
    b.z = (int)clip_ref(cy - ext, 0.0f, (float)(h - 1));
    float hy = cy + ext;
    if (MODE == M_GAUSS_MAX) hy = hy + 1.0f;
    b.w = (int)clip_ref(hy, (float)(b.z + 1), (float)h);
    return b;
}

// -------------------------------------------------------------------------------------
// Block fold (both CifHr kernels): lanes own the 64 pixels of an 8x8 block and fold them
// over the block's candidates in ascending splat order, in registers.  Per candidate the
// constant parts of the pixel test are prepared once (FoldCand):
//   - the box test is one packed 16-bit clamp of the lane's (x, y) key against the box
//     corners (v_pk_max_i16 / v_pk_min_i16) and a compare;
//   - the "closest pixel" branch (functional.pyx:132) is a key compare against the one
//     pixel with dx^2 < 0.25 and dy^2 < 0.25 (found per candidate with the same float ops);
//   - approx_exp's range test is dropped: a folded pixel has sum <= sigma^2, so
//     q in [-0.5, 0] (NaN keeps NaN either way);
//   - sigma^2's reciprocal is refined once (recip_of) instead of per pixel;
//   - blocks the circle misses entirely (distance from the center to the block's nearest
//     pixel > sigma * (1 + 2^-19), checked in f64) get no fold at all.
// Candidates are folded two at a time: both terms are independent of the accumulator, only
// the two updates are ordered.  All of this keeps per-(block, candidate) instructions low:
// the fold is issue-bound (rocprof: SQ_INSTS_VALU + SQ_INSTS_SALU per pair).
// -------------------------------------------------------------------------------------
struct FoldCand {  // 32 B in LDS
    float cx, cy, v, s2;
    float r;        // recip_of(s2).r (div_refined); the slow path divides
    uint32_t lo;    // box corner (x0, y0) as packed 16-bit (x | y << 16)
    uint32_t hi;    // box corner (x1 - 1, y1 - 1), end-inclusive
    uint32_t nkey;  // nearest pixel key (dx^2 < 0.25 and dy^2 < 0.25), ~0u: none
};

// the integer coordinate k with fl(fl(k - c)^2) < 0.25 (at most one exists), or -1
__device__ __forceinline__ int nearest_coord(float c) {
    if (!(fabsf(c) < 0x1p24f)) return -1;
    const int k = (int)floorf(c);
    for (int d = 0; d <= 1; d++) {
        const float dd = (float)(k + d) - c;
        if (dd * dd < 0.25f) return k + d;
    }
    return -1;
}

__device__ __forceinline__ uint32_t pix_key(int x, int y) {
    return (uint32_t)(x & 0xffff) | ((uint32_t)y << 16);
}

// candidates the fast fold cannot take exactly: div_refined outside its domain or a box
// the circle does not cover (make_cand sets r = 0 for both), or a non-finite v (v * 0 would
// not vanish for the pixels the fast term excludes)
__device__ __forceinline__ bool cand_slow(const FoldCand &c) {
    return !(c.r > 0.0f) || !(__builtin_fabsf(c.v) < __builtin_inff());
}

// Lanes whose pixel lies outside the map fold at these coordinates: dx^2 = 2^120 fails every
// fast candidate's circle test (s2 <= 2^100), and the key matches no candidate's nearest
// pixel (nkey is a pixel of the map, or ~0u).
constexpr float kOffMapCoord = 0x1p60f;
constexpr uint32_t kOffMapKey = 0xFFFFFFFEu;

typedef short pp_short2 __attribute__((ext_vector_type(2)));

// box: clamp the packed (x, y) key into [lo, hi] per 16-bit half; unchanged = inside
__device__ __forceinline__ bool in_box(const FoldCand &c, uint32_t key) {
    const pp_short2 k2 = __builtin_bit_cast(pp_short2, key);
    const pp_short2 cl = __builtin_elementwise_min(
        __builtin_elementwise_max(k2, __builtin_bit_cast(pp_short2, c.lo)),
        __builtin_bit_cast(pp_short2, c.hi));
    return __builtin_bit_cast(uint32_t, cl) == key;
}

// The fast fold has no box test (functional.pyx:122-129 bounds): the circle test alone
// excludes every pixel outside the box when the first pixel past each of the box's four
// edges fails it on its own axis, RN(d^2) > s2 with d = k - c.  Further out |d| only grows
// (rounding is monotone), and the fold's sum = RN(RN(dx^2) + RN(dy^2)) >= RN(dx^2).  The
// box ends at most a rounding error inside the circle's reach on the low side (x0 =
// trunc(cx - sigma)) and within one pixel on the high side (x1 = trunc(cx + sigma + 1)),
// so this fails only when an edge sits a few ulps from the circle; such candidates, and
// non-finite or huge centers, keep the box test on the slow path.  Pixels past the map's
// edge never fold (kOffMapCoord).
__device__ __forceinline__ bool box_in_circle(int4 b, float cx, float cy, float s2, int hh, int ww) {
    if (!(__builtin_fabsf(cx) < 0x1p20f && __builtin_fabsf(cy) < 0x1p20f)) return false;
    const auto out = [s2](int k, float c) {
        const float d = (float)k - c;
        return d * d > s2;
    };
    if (b.x > 0 && !out(b.x - 1, cx)) return false;
    if (b.y < ww && !out(b.y, cx)) return false;
    if (b.z > 0 && !out(b.z - 1, cy)) return false;
    if (b.w < hh && !out(b.w, cy)) return false;
    return true;
}

__device__ __forceinline__ FoldCand make_cand(int4 b, float4 p, int hh, int ww) {
    FoldCand c;
    c.cx = p.x;
    c.cy = p.y;
    c.v = p.z;
    c.s2 = p.w;
    c.r = (recip_ok(p.w) && box_in_circle(b, p.x, p.y, p.w, hh, ww)) ? recip_of(p.w).r : 0.0f;
    c.lo = pix_key(b.x, b.z);
    c.hi = pix_key(b.y - 1, b.w - 1);
    const int nx = nearest_coord(p.x), ny = nearest_coord(p.y);
    c.nkey = (nx < 0 || ny < 0) ? ~0u : pix_key(nx, ny);
    // the fast fold applies q = 0 after the box test: keep nkey only inside the box (the
    // box is clipped to the map, the nearest pixel may lie past its edge)
    if (c.nkey != ~0u && !in_box(c, c.nkey)) c.nkey = ~0u;
    return c;
}

// 8x8 blocks of the 64x64 tile at (tx0, ty0) (bit 8 * by + bx) that candidate c's box
// touches and its circle reaches.  Box corners unpack from the keys.
__device__ __forceinline__ uint64_t cand_live(const FoldCand &c, int tx0, int ty0) {
    const int x0 = (int)(c.lo & 0xffff), y0 = (int)(c.lo >> 16);
    const int x1 = (int)(c.hi & 0xffff) + 1, y1 = (int)(c.hi >> 16) + 1;
    if (x1 <= tx0 || x0 >= tx0 + kTile || y1 <= ty0 || y0 >= ty0 + kTile) return 0ull;
    const int bxa = max(x0 - tx0, 0) >> 3, bxb = (min(x1 - tx0, kTile) - 1) >> 3;
    const int bya = max(y0 - ty0, 0) >> 3, byb = (min(y1 - ty0, kTile) - 1) >> 3;
    const double cx = c.cx, cy = c.cy;
    const double thr = (double)c.s2 * (1.0 + 0x1p-19);  // NaN: never culled
    uint64_t live = 0ull;
    for (int by = bya; by <= byb; by++) {
        const int Y0 = ty0 + 8 * by;
        const double qy = fmin(fmax(cy, (double)Y0), (double)(Y0 + 7)) - cy;
        for (int bx = bxa; bx <= bxb; bx++) {
            const int X0 = tx0 + 8 * bx;
            const double qx = fmin(fmax(cx, (double)X0), (double)(X0 + 7)) - cx;
            if (!(qx * qx + qy * qy > thr)) live |= 1ull << (8 * by + bx);
        }
    }
    return live;
}


// fold_pixel<M_GAUSS_MAX> (truncate 1, max_value 1; functional.pyx:127-141): the term one
// candidate adds to this lane's pixel (vv) and whether the pixel takes it (slow path)
struct FoldTerm {
    float vv;
    bool take;
};

__device__ __forceinline__ FoldTerm fold_term_slow(const FoldCand &c, float fx, float fy,
                                                   uint32_t key) {
    const float dx = fx - c.cx, dy = fy - c.cy;
    const float dx2 = dx * dx, dy2 = dy * dy;  // powf(d, 2.0)
    const float sum = dx2 + dy2;
    // approx_exp(-0.5 * sum / s2) starts with 1 + x / 8: x = (-0.5 * sum) / s2 is
    // -0.5 * (sum / s2) exactly (scaling by a power of two commutes with rounding; where
    // sum / s2 is subnormal both give 1 + x / 8 = 1), so the -0.5 / 8 goes into the fma
    float q = sum / c.s2;
    q = (key == c.nkey) ? 0.0f : q;  // "closest pixel": q = 0 gives t = 1, v * t = v
    float t = __builtin_fmaf(q, -0.0625f, 1.0f);  // 1 + x / 8 (q * -0.0625 is exact)
    t = t * t;
    t = t * t;
    t = t * t;
    FoldTerm f;
    f.vv = c.v * t;
    f.take = !(sum > c.s2) & in_box(c, key);
    return f;
}

__device__ __forceinline__ float fold_apply(float acc, const FoldTerm &f) {
    const float a = acc + f.vv;
    return f.take ? ((a < 1.0f) ? a : 1.0f) : acc;  // min(max_value, f)
}

// The fast term (s2 in div_refined's domain, v finite, the box inside the circle's reach:
// make_cand): a pixel outside the circle gets q = 16, so t = (1 - 16 / 16)^8 = 0 and
// vv = v * 0 = +0, and the update min(acc + vv, 1) leaves it as it was (acc in [0, 1]).
// The closest pixel lies inside (sum < 0.5 <= sigma^2, sigma >= 1), so its q = 0 is applied
// last.  Every pixel then takes the same update, with the tests as selects on q (vector
// compares + cndmask: no scalar mask arithmetic).
__device__ __forceinline__ float fold_vv(const FoldCand &c, float fx, float fy, uint32_t key) {
    const float dx = fx - c.cx, dy = fy - c.cy;
    const float sum = dx * dx + dy * dy;
    float q = div_refined(sum, Recip{c.s2, c.r});
    q = (sum > c.s2) ? 16.0f : q;
    q = (key == c.nkey) ? 0.0f : q;
    float t = __builtin_fmaf(q, -0.0625f, 1.0f);
    t = t * t;
    t = t * t;
    t = t * t;
    return c.v * t;
}

__device__ __forceinline__ float fold_add(float acc, float vv) {
    return __builtin_fminf(acc + vv, 1.0f);  // (a < 1) ? a : 1; a NaN gives 1 either way
}

// Folds the candidates `q` (bits, ascending) of a candidate array into this lane's pixel:
// two at a time on the fast path, one at a time when the set holds a slow one.  `get(c)`
// returns candidate c (a FoldCand array, or an index list into the field's LDS list).
template <typename Get>
__device__ __forceinline__ float fold_block_g(float acc, Get get, uint64_t q, uint64_t slow,
                                              float fx, float fy, uint32_t key) {
    if (q & slow) {
        for (; q; q &= q - 1) {
            const int c = __builtin_ctzll(q);
            if ((slow >> c) & 1ull)
                acc = fold_apply(acc, fold_term_slow(get(c), fx, fy, key));
            else
                acc = fold_add(acc, fold_vv(get(c), fx, fy, key));
        }
        return acc;
    }
    // a counted loop over the pairs, the odd one after it: one scalar branch per pair
    const int np = __popcll(q);
    for (int i = 1; i < np; i += 2) {
        const int c1 = __builtin_ctzll(q);
        q &= ~(1ull << c1);
        const int c2 = __builtin_ctzll(q);
        q &= ~(1ull << c2);
        const float v1 = fold_vv(get(c1), fx, fy, key);
        const float v2 = fold_vv(get(c2), fx, fy, key);
        acc = fold_add(fold_add(acc, v1), v2);
    }
    if (np & 1) acc = fold_add(acc, fold_vv(get(__builtin_ctzll(q)), fx, fy, key));
    return acc;
}

__device__ __forceinline__ float fold_block(float acc, const FoldCand *cand, uint64_t q,
                                            uint64_t slow, float fx, float fy, uint32_t key) {
    return fold_block_g(acc, [cand](int c) -> const FoldCand & { return cand[c]; }, q, slow, fx,
                        fy, key);
}

// wave-wide OR of a 64-bit value through one LDS word
__device__ __forceinline__ uint64_t wave_or64(uint64_t v, uint64_t *s_slot) {
    if (lane_id() == 0) *s_slot = 0ull;
    wave_sync();
    if (v) atomicOr((unsigned long long *)s_slot, (unsigned long long)v);
    wave_sync();
    const uint64_t r = *s_slot;
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32);
}

// Row bins of a candidate list: bin r gets, in list order, every entry whose box rows meet
// tile row r (rows [64 r, 64 r + 64)), for maps of at most kMaxBinRows tile rows.  A counting
// sweep (LDS atomics per row, plus each row's first / last list index) sizes the bins,
// which are laid out back to back in `bins` (capacity bins_cap entries); then one block
// compaction per (row, 256 entries) over only that row's index range fills them in order.
// rowcnt[r] / rowoff[r] (LDS or global) = entries and offset of row r; rowcnt[r] = -1 for
// every row when the bins would exceed bins_cap (consumers then scan the whole list).
// Ends with a barrier.
constexpr int kMaxBinRows = 32;
constexpr int kBinMin = 512;  // shorter lists are scanned whole (binning would cost more)

__host__ __device__ inline int64_t bins_capacity(int64_t cells) { return cells + cells / 2 + 2048; }

struct RowBinLds {
    int cnt[kMaxBinRows], first[kMaxBinRows], last[kMaxBinRows], off[kMaxBinRows + 1];
    int tmp[4];
};

__device__ void hr_row_bins(const FoldCand *list, int total, FoldCand *bins, int64_t bins_cap,
                            int tiles_y, RowBinLds &L, int *rowcnt, int *rowoff) {
    if (threadIdx.x < kMaxBinRows) {
        L.cnt[threadIdx.x] = 0;
        L.first[threadIdx.x] = INT32_MAX;
        L.last[threadIdx.x] = -1;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += 256) {
        const FoldCand c = list[i];
        const int ra = (int)(c.lo >> 16) >> 6, rb = (int)(c.hi >> 16) >> 6;
        for (int r = ra; r <= rb && r < tiles_y; r++) {
            atomicAdd(&L.cnt[r], 1);
            atomicMin(&L.first[r], i);
            atomicMax(&L.last[r], i);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int o = 0;
        for (int r = 0; r < tiles_y; r++) {
            L.off[r] = o;
            o += L.cnt[r];
        }
        L.off[tiles_y] = o;
    }
    __syncthreads();
    const bool fits = L.off[tiles_y] <= bins_cap;
    if (threadIdx.x < tiles_y) {
        rowcnt[threadIdx.x] = fits ? L.cnt[threadIdx.x] : -1;
        rowoff[threadIdx.x] = L.off[threadIdx.x];
    }
    if (!fits) {
        __syncthreads();
        return;
    }
    for (int r = 0; r < tiles_y; r++) {
        if (L.cnt[r] == 0) continue;  // block-uniform
        FoldCand *bin = bins + L.off[r];
        const uint32_t lo_y = (uint32_t)(r * kTile), hi_y = lo_y + kTile;
        int running = 0;
        for (int base = L.first[r]; base <= L.last[r]; base += 256) {
            const int i = base + (int)threadIdx.x;
            FoldCand c;
            bool hit = false;
            if (i <= L.last[r]) {
                c = list[i];
                hit = (c.lo >> 16) < hi_y && (c.hi >> 16) >= lo_y;  // box rows y0 .. y1 - 1
            }
            int tot;
            const int slot = block_compact<4>(hit, L.tmp, tot);
            if (hit) bin[running + slot] = c;
            running += tot;
        }
    }
    __syncthreads();
}

// -------------------------------------------------------------------------------------
// K1: CIF cells -> splat records (cif_hr.py:26-40)
// -------------------------------------------------------------------------------------
constexpr int kTileBits = 1024;  // per-field tile bitmap capacity (32x32 tiles of 64x64 px)

// DET: CifDetHr.accumulate (cif_hr.py:84-100) on 7-channel fields [c, x, y, b, w, h, b2],
// min-scale masks on w and h, sigma = max(1, 0.1 * min(w, h) * stride); else CifHr
// (cif_hr.py:26-40), 5 channels.
//
// One workgroup per (image, field, CifHr group).  A group's members (cif_hr.py:42-57
// fill_multiple: one head, or heads g and g + n/2 with pairs) are compacted one after the
// other into one list, in the reference's accumulation order, at the group head's stride
// and min scale with v / neighbors / len_cifs.
struct HrSplatArgs {
    Heads h;
    int K, hh, ww;
    float v_th, neighbors;
    FoldCand *list;       // (n_img * K, list_cap); group g's list at goff[g]
    int64_t list_cap;     // cells of all heads
    int64_t goff[kMaxHeads];
    int *counts;          // (n_img * K, n_groups)
    uint32_t *tile_bits;  // (n_img * K, n_groups, kTileBits / 32)
    FoldCand *bins;       // (n_img * K, n_groups, bins_cap): the list per tile row (hr_row_bins)
    int *rowcnt, *rowoff; // (n_img * K, n_groups, kMaxBinRows): bin sizes (-1: none), offsets
    int64_t bins_cap;     // 0: no bins (maps of more than kMaxBinRows tile rows)
    int tiles_x, tiles, tiles_y;
};

template <bool DET>
__global__ __launch_bounds__(256) void cifhr_splats_kernel(HrSplatArgs a) {
    __shared__ int s_tmp[4];
    __shared__ RowBinLds s_rb;
    __shared__ uint32_t s_bits[kTileBits / 32];
    const bool use_bits = a.tiles <= kTileBits;
    if (threadIdx.x < kTileBits / 32) s_bits[threadIdx.x] = 0u;
    __syncthreads();
    const int ng = a.h.n_groups;
    const int64_t fld = blockIdx.x / ng;  // image * K + field
    const int g = (int)(blockIdx.x % ng);
    const float stride = (float)a.h.cstride[g];
    const bool ms_on = (a.h.ms_on >> g) & 1u;
    const float ms_th = a.h.ms_th[g];
    const float len_cifs = (float)a.h.group_size();
    FoldCand *out = a.list + fld * a.list_cap + a.goff[g];
    int running = 0;
    for (int i = 0; i < a.h.group_size(); i++) {
        const int m = a.h.member(g, i);
        const int hw = a.h.cH[m] * a.h.cW[m];
        const float *p = a.h.cif[m] + fld * (DET ? 7 : 5) * (int64_t)hw;
        // kU cells per thread per batch (cells base + k * 256 + tid): confidences, then the
        // rows of passing cells, each issued for the whole batch at once
        constexpr int kU = 8;
        for (int base = 0; base < hw; base += 256 * kU) {
            float c[kU], x[kU], y[kU], s4[kU], s5[kU];
#pragma unroll
            for (int k = 0; k < kU; k++) {
                const int cell = base + k * 256 + (int)threadIdx.x;
                c[k] = cell < hw ? p[cell] : NAN;  // NaN: never > v_th
                x[k] = y[k] = s4[k] = s5[k] = 0.0f;
            }
#pragma unroll
            for (int k = 0; k < kU; k++) {
                const int cell = base + k * 256 + (int)threadIdx.x;
                if (c[k] > a.v_th) {
                    x[k] = p[hw + cell];
                    y[k] = p[2 * hw + cell];
                    s4[k] = p[4 * hw + cell];
                    if (DET) s5[k] = p[5 * hw + cell];
                }
            }
#pragma unroll
            for (int k = 0; k < kU; k++) {
                bool keep = c[k] > a.v_th;
                if (keep && ms_on)  // p[4] (and for detections p[5]) > min_scale / stride
                    keep = DET ? (s4[k] > ms_th && s5[k] > ms_th) : s4[k] > ms_th;
                int total;
                const int slot = block_compact<4>(keep, s_tmp, total);
                if (keep) {
                    const float cx = x[k] * stride;
                    const float cy = y[k] * stride;
                    float sg;
                    if (DET) {  // np.minimum / np.maximum propagate NaN
                        const float w = s4[k], h = s5[k];
                        const float mn = (w != w) ? w : ((h != h) ? h : (h < w ? h : w));
                        sg = (0.1f * mn) * stride;
                    } else {
                        sg = (0.5f * s4[k]) * stride;
                    }
                    const float sigma = (sg != sg) ? sg : fmaxf(1.0f, sg);  // np.maximum keeps NaN
                    const float v = (c[k] / a.neighbors) / len_cifs;        // v / neighbors / len_cifs
                    const int4 box = splat_box<M_GAUSS_MAX>(cx, cy, 1.0f * sigma, a.hh, a.ww);
                    out[running + slot] = make_cand(box, make_float4(cx, cy, v, sigma * sigma), a.hh, a.ww);
                    if (use_bits) {  // mark the 64x64 output tiles this splat's box touches
                        for (int ty = box.z / kTile; ty <= (box.w - 1) / kTile; ty++)
                            for (int tx = box.x / kTile; tx <= (box.y - 1) / kTile; tx++) {
                                const int t = ty * a.tiles_x + tx;
                                atomicOr(&s_bits[t >> 5], 1u << (t & 31));
                            }
                    }
                }
                running += total;
            }
        }
    }
    if (threadIdx.x == 0) a.counts[blockIdx.x] = running;
    __syncthreads();
    if (threadIdx.x < kTileBits / 32)
        a.tile_bits[(int64_t)blockIdx.x * (kTileBits / 32) + threadIdx.x] =
            use_bits ? s_bits[threadIdx.x] : ~0u;
    // the list by tile row for the tile kernel (blockIdx.x = (image * K + field) * groups + g)
    if (a.bins_cap > 0 && running > kBinMin)
        hr_row_bins(out, running, a.bins + (int64_t)blockIdx.x * a.bins_cap, a.bins_cap,
                    a.tiles_y, s_rb, a.rowcnt + (int64_t)blockIdx.x * kMaxBinRows,
                    a.rowoff + (int64_t)blockIdx.x * kMaxBinRows);
}

// -------------------------------------------------------------------------------------
// primitive prep: point lists -> splat records (functional.pyx argument order, no filter)
// -------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void prep_splats_kernel(const float *__restrict__ x,
                                                          const float *__restrict__ y,
                                                          const float *__restrict__ s,
                                                          const float *__restrict__ v,
                                                          const float *__restrict__ wt,
                                                          int64_t n, int h, int w, float truncate,
                                                          Splat *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float cx = x[i], cy = y[i], sv = s[i];
    Splat r;
    if (MODE == M_CONST || MODE == M_CUMAVG) {
        r.box = splat_box<MODE>(cx, cy, sv, h, w);
        float cw = (MODE == M_CUMAVG) ? wt[i] : 0.0f;
        if (MODE == M_CUMAVG && cw <= 0.0f) r.box = make_int4(0, 0, 0, 0);  // `continue`
        r.par = make_float4(cx, cy, v[i], cw);
    } else {
        r.box = splat_box<MODE>(cx, cy, truncate * sv, h, w);
        r.par = make_float4(cx, cy, v[i], sv * sv);
    }
    out[i] = r;
}

// -------------------------------------------------------------------------------------
// K2: tile gather-fold
// -------------------------------------------------------------------------------------
struct TileArgs {
    float *field;           // (n_fields, h, pitch), fields back to back
    float *field2;          // cumw for M_CUMAVG
    const Splat *splats;    // n_fields * splat_cap
    int64_t splat_cap;
    int64_t n_splats;
    int64_t field_stride;   // elements between fields
    int h, w, pitch;
    int tiles_x, tiles;     // tiles per field
    int64_t n_work;         // n_fields * tiles
    float t2;               // truncate^2 (M_GAUSS_MAX circle test)
    float max_value;
};

template <int MODE>
__device__ __forceinline__ void fold_pixel(float &acc, float &acc2, bool in, float px, float py,
                                           const float4 &par, float t2s2, float maxv) {
    if (MODE == M_CONST) {
        if (in) acc = acc + par.z;
        return;
    }
    if (MODE == M_CUMAVG) {
        if (in) {
            const float cw = par.w, cv = par.z;
            acc = (cw * cv + acc2 * acc) / (acc2 + cw);  // functional.pyx:53 (cdivision)
            acc2 = acc2 + cw;
        }
        return;
    }
    const float dx = px - par.x, dy = py - par.y;
    const float dx2 = dx * dx, dy2 = dy * dy;  // powf(d, 2.0)
    const float sum = dx2 + dy2;
    if (MODE == M_GAUSS_MAX) in = in && !(sum > t2s2);
    if (!in) return;
    float vv;
    if (MODE != M_MAXG && dx2 < 0.25f && dy2 < 0.25f)
        vv = par.z;  // "closest pixel"
    else
        vv = par.z * approx_exp_ref((-0.5f * sum) / par.w);
    if (MODE == M_GAUSS_MAX) {
        acc = acc + vv;
        acc = (acc < maxv) ? acc : maxv;  // min(max_value, f) as emitted by Cython
    } else if (MODE == M_GAUSS) {
        acc = acc + vv;
    } else {
        acc = fmaxf(acc, vv);  // (float)fmax((double)f, (double)vv)
    }
}

// The functional.pyx primitives in place on one field: one workgroup per 64x64 tile reads
// the tile, folds the candidate splats in ascending order and writes it back.
template <int MODE>
__global__ __launch_bounds__(256) void splat_tile_kernel(TileArgs a) {
    __shared__ int4 s_box[kCand];
    __shared__ float4 s_par[kCand];
    __shared__ int s_tmp[4];

    const int64_t wid = xcd_remap(blockIdx.x, gridDim.x);
    if (wid >= a.n_work) return;
    const int tile = (int)(wid % a.tiles);
    const int64_t fld = wid / a.tiles;
    const int tx0 = (tile % a.tiles_x) * kTile;
    const int ty0 = (tile / a.tiles_x) * kTile;
    const Splat *sp = a.splats + fld * a.splat_cap;
    const int64_t ns = a.n_splats;
    float *out = a.field + fld * a.field_stride;
    float *out2 = (MODE == M_CUMAVG) ? a.field2 + fld * a.field_stride : nullptr;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int lx = lane & 7, ly = lane >> 3;
    const int wx0 = tx0, wy0 = ty0 + wave * 16;

    float acc[16], acc2[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        acc[r] = 0.0f;
        acc2[r] = 0.0f;
        const int px = wx0 + (r & 7) * 8 + lx, py = wy0 + (r >> 3) * 8 + ly;
        if (px < a.w && py < a.h) {
            acc[r] = out[(int64_t)py * a.pitch + px];
            if (MODE == M_CUMAVG) acc2[r] = out2[(int64_t)py * a.pitch + px];
        }
    }

    int64_t cursor = 0;
    while (cursor < ns) {
        // ---- gather: splats intersecting this tile, in splat order, into LDS ----
        int n = 0;
        while (cursor < ns) {
            const int64_t i = cursor + threadIdx.x;
            bool hit = false;
            int4 b = make_int4(0, 0, 0, 0);
            if (i < ns) {
                b = sp[i].box;
                hit = b.y > tx0 && b.x < tx0 + kTile && b.w > ty0 && b.z < ty0 + kTile;
            }
            int total;
            const int slot = block_compact<4>(hit, s_tmp, total);
            if (n + total > kCand) break;  // block-uniform; chunk re-read next pass
            if (hit) {
                s_box[n + slot] = b;
                s_par[n + slot] = sp[i].par;
            }
            n += total;
            cursor += 256;
        }
        __syncthreads();
        // ---- fold: per pixel, ascending candidate order ----
        for (int c = 0; c < n; c++) {
            const int bx0 = __builtin_amdgcn_readfirstlane(s_box[c].x);
            const int bx1 = __builtin_amdgcn_readfirstlane(s_box[c].y);
            const int by0 = __builtin_amdgcn_readfirstlane(s_box[c].z);
            const int by1 = __builtin_amdgcn_readfirstlane(s_box[c].w);
            if (bx1 <= wx0 || bx0 >= wx0 + kTile || by1 <= wy0 || by0 >= wy0 + 16) continue;
            const float4 par = s_par[c];
            const float t2s2 = a.t2 * par.w;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int rx0 = wx0 + (r & 7) * 8, ry0 = wy0 + (r >> 3) * 8;
                if (bx1 <= rx0 || bx0 >= rx0 + 8 || by1 <= ry0 || by0 >= ry0 + 8) continue;
                const int px = rx0 + lx, py = ry0 + ly;
                const bool in = px >= bx0 && px < bx1 && py >= by0 && py < by1;
                fold_pixel<MODE>(acc[r], acc2[r], in, (float)px, (float)py, par, t2s2,
                                 a.max_value);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int px = wx0 + (r & 7) * 8 + lx, py = wy0 + (r >> 3) * 8 + ly;
        if (px < a.w && py < a.h) {
            out[(int64_t)py * a.pitch + px] = acc[r];
            if (MODE == M_CUMAVG) out2[(int64_t)py * a.pitch + px] = acc2[r];
        }
    }
}

// -------------------------------------------------------------------------------------
// K2 for CifHr: one workgroup per (field, chunk of kChunkTiles tiles within one bitmap word)
// -------------------------------------------------------------------------------------
// The field's tile bitmap says which tiles any splat box touches.  Untouched tiles cost a
// zero-fill (one tile per workgroup streams best: many short workgroups keep every CU's
// store queue full, and a touched tile's fold delays no zero-fill).  In a touched tile each
// wave owns 16 rows (16 of the tile's 8x8 blocks): it gathers the candidates of its stripe
// from the tile row's bin (the splats kernel's hr_row_bins; the whole list when the bin
// overflowed) in passes of kSpCand, folds its blocks with fold_block into a private LDS
// stripe, and writes the stripe with 16-B nontemporal stores.  Waves never wait for each
// other.
//
// MULTI (CifHr over several groups, cif_hr.py:59-73): each group's list folds into a zero
// stripe and the groups combine by np.maximum(ta, accumulated) in registers.  A group
// with no splat on the stripe contributes max(0, acc) = acc (every fold value is >= 0 and
// the clamp maps NaN to max_value), so it is skipped.
constexpr int kChunkTiles = 1;  // tiles per workgroup: 1.209 ms vs 1.409 ms at 32 (cfg3)
constexpr int kHrPad = 68;    // stripe row pitch (floats)
// units per touched tile of a split field (small batches): 4 = a 16-row stripe (8, one block
// row each, measured slower: cfg2 uniform CifHr kernel 76.7 vs 69.6 us, planted equal)
constexpr int kSplitParts = 4;
static_assert(kSplitParts == 4 || kSplitParts == 8, "unit masks are written as u16 / u8 parts");

struct HrTileArgs {
    float *field;           // dense (n_fields, h, pitch)
    const FoldCand *list;   // field fld's group g list at list + fld * splat_cap + goff[g]
    const int *counts;      // (n_fields, n_groups)
    const uint32_t *tile_bits;  // (n_fields, n_groups, kTileBits / 32)
    const FoldCand *bins;   // (n_fields, n_groups, bins_cap)
    const int *rowcnt, *rowoff;  // (n_fields, n_groups, kMaxBinRows), rowcnt -1: scan the list
    int64_t bins_cap;       // 0: no bins
    int64_t splat_cap;
    int64_t field_stride;
    int h, w, pitch;
    int tiles_x, tiles, chunks;  // chunks per field
    int chunk_tiles;        // tiles per chunk: a power of two <= 32 (chunks never straddle a bitmap word)
    int64_t n_work;         // n_fields * chunks
    int n_groups;
    int64_t goff[kMaxHeads];
};

template <bool MULTI>
__global__ __launch_bounds__(256) void cifhr_tile_kernel(HrTileArgs a) {
    __shared__ FoldCand s_cand[4][kSpCand];
    __shared__ __attribute__((aligned(16))) float s_out[kTile * kHrPad];
    __shared__ uint64_t s_live[4];

    const int64_t wid = xcd_remap(blockIdx.x, gridDim.x);
    if (wid >= a.n_work) return;
    const int chunk = (int)(wid % a.chunks);
    const int64_t fld = wid / a.chunks;
    const int t0 = chunk * a.chunk_tiles, t1 = min(a.tiles, t0 + a.chunk_tiles);
    const int ng = MULTI ? a.n_groups : 1;

    // touched tiles of the chunk over all groups: one round trip of scalar loads (a list's
    // bitmap is all zero when the list is empty)
    uint32_t live = 0;
    for (int g = 0; g < ng; g++)
        live |= a.tile_bits[(fld * ng + g) * (kTileBits / 32) + (t0 >> 5)] >> (t0 & 31);
    live &= (t1 - t0 == 32) ? ~0u : ((1u << (t1 - t0)) - 1u);
    float *out = a.field + fld * a.field_stride;
    typedef float v4f __attribute__((ext_vector_type(4)));
    {  // untouched tiles are zero-filled, 16-B nontemporal stores
        const v4f z = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int t = t0; t < t1; t++) {
            if ((live >> (t - t0)) & 1u) continue;
            const int tx0 = (t % a.tiles_x) * kTile, ty0 = (t / a.tiles_x) * kTile;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int q = k * 256 + threadIdx.x;
                const int gy = ty0 + (q >> 4), gx = tx0 + (q & 15) * 4;
                if (gy < a.h && gx < a.pitch)
                    __builtin_nontemporal_store(z, reinterpret_cast<v4f *>(&out[(int64_t)gy * a.pitch + gx]));
            }
        }
    }
    if (!live) return;

    // touched tiles: wave w owns the tile's rows [16 w, 16 w + 16) = its blocks 16 w .. 16 w + 15
    // (block b = 8 * by + bx), folds them from its own candidate passes in a private LDS
    // stripe and writes the stripe; the waves never wait for each other
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int lx = lane & 7, ly = lane >> 3;
    float *s_acc = s_out + wave * 16 * kHrPad;  // this wave's 64 x 16 stripe
    FoldCand *cand = s_cand[wave];
    for (uint32_t rest = live; rest; rest &= rest - 1) {
        const int tile = t0 + __builtin_ctz(rest);
        const int tx0 = (tile % a.tiles_x) * kTile;
        const int ty0 = (tile / a.tiles_x) * kTile;
        const int row = tile / a.tiles_x;
        const int wy0 = ty0 + wave * 16;  // stripe rows [wy0, wy0 + 16)
        float res[MULTI ? 16 : 1];
#pragma unroll
        for (int r = 0; r < (MULTI ? 16 : 1); r++) res[r] = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; r++) s_acc[(r >> 3) * 8 * kHrPad + ly * kHrPad + (r & 7) * 8 + lx] = 0.0f;
        for (int g = 0; g < ng; g++) {
            const int64_t lst = fld * ng + g;
            const int ns = a.counts[lst];
            if (ns == 0 || !((a.tile_bits[lst * (kTileBits / 32) + (tile >> 5)] >> (tile & 31)) & 1u)) continue;
            if (MULTI && g > 0) {  // each group folds from zero (cif_hr.py:59-62)
                wave_sync();
#pragma unroll
                for (int r = 0; r < 16; r++) s_acc[(r >> 3) * 8 * kHrPad + ly * kHrPad + (r & 7) * 8 + lx] = 0.0f;
            }
            const int rc = (a.bins_cap > 0 && ns > kBinMin) ? a.rowcnt[lst * kMaxBinRows + row] : -1;
            const FoldCand *src = rc >= 0 ? a.bins + lst * a.bins_cap + a.rowoff[lst * kMaxBinRows + row]
                                          : a.list + fld * a.splat_cap + (MULTI ? a.goff[g] : 0);
            const int src_n = rc >= 0 ? rc : ns;
            bool hit_any = false;
            int cursor = 0;
            while (true) {
                // ---- the stripe's candidates in list order ----
                int n = 0;
                while (cursor < src_n) {
                    const int e = cursor + lane;
                    bool hit = false;
                    FoldCand c;
                    if (e < src_n) {
                        c = src[e];
                        const int x0 = (int)(c.lo & 0xffff), x1 = (int)(c.hi & 0xffff) + 1;
                        const int y0 = (int)(c.lo >> 16), y1 = (int)(c.hi >> 16) + 1;
                        hit = x1 > tx0 && x0 < tx0 + kTile && y1 > wy0 && y0 < wy0 + 16;
                    }
                    const uint64_t mk = __ballot(hit);
                    const int cnt = __popcll(mk);
                    if (n + cnt > kSpCand) break;  // wave-uniform; chunk re-read next pass
                    if (hit) cand[n + lane_prefix(mk)] = c;
                    n += cnt;
                    cursor += 64;
                }
                const bool last = cursor >= src_n;
                hit_any = hit_any || n > 0;
                wave_sync();
                // ---- lane = candidate: its blocks among the wave's 16 ----
                uint64_t cl = 0ull;
                bool slow_l = false;
                if (lane < n) {
                    cl = (cand_live(cand[lane], tx0, ty0) >> (16 * wave)) & 0xFFFFull;
                    slow_l = cand_slow(cand[lane]);
                }
                const uint64_t slow = __ballot(slow_l);
                const uint64_t lv = wave_or64(cl, &s_live[wave]);
                for (uint64_t bl = lv; bl; bl &= bl - 1) {
                    const int b = __builtin_ctzll(bl);
                    const int bx = b & 7, byl = b >> 3;
                    const int px = tx0 + 8 * bx + lx, py = wy0 + 8 * byl + ly;
                    const bool on = px < a.w && py < a.h;
                    float *cell = &s_acc[(byl * 8 + ly) * kHrPad + bx * 8 + lx];
                    *cell = fold_block(*cell, cand, __ballot((cl >> b) & 1ull), slow,
                                       on ? (float)px : kOffMapCoord, on ? (float)py : kOffMapCoord,
                                       on ? pix_key(px, py) : kOffMapKey);
                }
                if (last) break;
                wave_sync();  // the candidate array is rewritten by the next pass
            }
            if (MULTI) {
                wave_sync();
                if (hit_any) {
#pragma unroll
                    for (int r = 0; r < 16; r++) {  // np.maximum(ta, accumulated)
                        const float acc = s_acc[(r >> 3) * 8 * kHrPad + ly * kHrPad + (r & 7) * 8 + lx];
                        res[r] = (acc != acc || res[r] != res[r]) ? NAN : (acc > res[r] ? acc : res[r]);
                    }
                }
            }
        }
        if (MULTI) {
            wave_sync();
#pragma unroll
            for (int r = 0; r < 16; r++) s_acc[(r >> 3) * 8 * kHrPad + ly * kHrPad + (r & 7) * 8 + lx] = res[r];
        }
        wave_sync();
        // ---- write the wave's stripe: 16 rows x 64 floats, 16-B nontemporal stores ----
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int q = k * 64 + lane;  // float4 index in the stripe
            const int row16 = q >> 4, c4 = (q & 15) * 4;
            const v4f v = *reinterpret_cast<const v4f *>(&s_acc[row16 * kHrPad + c4]);
            const int gy = wy0 + row16, gx = tx0 + c4;
            if (gy < a.h && gx < a.pitch)
                __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(&out[(int64_t)gy * a.pitch + gx]));
        }
        wave_sync();  // the stripe is reused by the next tile
    }
}

// -------------------------------------------------------------------------------------
// The decoder's CifHr: block-sparse map (HrMap with masks), one workgroup per field
// -------------------------------------------------------------------------------------
// Phase 1 compacts the field's splats (every group, cif_hr.py:26-40, 55-57) in the
// reference's order into the field's global list of fold candidates (FoldCand): each
// thread loads kSpU cells per round, one barrier per round orders the (cell batch, wave)
// counts; a bitmap marks the 64x64 tiles the boxes touch.  Single-scale fields then bin the
// list by tile row (row r: the entries whose box meets rows [64 r, 64 r + 64), in list
// order, one block compaction per 256 entries), so a tile scans only its row's entries
// instead of the whole list (a bin that would overflow its capacity falls back to the list).
//
// Phase 2: the four waves take the touched tiles round robin, each on its own (no
// barriers).  Per tile a wave gathers the intersecting candidates in order (ballot
// compaction, kSpCand per pass), lane c computes the 8x8 blocks candidate c reaches, and
// for every block with candidates the 64 lanes fold their pixel over the block's
// candidates in ascending order in registers (fold_block) and store the block's 256
// contiguous bytes.  Blocks no splat box touches are never written: the
// tile's u64 mask says which blocks hold data, and HrMap::at reads the rest as 0.
// A tile with more than kSpCand candidates takes several passes; a block touched again
// reloads its fold state from the map (each lane reads back only the pixel it wrote).
//
// MULTI (cif_hr.py:59-73): groups fold into zero separately and combine by np.maximum;
// candidates carry their group, and a change of group closes the running fold into res.
// Across passes res stays in the map and the open group's fold in `aux`.
constexpr int kSpU = 32;      // cells per thread per compaction round (confidences in flight)
constexpr int kSplitSlots = 1024;  // small batches: workgroups per field = kSplitSlots / fields
constexpr int kMaxSplit = 64;
constexpr int kSpStage = 1024; // kept cells of a round staged in LDS (phase 2's s_cand space)

struct HrSparseArgs {
    Heads h;
    int hh, ww;
    float v_th, neighbors;
    FoldCand *list;   // (n_img * K, list_cap): each field's splats in the reference's order
    int64_t list_cap;
    FoldCand *bins;   // single-scale: (n_img * K, bins_cap) the list by tile row (hr_row_bins)
    int64_t bins_cap; // 0: no bins (multi-scale, or maps of more than kMaxBinRows tile rows)
    float *map;       // (n_img * K, tiles, 64 blocks, 64 px)
    float *aux;       // MULTI: open-group folds between passes, same shape as map
    uint64_t *masks;  // (n_img * K, tiles) written blocks
    int tiles_x, tiles, tiles_y;
    int split;        // workgroups per field (small batches): each folds every split-th
                      // touched tile of the field
    int split_list;   // prebuilt lists: a field uses ceil(list length / split_list) of its
                      // split workgroups (at most split), the others return at once
    // split > 1: the field's list, bins and tile bits are built once by
    // cifhr_list_kernel (prebuilt; NULL: every split workgroup builds its own copy)
    int *pre_total;         // (n_img * K) list lengths
    uint32_t *pre_bits;     // (n_img * K, kTileBits / 32) touched tiles
    int *pre_rowcnt;        // (n_img * K, kMaxBinRows) bin sizes (-1: none), offsets
    int *pre_rowoff;
    SeedSink seeds;         // cifhr_fused_kernel<true> / cifhr_list_kernel<true>: where the
                            // field's seeds go
    int *done;              // split fields with seeds: (n_img * K) workgroups finished
};

// a generic pointer as a global-address-space one (agent-scope atomics as global_ ops)
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T *as_global(T *p) {
    return (__attribute__((address_space(1))) T *)p;
}

__device__ __forceinline__ float nan_max(float a, float b) {  // np.maximum
    return (a != a || b != b) ? NAN : (a > b ? a : b);
}

#ifdef PP_STAMPS
// diagnostic build: per workgroup [start, phase 1 done, wave 0..3 done, hw_id, xcc_id, splats]
// in s_memrealtime ticks (100 MHz), dumped to $PP_HR_STAMPS_OUT by cifhr_sparse_launch
__device__ uint64_t *g_hr_stamps;
// per workgroup: [start, phase 1 done, end of waves 0-3, hw id, xcc id, list length,
// wave 0's shader cycles staging candidates, folding, its units]
constexpr int kHrSt = 12;
#define HR_ADD(slot, v)                                                                     \
    do {                                                                                    \
        if (g_hr_stamps && wave == 0 && lane == 0) g_hr_stamps[blockIdx.x * kHrSt + (slot)] += (v); \
    } while (0)
#define HR_STAMP(slot)                                                                      \
    do {                                                                                    \
        if (g_hr_stamps && lane == 0)                                                       \
            g_hr_stamps[blockIdx.x * kHrSt + (slot)] = __builtin_amdgcn_s_memrealtime();        \
    } while (0)
#else
#define HR_ADD(slot, v) \
    do {                \
    } while (0)
#define HR_STAMP(slot) \
    do {               \
    } while (0)
#endif

// Phase 3 of the seed emission (cif_seeds.py:35-47) for field `fld`, whose n_seed
// candidates (c, x, y, s; c > threshold, in cell order) are in the sink's segment: v =
// 0.9 * CifHr(x, y) + 0.1 * c from the finished block-sparse map, the seeds with v above
// the threshold compacted in place, in order; their count into f_counts.  Block-uniform.
__device__ void seeds_from_map(const HrSparseArgs &a, int64_t fld, int n_seed, int *s_tmp) {
    const SeedSink &ss = a.seeds;
    const int hw = a.h.cH[0] * a.h.cW[0];
    const int f = (int)(fld % ss.K);
    const int64_t img = fld / ss.K;
    float *sv = ss.g_keys + img * 4 * ss.cap + (int64_t)f * hw;
    float *sx = sv + ss.cap, *sy = sx + ss.cap, *sz = sy + ss.cap;
    HrMap hm{};
    hm.base = a.map;
    hm.masks = a.masks;
    hm.hh = a.hh;
    hm.ww = a.ww;
    hm.tiles_x = a.tiles_x;
    hm.tiles = a.tiles;
    int kept = 0;
    int *sf = ss.g_f + img * ss.cap + (int64_t)f * hw;
    // kSeedPer candidates per thread in flight (candidate e0 + 256 k + t), then one
    // compaction per k in candidate order
    constexpr int kSeedPer = 8;
    for (int e0 = 0; e0 < n_seed; e0 += 256 * kSeedPer) {  // block-uniform
        float v[kSeedPer], x[kSeedPer], y[kSeedPer], sc[kSeedPer];
        bool ok[kSeedPer];
#pragma unroll
        for (int k = 0; k < kSeedPer; k++) {
            const int e = e0 + 256 * k + (int)threadIdx.x;
            ok[k] = false;
            v[k] = x[k] = y[k] = sc[k] = 0.0f;
            if (e < n_seed) {
                const float c = sv[e];
                x[k] = sx[e];
                y[k] = sy[e];
                sc[k] = sz[e];
                const float hv = hm.at(fld, x[k], y[k], 0.0f);
                float vv = 0.9f * hv + 0.1f * c;  // 0.9 * v + 0.1 * c
                if (ss.score_scale != 1.0f) vv = vv * ss.score_scale;
                v[k] = vv;
                ok[k] = vv > ss.th;
            }
        }
        // every candidate of this pass is in registers before the first write below
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSeedPer; k++) {
            if (e0 + 256 * k >= n_seed) break;  // block-uniform
            int tot;
            const int slot = block_compact<4>(ok[k], s_tmp, tot);
            if (ok[k]) {
                const int pos = kept + slot;  // <= its candidate index: earlier slots only
                sv[pos] = v[k];
                sx[pos] = x[k];
                sy[pos] = y[k];
                sz[pos] = sc[k];
                sf[pos] = f;
            }
            kept += tot;
        }
    }
    if (threadIdx.x == 0) ss.f_counts[fld] = kept;
}

// Phase 1 of the CifHr kernel: the field's splat list in the reference's order (every
// group, cif_hr.py:26-40, 55-57) as fold candidates in the field's global list.  A round
// covers 256 * kSpU cells: each thread loads its kSpU confidences at once (plus the scale
// of the cells above threshold when a min scale applies), one barrier orders the (cell
// batch, wave) counts, and the kept cells are staged in LDS (`stage`: kSpStage cell
// indices) in list order; then one thread per staged cell reads its x, y, scale and writes
// its candidate.  So a round costs about three memory round trips however many cells it
// keeps (a round keeping more than kSpStage reads them per batch instead).  s_bits marks
// the 64x64 tiles the boxes touch (cleared by the caller before the first barrier).
// Returns the list length; s_gbeg[g] = start of group g's entries.  Ends with a barrier.
// SEEDS (one CIF head, one group): also the field's seed candidates (c > seed threshold,
// cif_seeds.py:28-33) into a.seeds' segment in cell order, their count into f_counts[fld]
// (seeds_from_map finishes them); s_tmp: 4 ints of LDS.
template <bool MULTI, bool SEEDS = false, int STAGE = kSpStage>
__device__ int hr_splat_list(const HrSparseArgs &a, int64_t fld, int64_t slot, uint32_t *s_bits,
                             int (*s_cnt)[kSpU][4], int *s_gbeg, int *stage,
                             int *s_tmp = nullptr) {
    static_assert(!(MULTI && SEEDS), "seed candidates of one CIF head only");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ng = MULTI ? a.h.n_groups : 1;
    FoldCand *glist = a.list + slot * a.list_cap;  // this workgroup's own copy
    int running = 0, buf = 0;
    const SeedSink &ss = a.seeds;
    const int sfield = SEEDS ? (int)(fld % ss.K) : 0;
    const bool seeding = SEEDS && !((ss.skip >> sfield) & 1u);
    const int shw = a.h.cH[0] * a.h.cW[0];
    float *sv = SEEDS ? ss.g_keys + (fld / (SEEDS ? ss.K : 1)) * 4 * ss.cap + (int64_t)sfield * shw
                      : nullptr;
    int n_seed = 0;
    // block-uniform: one seed-candidate compaction over the threads' (flag, cell)
    auto seed_cand = [&](bool cand, const float *p, int hw, int cell, float c, float stride) {
        if constexpr (SEEDS) {
            int tot;
            const int at = block_compact<4>(cand, s_tmp, tot);
            if (cand) {
                float *q = sv + n_seed + at;
                q[0] = c;
                q[ss.cap] = p[hw + cell] * stride;
                q[2 * ss.cap] = p[2 * hw + cell] * stride;
                q[3 * ss.cap] = p[4 * hw + cell] * stride;
            }
            n_seed += tot;
        }
    };
    for (int g = 0; g < ng; g++) {
        if (threadIdx.x == 0) s_gbeg[g] = running;
        const float stride = (float)a.h.cstride[g];
        const bool ms_on = (a.h.ms_on >> g) & 1u;
        const float ms_th = a.h.ms_th[g];
        const float len_cifs = (float)a.h.group_size();
        // candidate of cell `cell` (c > v_th, scale test passed) at list position pos
        auto emit = [&](const float *p, int hw, int cell, float c, int pos) {
            const float x = p[hw + cell], y = p[2 * hw + cell], s4 = p[4 * hw + cell];
            const float cx = x * stride, cy = y * stride;
            const float sg = (0.5f * s4) * stride;
            const float sigma = (sg != sg) ? sg : fmaxf(1.0f, sg);  // np.maximum keeps NaN
            const float v = (c / a.neighbors) / len_cifs;           // v / neighbors / len_cifs
            const int4 box = splat_box<M_GAUSS_MAX>(cx, cy, 1.0f * sigma, a.hh, a.ww);
            glist[pos] = make_cand(box, make_float4(cx, cy, v, sigma * sigma), a.hh, a.ww);
            for (int ty = box.z / kTile; ty <= (box.w - 1) / kTile; ty++)
                for (int tx = box.x / kTile; tx <= (box.y - 1) / kTile; tx++) {
                    const int t = ty * a.tiles_x + tx;
                    atomicOr(&s_bits[t >> 5], 1u << (t & 31));
                }
        };
        for (int i = 0; i < a.h.group_size(); i++) {
            const int m = a.h.member(g, i);
            const int hw = a.h.cH[m] * a.h.cW[m];
            const float *p = a.h.cif[m] + fld * 5 * (int64_t)hw;
            for (int base = 0; base < hw; base += 256 * kSpU) {
                float c[kSpU];
#pragma unroll
                for (int k = 0; k < kSpU; k++) {
                    const int cell = base + k * 256 + (int)threadIdx.x;
                    c[k] = cell < hw ? p[cell] : NAN;  // NaN: never > v_th
                }
                uint32_t keep = 0;
#pragma unroll
                for (int k = 0; k < kSpU; k++) keep |= (c[k] > a.v_th) ? (1u << k) : 0u;
                if (ms_on) {  // p[4] > min_scale / stride (cif_hr.py:29-30)
                    uint32_t km = keep;
#pragma unroll
                    for (int k = 0; k < kSpU; k++)
                        if ((keep >> k) & 1u) {
                            const int cell = base + k * 256 + (int)threadIdx.x;
                            if (!(p[4 * hw + cell] > ms_th)) km &= ~(1u << k);
                        }
                    keep = km;
                }
#pragma unroll
                for (int k = 0; k < kSpU; k++) {
                    const uint64_t bal = __ballot((keep >> k) & 1u);
                    if (lane == 0) s_cnt[buf][k][wave] = __popcll(bal);
                }
                __syncthreads();  // (also orders the s_bits clear before the first atomicOr)
                int off = 0;
#pragma unroll 4
                for (int k = 0; k < kSpU; k++) {
                    const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[buf][k][0]);
                    off += q.x + q.y + q.z + q.w;
                }
                // list position of batch k's kept cell in this thread (ballot order = cell order)
                auto place = [&](auto fn) {
                    int o = 0;
#pragma unroll 4
                    for (int k = 0; k < kSpU; k++) {
                        const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[buf][k][0]);
                        const uint64_t bal = __ballot((keep >> k) & 1u);
                        if ((keep >> k) & 1u)
                            fn(base + k * 256 + (int)threadIdx.x,
                               o + (wave > 0 ? q.x : 0) + (wave > 1 ? q.y : 0) + (wave > 2 ? q.z : 0) +
                                   lane_prefix(bal));
                        o += q.x + q.y + q.z + q.w;
                    }
                };
                if (off <= STAGE) {
                    place([&](int cell, int pos) { stage[pos] = cell; });
                    __syncthreads();
                    if constexpr (SEEDS) {
                        for (int e0 = 0; e0 < off; e0 += 256) {  // block-uniform
                            const int e = e0 + (int)threadIdx.x;
                            int cell = 0;
                            float c = 0.0f;
                            if (e < off) {
                                cell = stage[e];
                                c = p[cell];
                                emit(p, hw, cell, c, running + e);
                            }
                            seed_cand(seeding && e < off && c > ss.th, p, hw, cell, c, stride);
                        }
                    } else {
                        for (int e = threadIdx.x; e < off; e += 256) {
                            const int cell = stage[e];
                            emit(p, hw, cell, p[cell], running + e);
                        }
                    }
                } else {  // more than the stage holds: batch by batch (not unrolled)
                    int o = 0;
                    for (int k = 0; k < kSpU; k++) {
                        const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[buf][k][0]);
                        const uint64_t bal = __ballot((keep >> k) & 1u);
                        const int cell = base + k * 256 + (int)threadIdx.x;
                        float c = 0.0f;
                        if ((keep >> k) & 1u) {
                            c = p[cell];
                            emit(p, hw, cell, c,
                                 running + o + (wave > 0 ? q.x : 0) + (wave > 1 ? q.y : 0) +
                                     (wave > 2 ? q.z : 0) + lane_prefix(bal));
                        }
                        seed_cand(seeding && ((keep >> k) & 1u) && c > ss.th, p, hw, cell, c, stride);
                        o += q.x + q.y + q.z + q.w;
                    }
                }
                running += off;
                buf ^= 1;
                __syncthreads();  // the stage is rewritten by the next round
            }
        }
    }
    if (threadIdx.x == 0) s_gbeg[ng] = running;
    if (SEEDS && threadIdx.x == 0) ss.f_counts[fld] = n_seed;  // candidates (seeds_from_map)
    __syncthreads();
    return running;
}

// Phase 1 once per field (one CifHr group), into the field's list / bins / tile bits in
// global memory (pre_*): for small batches (split > 1) before cifhr_sparse_kernel, whose
// split workgroups then only fold, and for the dense map (pp_cifhr) before
// cifhr_tile_kernel, in HrSplatArgs' layout (masks NULL).  Untouched tiles of the sparse map
// get their empty block masks here.  8 waves per SIMD (64 VGPRs, as cifhr_sparse_kernel):
// uniform dense map 5.36 -> 5.32 ms per 256 images against 98 VGPRs, planted unchanged.
// SEEDS: the seed candidates too (hr_splat_list), and the field's completion counter of
// cifhr_sparse_kernel<false, true> zeroed (the kernel boundary orders it before that launch).
template <bool SEEDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void cifhr_list_kernel(HrSparseArgs a) {
    __shared__ uint32_t s_bits[kTileBits / 32];
    __shared__ RowBinLds s_rb;
    __shared__ __attribute__((aligned(16))) int s_cnt[2][kSpU][4];
    __shared__ int s_gbeg[kMaxHeads + 1];
    // with seeds a whole round's kept cells (uniform 80x80: ~2800) stay staged: the batch-by-
    // batch path would compact seed candidates once per 256-cell batch
    constexpr int kStage = SEEDS ? 256 * kSpU : kSpStage;
    __shared__ int s_stage[kStage];
    __shared__ int s_tmp[4];
    const int64_t fld = blockIdx.x;
    if (threadIdx.x < kTileBits / 32) s_bits[threadIdx.x] = 0u;
    if (SEEDS && threadIdx.x == 0) a.done[fld] = 0;
    const int total =
        hr_splat_list<false, SEEDS, kStage>(a, fld, fld, s_bits, s_cnt, s_gbeg, s_stage, s_tmp);
    int *rowcnt = a.pre_rowcnt + fld * kMaxBinRows, *rowoff = a.pre_rowoff + fld * kMaxBinRows;
    if (a.bins_cap > 0 && total > kBinMin)
        hr_row_bins(a.list + fld * a.list_cap, total, a.bins + fld * a.bins_cap, a.bins_cap,
                    a.tiles_y, s_rb, rowcnt, rowoff);
    else if (threadIdx.x < kMaxBinRows)
        rowcnt[threadIdx.x] = -1;
    if (threadIdx.x == 0) a.pre_total[fld] = total;
    if (threadIdx.x < kTileBits / 32) a.pre_bits[fld * (kTileBits / 32) + threadIdx.x] = s_bits[threadIdx.x];
    if (a.masks)
        for (int t = threadIdx.x; t < a.tiles; t += 256)  // untouched tiles: no block written
            if (!((s_bits[t >> 5] >> (t & 31)) & 1u)) a.masks[fld * a.tiles + t] = 0ull;
}

// SEEDS (split fields with a prebuilt list and seed candidates, cifhr_list_kernel<true>):
// the field's last workgroup to finish its fold emits the field's seeds (seeds_from_map).
// Completion is the write-through counter form of cdna_hip_programming.md Guideline 16: the
// map's blocks and the units' mask bits are stored sc1 (relaxed agent-scope atomic stores),
// so no release fence is needed; every wave drains its
// stores, the workgroup's barrier, one lane's relaxed agent-scope ticket; the last arriver
// acquires at agent scope, then reads the map with plain loads.  (With a release fence in
// every workgroup instead, cfg2 uniform's fold kernel took 99-110 vs 70 us.)
template <bool MULTI, bool SEEDS = false>
// 8 waves per SIMD (<= 64 VGPRs): the kernel is latency-bound, occupancy hides it
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void cifhr_sparse_kernel(HrSparseArgs a) {
    static_assert(!(MULTI && SEEDS), "seeds of one CIF head only");
    __shared__ uint32_t s_bits[kTileBits / 32];
    __shared__ RowBinLds s_rb;
    __shared__ int s_rowcnt[kMaxBinRows], s_rowoff[kMaxBinRows];  // bins (hr_row_bins)
    __shared__ __attribute__((aligned(16))) int s_cnt[2][kSpU][4];
    __shared__ int s_gbeg[kMaxHeads + 1];
    __shared__ FoldCand s_cand[4][kSpCand];
    __shared__ uint8_t s_cg[4][MULTI ? kSpCand : 1];
    __shared__ int8_t s_bg[4][MULTI ? 64 : 1];
    __shared__ uint64_t s_live[4];
    __shared__ int s_next;

    const int64_t fld = blockIdx.x / a.split;  // image * K + field
    const int part = (int)(blockIdx.x % a.split);
    const bool pre = !MULTI && a.pre_total;
    // list / bins copy of this workgroup (fld * split + part), or the field's prebuilt one
    const int64_t slot = pre ? fld : (int64_t)blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave == 0) HR_STAMP(0);
    if (threadIdx.x == 0) s_next = 0;
    int total;
    bool use_bins;
    int split = a.split;  // workgroups of this field that fold
    if (pre) {
        total = a.pre_total[fld];
        split = min(a.split, max(1, (total + a.split_list - 1) / a.split_list));
        if (part >= split) return;  // block-uniform: this field needs fewer workgroups
        if (threadIdx.x < kTileBits / 32) s_bits[threadIdx.x] = a.pre_bits[fld * (kTileBits / 32) + threadIdx.x];
        if (threadIdx.x < kMaxBinRows) {
            s_rowcnt[threadIdx.x] = a.pre_rowcnt[fld * kMaxBinRows + threadIdx.x];
            s_rowoff[threadIdx.x] = a.pre_rowoff[fld * kMaxBinRows + threadIdx.x];
        }
        use_bins = a.bins_cap > 0 && total > kBinMin;
        __syncthreads();
    } else {
        if (threadIdx.x < kTileBits / 32) s_bits[threadIdx.x] = 0u;
        total = hr_splat_list<MULTI>(a, fld, slot, s_bits, s_cnt, s_gbeg,
                                     reinterpret_cast<int *>(&s_cand[0][0]));
        use_bins = !MULTI && a.bins_cap > 0 && total > kBinMin;
        if (use_bins)
            hr_row_bins(a.list + slot * a.list_cap, total, a.bins + slot * a.bins_cap, a.bins_cap,
                        a.tiles_y, s_rb, s_rowcnt, s_rowoff);
    }
    const int ng = MULTI ? a.h.n_groups : 1;
    const FoldCand *glist = a.list + slot * a.list_cap;
#ifdef PP_STAMPS
    if (wave == 0) {
        HR_STAMP(1);
        if (g_hr_stamps && lane == 0) {
            g_hr_stamps[blockIdx.x * kHrSt + 6] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
            g_hr_stamps[blockIdx.x * kHrSt + 7] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
            g_hr_stamps[blockIdx.x * kHrSt + 8] = total;
        }
    }
#endif
    if (!pre)
        for (int t = threadIdx.x; t < a.tiles; t += 256)  // untouched tiles: no block written
            if (!((s_bits[t >> 5] >> (t & 31)) & 1u)) a.masks[fld * a.tiles + t] = 0ull;

    // ---- phase 2: units of touched tiles, one wave each, claimed from an LDS counter ----
    // A unit is a whole tile, or, for split fields (small batches, one group), a 16-row
    // stripe of one: the four stripes of a busy tile then fold on four waves.  (Stripes for
    // every batch measured slower: each stripe re-scans the tile's candidates; uniform cfg3
    // CifHr 7.6 -> 9.1 ms per overlapped step.)
    const int kParts = (!MULTI && a.split > 1) ? kSplitParts : 1;
    FoldCand *cand = s_cand[wave];
    const int lx = lane & 7, ly = lane >> 3;
    const int nwords = (a.tiles + 31) >> 5;
    int wd = 0, li = 0;  // this wave's walk over the set bits (live index li)
    uint32_t bits = __builtin_amdgcn_readfirstlane(s_bits[0]);
    while (true) {
        int claim = 0;
        if (lane == 0) claim = atomicAdd(&s_next, 1);
        // this workgroup's claim-th unit is the field's (claim * split + part)-th one: stripe
        // unit % kParts of the (unit / kParts)-th touched tile
        const int unit = __builtin_amdgcn_readfirstlane(claim) * split + part;
        const int target = unit / kParts, q = unit % kParts;
        // advance to the target-th touched tile (claims grow, so the walk only moves on)
        int t = -1;
        while (wd < nwords) {
            if (!bits) {
                if (++wd < nwords) bits = __builtin_amdgcn_readfirstlane(s_bits[wd]);
                continue;
            }
            if (li == target) {
                t = wd * 32 + __builtin_ctz(bits);
                break;
            }
            bits &= bits - 1;
            li++;
        }
        if (t < 0) break;
        const int tx0 = (t % a.tiles_x) * kTile, ty0 = (t / a.tiles_x) * kTile;
        const int kRows = kTile / kParts;
        const int wy0 = ty0 + q * kRows;  // the unit's rows [wy0, wy0 + kRows)
        const int kUnitBlocks = 64 / kParts;
        const uint64_t unit_blocks =
            kParts == 1 ? ~0ull : (((1ull << kUnitBlocks) - 1) << (kUnitBlocks * q));
        float *mp = a.map + (fld * a.tiles + t) * (int64_t)(kTile * kTile);
        float *ap = MULTI ? a.aux + (fld * a.tiles + t) * (int64_t)(kTile * kTile) : nullptr;
        uint64_t done = 0;  // blocks written by earlier passes
        // candidates come from the tile row's bin, or from the whole list (MULTI, overflow)
        const int row = t / a.tiles_x;
        const int rc = use_bins ? s_rowcnt[row] : -1;
        const FoldCand *src = rc >= 0 ? a.bins + slot * a.bins_cap + s_rowoff[row] : glist;
        const int src_n = rc >= 0 ? rc : total;
        int cursor = 0;
        HR_ADD(11, 1);
        while (true) {
#ifdef PP_STAMPS
            const uint64_t t_a = __builtin_amdgcn_s_memtime();
#endif
            // ---- this tile's candidates, in list order ----
            int n = 0;
            while (cursor < src_n) {
                const int e = cursor + lane;
                bool hit = false;
                FoldCand c;
                if (e < src_n) {
                    c = src[e];
                    const int x0 = (int)(c.lo & 0xffff), x1 = (int)(c.hi & 0xffff) + 1;
                    const int y0 = (int)(c.lo >> 16), y1 = (int)(c.hi >> 16) + 1;
                    hit = x1 > tx0 && x0 < tx0 + kTile && y1 > wy0 && y0 < wy0 + kRows;
                }
                const uint64_t mk = __ballot(hit);
                const int cnt = __popcll(mk);
                if (n + cnt > kSpCand) break;  // wave-uniform; chunk re-read next pass
                if (hit) {
                    const int pos = n + lane_prefix(mk);
                    cand[pos] = c;
                    if (MULTI) {  // list index e -> group
                        int gg = 0;
                        while (gg + 1 < ng && e >= s_gbeg[gg + 1]) gg++;
                        s_cg[wave][pos] = (uint8_t)gg;
                    }
                }
                n += cnt;
                cursor += 64;
            }
            const bool last = cursor >= src_n;
            wave_sync();
            // ---- lane = candidate: its blocks of the tile ----
            uint64_t cl = 0ull;
            bool slow_l = false;
            if (lane < n) {
                cl = cand_live(cand[lane], tx0, ty0) & unit_blocks;
                slow_l = cand_slow(cand[lane]);
            }
            const uint64_t slow = __ballot(slow_l);
            const uint64_t live = wave_or64(cl, &s_live[wave]);
#ifdef PP_STAMPS
            const uint64_t t_b = __builtin_amdgcn_s_memtime();
            HR_ADD(9, t_b - t_a);
#endif
            // ---- fold: block by block, lane = pixel, candidates ascending ----
            for (uint64_t rest = live; rest; rest &= rest - 1) {
                const int blk = __builtin_ctzll(rest);
                const int px = tx0 + 8 * (blk & 7) + lx, py = ty0 + 8 * (blk >> 3) + ly;
                const bool on = px < a.ww && py < a.hh;
                const float fx = on ? (float)px : kOffMapCoord, fy = on ? (float)py : kOffMapCoord;
                const uint32_t key = on ? pix_key(px, py) : kOffMapKey;
                const uint64_t bq = __ballot((cl >> blk) & 1ull);
                float acc = 0.0f, res = 0.0f;
                int gcur = -1;
                if ((done >> blk) & 1ull) {  // state of an earlier pass (own pixel)
                    if (MULTI) {
                        res = mp[blk * 64 + lane];
                        acc = ap[blk * 64 + lane];
                        gcur = s_bg[wave][blk];
                    } else {
                        acc = mp[blk * 64 + lane];
                    }
                }
                if (!MULTI) {
                    acc = fold_block(acc, cand, bq, slow, fx, fy, key);
                } else {
                    for (uint64_t q = bq; q; q &= q - 1) {
                        const int c = __builtin_ctzll(q);
                        const int gc = s_cg[wave][c];
                        if (gc != gcur) {  // np.maximum(ta, accumulated) per group
                            res = nan_max(acc, res);
                            acc = 0.0f;
                            gcur = gc;
                        }
                        acc = fold_block(acc, cand, 1ull << c, slow, fx, fy, key);
                    }
                }
                // nontemporal: the map is read by later kernels only, and streaming it past
                // L2 keeps the row bins the next tiles scan resident there
                if (!MULTI && SEEDS) {
                    __hip_atomic_store(as_global(&mp[blk * 64 + lane]),
                                       acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (!MULTI) {
                    __builtin_nontemporal_store(acc, &mp[blk * 64 + lane]);
                } else if (last) {
                    __builtin_nontemporal_store(nan_max(acc, res), &mp[blk * 64 + lane]);
                } else {
                    mp[blk * 64 + lane] = res;
                    ap[blk * 64 + lane] = acc;
                    if (lane == 0) s_bg[wave][blk] = (int8_t)gcur;
                }
            }
#ifdef PP_STAMPS
            HR_ADD(10, __builtin_amdgcn_s_memtime() - t_b);
#endif
            done |= live;
            if (last) {
                if (MULTI) {  // blocks of earlier passes the last pass did not touch
                    for (uint64_t rest = done & ~live; rest; rest &= rest - 1) {
                        const int blk = __builtin_ctzll(rest);
                        mp[blk * 64 + lane] = nan_max(ap[blk * 64 + lane], mp[blk * 64 + lane]);
                    }
                }
                break;
            }
            wave_sync();  // candidate arrays are rewritten by the next pass
        }
        if (lane == 0) {
            if (SEEDS && kSplitParts == 4)  // the unit's 16 bits, write-through (sc1)
                __hip_atomic_store(
                    as_global(reinterpret_cast<unsigned short *>(&a.masks[fld * a.tiles + t]) + q),
                    (unsigned short)(done >> (16 * q)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (SEEDS)  // the unit's 8 bits
                __hip_atomic_store(
                    as_global(reinterpret_cast<unsigned char *>(&a.masks[fld * a.tiles + t]) + q),
                    (unsigned char)(done >> (8 * q)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (kParts == 1)
                a.masks[fld * a.tiles + t] = done;
            else if (kSplitParts == 4)  // the unit's 16 bits of the tile's mask
                reinterpret_cast<uint16_t *>(&a.masks[fld * a.tiles + t])[q] = (uint16_t)(done >> (16 * q));
            else  // the unit's 8 bits (one block row)
                reinterpret_cast<uint8_t *>(&a.masks[fld * a.tiles + t])[q] = (uint8_t)(done >> (8 * q));
        }
    }
    HR_STAMP(2 + wave);
    if constexpr (SEEDS) {
        // Completion without a release fence: the blocks and masks above are
        // write-through (sc1 / nontemporal) stores, and on gfx9 stores count under vmcnt, so
        // the s_waitcnt below drains them to L2-coherent memory before the counter's atomic;
        // the last arriver's agent acquire then sees every unit's writes.  An agent release
        // fence would add a buffer_wbl2 of the whole L2 per workgroup on gfx950 (per-XCD
        // L2s).  This holds only where stores count under vmcnt: the guard at the top of this
        // file refuses any other device target.
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's blocks and masks
        __syncthreads();
        if (threadIdx.x == 0) {
            const int old = __hip_atomic_fetch_add(
                as_global(&a.done[fld]), 1,
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == split - 1;
            if (old == split - 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (s_last) {
            int *s_tmp = reinterpret_cast<int *>(&s_cand[0][0]);  // the fold's LDS is free
            seeds_from_map(a, fld, a.seeds.f_counts[fld], s_tmp);
        }
    }
}

// -------------------------------------------------------------------------------------
// The decoder's CifHr for batches whose fields each get one workgroup (one CIF head, one
// group, split 1), with the field's candidate list in LDS and, optionally (SEEDS), the
// field's seeds emitted by the same workgroup (cif_seeds.py:28-47).
//
// Phase 1 is hr_splat_list's (one confidence round per 8192 cells, kept cells staged in
// LDS, then their x / y / scale), but the first kFuList candidates stay in LDS: a field
// with at most kFuList splats (planted input: about 125) never writes or re-reads a list in
// global memory.  Longer lists go to the global list (the LDS part copied after it) and
// take cifhr_sparse_kernel's row bins and per-wave candidate copies, in the same LDS.
// SEEDS: the kept cells with c > seed_threshold (a subset: seed threshold >= CifHr
// threshold) are the seed candidates, in row-major order; their (c, x * stride,
// y * stride, s * stride) go to the field's segment of the seeds scratch in candidate
// order.
//
// Phase 2 as cifhr_sparse_kernel's, whole tiles per wave; with the list in LDS a wave's
// candidates for a tile are indices into it (no copies, no global reads).
//
// Phase 3 (SEEDS), after a barrier (the map's blocks and masks are this workgroup's own
// stores): each candidate looks up the map at its position (scalar_values, HrMap::at),
// v = 0.9 h + 0.1 c (times score_scale), and the ones with v > threshold are compacted in
// order into the same segment, as seeds_emit_kernel writes it; seeds_sort_kernel follows.
// -------------------------------------------------------------------------------------
constexpr int kFuList = 256;   // fold candidates of a field held in LDS
constexpr int kFuStage = 512;  // kept cells of a round staged in LDS

template <bool LDS>
__device__ __forceinline__ void fused_phase2(const HrSparseArgs &a, int64_t fld, int total,
                                             bool use_bins, const FoldCand *s_list,
                                             FoldCand *cand, uint8_t *idx,
                                             const uint32_t *s_bits, const int *s_rowcnt,
                                             const int *s_rowoff, uint64_t *s_live, int *s_next) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const FoldCand *glist = a.list + fld * a.list_cap;
    const int lx = lane & 7, ly = lane >> 3;
    const int nwords = (a.tiles + 31) >> 5;
    int wd = 0, li = 0;
    uint32_t bits = __builtin_amdgcn_readfirstlane(s_bits[0]);
    auto get = [&](int c) -> const FoldCand & {
        if constexpr (LDS) return s_list[idx[c]];
        else return cand[c];
    };
    while (true) {
        int claim = 0;
        if (lane == 0) claim = atomicAdd(s_next, 1);
        const int target = __builtin_amdgcn_readfirstlane(claim);
        int t = -1;
        while (wd < nwords) {
            if (!bits) {
                if (++wd < nwords) bits = __builtin_amdgcn_readfirstlane(s_bits[wd]);
                continue;
            }
            if (li == target) {
                t = wd * 32 + __builtin_ctz(bits);
                break;
            }
            bits &= bits - 1;
            li++;
        }
        if (t < 0) break;
        const int tx0 = (t % a.tiles_x) * kTile, ty0 = (t / a.tiles_x) * kTile;
        float *mp = a.map + (fld * a.tiles + t) * (int64_t)(kTile * kTile);
        uint64_t done = 0;
        const int row = t / a.tiles_x;
        const int rc = (!LDS && use_bins) ? s_rowcnt[row] : -1;
        const FoldCand *src = rc >= 0 ? a.bins + fld * a.bins_cap + s_rowoff[row] : glist;
        const int src_n = rc >= 0 ? rc : total;
        int cursor = 0;
        while (true) {
            int n = 0;
            while (cursor < src_n) {
                const int e = cursor + lane;
                bool hit = false;
                FoldCand c;
                uint32_t lo = 0, hi = 0;
                if (e < src_n) {
                    if constexpr (LDS) {
                        lo = s_list[e].lo;
                        hi = s_list[e].hi;
                    } else {
                        c = src[e];
                        lo = c.lo;
                        hi = c.hi;
                    }
                    const int x0 = (int)(lo & 0xffff), x1 = (int)(hi & 0xffff) + 1;
                    const int y0 = (int)(lo >> 16), y1 = (int)(hi >> 16) + 1;
                    hit = x1 > tx0 && x0 < tx0 + kTile && y1 > ty0 && y0 < ty0 + kTile;
                }
                const uint64_t mk = __ballot(hit);
                const int cnt = __popcll(mk);
                if (n + cnt > kSpCand) break;  // wave-uniform; chunk re-read next pass
                if (hit) {
                    const int pos = n + lane_prefix(mk);
                    if constexpr (LDS) idx[pos] = (uint8_t)e;
                    else cand[pos] = c;
                }
                n += cnt;
                cursor += 64;
            }
            const bool last = cursor >= src_n;
            wave_sync();
            uint64_t cl = 0ull;
            bool slow_l = false;
            if (lane < n) {
                cl = cand_live(get(lane), tx0, ty0);
                slow_l = cand_slow(get(lane));
            }
            const uint64_t slow = __ballot(slow_l);
            const uint64_t live = wave_or64(cl, &s_live[wave]);
            for (uint64_t rest = live; rest; rest &= rest - 1) {
                const int blk = __builtin_ctzll(rest);
                const int px = tx0 + 8 * (blk & 7) + lx, py = ty0 + 8 * (blk >> 3) + ly;
                const bool on = px < a.ww && py < a.hh;
                const float fx = on ? (float)px : kOffMapCoord, fy = on ? (float)py : kOffMapCoord;
                const uint32_t key = on ? pix_key(px, py) : kOffMapKey;
                const uint64_t bq = __ballot((cl >> blk) & 1ull);
                float acc = ((done >> blk) & 1ull) ? mp[blk * 64 + lane] : 0.0f;
                acc = fold_block_g(acc, get, bq, slow, fx, fy, key);
                __builtin_nontemporal_store(acc, &mp[blk * 64 + lane]);
            }
            done |= live;
            if (last) break;
            wave_sync();  // candidate arrays are rewritten by the next pass
        }
        if (lane == 0) a.masks[fld * a.tiles + t] = done;
    }
}

template <bool SEEDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void cifhr_fused_kernel(HrSparseArgs a) {
    // the field's list (<= kFuList entries), or with a longer list the per-wave candidate
    // copies of phase 2
    __shared__ __attribute__((aligned(16))) FoldCand s_list[kFuList];
    static_assert(kFuList >= 4 * kSpCand, "per-wave candidate copies share the list's LDS");
    __shared__ uint8_t s_idx[4][kSpCand];
    __shared__ uint32_t s_bits[kTileBits / 32];
    __shared__ RowBinLds s_rb;
    __shared__ int s_rowcnt[kMaxBinRows], s_rowoff[kMaxBinRows];
    __shared__ __attribute__((aligned(16))) int s_cnt[2][kSpU][4];
    __shared__ int s_stage[kFuStage];
    __shared__ int s_tmp[4];
    __shared__ uint64_t s_live[4];
    __shared__ int s_next;

    const int64_t fld = blockIdx.x;  // image * K + field
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave == 0) HR_STAMP(0);
    if (threadIdx.x == 0) s_next = 0;
    if (threadIdx.x < kTileBits / 32) s_bits[threadIdx.x] = 0u;
    FoldCand *glist = a.list + fld * a.list_cap;
    const float stride = (float)a.h.cstride[0];
    const bool ms_on = a.h.ms_on & 1u;
    const float ms_th = a.h.ms_th[0];
    const int hw = a.h.cH[0] * a.h.cW[0];
    const float *p = a.h.cif[0] + fld * 5 * (int64_t)hw;
    // seeds: field f of image img, its segment of the scratch (SeedArgs::seg_base(0, f))
    const SeedSink &ss = a.seeds;
    const int f = SEEDS ? (int)(fld % ss.K) : 0;
    const int64_t img = SEEDS ? fld / ss.K : 0;
    const bool seeding = SEEDS && !((ss.skip >> f) & 1u);
    float *sv = SEEDS ? ss.g_keys + img * 4 * ss.cap + (int64_t)f * hw : nullptr;
    float *sx = sv + ss.cap, *sy = sx + ss.cap, *sz = sy + ss.cap;
    int n_seed = 0;

    // ---- phase 1: the list (cif_hr.py:26-40) and the seed candidates (cif_seeds.py:28-33) ----
    // candidate of kept cell `cell` at list position pos; returns its (c, x, y, s) * stride
    auto emit = [&](int cell, int pos, float &c, float &x8, float &y8, float &s8) {
        c = p[cell];
        const float x = p[hw + cell], y = p[2 * hw + cell], s4 = p[4 * hw + cell];
        const float cx = x * stride, cy = y * stride;
        const float sg = (0.5f * s4) * stride;
        const float sigma = (sg != sg) ? sg : fmaxf(1.0f, sg);  // np.maximum keeps NaN
        const float v = (c / a.neighbors) / 1.0f;                 // v / neighbors / len_cifs
        const int4 box = splat_box<M_GAUSS_MAX>(cx, cy, 1.0f * sigma, a.hh, a.ww);
        const FoldCand fc = make_cand(box, make_float4(cx, cy, v, sigma * sigma), a.hh, a.ww);
        if (pos < kFuList)
            s_list[pos] = fc;
        else
            glist[pos] = fc;
        for (int ty = box.z / kTile; ty <= (box.w - 1) / kTile; ty++)
            for (int tx = box.x / kTile; tx <= (box.y - 1) / kTile; tx++) {
                const int t = ty * a.tiles_x + tx;
                atomicOr(&s_bits[t >> 5], 1u << (t & 31));
            }
        x8 = cx;
        y8 = cy;
        s8 = s4 * stride;
    };
    // block-uniform: one seed-candidate compaction over the threads' (flag, values)
    auto seed_cand = [&](bool cand, float c, float x8, float y8, float s8) {
        if constexpr (SEEDS) {
            int tot;
            const int slot = block_compact<4>(cand, s_tmp, tot);
            if (cand) {
                sv[n_seed + slot] = c;
                sx[n_seed + slot] = x8;
                sy[n_seed + slot] = y8;
                sz[n_seed + slot] = s8;
            }
            n_seed += tot;
        }
    };
    int running = 0, buf = 0;
    for (int base = 0; base < hw; base += 256 * kSpU) {
        float c[kSpU];
#pragma unroll
        for (int k = 0; k < kSpU; k++) {
            const int cell = base + k * 256 + (int)threadIdx.x;
            c[k] = cell < hw ? p[cell] : NAN;  // NaN: never > v_th
        }
        uint32_t keep = 0;
#pragma unroll
        for (int k = 0; k < kSpU; k++) keep |= (c[k] > a.v_th) ? (1u << k) : 0u;
        if (ms_on) {  // p[4] > min_scale / stride (cif_hr.py:29-30, cif_seeds.py:31-32)
            uint32_t km = keep;
#pragma unroll
            for (int k = 0; k < kSpU; k++)
                if ((keep >> k) & 1u) {
                    const int cell = base + k * 256 + (int)threadIdx.x;
                    if (!(p[4 * hw + cell] > ms_th)) km &= ~(1u << k);
                }
            keep = km;
        }
#pragma unroll
        for (int k = 0; k < kSpU; k++) {
            const uint64_t bal = __ballot((keep >> k) & 1u);
            if (lane == 0) s_cnt[buf][k][wave] = __popcll(bal);
        }
        __syncthreads();  // (also orders the s_bits clear before the first atomicOr)
        int off = 0;
#pragma unroll 4
        for (int k = 0; k < kSpU; k++) {
            const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[buf][k][0]);
            off += q.x + q.y + q.z + q.w;
        }
        if (off <= kFuStage) {
            int o = 0;
#pragma unroll 4
            for (int k = 0; k < kSpU; k++) {
                const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[buf][k][0]);
                const uint64_t bal = __ballot((keep >> k) & 1u);
                if ((keep >> k) & 1u)
                    s_stage[o + (wave > 0 ? q.x : 0) + (wave > 1 ? q.y : 0) + (wave > 2 ? q.z : 0) +
                            lane_prefix(bal)] = base + k * 256 + (int)threadIdx.x;
                o += q.x + q.y + q.z + q.w;
            }
            __syncthreads();
            for (int e0 = 0; e0 < off; e0 += 256) {  // block-uniform
                const int e = e0 + (int)threadIdx.x;
                float cc = 0.0f, x8 = 0.0f, y8 = 0.0f, s8 = 0.0f;
                if (e < off) emit(s_stage[e], running + e, cc, x8, y8, s8);
                seed_cand(seeding && e < off && cc > ss.th, cc, x8, y8, s8);
            }
        } else {  // more than the stage holds: batch by batch (not unrolled)
            int o = 0;
#pragma unroll 1
            for (int k = 0; k < kSpU; k++) {
                const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[buf][k][0]);
                const uint64_t bal = __ballot((keep >> k) & 1u);
                const bool kept = (keep >> k) & 1u;
                float cc = 0.0f, x8 = 0.0f, y8 = 0.0f, s8 = 0.0f;
                if (kept)
                    emit(base + k * 256 + (int)threadIdx.x,
                         running + o + (wave > 0 ? q.x : 0) + (wave > 1 ? q.y : 0) +
                             (wave > 2 ? q.z : 0) + lane_prefix(bal),
                         cc, x8, y8, s8);
                seed_cand(seeding && kept && cc > ss.th, cc, x8, y8, s8);
                o += q.x + q.y + q.z + q.w;
            }
        }
        running += off;
        buf ^= 1;
        __syncthreads();  // the stage is rewritten by the next round
    }
    const int total = running;
    if (wave == 0) {
        HR_STAMP(1);
        HR_ADD(8, total);
        HR_ADD(9, n_seed);
    }
    const bool lds = total <= kFuList;
    bool use_bins = false;
    if (!lds) {
        // the LDS part joins the global list; the LDS then holds phase 2's candidate copies
        if (threadIdx.x < kFuList) glist[threadIdx.x] = s_list[threadIdx.x];
        __syncthreads();
        use_bins = a.bins_cap > 0 && total > kBinMin;
        if (use_bins)
            hr_row_bins(glist, total, a.bins + fld * a.bins_cap, a.bins_cap, a.tiles_y, s_rb,
                        s_rowcnt, s_rowoff);
    }
    for (int t = threadIdx.x; t < a.tiles; t += 256)  // untouched tiles: no block written
        if (!((s_bits[t >> 5] >> (t & 31)) & 1u)) a.masks[fld * a.tiles + t] = 0ull;

    // ---- phase 2: the waves take the touched tiles from an LDS counter ----
    if (lds)
        fused_phase2<true>(a, fld, total, false, s_list, nullptr, s_idx[wave], s_bits, s_rowcnt,
                           s_rowoff, s_live, &s_next);
    else
        fused_phase2<false>(a, fld, total, use_bins, nullptr, s_list + wave * kSpCand, nullptr,
                            s_bits, s_rowcnt, s_rowoff, s_live, &s_next);

    // ---- phase 3: the seeds (cif_seeds.py:35-47) from the finished map ----
    if constexpr (SEEDS) {
        __syncthreads();  // every wave's blocks and masks are stored
        if (wave == 0) HR_STAMP(2);
        if (seeding) seeds_from_map(a, fld, n_seed, s_tmp);
        else if (threadIdx.x == 0) ss.f_counts[fld] = 0;
    }
#ifdef PP_STAMPS
    __syncthreads();
    if (wave == 0) HR_STAMP(3);
    if (g_hr_stamps && threadIdx.x == 0) {
        g_hr_stamps[blockIdx.x * kHrSt + 6] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        g_hr_stamps[blockIdx.x * kHrSt + 7] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    }
#endif
}

// -------------------------------------------------------------------------------------
// host launchers
// -------------------------------------------------------------------------------------
static inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

template <int MODE>
static void launch_tiles(TileArgs a, hipStream_t stream) {
    a.tiles_x = (a.w + kTile - 1) / kTile;
    const int tiles_y = (a.h + kTile - 1) / kTile;
    a.tiles = a.tiles_x * tiles_y;
    const int64_t n_fields = a.n_work;  // caller passes the field count here
    a.n_work = n_fields * a.tiles;
    const int64_t nblocks = round_up(a.n_work, 8);
    hipLaunchKernelGGL(splat_tile_kernel<MODE>, dim3((unsigned)nblocks), dim3(256), 0, stream, a);
}

}  // namespace pp

using namespace pp;

extern "C" {

int64_t pp_cifhr_pitch(int64_t w_hr) { return round_up(w_hr, 32); }

size_t pp_cifhr_workspace_size(int32_t n_img, int32_t K, int32_t H, int32_t W) {
    return pp::cifhr_heads_workspace_size(pp::single_head(nullptr, nullptr, H, W, 1), n_img, K);
}

}  // extern "C"

namespace pp {

// dense CifHr workspace: FoldCand lists, counts, tile bitmaps, row-bin sizes / offsets, row
// bins (bins_capacity entries per list, independent of the stride: pp_cifhr_workspace_size
// has no stride argument)
struct HeadsWs {
    size_t off_counts, off_bits, off_rowcnt, off_rowoff, off_bins, total;
};

static HeadsWs heads_ws(const Heads &h, int n_img, int K) {
    const size_t nf = (size_t)n_img * K, nl = nf * h.n_groups;
    HeadsWs w;
    w.off_counts = round_up((int64_t)(nf * (size_t)h.cif_cells() * sizeof(FoldCand)), 256);
    w.off_bits = w.off_counts + round_up((int64_t)(nl * sizeof(int)), 256);
    w.off_rowcnt = w.off_bits + round_up((int64_t)(nl * (kTileBits / 32) * sizeof(uint32_t)), 256);
    w.off_rowoff = w.off_rowcnt + round_up((int64_t)(nl * kMaxBinRows * sizeof(int)), 256);
    w.off_bins = w.off_rowoff + round_up((int64_t)(nl * kMaxBinRows * sizeof(int)), 256);
    w.total = w.off_bins +
              round_up((int64_t)(nl * (size_t)bins_capacity(h.cif_cells()) * sizeof(FoldCand)), 256);
    return w;
}

size_t cifhr_heads_workspace_size(const Heads &h, int n_img, int K) {
    return heads_ws(h, n_img, K).total;
}

// CifHr.fill (cif_hr.py:59-73) over the heads: the map has head 0's field size and stride
template <bool DET>
int cifhr_heads_launch(const Heads &h, int32_t n_img, int32_t K, const pp_config *cfg,
                       float *d_cifhr, void *d_workspace, size_t workspace_bytes, hipStream_t s,
                       const char *who) {
    if (!cfg || !d_cifhr || !d_workspace) return fail(PP_EINVAL, std::string(who) + ": NULL argument");
    for (int m = 0; m < h.n_cif; m++)
        if (!h.cif[m]) return fail(PP_EINVAL, std::string(who) + ": NULL field");
    if (n_img < 0 || K <= 0) return fail(PP_ESHAPE, std::string(who) + ": bad shape");
    if (n_img == 0) return PP_OK;
    if (workspace_bytes < cifhr_heads_workspace_size(h, n_img, K))
        return fail(PP_ENOMEM, std::string(who) + ": workspace too small");
    const int hh = h.hr_hh, ww = h.hr_ww;
    if (hh >= kMaxHrSide || ww >= kMaxHrSide)  // fold candidates pack pixel (x, y) as int16
        return fail(PP_ESHAPE, std::string(who) + ": CifHr map of 32768 px or more per side");
    const int64_t pitch = pp_cifhr_pitch(ww);
    const int64_t nf = (int64_t)n_img * K;
    HrSplatArgs sa{};
    sa.h = h;
    sa.K = K;
    sa.hh = hh;
    sa.ww = ww;
    sa.v_th = cfg->cif_threshold;
    sa.neighbors = (float)cfg->cif_neighbors;
    sa.list = (FoldCand *)d_workspace;
    sa.list_cap = h.cif_cells();
    int64_t o = 0;
    for (int g = 0; g < h.n_groups; g++) {
        sa.goff[g] = o;
        for (int i = 0; i < h.group_size(); i++) o += h.cif_hw(h.member(g, i));
    }
    const HeadsWs wl = heads_ws(h, n_img, K);
    sa.counts = (int *)((char *)d_workspace + wl.off_counts);
    sa.tile_bits = (uint32_t *)((char *)d_workspace + wl.off_bits);
    sa.rowcnt = (int *)((char *)d_workspace + wl.off_rowcnt);
    sa.rowoff = (int *)((char *)d_workspace + wl.off_rowoff);
    sa.bins = (FoldCand *)((char *)d_workspace + wl.off_bins);
    sa.tiles_x = (int)((pitch + kTile - 1) / kTile);
    sa.tiles_y = (hh + kTile - 1) / kTile;
    sa.tiles = sa.tiles_x * sa.tiles_y;
    sa.bins_cap = sa.tiles_y <= kMaxBinRows ? bins_capacity(h.cif_cells()) : 0;
    if (!DET && h.n_groups == 1) {
        // the decoder's phase 1 (hr_splat_list: 32 confidences per thread in flight, one
        // barrier per round, kept cells staged in LDS), writing this layout
        HrSparseArgs la{};
        la.h = h;
        la.hh = hh;
        la.ww = ww;
        la.v_th = sa.v_th;
        la.neighbors = sa.neighbors;
        la.list = sa.list;
        la.list_cap = sa.list_cap;
        la.bins = sa.bins;
        la.bins_cap = sa.bins_cap;
        la.tiles_x = sa.tiles_x;
        la.tiles = sa.tiles;
        la.tiles_y = sa.tiles_y;
        la.split = 1;
        la.pre_total = sa.counts;
        la.pre_bits = sa.tile_bits;
        la.pre_rowcnt = sa.rowcnt;
        la.pre_rowoff = sa.rowoff;
        if (sa.tiles > kTileBits) return fail(PP_ESHAPE, std::string(who) + ": CifHr map too large");
        hipLaunchKernelGGL(cifhr_list_kernel<false>, dim3((unsigned)nf), dim3(256), 0, s, la);
    } else {
        hipLaunchKernelGGL(cifhr_splats_kernel<DET>, dim3((unsigned)(nf * h.n_groups)), dim3(256), 0, s, sa);
    }
    HrTileArgs a{};
    a.field = d_cifhr;
    a.list = sa.list;
    a.counts = sa.counts;
    a.tile_bits = sa.tile_bits;
    a.bins = sa.bins;
    a.rowcnt = sa.rowcnt;
    a.rowoff = sa.rowoff;
    a.bins_cap = sa.bins_cap;
    a.splat_cap = sa.list_cap;
    a.h = hh;
    a.w = ww;
    a.pitch = (int)pitch;
    a.tiles_x = sa.tiles_x;
    a.tiles = sa.tiles;
    a.chunk_tiles = kChunkTiles;
    a.chunks = (sa.tiles + a.chunk_tiles - 1) / a.chunk_tiles;
    a.field_stride = (int64_t)hh * pitch;
    a.n_work = nf * a.chunks;
    a.n_groups = h.n_groups;
    for (int g = 0; g < h.n_groups; g++) a.goff[g] = sa.goff[g];
    if (sa.tiles > kTileBits) return fail(PP_ESHAPE, std::string(who) + ": CifHr map too large");
    const int64_t nblocks = round_up(a.n_work, 8);
    if (h.n_groups > 1)
        hipLaunchKernelGGL(cifhr_tile_kernel<true>, dim3((unsigned)nblocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(cifhr_tile_kernel<false>, dim3((unsigned)nblocks), dim3(256), 0, s, a);
    return check_launch(who);
}

template int cifhr_heads_launch<false>(const Heads &, int32_t, int32_t, const pp_config *, float *,
                                       void *, size_t, hipStream_t, const char *);
template int cifhr_heads_launch<true>(const Heads &, int32_t, int32_t, const pp_config *, float *,
                                      void *, size_t, hipStream_t, const char *);

// workgroups per field of cifhr_sparse_kernel: fewer fields than kSplitSlots split each
// field's tiles over several workgroups (each builds its own copy of the field's list: a
// re-read of its confidences, no extra round trip, no shared writes)
static int sparse_split(int64_t nf) {
#ifdef PP_STAMPS  // the diagnostic build only: PP_SPLIT_SLOTS (tools/cfg2_split.py)
    static const int64_t slots = [] {
        const char *e = getenv("PP_SPLIT_SLOTS");
        return e && atoi(e) > 0 ? (int64_t)atoi(e) : (int64_t)kSplitSlots;
    }();
#else
    constexpr int64_t slots = kSplitSlots;
#endif
    return (int)std::max<int64_t>(1, std::min<int64_t>(kMaxSplit, slots / std::max<int64_t>(1, nf)));
}

// candidates per split workgroup of a prebuilt field list: all of a field's split
// workgroups read the same bins, so a short list on many workgroups only queues them on
// the same L2 lines (cfg2 planted, 125 candidates per field: fold kernel 35.1 us on 60
// workgroups per field, 22.1 us on 3); PP_SPLIT_LIST overrides it in the diagnostic build
constexpr int kSplitList = 48;
static int split_list_len() {
#ifdef PP_STAMPS
    static const int v = [] {
        const char *e = getenv("PP_SPLIT_LIST");
        return e && atoi(e) > 0 ? atoi(e) : kSplitList;
    }();
    return v;
#else
    return kSplitList;
#endif
}

size_t cifhr_sparse_workspace_size(const Heads &h, int n_img, int K) {
    const size_t nf = (size_t)n_img * K * sparse_split((int64_t)n_img * K);
    size_t bytes = round_up((int64_t)(nf * (size_t)h.cif_cells() * sizeof(FoldCand)), 256);
    if (h.n_groups == 1)
        bytes += round_up((int64_t)(nf * (size_t)bins_capacity(h.cif_cells()) * sizeof(FoldCand)), 256);
    return bytes;
}

// the prebuilt-list mode of split fields: the field's list, lengths, tile bits, bin sizes
// and completion counters go past the nf lists (the workspace holds nf * split of them)
static size_t prebuilt_bytes(int64_t nf) {
    return (size_t)nf * (2 + kTileBits / 32 + 2 * kMaxBinRows) * sizeof(int);
}
static bool sparse_prebuilt(const Heads &h, int64_t nf) {
    const int split = sparse_split(nf);
    return split > 1 && h.n_groups == 1 &&
           (size_t)nf * (split - 1) * h.cif_cells() * sizeof(FoldCand) >= prebuilt_bytes(nf);
}

bool cifhr_fuses_seeds(const Heads &h, int n_img, int K, const pp_config *cfg) {
    const int64_t nf = (int64_t)n_img * K;
    // one workgroup per field: cifhr_fused_kernel<true>; split fields with a prebuilt list:
    // cifhr_list_kernel<true> + cifhr_sparse_kernel<false, true>
    return h.n_cif == 1 && h.n_groups == 1 && h.group_size() == 1 && n_img > 0 && K > 0 &&
           (sparse_split(nf) == 1 || sparse_prebuilt(h, nf)) &&
           cfg->seed_threshold >= cfg->cif_threshold;
}

int cifhr_sparse_launch(const Heads &h, int32_t n_img, int32_t K, const pp_config *cfg,
                        float *d_map, float *d_aux, uint64_t *d_masks, void *d_workspace,
                        size_t workspace_bytes, hipStream_t s, const char *who,
                        const SeedSink *sink) {
    if (!cfg || !d_map || !d_masks || !d_workspace || (h.n_groups > 1 && !d_aux))
        return fail(PP_EINVAL, std::string(who) + ": NULL argument");
    for (int m = 0; m < h.n_cif; m++)
        if (!h.cif[m]) return fail(PP_EINVAL, std::string(who) + ": NULL field");
    if (n_img < 0 || K <= 0) return fail(PP_ESHAPE, std::string(who) + ": bad shape");
    if (n_img == 0) return PP_OK;
    if (workspace_bytes < cifhr_sparse_workspace_size(h, n_img, K))
        return fail(PP_ENOMEM, std::string(who) + ": workspace too small");
    const int hh = h.hr_hh, ww = h.hr_ww;
    if (hh >= kMaxHrSide || ww >= kMaxHrSide)  // fold candidates pack pixel (x, y) as int16
        return fail(PP_ESHAPE, std::string(who) + ": CifHr map of 32768 px or more per side");
    const HrMap geo = dense_hr(nullptr, hh, ww);
    if (geo.tiles > kTileBits) return fail(PP_ESHAPE, std::string(who) + ": CifHr map too large");
    if (h.n_groups > 8) return fail(PP_ESHAPE, std::string(who) + ": too many CifHr groups");
    HrSparseArgs a{};
    a.h = h;
    a.hh = hh;
    a.ww = ww;
    a.v_th = cfg->cif_threshold;
    a.neighbors = (float)cfg->cif_neighbors;
    a.list = (FoldCand *)d_workspace;
    a.list_cap = h.cif_cells();
    a.tiles_x = geo.tiles_x;
    a.tiles = geo.tiles;
    a.tiles_y = (hh + kTile - 1) / kTile;
    // row bins for single-scale maps of at most kMaxBinRows tile rows
    a.bins_cap = (h.n_groups == 1 && a.tiles_y <= kMaxBinRows) ? bins_capacity(h.cif_cells()) : 0;
    a.bins = (FoldCand *)((char *)d_workspace +
                          round_up((int64_t)((size_t)n_img * K * sparse_split((int64_t)n_img * K) *
                                             a.list_cap * sizeof(FoldCand)), 256));
    a.map = d_map;
    a.aux = d_aux;
    a.masks = d_masks;
    const int64_t nf = (int64_t)n_img * K;
    a.split = sparse_split(nf);
    a.split_list = split_list_len();
    const unsigned nblocks = (unsigned)(nf * a.split);
    // one workgroup per field, one CIF head: the list-in-LDS kernel (with the seeds when a
    // sink is given); fields of small batches split over several workgroups, and
    // multi-scale groups, take cifhr_sparse_kernel
#ifdef PP_STAMPS
    uint64_t *st = nullptr;
    hipMalloc((void **)&st, (size_t)nblocks * kHrSt * sizeof(uint64_t));
    hipMemsetAsync(st, 0, (size_t)nblocks * kHrSt * sizeof(uint64_t), s);
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_hr_stamps), &st, sizeof(st), 0, hipMemcpyHostToDevice, s);
    // [start, ...]: dumped to $PP_HR_STAMPS_OUT after the launch (the stream synchronised)
    auto dump = [&]() {
        hipStreamSynchronize(s);
        std::vector<uint64_t> hbuf((size_t)nblocks * kHrSt);
        hipMemcpy(hbuf.data(), st, hbuf.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
        const char *path = getenv("PP_HR_STAMPS_OUT");
        FILE *fo = fopen(path ? path : "pp_hr_stamps.bin", "ab");
        if (fo) {
            fwrite(hbuf.data(), sizeof(uint64_t), hbuf.size(), fo);
            fclose(fo);
        }
        uint64_t *nul = nullptr;
        hipMemcpyToSymbol(HIP_SYMBOL(g_hr_stamps), &nul, sizeof(nul));
        hipFree(st);
    };
#endif
    if (a.split == 1 && h.n_cif == 1 && h.n_groups == 1 && h.group_size() == 1) {
        if (sink) {
            if (!cifhr_fuses_seeds(h, n_img, K, cfg) || sink->K != K)
                return fail(PP_EINVAL, std::string(who) + ": seeds cannot be fused here");
            a.seeds = *sink;
            hipLaunchKernelGGL(cifhr_fused_kernel<true>, dim3(nblocks), dim3(256), 0, s, a);
        } else {
            hipLaunchKernelGGL(cifhr_fused_kernel<false>, dim3(nblocks), dim3(256), 0, s, a);
        }
#ifdef PP_STAMPS
        dump();
#endif
        return check_launch(who);
    }
    // split fields: one list per field, built before the fold (cifhr_list_kernel);
    // (cfg2 uniform: CifHr stage 0.173 -> 0.125 ms with the prebuilt list and stripe units;
    // planted unchanged within noise).  With a sink the list kernel also writes the seed
    // candidates and the fold's last workgroup per field emits the seeds (cfg2: no
    // seeds_emit_kernel launch)
    const bool prebuilt = sparse_prebuilt(h, nf);
    if (sink && (!prebuilt || !cifhr_fuses_seeds(h, n_img, K, cfg) || sink->K != K))
        return fail(PP_EINVAL, std::string(who) + ": seeds cannot be fused here");
    if (prebuilt) {
        int *p = reinterpret_cast<int *>(a.list + nf * a.list_cap);
        a.pre_total = p;
        a.pre_bits = reinterpret_cast<uint32_t *>(p + nf);
        a.pre_rowcnt = p + nf * (1 + kTileBits / 32);
        a.pre_rowoff = a.pre_rowcnt + nf * kMaxBinRows;
        a.done = a.pre_rowoff + nf * kMaxBinRows;
        if (sink) {
            a.seeds = *sink;
            hipLaunchKernelGGL(cifhr_list_kernel<true>, dim3((unsigned)nf), dim3(256), 0, s, a);
        } else {
            hipLaunchKernelGGL(cifhr_list_kernel<false>, dim3((unsigned)nf), dim3(256), 0, s, a);
        }
    }
    if (h.n_groups > 1)
        hipLaunchKernelGGL(cifhr_sparse_kernel<true>, dim3(nblocks), dim3(256), 0, s, a);
    else if (sink)
        hipLaunchKernelGGL((cifhr_sparse_kernel<false, true>), dim3(nblocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(cifhr_sparse_kernel<false>, dim3(nblocks), dim3(256), 0, s, a);
#ifdef PP_STAMPS
    dump();
#endif
    return check_launch(who);
}

}  // namespace pp

extern "C" {

int pp_cifhr(const float *d_cif, int32_t n_img, int32_t K, int32_t H, int32_t W,
             const pp_config *cfg, float *d_cifhr, void *d_workspace, size_t workspace_bytes,
             void *stream) {
    if (!d_cif || !cfg) return fail(PP_EINVAL, "pp_cifhr: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_cifhr: bad shape");
    return cifhr_heads_launch<false>(single_head(d_cif, nullptr, H, W, cfg->stride), n_img, K, cfg,
                                     d_cifhr, d_workspace, workspace_bytes,
                                     (hipStream_t)stream, "pp_cifhr");
}

int32_t pp_cifhr_sparse_tiles(int32_t H, int32_t W, int32_t stride) {
    if (H <= 0 || W <= 0 || stride <= 0) return 0;
    return dense_hr(nullptr, (int)hr_dim(H, stride), (int)hr_dim(W, stride)).tiles;
}

size_t pp_cifhr_sparse_workspace_size(int32_t n_img, int32_t K, int32_t H, int32_t W) {
    return pp::cifhr_sparse_workspace_size(pp::single_head(nullptr, nullptr, H, W, 1), n_img, K);
}

int pp_cifhr_sparse(const float *d_cif, int32_t n_img, int32_t K, int32_t H, int32_t W,
                    const pp_config *cfg, float *d_map, uint64_t *d_masks, void *d_workspace,
                    size_t workspace_bytes, void *stream) {
    if (!d_cif || !cfg) return fail(PP_EINVAL, "pp_cifhr_sparse: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_cifhr_sparse: bad shape");
    return cifhr_sparse_launch(single_head(d_cif, nullptr, H, W, cfg->stride), n_img, K, cfg,
                               d_map, nullptr, d_masks, d_workspace, workspace_bytes,
                               (hipStream_t)stream, "pp_cifhr_sparse");
}

int pp_cifdet_hr(const float *d_det, int32_t n_img, int32_t K, int32_t H, int32_t W,
                 const pp_config *cfg, float *d_cifhr, void *d_workspace, size_t workspace_bytes,
                 void *stream) {
    if (!d_det || !cfg) return fail(PP_EINVAL, "pp_cifdet_hr: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_cifdet_hr: bad shape");
    return cifhr_heads_launch<true>(single_head(d_det, nullptr, H, W, cfg->stride), n_img, K, cfg,
                                    d_cifhr, d_workspace, workspace_bytes,
                                    (hipStream_t)stream, "pp_cifdet_hr");
}

size_t pp_cifhr_multi_workspace_size(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                     int32_t n_img, int32_t K) {
    Heads h;
    if (make_heads(scales, n_scales, cif_pairs, PP_ROLE_CIF, &h, "pp_cifhr_multi_workspace_size") ||
        n_img < 0 || K <= 0)
        return 0;
    return cifhr_heads_workspace_size(h, n_img, K);
}

int pp_cifdet_hr_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                       int32_t K, const pp_config *cfg, float *d_cifhr, void *d_workspace,
                       size_t workspace_bytes, void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, cif_pairs, PP_ROLE_CIF, &h, "pp_cifdet_hr_multi");
    if (rc) return rc;
    return cifhr_heads_launch<true>(h, n_img, K, cfg, d_cifhr, d_workspace, workspace_bytes,
                                    (hipStream_t)stream, "pp_cifdet_hr_multi");
}

int pp_cifhr_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                   int32_t K, const pp_config *cfg, float *d_cifhr, void *d_workspace,
                   size_t workspace_bytes, void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, cif_pairs, PP_ROLE_CIF, &h, "pp_cifhr_multi");
    if (rc) return rc;
    return cifhr_heads_launch<false>(h, n_img, K, cfg, d_cifhr, d_workspace, workspace_bytes,
                                     (hipStream_t)stream, "pp_cifhr_multi");
}

}  // extern "C"

// ---- functional.pyx square-splat primitives (in place on one (h, w) field) ----
namespace pp {

template <int MODE>
static int run_square_primitive(float *field, float *field2, int64_t h, int64_t w, int64_t pitch,
                                const float *x, const float *y, const float *s, const float *v,
                                const float *wt, int64_t n, float truncate, float max_value,
                                void *stream, const char *name) {
    if (!field || (n > 0 && (!x || !y || !s || !v))) return fail(PP_EINVAL, std::string(name) + ": NULL argument");
    if (h <= 0 || w <= 0 || pitch < w || h > (1 << 30) || w > (1 << 30))
        return fail(PP_ESHAPE, std::string(name) + ": bad field shape");
    if (n <= 0) return PP_OK;
    hipStream_t st = (hipStream_t)stream;
    Splat *splats = nullptr;
    if (hipMallocAsync((void **)&splats, (size_t)n * sizeof(Splat), st) != hipSuccess)
        return fail(PP_EHIP, std::string(name) + ": scratch allocation failed");
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL((prep_splats_kernel<MODE>), dim3((unsigned)blocks), dim3(256), 0, st, x, y,
                       s, v, wt, n, (int)h, (int)w, truncate, splats);
    TileArgs a{};
    a.field = field;
    a.field2 = field2;
    a.splats = splats;
    a.n_splats = n;
    a.splat_cap = n;
    a.field_stride = h * pitch;
    a.h = (int)h;
    a.w = (int)w;
    a.pitch = (int)pitch;
    a.n_work = 1;
    a.t2 = truncate * truncate;
    a.max_value = max_value;
    launch_tiles<MODE>(a, st);
    int rc = check_launch(name);
    hipFreeAsync(splats, st);
    return rc;
}

}  // namespace pp

extern "C" {

int pp_scalar_square_add_gauss_with_max(float *d_field, int64_t h, int64_t w, int64_t pitch,
                                        const float *d_x, const float *d_y, const float *d_sigma,
                                        const float *d_v, int64_t n, float truncate,
                                        float max_value, void *stream) {
    return run_square_primitive<M_GAUSS_MAX>(d_field, nullptr, h, w, pitch, d_x, d_y, d_sigma, d_v,
                                             nullptr, n, truncate, max_value, stream,
                                             "pp_scalar_square_add_gauss_with_max");
}

int pp_scalar_square_add_gauss(float *d_field, int64_t h, int64_t w, int64_t pitch,
                               const float *d_x, const float *d_y, const float *d_sigma,
                               const float *d_v, int64_t n, float truncate, void *stream) {
    return run_square_primitive<M_GAUSS>(d_field, nullptr, h, w, pitch, d_x, d_y, d_sigma, d_v,
                                         nullptr, n, truncate, 0.0f, stream,
                                         "pp_scalar_square_add_gauss");
}

int pp_scalar_square_max_gauss(float *d_field, int64_t h, int64_t w, int64_t pitch,
                               const float *d_x, const float *d_y, const float *d_sigma,
                               const float *d_v, int64_t n, float truncate, void *stream) {
    return run_square_primitive<M_MAXG>(d_field, nullptr, h, w, pitch, d_x, d_y, d_sigma, d_v,
                                        nullptr, n, truncate, 0.0f, stream,
                                        "pp_scalar_square_max_gauss");
}

int pp_scalar_square_add_constant(float *d_field, int64_t h, int64_t w, int64_t pitch,
                                  const float *d_x, const float *d_y, const float *d_width,
                                  const float *d_v, int64_t n, void *stream) {
    return run_square_primitive<M_CONST>(d_field, nullptr, h, w, pitch, d_x, d_y, d_width, d_v,
                                         nullptr, n, 0.0f, 0.0f, stream,
                                         "pp_scalar_square_add_constant");
}

int pp_cumulative_average(float *d_cuma, float *d_cumw, int64_t h, int64_t w, int64_t pitch,
                          const float *d_x, const float *d_y, const float *d_width,
                          const float *d_v, const float *d_w, int64_t n, void *stream) {
    if (!d_cumw || (n > 0 && !d_w)) return fail(PP_EINVAL, "pp_cumulative_average: NULL argument");
    return run_square_primitive<M_CUMAVG>(d_cuma, d_cumw, h, w, pitch, d_x, d_y, d_width, d_v, d_w,
                                          n, 0.0f, 0.0f, stream, "pp_cumulative_average");
}

}  // extern "C"
