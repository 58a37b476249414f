// stages.hip — CifSeeds and CafScored on gfx950.
//
//   seeds_emit_kernel  one workgroup per (image, CIF field): threshold + CifHr rescore +
//                      order-preserving ballot compaction (cif_seeds.py:28-47).
//   seeds_sort_kernel  one workgroup per image: fields concatenated in order, then a
//                      bitonic sort reproducing sorted(seeds, reverse=True)
//                      (cif_seeds.py:54) including its stability (ties broken by emission
//                      order).  LDS-resident up to kSortLds seeds, global network beyond.
//   caf_scored_kernel  one workgroup per (image, CAF field): threshold, x stride, CifHr
//                      lookups at both ends, forward/backward column sets in row-major
//                      cell order (caf_scored.py:32-87), one or two thresholds per pass.
//
// There is deliberately NO spatial NMS before the sort: v0.11.6 suppresses duplicate
// seeds only through the occupancy test in the seed loop (cifcaf.py:100-102).
#include "pp_common.hpp"

#ifdef PP_STAMPS
#include <stdio.h>
#include <stdlib.h>

#include <vector>
#endif

namespace pp {

#ifdef PP_STAMPS
// diagnostic build: seeds_sort_kernel per workgroup [start, offsets, keys loaded, sorted,
// done, n] in s_memtime ticks, dumped to $PP_SORT_STAMPS_OUT by launch_seeds
__device__ uint64_t *g_sort_stamps;
#define SORT_STAMP(slot)                                                                     \
    do {                                                                                     \
        if (g_sort_stamps && threadIdx.x == 0)                                               \
            g_sort_stamps[blockIdx.x * 6 + (slot)] = __builtin_amdgcn_s_memtime();           \
    } while (0)
#else
#define SORT_STAMP(slot) \
    do {                 \
    } while (0)
#endif

constexpr int kSortLds = 4096;

struct SeedKeys {
    const float *v, *x, *y, *s;
    const int *f;
    const int *loc;  // NULL, or emission index -> storage slot
    int n;
    __device__ __forceinline__ int at(int a) const { return loc ? loc[a] : a; }
    // true when seed a must come before seed b in sorted(..., reverse=True) order
    __device__ __forceinline__ bool before(int a, int b) const {
        if (a >= n) return false;  // padding sorts last
        if (b >= n) return true;
        const int pa = at(a), pb = at(b);
        if (v[pa] != v[pb]) return v[pa] > v[pb];
        if (f[pa] != f[pb]) return f[pa] > f[pb];
        if (x[pa] != x[pb]) return x[pa] > x[pb];
        if (y[pa] != y[pb]) return y[pa] > y[pb];
        if (s[pa] != s[pb]) return s[pa] > s[pb];
        return a < b;  // stable: emission order
    }
};

template <typename Perm>
__device__ __forceinline__ void bitonic_sort(Perm *p, int np, const SeedKeys &keys) {
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
    Heads h;            // CifSeeds.fill visits the heads in order (cif_seeds.py:56-64)
    HrMap hr;
    int K;
    float th, score_scale;
    uint32_t skip;      // pp_config.seed_skip_mask: fields that emit no seeds
    pp_seed *seeds;     // (n_img, cap) sorted output
    int cap;            // K * sum of the heads' H * W
    int *counts;        // (n_img) seeds per image
    float *g_keys;      // (n_img, 4, cap): per-segment emission slots (v, x, y, s)
    int *g_f;           // (n_img, cap): field of each slot
    int *f_counts;      // (n_img, n_heads * K) seeds per segment (head, field)
    int *g_perm;        // (n_img, np_cap)
    int np_cap;
    // first slot of segment (CIF head m, field f): K * cif_off[m] + f * H_m * W_m
    __device__ __forceinline__ int64_t seg_base(int m, int f) const {
        return (int64_t)K * h.cif_off[m] + (int64_t)f * h.cif_hw(m);
    }
    // seg_base of concatenated segment q = m * K + f with the head picked by selects: a
    // dynamic index into the kernel-argument struct makes the compiler copy the whole
    // struct to scratch for every lane
    __device__ __forceinline__ int64_t seg_base_q(int q) const {
        const int m = q / K, f = q % K;
        int64_t b = 0;
#pragma unroll
        for (int c = 0; c < kMaxHeads; c++)
            if (c == m) b = seg_base(c, f);
        return b;
    }
};

// stage 1: one workgroup per (image, head, field) — cif_seeds.py:28-47 for that field, in
// row-major cell order, into the segment's slot range.  A round covers 256 * kEmitU cells:
// every thread loads its kEmitU confidences at once, the cells above threshold are staged
// in LDS in cell order (one barrier orders the (cell batch, wave) counts), then one thread
// per staged cell reads x, y, scale and the CifHr value and the seeds are compacted in the
// staged order.  So a round is about four memory round trips however many cells it keeps
// (a round staging more than kEmitStage falls back to batches of 256).
constexpr int kEmitU = 32;
constexpr int kEmitStage = 256 * kEmitU;  // a whole round: no fallback for one 80x80 field

__global__ __launch_bounds__(256) void seeds_emit_kernel(SeedArgs a) {
    __shared__ int s_tmp[4];
    __shared__ __attribute__((aligned(16))) int s_cnt[kEmitU][4];
    __shared__ int s_stage[kEmitStage];
    const int nseg = a.h.n_cif * a.K;
    const int img = (int)(blockIdx.x / nseg), seg = (int)(blockIdx.x % nseg);
    const int m = seg / a.K, f = seg % a.K;
    const int hw = a.h.cH[m] * a.h.cW[m];
    const float stride = (float)a.h.cstride[m];
    const bool ms_on = (a.h.ms_on >> m) & 1u;
    const float ms_th = a.h.ms_th[m];
    const int64_t cap = a.cap;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *gv = a.g_keys + (int64_t)img * 4 * cap + a.seg_base(m, f);
    float *gx = gv + cap, *gy = gx + cap, *gs = gy + cap;
    int *gf = a.g_f + (int64_t)img * cap + a.seg_base(m, f);
    const float *p = a.h.cif[m] + ((int64_t)img * a.K + f) * 5 * hw;
    const int64_t plane = (int64_t)img * a.K + f;
    int running = 0;
    if ((a.skip >> f) & 1u) {  // `if seed_mask is not None and not seed_mask[field_i]: continue`
        if (threadIdx.x == 0) a.f_counts[blockIdx.x] = 0;
        return;
    }
    // cif_seeds.py:28-47 for one cell above threshold: (kept, v, x, y, s)
    auto score = [&](int cell, float c, float &v, float &x, float &y, float &sc) {
        x = p[hw + cell];
        y = p[2 * hw + cell];
        sc = p[4 * hw + cell];
        if (ms_on && !(sc > ms_th)) return false;  // then p[4] > min_scale / stride
        x = x * stride;
        y = y * stride;
        const float hv = a.hr.at(plane, x, y, 0.0f);
        float vv = 0.9f * hv + 0.1f * c;  // 0.9 * v + 0.1 * c
        if (a.score_scale != 1.0f) vv = vv * a.score_scale;
        v = vv;
        sc = sc * stride;
        return vv > a.th;
    };
    for (int base = 0; base < hw; base += 256 * kEmitU) {
        float c[kEmitU];
#pragma unroll
        for (int k = 0; k < kEmitU; k++) {
            const int cell = base + k * 256 + (int)threadIdx.x;
            c[k] = cell < hw ? p[cell] : NAN;  // NaN: never > threshold
        }
        uint32_t keep = 0;
#pragma unroll
        for (int k = 0; k < kEmitU; k++) keep |= (c[k] > a.th) ? (1u << k) : 0u;
#pragma unroll
        for (int k = 0; k < kEmitU; k++) {
            const uint64_t bal = __ballot((keep >> k) & 1u);
            if (lane == 0) s_cnt[k][wave] = __popcll(bal);
        }
        __syncthreads();
        int staged = 0;
#pragma unroll 4
        for (int k = 0; k < kEmitU; k++) {
            const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[k][0]);
            staged += q.x + q.y + q.z + q.w;
        }
        if (staged <= kEmitStage) {
            int o = 0;  // stage position of batch k's cell in this thread (ballot = cell order)
#pragma unroll 4
            for (int k = 0; k < kEmitU; k++) {
                const int4 q = *reinterpret_cast<const int4 *>(&s_cnt[k][0]);
                const uint64_t bal = __ballot((keep >> k) & 1u);
                if ((keep >> k) & 1u)
                    s_stage[o + (wave > 0 ? q.x : 0) + (wave > 1 ? q.y : 0) + (wave > 2 ? q.z : 0) +
                            lane_prefix(bal)] = base + k * 256 + (int)threadIdx.x;
                o += q.x + q.y + q.z + q.w;
            }
            __syncthreads();
            for (int e0 = 0; e0 < staged; e0 += 256) {  // block-uniform
                const int e = e0 + (int)threadIdx.x;
                float v = 0.0f, x = 0.0f, y = 0.0f, sc = 0.0f;
                bool ok = false;
                if (e < staged) {
                    const int cell = s_stage[e];
                    ok = score(cell, p[cell], v, x, y, sc);
                }
                int total;
                const int slot = block_compact<4>(ok, s_tmp, total);
                if (ok) {
                    const int pos = running + slot;
                    gv[pos] = v;
                    gx[pos] = x;
                    gy[pos] = y;
                    gs[pos] = sc;
                    gf[pos] = f;
                }
                running += total;
            }
        } else {  // more than the stage holds: batch by batch
#pragma unroll 1
            for (int k = 0; k < kEmitU; k++) {
                float v = 0.0f, x = 0.0f, y = 0.0f, sc = 0.0f;
                bool ok = false;
                const int cell = base + k * 256 + (int)threadIdx.x;
                if ((keep >> k) & 1u) ok = score(cell, p[cell], v, x, y, sc);  // no dynamic c[k]
                int total;
                const int slot = block_compact<4>(ok, s_tmp, total);
                if (ok) {
                    const int pos = running + slot;
                    gv[pos] = v;
                    gx[pos] = x;
                    gy[pos] = y;
                    gs[pos] = sc;
                    gf[pos] = f;
                }
                running += total;
            }
        }
        __syncthreads();  // s_cnt / s_stage are rewritten by the next round
    }
    if (threadIdx.x == 0) a.f_counts[blockIdx.x] = running;
}

// Seeds with v > threshold > 0 sort as 64-bit keys, descending: v's bits (positive
// floats order like integers), then the field, then the INVERTED emission index, so equal
// (v, field) stay in emission order.  The reference breaks (v, field) ties on x, y, s
// before emission order (tuple comparison, cif_seeds.py:54); such runs are rare and get
// re-sorted with the full comparator afterwards.
constexpr uint32_t kEmitMask = (1u << 27) - 1;

__device__ __forceinline__ uint64_t seed_key(float v, int f, int e) {
    return ((uint64_t)__float_as_uint(v) << 32) | ((uint32_t)f << 27) | (kEmitMask - (uint32_t)e);
}

__device__ __forceinline__ int key_emit(uint64_t k) { return (int)(kEmitMask - ((uint32_t)k & kEmitMask)); }

// stage 2: one workgroup per image — concatenate the segments in order and sort
// compare-exchange result for element i of the pair (i, i ^ j) in stage (k, j) of a
// descending bitonic network: the lower element of a descending block keeps the max
__device__ __forceinline__ uint64_t bitonic_pick(int i, int j, int k, uint64_t a, uint64_t b) {
    const bool lower = (i & j) == 0, desc = (i & k) == 0;
    const uint64_t mx = a > b ? a : b, mn = a > b ? b : a;
    return lower == desc ? mx : mn;
}

// lane ^ M for a constant M: DPP moves within a row of 16 (quad_perm for 1 and 2; the row
// half-mirror (lane ^ 7) or mirror (lane ^ 15) composed with a quad_perm / half-mirror for
// 4 and 8), a bpermute across rows
template <int M>
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v) {
    if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    } else if constexpr (M == 4) {  // (lane ^ 7) ^ 3
        const int h = __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
        return (uint32_t)__builtin_amdgcn_update_dpp(0, h, 0x1B, 0xF, 0xF, false);
    } else if constexpr (M == 8) {  // (lane ^ 15) ^ 7
        const int h = __builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
        return (uint32_t)__builtin_amdgcn_update_dpp(0, h, 0x141, 0xF, 0xF, false);
    } else {
        return (uint32_t)__shfl_xor((int)v, M);
    }
}

template <int M>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v) {
    return ((uint64_t)lane_xor32<M>((uint32_t)(v >> 32)) << 32) | lane_xor32<M>((uint32_t)v);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

// descending bitonic sort of the first NP (a power of two, KPT <= NP <= 1024 * KPT) u64
// keys held KPT (4 or 8) per thread of a 1024-thread block (element KPT * thread + e in
// key[e]; elements past NP are left alone); s_buf (kSortLds = 4096 keys) is scratch for the
// cross-wave stages, which only NP > 64 * KPT needs (8 keys per thread: in two passes of 4).
// Every stage (K, J) is a compile-time instance (BitonicMerge / BitonicStages below):
// register partners stay static register names and lane partners constant shuffle masks,
// which a runtime stage loop turns into select chains and bpermute address arithmetic.
static_assert(kSortLds == 4096, "bitonic_desc's LDS passes hold 4 keys per thread of 1024");
template <int KPT, int K, int J>
__device__ __forceinline__ void bitonic_stage(uint64_t key[KPT], uint64_t *s_buf) {
    const int t = threadIdx.x;
    if constexpr (J >= 64 * KPT) {  // partner thread t ^ (J / KPT) in another wave: via LDS
#pragma unroll
        for (int h = 0; h < KPT; h += 4) {
            __syncthreads();  // earlier readers of s_buf are done
#pragma unroll
            for (int e = 0; e < 4; e++) s_buf[4 * t + e] = key[h + e];
            __syncthreads();
            const int tp = t ^ (J / KPT);
#pragma unroll
            for (int e = 0; e < 4; e++)
                key[h + e] = bitonic_pick(KPT * t + h + e, J, K, key[h + e], s_buf[4 * tp + e]);
        }
    } else if constexpr (J >= KPT) {  // partner thread t ^ (J / KPT), same slot, same wave
#pragma unroll
        for (int e = 0; e < KPT; e++)
            key[e] = bitonic_pick(KPT * t + e, J, K, key[e], lane_xor64<(J / KPT)>(key[e]));
    } else {  // partner slot e ^ J of this thread
        uint64_t nk[KPT];
#pragma unroll
        for (int e = 0; e < KPT; e++) nk[e] = bitonic_pick(KPT * t + e, J, K, key[e], key[e ^ J]);
#pragma unroll
        for (int e = 0; e < KPT; e++) key[e] = nk[e];
    }
}

template <int KPT, int K, int J>
struct BitonicStages {  // stages J, J / 2, ..., 1 of the merge of blocks of K
    __device__ __forceinline__ static void run(uint64_t key[KPT], uint64_t *s_buf) {
        bitonic_stage<KPT, K, J>(key, s_buf);
        BitonicStages<KPT, K, J / 2>::run(key, s_buf);
    }
};
template <int KPT, int K>
struct BitonicStages<KPT, K, 0> {
    __device__ __forceinline__ static void run(uint64_t *, uint64_t *) {}
};

template <int KPT, int K, int NP>
struct BitonicMerge {  // merges of block sizes K, 2K, ..., NP
    __device__ __forceinline__ static void run(uint64_t key[KPT], uint64_t *s_buf) {
        BitonicStages<KPT, K, K / 2>::run(key, s_buf);
        BitonicMerge<KPT, 2 * K, NP>::run(key, s_buf);
    }
};
template <int KPT, int NP>
struct BitonicMerge<KPT, 2 * NP, NP> {
    __device__ __forceinline__ static void run(uint64_t *, uint64_t *) {}
};

template <int KPT, int NP>
__device__ __forceinline__ void bitonic_desc_np(uint64_t key[KPT], uint64_t *s_buf) {
    BitonicMerge<KPT, 2, NP>::run(key, s_buf);
}

// seeds_sort_kernel sorts up to 256 seeds with the bitonic network inside one wave, and
// 257..4096 with bucket_desc (or radix_desc, below); the network for 512..4096 keys took 56k
// of a planted image's 77k sort cycles (round 4)

// the sort of the first np keys (np a power of two, rounded up to 4), 4 keys per thread;
// block-uniform np
__device__ void bitonic_desc(uint64_t key[4], uint64_t *s_buf, int np) {
    switch (np <= 4 ? 4 : np) {
    case 4: bitonic_desc_np<4, 4>(key, s_buf); break;
    case 8: bitonic_desc_np<4, 8>(key, s_buf); break;
    case 16: bitonic_desc_np<4, 16>(key, s_buf); break;
    case 32: bitonic_desc_np<4, 32>(key, s_buf); break;
    case 64: bitonic_desc_np<4, 64>(key, s_buf); break;
    case 128: bitonic_desc_np<4, 128>(key, s_buf); break;
    default: bitonic_desc_np<4, 256>(key, s_buf); break;  // np <= 256 here
    }
}

// exclusive prefix sum over one int per thread of a 1024-thread block (wave shuffles, then
// the 16 wave totals through LDS); `total` = the block's sum.  s_w holds 16 ints.
__device__ __forceinline__ int block_scan_1024(int v, int *s_w, int &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(incl, d);
        if (lane >= d) incl += u;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const int c = s_w[w];
        before += w < wave ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return before + incl - v;
}

// LSD radix sort of up to kSortLds keys, descending on key >> 27 = (v bits, field) and
// stable: equal (v, field) keep their order, emission order, which is what the low 27 bits
// (the inverted emission index) give the full-key sort too.  Keys are held 4 per thread,
// striped: key[e] of thread (wave w, lane l) is element 256 w + 64 e + l; padding keys are
// 0 and stay last.  Digits are 7 bits of (key >> 27) - min over the keys, as many passes
// as that range needs (4 for seeds above 0.5: 23 mantissa bits + 5 field bits).  A pass:
// each wave ranks its 256 keys by digit with 7 ballots (peers = the lanes holding the same
// digit) and a per-wave count per digit in LDS, one block scan over (digit, wave), a
// scatter into s_key.  The bitonic network needs 78 compare-exchange stages for 4096 keys
// (56k of its 77k cycles per planted image, PP_STAMPS); this needs 4 passes.  Leaves the
// sorted keys in s_key[0, n).
constexpr int kRadixBits = 7, kRadixDigits = 1 << kRadixBits;
// per-wave digit counts, a row per wave: a wave's lanes read / write their digits' counts
// in one row (2 u16 per bank word), and the row pitch of 65 words spreads the scan's
// (digit, wave) column reads over the banks; [digit][wave] put 16 lanes on one bank
constexpr int kRadixPitch = kRadixDigits + 2;
constexpr int kRadixMin = 256;  // up to here the bitonic network stays inside one wave

// inclusive prefix sum over the wave on DPP (row shifts, then row_bcast15 / row_bcast31
// carry the row totals), no LDS round trip
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// radix_desc's LDS: s_rh (16 rows of kRadixPitch u16), s_w (2 x 16 wave totals, one half
// per pass parity so a pass's scan needs no barrier after reading them), s_mm (32 u64)
__device__ void radix_desc(uint64_t key[4], int n, uint64_t *s_key, uint16_t *s_rh, int *s_w,
                           uint64_t *s_mm) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // waves past the last key hold padding only, in every pass (padding stays at positions
    // >= n): they count nothing (their rows are zero when scanned, which only moves the
    // offsets of their own padding) and neither scatter nor reload; the others reload
    // positions >= n as 0
    const bool keys_here = 256 * w < n;
    uint16_t *row = s_rh + w * kRadixPitch;  // wave w's counts; only wave w writes them
    // zero this wave's row (65 words), before the range reduction's barrier
    reinterpret_cast<uint32_t *>(row)[lane] = 0u;
    if (lane == 0) reinterpret_cast<uint32_t *>(row)[64] = 0u;
    // range of key >> 27 over the real keys
    uint64_t lo = ~0ull, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; e++)
        if (key[e]) {
            lo = min(lo, key[e] >> 27);
            hi = max(hi, key[e] >> 27);
        }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        lo = min(lo, shfl_xor64(lo, m));
        hi = max(hi, shfl_xor64(hi, m));
    }
    if (lane == 0) {
        s_mm[w] = lo;
        s_mm[16 + w] = hi;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; q++) {
        lo = min(lo, s_mm[q]);
        hi = max(hi, s_mm[16 + q]);
    }
    const uint64_t range = hi > lo ? hi - lo : 0;
    const int passes = range ? (64 - __clzll(range) + kRadixBits - 1) / kRadixBits : 0;
    const uint64_t below_mask = (1ull << lane) - 1;
    // the scan's entries of thread t: (digit t / 8, waves 2 (t % 8) and 2 (t % 8) + 1)
    uint16_t *own = s_rh + 2 * (t & 7) * kRadixPitch + (t >> 3);
    for (int p = 0; p < passes; p++) {  // block-uniform
        const int sh = p * kRadixBits;
        // ---- rank: wave w's 256 keys by digit, counts in row w (zero: see below) ----
        uint32_t dg[4], rk[4];
#pragma unroll
        for (int e = 0; e < 4 && keys_here; e++) {
            const uint64_t dk = key[e] ? (key[e] >> 27) - lo : 0ull;
            const uint32_t d = (kRadixDigits - 1) - (uint32_t)((dk >> sh) & (kRadixDigits - 1));
            uint64_t peers = ~0ull;
#pragma unroll
            for (int b = 0; b < kRadixBits; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bal = __ballot(bit);
                peers &= bit ? bal : ~bal;
            }
            uint16_t *c = row + d;
            const uint32_t old = *c;
            rk[e] = old + (uint32_t)__popcll(peers & below_mask);
            dg[e] = d;
            if (lane == 63 - __clzll(peers)) *c = (uint16_t)(old + (uint32_t)__popcll(peers));
        }
        __syncthreads();  // every row counted
        // ---- exclusive offsets over (digit, wave) ----
        const int c0 = own[0], c1 = own[kRadixPitch];
        const int v = c0 + c1;
        const int incl = wave_incl_scan(v);
        int *sw = s_w + 16 * (p & 1);
        if (lane == 63) sw[w] = incl;
        __syncthreads();
        int before = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) before += q < w ? sw[q] : 0;
        const int base = before + incl - v;
        own[0] = (uint16_t)base;
        own[kRadixPitch] = (uint16_t)(base + c0);
        __syncthreads();  // offsets written
        // ---- scatter; then wave w zeroes its row for the next pass (its own reads of the
        // row are done: LDS operations of one wave complete in order) ----
        if (keys_here) {
            uint32_t pos[4];
#pragma unroll
            for (int e = 0; e < 4; e++) pos[e] = row[dg[e]] + rk[e];
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (pos[e] < (uint32_t)n) s_key[pos[e]] = key[e];  // padding lands at >= n
        }
        // every wave: the scan wrote offsets into every row
        reinterpret_cast<uint32_t *>(row)[lane] = 0u;
        if (lane == 0) reinterpret_cast<uint32_t *>(row)[64] = 0u;
        __syncthreads();  // s_key complete
        if (p + 1 < passes && keys_here) {
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int i = 256 * w + 64 * e + lane;
                key[e] = i < n ? s_key[i] : 0ull;
            }
            // the next pass's scatter comes after its first barrier: these reads are done
        }
    }
    if (passes == 0) {  // one (v, field) value: emission order is the order
#pragma unroll
        for (int e = 0; e < 4; e++) s_key[256 * w + 64 * e + lane] = key[e];
        __syncthreads();
    }
}

// The sort of 257..4096 keys.  The full 64-bit keys are distinct (the low 27 bits hold the
// inverted emission index), so the order needs no stable pass: one bucket pass on the top
// kBucketBits bits of (key >> 27) - min (LDS atomics; positions inside a bucket arbitrary),
// then each key's rank inside its bucket by counting the bucket's larger keys.  Five barriers
// and one LDS round trip per key, where radix_desc's four or five stable 7-bit passes took
// 32k of a planted image's 55k sort cycles (tools/sort_stamps.py).  A bucket holds the keys
// of one (v, field) value or of a narrow range of them, and ranking costs its length squared
// in LDS reads: the bench's fields put at most 23 keys in a bucket, but saturated fields
// (many seeds of one v) can put thousands in one.  So when a bucket passes kBucketMax keys,
// bucket_desc returns false before it writes anything, and the caller sorts with radix_desc
// (its cost does not depend on ties).  s_hist: kBuckets + 1 ints; s_w: 16 ints; s_flag: 1
// int.  Leaves s_key[0, n) sorted when it returns true.
constexpr int kBucketBits = 11, kBuckets = 1 << kBucketBits;
constexpr int kBucketMax = 256;
static_assert(kBuckets == 2 * 1024, "bucket_desc: two bucket counts per thread");

// min / max over the wave on DPP (prefix within rows, then row_bcast15 / row_bcast31, as
// wave_incl_scan), read from lane 63
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xA, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xC, 0xF, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ bool bucket_desc(uint64_t key[4], int n, uint64_t *s_key, int *s_hist, int *s_w,
                            uint64_t *s_mm, int *s_flag) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    s_hist[2 * t] = 0;
    s_hist[2 * t + 1] = 0;
    if (t == 0) *s_flag = 0;
    // the range of key >> 27 bounded through the v bits (key >> 32) alone: lo = min v << 5,
    // hi = max v << 5 | 31 (32-bit reductions; at most one bit wider than the exact range)
    uint32_t lo32 = ~0u, hi32n = ~0u;  // min of v, min of ~v
#pragma unroll
    for (int e = 0; e < 4; e++)
        if (256 * w + 64 * e + lane < n) {
            lo32 = min(lo32, (uint32_t)(key[e] >> 32));
            hi32n = min(hi32n, ~(uint32_t)(key[e] >> 32));
        }
    lo32 = wave_min_u32(lo32);
    hi32n = wave_min_u32(hi32n);
    uint32_t *s_mm32 = reinterpret_cast<uint32_t *>(s_mm);
    if (lane == 0) {
        s_mm32[w] = lo32;
        s_mm32[16 + w] = hi32n;
    }
    __syncthreads();  // range parts + zeroed counts
#pragma unroll
    for (int q = 0; q < 16; q++) {
        lo32 = min(lo32, s_mm32[q]);
        hi32n = min(hi32n, s_mm32[16 + q]);
    }
    const uint64_t lo = (uint64_t)lo32 << 5, hi = ((uint64_t)~hi32n << 5) | 31u;
    const uint64_t range = hi > lo ? hi - lo : 0;
    const int bits = range ? 64 - __clzll(range) : 0;
    const int sh = bits > kBucketBits ? bits - kBucketBits : 0;
    // bucket, descending: larger keys in lower buckets
    int bk[4], at[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        bk[e] = -1;
        if (256 * w + 64 * e + lane < n) {
            bk[e] = (kBuckets - 1) - (int)(((key[e] >> 27) - lo) >> sh);
            at[e] = atomicAdd(&s_hist[bk[e]], 1);
            if (at[e] == kBucketMax) *s_flag = 1;  // a crowded bucket: radix_desc instead
        }
    }
    __syncthreads();  // counts complete
    if (*s_flag) return false;  // block-uniform; nothing written but the counts
    // bucket starts: thread t scans buckets 2t, 2t + 1 (block_scan_1024 has two barriers,
    // after which nobody reads the counts again)
    const int c0 = s_hist[2 * t], c1 = s_hist[2 * t + 1];
    int total;
    const int base = block_scan_1024(c0 + c1, s_w, total);
    s_hist[2 * t] = base;
    s_hist[2 * t + 1] = base + c0;
    if (t == 0) s_hist[kBuckets] = total;
    __syncthreads();  // starts written
    int st[4], en[4];
#pragma unroll
    for (int e = 0; e < 4; e++)
        if (bk[e] >= 0) {
            st[e] = s_hist[bk[e]];
            en[e] = s_hist[bk[e] + 1];
            s_key[st[e] + at[e]] = key[e];
        }
    __syncthreads();  // bucketed
    int pos[4];
#pragma unroll
    for (int e = 0; e < 4; e++)
        if (bk[e] >= 0) {
            int r = 0;
            for (int j = st[e]; j < en[e]; j++) r += s_key[j] > key[e];
            pos[e] = st[e] + r;
        }
    __syncthreads();  // every rank counted
#pragma unroll
    for (int e = 0; e < 4; e++)
        if (bk[e] >= 0) s_key[pos[e]] = key[e];
    __syncthreads();
    return true;
}

// 41 KB of LDS (keys, bucket counts, segment offsets; x / y / s stay in the emission
// buffer), so a workgroup fits beside a seed-loop workgroup on one CU (DecodePipeline
// overlaps them)
__global__ __launch_bounds__(1024) void seeds_sort_kernel(SeedArgs a) {
    __shared__ uint64_t s_key[kSortLds];
    // radix_desc's per-wave digit rows (u16) or bucket_desc's kBuckets + 1 counts
    __shared__ __attribute__((aligned(16))) int s_rh_i[kBuckets + 1];
    static_assert(kBuckets + 1 >= 16 * kRadixPitch / 2, "radix_desc's rows fit the counts");
    __shared__ int s_flag;
    uint16_t *s_rh = reinterpret_cast<uint16_t *>(s_rh_i);
    __shared__ int s_rw[32];
    __shared__ uint64_t s_mm[32];
    __shared__ int s_off[kMaxHeads * PP_MAX_KP + 1];
    __shared__ int s_sb[kMaxHeads * PP_MAX_KP];  // seg_base of each segment
    __shared__ int s_scan[16];
    static_assert(kRadixDigits * 16 == 2 * 1024, "radix_desc: two counts per thread");
    static_assert(kMaxHeads * PP_MAX_KP < 1024, "one thread per segment");
    const int img = blockIdx.x;
    SORT_STAMP(0);
    const int nseg = a.h.n_cif * a.K;
    const int64_t cap = a.cap;
    const float *gv = a.g_keys + (int64_t)img * 4 * cap, *gx = gv + cap, *gy = gx + cap,
                *gs = gy + cap;
    int *gf = a.g_f + (int64_t)img * cap;
    // segment offsets: every segment's count in one round trip, then a block scan
    // (s_off[nseg] = the total: counts past nseg are 0)
    {
        const int q = threadIdx.x;
        const int cnt = q < nseg ? a.f_counts[(int64_t)img * nseg + q] : 0;
        int total;
        const int pre = block_scan_1024(cnt, s_scan, total);
        if (q <= nseg) s_off[q] = pre;
        if (q < nseg) s_sb[q] = (int)a.seg_base_q(q);
        if (q == 0) a.counts[img] = total;
    }
    __syncthreads();
    const int n = s_off[nseg];
    SORT_STAMP(1);
#ifdef PP_STAMPS
    if (g_sort_stamps && threadIdx.x == 0) g_sort_stamps[blockIdx.x * 6 + 5] = (uint64_t)n;
#endif
    int np = 1;
    while (np < n) np <<= 1;
    pp_seed *out = a.seeds + (int64_t)img * cap;
    // emission slot of concatenated seed i: its segment by binary search over the offsets
    auto slot = [&](int i) __attribute__((always_inline)) {
        int lo = 0, hi = nseg - 1;  // largest segment with s_off[seg] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= i)
                lo = mid;
            else
                hi = mid - 1;
        }
        return (int64_t)s_sb[lo] + (i - s_off[lo]);
    };
    // the sorted keys kb[0 .. n) (LDS, or global scratch for more than kSortLds keys):
    // runs of equal (v, field) re-sorted by (x, y, s) descending, then emission order (one
    // thread per run, insertion sort), then the records written in order
    auto finish = [&](uint64_t *kb) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t ki = kb[i] >> 27;
            const bool tie_prev = i > 0 && (kb[i - 1] >> 27) == ki;
            const bool tie_next = i + 1 < n && (kb[i + 1] >> 27) == ki;
            if (tie_prev || !tie_next) continue;
            int end = i + 1;
            while (end < n && (kb[end] >> 27) == ki) end++;
            auto before = [&](uint64_t p, uint64_t q) {  // p must precede q
                const int ep = key_emit(p), eq = key_emit(q);
                const int64_t kp = slot(ep), kq = slot(eq);
                if (gx[kp] != gx[kq]) return gx[kp] > gx[kq];
                if (gy[kp] != gy[kq]) return gy[kp] > gy[kq];
                if (gs[kp] != gs[kq]) return gs[kp] > gs[kq];
                return ep < eq;
            };
            for (int u = i + 1; u < end; u++) {
                const uint64_t cur = kb[u];
                int w = u;
                while (w > i && before(cur, kb[w - 1])) {
                    kb[w] = kb[w - 1];
                    w--;
                }
                kb[w] = cur;
            }
        }
        __syncthreads();
        // four records per thread per round: every slot search and load issued before the
        // stores (one global round trip per round, not per record)
        for (int i0 = 0; i0 < n; i0 += 4 * (int)blockDim.x) {
            uint64_t k[4];
            int64_t e[4];
            float x[4], y[4], z[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * (int)blockDim.x + (int)threadIdx.x;
                k[u] = i < n ? kb[i] : 0ull;
                e[u] = i < n ? slot(key_emit(k[u])) : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * (int)blockDim.x + (int)threadIdx.x;
                if (i < n) {
                    x[u] = gx[e[u]];
                    y[u] = gy[e[u]];
                    z[u] = gs[e[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * (int)blockDim.x + (int)threadIdx.x;
                if (i < n) {
                    pp_seed r;
                    r.v = __uint_as_float((uint32_t)(k[u] >> 32));
                    r.field = (int)((k[u] >> 27) & 31u);
                    r.x = x[u];
                    r.y = y[u];
                    r.s = z[u];
                    out[i] = r;
                }
            }
        }
    };
    if (n > kRadixMin && n <= kSortLds) {
        // thread (w, l) gathers seeds 256 w + 64 e + l (one round trip), then radix_desc
        uint64_t key[4];
        const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int i = 256 * w + 64 * e + l;
            key[e] = 0ull;
            if (i < n) {
                const int64_t k = slot(i);
                key[e] = seed_key(gv[k], gf[k], i);
            }
        }
        SORT_STAMP(2);
        if (!bucket_desc(key, n, s_key, s_rh_i, s_rw, s_mm, &s_flag)) {
            __syncthreads();  // every thread has read the flag before radix_desc's rows
            radix_desc(key, n, s_key, s_rh, s_rw, s_mm);
        }
        SORT_STAMP(3);
        finish(s_key);
        __syncthreads();
        SORT_STAMP(4);
        return;
    }
    if (n <= kSortLds) {
        // thread t gathers seeds 4t .. 4t + 3 (all loads independent: one round trip), the
        // keys straight into registers
        uint64_t key[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int i = 4 * (int)threadIdx.x + e;
            key[e] = 0ull;  // past n: sorts last
            if (i < n) {
                const int64_t k = slot(i);
                key[e] = seed_key(gv[k], gf[k], i);
            }
        }
        // bitonic network, descending, on the first max(4, np) keys held 4 per thread (keys
        // past n are 0 and sort last): only the stages whose partner lies in another wave go
        // through LDS (np > 256; 10 of 78 at 4096); the others exchange in registers / across
        // lanes
        SORT_STAMP(2);
        bitonic_desc(key, s_key, np < 4 ? 4 : np);
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 4; e++) s_key[4 * threadIdx.x + e] = key[e];
        __syncthreads();
        SORT_STAMP(3);
        finish(s_key);
        __syncthreads();
        SORT_STAMP(4);
        return;
    }
    if (n <= 2 * kSortLds) {
        // 4096 < n <= 8192: the same network with 8 keys per thread (cross-wave stages in
        // two LDS passes), output straight from the registers, or, when a run of equal
        // (v, field) needs the full comparator's insertion sort, through global scratch
        uint64_t key[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const int i = 8 * (int)threadIdx.x + e;
            key[e] = 0ull;
            if (i < n) {
                const int64_t k = slot(i);
                key[e] = seed_key(gv[k], gf[k], i);
            }
        }
        bitonic_desc_np<8, 2 * kSortLds>(key, s_key);
        __syncthreads();
        s_key[threadIdx.x] = key[0];  // each thread's first key, for its predecessor
        __syncthreads();
        // keys are nonzero for real seeds (v > 0), zero past n
        bool tie = false;
#pragma unroll
        for (int e = 0; e < 7; e++)
            tie |= key[e + 1] != 0ull && (key[e] >> 27) == (key[e + 1] >> 27);
        if (threadIdx.x + 1 < blockDim.x) {
            const uint64_t nx = s_key[threadIdx.x + 1];
            tie |= nx != 0ull && (key[7] >> 27) == (nx >> 27);
        }
        if (!__syncthreads_or(tie)) {
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int i = 8 * (int)threadIdx.x + e;
                if (i >= n) continue;
                const uint64_t k = key[e];
                const int64_t q = slot(key_emit(k));
                pp_seed r;
                r.v = __uint_as_float((uint32_t)(k >> 32));
                r.field = (int)((k >> 27) & 31u);
                r.x = gx[q];
                r.y = gy[q];
                r.s = gs[q];
                out[i] = r;
            }
            return;
        }
        // ties: the sorted keys to global scratch (the permutation buffer holds 2 * np
        // ints = np keys), then as the LDS path
        uint64_t *gk = reinterpret_cast<uint64_t *>(a.g_perm + (int64_t)img * a.np_cap);
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const int i = 8 * (int)threadIdx.x + e;
            if (i < n) gk[i] = key[e];
        }
        __syncthreads();
        finish(gk);
        return;
    }
    {
        // large seed sets: network over a permutation in global memory; keys are read
        // through an emission-index -> slot map
        int *perm = a.g_perm + (int64_t)img * a.np_cap;
        int *loc = perm + np;  // second half of the permutation buffer
        for (int q = 0; q < nseg; q++) {
            const int o = s_off[q], c = s_off[q + 1] - o;
            const int64_t sb = s_sb[q];
            for (int i = threadIdx.x; i < c; i += blockDim.x) loc[o + i] = (int)(sb + i);
        }
        for (int i = threadIdx.x; i < np; i += blockDim.x) perm[i] = i;
        __syncthreads();
        SeedKeys keys{gv, gx, gy, gs, gf, loc, n};
        bitonic_sort(perm, np, keys);
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int k = loc[perm[i]];
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
    Heads h;            // CafScored.fill visits the heads in order (caf_scored.py:88-98)
    HrMap hr;
    int K, C;
    int64_t col_cap;    // columns per set (>= cells of all heads)
    float cif_floor, one_minus_floor;
    int nt;             // number of thresholds (1 or 2)
    float th[2];
    float *cols[2];     // (n_img, C, 2, 9, col_cap): dir 0 backward, 1 forward
    int *counts[2];     // (n_img, C, 2)
    const int *gate;    // (n_img) or NULL: images with gate 0 are skipped (empty sets)
    int j1[kMaxCaf], j2[kMaxCaf];
};

// caf_scored.py:46-56: the min / max distance masks of head m on the raw (unstrided) vectors
__device__ __forceinline__ bool caf_distance_ok(const Heads &h, int m, const float *p, int64_t hw,
                                                int64_t cell) {
    const bool on_min = (h.dmin_on >> m) & 1u, on_max = (h.dmax_on >> m) & 1u;
    if (!on_min && !on_max) return true;
    const float dx = p[1 * hw + cell] - p[5 * hw + cell], dy = p[2 * hw + cell] - p[6 * hw + cell];
    const float dist = sqrtf(dx * dx + dy * dy);  // np.linalg.norm(nine[1:3] - nine[5:7], axis=0)
    if (on_min && !(dist > h.dmin_th[m])) return false;
    if (on_max && !(dist < h.dmax_th[m])) return false;
    return true;
}

__global__ __launch_bounds__(256) void caf_scored_kernel(CafArgs a) {
    __shared__ int s_tmp[4];
    const int64_t fld = blockIdx.x;  // image * C + caf field
    const int img = (int)(fld / a.C), ci = (int)(fld % a.C);
    if (a.gate && !a.gate[img]) {
        if (threadIdx.x < a.nt * 2) a.counts[threadIdx.x >> 1][fld * 2 + (threadIdx.x & 1)] = 0;
        return;
    }
    const int j1i = a.j1[ci], j2i = a.j2[ci];
    const bool use1 = a.cif_floor < 1.0f && j1i < a.K;
    const bool use2 = a.cif_floor < 1.0f && j2i < a.K;
    const int64_t t1 = (int64_t)img * a.K + (use1 ? j1i : 0);
    const int64_t t2 = (int64_t)img * a.K + (use2 ? j2i : 0);
    const int64_t cc = a.col_cap;
    int run_b[2] = {0, 0}, run_f[2] = {0, 0};
    const float th_min = a.nt == 2 ? fminf(a.th[0], a.th[1]) : a.th[0];
    for (int m = 0; m < a.h.n_caf; m++) {
        const int hw = a.h.aH[m] * a.h.aW[m];
        const float stride = (float)a.h.astride[m];
        const float *p = a.h.caf[m] + fld * 9 * hw;
        for (int base = 0; base < hw; base += 256) {
            const int cell = base + threadIdx.x;
            float nine[9];
            float sb = 0.0f, sf = 0.0f;
            bool any = false;
            if (cell < hw) {
                nine[0] = p[cell];
                any = nine[0] > th_min && caf_distance_ok(a.h, m, p, hw, cell);
                if (any) {
#pragma unroll
                    for (int r = 1; r < 9; r++) nine[r] = p[r * hw + cell] * stride;
                    const float score = nine[0];
                    sb = score;
                    sf = score;
                    if (use1)
                        sb = score * (a.cif_floor +
                                      a.one_minus_floor * a.hr.at(t1, nine[1], nine[2], 0.0f));
                    if (use2)
                        sf = score * (a.cif_floor +
                                      a.one_minus_floor * a.hr.at(t2, nine[5], nine[6], 0.0f));
                }
            }
            for (int t = 0; t < a.nt; t++) {
                const float th = a.th[t];
                const bool pass = any && nine[0] > th;  // mask = nine[0] > score_th
                const bool kb = pass && sb > th, kf = pass && sf > th;
                int tot_b, tot_f;
                const int slot_b = block_compact<4>(kb, s_tmp, tot_b);
                const int slot_f = block_compact<4>(kf, s_tmp, tot_f);
                float *bwd = a.cols[t] + (fld * 2 + 0) * 9 * cc;
                float *fwd = a.cols[t] + (fld * 2 + 1) * 9 * cc;
                if (kb) {
                    // backward rows (0, 5, 6, 7, 8, 1, 2, 3, 4) with row 0 = scores_b
                    const int64_t c = run_b[t] + slot_b;
                    bwd[c] = sb;
                    bwd[1 * cc + c] = nine[5];
                    bwd[2 * cc + c] = nine[6];
                    bwd[3 * cc + c] = nine[7];
                    bwd[4 * cc + c] = nine[8];
                    bwd[5 * cc + c] = nine[1];
                    bwd[6 * cc + c] = nine[2];
                    bwd[7 * cc + c] = nine[3];
                    bwd[8 * cc + c] = nine[4];
                }
                if (kf) {
                    const int64_t c = run_f[t] + slot_f;
                    fwd[c] = sf;
#pragma unroll
                    for (int r = 1; r < 9; r++) fwd[r * cc + c] = nine[r];
                }
                run_b[t] += tot_b;
                run_f[t] += tot_f;
            }
        }
    }
    if (threadIdx.x == 0) {
        for (int t = 0; t < a.nt; t++) {
            a.counts[t][fld * 2 + 0] = run_b[t];
            a.counts[t][fld * 2 + 1] = run_f[t];
        }
    }
}

// ------------------------------------------------------------------------------------
// CafScored for the device decoder: the same column sets, stored bucketed by SOURCE
// position so that caf_center_s (functional.pyx:338-359) in the grow kernel only visits
// the buckets its 2*scale box overlaps.  Row 9 keeps each column's index in the
// reference's row-major order, which is what ties are broken on; `offs` holds the
// bucket boundaries (bucket grid bw x bh of e x e px, plus one bucket for NaN sources).
// ------------------------------------------------------------------------------------
constexpr int kMaxBuckets = 1600 + 1;

struct CafBArgs {
    Heads h;
    HrMap hr;
    int K, C;
    int64_t col_cap;    // columns per set: cells of all heads
    float cif_floor, one_minus_floor, th;
    int bw, bh, nb;     // bucket grid and bucket count (bw * bh + 1)
    float inv_e;        // 1 / bucket edge (a power of two: exact)
    float *cols;        // (n_img, C, 2, kColRows, col_cap): dir 0 backward, 1 forward
    int *offs;          // (n_img, C, 2, nb + 1)
    // (n_img) or NULL: bitmask of the joints force-complete may still set.  Completion
    // only evaluates connections INTO unset joints (cifcaf.py:253, 272), so a direction
    // whose target joint is set everywhere is never read and its set is left empty.
    const int *gate;
    int j1[kMaxCaf], j2[kMaxCaf];
};

__device__ __forceinline__ int caf_bucket(float x, float y, int bw, int bh, float inv_e) {
    if (x != x || y != y) return bw * bh;  // NaN sources pass every box test: own bucket
    const int bx = (int)fminf(fmaxf(floorf(x * inv_e), 0.0f), (float)(bw - 1));
    const int by = (int)fminf(fmaxf(floorf(y * inv_e), 0.0f), (float)(bh - 1));
    return by * bw + bx;
}

// INDEX_ONLY (the force-complete set): bucket the cell index of every cell with c > th by
// its source position and store nothing else.  The rescoring by CifHr and the second
// threshold (caf_scored.py:63-81) are applied by the query (grow.hip, consider_raw) to the
// few columns in its box; both filters commute with the bucketing and the tie-break key is
// the cell index either way.
//
// STASH: the fields are read ONCE.  Pass 1 scores the cells, builds the bucket histograms
// and keeps what pass 2 scatters in LDS: for set A the kept columns themselves (any order:
// the grow kernel's merge ignores the order inside a bucket), for set B each cell's two
// bucket ids.  A set-A stash that overflows (more than kStashA kept columns in a direction)
// makes pass 2 recompute from the fields, as the non-STASH kernel always does.
constexpr int kStashA = 256;      // kept columns per direction (set A stash): 29 KB of LDS, 5 workgroups per CU
// Set A, one head: pass 1 first lists the cells above the threshold (confidence plane only,
// kConfU loads per thread in flight), then reads the other rows and the CifHr values of the
// listed cells only: three memory round trips per workgroup instead of three per
// NT * kU cells.  More than kCandA cells fall back to the batched scan.
constexpr int kCandA = 1024;
constexpr int kConfU = 16;
constexpr int kStashCells = kSetBIdx16Max; // cells of all heads (set B stash: u16 bucket per direction)
constexpr uint16_t kNoBucket = 0xFFFF;

struct StashCol {
    float v[7];  // score, source x, y, target x, y, target scale, index bits
    int bucket;
};

template <bool INDEX_ONLY, bool STASH>
__global__ __launch_bounds__(STASH && INDEX_ONLY ? 512 : 256) void caf_bucketed_kernel(CafBArgs a) {
    constexpr int NT = STASH && INDEX_ONLY ? 512 : 256;
    constexpr int NW = NT / 64;
    // The set-B build (PK) keeps its LDS small enough to run beside a seed-loop workgroup
    // (whose LDS leaves ~38 KB of a CU): bucket counts / cursors as u16 pairs (a bucket holds
    // at most kStashCells cells), and the stash sized by the launch to the field's cells.
    constexpr bool PK = INDEX_ONLY && STASH;
    __shared__ int s_cnt[2][PK ? (kMaxBuckets + 2) / 2 : kMaxBuckets + 1];
    __shared__ int s_wsum[2][NW];
    __shared__ __attribute__((aligned(16))) char s_stash[STASH && !INDEX_ONLY ? 2 * kStashA * (int)sizeof(StashCol) : 16];
    extern __shared__ __attribute__((aligned(16))) char s_dyn[];  // PK: 2 * col_cap u16
    __shared__ int s_sn[2], s_ovf, s_nc;
    constexpr bool kList = STASH && !INDEX_ONLY;
    __shared__ int s_cand[kList ? kCandA : 1];
    __shared__ float s_cand_c[kList ? kCandA : 1];
    StashCol *stash_a = reinterpret_cast<StashCol *>(s_stash);       // [2][kStashA]
    uint16_t *stash_b = reinterpret_cast<uint16_t *>(s_dyn);         // [2][col_cap]
    const int scell = (int)a.col_cap;                                 // stash_b's direction stride
    // bucket b of direction d: add one (returns the old count / cursor), read
    auto h_add = [&](int d, int b) -> int {
        if constexpr (PK) {
            const unsigned sh = (unsigned)(b & 1) * 16u;
            return (int)((atomicAdd(reinterpret_cast<unsigned *>(&s_cnt[d][b >> 1]), 1u << sh) >> sh) & 0xFFFFu);
        } else {
            return atomicAdd(&s_cnt[d][b], 1);
        }
    };
    auto h_get = [&](int d, int b) -> int {
        if constexpr (PK) return (int)(((unsigned)s_cnt[d][b >> 1] >> ((b & 1) * 16)) & 0xFFFFu);
        else return s_cnt[d][b];
    };
    const int64_t fld = blockIdx.x;  // image * C + caf field
    const int img = (int)(fld / a.C), ci = (int)(fld % a.C);
    const int nb = a.nb;
    int *offs_b = a.offs + (fld * 2 + 0) * (int64_t)(nb + 1);
    int *offs_f = a.offs + (fld * 2 + 1) * (int64_t)(nb + 1);
    const int j1i = a.j1[ci], j2i = a.j2[ci];
    // backward columns end at j1, forward ones at j2
    const bool need_b = !a.gate || ((a.gate[img] >> j1i) & 1);
    const bool need_f = !a.gate || ((a.gate[img] >> j2i) & 1);
    if (!need_b && !need_f) {
        for (int i = threadIdx.x; i <= nb; i += NT) {
            offs_b[i] = 0;
            offs_f[i] = 0;
        }
        return;
    }
    const bool use1 = need_b && a.cif_floor < 1.0f && j1i < a.K;
    const bool use2 = need_f && a.cif_floor < 1.0f && j2i < a.K;
    const int64_t t1 = (int64_t)img * a.K + (use1 ? j1i : 0);
    const int64_t t2 = (int64_t)img * a.K + (use2 ? j2i : 0);
    for (int i = threadIdx.x; i < (PK ? (nb + 2) / 2 : nb + 1); i += NT) {
        s_cnt[0][i] = 0;
        s_cnt[1][i] = 0;
    }
    if (threadIdx.x == 0) {
        s_sn[0] = s_sn[1] = 0;
        s_ovf = 0;
        s_nc = 0;
    }
    __syncthreads();

    // caf_scored.py:42-81 (both directions) for kU cells per thread of head m at once:
    // cells base + k * NT + tid.  The loads of the batch (confidences, then the rows of
    // passing cells, then the CifHr lookups) are issued together, so one batch costs three
    // memory round trips instead of three per cell.
    constexpr int kU = INDEX_ONLY ? 8 : 4;
    struct Batch {
        float nine[kU][9];
        float sb[kU], sf[kU];
        bool kb[kU], kf[kU];
    };
    auto score_batch = [&](const float *p, int hw, float stride, int m, int base, Batch &B) {
        const bool on_min = (a.h.dmin_on >> m) & 1u, on_max = (a.h.dmax_on >> m) & 1u;
#pragma unroll
        for (int k = 0; k < kU; k++) {
            const int cell = base + k * NT + (int)threadIdx.x;
            B.nine[k][0] = cell < hw ? p[cell] : NAN;  // NaN: never > score_th
            B.kb[k] = B.kf[k] = false;
        }
#pragma unroll
        for (int k = 0; k < kU; k++) {
            const int cell = base + k * NT + (int)threadIdx.x;
            if (!(B.nine[k][0] > a.th)) continue;  // mask = nine[0] > score_th
#pragma unroll
            for (int r = 1; r < 9; r++) {
                const bool need = (r == 1 || r == 2 || r == 5 || r == 6) ||
                                  (!INDEX_ONLY && (r == 4 || r == 8));
                B.nine[k][r] = need ? p[r * hw + cell] : 0.0f;  // b1, b2 are never read
            }
        }
#pragma unroll
        for (int k = 0; k < kU; k++) {
            if (!(B.nine[k][0] > a.th)) continue;
            if (on_min || on_max) {  // caf_scored.py:46-56 on the raw (unstrided) vectors
                const float dx = B.nine[k][1] - B.nine[k][5], dy = B.nine[k][2] - B.nine[k][6];
                const float dist = sqrtf(dx * dx + dy * dy);
                if ((on_min && !(dist > a.h.dmin_th[m])) || (on_max && !(dist < a.h.dmax_th[m])))
                    continue;
            }
#pragma unroll
            for (int r = 1; r < 9; r++) B.nine[k][r] = B.nine[k][r] * stride;
            if (INDEX_ONLY) {  // source positions only: forward (x1, y1), backward (x2, y2)
                B.kb[k] = need_b;
                B.kf[k] = need_f;
                continue;
            }
            const float score = B.nine[k][0];
            float sb = score, sf = score;
            if (use1)
                sb = score * (a.cif_floor + a.one_minus_floor * a.hr.at(t1, B.nine[k][1], B.nine[k][2], 0.0f));
            if (use2)
                sf = score * (a.cif_floor + a.one_minus_floor * a.hr.at(t2, B.nine[k][5], B.nine[k][6], 0.0f));
            B.sb[k] = sb;
            B.sf[k] = sf;
            B.kb[k] = need_b && sb > a.th;
            B.kf[k] = need_f && sf > a.th;
        }
    };

    // pass 1: bucket histograms (backward sources are (x2, y2), forward (x1, y1)); no
    // barrier inside the loop, so the cells' loads overlap freely
    // one scored cell of pass 1: histogram counts and the stash
    auto account = [&](const Batch &B, int k, int cell, int hw, int coff) {
        const float *nine = B.nine[k];
        const int bkb = B.kb[k] ? caf_bucket(nine[5], nine[6], a.bw, a.bh, a.inv_e) : -1;
        const int bkf = B.kf[k] ? caf_bucket(nine[1], nine[2], a.bw, a.bh, a.inv_e) : -1;
        if (bkb >= 0) h_add(0, bkb);
        if (bkf >= 0) h_add(1, bkf);
        if (STASH && INDEX_ONLY) {
            if (cell < hw) {
                stash_b[coff + cell] = bkb >= 0 ? (uint16_t)bkb : kNoBucket;
                stash_b[scell + coff + cell] = bkf >= 0 ? (uint16_t)bkf : kNoBucket;
            }
        } else if (STASH) {
            const float key = __int_as_float(coff + cell);
            if (bkb >= 0) {
                const int sl = atomicAdd(&s_sn[0], 1);
                if (sl < kStashA) {
                    StashCol &e = stash_a[sl];
                    e.v[0] = B.sb[k];
                    e.v[1] = nine[5];
                    e.v[2] = nine[6];
                    e.v[3] = nine[1];
                    e.v[4] = nine[2];
                    e.v[5] = nine[4];
                    e.v[6] = key;
                    e.bucket = bkb;
                } else {
                    s_ovf = 1;
                }
            }
            if (bkf >= 0) {
                const int sl = atomicAdd(&s_sn[1], 1);
                if (sl < kStashA) {
                    StashCol &e = stash_a[kStashA + sl];
                    e.v[0] = B.sf[k];
                    e.v[1] = nine[1];
                    e.v[2] = nine[2];
                    e.v[3] = nine[5];
                    e.v[4] = nine[6];
                    e.v[5] = nine[8];
                    e.v[6] = key;
                    e.bucket = bkf;
                } else {
                    s_ovf = 1;
                }
            }
        }
    };

    bool listed = false;
    if (kList && a.h.n_caf == 1) {
        // list the cells above the threshold (confidence plane only)
        const int hw = a.h.aH[0] * a.h.aW[0];
        const float *p = a.h.caf[0] + fld * 9 * hw;
        const int lane = threadIdx.x & 63;
        for (int base = 0; base < hw; base += NT * kConfU) {
            float v[kConfU];
#pragma unroll
            for (int k = 0; k < kConfU; k++) {
                const int cell = base + k * NT + (int)threadIdx.x;
                v[k] = cell < hw ? p[cell] : NAN;
            }
#pragma unroll
            for (int k = 0; k < kConfU; k++) {
                const bool pass = v[k] > a.th;  // mask = nine[0] > score_th
                const uint64_t bm = __ballot(pass);
                if (!bm) continue;
                int wb = 0;
                if (lane == 0) wb = atomicAdd(&s_nc, __popcll(bm));
                wb = __shfl(wb, 0);
                if (pass) {
                    const int i = wb + __popcll(bm & ((1ull << lane) - 1));
                    if (i < kCandA) {
                        s_cand[i] = base + k * NT + (int)threadIdx.x;
                        s_cand_c[i] = v[k];
                    }
                }
            }
        }
        __syncthreads();
        listed = s_nc <= kCandA;
    }
    if (listed) {
        const int n = s_nc;
        const int hw = a.h.aH[0] * a.h.aW[0];
        const float stride = (float)a.h.astride[0];
        const float *p = a.h.caf[0] + fld * 9 * hw;
        const int coff = (int)a.h.caf_off[0];
        const bool on_min = a.h.dmin_on & 1u, on_max = a.h.dmax_on & 1u;
        for (int i0 = 0; i0 < n; i0 += NT * kU) {
            Batch B;
            int cells[kU];
#pragma unroll
            for (int k = 0; k < kU; k++) {
                const int i = i0 + k * NT + (int)threadIdx.x;
                cells[k] = i < n ? s_cand[i] : 0;
                B.nine[k][0] = i < n ? s_cand_c[i] : NAN;
                B.kb[k] = B.kf[k] = false;
            }
#pragma unroll
            for (int k = 0; k < kU; k++) {
                if (!(B.nine[k][0] > a.th)) continue;
#pragma unroll
                for (int r = 1; r < 9; r++) {
                    const bool need = r == 1 || r == 2 || r == 4 || r == 5 || r == 6 || r == 8;
                    B.nine[k][r] = need ? p[r * hw + cells[k]] : 0.0f;  // b1, b2 never read
                }
            }
#pragma unroll
            for (int k = 0; k < kU; k++) {
                if (!(B.nine[k][0] > a.th)) continue;
                if (on_min || on_max) {  // caf_scored.py:46-56 on the raw (unstrided) vectors
                    const float dx = B.nine[k][1] - B.nine[k][5], dy = B.nine[k][2] - B.nine[k][6];
                    const float dist = sqrtf(dx * dx + dy * dy);
                    if ((on_min && !(dist > a.h.dmin_th[0])) || (on_max && !(dist < a.h.dmax_th[0])))
                        continue;
                }
#pragma unroll
                for (int r = 1; r < 9; r++) B.nine[k][r] = B.nine[k][r] * stride;
                const float score = B.nine[k][0];
                float sb = score, sf = score;
                if (use1)
                    sb = score * (a.cif_floor + a.one_minus_floor * a.hr.at(t1, B.nine[k][1], B.nine[k][2], 0.0f));
                if (use2)
                    sf = score * (a.cif_floor + a.one_minus_floor * a.hr.at(t2, B.nine[k][5], B.nine[k][6], 0.0f));
                B.sb[k] = sb;
                B.sf[k] = sf;
                B.kb[k] = need_b && sb > a.th;
                B.kf[k] = need_f && sf > a.th;
            }
#pragma unroll
            for (int k = 0; k < kU; k++) account(B, k, cells[k], hw, coff);
        }
    } else {
    for (int m = 0; m < a.h.n_caf; m++) {
        const int hw = a.h.aH[m] * a.h.aW[m];
        const float stride = (float)a.h.astride[m];
        const float *p = a.h.caf[m] + fld * 9 * hw;
        const int coff = (int)a.h.caf_off[m];
        for (int base = 0; base < hw; base += NT * kU) {
            Batch B;
            score_batch(p, hw, stride, m, base, B);
#pragma unroll
            for (int k = 0; k < kU; k++) account(B, k, base + k * NT + (int)threadIdx.x, hw, coff);
        }
    }
    }
    __syncthreads();
    // exclusive prefix over the buckets (thread-contiguous ranges + block scan); PK: even
    // ranges, so that each thread owns the u16 pairs of its range
    const int per = PK ? (((nb + NT - 1) / NT + 1) & ~1) : (nb + NT - 1) / NT;
    const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    int sum[2] = {0, 0};
    for (int d = 0; d < 2; d++)
        for (int i = b0; i < b1; i++) sum[d] += h_get(d, i);
    int incl[2];
    for (int d = 0; d < 2; d++) {
        int v = sum[d];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(v, off);
            if ((threadIdx.x & 63) >= off) v += o;
        }
        incl[d] = v;
        if ((threadIdx.x & 63) == 63) s_wsum[d][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    for (int d = 0; d < 2; d++) {
        int base = incl[d] - sum[d];
        for (int w = 0; w < (int)(threadIdx.x >> 6); w++) base += s_wsum[d][w];
        int *offs = d == 0 ? offs_b : offs_f;
        if constexpr (PK) {
            for (int i = b0; i < b1; i += 2) {  // the pair (i, i + 1) becomes two cursors
                const unsigned w = (unsigned)s_cnt[d][i >> 1];
                const int c0 = (int)(w & 0xFFFFu), c1 = i + 1 < b1 ? (int)(w >> 16) : 0;
                offs[i] = base;
                if (i + 1 < b1) offs[i + 1] = base + c0;
                s_cnt[d][i >> 1] = (int)((unsigned)base | ((unsigned)(base + c0) << 16));
                base += c0 + c1;
            }
        } else {
            for (int i = b0; i < b1; i++) {
                const int c = s_cnt[d][i];
                s_cnt[d][i] = base;  // becomes the bucket cursor
                offs[i] = base;
                base += c;
            }
        }
        if (threadIdx.x == NT - 1) {
            int tot = 0;
            for (int w = 0; w < NW; w++) tot += s_wsum[d][w];
            offs[nb] = tot;
        }
    }
    __syncthreads();

    // pass 2: scatter into buckets.  A column's tie-break key is its concatenated cell index
    // (cell_off[m] + row-major cell): it orders the kept columns exactly as their rank in the
    // reference's concatenated array does, and the grow kernel's merge is independent of the
    // order inside a bucket.
    const int rows = INDEX_ONLY ? 1 : kColRows;
    const int64_t cc = a.col_cap;
    float *bwd = a.cols + (fld * 2 + 0) * rows * cc;
    float *fwd = a.cols + (fld * 2 + 1) * rows * cc;
    if (STASH && INDEX_ONLY) {
        const int ncell = (int)cc;
        for (int cell = threadIdx.x; cell < ncell; cell += NT) {
            const uint16_t bb = stash_b[cell], bf = stash_b[scell + cell];
            // u16 cell indices (cells <= kSetBIdx16Max): half the bytes to write and to read
            if (bb != kNoBucket) reinterpret_cast<uint16_t *>(bwd)[h_add(0, bb)] = (uint16_t)cell;
            if (bf != kNoBucket) reinterpret_cast<uint16_t *>(fwd)[h_add(1, bf)] = (uint16_t)cell;
        }
        return;
    }
    if (STASH && !s_ovf) {
        for (int d = 0; d < 2; d++) {
            float *out = d ? fwd : bwd;
            const int n = s_sn[d];
            for (int i = threadIdx.x; i < n; i += NT) {
                const StashCol &e = stash_a[d * kStashA + i];
                const int64_t c = atomicAdd(&s_cnt[d][e.bucket], 1);
#pragma unroll
                for (int r = 0; r < kColRows; r++) out[r * cc + c] = e.v[r];
            }
        }
        return;
    }
    for (int m = 0; m < a.h.n_caf; m++) {
        const int hw = a.h.aH[m] * a.h.aW[m];
        const float stride = (float)a.h.astride[m];
        const float *p = a.h.caf[m] + fld * 9 * hw;
        const int coff = (int)a.h.caf_off[m];
        for (int base = 0; base < hw; base += NT * kU) {
            Batch B;
            score_batch(p, hw, stride, m, base, B);
#pragma unroll
            for (int k = 0; k < kU; k++) {
                const int key = coff + base + k * NT + (int)threadIdx.x;
                const float *nine = B.nine[k];
                if (INDEX_ONLY) {
                    if (B.kb[k])
                        reinterpret_cast<int *>(bwd)[atomicAdd(
                            &s_cnt[0][caf_bucket(nine[5], nine[6], a.bw, a.bh, a.inv_e)], 1)] = key;
                    if (B.kf[k])
                        reinterpret_cast<int *>(fwd)[atomicAdd(
                            &s_cnt[1][caf_bucket(nine[1], nine[2], a.bw, a.bh, a.inv_e)], 1)] = key;
                    continue;
                }
                // the kColRows rows the grow kernel reads: score, source x, y, target x, y,
                // target scale, index.  Backward sets are the reference's rows (0, 5, 6, 7, 8,
                // 1, 2, 3, 4) with row 0 = scores_b, so their source is (x2, y2) and their
                // target (x1, y1, s1).
                if (B.kb[k]) {
                    const int64_t c = atomicAdd(&s_cnt[0][caf_bucket(nine[5], nine[6], a.bw, a.bh, a.inv_e)], 1);
                    bwd[c] = B.sb[k];
                    bwd[1 * cc + c] = nine[5];
                    bwd[2 * cc + c] = nine[6];
                    bwd[3 * cc + c] = nine[1];
                    bwd[4 * cc + c] = nine[2];
                    bwd[5 * cc + c] = nine[4];
                    bwd[6 * cc + c] = __int_as_float(key);
                }
                if (B.kf[k]) {
                    const int64_t c = atomicAdd(&s_cnt[1][caf_bucket(nine[1], nine[2], a.bw, a.bh, a.inv_e)], 1);
                    fwd[c] = B.sf[k];
                    fwd[1 * cc + c] = nine[1];
                    fwd[2 * cc + c] = nine[2];
                    fwd[3 * cc + c] = nine[5];
                    fwd[4 * cc + c] = nine[6];
                    fwd[5 * cc + c] = nine[8];
                    fwd[6 * cc + c] = __int_as_float(key);
                }
            }
        }
    }
}

static inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

SeedSink seed_sink(int n_img, int K, const pp_config *cfg, int cap, void *scratch) {
    SeedSink k{};
    char *w = (char *)scratch;
    k.g_keys = (float *)w;
    w += round_up((int64_t)n_img * 4 * cap * sizeof(float), 256);
    k.g_f = (int *)w;
    w += round_up((int64_t)n_img * cap * sizeof(int), 256);
    k.f_counts = (int *)w;
    k.cap = cap;
    k.K = K;
    k.th = cfg->seed_threshold;
    k.score_scale = cfg->seed_score_scale;
    k.skip = cfg->seed_skip_mask;
    return k;
}

// `emitted`: the decoder's CifHr kernel already wrote the seed segments (cifhr_fuses_seeds,
// SeedSink): only the sort runs
int launch_seeds(const Heads &h, const HrMap &hr, int n_img, int K, const pp_config *cfg,
                 pp_seed *seeds, int cap, int *counts, void *scratch, hipStream_t s,
                 bool emitted) {
    if (K > PP_MAX_KP) return fail(PP_ESHAPE, "seeds: more than PP_MAX_KP CIF fields");
    if ((int64_t)cap < (int64_t)K * h.cif_cells())
        return fail(PP_ESHAPE, "seeds: capacity < K * cells");
    SeedArgs a{};
    a.h = h;
    a.hr = hr;
    a.K = K;
    a.th = cfg->seed_threshold;
    a.score_scale = cfg->seed_score_scale;
    a.skip = cfg->seed_skip_mask;
    a.seeds = seeds;
    a.cap = cap;
    a.counts = counts;
    int np = 1;
    while (np < cap) np <<= 1;
    a.np_cap = 2 * np;
    char *w = (char *)scratch;
    a.g_keys = (float *)w;
    w += round_up((int64_t)n_img * 4 * cap * sizeof(float), 256);
    a.g_f = (int *)w;
    w += round_up((int64_t)n_img * cap * sizeof(int), 256);
    a.f_counts = (int *)w;
    w += round_up((int64_t)n_img * kMaxHeads * PP_MAX_KP * sizeof(int), 256);
    a.g_perm = (int *)w;
    if (!emitted)
        hipLaunchKernelGGL(seeds_emit_kernel, dim3((unsigned)((int64_t)n_img * h.n_cif * K)), dim3(256), 0, s, a);
#ifdef PP_STAMPS
    uint64_t *st = nullptr;
    hipMalloc((void **)&st, (size_t)n_img * 6 * sizeof(uint64_t));
    hipMemsetAsync(st, 0, (size_t)n_img * 6 * sizeof(uint64_t), s);
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sort_stamps), &st, sizeof(st), 0, hipMemcpyHostToDevice, s);
#endif
    hipLaunchKernelGGL(seeds_sort_kernel, dim3(n_img), dim3(1024), 0, s, a);
#ifdef PP_STAMPS
    {
        hipStreamSynchronize(s);
        std::vector<uint64_t> hb((size_t)n_img * 6);
        hipMemcpy(hb.data(), st, hb.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
        const char *path = getenv("PP_SORT_STAMPS_OUT");
        FILE *fo = fopen(path ? path : "pp_sort_stamps.bin", "ab");
        if (fo) {
            fwrite(hb.data(), sizeof(uint64_t), hb.size(), fo);
            fclose(fo);
        }
        uint64_t *nul = nullptr;
        hipMemcpyToSymbol(HIP_SYMBOL(g_sort_stamps), &nul, sizeof(nul));
        hipFree(st);
    }
#endif
    return check_launch("pp_seeds");
}

size_t seeds_scratch_size(int n_img, int cap) {
    int64_t np = 1;
    while (np < cap) np <<= 1;
    return round_up((int64_t)n_img * 4 * cap * sizeof(float), 256) +
           round_up((int64_t)n_img * cap * sizeof(int), 256) +
           round_up((int64_t)n_img * kMaxHeads * PP_MAX_KP * sizeof(int), 256) +
           round_up((int64_t)n_img * 2 * np * sizeof(int), 256);
}

int launch_caf_scored(const Heads &h, const HrMap &hr, int n_img, int K, int C,
                      const int32_t *skeleton, const pp_config *cfg, int nt, const float *th,
                      float *const *cols, int64_t col_cap, int *const *counts, hipStream_t s,
                      const int *gate) {
    if (C > kMaxCaf) return fail(PP_ESHAPE, "caf_scored: more than PP_MAX_EDGES CAF fields");
    if (col_cap < h.caf_cells()) return fail(PP_ESHAPE, "caf_scored: column capacity < cells");
    CafArgs a{};
    a.h = h;
    a.hr = hr;
    a.K = K;
    a.C = C;
    a.col_cap = col_cap;
    a.cif_floor = cfg->cif_floor;
    a.one_minus_floor = (float)(1.0 - (double)cfg->cif_floor);  // (1.0 - self.cif_floor)
    a.nt = nt;
    a.gate = gate;
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

// bucket geometry for the CifHr map (head 0): edge e = stride * 2^k px with <= 1600 buckets
void caf_bucket_grid(int H, int W, int stride, int *bw, int *bh, int *nb, float *inv_e) {
    const int hh = (int)hr_dim(H, stride), ww = (int)hr_dim(W, stride);
    int e = stride;
    while (((hh + e - 1) / e) * ((ww + e - 1) / e) > kMaxBuckets - 1) e *= 2;
    *bw = (ww + e - 1) / e;
    *bh = (hh + e - 1) / e;
    *nb = *bw * *bh + 1;
    *inv_e = 1.0f / (float)e;
}

int launch_caf_bucketed(const Heads &h, const HrMap &hr, int n_img, int K, int C,
                        const int32_t *skeleton, const pp_config *cfg, float th, float *cols,
                        int *offs, const int *gate, bool index_only, hipStream_t s) {
    if (C > kMaxCaf) return fail(PP_ESHAPE, "caf_scored: more than PP_MAX_EDGES CAF fields");
    CafBArgs a{};
    a.h = h;
    a.hr = hr;
    a.K = K;
    a.C = C;
    a.col_cap = h.caf_cells();
    a.cif_floor = cfg->cif_floor;
    a.one_minus_floor = (float)(1.0 - (double)cfg->cif_floor);
    a.th = th;
    caf_bucket_grid(h.cH[0], h.cW[0], h.cstride[0], &a.bw, &a.bh, &a.nb, &a.inv_e);
    a.cols = cols;
    a.offs = offs;
    a.gate = gate;
    for (int i = 0; i < C; i++) {
        a.j1[i] = skeleton[2 * i] - 1;
        a.j2[i] = skeleton[2 * i + 1] - 1;
    }
    const dim3 grid((unsigned)((int64_t)n_img * C));
    if (index_only && a.col_cap <= kStashCells)
        hipLaunchKernelGGL((caf_bucketed_kernel<true, true>), grid, dim3(512),
                           (size_t)(2 * a.col_cap * sizeof(uint16_t)), s, a);
    else if (index_only)
        hipLaunchKernelGGL((caf_bucketed_kernel<true, false>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((caf_bucketed_kernel<false, true>), grid, dim3(256), 0, s, a);
    return check_launch("caf_scored(bucketed)");
}

}  // namespace pp

using namespace pp;

extern "C" {

static int seeds_entry(const Heads &h, const float *d_cifhr, int32_t n_img, int32_t K,
                       const pp_config *cfg, pp_seed *d_seeds, int32_t seed_capacity,
                       int32_t *d_counts, void *stream) {
    if (!d_cifhr || !cfg || !d_seeds || !d_counts) return fail(PP_EINVAL, "pp_seeds: NULL argument");
    if (n_img < 0 || K <= 0 || seed_capacity <= 0) return fail(PP_ESHAPE, "pp_seeds: bad shape");
    if (n_img == 0) return PP_OK;
    void *scratch = nullptr;
    hipStream_t s = (hipStream_t)stream;
    if (hipMallocAsync(&scratch, seeds_scratch_size(n_img, seed_capacity), s) != hipSuccess)
        return fail(PP_EHIP, "pp_seeds: scratch allocation failed");
    const HrMap hr = dense_hr(d_cifhr, h.hr_hh, h.hr_ww);
    int rc = launch_seeds(h, hr, n_img, K, cfg, d_seeds, seed_capacity, d_counts, scratch, s,
                          false);
    if (hipFreeAsync(scratch, s) != hipSuccess && rc == PP_OK)
        rc = fail(PP_EHIP, "pp_seeds: scratch release failed");
    return rc;
}

int pp_seeds(const float *d_cif, const float *d_cifhr, int32_t n_img, int32_t K, int32_t H,
             int32_t W, const pp_config *cfg, pp_seed *d_seeds, int32_t seed_capacity,
             int32_t *d_counts, void *stream) {
    if (!d_cif || !cfg) return fail(PP_EINVAL, "pp_seeds: NULL argument");
    if (H <= 0 || W <= 0 || cfg->stride <= 0) return fail(PP_ESHAPE, "pp_seeds: bad shape");
    return seeds_entry(single_head(d_cif, nullptr, H, W, cfg->stride), d_cifhr, n_img, K, cfg,
                       d_seeds, seed_capacity, d_counts, stream);
}

int pp_seeds_multi(const pp_scale *scales, int32_t n_scales, const float *d_cifhr, int32_t n_img,
                   int32_t K, const pp_config *cfg, pp_seed *d_seeds, int32_t seed_capacity,
                   int32_t *d_counts, void *stream) {
    Heads h;
    const int rc = make_heads(scales, n_scales, 0, PP_ROLE_CIF, &h, "pp_seeds_multi");
    if (rc) return rc;
    for (int m = 0; m < h.n_cif; m++)
        if (!h.cif[m]) return fail(PP_EINVAL, "pp_seeds_multi: NULL field");
    return seeds_entry(h, d_cifhr, n_img, K, cfg, d_seeds, seed_capacity, d_counts, stream);
}

int pp_caf_scored(const float *d_caf, const float *d_cifhr, int32_t n_img, int32_t K, int32_t C,
                  int32_t H, int32_t W, const int32_t *skeleton, float score_th,
                  const pp_config *cfg, float *d_cols, int32_t *d_counts, void *stream) {
    if (!d_caf || !d_cifhr || !skeleton || !cfg || !d_cols || !d_counts)
        return fail(PP_EINVAL, "pp_caf_scored: NULL argument");
    if (n_img < 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0 || cfg->stride <= 0)
        return fail(PP_ESHAPE, "pp_caf_scored: bad shape");
    if (n_img == 0) return PP_OK;
    float *cols[1] = {d_cols};
    int *counts[1] = {d_counts};
    return launch_caf_scored(single_head(nullptr, d_caf, H, W, cfg->stride),
                             dense_hr(d_cifhr, (int)hr_dim(H, cfg->stride), (int)hr_dim(W, cfg->stride)),
                             n_img, K, C, skeleton, cfg, 1, &score_th, cols, (int64_t)H * W, counts,
                             (hipStream_t)stream, nullptr);
}

int pp_caf_scored_multi(const pp_scale *scales, int32_t n_scales, const float *d_cifhr,
                        int32_t n_img, int32_t K, int32_t C, const int32_t *skeleton,
                        float score_th, const pp_config *cfg, float *d_cols,
                        int64_t col_capacity, int32_t *d_counts, void *stream) {
    Heads h;
    // CIF head 0 (or a PP_ROLE_HRMAP entry) gives the CifHr map's geometry; CIF fields are
    // not read
    const int rc = make_heads(scales, n_scales, 0, PP_ROLE_CAF, &h, "pp_caf_scored_multi");
    if (rc) return rc;
    if (h.hr_hh <= 0) return fail(PP_EINVAL, "pp_caf_scored_multi: no CIF head or PP_ROLE_HRMAP entry");
    if (!d_cifhr || !skeleton || !cfg || !d_cols || !d_counts)
        return fail(PP_EINVAL, "pp_caf_scored_multi: NULL argument");
    for (int m = 0; m < h.n_caf; m++)
        if (!h.caf[m]) return fail(PP_EINVAL, "pp_caf_scored_multi: NULL field");
    if (n_img < 0 || K <= 0 || C <= 0) return fail(PP_ESHAPE, "pp_caf_scored_multi: bad shape");
    if (n_img == 0) return PP_OK;
    float *cols[1] = {d_cols};
    int *counts[1] = {d_counts};
    return launch_caf_scored(h,
                             dense_hr(d_cifhr, h.hr_hh, h.hr_ww),
                             n_img, K, C, skeleton, cfg, 1, &score_th, cols, col_capacity, counts,
                             (hipStream_t)stream, nullptr);
}

}  // extern "C"
