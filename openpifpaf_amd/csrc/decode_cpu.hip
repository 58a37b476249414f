// decode_cpu.hip — host twin of the whole CifCaf decode (pp_decode_batch_cpu): the seed loop
// with its occupancy, the frontier grow, force-complete with the flood fill, and
// nms.Keypoints, after the front stages' host twins (stages_cpu.hip), on host pointers.
//
// SURVEY.md §7 asks for a C++ CPU twin of every kernel and §8(d) decodes cfg1 "with the CPU
// twin": this is that path for a batch of one-head fields, and bench.py's `cpu_baseline`
// (kind "twin").  Nothing falls back to it: the decoder computes on the device and raises
// without one; openpifpaf_amd.stages_cpu.decode_batch names this path explicitly.
//
// The arithmetic is the reference's, in its order, and the device's: the per-element
// helpers are pp_common.hpp's (np_exp_f32 / np_pow2_f32 for the scores, hr_lookup,
// occupancy_mark_box, clip_ref).  The column queries differ from the reference only in
// which columns they visit: a set's columns are indexed by source y (NaN sources apart), so
// a query scans the rows its 2 * scale box spans instead of every column; the top-2 merge
// ranks (score, column index) keys exactly as the stable argsort / argmax do, so the visiting
// order never matters.  Images run in parallel on `n_threads` host threads.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "pp_common.hpp"

namespace {

using pp::clip_ref;

// by_source (cifcaf.py:62-65): per start joint, its (end, CAF, forward) entries in dict
// insertion order; a later duplicate key overwrites the value in place
struct BySource {
    int n[PP_MAX_KP] = {};
    int end[PP_MAX_KP][PP_MAX_KP];
    int caf[PP_MAX_KP][PP_MAX_KP];
    bool fwd[PP_MAX_KP][PP_MAX_KP];

    BySource(const int32_t *skeleton, int C) {
        for (int ci = 0; ci < C; ci++) {
            const int j1 = skeleton[2 * ci] - 1, j2 = skeleton[2 * ci + 1] - 1;
            put(j1, j2, ci, true);
            put(j2, j1, ci, false);
        }
    }
    void put(int s, int e, int ci, bool f) {
        int at = -1;
        for (int i = 0; i < n[s]; i++)
            if (end[s][i] == e) at = i;
        if (at < 0) at = n[s]++;
        end[s][at] = e;
        caf[s][at] = ci;
        fwd[s][at] = f;
    }
};

// one CafScored direction set (pp_caf_scored_cpu layout: rows 0 score, 1-2 source, 5-6
// target, 8 target scale; pitch hw) with its columns ordered by source y for the queries
struct ColSet {
    const float *rows = nullptr;
    int64_t pitch = 0;
    int n = 0;
    std::vector<int> by_y;   // columns with a number as source y, ascending y
    std::vector<float> ys;   // their y
    std::vector<int> nan_y;  // columns whose source y is NaN (every y test passes them)

    void index(const float *r, int64_t p, int count) {
        rows = r;
        pitch = p;
        n = count;
        by_y.clear();
        nan_y.clear();
        for (int i = 0; i < n; i++) {
            if (r[2 * p + i] != r[2 * p + i])
                nan_y.push_back(i);
            else
                by_y.push_back(i);
        }
        std::stable_sort(by_y.begin(), by_y.end(),
                         [&](int a, int b) { return r[2 * p + a] < r[2 * p + b]; });
        ys.resize(by_y.size());
        for (size_t i = 0; i < by_y.size(); i++) ys[i] = r[2 * p + by_y[i]];
    }
};

// top-2 key of a candidate column: the score's bits above (scores are >= 0, so float order
// is integer order; NaN, last in np.argsort and first for np.argmax, above every number),
// the column index below (blend: a stable ascending argsort ranks equal scores by index,
// so the higher index wins; max: np.argmax takes the first maximum)
inline uint64_t cand_key(float score, int i, bool maxm) {
    const uint32_t hi = score != score ? 0xFFFFFFFFu : pp::u32_of(score);
    const uint32_t lo = maxm ? (uint32_t)(0x7FFFFFFF - i) : (uint32_t)(i + 1);
    return ((uint64_t)hi << 32) | lo;
}

inline float key_score(uint64_t k) { return pp::f32_of((uint32_t)(k >> 32)); }

// _grow_connection + _target_with_blend / _target_with_maxscore (cifcaf.py:124-192)
void grow_connection(const ColSet &s, float x, float y, float xy_scale, bool maxm, int exp_mode,
                     float out[4]) {
    const float sbox = 2.0f * xy_scale;  // caf_center_s(..., sigma=2.0 * xy_scale)
    const float lo_x = x - sbox, hi_x = x + sbox, lo_y = y - sbox, hi_y = y + sbox;
    const float sigma = 0.5f * xy_scale;
    const float sigma2 = pp::np_pow2_f32(sigma);
    const float *r = s.rows;
    const int64_t p = s.pitch;
    uint64_t k1 = 0, k2 = 0;
    int i1 = -1, i2 = -1;
    auto consider = [&](int i) {
        const float c1 = r[p + i], c2 = r[2 * p + i];
        if (c1 < lo_x || c1 > hi_x || c2 < lo_y || c2 > hi_y) return;
        const float dx = x - c1, dy = y - c2;
        const float dd = std::sqrt(dx * dx + dy * dy);  // np.linalg.norm(axis=0)
        const float score = pp::caf_exp((-0.5f * (dd * dd)) / sigma2, exp_mode) * r[i];
        const uint64_t k = cand_key(score, i, maxm);
        if (k > k1) {
            k2 = k1;
            i2 = i1;
            k1 = k;
            i1 = i;
        } else if (k > k2) {
            k2 = k;
            i2 = i;
        }
    };
    if (lo_x != lo_x || hi_x != hi_x || lo_y != lo_y || hi_y != hi_y) {
        for (int i = 0; i < s.n; i++) consider(i);  // NaN bounds pass every column
    } else {
        const auto b = std::lower_bound(s.ys.begin(), s.ys.end(), lo_y);
        const auto e = std::upper_bound(b, s.ys.end(), hi_y);
        for (auto it = b; it != e; ++it) consider(s.by_y[it - s.ys.begin()]);
        for (int i : s.nan_y) consider(i);
    }
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    if (i1 < 0) return;  // caf_field.shape[1] == 0
    const float *tx = r + 5 * p, *ty = r + 6 * p, *ts = r + 8 * p;
    const float s1 = key_score(k1);
    if (maxm || i2 < 0) {  // argmax, or len(scores) == 1: scores[0] * 0.5
        out[0] = tx[i1];
        out[1] = ty[i1];
        out[2] = ts[i1];
        out[3] = maxm ? s1 : s1 * 0.5f;
        return;
    }
    const float s2 = key_score(k2);
    if (s2 < 0.01f || s2 < 0.5f * s1) {
        out[0] = tx[i1];
        out[1] = ty[i1];
        out[2] = ts[i1];
        out[3] = s1 * 0.5f;
        return;
    }
    const float ex = tx[i1] - tx[i2], ey = ty[i1] - ty[i2];
    const float d = std::sqrt(ex * ex + ey * ey);
    if (d > ts[i1] / 2.0f) {
        out[0] = tx[i1];
        out[1] = ty[i1];
        out[2] = ts[i1];
        out[3] = s1 * 0.5f;
        return;
    }
    const float ssum = s1 + s2;
    out[0] = (s1 * tx[i1] + s2 * tx[i2]) / ssum;
    out[1] = (s1 * ty[i1] + s2 * ty[i2]) / ssum;
    out[2] = (s1 * ts[i1] + s2 * ts[i2]) / ssum;
    out[3] = 0.5f * (s1 + s2);
}

inline float max0(float v) { return v > 0.0f ? v : 0.0f; }  // max(0.0, v)

// frontier entry (-score, None | xysv, start, end) (cifcaf.py:261, 285); a None / tuple tie
// would raise TypeError in the reference (never in a successful run): None first here
struct FEntry {
    float neg;
    bool eval;
    float xysv[4];
    int j, k;
};

inline bool fentry_greater(const FEntry &a, const FEntry &b) {  // for a min-heap
    if (a.neg != b.neg) return a.neg > b.neg;
    if (a.eval != b.eval) return a.eval > b.eval;
    if (a.eval)
        for (int t = 0; t < 4; t++)
            if (a.xysv[t] != b.xysv[t]) return a.xysv[t] > b.xysv[t];
    if (a.j != b.j) return a.j > b.j;
    return a.k > b.k;
}

// flood-fill entry (-v, end, start xyv, s) (cifcaf.py:317)
struct FFEntry {
    float neg;
    int end;
    float sxyv[3];
    float s;
};

inline bool ffentry_greater(const FFEntry &a, const FFEntry &b) {
    if (a.neg != b.neg) return a.neg > b.neg;
    if (a.end != b.end) return a.end > b.end;
    for (int t = 0; t < 3; t++)
        if (a.sxyv[t] != b.sxyv[t]) return a.sxyv[t] > b.sxyv[t];
    return a.s > b.s;
}

struct Decoder {
    const pp_config &cfg;
    const BySource &bs;
    int K, C;
    const std::vector<ColSet> *sets = nullptr;  // (C, 2): dir 0 backward, 1 forward
    std::vector<FEntry> heap;

    Decoder(const pp_config &c, const BySource &b, int k, int nc) : cfg(c), bs(b), K(k), C(nc) {}

    // cifcaf.py:194-217 (set: the current CafScored, reverse_match as the caller asks)
    void connection_value(const pp_ann &a, int start, int e, bool reverse_match, float out[4]) {
        const int ci = bs.caf[start][e];
        const bool fwd = bs.fwd[start][e];
        const ColSet &sf = (*sets)[2 * ci + (fwd ? 1 : 0)], &sb = (*sets)[2 * ci + (fwd ? 0 : 1)];
        const bool maxm = cfg.connection_method == 1;
        const float *xyv = a.data[start];
        const float xy_scale_s = max0(a.joint_scales[start]);
        float nx[4];
        grow_connection(sf, xyv[0], xyv[1], xy_scale_s, maxm, cfg.exp_mode, nx);
        out[0] = out[1] = out[2] = out[3] = 0.0f;
        const float ks = std::sqrt(nx[3] * xyv[2]);  // geometric mean
        if (ks < cfg.keypoint_threshold) return;
        if (nx[3] == 0.0f) return;
        const float xy_scale_t = max0(nx[2]);
        if (reverse_match) {
            float rv[4];
            grow_connection(sb, nx[0], nx[1], xy_scale_t, maxm, cfg.exp_mode, rv);
            if (rv[2] == 0.0f) return;  // tests the scale (cifcaf.py:212)
            if (std::fabs(xyv[0] - rv[0]) + std::fabs(xyv[1] - rv[1]) > xy_scale_s) return;
        }
        out[0] = nx[0];
        out[1] = nx[1];
        out[2] = nx[2];
        out[3] = ks;
    }

    // _grow (cifcaf.py:247-307); false when a record list overflowed
    bool grow(pp_ann &a, bool reverse_match) {
        heap.clear();
        bool in_frontier[PP_MAX_KP][PP_MAX_KP] = {};
        bool ok = true;
        auto push = [&](const FEntry &x) {
            heap.push_back(x);
            std::push_heap(heap.begin(), heap.end(), fentry_greater);
        };
        auto add_to_frontier = [&](int start) {
            for (int e = 0; e < bs.n[start]; e++) {
                const int end = bs.end[start][e];
                if (a.data[end][2] > 0.0f) continue;
                if (in_frontier[start][end]) continue;
                FEntry x{};
                const float mps = std::sqrt(a.data[start][2]);  // max_possible_score
                x.neg = cfg.confidence_scales ? -(mps * cfg.confidence_scales[bs.caf[start][e]]) : -mps;
                x.eval = false;
                x.j = start;
                x.k = end;
                push(x);
                in_frontier[start][end] = true;
                if (a.n_frontier < PP_MAX_FRONTIER) {
                    a.frontier_pairs[a.n_frontier][0] = (uint8_t)start;
                    a.frontier_pairs[a.n_frontier][1] = (uint8_t)end;
                } else {
                    ok = false;
                }
                a.n_frontier++;
            }
        };
        auto edge_of = [&](int start, int end) {
            for (int e = 0; e < bs.n[start]; e++)
                if (bs.end[start][e] == end) return e;
            return -1;
        };
        for (int j = 0; j < K; j++)
            if (a.data[j][2] != 0.0f) add_to_frontier(j);
        for (;;) {
            FEntry got{};
            bool have = false;
            while (!heap.empty()) {  // frontier_get (cifcaf.py:265-285)
                std::pop_heap(heap.begin(), heap.end(), fentry_greater);
                FEntry en = heap.back();
                heap.pop_back();
                if (en.eval) {
                    got = en;
                    have = true;
                    break;
                }
                if (a.data[en.k][2] > 0.0f) continue;
                const int e = edge_of(en.j, en.k);
                float nx[4];
                connection_value(a, en.j, e, reverse_match, nx);
                if (nx[3] == 0.0f) continue;
                FEntry ev = en;
                ev.eval = true;
                std::memcpy(ev.xysv, nx, sizeof(nx));
                float score = nx[3];
                if (cfg.greedy) {
                    ev.neg = -score;
                    got = ev;
                    have = true;
                    break;
                }
                if (cfg.confidence_scales) score = score * cfg.confidence_scales[bs.caf[en.j][e]];
                ev.neg = -score;
                push(ev);
            }
            if (!have) break;
            const int jsi = got.j, jti = got.k;
            if (a.data[jti][2] > 0.0f) continue;
            a.data[jti][0] = got.xysv[0];
            a.data[jti][1] = got.xysv[1];
            a.data[jti][2] = got.xysv[3];
            a.joint_scales[jti] = got.xysv[2];
            if (a.n_decoding < PP_MAX_KP) {
                const int t = a.n_decoding;
                a.decoding_pairs[t][0] = (uint8_t)jsi;
                a.decoding_pairs[t][1] = (uint8_t)jti;
                std::memcpy(&a.decoding_xyv[t][0], a.data[jsi], 3 * sizeof(float));
                std::memcpy(&a.decoding_xyv[t][3], a.data[jti], 3 * sizeof(float));
            } else {
                ok = false;
            }
            a.n_decoding++;
            add_to_frontier(jti);
        }
        return ok;
    }

    // _flood_fill (cifcaf.py:309-331): the key is the ENCLOSING xyv's v (App. D item 5)
    void flood_fill(pp_ann &a) {
        std::vector<FFEntry> h;
        auto add = [&](int start, float key_v) {
            for (int e = 0; e < bs.n[start]; e++) {
                const int end = bs.end[start][e];
                if (a.data[end][2] > 0.0f) continue;
                FFEntry x;
                x.neg = -key_v;
                x.end = end;
                std::memcpy(x.sxyv, a.data[start], 3 * sizeof(float));
                x.s = a.joint_scales[start];
                h.push_back(x);
                std::push_heap(h.begin(), h.end(), ffentry_greater);
            }
        };
        for (int j = 0; j < K; j++)
            if (a.data[j][2] != 0.0f) add(j, a.data[j][2]);
        while (!h.empty()) {
            std::pop_heap(h.begin(), h.end(), ffentry_greater);
            const FFEntry top = h.back();
            h.pop_back();
            if (a.data[top.end][2] > 0.0f) continue;
            a.data[top.end][0] = top.sxyv[0];
            a.data[top.end][1] = top.sxyv[1];
            a.data[top.end][2] = 0.00001f;
            a.joint_scales[top.end] = top.s;
            add(top.end, top.sxyv[2]);
        }
    }
};

// the seed loop's Occupancy(cifhr.shape, 2, min_scale=4) (cifcaf.py:84, occupancy.py)
struct Occ {
    std::vector<uint8_t> p;
    int64_t h = 0, w = 0;
    int K = 0;
    float red = 2.0f, msr = 2.0f;
    bool get(int f, float x, float y) const {  // occupancy.py:41-47
        if (f >= K) return true;
        if (h <= 0 || w <= 0) return false;  // the reference reads out of bounds here
        const int64_t xi = (int64_t)clip_ref(x / red, 0.0f, (float)(w - 1));
        const int64_t yi = (int64_t)clip_ref(y / red, 0.0f, (float)(h - 1));
        return p[((int64_t)f * h + yi) * w + xi] != 0;
    }
    void set(int f, float x, float y, float s) {  // occupancy.py:31-39, utils.py:61-66
        int64_t x0, x1, y0, y1;
        if (!pp::occupancy_mark_box(f, K, h, w, x, y, s, red, msr, x0, x1, y0, y1)) return;
        for (int64_t yy = y0; yy < y1; yy++)
            for (int64_t xx = x0; xx < x1; xx++) {
                uint8_t &c = p[((int64_t)f * h + yy) * w + xx];
                c = (uint8_t)(c + 1);
            }
    }
};

// per-thread scratch of one image's decode
struct Scratch {
    std::vector<float> cifhr, cols_a, cols_b;
    std::vector<int32_t> cnt_a, cnt_b;
    std::vector<pp_seed> seeds;
    std::vector<ColSet> sets_a, sets_b;
    std::vector<pp_ann> work;
};

// one image: CifCaf.__call__ (cifcaf.py:67-122) with the front stages' host twins
int decode_image(const float *cif, const float *caf, int K, int C, int H, int W,
                 const int32_t *skeleton, const pp_config &cfg, const BySource &bs,
                 pp_ann *out, int cap, int32_t *count, int32_t *status, Scratch &S) {
    const int64_t hw = (int64_t)H * W;
    const int64_t hh = pp::hr_dim(H, cfg.stride), ww = pp::hr_dim(W, cfg.stride);
    const int64_t pitch = (ww + 31) / 32 * 32;
    S.cifhr.resize((size_t)K * hh * pitch);
    int rc = pp_cifhr_cpu(cif, 1, K, H, W, &cfg, S.cifhr.data());
    if (rc) return rc;
    const int seed_cap = (int)std::min<int64_t>((int64_t)K * hw, INT32_MAX);
    S.seeds.resize((size_t)seed_cap);
    int32_t n_seeds = 0;
    rc = pp_seeds_cpu(cif, S.cifhr.data(), 1, K, H, W, &cfg, S.seeds.data(), seed_cap, &n_seeds);
    if (rc) return rc;
    auto build_sets = [&](float th, std::vector<float> &cols, std::vector<int32_t> &cnt,
                          std::vector<ColSet> &sets) {
        cols.resize((size_t)C * 2 * 9 * hw);
        cnt.resize((size_t)C * 2);
        const int r = pp_caf_scored_cpu(caf, S.cifhr.data(), 1, K, C, H, W, skeleton, th, &cfg,
                                        cols.data(), cnt.data());
        if (r) return r;
        sets.resize((size_t)C * 2);
        for (int q = 0; q < 2 * C; q++) sets[q].index(cols.data() + (int64_t)q * 9 * hw, hw, cnt[q]);
        return (int)PP_OK;
    };
    rc = build_sets(cfg.caf_threshold, S.cols_a, S.cnt_a, S.sets_a);
    if (rc) return rc;
    Decoder dec(cfg, bs, K, C);
    dec.sets = &S.sets_a;
    Occ occ;
    occ.K = K;
    occ.red = (float)cfg.occupancy_reduction;
    occ.msr = (float)((double)cfg.occupancy_min_scale / cfg.occupancy_reduction);
    occ.h = (int64_t)((double)hh / cfg.occupancy_reduction);  // int(shape[1] / reduction)
    occ.w = (int64_t)((double)ww / cfg.occupancy_reduction);
    occ.p.assign((size_t)(K * occ.h * occ.w), 0);
    S.work.clear();
    int st = 0;
    for (int i = 0; i < n_seeds; i++) {  // cifcaf.py:100-108
        const pp_seed &sd = S.seeds[i];
        if (occ.get(sd.field, sd.x, sd.y)) continue;
        if ((int)S.work.size() >= cap) {
            st |= PP_ST_ANN_OVERFLOW;
            break;
        }
        pp_ann a;
        std::memset(&a, 0, sizeof(a));
        a.n_keypoints = K;
        a.data[sd.field][0] = sd.x;
        a.data[sd.field][1] = sd.y;
        a.data[sd.field][2] = sd.v;
        a.joint_scales[sd.field] = sd.s;
        if (!dec.grow(a, true)) st |= PP_ST_DEC_OVERFLOW;
        S.work.push_back(a);
        for (int j = 0; j < K; j++)  // mark_occupied (cifcaf.py:87-93)
            if (a.data[j][2] != 0.0f) occ.set(j, a.data[j][0], a.data[j][1], a.joint_scales[j]);
    }
    if (cfg.force_complete) {  // complete_annotations (cifcaf.py:333-351)
        rc = build_sets(cfg.complete_caf_threshold, S.cols_b, S.cnt_b, S.sets_b);
        if (rc) return rc;
        dec.sets = &S.sets_b;
        for (pp_ann &a : S.work) {
            bool unfilled[PP_MAX_KP];
            for (int j = 0; j < K; j++) unfilled[j] = a.data[j][2] == 0.0f;
            if (!dec.grow(a, false)) st |= PP_ST_DEC_OVERFLOW;
            bool any_zero = false;
            for (int j = 0; j < K; j++) {
                if (unfilled[j] && a.data[j][2] > 0.0f)
                    a.data[j][2] = std::min(0.001f, a.data[j][2]);  // np.minimum(0.001, v)
                any_zero = any_zero || a.data[j][2] == 0.0f;
            }
            if (any_zero) dec.flood_fill(a);
        }
    }
    const int32_t n = (int32_t)S.work.size();
    if (n == 0) {
        *count = 0;
    } else if (cfg.apply_nms) {  // nms.Keypoints (nms.py:17-57)
        rc = pp_nms_keypoints_cpu(S.work.data(), &n, 1, K, std::max(1, n), &cfg, out, count,
                                  nullptr);
        if (rc) return rc;
    } else {
        for (int32_t i = 0; i < n; i++) {
            out[i] = S.work[i];
            out[i].score = pp::ann_score_cpu(out[i], K);
        }
        *count = n;
    }
    *status = st;
    return PP_OK;
}

}  // namespace

extern "C" {

int pp_decode_batch_cpu(const float *cif, const float *caf, int32_t n_img, int32_t K, int32_t C,
                        int32_t H, int32_t W, const int32_t *skeleton, const pp_config *cfg,
                        pp_ann *anns, int32_t ann_capacity, int32_t *counts, int32_t *status,
                        int32_t n_threads) {
    if (!cif || !caf || !skeleton || !cfg || !anns || !counts || !status)
        return pp::fail(PP_EINVAL, "pp_decode_batch_cpu: NULL argument");
    if (n_img < 0 || K <= 0 || K > PP_MAX_KP || C <= 0 || C > PP_MAX_EDGES || H <= 0 || W <= 0 ||
        ann_capacity <= 0 || cfg->stride <= 0 || cfg->occupancy_reduction <= 0)
        return pp::fail(PP_ESHAPE, "pp_decode_batch_cpu: shape outside the supported envelope");
    if (cfg->connection_method != 0 && cfg->connection_method != 1)
        return pp::fail(PP_EINVAL, "connection method not known");
    for (int i = 0; i < 2 * C; i++)
        if (skeleton[i] < 1 || skeleton[i] > K)
            return pp::fail(PP_EINVAL, "pp_decode_batch_cpu: skeleton joint index out of 1..K");
    if (n_img == 0) return PP_OK;
    const BySource bs(skeleton, C);
    const int64_t hw = (int64_t)H * W;
    int threads = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    threads = std::max(1, std::min(threads, (int)n_img));
    std::atomic<int> next{0};
    std::atomic<int> err{PP_OK};
    auto worker = [&]() {
        Scratch S;
        for (;;) {
            const int img = next.fetch_add(1);
            if (img >= n_img || err.load() != PP_OK) return;
            const int rc = decode_image(cif + (int64_t)img * K * 5 * hw, caf + (int64_t)img * C * 9 * hw,
                                        K, C, H, W, skeleton, *cfg, bs,
                                        anns + (int64_t)img * ann_capacity, ann_capacity,
                                        counts + img, status + img, S);
            if (rc != PP_OK) err.store(rc);
        }
    };
    if (threads == 1) {
        worker();
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
    }
    return err.load();
}

}  // extern "C"
