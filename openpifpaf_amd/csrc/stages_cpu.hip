// stages_cpu.hip — host twins of the decoder's front stages (pp_cifhr_cpu, pp_seeds_cpu,
// pp_caf_scored_cpu): CifHr.fill, CifSeeds.fill + get and CafScored.fill for one CIF and one
// CAF head, with the device forms' layouts (pp_cifhr / pp_seeds / pp_caf_scored) but host
// pointers, run on the calling thread.
//
// As functional_cpu.hip does for the primitives, these exist for callers holding host
// buffers (the reference's stage classes are CPU-only: cif_hr.py, cif_seeds.py,
// caf_scored.py); no product path reaches them by fallback.  The arithmetic is the
// reference's, in its order: the CifHr splats go through the primitive's host twin
// (pp_scalar_square_add_gauss_with_max_cpu), the lookups through pp_common.hpp's hr_lookup,
// and the seed order is the device sort's (u64 keys, then the full tuple comparator on runs
// of equal (v, field)).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "pp_common.hpp"

namespace {

struct HrGeom {
    int64_t hh, ww, pitch;
};

HrGeom hr_geom(int H, int W, int stride) {
    HrGeom g;
    g.hh = pp::hr_dim(H, stride);
    g.ww = pp::hr_dim(W, stride);
    g.pitch = (g.ww + 31) / 32 * 32;  // pp_cifhr_pitch
    return g;
}

bool bad_cfg(const pp_config *cfg) { return !cfg || cfg->stride <= 0; }

constexpr uint32_t kEmitMask = (1u << 27) - 1;

uint32_t f32_bits(float v) {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    return u;
}

// numpy's pairwise sum (n <= 128), as Annotation.score()'s np.sum adds its K products
double pw_sum_cpu(const double *a, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
}

}  // namespace

namespace pp {
// Annotation.score() (annotation.py:60-71) with the default weights: 3 / (3 min(K, 3) +
// K - min(K, 3)) for the three largest v, 1 / (...) for the rest, np.sort(v)[::-1] order
// (zero_j >= 0: suppress_score_index, v[zero_j] reads as 0; w: the record's own score_weights)
double ann_score_cpu(const pp_ann &a, int K, int zero_j, const double *w) {
    float v[PP_MAX_KP];
    for (int j = 0; j < K; j++) v[j] = j == zero_j ? 0.0f : a.data[j][2];
    std::stable_sort(v, v + K, [](float p, float q) { return p > q; });
    const double ws = (double)(3 * std::min(K, 3) + (K - std::min(K, 3)));
    double prod[PP_MAX_KP];
    for (int r = 0; r < K; r++) prod[r] = (w ? w[r] : (r < 3 ? 3.0 : 1.0) / ws) * (double)v[r];
    return pw_sum_cpu(prod, K);
}
}  // namespace pp

namespace {
using pp::ann_score_cpu;

// Occupancy of nms.Keypoints (nms.py:27-31): (K, int(max y + 1) / r, int(max x + 1) / r) u8
struct NmsOcc {
    std::vector<uint8_t> p;
    int64_t h = 0, w = 0;
    int K = 0;
    float red = 2.0f, msr = 2.0f;
    bool get(int f, float x, float y) const {  // occupancy.py:41-47
        if (f >= K) return true;
        if (h <= 0 || w <= 0) return false;
        const int64_t xi = (int64_t)pp::clip_ref(x / red, 0.0f, (float)(w - 1));
        const int64_t yi = (int64_t)pp::clip_ref(y / red, 0.0f, (float)(h - 1));
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

}  // namespace

extern "C" {

// nms.Keypoints.annotations (nms.py:17-57) per group of records, as pp_nms_keypoints: anns
// edited in place (joints below keypoint_threshold zeroed, suppressed v scaled), survivors
// sorted by -score into out with their score, out_counts, out_index (optional) = input index.
static int nms_keypoints_host(pp_ann *anns, const int32_t *counts, int32_t n_img, int32_t K,
                              int32_t ann_capacity, const pp_config *cfg, double it,
                              const int32_t *spec, const double *sw, const double *fixed,
                              pp_ann *out, int32_t *out_counts, int32_t *out_index) {
    const float kt = cfg->nms_keypoint_threshold;
    std::vector<int> keep;
    std::vector<double> score;
    for (int img = 0; img < n_img; img++) {
        pp_ann *a = anns + (int64_t)img * ann_capacity;
        const int n = std::min(counts[img], ann_capacity);
        if (n < 0) return pp::fail(PP_ESHAPE, "pp_nms_keypoints_cpu: negative count");
        auto threshold_filter = [&](std::vector<int> &idx) {  // nms.py:20-21 / 47-49
            std::vector<int> kept;
            for (int i : idx) {
                for (int j = 0; j < K; j++)
                    if (a[i].data[j][2] < kt) a[i].data[j][0] = a[i].data[j][1] = a[i].data[j][2] = 0.0f;
                const int64_t gi = (int64_t)img * ann_capacity + i;
                if (spec && spec[gi] == -2)
                    score[i] = fixed[gi];  // fixed_score
                else if (spec)
                    score[i] = ann_score_cpu(a[i], K, spec[gi], sw + gi * K);
                else
                    score[i] = ann_score_cpu(a[i], K);
                if (score[i] >= it) kept.push_back(i);
            }
            std::stable_sort(kept.begin(), kept.end(),
                             [&](int p, int q) { return -score[p] < -score[q]; });
            idx.swap(kept);
        };
        keep.resize(n);
        score.assign(n, 0.0);
        for (int i = 0; i < n; i++) keep[i] = i;
        threshold_filter(keep);
        if (!keep.empty()) {
            NmsOcc occ;
            occ.K = K;
            occ.red = (float)cfg->occupancy_reduction;
            occ.msr = (float)((double)cfg->occupancy_min_scale / cfg->occupancy_reduction);
            float mx = 0.0f, my = 0.0f;
            bool first = true;
            std::vector<char> kept(n, 0);
            for (int i : keep) kept[i] = 1;
            for (int i = 0; i < n; i++) {  // max over the kept annotations in input order
                if (!kept[i]) continue;
                float ax = a[i].data[0][0], ay = a[i].data[0][1];
                for (int j = 1; j < K; j++) {
                    ax = a[i].data[j][0] > ax ? a[i].data[j][0] : ax;
                    ay = a[i].data[j][1] > ay ? a[i].data[j][1] : ay;
                }
                if (first || ax > mx) mx = ax;
                if (first || ay > my) my = ay;
                first = false;
            }
            const int64_t oh = (int64_t)((double)(int64_t)(my + 1.0f) / cfg->occupancy_reduction);
            const int64_t ow = (int64_t)((double)(int64_t)(mx + 1.0f) / cfg->occupancy_reduction);
            occ.h = oh > 0 ? oh : 0;
            occ.w = ow > 0 ? ow : 0;
            occ.p.assign((size_t)(K * occ.h * occ.w), 0);
            for (int i : keep)  // nms.py:33-45, in score order
                for (int f = 0; f < K; f++) {
                    float *xyv = a[i].data[f];
                    if (xyv[2] == 0.0f) continue;
                    if (occ.get(f, xyv[0], xyv[1]))
                        xyv[2] = xyv[2] * cfg->nms_suppression;
                    else
                        occ.set(f, xyv[0], xyv[1], a[i].joint_scales[f]);
                }
            threshold_filter(keep);
        }
        pp_ann *o = out + (int64_t)img * ann_capacity;
        for (size_t r = 0; r < keep.size(); r++) {
            o[r] = a[keep[r]];
            o[r].score = score[keep[r]];
            if (out_index) out_index[(int64_t)img * ann_capacity + r] = keep[r];
        }
        out_counts[img] = (int32_t)keep.size();
    }
    return PP_OK;
}

int pp_nms_keypoints_cpu(pp_ann *anns, const int32_t *counts, int32_t n_img, int32_t K,
                         int32_t ann_capacity, const pp_config *cfg, pp_ann *out,
                         int32_t *out_counts, int32_t *out_index) {
    if (!anns || !counts || !cfg || !out || !out_counts)
        return pp::fail(PP_EINVAL, "pp_nms_keypoints_cpu: NULL argument");
    if (n_img < 0 || K <= 0 || K > PP_MAX_KP || ann_capacity <= 0 || cfg->occupancy_reduction <= 0)
        return pp::fail(PP_ESHAPE, "pp_nms_keypoints_cpu: bad shape");
    return nms_keypoints_host(anns, counts, n_img, K, ann_capacity, cfg,
                              (double)cfg->nms_instance_threshold, nullptr, nullptr, nullptr, out,
                              out_counts, out_index);
}

// pp_nms_keypoints_scored on host records: each record's own Annotation.score()
// (annotation.py:60-71; spec -2 fixed_score, -1 none, j suppress_score_index), the instance
// threshold compared in float64
int pp_nms_keypoints_scored_cpu(pp_ann *anns, const int32_t *counts, int32_t n_img, int32_t K,
                                int32_t ann_capacity, const pp_config *cfg,
                                double instance_threshold, const int32_t *score_spec,
                                const double *score_weights, const double *fixed_score,
                                pp_ann *out, int32_t *out_counts, int32_t *out_index) {
    if (!anns || !counts || !cfg || !out || !out_counts ||
        (score_spec && (!score_weights || !fixed_score)))
        return pp::fail(PP_EINVAL, "pp_nms_keypoints_scored_cpu: NULL argument");
    if (n_img < 0 || K <= 0 || K > PP_MAX_KP || ann_capacity <= 0 || cfg->occupancy_reduction <= 0)
        return pp::fail(PP_ESHAPE, "pp_nms_keypoints_scored_cpu: bad shape");
    return nms_keypoints_host(anns, counts, n_img, K, ann_capacity, cfg, instance_threshold,
                              score_spec, score_weights, fixed_score, out, out_counts, out_index);
}

// CifHr.fill (cif_hr.py:23-81) for one head: per image and field, the cells with
// c > v_threshold in row-major order as truncate-1 splats of v / neighbors / len_cifs at
// (x, y) * stride with sigma = max(1, 0.5 * scale * stride) (cif_hr.py:26-40), into a zeroed
// (n_img, K, H', pitch) map.
int pp_cifhr_cpu(const float *cif, int32_t n_img, int32_t K, int32_t H, int32_t W,
                 const pp_config *cfg, float *cifhr) {
    if (!cif || !cifhr || bad_cfg(cfg)) return pp::fail(PP_EINVAL, "pp_cifhr_cpu: bad argument");
    if (n_img < 0 || K <= 0 || H <= 0 || W <= 0) return pp::fail(PP_ESHAPE, "pp_cifhr_cpu: bad shape");
    const HrGeom g = hr_geom(H, W, cfg->stride);
    const int64_t hw = (int64_t)H * W;
    const float stride = (float)cfg->stride, nb = (float)cfg->cif_neighbors;
    std::fill(cifhr, cifhr + (int64_t)n_img * K * g.hh * g.pitch, 0.0f);
    std::vector<float> x, y, s, v;
    for (int64_t f = 0; f < (int64_t)n_img * K; f++) {
        const float *p = cif + f * 5 * hw;
        x.clear();
        y.clear();
        s.clear();
        v.clear();
        for (int64_t c = 0; c < hw; c++) {
            if (!(p[c] > cfg->cif_threshold)) continue;  // p[:, p[0] > v_threshold]
            x.push_back(p[hw + c] * stride);
            y.push_back(p[2 * hw + c] * stride);
            const float sg = (0.5f * p[4 * hw + c]) * stride;
            s.push_back(sg != sg ? sg : std::fmax(1.0f, sg));  // np.maximum keeps NaN
            v.push_back((p[c] / nb) / 1.0f);                    // v / neighbors / len_cifs
        }
        const int rc = pp_scalar_square_add_gauss_with_max_cpu(
            cifhr + f * g.hh * g.pitch, g.hh, g.ww, g.pitch, x.data(), y.data(), s.data(),
            v.data(), (int64_t)x.size(), 1.0f, 1.0f);
        if (rc) return rc;
    }
    return PP_OK;
}

// CifSeeds.fill + get (cif_seeds.py:23-64) for one head: per image, fields in order (bit f
// of seed_skip_mask: FieldConfig.seed_mask[f] false), cells with c > threshold in row-major
// order, v = 0.9 * CifHr(x, y) + 0.1 * c (times score_scale), kept where v > threshold, as
// (v, field, x, y, s) scaled by the stride; sorted(seeds, reverse=True).
int pp_seeds_cpu(const float *cif, const float *cifhr, int32_t n_img, int32_t K, int32_t H,
                 int32_t W, const pp_config *cfg, pp_seed *seeds, int32_t seed_capacity,
                 int32_t *counts) {
    if (!cif || !cifhr || !seeds || !counts || bad_cfg(cfg))
        return pp::fail(PP_EINVAL, "pp_seeds_cpu: bad argument");
    if (n_img < 0 || K <= 0 || H <= 0 || W <= 0 || seed_capacity <= 0)
        return pp::fail(PP_ESHAPE, "pp_seeds_cpu: bad shape");
    const HrGeom g = hr_geom(H, W, cfg->stride);
    const int64_t hw = (int64_t)H * W;
    const float stride = (float)cfg->stride, th = cfg->seed_threshold;
    std::vector<pp_seed> em;     // emission order
    std::vector<uint64_t> keys;  // (v bits, field, inverted emission index), descending
    for (int img = 0; img < n_img; img++) {
        em.clear();
        keys.clear();
        for (int f = 0; f < K; f++) {
            if ((cfg->seed_skip_mask >> f) & 1u) continue;
            const float *p = cif + ((int64_t)img * K + f) * 5 * hw;
            const float *plane = cifhr + ((int64_t)img * K + f) * g.hh * g.pitch;
            for (int64_t c = 0; c < hw; c++) {
                const float conf = p[c];
                if (!(conf > th)) continue;
                const float hv = pp::hr_lookup(plane, (int)g.hh, (int)g.ww, g.pitch,
                                               p[hw + c] * stride, p[2 * hw + c] * stride, 0.0f);
                float vv = 0.9f * hv + 0.1f * conf;
                if (cfg->seed_score_scale != 1.0f) vv = vv * cfg->seed_score_scale;
                if (!(vv > th)) continue;
                if ((int64_t)em.size() >= seed_capacity)
                    return pp::fail(PP_ESHAPE, "pp_seeds_cpu: more seeds than seed_capacity");
                pp_seed r;
                r.v = vv;
                r.field = f;
                r.x = p[hw + c] * stride;
                r.y = p[2 * hw + c] * stride;
                r.s = p[4 * hw + c] * stride;
                keys.push_back(((uint64_t)f32_bits(vv) << 32) | ((uint64_t)f << 27) |
                               (kEmitMask - (uint32_t)em.size()));
                em.push_back(r);
            }
        }
        std::sort(keys.begin(), keys.end(), [](uint64_t a, uint64_t b) { return a > b; });
        auto emit = [](uint64_t k) { return (int64_t)(kEmitMask - ((uint32_t)k & kEmitMask)); };
        // runs of equal (v, field): (x, y, s) descending, then emission order (tuple order)
        auto before = [&](uint64_t p, uint64_t q) {
            const pp_seed &a = em[emit(p)], &b = em[emit(q)];
            if (a.x != b.x) return a.x > b.x;
            if (a.y != b.y) return a.y > b.y;
            if (a.s != b.s) return a.s > b.s;
            return emit(p) < emit(q);
        };
        const int64_t n = (int64_t)keys.size();
        for (int64_t i = 0; i < n;) {
            int64_t end = i + 1;
            while (end < n && (keys[end] >> 27) == (keys[i] >> 27)) end++;
            for (int64_t u = i + 1; u < end; u++) {  // insertion sort, as the device's
                const uint64_t cur = keys[u];
                int64_t w = u;
                while (w > i && before(cur, keys[w - 1])) {
                    keys[w] = keys[w - 1];
                    w--;
                }
                keys[w] = cur;
            }
            i = end;
        }
        pp_seed *out = seeds + (int64_t)img * seed_capacity;
        for (int64_t i = 0; i < n; i++) out[i] = em[emit(keys[i])];
        counts[img] = (int32_t)n;
    }
    return PP_OK;
}

// CafScored.fill (caf_scored.py:32-98) for one head: per image and CAF field, the cells with
// c > score_th in row-major order, rows 1-8 times the stride, rescored by the CifHr of the
// direction's target joint (cif_floor + (1 - cif_floor) * CifHr) and kept where the rescored
// value passes; backward columns in row order (0, 5, 6, 7, 8, 1, 2, 3, 4).  Layout as
// pp_caf_scored: cols (n_img, C, 2, 9, H*W), dir 0 backward, 1 forward; counts (n_img, C, 2).
int pp_caf_scored_cpu(const float *caf, const float *cifhr, int32_t n_img, int32_t K, int32_t C,
                      int32_t H, int32_t W, const int32_t *skeleton, float score_th,
                      const pp_config *cfg, float *cols, int32_t *counts) {
    if (!caf || !cifhr || !skeleton || !cols || !counts || bad_cfg(cfg))
        return pp::fail(PP_EINVAL, "pp_caf_scored_cpu: bad argument");
    if (n_img < 0 || K <= 0 || C <= 0 || H <= 0 || W <= 0)
        return pp::fail(PP_ESHAPE, "pp_caf_scored_cpu: bad shape");
    for (int i = 0; i < C; i++)
        if (skeleton[2 * i] < 1 || skeleton[2 * i + 1] < 1)
            return pp::fail(PP_EINVAL, "pp_caf_scored_cpu: skeleton is 1-based");
    const HrGeom g = hr_geom(H, W, cfg->stride);
    const int64_t hw = (int64_t)H * W;
    const float stride = (float)cfg->stride;
    const float floor_ = cfg->cif_floor, omf = (float)(1.0 - (double)cfg->cif_floor);
    for (int img = 0; img < n_img; img++)
        for (int ci = 0; ci < C; ci++) {
            const int64_t fld = (int64_t)img * C + ci;
            const float *p = caf + fld * 9 * hw;
            float *bwd = cols + (fld * 2 + 0) * 9 * hw, *fwd = cols + (fld * 2 + 1) * 9 * hw;
            const int j1 = skeleton[2 * ci] - 1, j2 = skeleton[2 * ci + 1] - 1;
            const bool use1 = floor_ < 1.0f && j1 < K, use2 = floor_ < 1.0f && j2 < K;
            const float *t1 = cifhr + ((int64_t)img * K + (use1 ? j1 : 0)) * g.hh * g.pitch;
            const float *t2 = cifhr + ((int64_t)img * K + (use2 ? j2 : 0)) * g.hh * g.pitch;
            int64_t nb = 0, nf = 0;
            for (int64_t c = 0; c < hw; c++) {
                const float score = p[c];
                if (!(score > score_th)) continue;  // mask = nine[0] > score_th
                float nine[9];
                nine[0] = score;
                for (int r = 1; r < 9; r++) nine[r] = p[r * hw + c] * stride;
                float sb = score, sf = score;
                if (use1)
                    sb = score * (floor_ + omf * pp::hr_lookup(t1, (int)g.hh, (int)g.ww, g.pitch,
                                                               nine[1], nine[2], 0.0f));
                if (use2)
                    sf = score * (floor_ + omf * pp::hr_lookup(t2, (int)g.hh, (int)g.ww, g.pitch,
                                                               nine[5], nine[6], 0.0f));
                if (sb > score_th) {
                    static const int order[9] = {0, 5, 6, 7, 8, 1, 2, 3, 4};
                    bwd[nb] = sb;
                    for (int r = 1; r < 9; r++) bwd[r * hw + nb] = nine[order[r]];
                    nb++;
                }
                if (sf > score_th) {
                    fwd[nf] = sf;
                    for (int r = 1; r < 9; r++) fwd[r * hw + nf] = nine[r];
                    nf++;
                }
            }
            counts[fld * 2 + 0] = (int32_t)nb;
            counts[fld * 2 + 1] = (int32_t)nf;
        }
    return PP_OK;
}

}  // extern "C"
