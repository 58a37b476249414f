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

}  // namespace

extern "C" {

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
