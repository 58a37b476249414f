// pp_host.hip — C-ABI plumbing: error reporting, version, default configuration.
#include "pp_common.hpp"

namespace pp {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int status, const std::string &msg) {
    set_error(msg);
    return status;
}

int check_launch(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(PP_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return PP_OK;
}

int make_heads(const pp_scale *sc, int n, int pairs, int need, Heads *h, const char *who) {
    if (!sc || !h) return fail(PP_EINVAL, std::string(who) + ": NULL scale list");
    if (n <= 0 || n > 2 * kMaxHeads) return fail(PP_ESHAPE, std::string(who) + ": bad scale count");
    *h = Heads{};
    int64_t coff = 0, aoff = 0;
    int64_t geo_hh = 0, geo_ww = 0;
    for (int i = 0; i < n; i++) {
        const pp_scale &s = sc[i];
        const int role = s.role ? s.role : (PP_ROLE_CIF | PP_ROLE_CAF);
        if (role & ~(PP_ROLE_CIF | PP_ROLE_CAF | PP_ROLE_HRMAP) ||
            ((role & PP_ROLE_HRMAP) && role != PP_ROLE_HRMAP))
            return fail(PP_EINVAL, std::string(who) + ": bad role");
        if (s.H <= 0 || s.W <= 0 || s.stride <= 0)
            return fail(PP_ESHAPE, std::string(who) + ": bad head shape / stride");
        if (role == PP_ROLE_HRMAP) {  // geometry only: no field is read
            if (geo_hh) return fail(PP_EINVAL, std::string(who) + ": two PP_ROLE_HRMAP entries");
            geo_hh = hr_dim(s.H, s.stride);
            geo_ww = hr_dim(s.W, s.stride);
            continue;
        }
        // `if min_scale:` / `if min_distance:` / `if max_distance:` (truthiness); the
        // thresholds are Python float / int divisions rounded to the f32 comparand
        if (role & PP_ROLE_CIF) {
            const int m = h->n_cif++;
            if (m >= kMaxHeads) return fail(PP_ESHAPE, std::string(who) + ": more than PP_MAX_SCALES CIF heads");
            h->cif[m] = s.cif;
            h->cH[m] = s.H;
            h->cW[m] = s.W;
            h->cstride[m] = s.stride;
            h->cif_off[m] = coff;
            coff += (int64_t)s.H * s.W;
            if (s.cif_min_scale != 0.0f) h->ms_on |= 1u << m;
            h->ms_th[m] = (float)((double)s.cif_min_scale / s.stride);
        }
        if (role & PP_ROLE_CAF) {
            const int m = h->n_caf++;
            if (m >= kMaxHeads) return fail(PP_ESHAPE, std::string(who) + ": more than PP_MAX_SCALES CAF heads");
            h->caf[m] = s.caf;
            h->aH[m] = s.H;
            h->aW[m] = s.W;
            h->astride[m] = s.stride;
            h->caf_off[m] = aoff;
            aoff += (int64_t)s.H * s.W;
            if (s.caf_min_distance != 0.0f) h->dmin_on |= 1u << m;
            if (s.caf_max_distance != 0.0f) h->dmax_on |= 1u << m;
            h->dmin_th[m] = (float)((double)s.caf_min_distance / s.stride);
            h->dmax_th[m] = (float)((double)s.caf_max_distance / s.stride);
        }
    }
    h->cif_off[h->n_cif] = coff;
    h->caf_off[h->n_caf] = aoff;
    if ((need & PP_ROLE_CIF) && h->n_cif == 0) return fail(PP_EINVAL, std::string(who) + ": no CIF head");
    if ((need & PP_ROLE_CAF) && h->n_caf == 0) return fail(PP_EINVAL, std::string(who) + ": no CAF head");
    // cif_pairs: 0 = one CifHr group per head, 1 = hflip pairs (2 heads per group),
    // n >= 2 = n heads per group
    const int gsize = pairs <= 0 ? 1 : (pairs == 1 ? 2 : pairs);
    if (h->n_cif % gsize)
        return fail(PP_ESHAPE, std::string(who) + ": CIF head count is not a multiple of the "
                                                  "CifHr group size");
    h->gsize = gsize;
    h->n_groups = h->n_cif / gsize;
    if (geo_hh) {
        h->hr_hh = (int)geo_hh;
        h->hr_ww = (int)geo_ww;
    } else if (h->n_cif) {
        h->hr_hh = (int)hr_dim(h->cH[0], h->cstride[0]);
        h->hr_ww = (int)hr_dim(h->cW[0], h->cstride[0]);
    }
    if (geo_hh > INT32_MAX / 2 || geo_ww > INT32_MAX / 2)
        return fail(PP_ESHAPE, std::string(who) + ": CifHr map too large");
    if (coff * PP_MAX_KP > INT32_MAX || aoff > INT32_MAX)
        return fail(PP_ESHAPE, std::string(who) + ": too many cells");
    return PP_OK;
}

Heads single_head(const float *cif, const float *caf, int H, int W, int stride) {
    pp_scale s{};
    s.cif = cif;
    s.caf = caf;
    s.H = H;
    s.W = W;
    s.stride = stride;
    Heads h{};
    make_heads(&s, 1, 0, 0, &h, "single");
    return h;
}

}  // namespace pp

extern "C" {

int pp_version(void) { return PP_ABI_VERSION; }

const char *pp_last_error(void) { return pp::g_last_error.c_str(); }

// Reference defaults as eval_coco configures them (decoder/factory.py:17-22,64-98;
// eval_coco.py:215): force_complete_pose=True, seed_threshold=0.2, keypoint/instance 0.
void pp_default_config(pp_config *c) {
    if (!c) return;
    c->cif_threshold = 0.1f;           // CifHr.v_threshold
    c->seed_threshold = 0.2f;          // --seed-threshold default
    c->seed_score_scale = 1.0f;        // CifSeeds.score_scale
    c->caf_threshold = 0.1f;           // CafScored.default_score_th
    c->complete_caf_threshold = 0.0001f;
    c->cif_floor = 0.1f;
    c->keypoint_threshold = 0.0f;
    c->nms_keypoint_threshold = 0.0f;
    c->nms_instance_threshold = 0.0f;
    c->nms_suppression = 0.0f;
    c->stride = 8;
    c->cif_neighbors = 16;
    c->force_complete = 1;
    c->greedy = 0;
    c->connection_method = 0;
    c->apply_nms = 1;
    c->occupancy_reduction = 2;
    c->occupancy_min_scale = 4;
    c->seed_skip_mask = 0u;
    c->confidence_scales = nullptr;
}

}  // extern "C"
