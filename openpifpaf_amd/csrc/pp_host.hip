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
}

}  // extern "C"
