/*
 * pifpaf_amd.h — C ABI of libpifpaf_amd.so, the MI355X (gfx950) CIF/CAF pose decoder.
 *
 * Drop-in boundary for openpifpaf v0.11.6's decoder hot path.  The reference exposes
 * this path as the Cython extension module `openpifpaf.functional`
 * (openpifpaf/functional.pyx) plus the pure-Python decoder classes in
 * openpifpaf/decoder/ (cif_hr.py, cif_seeds.py, caf_scored.py, generator/cifcaf.py,
 * nms.py, occupancy.py).  Every entry point below names the reference interface it
 * replaces (file:line).  The Python mirror of those interfaces is the package
 * openpifpaf_amd (ctypes over this header).
 *
 * Conventions (all entry points):
 *   - plain pointers + sizes, no C++/torch types; arrays are C-contiguous float32 unless
 *     a pitch/stride argument says otherwise.  Element strides, not byte strides.
 *   - every pointer named d_* is DEVICE memory (hipMalloc / torch device tensors).
 *     The caller owns all buffers; the library never allocates or frees them.
 *   - calls are asynchronous on `stream` (a hipStream_t; NULL = legacy default stream).
 *     No host synchronisation inside (graph-capturable).
 *   - return 0 on success or a negative pp_status; pp_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - the library has no global mutable state; calls on distinct streams are thread-safe.
 */
#ifndef PIFPAF_AMD_H
#define PIFPAF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PP_ABI_VERSION 4

/* capacities of one annotation record (COCO person: 17 keypoints, 19 or 44 edges) */
#define PP_MAX_KP 24
#define PP_MAX_EDGES 64
#define PP_MAX_FRONTIER (4 * PP_MAX_EDGES)
#define PP_MAX_SCALES 16   /* CIF / CAF heads of one multi-scale decode */

typedef enum pp_status {
    PP_OK = 0,
    PP_EINVAL = -1,     /* bad argument (NULL pointer, negative size, bad enum) */
    PP_ESHAPE = -2,     /* shape outside the supported envelope                 */
    PP_EOVERFLOW = -3,  /* a capacity was exceeded; see the per-image status     */
    PP_EHIP = -4,       /* HIP runtime error (launch / device)                   */
    PP_ENOMEM = -5      /* workspace too small                                   */
} pp_status;

/*
 * Decoder configuration.  The reference keeps these as CLASS ATTRIBUTES written by
 * decoder/factory.py:configure (factory.py:64-98); pp_default_config() fills the
 * reference defaults (eval_coco: force_complete=1, seed_threshold=0.2).
 */
typedef struct pp_config {
    float cif_threshold;          /* CifHr.v_threshold                cif_hr.py:16          */
    float seed_threshold;         /* CifSeeds.threshold               cif_seeds.py:14       */
    float seed_score_scale;       /* CifSeeds.score_scale             cif_seeds.py:15       */
    float caf_threshold;          /* CafScored.default_score_th       caf_scored.py:14      */
    float complete_caf_threshold; /* score_th of the force-complete CafScored cifcaf.py:337 */
    float cif_floor;              /* CafScored(cif_floor=0.1)         caf_scored.py:16      */
    float keypoint_threshold;     /* CifCaf.keypoint_threshold        cifcaf.py:33          */
    float nms_keypoint_threshold; /* nms.Keypoints.keypoint_threshold nms.py:14             */
    float nms_instance_threshold; /* nms.Keypoints.instance_threshold nms.py:13             */
    float nms_suppression;        /* nms.Keypoints.suppression        nms.py:12             */
    int32_t stride;               /* FieldConfig.cif_strides[0] == caf_strides[0]  field_config.py:9-10 */
    int32_t cif_neighbors;        /* CifHr.neighbors                  cif_hr.py:15          */
    int32_t force_complete;       /* CifCaf.force_complete            cifcaf.py:31          */
    int32_t greedy;               /* CifCaf.greedy                    cifcaf.py:32          */
    int32_t connection_method;    /* CifCaf.connection_method: 0 'blend', 1 'max'  cifcaf.py:29 */
    int32_t apply_nms;            /* CifCaf(nms=True) -> nms.Keypoints()  cifcaf.py:43-44   */
    int32_t occupancy_reduction;  /* Occupancy(shape, 2, min_scale=4)  cifcaf.py:84         */
    int32_t occupancy_min_scale;
    uint32_t seed_skip_mask;      /* bit f set: field f emits no seeds, FieldConfig.seed_mask[f]
                                     falsy (cif_seeds.py:28-29); 0 = every field seeds       */
    int32_t exp_mode;             /* np.exp of the CAF scores (cifcaf.py:139): 0 = NumPy's
                                     float32 SIMD exp (the FMA3 / AVX512F routine NumPy runs on
                                     any x86-64 since 2013; bit-exact over every float32 in
                                     [-104, 0], tests/test_np_exp.py), 1 = correctly rounded
                                     (NumPy's scalar loop on CPUs without FMA3)              */
    const float *confidence_scales; /* HOST array (C): CifCaf(confidence_scales=...)
                                     (cifcaf.py:39,52), each CAF's weight on the frontier
                                     priorities of _grow (cifcaf.py:259-260, 282-284), f32
                                     products as NumPy forms them from a list of Python
                                     floats; NULL = none (the default)                       */
} pp_config;

/*
 * One output annotation (openpifpaf/annotation.py:9-28).  data/joint_scales are the
 * reference's float32 arrays; score is Annotation.score() (float64, annotation.py:60-71).
 * decoding_order entries (jsi, jti, xyv_jsi, xyv_jti) and frontier_order pairs as
 * appended by CifCaf._grow (cifcaf.py:263,305-306), 0-based joint indices.
 */
typedef struct pp_ann {
    float data[PP_MAX_KP][3];
    float joint_scales[PP_MAX_KP];
    double score;
    int32_t n_keypoints;
    int32_t n_decoding;
    int32_t n_frontier;
    int32_t image;
    uint8_t decoding_pairs[PP_MAX_KP][2];
    float decoding_xyv[PP_MAX_KP][6];
    uint8_t frontier_pairs[PP_MAX_FRONTIER][2];
} pp_ann;

/* one seed (cif_seeds.py:47 tuple (v, field, x, y, s)) */
typedef struct pp_seed {
    float v;
    int32_t field;
    float x;
    float y;
    float s;
} pp_seed;

/* One detection: AnnotationDet (annotation.py:122-137) with its image */
typedef struct pp_det {
    int32_t field;       /* category index (field_i)                                     */
    float score;
    float bbox[4];       /* x, y, w, h                                                   */
    int32_t image;
    int32_t pad_;
} pp_det;

/* nms.Detection class attributes (nms.py:60-65) */
typedef struct pp_det_nms {
    float suppression;        /* 0.1 */
    float suppression_soft;   /* 0.3 */
    float instance_threshold; /* 0.1 */
    float iou_threshold;      /* 0.7 */
    float iou_threshold_soft; /* 0.5 */
    int32_t apply;            /* 1 */
} pp_det_nms;

/* The meta of one image that Preprocess.annotations_inverse reads
 * (transforms/annotations.py:39-44): offset and scale float64, width_height[0], hflip,
 * rotation angle / width / height */
typedef struct pp_inverse_meta {
    double offset[2];
    double scale[2];
    double rotation_angle;
    double rotation_width;
    double rotation_height;
    double width;
    int32_t hflip;
    int32_t pad_;
} pp_inverse_meta;

/* One head of a multi-scale decode: FieldConfig entries (field_config.py:7-13,
 * factory.py:153-180).  The entries with the PP_ROLE_CIF bit form the CIF head list
 * (cif_indices order), those with PP_ROLE_CAF the CAF head list (caf_indices order); role 0
 * means both (one stride shared by a CIF and a CAF head).  0 for a min scale / distance
 * means unused (the reference tests them for truthiness). */
#define PP_ROLE_CIF 1
#define PP_ROLE_CAF 2
/* An entry that only names the CifHr map's geometry, (H-1)*stride+1 x (W-1)*stride+1,
 * instead of CIF head 0's (no field is read): the stage entry points then read or write a
 * map made at another head's size (CifSeeds.fill_cif / CafScored.fill_caf at any stride,
 * CifHr.fill_multiple into an existing map, cif_hr.py:42-57). */
#define PP_ROLE_HRMAP 4
typedef struct pp_scale {
    const float *cif;        /* (n_img, K, 5, H, W) when a CIF head */
    const float *caf;        /* (n_img, C, 9, H, W) when a CAF head */
    int32_t H, W, stride;
    float cif_min_scale;     /* cif_min_scales[i] */
    float caf_min_distance;  /* caf_min_distances[i] */
    float caf_max_distance;  /* caf_max_distances[i] (None -> 0) */
    int32_t role;            /* PP_ROLE_* bits, 0 = both */
} pp_scale;

/* per-image status bits written by pp_decode_batch (d_status) */
#define PP_ST_ANN_OVERFLOW 1   /* more annotations than ann_capacity               */
#define PP_ST_NMS_OVERFLOW 2   /* NMS occupancy larger than the occupancy workspace */
#define PP_ST_SEED_OVERFLOW 4  /* more seeds than the seed workspace               */
#define PP_ST_DEC_OVERFLOW 8   /* decoding/frontier order longer than the record   */

int pp_version(void);
const char *pp_last_error(void);
void pp_default_config(pp_config *cfg);

/* ---------------------------------------------------------------------------------
 * Decoder stages.  Batched: n_img images, fields (n_img, K, 5, H, W) and
 * (n_img, C, 9, H, W) resident in device memory.  The high-resolution CIF map is laid
 * out (n_img, K, H', pitch) with H' = (H-1)*stride+1, W' = (W-1)*stride+1 and
 * pitch = pp_cifhr_pitch(W') (a multiple of 32 floats, so each row starts on a 128-B line).
 * --------------------------------------------------------------------------------- */
int64_t pp_cifhr_pitch(int64_t w_hr);

/* bytes of scratch pp_decode_batch needs (pass the same arguments) */
size_t pp_decode_workspace_size(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                                const pp_config *cfg, int32_t ann_capacity);

/*
 * CifHr (cif_hr.py:14-81): zero-init + accumulate every CIF cell with c > cif_threshold
 * as a truncate=1 Gaussian splat (functional.pyx:105-141) into d_cifhr.  Bit-exact.
 * d_workspace >= pp_cifhr_workspace_size(n_img, K, H, W).
 */
size_t pp_cifhr_workspace_size(int32_t n_img, int32_t K, int32_t H, int32_t W);
int pp_cifhr(const float *d_cif, int32_t n_img, int32_t K, int32_t H, int32_t W,
             const pp_config *cfg, float *d_cifhr, void *d_workspace, size_t workspace_bytes,
             void *stream);

/*
 * The same CifHr as the block-sparse map the decoder keeps (cif_hr.py:14-81, values bit-equal
 * to pp_cifhr): the (H', pitch) plane is cut into T = pp_cifhr_sparse_tiles(H, W, stride)
 * 64x64 tiles (row-major, ceil(pitch/64) per row) of 64 8x8 blocks.  d_map
 * (n_img, K, T, 64 blocks, 64 px): block b = 8*by + bx of a tile holds its 8 rows of 8
 * pixels back to back; d_masks (n_img, K, T) u64 with bit b set iff block b was written.
 * Only blocks some splat box touches are written; every other pixel is 0.
 * d_workspace >= pp_cifhr_sparse_workspace_size(n_img, K, H, W).
 */
int32_t pp_cifhr_sparse_tiles(int32_t H, int32_t W, int32_t stride);
size_t pp_cifhr_sparse_workspace_size(int32_t n_img, int32_t K, int32_t H, int32_t W);
int pp_cifhr_sparse(const float *d_cif, int32_t n_img, int32_t K, int32_t H, int32_t W,
                    const pp_config *cfg, float *d_map, uint64_t *d_masks, void *d_workspace,
                    size_t workspace_bytes, void *stream);

/*
 * CifSeeds (cif_seeds.py:23-64): per image, the seeds sorted as
 * sorted(seeds, reverse=True) (cif_seeds.py:54).  d_seeds (n_img, seed_capacity) with
 * seed_capacity >= K*H*W (every cell can seed, so no overflow is possible);
 * d_counts (n_img) = number of seeds.
 */
int pp_seeds(const float *d_cif, const float *d_cifhr, int32_t n_img, int32_t K, int32_t H,
             int32_t W, const pp_config *cfg, pp_seed *d_seeds, int32_t seed_capacity,
             int32_t *d_counts, void *stream);

/*
 * CafScored (caf_scored.py:32-98) for one score threshold: per image and CAF field, the
 * backward and forward (9, N) column sets.  Layout d_cols (n_img, C, 2, 9, H*W) with
 * direction 0 = backward, 1 = forward; d_counts (n_img, C, 2).
 */
int pp_caf_scored(const float *d_caf, const float *d_cifhr, int32_t n_img, int32_t K,
                  int32_t C, int32_t H, int32_t W, const int32_t *skeleton, float score_th,
                  const pp_config *cfg, float *d_cols, int32_t *d_counts, void *stream);

/*
 * Full decode, CifCaf.__call__ (cifcaf.py:67-122) for a batch: CifHr -> CifSeeds ->
 * CafScored -> seed loop / _grow -> complete_annotations -> nms.Keypoints.
 *   skeleton      HOST array (C, 2) of 1-based joint pairs (cifcaf.py:50)
 *   d_anns        (n_img, ann_capacity) records, image-major, in the reference's final order
 *   d_counts      (n_img) number of annotations per image (true count)
 *   d_status      (n_img) PP_ST_* bits; a non-zero bit means "re-run with more capacity"
 *   d_cifhr       optional (n_img, K, H', pitch) output of the CifHr stage (NULL: scratch)
 */
int pp_decode_batch(const float *d_cif, const float *d_caf, int32_t n_img, int32_t K,
                    int32_t C, int32_t H, int32_t W, const int32_t *skeleton,
                    const pp_config *cfg, float *d_cifhr, pp_ann *d_anns,
                    int32_t ann_capacity, int32_t *d_counts, int32_t *d_status,
                    void *d_workspace, size_t workspace_bytes, void *stream);

/*
 * Multi-scale decode: the same stages over a FieldConfig of CIF and CAF heads
 * (field_config.py:7-13; the heads' scale / min-distance lists of factory.py:153-180) given
 * as n_scales pp_scale entries (see PP_ROLE_*), device arrays of each head's own size.
 * cif_pairs groups the CIF heads for CifHr (fill_multiple, cif_hr.py:42-57): 0 = one group
 * per head; 1 = the reference's 10-head hflip layout (cif_hr.py:63-68), heads g and g + n/2
 * accumulated into one map at head g's stride and min scale (the reference pairs exactly
 * when len(cif_indices) == 10); m >= 2 = groups of m heads, head g + i * (n / m) being
 * member i of group g, each splat weighted v / neighbors / m.  The groups' maps are combined
 * by np.maximum.  The CifHr map has CIF head 0's size, (n_img, K, H', pitch) with
 * H' = (H_0 - 1) * stride_0 + 1, unless a PP_ROLE_HRMAP entry names another.  cfg->stride
 * is unused.
 *   pp_cifhr_multi       CifHr.fill (cif_hr.py:59-73), maps combined by np.maximum
 *   pp_seeds_multi       CifSeeds.fill over every CIF head (cif_seeds.py:56-64), sorted;
 *                        seed_capacity >= K * (sum of the CIF heads' H * W)
 *   pp_caf_scored_multi  CafScored.fill over every CAF head (caf_scored.py:88-98): per field
 *                        the heads' columns concatenated; d_cols (n_img, C, 2, 9,
 *                        col_capacity) with col_capacity >= the CAF heads' cells,
 *                        d_counts (n_img, C, 2); the list must hold the CIF heads too
 *                        (CIF head 0 gives the CifHr geometry; CIF fields are not read)
 *   pp_decode_multi      CifCaf.__call__ (cifcaf.py:67-122) over the heads, `stages` as
 *                        pp_decode_stages (15 = the full decode); outputs and status as
 *                        pp_decode_batch, workspace contract as pp_decode_stages (zero
 *                        region from pp_decode_multi_workspace_zero_offset).
 */
size_t pp_cifhr_multi_workspace_size(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                     int32_t n_img, int32_t K);
int pp_cifhr_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                   int32_t K, const pp_config *cfg, float *d_cifhr, void *d_workspace,
                   size_t workspace_bytes, void *stream);
int pp_seeds_multi(const pp_scale *scales, int32_t n_scales, const float *d_cifhr, int32_t n_img,
                   int32_t K, const pp_config *cfg, pp_seed *d_seeds, int32_t seed_capacity,
                   int32_t *d_counts, void *stream);
int pp_caf_scored_multi(const pp_scale *scales, int32_t n_scales, const float *d_cifhr,
                        int32_t n_img, int32_t K, int32_t C, const int32_t *skeleton,
                        float score_th, const pp_config *cfg, float *d_cols,
                        int64_t col_capacity, int32_t *d_counts, void *stream);
size_t pp_decode_multi_workspace_size(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                      int32_t n_img, int32_t K, int32_t C, const pp_config *cfg,
                                      int32_t ann_capacity);
size_t pp_decode_multi_workspace_zero_offset(const pp_scale *scales, int32_t n_scales,
                                             int32_t cif_pairs, int32_t n_img, int32_t K,
                                             int32_t C, const pp_config *cfg,
                                             int32_t ann_capacity);
int pp_decode_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                    int32_t K, int32_t C, const int32_t *skeleton, const pp_config *cfg,
                    float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                    int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                    uint32_t stages, void *stream);

/*
 * CifCaf.__call__(fields, initial_annotations) (cifcaf.py:67-71, 95-98): pp_decode_multi
 * where each image first grows its initial annotations d_initial[img * initial_capacity + i],
 * i < d_initial_counts[img] (set A, reverse matching, from every joint with v != 0; the
 * records' decoding / frontier orders are kept and appended to), appends them to its
 * annotation list in that order and marks them occupied, then runs the seed loop; force-
 * complete and NMS see them like any other annotation.  A record needs data,
 * joint_scales, n_decoding, decoding_pairs / decoding_xyv, n_frontier and frontier_pairs;
 * image and n_keypoints are set by the decoder.  d_initial / d_initial_counts may be NULL
 * (then this is pp_decode_multi).  d_out_index (optional, (n_img, ann_capacity) int32):
 * for each output record its position in the image's annotation list before NMS, so
 * positions < d_initial_counts[img] are the initial annotations (the reference returns those
 * objects, mutated).  Workspace as pp_decode_multi (pp_decode_multi_workspace_size).
 * Reference interface: openpifpaf.decoder.CifCaf.__call__ (cifcaf.py:67).
 */
/*
 * Byte offset, inside a decode workspace of that shape, of the (n_img, ann_capacity) pp_ann
 * working records: after a decode with the grow stage, image img's annotation list before
 * NMS (positions as d_out_index reports them), in the state NMS left every one of them in,
 * including those it dropped (nms.py:20-53 edits the Annotation objects in place before it
 * filters them).  Valid until the next decode into the workspace.  pp_decode_work_offset
 * for pp_decode_batch / pp_decode_stages workspaces, pp_decode_multi_work_offset for
 * pp_decode_multi / pp_decode_initial ones; 0 on a bad shape.
 * Reference interface: the initial_annotations objects CifCaf.__call__ mutates
 * (cifcaf.py:67-71, 95-98, 117-118).
 */
size_t pp_decode_work_offset(int32_t n_img, int32_t K, int32_t C, int32_t H, int32_t W,
                             const pp_config *cfg, int32_t ann_capacity);
size_t pp_decode_multi_work_offset(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                   int32_t n_img, int32_t K, int32_t C, const pp_config *cfg,
                                   int32_t ann_capacity);

int pp_decode_initial(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                      int32_t K, int32_t C, const int32_t *skeleton, const pp_config *cfg,
                      float *d_cifhr, pp_ann *d_anns, int32_t ann_capacity, int32_t *d_counts,
                      int32_t *d_status, const pp_ann *d_initial, const int32_t *d_initial_counts,
                      int32_t initial_capacity, int32_t *d_out_index, void *d_workspace,
                      size_t workspace_bytes, uint32_t stages, void *stream);

/*
 * CifDet detection decoder (decoder/generator/cifdet.py:27-52), batched:
 *   d_det     (n_img, K, 7, H, W) CifDet fields [c, x, y, b, w, h, b2] (heads.py:127-144)
 *   d_cifhr   optional (n_img, K, H', pitch) output of CifDetHr (NULL: scratch)
 *   d_out     (n_img, det_capacity) pp_det, d_counts (n_img), d_status (n_img) PP_ST_* bits
 * Uses cfg's cif_threshold (CifHr.v_threshold), seed_threshold (>= 0), seed_score_scale,
 * stride and cif_neighbors; the occupancy is the reference's fixed Occupancy(cifhr.shape,
 * 2, min_scale=2.0); nms.Detection runs with *nms (pp_default_det_nms) when nms->apply.
 * pp_cifdet_hr is the CifDetHr stage alone (cif_hr.py:84-100), workspace as pp_cifhr.
 */
void pp_default_det_nms(pp_det_nms *nms);
int pp_cifdet_hr(const float *d_det, int32_t n_img, int32_t K, int32_t H, int32_t W,
                 const pp_config *cfg, float *d_cifhr, void *d_workspace, size_t workspace_bytes,
                 void *stream);
/* CifDetHr.fill over several detection heads (cif_hr.py:67-80 as CifDetHr inherits it: each
 * head its own map at its stride, min-scale masks p[4] and p[5] > cif_min_scale / stride
 * (cif_hr.py:84-90), combined by np.maximum; cif_pairs as pp_cifhr_multi for the 10-head
 * layout).  scales: PP_ROLE_CIF entries whose `cif` points at (n_img, K, 7, H, W) detection
 * fields; d_cifhr has head 0's size (or a PP_ROLE_HRMAP entry's); workspace
 * pp_cifhr_multi_workspace_size of the same list. */
int pp_cifdet_hr_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs, int32_t n_img,
                       int32_t K, const pp_config *cfg, float *d_cifhr, void *d_workspace,
                       size_t workspace_bytes, void *stream);
/* nms.Detection.annotations (nms.py:79-102) over caller records: n_img groups, d_in
 * (n_img, capacity) with d_counts[i] records (field, score, bbox) in list order.  Output
 * as pp_cifdet_decode; d_out_index (optional) = input index of each output record;
 * d_scores_out (optional, (n_img, capacity)) = every input record's score after the
 * reference's in-place edits (soft suppression; nms.py:90-99), in input order. */
size_t pp_nms_detection_workspace_size(int32_t n_img, int32_t capacity);
int pp_nms_detection(const pp_det *d_in, const int32_t *d_counts, int32_t n_img, int32_t capacity,
                     const pp_det_nms *nms, pp_det *d_out, int32_t *d_out_counts,
                     int32_t *d_out_index, float *d_scores_out, void *d_workspace,
                     size_t workspace_bytes, void *stream);
/* CifDetSeeds.fill_cif (cif_seeds.py:67-90) per (image, field), in cell order:
 * d_seg (n_img, K, 5, H*W) = v, x, y, w, h of the first d_seg_counts[i, f] entries;
 * d_cifhr (n_img, K, H', pitch).  get() = sorted((v, f, x, y, w, h), reverse=True). */
int pp_cifdet_seeds(const float *d_det, const float *d_cifhr, int32_t n_img, int32_t K, int32_t H,
                    int32_t W, const pp_config *cfg, float *d_seg, int32_t *d_seg_counts,
                    void *stream);
/* CifDetSeeds.fill over several detection heads (cif_seeds.py:56-64, 67-90: each head's
 * cells, min-scale masks on p[4] and p[5], x / y / w / h at the head's stride, v from the
 * one d_cifhr map), each field's seeds appended head after head: d_seg (n_img, K, 5, cells)
 * with cells = the heads' H * W summed. */
int pp_cifdet_seeds_multi(const pp_scale *scales, int32_t n_scales, const float *d_cifhr,
                          int32_t n_img, int32_t K, const pp_config *cfg, float *d_seg,
                          int32_t *d_seg_counts, void *stream);
size_t pp_cifdet_workspace_size(int32_t n_img, int32_t K, int32_t H, int32_t W,
                                const pp_config *cfg, int32_t det_capacity);
int pp_cifdet_decode(const float *d_det, int32_t n_img, int32_t K, int32_t H, int32_t W,
                     const pp_config *cfg, const pp_det_nms *nms, float *d_cifhr, pp_det *d_out,
                     int32_t det_capacity, int32_t *d_counts, int32_t *d_status,
                     void *d_workspace, size_t workspace_bytes, void *stream);
/* CifDet.__call__ (generator/cifdet.py:27-52) over a FieldConfig of several detection heads
 * and / or min scales: CifDetHr as pp_cifdet_hr_multi, CifDetSeeds as pp_cifdet_seeds_multi,
 * then the occupancy loop and nms.Detection as pp_cifdet_decode. */
size_t pp_cifdet_multi_workspace_size(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                                      int32_t n_img, int32_t K, int32_t det_capacity);
int pp_cifdet_decode_multi(const pp_scale *scales, int32_t n_scales, int32_t cif_pairs,
                           int32_t n_img, int32_t K, const pp_config *cfg, const pp_det_nms *nms,
                           float *d_cifhr, pp_det *d_out, int32_t det_capacity, int32_t *d_counts,
                           int32_t *d_status, void *d_workspace, size_t workspace_bytes,
                           void *stream);

/*
 * Preprocess.annotations_inverse (transforms/preprocess.py:35-95) on device records, one
 * meta per image (d_metas (n_img) device array):
 *   pp_annotations_inverse  poses: rotation, offset, scale (data, joint_scales,
 *                           decoding_order), hflip with the optional horizontal swap
 *                           d_hswap (K) = target row of each source row (hflip.py:17-29);
 *                           d_nan_flags[i] |= 1 where the reference's NaN assert fires
 *   pp_dets_inverse         boxes: rotate_box (transforms/utils.py:5-28), offset, scale
 */
int pp_annotations_inverse(pp_ann *d_anns, const int32_t *d_counts, int32_t n_img,
                           int32_t capacity, int32_t K, const pp_inverse_meta *d_metas,
                           const int32_t *d_hswap, int32_t *d_nan_flags, void *stream);
int pp_dets_inverse(pp_det *d_dets, const int32_t *d_counts, int32_t n_img, int32_t capacity,
                    const pp_inverse_meta *d_metas, void *stream);

/*
 * Field ingestion: the raw output of a CompositeFieldFused head's conv (network/heads.py:
 * 406-455, eval mode) -> the decoder's field layout, as CifCafCollector /
 * CifdetCollector.forward (heads.py:65-88, 127-144) produce it: `quad` PixelShuffle(2)
 * dequads with the last row / column cropped, sigmoid on confidences, exp on scales, the
 * index grid added to the vector components and the channel reorder, in one pass.
 *   d_conv  (n_img, F * 4^quad, h, w) with F = n_fields * (5 | 9 | 7) for layout
 *           0 CIF (IntensityMeta), 1 CAF (AssociationMeta), 2 CifDet (DetectionMeta)
 *   d_out   (n_img, n_fields, 5 | 9 | 7, H, W) with H = pp_fields_dim(h, quad)
 * Floats: sigmoid / exp are evaluated in f64 and rounded (within 1 ulp of torch's).
 */
int64_t pp_fields_dim(int64_t n, int32_t quad);
int pp_fields_from_conv(const float *d_conv, int32_t n_img, int32_t n_fields, int32_t layout,
                        int32_t h, int32_t w, int32_t quad, float *d_out, void *stream);

/*
 * nms.Keypoints.annotations (nms.py:17-57) over caller records, n_img independent groups:
 * d_anns (n_img, ann_capacity) with d_counts[i] records in group i (modified in place as
 * the reference modifies its Annotation objects: joints below keypoint_threshold zeroed,
 * suppressed joints' v scaled by nms_suppression).  Survivors sorted by -score go to
 * d_out (n_img, ann_capacity) with their score set, d_out_counts (n_img), and optionally
 * d_out_index (n_img, ann_capacity) = the input index of each survivor.  Uses cfg's
 * nms_* thresholds and occupancy_reduction / occupancy_min_scale.  Scores are the
 * default Annotation.score() (annotation.py:60-71 without fixed_score or
 * suppress_score_index).
 */
size_t pp_nms_workspace_size(int32_t n_img, int32_t ann_capacity);
int pp_nms_keypoints(pp_ann *d_anns, const int32_t *d_counts, int32_t n_img, int32_t K,
                     int32_t ann_capacity, const pp_config *cfg, pp_ann *d_out,
                     int32_t *d_out_counts, int32_t *d_out_index, void *d_workspace,
                     size_t workspace_bytes, void *stream);

/*
 * pp_nms_keypoints with each record's own Annotation.score() (annotation.py:60-71), for
 * annotations carrying fixed_score, suppress_score_index or non-default score_weights
 * (nms.py:21, 33, 53-54 sort and filter by it).  Per (image, record), laid out like d_anns:
 * d_score_spec -2 = fixed_score (d_fixed_score holds it), -1 = none, j in [0, K) =
 * suppress_score_index (v[j] reads as 0, negative Python indices normalised by the
 * caller); d_score_weights (n_img, ann_capacity, K) float64 = the record's score_weights;
 * d_fixed_score (n_img, ann_capacity) float64.  instance_threshold replaces cfg's float32
 * nms_instance_threshold: the reference compares score() >= it in float64 (a fixed_score
 * equal to the threshold is kept).  NULL d_score_spec = the default score().
 */
int pp_nms_keypoints_scored(pp_ann *d_anns, const int32_t *d_counts, int32_t n_img, int32_t K,
                            int32_t ann_capacity, const pp_config *cfg,
                            double instance_threshold, const int32_t *d_score_spec, const double *d_score_weights,
                            const double *d_fixed_score, pp_ann *d_out, int32_t *d_out_counts,
                            int32_t *d_out_index, void *d_workspace, size_t workspace_bytes,
                            void *stream);

/*
 * Packs a decode's records (d_anns (n_img, ann_capacity), d_counts[i] valid in slot row i)
 * image after image into `out` and copies the counts to out_counts: the flattened
 * per-image Annotation lists that Generator.batch returns (generator.py:96-97), in one
 * launch.  `out` / `out_counts` may be device memory or pinned host memory
 * (hipHostMalloc / hipHostRegister; written zero-copy through its mapped device address,
 * so one stream synchronisation hands the caller every record).  Records whose packed
 * index is >= out_capacity are not written; out_counts is always complete, so the caller
 * can size a retry.
 */
int pp_pack_records(const pp_ann *d_anns, const int32_t *d_counts, int32_t n_img,
                    int32_t ann_capacity, pp_ann *out, int64_t out_capacity, int32_t *out_counts,
                    void *stream);

/*
 * The same hand-over with COMPACT records (the wire format of the host fetch and the
 * multi-GPU gather): a pp_ann cut to K keypoints, pp_packed_record_size(K, C, flags) bytes
 * (a multiple of 16), little-endian:
 *   0   f64 score                       Annotation.score()        annotation.py:60-71
 *   8   i32 image
 *   12  u16 n_decoding | PP_PACK_REFETCH (bit 15), 14 u16 n_frontier
 *   16  f32 data[K][3], f32 joint_scales[K]                       annotation.py:17-18
 *   PP_PACK_DECODING: u8 decoding_pairs[K][2] (padded to 4 B), f32 decoding_v[K][2],
 *       f32 decoding_xy[K][2]: the (jsi, jti) pairs of decoding_order (cifcaf.py:305-306),
 *       v of xyv_jsi / xyv_jti, and per joint the x / y it had when it entered the order:
 *       xyv_jsi = (decoding_xy[jsi], v[0]), xyv_jti = (decoding_xy[jti], v[1]) (checked on
 *       the device for every entry)
 *   PP_PACK_FRONTIER: u8 frontier_pairs[F][2] (padded to 4 B), F = min(PP_MAX_FRONTIER, 4*C)
 * A record whose decoding entries disagree with the per-joint x / y, or whose orders exceed
 * K / F entries, carries PP_PACK_REFETCH: fetch that decode's full pp_ann records instead.
 * `out_flags` (optional, NULL to skip; device or pinned host memory, n_img int32): set to 1
 * for an image with at least one flagged record, else 0 -- so a caller whose records stay in
 * device memory (the multi-GPU gather) learns of a refetch without reading them.
 * `out` (16-byte aligned) holds out_capacity records; device or pinned host memory as for
 * pp_pack_records.  Reference consumer: Generator.batch's per-image lists
 * (generator.py:96-97).
 */
#define PP_PACK_DECODING 1u
#define PP_PACK_FRONTIER 2u
#define PP_PACK_REFETCH 0x8000u
int64_t pp_packed_record_size(int32_t K, int32_t C, uint32_t flags);
int pp_pack_compact(const pp_ann *d_anns, const int32_t *d_counts, int32_t n_img,
                    int32_t ann_capacity, int32_t K, int32_t C, uint32_t flags, void *out,
                    int64_t out_capacity, int32_t *out_counts, int32_t *out_flags,
                    void *stream);

/*
 * The same decode split into stages for measurement: bit 1 CifHr, 2 CifSeeds,
 * 4 CafScored at caf_threshold, 8 seed loop + grow + complete + NMS (stage 8 also builds
 * the complete_caf_threshold column sets, only where force-complete needs them).  Stage buffers live
 * in the workspace, so calling the stages in order with the same workspace equals one
 * pp_decode_batch call.  pp_decode_batch == pp_decode_stages(..., 15, stream).
 * Bit 16 (PP_STAGE_COMPLETE_SETS_EARLY) moves the complete_caf_threshold column sets into
 * stage 4, built for every (field, direction) (stage 8 then reads them): the same result,
 * for callers that overlap one batch's stages 1-4 with the previous batch's stage 8.  In a
 * call with stage 1 (and without 8) they start on the library's side stream before the
 * CifHr map instead (they read only the CAF fields); a later call with stages 2 | 4 joins
 * that stream.
 * With bit 16, stage 8 may run in two calls on the same workspace and outputs: first with
 * PP_STAGE_SEED_LOOP_ONLY (32), then with PP_STAGE_AFTER_SEED_LOOP (64: force-complete and
 * NMS), so the second part can run on another stream beside the next batch's seed loop.
 * The second part may itself run as two calls: PP_STAGE_AFTER_SEED_LOOP | PP_STAGE_COMPLETE_ONLY
 * (128: force-complete), then PP_STAGE_AFTER_SEED_LOOP | PP_STAGE_NMS_ONLY (256).  NMS reads
 * only the annotation records and NMS scratch, none of which stages 1-4 write, so the
 * workspace's next stages 1-4 need wait only for the force-complete call.
 * PP_STAGE_NMS_WIDE (512, a hint for dense batches): NMS in workgroups of 8 waves instead of
 * 4 when the batch runs the one-CU seed loop (at least about CUs / 2 images).  The 4-wave
 * form fits on a CU beside a seed-loop workgroup, so an overlapped caller's NMS runs beside
 * the next batch's seed loop; the 8-wave form is faster per image on dense input
 * (hundreds of annotations per image).  With force-complete it also selects the number of
 * force-complete workgroups per image (more for dense batches).  Same results either way.
 * PP_STAGE_NMS_BITMAP (1024): NMS as three launches whose middle one decides each (image,
 * joint plane) with the plane's occupancy as a bitmap in LDS (one wave each) instead of
 * one launch walking box lists.  Same results; faster one step at a time, slower beside
 * another batch's seed loop (the many one-wave workgroups), hence opt-in.
 *
 * Workspace contract: bytes [pp_decode_workspace_zero_offset(), end) must be zero before
 * the first call (e.g. hipMemset once at allocation); every call leaves them zero again.
 */
#define PP_STAGE_COMPLETE_SETS_EARLY 16u
#define PP_STAGE_SEED_LOOP_ONLY 32u
#define PP_STAGE_AFTER_SEED_LOOP 64u
#define PP_STAGE_COMPLETE_ONLY 128u
#define PP_STAGE_NMS_ONLY 256u
#define PP_STAGE_NMS_WIDE 512u
#define PP_STAGE_NMS_BITMAP 1024u
int pp_decode_stages(const float *d_cif, const float *d_caf, int32_t n_img, int32_t K,
                     int32_t C, int32_t H, int32_t W, const int32_t *skeleton,
                     const pp_config *cfg, float *d_cifhr, pp_ann *d_anns,
                     int32_t ann_capacity, int32_t *d_counts, int32_t *d_status,
                     void *d_workspace, size_t workspace_bytes, uint32_t stages, void *stream);
size_t pp_decode_workspace_zero_offset(int32_t n_img, int32_t K, int32_t C, int32_t H,
                                       int32_t W, const pp_config *cfg, int32_t ann_capacity);

/* ---------------------------------------------------------------------------------
 * openpifpaf.functional primitives (functional.pyx).  `field` arguments are
 * (h, w) float32 with row pitch `pitch` (elements).  Point lists are length-n device
 * arrays.  All are bit-exact restatements run as HIP kernels.
 * --------------------------------------------------------------------------------- */

/* functional.pyx:105-141 */
int pp_scalar_square_add_gauss_with_max(float *d_field, int64_t h, int64_t w, int64_t pitch,
                                        const float *d_x, const float *d_y,
                                        const float *d_sigma, const float *d_v, int64_t n,
                                        float truncate, float max_value, void *stream);
/* functional.pyx:71-102 */
int pp_scalar_square_add_gauss(float *d_field, int64_t h, int64_t w, int64_t pitch,
                               const float *d_x, const float *d_y, const float *d_sigma,
                               const float *d_v, int64_t n, float truncate, void *stream);
/* functional.pyx:7-26 */
int pp_scalar_square_add_constant(float *d_field, int64_t h, int64_t w, int64_t pitch,
                                  const float *d_x, const float *d_y, const float *d_width,
                                  const float *d_v, int64_t n, void *stream);
/* functional.pyx:144-169 */
int pp_scalar_square_max_gauss(float *d_field, int64_t h, int64_t w, int64_t pitch,
                               const float *d_x, const float *d_y, const float *d_sigma,
                               const float *d_v, int64_t n, float truncate, void *stream);
/* functional.pyx:29-54 */
int pp_cumulative_average(float *d_cuma, float *d_cumw, int64_t h, int64_t w, int64_t pitch,
                          const float *d_x, const float *d_y, const float *d_width,
                          const float *d_v, const float *d_w, int64_t n, void *stream);
/* functional.pyx:172-211: x (n, d) row pitch x_pitch, y (>=2) updated in place,
 * d_denom (n) out; d_out_steps (1 int32) = iterations run */
int pp_weiszfeld_nd(const float *d_x, int64_t n, int64_t d, int64_t x_pitch, float *d_y,
                    const float *d_weights, float epsilon, int64_t max_steps, float *d_denom,
                    void *stream);
/* functional.pyx:231-244 */
int pp_scalar_values(const float *d_field, int64_t h, int64_t w, int64_t pitch,
                     const float *d_x, const float *d_y, int64_t n, float default_value,
                     float *d_out, void *stream);
/*
 * Single-point lookups, batched (functional.pyx:247-286).  mode:
 *   0 scalar_value(default)  1 scalar_value_clipped  (float field, float out)
 *   2 scalar_nonzero(default) 3 scalar_nonzero_clipped 4 ..._with_reduction(r)  (u8 field)
 */
int pp_scalar_lookup(const void *d_field, int64_t h, int64_t w, int64_t pitch, int32_t mode,
                     const float *d_x, const float *d_y, int64_t n, float default_value,
                     float reduction, void *d_out, void *stream);
/*
 * Occupancy.set (decoder/occupancy.py:36-44) with scalar_square_add_single
 * (decoder/utils.py:61-66) for n marks, in order: plane d_f[i] of d_occ (n_planes, h, w) u8
 * with row pitch `pitch` gets += 1 (wrapping) on the box of half-width
 * round(max(min_scale_reduced, sigma / reduction)) around (round(x / reduction),
 * round(y / reduction)); f32 division, round half to even, NumPy slice clipping.  Marks
 * with d_f[i] outside [0, n_planes) are skipped, as the reference's early return; marks
 * with non-finite coordinates are skipped (the reference's round() raises).  Occupancy.get
 * is pp_scalar_lookup mode 4.
 */
int pp_occupancy_set(uint8_t *d_occ, int32_t n_planes, int64_t h, int64_t w, int64_t pitch,
                     const int32_t *d_f, const float *d_x, const float *d_y, const float *d_sigma,
                     int64_t n, float reduction, float min_scale_reduced, void *stream);

/*
 * Column filters over a (rows, n) field with row pitch `pitch` (functional.pyx:214-228,
 * 289-359), order preserving.  mode: 0 caf_center_s, 1 paf_center, 2 paf_center_b,
 * 3 paf_mask_center (d_out = u8 mask (n)).  Modes 0-2 write the kept columns to
 * d_out (rows, out_pitch) and the kept count to d_count (1 int32).
 */
int pp_center_filter(const float *d_field, int64_t rows, int64_t n, int64_t pitch, int32_t mode,
                     float x, float y, float sigma, void *d_out, int64_t out_pitch,
                     int32_t *d_count, void *stream);

/*
 * CifCaf._grow_connection + _target_with_blend / _target_with_maxscore
 * (cifcaf.py:124-192; the north star's "grow_connection_blend") for one query point on a
 * (9, n) column set with row pitch `pitch`.  method bit 0: 0 blend, 1 max; bit 1: the
 * scores' np.exp correctly rounded (pp_config.exp_mode 1) instead of NumPy's SIMD exp.
 * d_out = 4 floats (x, y, scale, score); all zero when no column lies in the 2*xy_scale box.
 */
int pp_grow_connection(const float *d_cols, int64_t n, int64_t pitch, float x, float y,
                       float xy_scale, int32_t method, float *d_out, void *stream);

/*
 * np.exp of float32 values as the decoder's CAF scores take it (cifcaf.py:139, the
 * score's exp): d_y[i] = exp(d_x[i]) with pp_config.exp_mode's rounding (0 NumPy's SIMD
 * float32 routine, 1 correctly rounded).  The device form of the decoder's own function
 * (caf_exp, pp_common.hpp), for checking it against np.exp.
 */
int pp_np_exp(const float *d_x, float *d_y, int64_t n, int32_t exp_mode, void *stream);

/*
 * d_y[i] = d_x[i] ** 2 as NumPy computes it for a float32 SCALAR (cifcaf.py:139 `sigma**2`):
 * the C library's powf(x, 2.0f), glibc 2.35's FMA build, which differs from x * x in about
 * 0.07 % of inputs.  The device form of the decoder's own function (np_pow2_f32).
 */
int pp_np_square(const float *d_x, float *d_y, int64_t n, void *stream);

/* ---------------------------------------------------------------------------------
 * Host twins of the functional.pyx primitives above (SURVEY.md §8(b) `_cpu` variants):
 * the same arguments as the device entry points minus the stream, HOST pointers, run
 * sequentially on the calling thread in the reference's loop order (functional.pyx is
 * CPU-only Cython), bit-exact with it and with the kernels.  Explicit entry points only:
 * nothing in the library or its Python API falls back to them.
 * --------------------------------------------------------------------------------- */
int pp_scalar_square_add_gauss_with_max_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                            const float *x, const float *y, const float *sigma,
                                            const float *v, int64_t n, float truncate,
                                            float max_value);
int pp_scalar_square_add_gauss_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                   const float *x, const float *y, const float *sigma,
                                   const float *v, int64_t n, float truncate);
int pp_scalar_square_max_gauss_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                   const float *x, const float *y, const float *sigma,
                                   const float *v, int64_t n, float truncate);
int pp_scalar_square_add_constant_cpu(float *field, int64_t h, int64_t w, int64_t pitch,
                                      const float *x, const float *y, const float *width,
                                      const float *v, int64_t n);
int pp_cumulative_average_cpu(float *cuma, float *cumw, int64_t h, int64_t w, int64_t pitch,
                              const float *x, const float *y, const float *width,
                              const float *v, const float *w_, int64_t n);
/* pp_np_exp / pp_np_square on host pointers */
int pp_np_exp_cpu(const float *x, float *y, int64_t n, int32_t exp_mode);
int pp_np_square_cpu(const float *x, float *y, int64_t n);
/* out_steps (optional, 1 int64) = iterations run */
int pp_weiszfeld_nd_cpu(const float *x, int64_t n, int64_t d, int64_t x_pitch, float *y,
                        const float *weights, float epsilon, int64_t max_steps, float *denom,
                        int64_t *out_steps);
int pp_scalar_values_cpu(const float *field, int64_t h, int64_t w, int64_t pitch, const float *x,
                         const float *y, int64_t n, float default_value, float *out);
int pp_scalar_lookup_cpu(const void *field, int64_t h, int64_t w, int64_t pitch, int32_t mode,
                         const float *x, const float *y, int64_t n, float default_value,
                         float reduction, void *out);
int pp_occupancy_set_cpu(uint8_t *occ, int32_t n_planes, int64_t h, int64_t w, int64_t pitch,
                         const int32_t *f, const float *x, const float *y, const float *sigma,
                         int64_t n, float reduction, float min_scale_reduced);
int pp_center_filter_cpu(const float *field, int64_t rows, int64_t n, int64_t pitch, int32_t mode,
                         float x, float y, float sigma, void *out, int64_t out_pitch,
                         int32_t *count);

/* ---------------------------------------------------------------------------------
 * Host twins of the front stages (csrc/stages_cpu.hip): pp_cifhr / pp_seeds /
 * pp_caf_scored for one CIF and one CAF head with the same layouts, HOST pointers, run on
 * the calling thread in the reference's order (the stage classes are CPU-only NumPy code).
 * Explicit entry points only, as the primitives' twins above.
 *   pp_cifhr_cpu       CifHr.fill / fill_cif (cif_hr.py:23-81): cifhr (n_img, K, H', pitch),
 *                      pitch = pp_cifhr_pitch(W'), zeroed then accumulated
 *   pp_seeds_cpu       CifSeeds.fill + get (cif_seeds.py:23-64): seeds (n_img, seed_capacity)
 *                      sorted as sorted(seeds, reverse=True), counts (n_img); PP_ESHAPE when
 *                      an image has more than seed_capacity seeds
 *   pp_caf_scored_cpu  CafScored.fill (caf_scored.py:32-98) at score_th: cols
 *                      (n_img, C, 2, 9, H*W), dir 0 backward, 1 forward; counts (n_img, C, 2)
 * --------------------------------------------------------------------------------- */
int pp_cifhr_cpu(const float *cif, int32_t n_img, int32_t K, int32_t H, int32_t W,
                 const pp_config *cfg, float *cifhr);
int pp_seeds_cpu(const float *cif, const float *cifhr, int32_t n_img, int32_t K, int32_t H,
                 int32_t W, const pp_config *cfg, pp_seed *seeds, int32_t seed_capacity,
                 int32_t *counts);
int pp_caf_scored_cpu(const float *caf, const float *cifhr, int32_t n_img, int32_t K, int32_t C,
                      int32_t H, int32_t W, const int32_t *skeleton, float score_th,
                      const pp_config *cfg, float *cols, int32_t *counts);
/* nms.Keypoints.annotations (nms.py:17-57) as pp_nms_keypoints, on host records (no workspace):
 * anns edited in place, survivors sorted by -score in out with their score, out_counts,
 * out_index (optional) = each survivor's input index. */
int pp_nms_keypoints_cpu(pp_ann *anns, const int32_t *counts, int32_t n_img, int32_t K,
                         int32_t ann_capacity, const pp_config *cfg, pp_ann *out,
                         int32_t *out_counts, int32_t *out_index);
/* pp_nms_keypoints_scored on host records (each record's own Annotation.score()). */
int pp_nms_keypoints_scored_cpu(pp_ann *anns, const int32_t *counts, int32_t n_img, int32_t K,
                                int32_t ann_capacity, const pp_config *cfg,
                                double instance_threshold, const int32_t *score_spec,
                                const double *score_weights, const double *fixed_score,
                                pp_ann *out, int32_t *out_counts, int32_t *out_index);

/*
 * Host twin of pp_decode_batch (CifCaf.__call__, cifcaf.py:67-122, for a batch of one-head
 * fields; no initial annotations): CifHr, seeds and both CafScored sets through the front
 * stages' twins, the seed loop with its occupancy, _grow, complete_annotations with
 * _flood_fill (force_complete) and nms.Keypoints (apply_nms), on HOST pointers, one image
 * per task on n_threads host threads (0: one per hardware thread).  Outputs as
 * pp_decode_batch: per image ann_capacity records (counts[i] of them used, sorted by
 * nms.Keypoints) and status flags (PP_ST_*; PP_ST_ANN_OVERFLOW: more annotations than
 * ann_capacity, retry with a larger one).  Bit-exact with the device decode and with the
 * reference's fixtures (tests/test_decode_cpu.py).
 */
int pp_decode_batch_cpu(const float *cif, const float *caf, int32_t n_img, int32_t K, int32_t C,
                        int32_t H, int32_t W, const int32_t *skeleton, const pp_config *cfg,
                        pp_ann *anns, int32_t ann_capacity, int32_t *counts, int32_t *status,
                        int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif /* PIFPAF_AMD_H */
