/*
 * asan_main.c — sanitizer driver for the oracle (TEST INFRASTRUCTURE; SURVEY.md §5
 * "Race detection / sanitizers").  Built by `make -C oracle asan` with
 * -fsanitize=address,undefined together with pp_oracle.c, run by
 * tests/test_oracle_asan.py: random uniform-style fields (synthetic.uniform's recipe with a
 * xorshift generator) through every decode entry point at odd shapes, both modes, the COCO
 * skeleton and a 44-edge one, a 2-head multi-scale list, CifDet, NMS and the primitives'
 * edge cases (empty lists, boxes past the field).  Any invalid access or UB aborts.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pifpaf_amd.h"

long orc_decode(const float *, const float *, int, int, int, int, const int32_t *,
                const pp_config *, pp_ann *, long);
long orc_decode_multi(const pp_scale *, int, int, int, int, const int32_t *, const pp_config *,
                      pp_ann *, long);
long orc_cifdet_decode(const float *, int, int, int, const pp_config *, const pp_det_nms *,
                       pp_det *, long);
long orc_nms_keypoints(pp_ann *, long, int, const pp_config *);
void orc_scalar_square_add_gauss_with_max(float *, long, long, long, long, const float *,
                                          const float *, const float *, const float *, long,
                                          float, float);

static uint64_t rng = 88172645463325252ull;
static float urand(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (float)((rng >> 40) * (1.0 / 16777216.0));
}

/* COCO person skeleton (1-based), then 25 further joint pairs for a 44-edge skeleton */
static const int32_t COCO[19][2] = {{16, 14}, {14, 12}, {17, 15}, {15, 13}, {12, 13}, {6, 12},
                                    {7, 13},  {6, 7},   {6, 8},   {7, 9},   {8, 10},  {9, 11},
                                    {2, 3},   {1, 2},   {1, 3},   {2, 4},   {3, 5},   {4, 6},
                                    {5, 7}};

static void fields(float *cif, float *caf, int K, int C, int H, int W) {
    for (int f = 0; f < K; f++)
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                float *p = cif + (size_t)f * 5 * H * W + (size_t)y * W + x;
                const float c = urand();
                p[0] = c * c * c * c;
                p[(size_t)H * W] = (float)x + urand() - 0.5f;
                p[(size_t)2 * H * W] = (float)y + urand() - 0.5f;
                p[(size_t)3 * H * W] = urand();
                p[(size_t)4 * H * W] = 0.5f + 3.0f * urand();
            }
    for (int f = 0; f < C; f++)
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                float *p = caf + (size_t)f * 9 * H * W + (size_t)y * W + x;
                const size_t s = (size_t)H * W;
                const float c = urand();
                p[0] = c * c * c * c;
                p[s] = (float)x + urand() - 0.5f;
                p[2 * s] = (float)y + urand() - 0.5f;
                p[3 * s] = urand();
                p[4 * s] = 0.5f + 3.0f * urand();
                p[5 * s] = (float)x + 4.0f * (urand() - 0.5f);
                p[6 * s] = (float)y + 4.0f * (urand() - 0.5f);
                p[7 * s] = urand();
                p[8 * s] = 0.5f + 3.0f * urand();
            }
}

static pp_config config(int eval) {
    pp_config c;
    memset(&c, 0, sizeof(c));
    c.cif_threshold = 0.1f;
    c.seed_threshold = eval ? 0.2f : 0.5f;
    c.seed_score_scale = 1.0f;
    c.caf_threshold = 0.1f;
    c.complete_caf_threshold = 0.0001f;
    c.cif_floor = 0.1f;
    c.keypoint_threshold = eval ? 0.0f : 0.001f;
    c.nms_keypoint_threshold = eval ? 0.0f : 0.001f;
    c.nms_instance_threshold = eval ? 0.0f : 0.1f;
    c.stride = 8;
    c.cif_neighbors = 16;
    c.force_complete = eval;
    c.apply_nms = 1;
    c.occupancy_reduction = 2;
    c.occupancy_min_scale = 4;
    return c;
}

int main(void) {
    const int K = 17, cap = 4096;
    int32_t skel[44][2];
    for (int e = 0; e < 19; e++) skel[e][0] = COCO[e][0], skel[e][1] = COCO[e][1];
    for (int e = 19; e < 44; e++) {  /* extra pairs of distinct joints */
        skel[e][0] = 1 + (e * 7) % K;
        skel[e][1] = 1 + (e * 7 + 3 + e % 5) % K;
    }
    pp_ann *out = (pp_ann *)malloc(sizeof(pp_ann) * cap);
    const int shapes[][2] = {{1, 1}, {3, 7}, {10, 10}, {16, 21}, {24, 24}};
    long total = 0;
    for (int si = 0; si < 5; si++) {
        const int H = shapes[si][0], W = shapes[si][1];
        for (int C = 19; C <= 44; C += 25) {
            float *cif = (float *)malloc(sizeof(float) * K * 5 * H * W);
            float *caf = (float *)malloc(sizeof(float) * C * 9 * H * W);
            fields(cif, caf, K, C, H, W);
            for (int eval = 0; eval < 2; eval++) {
                pp_config cfg = config(eval);
                for (int method = 0; method < 2; method++) {
                    cfg.connection_method = method;
                    cfg.greedy = method;
                    long n = orc_decode(cif, caf, K, C, H, W, &skel[0][0], &cfg, out, cap);
                    if (n < 0 || n > cap) return 1;
                    total += n;
                    if (n > 1) orc_nms_keypoints(out, n, K, &cfg);
                }
            }
            free(cif);
            free(caf);
        }
        /* two heads: stride 8 and stride 16 over the same image size */
        {
            const int H2 = (H - 1) / 2 + 1, W2 = (W - 1) / 2 + 1;
            float *c1 = (float *)malloc(sizeof(float) * K * 5 * H * W);
            float *a1 = (float *)malloc(sizeof(float) * 19 * 9 * H * W);
            float *c2 = (float *)malloc(sizeof(float) * K * 5 * H2 * W2);
            float *a2 = (float *)malloc(sizeof(float) * 19 * 9 * H2 * W2);
            fields(c1, a1, K, 19, H, W);
            fields(c2, a2, K, 19, H2, W2);
            pp_scale sc[2];
            memset(sc, 0, sizeof(sc));
            sc[0].cif = c1, sc[0].caf = a1, sc[0].H = H, sc[0].W = W, sc[0].stride = 8;
            sc[1].cif = c2, sc[1].caf = a2, sc[1].H = H2, sc[1].W = W2, sc[1].stride = 16;
            sc[1].cif_min_scale = 12.0f, sc[1].caf_min_distance = 36.0f;
            sc[0].caf_max_distance = 160.0f;
            pp_config cfg = config(1);
            long n = orc_decode_multi(sc, 2, 0, K, 19, &skel[0][0], &cfg, out, cap);
            if (n < 0 || n > cap) return 2;
            total += n;
            free(c1), free(a1), free(c2), free(a2);
        }
        /* CifDet: 3 categories, 7-channel fields */
        {
            float *det = (float *)malloc(sizeof(float) * 3 * 7 * H * W);
            for (long i = 0; i < 3L * 7 * H * W; i++) det[i] = urand() * 4.0f;
            pp_det *dets = (pp_det *)malloc(sizeof(pp_det) * cap);
            pp_det_nms z = {0.1f, 0.3f, 0.1f, 0.7f, 0.5f, 1};
            pp_config cfg = config(1);
            cfg.seed_threshold = 0.1f;
            long n = orc_cifdet_decode(det, 3, H, W, &cfg, &z, dets, cap);
            if (n < 0) return 3;
            free(det), free(dets);
        }
    }
    /* primitive edge cases: empty list, splats far outside the field */
    {
        float field[6 * 5] = {0};
        const float x[3] = {-100.0f, 2.5f, 1e9f}, y[3] = {2.0f, -50.0f, 3.0f},
                    s[3] = {1.0f, 40.0f, 2.0f}, v[3] = {0.5f, 0.5f, 0.5f};
        orc_scalar_square_add_gauss_with_max(field, 6, 5, 5, 1, x, y, s, v, 0, 2.0f, 1.0f);
        orc_scalar_square_add_gauss_with_max(field, 6, 5, 5, 1, x, y, s, v, 3, 2.0f, 1.0f);
    }
    free(out);
    printf("asan ok: %ld annotations\n", total);
    return 0;
}
