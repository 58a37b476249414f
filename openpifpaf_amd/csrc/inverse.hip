// inverse.hip — Preprocess.annotations_inverse (transforms/preprocess.py:35-95) on decoded
// records: image-space poses and boxes from network-input coordinates, one thread per
// record, batched over images (each image has its own meta).
//
// NumPy semantics, step by step: the meta's offset / scale are float64 arrays and
// width_height an int64 array (transforms/annotations.py:39-44), so those in-place steps
// on the float32 records compute in float64 and round to float32; the rotation mixes
// float32 arrays with Python floats, so it runs in float32 with the constants rounded.
#include "pp_common.hpp"

#include <math.h>

namespace pp {

__device__ __forceinline__ float npmin3(float a, float b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }
__device__ __forceinline__ float npmax3(float a, float b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }

__global__ __launch_bounds__(256) void ann_inverse_kernel(pp_ann *anns, const int *counts, int cap,
                                                          int K, const pp_inverse_meta *metas,
                                                          const int *hswap, int *nan_flags) {
    const int img = blockIdx.y;
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= min(counts[img], cap)) return;
    pp_ann &a = anns[(int64_t)img * cap + r];
    const pp_inverse_meta m = metas[img];
    const double angle = -m.rotation_angle;
    if (angle != 0.0) {  // preprocess.py:51-56, float32 with the Python floats rounded
        const float c = (float)cos(angle / 180.0 * M_PI), s = (float)sin(angle / 180.0 * M_PI);
        const float hw = (float)((m.rotation_width - 1.0) / 2.0);
        const float hh = (float)((m.rotation_height - 1.0) / 2.0);
        for (int j = 0; j < K; j++) {
            const float xo = a.data[j][0] - hw, yo = a.data[j][1] - hh;
            a.data[j][0] = (hw + c * xo) + s * yo;
            a.data[j][1] = (hh - s * xo) + c * yo;
        }
    }
    bool nan = false;
    for (int j = 0; j < K; j++) {  // offset, then scale (float64, rounded to float32)
        float x = (float)((double)a.data[j][0] + m.offset[0]);
        float y = (float)((double)a.data[j][1] + m.offset[1]);
        x = (float)((double)x / m.scale[0]);
        y = (float)((double)y / m.scale[1]);
        a.data[j][0] = x;
        a.data[j][1] = y;
        a.joint_scales[j] = (float)((double)a.joint_scales[j] / m.scale[0]);
        nan = nan || x != x || y != y || a.data[j][2] != a.data[j][2];
    }
    if (nan) atomicOr(&nan_flags[img], 1);  // the reference asserts here (preprocess.py:67)
    if (m.hflip) {
        for (int j = 0; j < K; j++)
            a.data[j][0] = (float)(-(double)a.data[j][0] + (m.width - 1.0));
        if (hswap) {  // _HorizontalSwap (hflip.py:17-29): target rows, last writer wins
            float t[PP_MAX_KP][3];
            for (int j = 0; j < K; j++) t[j][0] = t[j][1] = t[j][2] = 0.0f;
            for (int sj = 0; sj < K; sj++) {
                const int tj = hswap[sj];
                t[tj][0] = a.data[sj][0];
                t[tj][1] = a.data[sj][1];
                t[tj][2] = a.data[sj][2];
            }
            for (int j = 0; j < K; j++) {
                a.data[j][0] = t[j][0];
                a.data[j][1] = t[j][1];
                a.data[j][2] = t[j][2];
            }
        }
    }
    const int nd = min(a.n_decoding, PP_MAX_KP);
    for (int d = 0; d < nd; d++) {  // decoding_order: offset and scale only (preprocess.py:76-81)
        for (int c = 0; c < 2; c++) {
            for (int h = 0; h < 2; h++) {
                float v = (float)((double)a.decoding_xyv[d][3 * h + c] + m.offset[c]);
                a.decoding_xyv[d][3 * h + c] = (float)((double)v / m.scale[c]);
            }
        }
    }
}

// anndet_inverse (preprocess.py:84-95) with utils.rotate_box (transforms/utils.py:5-28)
__global__ __launch_bounds__(256) void det_inverse_kernel(pp_det *dets, const int *counts, int cap,
                                                          const pp_inverse_meta *metas) {
    const int img = blockIdx.y;
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= min(counts[img], cap)) return;
    pp_det &d = dets[(int64_t)img * cap + r];
    const pp_inverse_meta m = metas[img];
    const double angle = -m.rotation_angle;
    float b[4] = {d.bbox[0], d.bbox[1], d.bbox[2], d.bbox[3]};
    if (angle != 0.0) {
        const float c = (float)cos(angle / 180.0 * M_PI), s = (float)sin(angle / 180.0 * M_PI);
        const float w2 = (float)((m.rotation_width - 1.0) / 2.0);
        const float h2 = (float)((m.rotation_height - 1.0) / 2.0);
        const float cx[4] = {b[0], b[0] + b[2], b[0], b[0] + b[2]};
        const float cy[4] = {b[1], b[1], b[1] + b[3], b[1] + b[3]};
        float rx[4], ry[4];
        for (int i = 0; i < 4; i++) {
            const float xo = cx[i] - w2, yo = cy[i] - h2;
            rx[i] = (w2 + c * xo) + s * yo;
            ry[i] = (h2 - s * xo) + c * yo;
        }
        float x = rx[0], y = ry[0], xm = rx[0], ym = ry[0];
        for (int i = 1; i < 4; i++) {
            x = npmin3(x, rx[i]);
            y = npmin3(y, ry[i]);
            xm = npmax3(xm, rx[i]);
            ym = npmax3(ym, ry[i]);
        }
        b[0] = x;
        b[1] = y;
        b[2] = xm - x;
        b[3] = ym - y;
    }
    b[0] = (float)((double)b[0] + m.offset[0]);
    b[1] = (float)((double)b[1] + m.offset[1]);
    b[0] = (float)((double)b[0] / m.scale[0]);
    b[1] = (float)((double)b[1] / m.scale[1]);
    b[2] = (float)((double)b[2] / m.scale[0]);
    b[3] = (float)((double)b[3] / m.scale[1]);
    for (int i = 0; i < 4; i++) d.bbox[i] = b[i];
}

// -------------------------------------------------------------------------------------
// record packing: the per-image record slots of a decode, image after image, into one
// caller buffer (Generator.batch's list of per-image Annotation lists, generator.py:96-97,
// flattened); the destination may be mapped pinned host memory (zero-copy)
// -------------------------------------------------------------------------------------
// One workgroup per image: the image's offset is the sum of the earlier counts (read by
// the whole workgroup, n is small), then its records are copied as 8-byte words (a record
// is 1544 = 8 * 193 bytes).  Records at packed index >= out_cap are not written.
__global__ __launch_bounds__(256) void pack_records_kernel(const pp_ann *__restrict__ anns,
                                                           const int *__restrict__ counts, int n,
                                                           int cap, pp_ann *out, int64_t out_cap,
                                                           int *out_counts) {
    __shared__ int s_off;
    const int img = blockIdx.x;
    if (threadIdx.x == 0) s_off = 0;
    __syncthreads();
    int part = 0;
    for (int j = threadIdx.x; j < img; j += 256) part += counts[j];
    if (part) atomicAdd(&s_off, part);
    __syncthreads();
    const int64_t off = s_off;
    const int cnt = counts[img];
    if (threadIdx.x == 0) out_counts[img] = cnt;
    const int64_t fit = min((int64_t)cnt, max((int64_t)0, out_cap - off));
    constexpr int kWords = sizeof(pp_ann) / 8;
    static_assert(sizeof(pp_ann) % 8 == 0, "pp_ann is copied in 8-byte words");
    const uint64_t *src = reinterpret_cast<const uint64_t *>(anns + (int64_t)img * cap);
    uint64_t *dst = reinterpret_cast<uint64_t *>(out + off);
    // 16-byte stores (the destination is usually across PCIe, where wide writes pay):
    // one leading 8-byte word when the destination is 8 mod 16, then word pairs, each
    // assembled from two 8-byte loads, then a trailing word
    const int64_t words = fit * kWords;
    const int64_t lead = (reinterpret_cast<uintptr_t>(dst) & 8) ? min(words, (int64_t)1) : 0;
    const int64_t pairs = (words - lead) >> 1;
    if (threadIdx.x == 0 && lead) dst[0] = src[0];
    typedef uint64_t v2u __attribute__((ext_vector_type(2)));
    v2u *dst2 = reinterpret_cast<v2u *>(dst + lead);
    for (int64_t i = threadIdx.x; i < pairs; i += 256) {
        v2u v;
        v.x = src[lead + 2 * i];
        v.y = src[lead + 2 * i + 1];
        dst2[i] = v;
    }
    if (threadIdx.x == 0 && lead + 2 * pairs < words) dst[words - 1] = src[words - 1];
}

// -------------------------------------------------------------------------------------
// compact records (pp_pack_compact): a pp_ann cut to K keypoints and the skeleton's frontier
// bound, for the PCIe hand-over and the multi-GPU gather.  decoding_order keeps the pairs,
// the two v of each entry and, once per joint, the x / y the joint had when it entered the
// order (set once by _grow, cifcaf.py:300-306; nms.Keypoints may zero the data row later,
// nms.py:22, so the data rows cannot stand in for them).  The kernel checks that every
// entry's coordinates equal its joints' recorded x / y bit for bit; a record where that does
// not hold, or whose orders exceed the compact bounds, is flagged PP_PACK_REFETCH for a
// full-record fetch.
// -------------------------------------------------------------------------------------
struct PackLayout {
    int K, F, dec, front;
    int off_data, off_scales, off_pairs, off_decv, off_decxy, off_front, size;
};

__host__ __device__ inline PackLayout pack_layout(int K, int C, uint32_t flags) {
    PackLayout L{};
    L.K = K;
    L.F = min(PP_MAX_FRONTIER, 4 * C);  // frontier_order: <= 2C edges per _grow, grow + complete
    L.dec = (flags & PP_PACK_DECODING) != 0;
    L.front = (flags & PP_PACK_FRONTIER) != 0;
    int o = 16;
    L.off_data = o;
    o += 12 * K;
    L.off_scales = o;
    o += 4 * K;
    L.off_pairs = o;
    if (L.dec) o += (2 * K + 3) / 4 * 4;
    L.off_decv = o;
    if (L.dec) o += 8 * K;
    L.off_decxy = o;
    if (L.dec) o += 8 * K;
    L.off_front = o;
    if (L.front) o += (2 * L.F + 3) / 4 * 4;
    L.size = (o + 15) / 16 * 16;
    return L;
}

// 4-byte word i of the compact record of `a` (w3 = the count word; jxy = the wave's LDS
// copy of the recorded joint coordinates)
__device__ __forceinline__ uint32_t packed_word(const pp_ann &a, const PackLayout &L, int i,
                                                uint32_t w3, const float *jxy) {
    const uint32_t *s = reinterpret_cast<const uint32_t *>(&a);
    const int b = 4 * i;
    if (i < 2) return s[offsetof(pp_ann, score) / 4 + i];
    if (i == 2) return (uint32_t)a.image;
    if (i == 3) return w3;
    if (b < L.off_scales) return s[offsetof(pp_ann, data) / 4 + (b - L.off_data) / 4];
    if (b < L.off_pairs) return s[offsetof(pp_ann, joint_scales) / 4 + (b - L.off_scales) / 4];
    const int nd = min(a.n_decoding, L.K), nf = min(a.n_frontier, L.F);
    if (b < L.off_decv) {  // pairs bytes [q, q + 4) of the first nd entries
        const int q = b - L.off_pairs;
        uint32_t w = s[offsetof(pp_ann, decoding_pairs) / 4 + q / 4];
        const int keep = min(max(2 * nd - q, 0), 4);
        return keep == 4 ? w : (w & ((1u << (8 * keep)) - 1u));
    }
    if (b < L.off_decxy) {  // (v of the source joint, v of the target joint) per entry
        const int t = (b - L.off_decv) / 4, e = t >> 1;
        return e < nd ? __float_as_uint(a.decoding_xyv[e][2 + 3 * (t & 1)]) : 0u;
    }
    if (b < L.off_front) {  // (x, y) per joint as it entered decoding_order
        return __float_as_uint(jxy[(b - L.off_decxy) / 4]);
    }
    if (b < L.off_front + (2 * L.F + 3) / 4 * 4 && L.front) {
        const int q = b - L.off_front;
        uint32_t w = s[offsetof(pp_ann, frontier_pairs) / 4 + q / 4];
        const int keep = min(max(2 * nf - q, 0), 4);
        return keep == 4 ? w : (w & ((1u << (8 * keep)) - 1u));
    }
    return 0u;
}

// One workgroup per image (offset = the sum of the earlier counts), one wave per record,
// lane = one 16-byte chunk of the compact record (16-byte stores; the destination is
// usually mapped host memory across PCIe).
__global__ __launch_bounds__(256) void pack_compact_kernel(const pp_ann *__restrict__ anns,
                                                           const int *__restrict__ counts, int n,
                                                           int cap, PackLayout L, char *out,
                                                           int64_t out_cap, int *out_counts,
                                                           int *out_flags) {
    __shared__ int s_off, s_bad;
    __shared__ float s_jxy[4][2 * PP_MAX_KP];
    const int img = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) s_off = s_bad = 0;
    __syncthreads();
    int part = 0;
    for (int j = threadIdx.x; j < img; j += 256) part += counts[j];
    if (part) atomicAdd(&s_off, part);
    __syncthreads();
    const int64_t off = s_off;
    const int cnt = counts[img];
    if (threadIdx.x == 0) out_counts[img] = cnt;
    const int fit = (int)min((int64_t)min(cnt, cap), max((int64_t)0, out_cap - off));
    const int chunks = L.size / 16;
    for (int r = wave; r < fit; r += 4) {
        const pp_ann &a = anns[(int64_t)img * cap + r];
        // compact form: lane j records joint j's x / y at its first appearance in
        // decoding_order; every entry must agree with its joints' records
        const int nd = a.n_decoding, nf = a.n_frontier;
        const int ndc = min(max(nd, 0), L.K);
        bool bad = (L.dec && nd > L.K) || (L.front && nf > L.F) || nd < 0 || nf < 0;
        float jx = 0.0f, jy = 0.0f;
        if (L.dec) {
            bool found = false;
            for (int e = 0; e < ndc; e++) {  // wave-uniform walk, nd <= K entries
                const int js = a.decoding_pairs[e][0], jt = a.decoding_pairs[e][1];
                if (!found && (js == lane || jt == lane)) {
                    const int h = js == lane ? 0 : 3;
                    jx = a.decoding_xyv[e][h];
                    jy = a.decoding_xyv[e][h + 1];
                    found = true;
                }
            }
            int js = 0, jt = 0;
            if (lane < ndc) {
                js = a.decoding_pairs[lane][0];
                jt = a.decoding_pairs[lane][1];
                bad |= js >= L.K || jt >= L.K;
            }
            const float sx = __shfl(jx, js), sy = __shfl(jy, js);
            const float tx = __shfl(jx, jt), ty = __shfl(jy, jt);
            if (lane < ndc) {
                const float *x = a.decoding_xyv[lane];
                bad |= __float_as_uint(x[0]) != __float_as_uint(sx) ||
                       __float_as_uint(x[1]) != __float_as_uint(sy) ||
                       __float_as_uint(x[3]) != __float_as_uint(tx) ||
                       __float_as_uint(x[4]) != __float_as_uint(ty);
            }
        }
        bad = __ballot(bad) != 0ull;
        if (bad && lane == 0) s_bad = 1;
        if (lane < L.K) {
            s_jxy[wave][2 * lane] = jx;
            s_jxy[wave][2 * lane + 1] = jy;
        }
        wave_sync();
        const uint32_t w3 = (uint32_t)(L.dec ? min(nd, L.K) : 0) | (bad ? PP_PACK_REFETCH : 0u) |
                            ((uint32_t)(L.front ? min(nf, L.F) : 0) << 16);
        uint4 *dst = reinterpret_cast<uint4 *>(out + (off + r) * (int64_t)L.size);
        for (int c = lane; c < chunks; c += 64) {
            uint4 v;
            v.x = packed_word(a, L, 4 * c, w3, s_jxy[wave]);
            v.y = packed_word(a, L, 4 * c + 1, w3, s_jxy[wave]);
            v.z = packed_word(a, L, 4 * c + 2, w3, s_jxy[wave]);
            v.w = packed_word(a, L, 4 * c + 3, w3, s_jxy[wave]);
            dst[c] = v;
        }
        wave_sync();  // s_jxy is rewritten for the wave's next record
    }
    if (out_flags) {  // one plain store per image: no atomics across PCIe
        __syncthreads();
        if (threadIdx.x == 0) out_flags[img] = s_bad;
    }
}

}  // namespace pp

using namespace pp;

extern "C" {

int pp_annotations_inverse(pp_ann *d_anns, const int32_t *d_counts, int32_t n_img,
                           int32_t capacity, int32_t K, const pp_inverse_meta *d_metas,
                           const int32_t *d_hswap, int32_t *d_nan_flags, void *stream) {
    if (!d_anns || !d_counts || !d_metas || !d_nan_flags)
        return fail(PP_EINVAL, "pp_annotations_inverse: NULL argument");
    if (n_img < 0 || capacity <= 0 || K <= 0 || K > PP_MAX_KP)
        return fail(PP_ESHAPE, "pp_annotations_inverse: bad shape");
    if (n_img == 0) return PP_OK;
    const dim3 grid((unsigned)((capacity + 255) / 256), (unsigned)n_img);
    hipLaunchKernelGGL(ann_inverse_kernel, grid, dim3(256), 0, (hipStream_t)stream, d_anns,
                       d_counts, capacity, K, d_metas, d_hswap, d_nan_flags);
    return check_launch("pp_annotations_inverse");
}

int pp_dets_inverse(pp_det *d_dets, const int32_t *d_counts, int32_t n_img, int32_t capacity,
                    const pp_inverse_meta *d_metas, void *stream) {
    if (!d_dets || !d_counts || !d_metas) return fail(PP_EINVAL, "pp_dets_inverse: NULL argument");
    if (n_img < 0 || capacity <= 0) return fail(PP_ESHAPE, "pp_dets_inverse: bad shape");
    if (n_img == 0) return PP_OK;
    const dim3 grid((unsigned)((capacity + 255) / 256), (unsigned)n_img);
    hipLaunchKernelGGL(det_inverse_kernel, grid, dim3(256), 0, (hipStream_t)stream, d_dets,
                       d_counts, capacity, d_metas);
    return check_launch("pp_dets_inverse");
}

int pp_pack_records(const pp_ann *d_anns, const int32_t *d_counts, int32_t n_img,
                    int32_t ann_capacity, pp_ann *out, int64_t out_capacity, int32_t *out_counts,
                    void *stream) {
    if (!d_anns || !d_counts || !out || !out_counts)
        return fail(PP_EINVAL, "pp_pack_records: NULL argument");
    if (n_img < 0 || ann_capacity <= 0 || out_capacity < 0)
        return fail(PP_ESHAPE, "pp_pack_records: bad shape");
    if (n_img == 0) return PP_OK;
    // destinations as the device sees them: device memory as is, pinned host memory
    // (hipHostMalloc / registered) through its mapped device address
    void *dst[2] = {out, out_counts};
    for (void *&d : dst) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, d) != hipSuccess || !at.devicePointer ||
            (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeHost)) {
            (void)hipGetLastError();
            return fail(PP_EINVAL, "pp_pack_records: destination is neither device memory nor "
                                   "pinned host memory");
        }
        d = at.devicePointer;
    }
    hipLaunchKernelGGL(pack_records_kernel, dim3((unsigned)n_img), dim3(256), 0,
                       (hipStream_t)stream, d_anns, d_counts, n_img, ann_capacity,
                       (pp_ann *)dst[0], out_capacity, (int *)dst[1]);
    return check_launch("pp_pack_records");
}

int64_t pp_packed_record_size(int32_t K, int32_t C, uint32_t flags) {
    if (K <= 0 || K > PP_MAX_KP || C <= 0 || C > PP_MAX_EDGES) return 0;
    return pack_layout(K, C, flags).size;
}

int pp_pack_compact(const pp_ann *d_anns, const int32_t *d_counts, int32_t n_img,
                    int32_t ann_capacity, int32_t K, int32_t C, uint32_t flags, void *out,
                    int64_t out_capacity, int32_t *out_counts, int32_t *out_flags,
                    void *stream) {
    if (!d_anns || !d_counts || !out || !out_counts)
        return fail(PP_EINVAL, "pp_pack_compact: NULL argument");
    if (n_img < 0 || ann_capacity <= 0 || out_capacity < 0 || K <= 0 || K > PP_MAX_KP || C <= 0 ||
        C > PP_MAX_EDGES)
        return fail(PP_ESHAPE, "pp_pack_compact: bad shape");
    if (flags & ~(uint32_t)(PP_PACK_DECODING | PP_PACK_FRONTIER))
        return fail(PP_EINVAL, "pp_pack_compact: unknown flag");
    if (n_img == 0) return PP_OK;
    void *dst[3] = {out, out_counts, out_flags};
    for (void *&d : dst) {
        if (!d) continue;  // out_flags is optional
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, d) != hipSuccess || !at.devicePointer ||
            (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeHost)) {
            (void)hipGetLastError();
            return fail(PP_EINVAL, "pp_pack_compact: destination is neither device memory nor "
                                   "pinned host memory");
        }
        d = at.devicePointer;
    }
    if (reinterpret_cast<uintptr_t>(dst[0]) & 15)
        return fail(PP_EINVAL, "pp_pack_compact: destination not 16-byte aligned");
    hipLaunchKernelGGL(pack_compact_kernel, dim3((unsigned)n_img), dim3(256), 0,
                       (hipStream_t)stream, d_anns, d_counts, n_img, ann_capacity,
                       pack_layout(K, C, flags), (char *)dst[0], out_capacity, (int *)dst[1],
                       (int *)dst[2]);
    return check_launch("pp_pack_compact");
}

}  // extern "C"
