// ingest.hip — head conv outputs -> decoder fields, one pass over HBM.
//
// Replaces the eval-mode tail of CompositeFieldFused.forward (network/heads.py:406-455):
// `quad` PixelShuffle(2) dequads with the last row / column cropped, sigmoid on the
// confidences, exp on the scales; and CifCafCollector / CifdetCollector.forward
// (heads.py:65-88, 127-144): per-field concatenation, the index grid added to the vector
// components, the channel reorder.  The result is what the decoder consumes, written
// straight from the conv output (no intermediate tensors, no host copy).
//
// Work unit: one thread per output pixel of one (image, field); it writes every output
// channel of that field.  Reads and writes are coalesced along x.
#include "pp_common.hpp"

namespace pp {

constexpr int kMaxOutCh = 16;

struct IngestArgs {
    const float *conv;   // (n_img, n_fields * n_per_field * 4^quad, h, w)
    float *out;          // (n_img, n_fields, n_out, H, W)
    int n_img, n_fields, h, w, H, W, quad;
    int n_conf, n_vec, n_scales, n_out;
    int64_t conv_ch;     // channels per image of the conv output
    // per output channel: conv channel group offset and stride per field, component, op
    int grp_off[kMaxOutCh];  // first conv channel of the component's group (pre-dequad units)
    int fld_mul[kMaxOutCh];  // channels per field inside the group
    int comp[kMaxOutCh];     // component inside the field
    int op[kMaxOutCh];       // 0 copy, 1 sigmoid, 2 exp, 3 + x index, 4 + y index
};

__global__ __launch_bounds__(256) void ingest_kernel(IngestArgs a) {
    const int64_t pix = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t HW = (int64_t)a.H * a.W;
    const int f = blockIdx.y, img = blockIdx.z;
    if (pix >= HW) return;
    const int Y = (int)(pix / a.W), X = (int)(pix % a.W);
    // undo the dequads: T_q[c, Y, X] = T_{q-1}[4c + 2(Y&1) + (X&1), Y>>1, X>>1], so the
    // conv channel is 4^quad * c + sub with the finest level's offset the most significant
    int sub = 0, y0 = Y, x0 = X, mul = 1;
    for (int q = 0; q < a.quad; q++) {
        sub = 4 * sub + (2 * (y0 & 1) + (x0 & 1));
        mul *= 4;
        y0 >>= 1;
        x0 >>= 1;
    }
    const float *src = a.conv + (int64_t)img * a.conv_ch * a.h * a.w + (int64_t)y0 * a.w + x0;
    float *dst = a.out + (((int64_t)img * a.n_fields + f) * a.n_out) * HW + pix;
    for (int o = 0; o < a.n_out; o++) {
        const int64_t ch = (int64_t)(a.grp_off[o] + f * a.fld_mul[o] + a.comp[o]) * mul + sub;
        const float v = src[ch * a.h * a.w];
        float r;
        switch (a.op[o]) {
            case 1: r = (float)(1.0 / (1.0 + exp(-(double)v))); break;  // torch.sigmoid
            case 2: r = (float)exp((double)v); break;                  // torch.exp
            case 3: r = v + (float)X; break;                           // + index_field x
            case 4: r = v + (float)Y; break;                           // + index_field y
            default: r = v;
        }
        dst[(int64_t)o * HW] = r;
    }
}

}  // namespace pp

using namespace pp;

extern "C" {

int64_t pp_fields_dim(int64_t n, int32_t quad) {
    for (int q = 0; q < quad; q++) n = 2 * n - 1;  // PixelShuffle(2) then [:-1]
    return n;
}

int pp_fields_from_conv(const float *d_conv, int32_t n_img, int32_t n_fields, int32_t layout,
                        int32_t h, int32_t w, int32_t quad, float *d_out, void *stream) {
    if (!d_conv || !d_out) return fail(PP_EINVAL, "pp_fields_from_conv: NULL argument");
    if (n_img < 0 || n_fields <= 0 || h <= 0 || w <= 0 || quad < 0 || quad > 4)
        return fail(PP_ESHAPE, "pp_fields_from_conv: bad shape");
    IngestArgs a{};
    // (n_confidences, n_vectors, n_scales) of IntensityMeta / AssociationMeta /
    // DetectionMeta (heads.py:218-265) and the collector's output channel order
    static const int metas[3][3] = {{1, 1, 1}, {1, 2, 2}, {1, 2, 0}};
    // concatenated per-field channels: conf..., vec0 x, vec0 y, vec1 x, ..., logb..., scale...
    // output channel -> concatenated channel (heads.py:87 for CAF, :142 for CifDet)
    static const int perm[3][9] = {{0, 1, 2, 3, 4, 0, 0, 0, 0},
                                   {0, 1, 2, 5, 7, 3, 4, 6, 8},
                                   {0, 1, 2, 5, 3, 4, 6, 0, 0}};
    static const int n_out[3] = {5, 9, 7};
    if (layout < 0 || layout > 2) return fail(PP_EINVAL, "pp_fields_from_conv: layout 0 CIF, 1 CAF, 2 CifDet");
    a.conv = d_conv;
    a.out = d_out;
    a.n_img = n_img;
    a.n_fields = n_fields;
    a.h = h;
    a.w = w;
    a.quad = quad;
    a.H = (int)pp_fields_dim(h, quad);
    a.W = (int)pp_fields_dim(w, quad);
    a.n_conf = metas[layout][0];
    a.n_vec = metas[layout][1];
    a.n_scales = metas[layout][2];
    a.n_out = n_out[layout];
    const int F0 = a.n_conf * n_fields, F1 = F0 + 2 * a.n_vec * n_fields,
              F2 = F1 + a.n_vec * n_fields, F3 = F2 + a.n_scales * n_fields;
    a.conv_ch = (int64_t)F3 << (2 * quad);
    const int nc = a.n_conf, nv2 = 2 * a.n_vec, nv = a.n_vec;
    for (int o = 0; o < a.n_out; o++) {
        const int q = perm[layout][o];
        if (q < nc) {  // confidences: sigmoid
            a.grp_off[o] = 0;
            a.fld_mul[o] = nc;
            a.comp[o] = q;
            a.op[o] = 1;
        } else if (q < nc + nv2) {  // vectors: index added to the first (CifDet) or all
            const int c = q - nc;
            a.grp_off[o] = F0;
            a.fld_mul[o] = nv2;
            a.comp[o] = c;
            const bool indexed = layout != 2 || c < 2;
            a.op[o] = indexed ? ((c & 1) ? 4 : 3) : 0;
        } else if (q < nc + nv2 + nv) {  // logb: as is
            a.grp_off[o] = F1;
            a.fld_mul[o] = nv;
            a.comp[o] = q - nc - nv2;
            a.op[o] = 0;
        } else {  // scales: exp
            a.grp_off[o] = F2;
            a.fld_mul[o] = a.n_scales;
            a.comp[o] = q - nc - nv2 - nv;
            a.op[o] = 2;
        }
    }
    if (n_img == 0) return PP_OK;
    const int64_t HW = (int64_t)a.H * a.W;
    const dim3 grid((unsigned)((HW + 255) / 256), (unsigned)n_fields, (unsigned)n_img);
    hipLaunchKernelGGL(ingest_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
    return check_launch("pp_fields_from_conv");
}

}  // extern "C"
