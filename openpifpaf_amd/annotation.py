"""Output record of the decoder: same interface as openpifpaf/annotation.py:9-119."""
import numpy as np

NOTSET = '__notset__'


class Annotation:
    """One pose.  data (K, 3) float32 [x, y, v], joint_scales (K,) float32."""

    def __init__(self, keypoints, skeleton, *, category_id=1, suppress_score_index=None):
        self.keypoints = keypoints
        self.skeleton = skeleton
        self.category_id = category_id
        self.suppress_score_index = suppress_score_index
        k = len(keypoints)
        self.data = np.zeros((k, 3), dtype=np.float32)
        self.joint_scales = np.zeros((k,), dtype=np.float32)
        self.fixed_score = NOTSET
        self.decoding_order = []
        self.frontier_order = []
        self.skeleton_m1 = (np.asarray(skeleton) - 1).tolist()
        # annotation.py:24-28: weight 3 for the first three joints, normalised in float64
        w = np.ones((k,))
        if suppress_score_index:
            w[-1] = 0.0
        w[:3] = 3.0
        self.score_weights = w / np.sum(w)

    @classmethod
    def from_record(cls, rec, keypoints, skeleton):
        """Build from one pp_ann record (include/pifpaf_amd.h)."""
        k = len(keypoints)
        ann = cls(keypoints, skeleton)
        ann.data = np.array(rec['data'][:k], dtype=np.float32)
        ann.joint_scales = np.array(rec['joint_scales'][:k], dtype=np.float32)
        nd = int(rec['n_decoding'])
        pairs = rec['decoding_pairs']
        xyv = rec['decoding_xyv']
        ann.decoding_order = [(int(pairs[t, 0]), int(pairs[t, 1]), xyv[t, :3].copy(),
                               xyv[t, 3:].copy()) for t in range(min(nd, len(pairs)))]
        fr = rec['frontier_pairs']
        ann.frontier_order = [(int(fr[t, 0]), int(fr[t, 1]))
                              for t in range(min(int(rec['n_frontier']), len(fr)))]
        return ann

    def update_from_record(self, rec):
        """Take data, joint scales and both orders from a pp_ann record: what the
        reference's decoder does to an initial annotation in place (cifcaf.py:95-98 grows
        it, complete_annotations and nms.Keypoints mutate it)."""
        new = Annotation.from_record(rec, self.keypoints, self.skeleton)
        self.data = new.data
        self.joint_scales = new.joint_scales
        self.decoding_order = new.decoding_order
        self.frontier_order = new.frontier_order
        return self

    def to_record(self):
        """This annotation as a pp_ann record (the input form of pp_decode_initial)."""
        from ._abi import ANN_DTYPE, PP_MAX_FRONTIER, PP_MAX_KP  # pylint: disable=import-outside-toplevel
        k = len(self.data)
        if k > PP_MAX_KP or len(self.decoding_order) > PP_MAX_KP or \
                len(self.frontier_order) > PP_MAX_FRONTIER:
            raise ValueError('annotation exceeds the record bounds (PP_MAX_KP keypoints / '
                             'decoding entries, PP_MAX_FRONTIER frontier entries)')
        r = np.zeros((), ANN_DTYPE)
        r['data'][:k] = self.data
        r['joint_scales'][:k] = self.joint_scales
        r['n_keypoints'] = k
        r['n_decoding'] = len(self.decoding_order)
        for t, (js, jt, xa, xb) in enumerate(self.decoding_order):
            r['decoding_pairs'][t] = (js, jt)
            r['decoding_xyv'][t, :3] = xa
            r['decoding_xyv'][t, 3:] = xb
        r['n_frontier'] = len(self.frontier_order)
        for t, pair in enumerate(self.frontier_order):
            r['frontier_pairs'][t] = pair
        return r

    @classmethod
    def from_packed(cls, rec, keypoints, skeleton):
        """Build from one compact record (pp_pack_compact, include/pifpaf_amd.h): each
        decoding_order entry is (jsi, jti, (x, y of jsi, v), (x, y of jti, v)) from the
        per-joint coordinates and the entry's two v values."""
        k = len(keypoints)
        ann = cls(keypoints, skeleton)
        ann.data = np.array(rec['data'][:k], dtype=np.float32)
        ann.joint_scales = np.array(rec['joint_scales'][:k], dtype=np.float32)
        names = rec.dtype.names
        if int(rec['n_decoding']) & 0x8000:  # PP_PACK_REFETCH: the compact form is incomplete
            raise ValueError('compact record flagged PP_PACK_REFETCH: its decoding / frontier '
                             'order does not fit; fetch the full pp_ann record instead')
        if 'decoding_pairs' in names:
            nd = int(rec['n_decoding'])
            pairs, dv, dxy = rec['decoding_pairs'], rec['decoding_v'], rec['decoding_xy']
            order = []
            for t in range(nd):
                js, jt = int(pairs[t, 0]), int(pairs[t, 1])
                a = np.array([dxy[js, 0], dxy[js, 1], dv[t, 0]], dtype=np.float32)
                b = np.array([dxy[jt, 0], dxy[jt, 1], dv[t, 1]], dtype=np.float32)
                order.append((js, jt, a, b))
            ann.decoding_order = order
        if 'frontier_pairs' in names:
            fr = rec['frontier_pairs']
            ann.frontier_order = [(int(fr[t, 0]), int(fr[t, 1]))
                                  for t in range(int(rec['n_frontier']))]
        return ann

    @classmethod
    def from_any(cls, rec, keypoints, skeleton):
        """Full pp_ann record or compact record."""
        if 'decoding_xyv' in rec.dtype.names:
            return cls.from_record(rec, keypoints, skeleton)
        return cls.from_packed(rec, keypoints, skeleton)

    def add(self, joint_i, xyv):
        self.data[joint_i] = xyv
        return self

    def set(self, data, joint_scales=None, *, fixed_score=NOTSET):
        self.data = data
        if joint_scales is not None:
            self.joint_scales = joint_scales
        else:
            self.joint_scales[:] = 0.0
        self.fixed_score = fixed_score
        return self

    def rescale(self, scale_factor):
        self.data[:, 0:2] *= scale_factor
        if self.joint_scales is not None:
            self.joint_scales *= scale_factor
        for _, __, c1, c2 in self.decoding_order:
            c1[:2] *= scale_factor
            c2[:2] *= scale_factor
        return self

    def fill_joint_scales(self, scales, hr_scale=1.0):
        from .functional import scalar_value_clipped  # pylint: disable=import-outside-toplevel
        self.joint_scales = np.zeros((self.data.shape[0],))
        for i, xyv in enumerate(self.data):
            if xyv[2] == 0.0:
                continue
            s = scalar_value_clipped(scales[i], xyv[0] * hr_scale, xyv[1] * hr_scale)
            self.joint_scales[i] = s / hr_scale

    def score(self):
        """annotation.py:60-71: weighted sum of the sorted visibilities (float64)."""
        if self.fixed_score != NOTSET:
            return self.fixed_score
        v = self.data[:, 2]
        if self.suppress_score_index is not None:
            v = np.copy(v)
            v[self.suppress_score_index] = 0.0
        return np.sum(self.score_weights * np.sort(v)[::-1])

    def scale(self, v_th=0.5):
        m = self.data[:, 2] > v_th
        if not np.any(m):
            return 0.0
        return max(np.max(self.data[m, 0]) - np.min(self.data[m, 0]),
                   np.max(self.data[m, 1]) - np.min(self.data[m, 1]))

    def json_data(self):
        """annotation.py:82-104: rounded to 2 decimals, visible keypoints kept >= 0.01."""
        v_mask = self.data[:, 2] > 0.0
        keypoints = np.copy(self.data)
        keypoints[v_mask, 2] = np.maximum(0.01, keypoints[v_mask, 2])
        keypoints = np.around(keypoints.astype(np.float64), 2)
        data = {
            'keypoints': keypoints.reshape(-1).tolist(),
            'bbox': [round(float(c), 2) for c in self.bbox()],
            'score': max(0.001, round(self.score(), 3)),
            'category_id': self.category_id,
        }
        id_ = getattr(self, 'id_', None)
        if id_:
            data['id_'] = id_
        return data

    def bbox(self):
        return self.bbox_from_keypoints(self.data, self.joint_scales)

    @staticmethod
    def bbox_from_keypoints(kps, joint_scales):
        m = kps[:, 2] > 0
        if not np.any(m):
            return [0, 0, 0, 0]
        x = np.min(kps[:, 0][m] - joint_scales[m])
        y = np.min(kps[:, 1][m] - joint_scales[m])
        w = np.max(kps[:, 0][m] + joint_scales[m]) - x
        h = np.max(kps[:, 1][m] + joint_scales[m]) - y
        return [x, y, w, h]


class AnnotationDet:
    """One detection (annotation.py:122-145): category field_i, score, bbox (x, y, w, h)."""

    def __init__(self, categories):
        self.categories = categories
        self.field_i = None
        self.score = None
        self.bbox = None

    def set(self, field_i, score, bbox):
        """Set score to None for a ground truth annotation."""
        self.field_i = field_i
        self.score = score
        self.bbox = np.asarray(bbox)
        return self

    @classmethod
    def from_record(cls, rec, categories):
        """Build from one pp_det record (include/pifpaf_amd.h)."""
        return cls(categories).set(int(rec['field']), np.float32(rec['score']),
                                   np.array(rec['bbox'], dtype=np.float32))

    @property
    def category(self):
        return self.categories[self.field_i]

    def json_data(self):
        return {
            'category_id': self.field_i + 1,
            'category': self.category,
            'score': max(0.001, round(float(self.score), 3)),
            'bbox': [round(float(c), 2) for c in self.bbox],
        }
