"""Synthetic CIF/CAF field generators.

There is no checkpoint or dataset offline, so every benchmark and parity case runs on
synthetic fields with the reference's field layout (network/heads.py:65-88):
  CIF  (17, 5, H, W)  channels [c, x, y, b, s], x/y absolute field-cell coordinates
  CAF  (C, 9, H, W)   channels [c, x1, y1, b1, s1, x2, y2, b2, s2] (after heads.py:86 reorder)

* uniform(...)  - the literal "synthetic random" stress input (≈44% of CIF cells over 0.1,
                  ≈400 annotations per 80x80 image under eval defaults).
* planted(...)  - realistic input: a low-confidence background plus n people whose joints
                  get 4x4 CIF patches (encoder/cif.py:118-145 places 4x4 patches) and whose
                  limbs get one 4x4 CAF patch at the limb midpoint pointing joint1 -> joint2.
* det_planted / det_uniform(...) - CifDet fields (n_categories, 7, H, W), channels
                  [c, x, y, b, w, h, b2] (CifdetCollector, heads.py:127-144): boxes whose
                  centre cells carry the box centre and size, or random fields.

Both are deterministic functions of their arguments (numpy PCG64 streams).  The golden
fixtures record a SHA-256 of the generated inputs so a change here is caught by the tests.
"""
import hashlib

import numpy as np

from .constants import COCO_PERSON_SKELETON, COCO_UPRIGHT_POSE


def _grid(h, w):
    # (2, H, W): [0] = x (column), [1] = y (row)
    return np.indices((h, w), dtype=np.float32)[::-1]


def uniform(h, w, n_caf=19, seed=0):
    rng = np.random.default_rng(seed)
    g = _grid(h, w)
    cif = rng.random((17, 5, h, w), dtype=np.float32)
    cif[:, 0] **= 4
    cif[:, 1:3] += g - 0.5
    cif[:, 4] = 0.5 + 3 * cif[:, 4]
    caf = rng.random((n_caf, 9, h, w), dtype=np.float32)
    caf[:, 0] **= 4
    caf[:, 1:3] += g - 0.5
    caf[:, 5:7] = g + 4 * (caf[:, 5:7] - 0.5)
    caf[:, 4] = 0.5 + 3 * caf[:, 4]
    caf[:, 8] = 0.5 + 3 * caf[:, 8]
    return cif, caf


def _patch_cells(px, py, h, w):
    """Cells of the 4x4 patch around point (px, py) (field-cell units) inside the grid."""
    x0 = int(np.floor(px)) - 1
    y0 = int(np.floor(py)) - 1
    xs = np.arange(max(0, x0), min(w, x0 + 4))
    ys = np.arange(max(0, y0), min(h, y0 + 4))
    return xs, ys


def _plant_person(cif, caf, kps, scale, skeleton, rng):
    """4x4 CIF patches at the joints kps (17, 2) and one 4x4 CAF patch per limb midpoint
    (field-cell units), confidences 0.7-1.0."""
    h, w = cif.shape[2:]
    for j in range(17):
        xs, ys = _patch_cells(kps[j, 0], kps[j, 1], h, w)
        conf = rng.uniform(0.7, 1.0, (len(ys), len(xs))).astype(np.float32)
        if conf.size == 0:
            continue
        sub = cif[j, :, ys[0]:ys[-1] + 1, xs[0]:xs[-1] + 1]
        m = conf > sub[0]
        sub[0][m] = conf[m]
        sub[1][m] = kps[j, 0]
        sub[2][m] = kps[j, 1]
        sub[3][m] = 0.5
        sub[4][m] = scale

    for e, (j1, j2) in enumerate(skeleton):
        a = kps[j1 - 1]
        b = kps[j2 - 1]
        mid = 0.5 * (a + b)
        xs, ys = _patch_cells(mid[0], mid[1], h, w)
        conf = rng.uniform(0.7, 1.0, (len(ys), len(xs))).astype(np.float32)
        if conf.size == 0:
            continue
        sub = caf[e, :, ys[0]:ys[-1] + 1, xs[0]:xs[-1] + 1]
        m = conf > sub[0]
        sub[0][m] = conf[m]
        sub[1][m] = a[0]
        sub[2][m] = a[1]
        sub[3][m] = 0.5
        sub[4][m] = scale
        sub[5][m] = b[0]
        sub[6][m] = b[1]
        sub[7][m] = 0.5
        sub[8][m] = scale


def _background(h, w, n_caf, rng, noise):
    g = _grid(h, w)
    cif = np.zeros((17, 5, h, w), dtype=np.float32)
    cif[:, 0] = rng.uniform(0.0, noise, (17, h, w))
    cif[:, 1:3] = g + rng.uniform(-0.5, 0.5, (17, 2, h, w))
    cif[:, 3] = 0.5
    cif[:, 4] = 1.0
    caf = np.zeros((n_caf, 9, h, w), dtype=np.float32)
    caf[:, 0] = rng.uniform(0.0, noise, (n_caf, h, w))
    caf[:, 1:3] = g
    caf[:, 5:7] = g + 4.0 * rng.uniform(-0.5, 0.5, (n_caf, 2, h, w))
    caf[:, 3] = 0.5
    caf[:, 4] = 1.0
    caf[:, 7] = 0.5
    caf[:, 8] = 1.0
    return cif, caf


def planted_multi(h_px, w_px, strides, n_people=4, seed=0, skeleton=None, noise=0.08):
    """The same people seen at several strides (multi-scale heads): a list of (cif, caf),
    one per stride, with fields of (h_px - 1) // stride + 1 rows."""
    if skeleton is None:
        skeleton = COCO_PERSON_SKELETON
    rng = np.random.default_rng(seed)
    people = []
    for _ in range(n_people):
        u = rng.uniform(8.0, 28.0)  # pixels per pose unit
        cx = rng.uniform(0.15 * w_px, 0.85 * w_px)
        cy = rng.uniform(0.15 * h_px, 0.85 * h_px)
        kps = np.stack([cx + u * COCO_UPRIGHT_POSE[:, 0],
                        cy - u * (COCO_UPRIGHT_POSE[:, 1] - 5.0)], axis=1)
        # joint scale in pixels: ~0.4 u as planted() (0.4 pose units), spread over people so
        # that the heads' min-scale masks keep some joints and drop others
        people.append((kps + rng.normal(0.0, 2.0, (17, 2)), u * rng.uniform(0.3, 1.2)))
    out = []
    for si, stride in enumerate(strides):
        h, w = (h_px - 1) // stride + 1, (w_px - 1) // stride + 1
        srng = np.random.default_rng(seed * 1000 + si)
        cif, caf = _background(h, w, len(skeleton), srng, noise)
        for kps, scale_px in people:
            _plant_person(cif, caf, kps / stride, scale_px / stride, skeleton, srng)
        out.append((cif, caf))
    return out


# multi-scale FieldConfigs (factory.py:153-180): strides per head, cif min scales,
# caf min / max distances.  'ms10' has 10 heads: CifHr pairs i with i + 5 (cif_hr.py:63).
MULTI_CASES = {
    'ms2': ([8, 16], [0.0, 12.0], [0.0, 36.0], [160.0, None]),
    'ms10': ([8, 16, 8, 16, 8] * 2, [0.0, 12.0, 16.0, 24.0, 40.0] * 2,
             [0.0, 36.0, 48.0, 72.0, 120.0] * 2, [160.0, 240.0, 320.0, 480.0, None] * 2),
}


def multi_case(name, seed=0, h_px=321, w_px=321, n_people=4):
    """fields list [cif_0, caf_0, cif_1, caf_1, ...] and the FieldConfig kwargs of a case."""
    strides, mins, dmin, dmax = MULTI_CASES[name]
    fields = []
    for cif, caf in planted_multi(h_px, w_px, strides, n_people=n_people, seed=seed):
        fields += [cif, caf]
    n = len(strides)
    kw = dict(cif_indices=[2 * i for i in range(n)], caf_indices=[2 * i + 1 for i in range(n)],
              cif_strides=list(strides), caf_strides=list(strides), cif_min_scales=list(mins),
              caf_min_distances=list(dmin), caf_max_distances=list(dmax))
    return fields, kw


def planted(h, w, n_people=8, seed=0, skeleton=None, noise=0.08):
    if skeleton is None:
        skeleton = COCO_PERSON_SKELETON
    n_caf = len(skeleton)
    rng = np.random.default_rng(seed)
    g = _grid(h, w)

    cif = np.zeros((17, 5, h, w), dtype=np.float32)
    cif[:, 0] = rng.uniform(0.0, noise, (17, h, w))
    cif[:, 1:3] = g + rng.uniform(-0.5, 0.5, (17, 2, h, w))
    cif[:, 3] = 0.5
    cif[:, 4] = 1.0

    caf = np.zeros((n_caf, 9, h, w), dtype=np.float32)
    caf[:, 0] = rng.uniform(0.0, noise, (n_caf, h, w))
    caf[:, 1:3] = g
    caf[:, 5:7] = g + 4.0 * rng.uniform(-0.5, 0.5, (n_caf, 2, h, w))
    caf[:, 3] = 0.5
    caf[:, 4] = 1.0
    caf[:, 7] = 0.5
    caf[:, 8] = 1.0

    for _ in range(n_people):
        u = rng.uniform(1.0, 3.5)
        cx = rng.uniform(6.0, w - 6.0)
        cy = rng.uniform(6.0, h - 6.0)
        kps = np.stack([
            cx + u * COCO_UPRIGHT_POSE[:, 0],
            cy - u * (COCO_UPRIGHT_POSE[:, 1] - 5.0),
        ], axis=1) + rng.normal(0.0, 0.3, (17, 2))
        _plant_person(cif, caf, kps, 0.4 * u, skeleton, rng)

    return cif, caf


def det_uniform(h, w, n_categories=3, seed=0):
    rng = np.random.default_rng(seed)
    det = rng.random((n_categories, 7, h, w), dtype=np.float32)
    det[:, 0] **= 4
    det[:, 1:3] += _grid(h, w) - 0.5
    det[:, 4:6] = 0.5 + 8.0 * det[:, 4:6]
    return det


def det_planted(h, w, n_categories=3, n_objects=10, seed=0, noise=0.08):
    """Objects of random category, centre and size (field cells); the 4x4 patch of cells
    around each centre predicts it."""
    rng = np.random.default_rng(seed)
    g = _grid(h, w)
    det = np.zeros((n_categories, 7, h, w), dtype=np.float32)
    det[:, 0] = rng.uniform(0.0, noise, (n_categories, h, w))
    det[:, 1:3] = g + rng.uniform(-0.5, 0.5, (n_categories, 2, h, w))
    det[:, 3] = 0.5
    det[:, 4:6] = rng.uniform(0.5, 3.0, (n_categories, 2, h, w))
    det[:, 6] = 0.5
    for _ in range(n_objects):
        f = int(rng.integers(n_categories))
        cx, cy = rng.uniform(2.0, w - 2.0), rng.uniform(2.0, h - 2.0)
        bw, bh = rng.uniform(2.0, w / 2.0), rng.uniform(2.0, h / 2.0)
        xs, ys = _patch_cells(cx, cy, h, w)
        conf = rng.uniform(0.7, 1.0, (len(ys), len(xs))).astype(np.float32)
        sub = det[f, :, ys[0]:ys[-1] + 1, xs[0]:xs[-1] + 1]
        m = conf > sub[0]
        sub[0][m] = conf[m]
        sub[1][m] = cx + rng.normal(0.0, 0.1, m.sum())
        sub[2][m] = cy + rng.normal(0.0, 0.1, m.sum())
        sub[4][m] = bw
        sub[5][m] = bh
    return det


def det_batch(kind, n, h, w, first_seed=0, **kwargs):
    """(n, n_categories, 7, H, W) CifDet fields, image i from seed first_seed + i."""
    fn = {'planted': det_planted, 'uniform': det_uniform}[kind]
    return np.stack([fn(h, w, seed=first_seed + i, **kwargs) for i in range(n)])


def generate(kind, h, w, seed, n_caf=19, skeleton=None, n_people=8):
    if kind == 'uniform':
        return uniform(h, w, n_caf=n_caf, seed=seed)
    if kind == 'planted':
        return planted(h, w, n_people=n_people, seed=seed, skeleton=skeleton)
    raise ValueError('unknown generator: {}'.format(kind))


def batch(kind, n, h, w, first_seed=0, **kwargs):
    """(n, 17, 5, H, W), (n, C, 9, H, W) with image i generated from seed first_seed + i."""
    cifs, cafs = zip(*(generate(kind, h, w, first_seed + i, **kwargs) for i in range(n)))
    return np.stack(cifs), np.stack(cafs)


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
