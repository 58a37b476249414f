"""Duck-typed head networks / metas for factory_decode tests (network/heads.py metas:
IntensityMeta .keypoints, AssociationMeta .skeleton, DetectionMeta .categories; a head
network has .meta and .stride(basenet_stride))."""
import types

from openpifpaf_amd import constants


def meta(name, **kw):
    return types.SimpleNamespace(name=name, **kw)


class Head:
    def __init__(self, m, stride=8):
        self.meta = m
        self._stride = stride

    def stride(self, basenet_stride):
        del basenet_stride
        return self._stride


def cif_head(stride=8):
    return Head(meta('cif', keypoints=constants.COCO_KEYPOINTS), stride)


def caf_head(stride=8, skeleton=None):
    return Head(meta('caf', keypoints=constants.COCO_KEYPOINTS,
                     skeleton=list(skeleton or constants.COCO_PERSON_SKELETON)), stride)


def caf25_head(stride=8):
    return Head(meta('caf25', keypoints=constants.COCO_KEYPOINTS,
                     skeleton=list(constants.DENSER_COCO_PERSON_CONNECTIONS)), stride)


def multi_heads(strides, dense=False):
    """Per scale: cif, caf(, caf25) as the reference's multi-scale models lay them out."""
    heads = []
    for s in strides:
        heads += [cif_head(s), caf_head(s)]
        if not dense:
            heads.append(caf25_head(s))
    return heads


def det_head(categories):
    return Head(meta('cifdet', categories=list(categories)))
