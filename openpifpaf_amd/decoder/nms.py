"""Keypoint NMS configuration (nms.py:11-57).

The suppression itself runs inside the device decode (csrc/grow.hip, after the seed loop
and force-complete), configured from these class attributes exactly as the reference's
CifCaf(nms=nms.Keypoints()) is.
"""


class Keypoints:
    suppression = 0.0
    instance_threshold = 0.0
    keypoint_threshold = 0.0
    occupancy_visualizer = None

    def annotations(self, anns):
        raise NotImplementedError(
            'nms.Keypoints runs inside the device decode (CifCaf); standalone NMS over '
            'host Annotation lists is not provided')
