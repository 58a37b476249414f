"""COCO person keypoint configuration the decoder is parameterised with.

Values follow openpifpaf/datasets/constants.py (reference v0.11.6):
  keypoint names      constants.py:23-41
  COCO skeleton       constants.py:4-8   (1-based joint indices, 19 edges)
  dense skeleton      constants.py:106-126 (44 edges; the 25 "connections" are the
                      DENSER edges that are not in the COCO skeleton)
  upright pose        constants.py:44-62 (only used by the synthetic "planted" generator)
"""
import numpy as np

COCO_KEYPOINTS = [
    'nose', 'left_eye', 'right_eye', 'left_ear', 'right_ear',
    'left_shoulder', 'right_shoulder', 'left_elbow', 'right_elbow',
    'left_wrist', 'right_wrist', 'left_hip', 'right_hip',
    'left_knee', 'right_knee', 'left_ankle', 'right_ankle',
]

COCO_PERSON_SKELETON = [
    (16, 14), (14, 12), (17, 15), (15, 13), (12, 13), (6, 12), (7, 13),
    (6, 7), (6, 8), (7, 9), (8, 10), (9, 11), (2, 3), (1, 2), (1, 3),
    (2, 4), (3, 5), (4, 6), (5, 7),
]

DENSER_COCO_PERSON_SKELETON = [
    (1, 2), (1, 3), (2, 3), (1, 4), (1, 5), (4, 5),
    (1, 6), (1, 7), (2, 6), (3, 7),
    (2, 4), (3, 5), (4, 6), (5, 7), (6, 7),
    (6, 12), (7, 13), (6, 13), (7, 12), (12, 13),
    (6, 8), (7, 9), (8, 10), (9, 11), (6, 10), (7, 11),
    (8, 9), (10, 11),
    (10, 12), (11, 13),
    (10, 14), (11, 15),
    (14, 12), (15, 13), (12, 15), (13, 14),
    (12, 16), (13, 17),
    (16, 14), (17, 15), (14, 17), (15, 16),
    (14, 15), (16, 17),
]

DENSER_COCO_PERSON_CONNECTIONS = [
    c for c in DENSER_COCO_PERSON_SKELETON if c not in COCO_PERSON_SKELETON]

# decode skeleton for --dense-connections (factory.py:182-188): COCO 19 + 25 dense = 44
DENSE_DECODE_SKELETON = COCO_PERSON_SKELETON + DENSER_COCO_PERSON_CONNECTIONS

# (x, y) of an upright person in units of "person scale"; column 2 (visibility) dropped.
COCO_UPRIGHT_POSE = np.array([
    [0.0, 9.3], [-0.35, 9.7], [0.35, 9.7], [-0.7, 9.5], [0.7, 9.5],
    [-1.4, 8.0], [1.4, 8.0], [-1.75, 6.0], [1.75, 6.2], [-1.75, 4.0],
    [1.75, 4.2], [-1.26, 4.0], [1.26, 4.0], [-1.4, 2.0], [1.4, 2.1],
    [-1.4, 0.0], [1.4, 0.1],
], dtype=np.float64)


# datasets/constants.py: left / right keypoint pairs swapped by a horizontal flip
HFLIP = {
    'left_eye': 'right_eye', 'right_eye': 'left_eye',
    'left_ear': 'right_ear', 'right_ear': 'left_ear',
    'left_shoulder': 'right_shoulder', 'right_shoulder': 'left_shoulder',
    'left_elbow': 'right_elbow', 'right_elbow': 'left_elbow',
    'left_wrist': 'right_wrist', 'right_wrist': 'left_wrist',
    'left_hip': 'right_hip', 'right_hip': 'left_hip',
    'left_knee': 'right_knee', 'right_knee': 'left_knee',
    'left_ankle': 'right_ankle', 'right_ankle': 'left_ankle',
}
