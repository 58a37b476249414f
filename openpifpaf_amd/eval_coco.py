"""COCO prediction records (eval_coco.py:108-158, EvalCoco.from_predictions).

`coco_predictions(predictions, meta)` maps decoded annotations to image coordinates on
the device (transforms.Preprocess.annotations_inverse), applies EvalCoco's small-object
filter and per-image cap, and returns the json records pycocotools reads.  The COCO
evaluation itself (pycocotools) is not part of this package.
"""
import numpy as np

from . import transforms

KEYS = ('category_id', 'score', 'keypoints', 'bbox', 'image_id')


def coco_predictions(predictions, meta, *, small_threshold=0.0, max_per_image=20,
                     n_keypoints=17):
    image_id = int(meta['image_id'])
    predictions = transforms.Preprocess.annotations_inverse(predictions, meta)
    if small_threshold:
        predictions = [pred for pred in predictions
                       if pred.scale(v_th=0.01) >= small_threshold]
    if len(predictions) > max_per_image:
        predictions = predictions[:max_per_image]
    image_annotations = []
    for pred in predictions:
        pred_data = pred.json_data()
        pred_data['image_id'] = image_id
        image_annotations.append({k: v for k, v in pred_data.items() if k in KEYS})
    if not image_annotations:  # at least one record per image (for pycocotools)
        image_annotations.append({
            'image_id': image_id,
            'category_id': 1,
            'keypoints': np.zeros((n_keypoints * 3,)).tolist(),
            'bbox': [0, 0, 1, 1],
            'score': 0.001,
        })
    return image_annotations
