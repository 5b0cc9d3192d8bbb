"""Part-segmentation IoU (utils/metric.py): object_names, seg_classes and the
per-shape mean part IoU used by run_testing_seg (host numpy, evaluation only)."""
import numpy as np

object_names = ['Airplane', 'Bag', 'Cap', 'Car', 'Chair', 'Earphone', 'Guitar', 'Knife', 'Lamp',
                'Laptop', 'Motorbike', 'Mug', 'Pistol', 'Rocket', 'Skateboard', 'Table']
# utils/metric.py:5: the part labels of each object category
seg_classes = {'Airplane': [0, 1, 2, 3], 'Bag': [4, 5], 'Cap': [6, 7], 'Car': [8, 9, 10, 11],
               'Chair': [12, 13, 14, 15], 'Earphone': [16, 17, 18], 'Guitar': [19, 20, 21],
               'Knife': [22, 23], 'Lamp': [24, 25, 26, 27], 'Laptop': [28, 29],
               'Motorbike': [30, 31, 32, 33, 34, 35], 'Mug': [36, 37], 'Pistol': [38, 39, 40],
               'Rocket': [41, 42, 43], 'Skateboard': [44, 45, 46], 'Table': [47, 48, 49]}


def get_iou(gt, pred, cls_gt):
    """utils/metric.py:19-30: mean over the category's parts of |gt & pred| /
    |gt | pred|, a part absent from both counting 1."""
    parts = seg_classes[object_names[cls_gt]]
    ious = []
    for lab in parts:
        g, p = gt == lab, pred == lab
        if not p.any() and not g.any():
            ious.append(1.0)
        else:
            ious.append(np.sum(g & p) / float(np.sum(g | p)))
    return float(np.mean(ious))


def batch_get_iou(batch_pred, batch_seg, batch_cls):
    """utils/metric.py:32-38."""
    return [get_iou(batch_seg[i], batch_pred[i], int(np.argmax(batch_cls[i, :])))
            for i in range(batch_pred.shape[0])]
