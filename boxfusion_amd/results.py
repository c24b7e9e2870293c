"""Result writers of the run (demo.py:368-387, tools/utils.py:302-331), kept off the timed path.

  post_process(corners, threshold)       tools/utils.py:302-317 (ScanNet: drop boxes thinner than
                                         `threshold` along any world axis)
  save_box(data, filename)               tools/utils.py:322-331 (pickle, highest protocol)
  global_save_list(all_pred_box, ...)    demo.py:368-379: [[(0, corners[n], 1.0) ...]]
  framewise_save_list(per_frame_ins, ..) demo.py:382-387: [[(class_idx, corners, feature) ...]]
  export(...)                            both files, under the same conditions as demo.py

Corners come from the device (`GeneralInstance3DBoxes.corners`, bf_box_corners); the rest is host
bookkeeping on at most a few thousand boxes.
"""
from __future__ import annotations

import os
import pickle

import numpy as np


def post_process(boxes, threshold=0.3):
    """corners [N,8,3] -> the boxes whose extent along x, y and z is each >= threshold"""
    boxes = np.asarray(boxes)
    ranges = boxes.max(axis=1) - boxes.min(axis=1)
    return boxes[(ranges >= threshold).all(axis=1)]


def save_box(data, filename):
    with open(filename, "wb") as f:
        pickle.dump(data, f, protocol=pickle.HIGHEST_PROTOCOL)
    print(f"Results successfully saved to {filename}")


def _corners(inst):
    return inst.pred_boxes_3d.corners.detach().cpu().numpy()


def _class_index(class_list, categories):
    class_list = list(class_list)
    return np.array([class_list.index(c) for c in categories])


def global_save_list(all_pred_box, class_list, dataset):
    """demo.py:371-379.  The class index is computed (so an unknown category raises like the
    reference's list.index) but, as in the reference, every record is written with class 0 and
    score 1.0.  Returns None when no box survives (nothing is written then)."""
    if getattr(all_pred_box, "categories", None) is not None:
        _class_index(class_list, all_pred_box.categories)
    boxes = _corners(all_pred_box)
    if dataset == "scannet":
        boxes = post_process(boxes)
    if boxes.shape[0] == 0:
        return None
    # demo.py:378 iterates over len(all_pred_box), not over the post-processed count: a box
    # dropped by post_process makes it raise IndexError, as the reference does
    return [[(int(0), boxes[n], 1.0) for n in range(len(all_pred_box))]]


def framewise_save_list(per_frame_ins, class_list):
    """demo.py:383-386: every per-frame detection with its class index and CLIP feature"""
    idx = _class_index(class_list, per_frame_ins.categories)
    boxes = _corners(per_frame_ins)
    feats = per_frame_ins.features
    return [[(idx[n], boxes[n], feats[n]) for n in range(len(per_frame_ins))]]


def export(all_pred_box, per_frame_ins, class_list, cfg, video_id):
    """demo.py:368-387: `<output_dir>/<video_id>_boxes.pkl` when cfg['eval'], and
    `<output_dir>/framewise_boxes.pkl`, when cfg['data']['output_dir'] is set."""
    out_dir = cfg["data"].get("output_dir")
    written = []
    if out_dir is None:
        return written
    if cfg.get("eval"):
        lst = global_save_list(all_pred_box, class_list, cfg["dataset"])
        if lst is not None:
            fn = os.path.join(out_dir, video_id + "_boxes.pkl")
            save_box(lst, fn)
            written.append(fn)
    fn = os.path.join(out_dir, "framewise_boxes.pkl")
    save_box(framewise_save_list(per_frame_ins, class_list), fn)
    written.append(fn)
    return written
