"""Fusion bookkeeping (reference: boxfusion/box_manager.py).

Same public state as the reference — `fusion_list` (list of sorted init_id lists),
`fusion_flag`, `already_fusion`, `num_record` — kept as Python lists for API compatibility.
The record()/record_corr() logic itself runs inside the association kernels (bf_nms_scan,
bf_corr_assoc); `pack`/`unpack` move the lists to and from the kernels' fixed-capacity rows, and
`replay_flags` applies the kernels' event log to `fusion_flag` (box_manager.py:85-86,126-127).
"""
from __future__ import annotations

import copy
import itertools

import numpy as np
import torch

from boxfusion_amd import _lib

DEFAULT_LIST_CAPACITY = 64


class _TrackedList(list):
    """already_fusion: a list whose in-place changes bump `version`, so the membership mirror of
    BoxManager.check_if_fusion is rebuilt after any outside edit (append, item assignment, pop,
    slice writes, ...), not only after length changes.  Rows themselves are treated as values
    (the reference deep-copies them on insertion, box_manager.py:31)."""
    __slots__ = ("version",)

    def __init__(self, *a):
        super().__init__(*a)
        self.version = 0


def _bumping(name):
    base = getattr(list, name)

    def f(self, *a, **k):
        self.version += 1
        return base(self, *a, **k)
    f.__name__ = name
    return f


for _m in ("append", "extend", "insert", "pop", "remove", "clear", "sort", "reverse", "__setitem__",
           "__delitem__", "__iadd__", "__imul__"):
    setattr(_TrackedList, _m, _bumping(_m))


class BoxManager:
    def __init__(self, cfg):
        self.fusion_list = []
        self.last_fusion_frame = []
        self._fusion_flag = []
        self._already_fusion = _TrackedList()
        self._already_set, self._already_ver = set(), 0   # tuple mirror of already_fusion (membership)
        self._pending = None      # resolves a deferred BoxFusion result (box_fusion.py)
        self.num_record = {}
        self.cfg = cfg
        self.rotation_gap = cfg["association"]["rotation_gap"]
        self.translation_gap = cfg["association"]["translation_gap"]
        self.small_size = cfg["box_fusion"]["small_size"]
        self.list_capacity = int(cfg.get("box_fusion", {}).get("list_capacity", DEFAULT_LIST_CAPACITY))
        self.merge_log = []

    # fusion_flag / already_fusion are plain lists in the reference; here every read first applies
    # a deferred BoxFusion.boxfusion result, so callers always see the reference's state
    @property
    def fusion_flag(self):
        self.flush()
        return self._fusion_flag

    @fusion_flag.setter
    def fusion_flag(self, v):
        self._fusion_flag = v

    @property
    def already_fusion(self):
        self.flush()
        return self._already_fusion

    @already_fusion.setter
    def already_fusion(self, v):
        self._already_fusion = _TrackedList(v)
        self._already_ver = -1               # rebuild the membership mirror on the next check

    def flush(self):
        if self._pending is not None:
            f, self._pending = self._pending, None
            f()

    # -- reference API ---------------------------------------------------------------------------
    def init_new_predictions(self, box_num, all_num):
        for i in range(box_num):
            self.fusion_list.append([i + all_num])
            self.last_fusion_frame.append([0])
            self._fusion_flag.append(0)     # order-independent of a pending fusion result

    def add_fusion_ind(self, idx_list):
        row = copy.deepcopy(idx_list)
        af = self._already_fusion
        in_sync = self._already_ver == af.version
        af.append(row)
        if in_sync:                          # keep the mirror incrementally
            self._already_set.add(tuple(row))
            self._already_ver = af.version

    def check_if_fusion(self, idx_list):
        """`idx_list in already_fusion` (list equality) as a set lookup on a tuple mirror: the list
        grows with every fused box and is searched for every candidate of every keyframe"""
        af = self.already_fusion
        if self._already_ver != af.version:  # changed from outside: rebuild
            self._already_set = {tuple(r) for r in af}
            self._already_ver = af.version
        return tuple(idx_list) in self._already_set

    def update(self, keep_idx):
        self.fusion_list = [self.fusion_list[i] for i in keep_idx]

    def update_fusion_flag(self, idx):
        self._fusion_flag[idx] = 1

    def get_fusion_idx(self):
        return [i for i in range(len(self.fusion_flag)) if self.fusion_flag[i] == 1]

    def get_nofusion_idx(self):
        return [i for i in range(len(self.fusion_flag)) if self.fusion_flag[i] == 0]

    def check_valid_num(self, all_pred_box, count, gap):
        """box_manager.py:151-166 (off in every shipped config)."""
        fid = all_pred_box.frame_id
        vn = all_pred_box.valid_num
        zero = torch.where((vn == 0) & (fid < (count - gap)))[0]
        valid = torch.arange(len(all_pred_box))
        for idx in zero.tolist():
            valid = valid[valid != idx]
        self.fusion_list = [self.fusion_list[int(i)] for i in valid]
        return all_pred_box[valid]

    @staticmethod
    def check_uv_bounds(uv_coords, W, H, ratio=1.0):
        """box_manager.py:217-225 (gap = int((1 - ratio) * size): 63 / 47 at 640 / 480, 0.9)."""
        gap_w = int((1 - ratio) * W)
        gap_h = int((1 - ratio) * H)
        u, v = uv_coords[:, 0], uv_coords[:, 1]
        return (u > gap_w) & (u < (W - gap_w)) & (v > gap_h) & (v < (H - gap_h))

    @staticmethod
    def check_floor_mask(box_3d, ratio=20):
        size = box_3d[:, 3:]
        mx = torch.amax(size, dim=1)
        mn = torch.amin(size, dim=1)
        second = torch.sort(size, dim=1, descending=True)[0][:, 1]
        mask = mx / mn > ratio
        second_mask = ((mx / mn > ratio / 2) & (mx / second > ratio / 2) & (second / mn < 2.0) &
                       (second < 0.15) & (mn < 0.15))
        return mask | second_mask

    @staticmethod
    def check_large_mask(box_3d, thres=0.5):
        return torch.amax(box_3d[:, 3:], dim=1) > thres

    # -- device exchange ---------------------------------------------------------------------------
    def pack(self, device):
        n = len(self.fusion_list)
        cap = self.list_capacity
        items = np.full((max(n, 1), cap), -1, np.int32)
        lens = np.zeros(max(n, 1), np.int32)
        for i, row in enumerate(self.fusion_list):
            if len(row) > cap:
                raise _lib.HipError(f"fusion list of {len(row)} > capacity {cap}; raise "
                                    "box_fusion.list_capacity")
            items[i, :len(row)] = row
            lens[i] = len(row)
        return _lib.h2d(items, device), _lib.h2d(lens, device)

    def pack_host(self):
        """fusion lists as host arrays (items [n, cap] padded with -1, lengths [n])"""
        fl = self.fusion_list
        n = len(fl)
        cap = self.list_capacity
        items = np.full((max(n, 1), cap), -1, np.int32)
        lens = np.zeros(max(n, 1), np.int32)
        if n:
            ln = np.fromiter(map(len, fl), np.int64, n)
            if int(ln.max()) > cap:
                raise _lib.HipError(f"fusion list of {int(ln.max())} > capacity {cap}; raise "
                                    "box_fusion.list_capacity")
            lens[:n] = ln
            rows = np.repeat(np.arange(n), ln)
            cols = np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln)
            items[rows, cols] = np.fromiter(itertools.chain.from_iterable(fl), np.int64, int(ln.sum()))
        return items, lens

    def unpack_host(self, items, lens):
        self.fusion_list = [items[i, :lens[i]].tolist() for i in range(len(self.fusion_list))]

    def unpack(self, items, lens):
        it = items.cpu().numpy()
        ln = lens.cpu().numpy()
        self.fusion_list = [[int(v) for v in it[i, :ln[i]]] for i in range(len(self.fusion_list))]

    def replay_flags(self, events):
        """fusion_flag propagation of record/record_corr's branch 2 (the flag is never pruned by
        update(), so indices refer to a stale layout exactly as in the reference)."""
        for cur, idx, branch in events:
            if branch == 2 and idx < len(self.fusion_flag) and self.fusion_flag[idx] == 1:
                self.fusion_flag[cur] = 1

    def nms_cfg(self, iou_threshold):
        c = _lib.NmsCfg()
        c.iou_threshold = float(iou_threshold)
        c.translation_gap = float(self.translation_gap)
        c.rotation_gap = float(self.rotation_gap)
        c.center_gap = 0.5
        c.max_list = 5
        c.list_capacity = self.list_capacity
        return c

    def corr_cfg(self, threshold, W, H):
        c = _lib.CorrCfg()
        c.small_size = float(self.small_size)
        c.threshold = float(threshold)
        c.translation_gap = float(self.translation_gap)
        c.rotation_gap = float(self.rotation_gap)
        c.W, c.H = float(W), float(H)
        c.max_list = 5
        c.list_capacity = self.list_capacity
        return c
