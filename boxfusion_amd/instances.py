"""Instances3D field container + association entry points (reference: boxfusion/instances.py).

The container semantics follow the reference (Detectron2-style fields, `cat`, `__getitem__` with
int / slice / bool / long / numpy indices).  The association methods keep the reference's
signatures and return values but run on the GPU:

  spatial_association         -> bf_obb_iou_matrix + bf_nms_scan       (instances.py:22-101,372-397)
  correspondence_association  -> bf_corr_assoc                          (instances.py:411-490)
  project_3d_boxes            -> bf_project_boxes                       (instances.py:333-369)
"""
from __future__ import annotations

import itertools
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

from boxfusion_amd import _lib


class Exchange:
    """One int32 host<->device exchange buffer for an association kernel: named host arrays are
    uploaded with a single copy, named sizes are device outputs; `fetch()` reads everything back
    with a single copy (one synchronisation per association step)."""

    def __init__(self, dev, **fields):
        self.layout = {}
        off = 0
        for k, v in fields.items():
            n = int(np.asarray(v).size) if isinstance(v, np.ndarray) else int(v)
            shape = v.shape if isinstance(v, np.ndarray) else (n,)
            self.layout[k] = (off, n, shape)
            off += n
        host = np.zeros(max(off, 1), np.int32)
        for k, v in fields.items():
            if isinstance(v, np.ndarray):
                o, n, _ = self.layout[k]
                host[o:o + n] = v.reshape(-1)
        self.buf = _lib.h2d(host, dev)
        self.dev = {k: self.buf[o:o + n].view(*shape) for k, (o, n, shape) in self.layout.items()}

    def fetch(self):
        h = self.buf.cpu().numpy()
        return {k: h[o:o + n].reshape(shape) for k, (o, n, shape) in self.layout.items()}


class Instances3D:
    def __init__(self, image_size: Tuple[int, int] = (0, 0), **kwargs: Any):
        self._image_size = image_size
        self._fields: Dict[str, Any] = {}
        self._len = None
        for k, v in kwargs.items():
            self.set(k, v)

    @property
    def image_size(self):
        return self._image_size

    def __setattr__(self, name, val):
        if name.startswith("_"):
            super().__setattr__(name, val)
        else:
            self.set(name, val)

    def __getattr__(self, name):
        if name == "_fields" or name not in self._fields:
            raise AttributeError(f"Cannot find field '{name}' in the given Instances3D!")
        return self._fields[name]

    def set(self, name, value):
        n = value.shape[0] if isinstance(value, (torch.Tensor, np.ndarray)) else len(value)
        if self._fields and not (len(self._fields) == 1 and name in self._fields):
            assert self._len == n, f"Adding a field of length {n} to a Instances3D of length {self._len}"
        self._fields[name] = value
        self._len = n

    def has(self, name):
        return name in self._fields

    def remove(self, name):
        del self._fields[name]
        if not self._fields:
            self._len = None

    def get(self, name):
        return self._fields[name]

    def get_fields(self):
        return self._fields

    def to(self, *args, **kwargs):
        ret = Instances3D(self._image_size)
        for k, v in self._fields.items():
            ret.set(k, v.to(*args, **kwargs) if hasattr(v, "to") else v)
        return ret

    def _device_rows(self, others, idx=None):
        """cat([self] + others) (one other) or self[idx] (idx: int64 device tensor) for instance
        sets whose fields are all device tensors / boxes: one bf_rows_gather launch.  None when a
        field needs the generic path."""
        pairs, plan = [], []
        narrow_id = None
        for k, v in self._fields.items():
            w = others[0]._fields.get(k) if others else None
            if isinstance(v, torch.Tensor):
                if v.element_size() < 4 and (v.element_size() * int(np.prod(v.shape[1:], dtype=np.int64))) % 4:
                    return None
                if not v.is_cuda or (others and not (isinstance(w, torch.Tensor) and w.dtype == v.dtype
                                                     and w.shape[1:] == v.shape[1:] and w.is_cuda)):
                    return None
                plan.append((k, None))
                pairs.append((v.contiguous(), w.contiguous() if others else None))
            elif hasattr(v, "tensor") and hasattr(v, "R") and isinstance(v.tensor, torch.Tensor):
                if not v.tensor.is_cuda or (others and not hasattr(w, "R")):
                    return None
                plan.append((k, type(v)))
                pairs.append((v.tensor.contiguous(), w.tensor.contiguous() if others else None))
                pairs.append((v.R.contiguous(), w.R.contiguous() if others else None))
            else:
                return None
        if "init_id" in self._fields and isinstance(self._fields["init_id"], torch.Tensor) \
                and self._fields["init_id"].dtype == torch.int64 and self._fields["init_id"].dim() == 1:
            # the association kernels' int32 copy of init_id, produced by the same launch
            narrow_id = len(pairs)
            v = self._fields["init_id"]
            pairs.append((v.contiguous(), others[0]._fields["init_id"].contiguous() if others else None, True))
        if not pairs or len(pairs) > _lib.ROWS_MAX_FIELDS:
            return None
        if others and set(others[0]._fields) != set(self._fields):
            return None
        outs = _lib.rows_gather(pairs, idx)
        ret = Instances3D(self._image_size)
        o = 0
        for k, box_type in plan:
            if box_type is None:
                ret.set(k, outs[o])
                o += 1
            else:
                ret.set(k, box_type._views(outs[o], outs[o + 1]))
                o += 2
        if narrow_id is not None:
            ret._init_id32 = outs[narrow_id]
        return ret

    def __getitem__(self, item):
        if isinstance(item, np.ndarray) and item.dtype.kind in "iu" and item.ndim == 1 and self._fields:
            dev = next((v.device if isinstance(v, torch.Tensor) else getattr(getattr(v, "tensor", None), "device", None)
                        for v in self._fields.values()), None)
            if dev is not None and dev.type == "cuda":
                r = self._device_rows([], _lib.h2d(item.astype(np.int64), dev))
                if r is not None:
                    return r
        if type(item) == int:
            if item >= len(self) or item < -len(self):
                raise IndexError("Instances3D index out of range!")
            item = slice(item, None, len(self))
        ret = Instances3D(self._image_size)
        # a host index used on device fields is uploaded once, not once per field
        dev_index = {}

        def on(device):
            if device not in dev_index:
                dev_index[device] = (_lib.h2d(item, device) if isinstance(item, np.ndarray)
                                     else torch.as_tensor(item, device=device))
            return dev_index[device]
        for k, v in self._fields.items():
            if isinstance(v, (torch.Tensor, np.ndarray)) or hasattr(v, "tensor"):
                if isinstance(v, np.ndarray) and isinstance(item, torch.Tensor):
                    ret.set(k, v[item.cpu().numpy()])
                elif isinstance(v, torch.Tensor) and isinstance(item, np.ndarray):
                    ix = on(v.device)
                    ret.set(k, v.index_select(0, ix) if ix.dtype == torch.int64 and ix.dim() == 1 else v[ix])
                elif hasattr(v, "tensor") and isinstance(item, np.ndarray):
                    ret.set(k, v[on(v.tensor.device)])
                else:
                    ret.set(k, v[item])
            elif hasattr(v, "__iter__"):
                if isinstance(item, np.ndarray) and item.dtype == np.bool_:
                    ret.set(k, [x for i, x in enumerate(v) if item[i]])
                elif isinstance(item, torch.Tensor) and item.dtype == torch.bool:
                    m = item.cpu().tolist()
                    ret.set(k, [x for i, x in enumerate(v) if m[i]])
                elif isinstance(item, torch.Tensor) and item.dtype == torch.int64:
                    ret.set(k, [v[i] for i in item.cpu().tolist()])
                elif isinstance(item, np.ndarray):
                    ret.set(k, [v[int(i)] for i in item])
                elif isinstance(item, slice):
                    ret.set(k, v[item])
                else:
                    raise ValueError("Expected Bool or Long Tensor")
            else:
                raise ValueError("Not supported!")
        return ret

    def __len__(self):
        if self._len is None:
            raise NotImplementedError("Empty Instances3D does not support __len__!")
        return self._len

    def __iter__(self):
        raise NotImplementedError("`Instances3D` object is not iterable!")

    def clone(self):
        ret = Instances3D(self._image_size)
        for k, v in self._fields.items():
            if hasattr(v, "clone"):
                v = v.clone()
            elif isinstance(v, np.ndarray):
                v = np.copy(v)
            elif isinstance(v, (str, list, tuple)):
                v = list(v)
            ret.set(k, v)
        return ret

    @staticmethod
    def cat(instance_lists: List["Instances3D"]) -> "Instances3D":
        assert len(instance_lists) > 0
        if len(instance_lists) == 1:
            return instance_lists[0]
        if len(instance_lists) == 2:
            r = instance_lists[0]._device_rows([instance_lists[1]])
            if r is not None:
                return r
        ret = Instances3D(instance_lists[0]._image_size)
        for k in instance_lists[0]._fields.keys():
            vals = [i.get(k) for i in instance_lists]
            v0 = vals[0]
            if isinstance(v0, torch.Tensor):
                vals = torch.cat(vals, 0)
            elif isinstance(v0, np.ndarray):
                vals = np.concatenate(vals, 0)
            elif isinstance(v0, list):
                vals = list(itertools.chain(*vals))
            elif hasattr(type(v0), "cat"):
                vals = type(v0).cat(vals)
            else:
                raise ValueError(f"Unsupported type {type(v0)} for concatenation")
            ret.set(k, vals)
        return ret

    def __str__(self):
        return f"Instances3D(num_instances={len(self)}, fields=[{', '.join(self._fields)}])"

    __repr__ = __str__

    # ------------------------------------------------------------------------------------------
    # GPU geometry and association
    # ------------------------------------------------------------------------------------------
    def project_3d_boxes(self, K, H=480, W=640):
        boxes = self.get("pred_boxes_3d")
        corners = boxes.corners
        K = torch.as_tensor(np.asarray(K, dtype=np.float32) if not isinstance(K, torch.Tensor) else K)
        self.projected_boxes = _lib.project_boxes(corners, self.cam_pose.to(corners.device, torch.float32),
                                                  K.to(corners.device, torch.float32), float(W), float(H))

    def spatial_association(instance_lists, threshold, box_manager, cam_poses, corners=None):
        """nms_3d over all boxes; returns (keep, success_nms) as sorted lists.
        corners: the boxes' [N,8,3] corners when the caller already has them."""
        assert len(instance_lists) > 0
        if len(instance_lists) == 1:
            return instance_lists  # reference quirk (instances.py:381-382)
        boxes = instance_lists.get("pred_boxes_3d")
        dev = boxes.device
        if corners is None:
            corners = boxes.corners
        iou = _lib.obb_iou_matrix(corners)
        scores = instance_lists.scores.to(dev, torch.float32).contiguous()
        init_id = instance_lists.init_id.to(dev, torch.int32).contiguous()
        poses = cam_poses.to(dev, torch.float32).contiguous()
        vn = instance_lists.valid_num
        if not (isinstance(vn, torch.Tensor) and vn.is_cuda and vn.dtype == torch.float32 and vn.is_contiguous()):
            vn = torch.as_tensor(vn).to(dev, torch.float32).contiguous()
            instance_lists.valid_num = vn
        # one host->device copy in (fusion lists), one device->host copy out (lists + results)
        items, lens = box_manager.pack_host()
        n = scores.shape[0]
        x = Exchange(dev, items=items, lens=lens, counts=np.zeros(4, np.int32),
                     keep=n + 1, succ=n + 1, events=3 * (n + 1))
        _lib.nms_scan(iou, corners, scores, init_id, poses, x.dev["items"], x.dev["lens"], vn,
                      box_manager.nms_cfg(threshold),
                      out=(x.dev["keep"], x.dev["succ"], x.dev["events"].view(-1, 3), x.dev["counts"]))
        h = x.fetch()
        c = h["counts"]
        if c[3]:
            raise _lib.HipError(f"bf_nms_scan device status {c[3]} (fusion list capacity)")
        box_manager.unpack_host(h["items"], h["lens"])
        box_manager.replay_flags(h["events"].reshape(-1, 3)[:c[2]].tolist())
        keep = h["keep"][:c[0]].astype(np.int64).tolist()
        success = h["succ"][:c[1]].astype(np.int64).tolist()
        return keep, success

    def correspondence_association(cfg, box_manager, cur_keep_idx, cur_success_nms, pred_instances,
                                   global_pred_box, all_pred_box, all_poses, per_frame_ins_cam_pose,
                                   frame_id, mask, intrinsic, all_kf_pose, threshold=0.33, H=480,
                                   W=640, corners=None, cur_pose=None):
        """small-box 2-D association against the previous global boxes; returns
        (all_pred_box[keep_idx], all_poses[keep_idx], keep_idx).
        corners / cur_pose: all_pred_box's corners and this keyframe's pose as device tensors
        when the caller already has them (`intrinsic` may also be a device tensor)."""
        n_glo = len(global_pred_box)
        boxes = all_pred_box.get("pred_boxes_3d")
        dev = boxes.device
        if corners is None:
            corners = boxes.corners
        mask_np = np.asarray(mask, dtype=np.int64)
        success_all = [i + n_glo for i in cur_success_nms]
        vn = all_pred_box.valid_num
        items, lens = box_manager.pack_host()
        n_all = len(all_pred_box)
        x = Exchange(dev, items=items, lens=lens, mask=mask_np.astype(np.int32),
                     succ=np.asarray(success_all if success_all else [0], np.int32),
                     counts=np.zeros(3, np.int32), keep=max(1, len(mask_np)), events=3 * (n_all + 1))
        if cur_pose is None:
            cur_pose = _lib.h2d(np.asarray(all_kf_pose[frame_id], dtype=np.float32), dev)
        K = torch.as_tensor(intrinsic).to(dev, torch.float32)
        succ_dev = x.dev["succ"][:len(success_all)]
        _lib.corr_assoc(
            corners, boxes.dims.contiguous(), all_pred_box.scores.to(dev, torch.float32).contiguous(),
            all_pred_box.pred_boxes.to(dev, torch.float32).contiguous(),
            all_pred_box.init_id.to(dev, torch.int32).contiguous(),
            per_frame_ins_cam_pose.to(dev, torch.float32).contiguous(), cur_pose, K, n_glo,
            x.dev["mask"], succ_dev, x.dev["items"], x.dev["lens"], vn,
            box_manager.corr_cfg(threshold, W, H),
            out=(x.dev["keep"], x.dev["events"].view(-1, 3), x.dev["counts"]))
        h = x.fetch()
        c = h["counts"]
        if c[2]:
            raise _lib.HipError(f"bf_corr_assoc device status {c[2]} (fusion list capacity)")
        box_manager.unpack_host(h["items"], h["lens"])
        box_manager.replay_flags(h["events"].reshape(-1, 3)[:c[1]].tolist())
        keep_idx = h["keep"][:c[0]].astype(np.int64)
        return all_pred_box[keep_idx], all_poses[keep_idx], keep_idx

    def joint_association(all_pred_box, n_glo, threshold, small_threshold, box_manager,
                          per_frame_ins_cam_pose, cur_pose, intrinsic, corners, H=480, W=640):
        """spatial_association followed by correspondence_association (demo.py:243-262) with ONE
        host round trip: bf_nms_scan and bf_corr_assoc_chained run back to back on the stream,
        the second on the first's device outputs.  Returns (mask, success, keep_idx, cur_keep):
        mask / success as spatial_association's, keep_idx = correspondence_association's keep
        (equal to mask when no new box survived the NMS, the case where the reference skips the
        second step), cur_keep = whether a new box (index >= n_glo) is in mask, and the kept rows
        (keep_idx, or mask without cur_keep) as an int32 device tensor."""
        boxes = all_pred_box.get("pred_boxes_3d")
        dev = boxes.device
        iou = _lib.obb_iou_matrix(corners)
        scores = all_pred_box.scores.to(dev, torch.float32).contiguous()
        init_id = getattr(all_pred_box, "_init_id32", None)
        if init_id is None or init_id.shape[0] != len(all_pred_box):
            init_id = all_pred_box.init_id.to(dev, torch.int32).contiguous()
        poses = per_frame_ins_cam_pose.to(dev, torch.float32).contiguous()
        vn = all_pred_box.valid_num
        if not (isinstance(vn, torch.Tensor) and vn.is_cuda and vn.dtype == torch.float32 and vn.is_contiguous()):
            vn = torch.as_tensor(vn).to(dev, torch.float32).contiguous()
            all_pred_box.valid_num = vn
        items, lens = box_manager.pack_host()
        n = scores.shape[0]
        x = Exchange(dev, items=items, lens=lens, counts=np.zeros(4, np.int32), keep=n + 1,
                     succ=n + 1, events=3 * (n + 1), ccounts=np.zeros(3, np.int32), ckeep=n + 1,
                     cevents=3 * (n + 1))
        d = x.dev
        _lib.nms_scan(iou, corners, scores, init_id, poses, d["items"], d["lens"], vn,
                      box_manager.nms_cfg(threshold),
                      out=(d["keep"], d["succ"], d["events"].view(-1, 3), d["counts"]))
        _lib.corr_assoc_chained(
            corners, boxes.dims.contiguous(), scores,
            all_pred_box.pred_boxes.to(dev, torch.float32).contiguous(), init_id, poses, cur_pose,
            torch.as_tensor(intrinsic).to(dev, torch.float32), n_glo, d["keep"], d["counts"][0:1],
            d["succ"], d["counts"][1:2], d["items"], d["lens"], vn,
            box_manager.corr_cfg(small_threshold, W, H),
            out=(d["ckeep"], d["cevents"].view(-1, 3), d["ccounts"]))
        h = x.fetch()
        c, cc = h["counts"], h["ccounts"]
        if c[3]:
            raise _lib.HipError(f"bf_nms_scan device status {c[3]} (fusion list capacity)")
        if cc[2]:
            raise _lib.HipError(f"bf_corr_assoc device status {cc[2]} (fusion list capacity)")
        box_manager.unpack_host(h["items"], h["lens"])
        # the NMS events, then the correspondence events, exactly as the two calls replay them
        box_manager.replay_flags(h["events"].reshape(-1, 3)[:c[2]].tolist())
        box_manager.replay_flags(h["cevents"].reshape(-1, 3)[:cc[1]].tolist())
        mask = h["keep"][:c[0]].astype(np.int64)
        success = h["succ"][:c[1]].astype(np.int64).tolist()
        keep_idx = h["ckeep"][:cc[0]].astype(np.int64)
        any_cur = bool((mask >= n_glo).any())
        # the row set to keep, still on the device (int32): gather without another upload
        keep_dev = d["ckeep"][:cc[0]] if any_cur else d["keep"][:c[0]]
        return mask.tolist(), success, keep_idx, any_cur, keep_dev
