"""The keyframe state machine of demo.py:200-305 on the GPU kernels.

`FusionStage.keyframe(count, pose, pred)` performs exactly the reference's per-keyframe sequence
with the reference's containers (Instances3D, BoxManager, BoxFusion):

  cam_pose / frame_id / init_id / valid_num fields            demo.py:215-219
  transform2world -> bf_box_transform2world                    demo.py:220, boxes.py:825-833
  project_3d_boxes -> bf_project_boxes                         demo.py:221, instances.py:333-369
  first keyframe: initialise                                   demo.py:226-241
  else: cat, spatial_association (bf_obb_iou_matrix + bf_nms_scan), then
        new boxes kept: correspondence_association (bf_corr_assoc), update, check_valid_num,
                        boxfusion (bf_fusion_fit, one launch for every box)   demo.py:243-299
        none kept:      all_pred_box[mask]                                     demo.py:300-304

`finish(count, pose)` reproduces the last-frame re-entry of demo.py:200 (`count == len-1` on a
non-keyframe): the previous keyframe's already world-space `pred_instances` are transformed by the
last pose a second time and go through association again (`stale_last_frame`
flag, default on as in the reference).
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time
import warnings

import numpy as np
import torch

from boxfusion_amd import _lib
from boxfusion_amd.box_fusion import BoxFusion, _warn_hull_once
from boxfusion_amd.box_manager import BoxManager
from boxfusion_amd.instances import Instances3D

# last_pred marker of a keyframe without detections: demo.py:206-212 still runs on the last-frame
# re-entry with an empty pred_instances and records num_record[count] (None = no keyframe yet)
EMPTY_KEYFRAME = "empty keyframe"
_PROFILE = bool(os.environ.get("BF_FSEQ_PROFILE"))   # diagnostic: per-call phase times on stderr


class FusionStage:
    """`native` (default: env BF_NATIVE_FUSION, on): the keyframe sequence after the per-box
    geometry runs in the library's sequencer (bf_fseq, one call per batch of keyframes), with
    all_pred_box's rows and BoxManager's lists owned there; `box_manager`, `all_pred_box`,
    `all_poses`, `fuser` and `stats` are then read-only mirrors refreshed on access.  native=False
    (or the non-joint association, or box_fusion.check_valid) drives the same kernels from Python
    with the reference's containers.  Both give bit-identical results."""

    def __init__(self, cfg, K3, H=480, W=640, device="cuda", legacy_promotion=True,
                 stale_last_frame=True, native=None):
        self.cfg = cfg
        self.dev = torch.device(device)
        self.K3 = np.asarray(K3, np.float32)
        self.H, self.W = H, W
        self.gap = int(cfg["data"].get("gap", 1)) if "data" in cfg else 1
        self._bm = BoxManager(cfg)
        with warnings.catch_warnings():
            # the CA-1M branch's missing K_depth.txt: the stream's K replaces it right below
            # (demo.py:117-118 does the same before the first fusion)
            warnings.filterwarnings("ignore", message="BoxFusion: .*K_depth.txt not found")
            self._fuser = BoxFusion(cfg, device=device, legacy_promotion=legacy_promotion)
        self._fuser.update_intrinsics((W, H), self.K3)
        self._fuser.update_K_flag = True
        self.stale_last_frame = stale_last_frame
        self._apb = None
        self._all_poses = None
        self.per_frame_ins = None
        self.all_kf_pose = {}
        self.box_count = 0
        self._last_pred = None
        self._stats = dict(keyframes=0, suppressed=0)
        self.K_dev = torch.from_numpy(self.K3).to(self.dev)     # uploaded once
        self._pf_table = None    # append-only device table behind per_frame_ins
        # nms + correspondence association chained on the device (one host round trip);
        # False: the reference's two separate calls (same results)
        self.joint = os.environ.get("BF_JOINT_ASSOC", "1") != "0"
        self.native = (os.environ.get("BF_NATIVE_FUSION", "1") != "0") if native is None else bool(native)
        self._mode = None        # "native" | "python", fixed by the first keyframe
        self._seq = None         # _lib.FusionSequencer in native mode
        self._ver = 0            # sequencer calls so far (mirror cache key)
        self._mirror_ver = -1
        self._apb_ver = -1
        self._seq_cfg = None

    # -- mode and mirrors ------------------------------------------------------------------------
    def _select_mode(self):
        if self._mode is None:
            bf = self.cfg["box_fusion"]
            ok = self.native and self.joint and not bf.get("check_valid", False)
            self._mode = "native" if ok else "python"
        return self._mode

    def _refresh(self):
        """pull the sequencer's BoxManager / BoxFusion state into the mirrors (one wait)"""
        if self._mode != "native" or self._seq is None or self._mirror_ver == self._ver:
            return
        st = self._seq.state()
        bm, f = self._bm, self._fuser
        bm.fusion_list = self._seq.lists(0, int(st[1]), int(st[2]))
        bm._fusion_flag = self._seq.flags(int(st[3]))
        bm.already_fusion = self._seq.lists(1, int(st[4]), int(st[5]))
        if int(st[9]) > f.hull_overflow_calls:
            _warn_hull_once()
        f.hull_overflow_calls, f.fit_calls, f.updated_total = int(st[9]), int(st[8]), int(st[7])
        f.last_stats = dict(jobs=int(st[10]), updated=int(st[11]), views=int(st[13]), iters=int(st[12]))
        self._stats["suppressed"] = int(st[6])
        self._mirror_ver = self._ver

    @property
    def box_manager(self):
        self._refresh()
        return self._bm

    @property
    def fuser(self):
        self._refresh()
        return self._fuser

    @property
    def all_pred_box(self):
        if self._mode != "native" or self._seq is None:
            return self._apb
        if self._apb_ver != self._ver:
            st = self._seq.state()
            n = int(st[0])
            if n < 0:
                self._apb = None
            else:
                ids, xyz, vn = self._seq.global_rows(n, self.dev)
                apb = self.per_frame_ins[ids.astype(np.int64)]
                b = apb.pred_boxes_3d
                apb.pred_boxes_3d = type(b)._views(xyz, b.R)      # fused rows refined
                apb.valid_num = vn
                self._apb = apb
            self._apb_ver = self._ver
        return self._apb

    @all_pred_box.setter
    def all_pred_box(self, v):
        if self._mode == "native":
            raise _lib.HipError("all_pred_box is owned by the native sequencer (native=False to edit it)")
        self._apb = v

    @property
    def all_poses(self):
        if self._mode != "native" or self._seq is None:
            return self._all_poses
        apb = self.all_pred_box
        return None if apb is None else apb.cam_pose.cpu().numpy()

    @all_poses.setter
    def all_poses(self, v):
        if self._mode == "native":
            raise _lib.HipError("all_poses is owned by the native sequencer")
        self._all_poses = v

    @property
    def last_pred(self):
        lp = self._last_pred
        if isinstance(lp, tuple):        # native batches: (batch, first row, rows), sliced lazily
            preds, off, n = lp
            lp = self._last_pred = preds[off:off + n]
        return lp

    @last_pred.setter
    def last_pred(self, v):
        self._last_pred = v

    @property
    def stats(self):
        """keyframes, suppressed boxes, fused boxes (resolves a deferred fusion result)"""
        bm = self.box_manager
        bm.flush()
        return dict(self._stats, fused=self._fuser.updated_total)

    def _to_python(self):
        """hand the state from the sequencer to the Python-driven path (same values)"""
        if self._mode != "native":
            return
        if self._seq is not None:
            self._refresh()
            apb = self.all_pred_box
            self._all_poses = self.all_poses
            self._apb = apb
            self._seq = None
        self._mode = "python"

    def _fseq_cfg(self):
        f = self._fuser
        key = (f.H, f.W, f.K.tobytes(), f.legacy_promotion, f.strict_hull, f.fusion_iters, f.pst_size)
        if self._seq_cfg is None or self._seq_cfg[0] != key:
            c = _lib.FseqCfg()
            bf = self.cfg["box_fusion"]
            c.nms = self._bm.nms_cfg(bf["nms_threshold"])
            c.corr = self._bm.corr_cfg(self.cfg["association"]["small_threshold"], self.W, self.H)
            c.fuse = f.fuse_cfg()
            c.use_fusion = 1 if bf.get("use", True) else 0
            c.strict_hull = 1 if f.strict_hull else 0
            self._seq_cfg = (key, c)
        return self._seq_cfg[1]

    # -- keyframes -------------------------------------------------------------------------------
    def keyframes(self, counts, poses, preds, sizes):
        """Several keyframes in frame order whose detections arrive as ONE Instances3D `preds`
        (camera frame, keyframe j's boxes are rows [off_j, off_j + sizes[j])): the per-box
        geometry (world transform, projection, ids) runs once for all of them, then each keyframe
        goes through the serial association / fusion exactly like keyframe()."""
        t_prof = time.perf_counter() if _PROFILE else 0.0
        sizes = np.asarray(sizes, np.int64)
        n_tot = int(sizes.sum())
        poses = np.asarray(poses, np.float32)
        if n_tot:
            kf = np.repeat(np.arange(len(sizes)), sizes)
            preds.cam_pose = _lib.h2d(poses[kf], self.dev)
            ids = np.empty((2, n_tot), np.int64)
            ids[0] = np.asarray(counts, np.int64)[kf]
            # init_id of keyframe j = box_count before it + row: box_count grows by n per keyframe
            ids[1] = self.box_count + np.arange(n_tot)
            idd = _lib.h2d(ids, self.dev)
            preds.frame_id, preds.init_id = idd[0], idd[1]
            preds.valid_num = torch.zeros(n_tot, device=self.dev)
            preds.pred_boxes_3d.transform2world(preds.cam_pose)
            preds.project_3d_boxes(self.K_dev, H=self.H, W=self.W)
        if self._select_mode() == "native":
            self._native_batch(counts, poses, preds if n_tot else None, sizes, t_prof)
            # the batch's row gathers flag BF_DEV_INDEX_RANGE in the status word (one read per
            # batch; the sequencer has already waited on the device)
            if _PROFILE:
                print(f"keyframes() before status: {1e3 * (time.perf_counter() - t_prof):.2f} ms",
                      file=sys.stderr, flush=True)
            if n_tot:
                _lib.check_status(self.dev)
            if _PROFILE:
                print(f"keyframes() {len(sizes)} kf: {1e3 * (time.perf_counter() - t_prof):.2f} ms",
                      file=sys.stderr, flush=True)
            return
        off = 0
        for j, c in enumerate(counts):
            n = int(sizes[j])
            self.keyframe(c, poses[j], preds[off:off + n] if n else None, prepared=True)
            off += n
        _lib.check_status(self.dev)     # row gathers of the batch (one read per batch)

    def _native_batch(self, counts, poses, preds, sizes, t_prof=0.0):
        if self._seq is None:
            self._seq = _lib.FusionSequencer()
        n_tot = int(sizes.sum())
        p_base = len(self.per_frame_ins) if self.per_frame_ins is not None else 0
        if n_tot:
            # per_frame_ins = cat(per_frame_ins, pred) for the whole batch (one gather)
            cur = self.per_frame_ins if self.per_frame_ins is not None else preds[0:0]
            self.per_frame_ins = self._per_frame_append(preds, cur)
            pf = self.per_frame_ins
            b3 = pf.pred_boxes_3d
            fields = [t if t.dtype == torch.float32 and t.is_contiguous() else t.float().contiguous()
                      for t in (b3.tensor, b3.R, pf.scores, pf.pred_boxes, pf.cam_pose, pf.projected_boxes)]
            self._ver += 1
            if _PROFILE:
                print(f"keyframes() geometry + append: {1e3 * (time.perf_counter() - t_prof):.2f} ms",
                      file=sys.stderr, flush=True)
            self._seq.keyframes(self._fseq_cfg(), sizes, p_base, fields, self.K_dev, self._fuser._pst_dev)
            if _PROFILE:
                print(f"keyframes() after native: {1e3 * (time.perf_counter() - t_prof):.2f} ms",
                      file=sys.stderr, flush=True)
        bm = self._bm
        off = 0
        for j, c in enumerate(counts):
            n = int(sizes[j])
            self.all_kf_pose[c] = np.asarray(poses[j], np.float32)
            if n:
                self._stats["keyframes"] += 1
                self.box_count += n
                bm.last_fusion_frame.extend([0] for _ in range(n))
                self._last_pred = (preds, off, n)
            else:
                self._last_pred = EMPTY_KEYFRAME
            bm.num_record[c] = self.box_count
            off += n

    def keyframe(self, count, pose, pred, prepared=False):
        """pred: Instances3D of this keyframe in CAMERA coordinates (after the detection filters
        and the CLIP step), tensors on the device; it is modified in place like the reference's.
        prepared=True: world transform, projection and the id fields were already applied
        (keyframes())."""
        if not prepared and self._select_mode() == "native":
            n = len(pred) if pred is not None and len(pred._fields) else 0
            self.keyframes([count], np.asarray(pose, np.float32)[None], pred if n else None, [n])
            return
        cfg, bm = self.cfg, self._bm
        self.last_pred = pred
        pose = np.asarray(pose, np.float32)
        self.all_kf_pose[count] = pose
        n = len(pred) if pred is not None and len(pred._fields) else 0
        pose_np = np.repeat(pose[None], n, 0)
        if n == 0:
            self._last_pred = EMPTY_KEYFRAME
            bm.num_record[count] = self.box_count
            return
        self._stats["keyframes"] += 1
        if not prepared:
            pred.cam_pose = _lib.h2d(pose_np, self.dev)
            pred.frame_id = torch.full((n,), count, dtype=torch.int64, device=self.dev)
            pred.init_id = self.box_count + torch.arange(n, device=self.dev)
            pred.valid_num = torch.zeros(n, device=self.dev)
            pred.pred_boxes_3d.transform2world(pred.cam_pose)
            pred.project_3d_boxes(self.K_dev, H=self.H, W=self.W)
        self.box_count += n
        bm.num_record[count] = self.box_count
        if self._apb is None and (count < self.gap or self.per_frame_ins is None):
            self._apb = pred
            self._all_poses = pose_np
            self.per_frame_ins = pred
            bm.init_new_predictions(n, 0)
            return
        bm.init_new_predictions(n, len(self.per_frame_ins))
        n_before = len(self._apb)
        cur_global = self._apb
        all_pred_box = Instances3D.cat([self._apb, pred])
        self.per_frame_ins = self._per_frame_append(pred)
        all_poses = np.concatenate((self._all_poses, pose_np), axis=0)
        corners = all_pred_box.pred_boxes_3d.corners       # shared by both association steps
        if self.joint and len(all_pred_box) > 1:
            # nms + correspondence back to back on the device, one read-back
            mask, success, keep_idx, any_cur, keep_dev = Instances3D.joint_association(
                all_pred_box, n_before, cfg["box_fusion"]["nms_threshold"],
                cfg["association"]["small_threshold"], bm, self.per_frame_ins.cam_pose,
                pred.cam_pose[0], self.K_dev, corners, H=self.H, W=self.W)
            if not any_cur:
                keep_idx = np.asarray(mask)
            kept = all_pred_box._device_rows([], keep_dev)
            all_pred_box = kept if kept is not None else all_pred_box[keep_idx]
            all_poses = all_poses[keep_idx]
            if not any_cur:
                self._stats["suppressed"] += len(success)
                bm.update(keep_idx)
                self._apb, self._all_poses = all_pred_box, all_poses
                return
        else:
            mask, success = Instances3D.spatial_association(all_pred_box, cfg["box_fusion"]["nms_threshold"],
                                                            bm, self.per_frame_ins.cam_pose, corners=corners)
            cur_keep = [i - n_before for i in mask if i >= n_before]
            any_cur = bool(cur_keep)
            keep_idx = np.asarray(mask)
            if any_cur:
                cur_success = [i - n_before for i in success if i >= n_before]
                all_pred_box, all_poses, keep_idx = Instances3D.correspondence_association(
                    cfg, bm, cur_keep, cur_success, pred, cur_global, all_pred_box, all_poses,
                    self.per_frame_ins.cam_pose, count, mask, self.K_dev, self.all_kf_pose,
                    threshold=cfg["association"]["small_threshold"], H=self.H, W=self.W,
                    corners=corners, cur_pose=pred.cam_pose[0])
        self._stats["suppressed"] += len(success)
        if any_cur:
            bm.update(keep_idx)
            if cfg["box_fusion"].get("check_valid", False):
                all_pred_box = bm.check_valid_num(all_pred_box, count, self.gap)
            if cfg["box_fusion"].get("use", True):
                self._fuser.boxfusion(all_pred_box, self.per_frame_ins, bm, defer=True)
        else:
            all_pred_box = all_pred_box[_lib.h2d(np.asarray(keep_idx, np.int64), self.dev)]
            all_poses = all_poses[keep_idx]
            bm.update(keep_idx)
        self._apb, self._all_poses = all_pred_box, all_poses

    def _per_frame_append(self, pred, cur=None):
        """per_frame_ins = cat(per_frame_ins, pred) on an append-only table: every field lives in a
        preallocated device buffer (capacity doubling), the new rows are written into its tail by
        one bf_rows_gather launch and per_frame_ins becomes views of the first n rows.  Rows never
        change once written, so earlier views stay valid.  `cur`: the rows to append to (default
        per_frame_ins)."""
        cur = self.per_frame_ins if cur is None else cur
        n, m = len(cur), len(pred)
        specs = []   # (key, box_type or None, [tensors of cur], [tensors of pred])
        for k, v in cur._fields.items():
            w = pred._fields.get(k)
            if isinstance(v, torch.Tensor) and isinstance(w, torch.Tensor) and v.is_cuda and \
                    w.dtype == v.dtype and w.shape[1:] == v.shape[1:]:
                specs.append((k, None, [v], [w]))
            elif hasattr(v, "tensor") and hasattr(v, "R") and hasattr(w, "R") and v.tensor.is_cuda:
                specs.append((k, type(v), [v.tensor, v.R], [w.tensor, w.R]))
            else:
                return Instances3D.cat([cur, pred])
        if set(pred._fields) != set(cur._fields) or \
                sum(len(t) for _, _, t, _ in specs) > _lib.ROWS_MAX_FIELDS:
            return Instances3D.cat([cur, pred])
        tab = self._pf_table
        flat_cur = [t for _, _, ts, _ in specs for t in ts]
        if tab is None or tab["n"] != n or tab["keys"] != [k for k, _, _, _ in specs] or \
                any(t.data_ptr() != b.data_ptr() for t, b in zip(flat_cur, tab["bufs"])):
            tab = None                                   # (re)build from the current rows
        if tab is None or n + m > tab["cap"]:
            cap = max(4096, 2 * (n + m))
            bufs = [torch.empty((cap,) + t.shape[1:], dtype=t.dtype, device=t.device) for t in flat_cur]
            if n:
                _lib.rows_gather([(t.contiguous(), None) for t in flat_cur], n_out=n,
                                 outs=[b[:n] for b in bufs])
            tab = dict(cap=cap, bufs=bufs, keys=[k for k, _, _, _ in specs], n=n)
        bufs = tab["bufs"]
        flat_new = [t.contiguous() for _, _, _, ts in specs for t in ts]
        if m:
            _lib.rows_gather([(t, None) for t in flat_new], n_out=m, outs=[b[n:n + m] for b in bufs])
        tab["n"] = n + m
        ret = Instances3D(cur.image_size)
        o = 0
        for k, box_type, ts, _ in specs:
            if box_type is None:
                ret.set(k, bufs[o][:n + m])
                o += 1
            else:
                ret.set(k, box_type._views(bufs[o][:n + m], bufs[o + 1][:n + m]))
                o += 2
        self._pf_table = tab
        return ret

    def finish(self, count, pose, last_was_keyframe):
        """demo.py:200 `count == len(dataset) - 1` re-entry on a non-keyframe last frame."""
        if last_was_keyframe or not self.stale_last_frame or self._last_pred is None:
            return
        if self._last_pred is EMPTY_KEYFRAME:
            # demo.py:202-212: the re-entry with an empty pred_instances records the count only
            self.all_kf_pose[count] = np.asarray(pose, np.float32)
            self._bm.num_record[count] = self.box_count
            return
        if self._mode == "native" and self._stats["keyframes"] == 1:
            # one keyframe so far: the reference's all_pred_box and per_frame_ins ARE that
            # keyframe's pred object (demo.py:226-241), and the re-entry transforms it in place
            # through those aliases; the Python path reproduces the aliasing
            last = self.last_pred
            self._to_python()
            self._apb = self.per_frame_ins = last
            self._pf_table = None
        self.keyframe(count, pose, self.last_pred)

    # -- results ---------------------------------------------------------------------------------
    def boxes(self):
        """global boxes (xyzlhw [N,6], R [N,3,3]) on the host"""
        apb = self.all_pred_box
        if apb is None:
            return np.zeros((0, 6), np.float32), np.zeros((0, 3, 3), np.float32)
        b = apb.pred_boxes_3d
        return b.tensor.cpu().numpy(), b.R.cpu().numpy()


class AsyncFusion:
    """Runs a FusionStage on a worker thread with its own HIP stream, so the serial keyframe
    state machine of keyframes k overlaps the (independent) detection of later frames on the
    main stream.  Keyframes are consumed strictly in submission (= frame) order; `make_pred` is
    called on the worker, after its stream waited for `ready` (an event on the producer stream),
    so it may read the producer's buffers."""

    def __init__(self, stage: FusionStage, stream=None):
        self.stage = stage
        self.device_index = stage.dev.index if stage.dev.index is not None else torch.cuda.current_device()
        self.stream = stream if stream is not None else torch.cuda.Stream(device=self.device_index)
        self.q = queue.Queue()
        self.err = None
        self.busy_s = 0.0      # wall time the worker spent inside keyframe jobs (after their input was ready)
        self.thread = threading.Thread(target=self._run, name="boxfusion-fusion", daemon=True)
        self.thread.start()
        _lib.register_worker(self)

    def submit(self, count, pose, make_pred, ready=None):
        self.q.put((count, pose, make_pred, ready))

    def submit_call(self, fn, ready=None):
        """fn(stage) on the worker (e.g. stage.keyframes for a whole batch of keyframes)"""
        self.q.put((None, None, fn, ready))

    def _run(self):
        if os.environ.get("BF_PROFILE_FUSION"):      # diagnostic: cProfile of the worker thread
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            try:
                self._loop()
            finally:
                pr.disable()
                st = pstats.Stats(pr, stream=sys.stderr)
                st.sort_stats("tottime").print_stats(25)
                st.sort_stats("cumulative").print_stats(40)
            return
        self._loop()

    def _loop(self):
        torch.cuda.set_device(self.device_index)
        with torch.cuda.stream(self.stream):
            while True:
                item = self.q.get()
                if item is None:
                    return
                if self.err is not None:
                    continue
                count, pose, make_pred, ready = item
                try:
                    if ready is not None:
                        # the job reads the producer's outputs on the host right away (record
                        # counts), so wait here: busy_s then counts fusion work only, not the wait
                        # for the detect stream
                        ready.synchronize()
                        self.stream.wait_event(ready)
                    t0 = time.perf_counter()
                    if count is None:
                        make_pred(self.stage)
                    else:
                        self.stage.keyframe(count, pose, make_pred())
                    self.busy_s += time.perf_counter() - t0
                except BaseException as e:  # noqa: BLE001 - re-raised on join()
                    self.err = e

    def join(self):
        self.q.put(None)
        self.thread.join()
        self.stream.synchronize()
        if self.err is not None:
            raise self.err
        return self.stage

    def stop(self, timeout=None):
        """interpreter exit (_lib._shutdown): drop queued jobs, let the running one finish, and
        drain the worker's stream before the streams and sequencers it uses are released"""
        if not self.thread.is_alive():
            return True
        try:
            while True:
                self.q.get_nowait()
        except queue.Empty:
            pass
        self.q.put(None)
        self.thread.join(timeout)
        if self.thread.is_alive():
            # still launching (a long batch): its sequencers and CU-masked streams must outlive it,
            # so _shutdown leaves them to process teardown instead of releasing them under it
            import warnings
            warnings.warn("fusion worker still running at exit: its HIP resources are not released",
                          RuntimeWarning)
            return False
        self.stream.synchronize()
        return True
