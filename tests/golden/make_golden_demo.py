"""Golden fixture: the REFERENCE's own demo.py `run()` (demo.py:33-387) over a synthetic stream at
gap 25 whose last frame is not a keyframe (so the stale last-frame re-fusion of demo.py:200,
SURVEY §8 quirk 1, fires), recording what run() writes: the global boxes and the framewise
boxes / class indices / CLIP features (save_box, demo.py:368-387), the box manager's final
fusion lists, every box's world-space geometry (transform2world + project_3d_boxes as the
reference computed them, keyed by init_id), and every rerun.log call of the run with vis.rerun on
(demo.py:93-197, 329-330; tools/utils.py:37-96) through a recording rerun stand-in.

run()'s arguments are the only things supplied from outside:
  * model: returns the seeded scene's detections of the next keyframe as Instances3D in the
    camera frame (random-weight CuTR boxes would be noise), with `pixel_mean` for demo.py:70;
  * clip_model: a stand-in for the absent SAMCLIP (demo.py:458), get_batch_images_clip_features
    returning seeded features (near a text row for 3 of 4 crops, so categories survive the
    threshold), one draw per call;
  * dataset: samples packed like the ScanNet iterator (make_golden_cutr.make_sample).
Absent third-party modules are stand-ins (rerun, open3d, open_clip, torchvision, cv2, pycuda
with the oracle's fitness as in make_golden.py).  Run:
  python tests/golden/make_golden_demo.py  ->  tests/golden/demo_gap25.npz
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden_results  # noqa: E402,F401  (stand-ins; tools.utils imported)
import make_golden as MG  # noqa: E402
from make_golden_cutr import make_sample  # noqa: E402


class _Any:
    """permissive stand-in object (rerun blueprint builders are called at run() start)"""

    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Any()

    def __getattr__(self, name):
        return _Any()


for name in ("rerun", "rerun.blueprint", "open_clip"):
    mod = sys.modules.get(name) or types.ModuleType(name)
    mod.__getattr__ = lambda attr: _Any()
    sys.modules[name] = mod
sys.modules["rerun"].blueprint = sys.modules["rerun.blueprint"]

# A recording rerun: demo.py's (and tools/utils.visualize_online_boxes's) rerun.log calls become
# plain records -- entity path, time, archetype and its fields (images as shape + adler32, the
# trajectory strip as its length, sum and last point) -- in call order.
RERUN_LOG = []
_RR_TIME = [None]


class _Arch(dict):
    def __init__(self, kind, **fields):
        super().__init__(fields)
        self.kind = kind

    def compress(self, *a, **k):          # rerun.Image(...).compress()
        return self


def _arch(kind):
    return lambda *a, **k: _Arch(kind, _args=a, **k)


def _f(x):
    return np.asarray(x, np.float64).tolist()


def _rr_log(path, arch, *a, **k):
    import zlib
    kind = arch.kind
    rec = {"path": path, "time": _RR_TIME[0], "kind": kind}
    if kind == "Transform3D":
        rec.update(translation=_f(arch["translation"]), quaternion_xyzw=_f(arch["rotation"]["xyzw"]))
    elif kind == "Pinhole":
        rec.update(image_from_camera=_f(arch["image_from_camera"]), resolution=_f(arch["resolution"]))
    elif kind in ("Image", "DepthImage"):
        img = np.ascontiguousarray(np.asarray(arch["_args"][0]))
        rec.update(shape=list(img.shape), dtype=str(img.dtype), adler32=zlib.adler32(img.tobytes()))
    elif kind == "LineStrips3D":
        strip = np.asarray(arch["_args"][0][0], np.float64).reshape(-1, 3)
        rec.update(n=len(strip), sum=float(strip.sum()), last=_f(strip[-1]) if len(strip) else [],
                   colors=_f(arch["colors"]))
    elif kind == "Boxes3D":
        rec.update(centers=_f(arch["centers"]), sizes=_f(arch["sizes"]),
                   quaternions_xyzw=[_f(q["xyzw"]) for q in arch["quaternions"]],
                   colors=[_f(c) for c in arch["colors"]], labels=[str(x) for x in arch["labels"]],
                   show_labels=bool(arch["show_labels"]))
    else:
        rec.update(fields=sorted(arch))
    RERUN_LOG.append(rec)


_rr = sys.modules["rerun"]
_rr.log = _rr_log
_rr.set_time_seconds = lambda timeline, t, **k: _RR_TIME.__setitem__(0, [timeline, float(t)])
_rr.new_recording = lambda *a, **k: _Any()
_rr.spawn = lambda *a, **k: None
_rr.Quaternion = lambda xyzw: {"xyzw": np.asarray(xyzw, np.float64)}
for _kind in ("Transform3D", "Pinhole", "Image", "DepthImage", "Points3D", "LineStrips3D", "Boxes3D"):
    setattr(_rr, _kind, _arch(_kind))
# retriev's cv2.resize (tools/utils.py:395): the stand-in CLIP ignores pixels
sys.modules["cv2"].resize = lambda img, size, *a, **k: np.zeros((size[1], size[0], 3), np.uint8)

import demo  # noqa: E402  (the reference's demo.py)
from boxfusion.boxes import GeneralInstance3DBoxes  # noqa: E402
from boxfusion.instances import Instances3D  # noqa: E402
from boxfusion.preprocessor import Augmentor, Preprocessor  # noqa: E402

REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from boxfusion_amd.synthetic import SCANNET_K, Scene, frame_rgbd  # noqa: E402

GAP, N_FRAMES = 25, 188            # keyframes 0, 25, ..., 175; frame 187 is the stale last frame
SCENE = dict(seed=7, period=400)
CLIP_SEED = 123


def cfg_demo(out_dir):
    c = dict(MG.SCANNET_CFG)
    # dataset 'online': demo.py:374's post_process (ScanNet only) would make the save loop raise
    # IndexError when it drops a box; a datadir naming scannet keeps BoxFusion's ScanNet
    # intrinsics branch (box_fusion.py:36-42)
    c["dataset"] = "online"
    c["data"] = dict(datadir="/synthetic/scannet", gap=GAP, start=0, output_dir=out_dir)
    c["detection"] = dict(score_thresh=0.5, uv_bound=True, uv_bound_value=0.9, floor_mask=True,
                          floor_ratio=15, scale_box=1.5, class_sim_thres=25.0, size_max_thres=None)
    c["box_fusion"] = dict(c["box_fusion"], clip_sim_coeff=1.0)
    # demo.py's rerun logging on (re_vis=True below; it only gates the log calls), recorded
    c["vis"] = dict(rerun=True, show_class=False, show_label=False, trajectory=True)
    c["eval"] = True
    return c


def scene_instances(det, H=480, W=640):
    p = Instances3D((H, W))
    p.scores = torch.from_numpy(det["scores"].copy())
    p.pred_boxes = torch.from_numpy(det["pred_boxes"].copy())
    p.pred_boxes_3d = GeneralInstance3DBoxes(torch.from_numpy(det["xyzlhw"].copy()),
                                             torch.from_numpy(det["R"].copy()))
    p.pred_proj_xy = torch.from_numpy(det["proj_xy"].copy())
    return p


class SceneModel:
    """stand-in CuTR: the scene detections of keyframe k on its k-th call"""

    def __init__(self, scene, keyframes):
        self.scene, self.keyframes, self.calls = scene, keyframes, 0
        self.pixel_mean = torch.zeros(3, 1, 1)

    def __call__(self, packaged):
        f = self.keyframes[self.calls]
        self.calls += 1
        return [scene_instances(self.scene.detections(f))]


class StubCLIP:
    """stand-in for SAMCLIP: seeded features, 3 of 4 near a text row (similarity above 25)"""

    def __init__(self, text, seed=CLIP_SEED):
        self.text = text.numpy().astype(np.float32)
        self.seed, self.calls = seed, 0

    def features(self, n):
        rng = np.random.default_rng(self.seed + self.calls)
        self.calls += 1
        f = rng.normal(0, 1, (n, self.text.shape[1])).astype(np.float32)
        pick = rng.integers(0, len(self.text), n)
        near = np.arange(n) % 4 != 3
        f[near] = self.text[pick[near]] * 30.0 + f[near] * 0.4
        return f

    def get_batch_images_clip_features(self, images):
        return torch.from_numpy(self.features(len(images))), None


class Stream:
    def __init__(self, scene):
        self.scene = scene

    def __len__(self):
        return N_FRAMES

    def __iter__(self):
        for i in range(N_FRAMES):
            rgb, depth = frame_rgbd(i)
            s, _, _ = make_sample(rgb, depth, SCANNET_K, self.scene.pose(i))
            s["meta"] = dict(video_id=["synthetic"], timestamp=i)
            yield s


def main():
    torch.set_num_threads(8)
    scene = Scene(**SCENE)
    keyframes = [f for f in range(N_FRAMES) if f % GAP == 0]
    names = np.genfromtxt(os.path.join(REPO, "boxfusion_amd", "data", "panoptic_categories_nomerge.txt"),
                          delimiter="\n", dtype=str)
    text = torch.from_numpy(np.load(os.path.join(REPO, "boxfusion_amd", "data", "class_features.npy")).astype(np.float32))
    saved = {}
    demo.save_box = lambda data, fn: saved.__setitem__(os.path.basename(fn), data)
    managers = []
    _BM = demo.BoxManager

    class RecBM(_BM):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            managers.append(self)

    demo.BoxManager = RecBM
    # record every box's world-space geometry as the reference computed it (transform2world and
    # project_3d_boxes on torch CPU), keyed by init_id, so the GPU replay can run its association
    # and fusion kernels on bit-identical inputs (the particle search amplifies ulps)
    geom = {}
    _proj = Instances3D.project_3d_boxes

    def project_rec(self, K, H=480, W=640):
        r = _proj(self, K, H=H, W=W)
        for j, i in enumerate(self.init_id.numpy().tolist()):
            geom[int(i)] = (self.pred_boxes_3d.tensor[j].numpy().copy(), self.pred_boxes_3d.R[j].numpy().copy(),
                            self.projected_boxes[j].numpy().copy())
        return r

    Instances3D.project_3d_boxes = project_rec
    MG.STUB_STATE["cfg"] = MG.OR.fuse_cfg(MG.SCANNET_CFG, np.eye(4), 480, 640, legacy=False)
    MG.OR.hull_overflow()
    with tempfile.TemporaryDirectory() as out_dir, MG.quiet():
        cfg = cfg_demo(out_dir)
        demo.run(cfg, SceneModel(scene, keyframes), Stream(scene), StubCLIP(text), None, names, text.clone(),
                 Augmentor(("wide/image", "wide/depth")), Preprocessor(),
                 score_thresh=cfg["detection"]["score_thresh"], viz_on_gt_points=False, gap=GAP,
                 re_vis=True)
    # fitness evaluations past the reference kernel's corners_i[36] / convex_inter[8]
    # (box_fusion.py:378-384): the run is the reference's with the exact hull there
    hull_over = np.asarray(MG.OR.hull_overflow(), np.int64)
    glob_list = saved["synthetic_boxes.pkl"][0]
    fw = saved["framewise_boxes.pkl"][0]
    bm = managers[0]
    fl_flat, fl_off = MG.ragged([list(map(int, r)) for r in bm.fusion_list])
    af_flat, af_off = MG.ragged([list(map(int, r)) for r in bm.already_fusion])
    out = dict(gap=np.int32(GAP), n_frames=np.int32(N_FRAMES), scene_seed=np.int32(SCENE["seed"]),
               scene_period=np.int32(SCENE["period"]), clip_seed=np.int32(CLIP_SEED),
               global_corners=np.stack([t[1] for t in glob_list]).astype(np.float32),
               fw_class=np.array([int(t[0]) for t in fw], np.int64),
               fw_corners=np.stack([np.asarray(t[1]) for t in fw]).astype(np.float32),
               fw_features=np.stack([np.asarray(t[2]) for t in fw]).astype(np.float32),
               fusion_list_flat=fl_flat, fusion_list_off=fl_off,
               already_fusion_flat=af_flat, already_fusion_off=af_off,
               num_record_frames=np.array(sorted(bm.num_record), np.int32),
               num_record=np.array([bm.num_record[k] for k in sorted(bm.num_record)], np.int64),
               geom_tensor=np.stack([geom[i][0] for i in range(len(geom))]),
               geom_R=np.stack([geom[i][1] for i in range(len(geom))]),
               geom_proj=np.stack([geom[i][2] for i in range(len(geom))]), hull_over=hull_over,
               rerun_json=np.array(__import__("json").dumps(RERUN_LOG)))
    assert sorted(geom) == list(range(len(geom)))
    np.savez_compressed(os.path.join(HERE, "demo_gap25.npz"), **out)
    print("demo golden:", {k: getattr(v, "shape", v) for k, v in out.items()})


if __name__ == "__main__":
    main()
