"""The demo.py keyframe state machine (FusionStage) and the per-frame DetectStage on the GPU.

FusionStage is compared bit for bit with the reference's recorded traces and with oracle/chain.py,
given the same world-space boxes and projections.  The GPU transform2world / projection differ from
the reference's torch-CPU ones by ~1 ulp (test_gpu_fusion.py pins them at 2e-6 / 2e-3 px), and the
particle search amplifies ulps, so with its own geometry the chain is checked only over the first
keyframes (test_fusion_stage_own_geometry)."""
import json

import numpy as np
import pytest
import torch

from tests import trace_util as TU

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda")


def _inject_geometry(monkeypatch, dev, src):
    """Make FusionStage use given world-space boxes and projections (indexed by init_id) in place
    of its own transform2world / projection kernels, so the association and fusion kernels see
    bit-identical inputs to the run they are compared with."""
    from boxfusion_amd.instances import Instances3D

    def project(self, K, H=480, W=640):
        ids = self.init_id.cpu().numpy()
        self.pred_boxes_3d.tensor = torch.from_numpy(np.ascontiguousarray(src["tensor"][ids])).to(dev)
        self.pred_boxes_3d.R = torch.from_numpy(np.ascontiguousarray(src["R"][ids])).to(dev)
        self.projected_boxes = torch.from_numpy(np.ascontiguousarray(src["proj"][ids])).to(dev)
    monkeypatch.setattr(Instances3D, "project_3d_boxes", project)


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("name", TU.TRACES)
def test_fusion_stage_vs_trace(dev, name, native, monkeypatch):
    """demo.py keyframe state machine on the GPU == the reference's recorded chain, bit for bit,
    given the reference's own world-space boxes and projections (pf_* of the trace).  The trace
    is the reference's control flow with the exact hull wherever its kernel overruns
    convex_inter[8] (recorded per keyframe, hull_over): the keyframes before the first such
    fusion are reference-pinned outright, and BoxFusion's BF_DEV_HULL_OVERFLOW count matches the
    record keyframe by keyframe.  fusion_trace_faceon.npz has no overrun anywhere (every keyframe
    pinned); fusion_trace_ca1m.npz runs ca1m.yaml's thresholds on 384 x 512 portrait frames.
    native: the library's keyframe sequencer (bf_fseq) runs the state machine; else Python
    drives the same kernels."""
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    t = TU.load(name)
    cfg, K, H, W = TU.trace_setup(t)
    _inject_geometry(monkeypatch, dev, dict(tensor=t["pf_tensor"], R=t["pf_R"], proj=t["pf_proj"]))
    st = FusionStage(cfg, K, H=H, W=W, device=dev, legacy_promotion=False, native=native)
    nd = t["n_det"]
    fused = 0
    for k, frame in enumerate(t["frame"]):
        a, b = int(nd[:k].sum()), int(nd[:k + 1].sum())
        det = {key: t["det_" + key][a:b] for key in ["scores", "pred_boxes", "xyzlhw", "R", "proj_xy"]}
        calls = st.fuser.hull_overflow_calls
        st.keyframe(int(frame), t["pose"][k], scene_instances(det, dev, H, W))
        got, _ = st.boxes()
        assert st.box_manager.fusion_list == TU._lists(t, "post_fl", k), f"kf {k}"
        assert st.box_manager.already_fusion == TU._lists(t, "fused", k), f"kf {k}"
        # (the read of already_fusion above resolved the deferred fusion result)
        assert (st.fuser.hull_overflow_calls > calls) == bool(t["hull_over"][k].any()), f"kf {k}"
        np.testing.assert_array_equal(got, TU._rows(t, "post_tensor", k), err_msg=f"kf {k}")
        np.testing.assert_array_equal(st.all_pred_box.valid_num.cpu().numpy(),
                                      TU._rows(t, "post_valid_num", k), err_msg=f"kf {k}")
        fused = len(st.box_manager.already_fusion)
    assert fused >= 10


def test_fusion_stage_own_geometry(dev):
    """Without injection (GPU transform2world / projection, equal to torch-CPU within ~1 ulp):
    the first keyframes agree exactly in state; unfused boxes within 1e-4, fused boxes (a random
    search that amplifies ulp-level hull differences) within 5 cm."""
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K
    t = TU.load("fusion_trace.npz")
    st = FusionStage(TU.SCANNET_CFG, SCANNET_K, device=dev, legacy_promotion=False)
    nd = t["n_det"]
    for k in range(4):
        a, b = int(nd[:k].sum()), int(nd[:k + 1].sum())
        det = {key: t["det_" + key][a:b] for key in ["scores", "pred_boxes", "xyzlhw", "R", "proj_xy"]}
        st.keyframe(int(t["frame"][k]), t["pose"][k], scene_instances(det, dev))
        assert st.box_manager.fusion_list == TU._lists(t, "post_fl", k), f"kf {k}"
        got, want = st.boxes()[0], TU._rows(t, "post_tensor", k)
        fused = np.array([fl in st.box_manager.already_fusion for fl in st.box_manager.fusion_list])
        np.testing.assert_allclose(got[~fused], want[~fused], rtol=0, atol=1e-4, err_msg=f"kf {k}")
        np.testing.assert_allclose(got[fused], want[fused], rtol=0, atol=5e-2, err_msg=f"kf {k}")


# first keyframe whose decisions (fusion lists, fused lists) differ from the reference when the
# chain runs on the GPU's own transform2world / projection (None: identical to the end); measured
# on MI355X, see DESIGN.md §2
OWN_GEOMETRY_FIRST_DIVERGENCE = {"fusion_trace.npz": None, "fusion_trace_small.npz": 13,
                                 "fusion_trace_ca1m.npz": None, "fusion_trace_faceon.npz": None}


@pytest.mark.parametrize("name", TU.TRACES)
def test_fusion_stage_own_geometry_decisions(dev, name):
    """The whole chain WITHOUT injection (the GPU's own transform2world / projection, ~1 ulp from
    the reference's torch-CPU ones) over every keyframe of each trace: NMS keep / association
    decisions are compared through the fusion lists and the fused lists keyframe by keyframe;
    until the first divergence, unfused boxes agree within 1e-4 (north_star's box tolerance) and
    the fused boxes' error (the particle search amplifies ulp-level hull differences) is
    reported.  Writes gpurun_out/own_geometry_<trace>.json when that directory exists."""
    import os
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    t = TU.load(name)
    cfg, K, H, W = TU.trace_setup(t)
    st = FusionStage(cfg, K, H=H, W=W, device=dev, legacy_promotion=False)
    nd = t["n_det"]
    rep = dict(trace=name, keyframes=len(t["frame"]), first_divergence=None, max_unfused=0.0,
               max_fused=0.0, fused_boxes=0)
    for k, frame in enumerate(t["frame"]):
        a, b = int(nd[:k].sum()), int(nd[:k + 1].sum())
        det = {key: t["det_" + key][a:b] for key in ["scores", "pred_boxes", "xyzlhw", "R", "proj_xy"]}
        st.keyframe(int(frame), t["pose"][k], scene_instances(det, dev, H, W))
        bm = st.box_manager
        if bm.fusion_list != TU._lists(t, "post_fl", k) or bm.already_fusion != TU._lists(t, "fused", k):
            pf = st.per_frame_ins
            n = len(t["pf_tensor"]) if k == len(t["frame"]) - 1 else int(nd[:k + 1].sum())
            rep["first_divergence"] = dict(
                keyframe=k, lists_equal=bm.fusion_list == TU._lists(t, "post_fl", k),
                fused_equal=bm.already_fusion == TU._lists(t, "fused", k),
                world_box_err=float(np.abs(pf.pred_boxes_3d.tensor.cpu().numpy()[:n] - t["pf_tensor"][:n]).max()),
                proj_err_px=float(np.abs(pf.projected_boxes.cpu().numpy()[:n] - t["pf_proj"][:n]).max()))
            break
        got, want = st.boxes()[0], TU._rows(t, "post_tensor", k)
        fused = np.array([fl in bm.already_fusion for fl in bm.fusion_list], bool)
        if (~fused).any():
            rep["max_unfused"] = max(rep["max_unfused"], float(np.abs(got[~fused] - want[~fused]).max()))
        if fused.any():
            rep["max_fused"] = max(rep["max_fused"], float(np.abs(got[fused] - want[fused]).max()))
        rep["fused_boxes"] = int(fused.sum())
    print("own geometry", json.dumps(rep))
    if os.path.isdir("gpurun_out"):
        with open(f"gpurun_out/own_geometry_{name.replace('.npz', '')}.json", "w") as f:
            json.dump(rep, f)
    assert rep["max_unfused"] < 1e-4
    want_div = OWN_GEOMETRY_FIRST_DIVERGENCE.get(name, "unmeasured")
    if want_div != "unmeasured":
        got_div = rep["first_divergence"]["keyframe"] if rep["first_divergence"] else None
        assert got_div is None or (want_div is not None and got_div >= want_div), rep
    else:
        assert rep["first_divergence"] is None or rep["first_divergence"]["keyframe"] >= 4, rep


# The same decision-identity limit on a dense scene (150 objects, ~125 boxes per association, the
# n > 96 bit-mask NMS scan) without a reference trace: the GPU chain on its own geometry against
# oracle/chain.py (the reference-pinned restatement) on its own CPU geometry, at demo.py's ScanNet
# thresholds and at config/ca1m.yaml's (score 0.4, small_threshold 0.2, small_size 0.5; the 384 x
# 512 portrait CA-1M camera).  Value = first keyframe whose fusion / fused lists differ (None:
# identical over all SCENE150_KEYFRAMES); measured on MI355X (gpurun_out/own_geometry_scene150_*.json)
SCENE150_KEYFRAMES = 24
# (round 5: unfused boxes bit-equal to the oracle's until the divergence; the divergence is a
# fitness accept / reject on ulp-different projected hulls: fused boxes 5.4e-2 m apart at
# ScanNet thresholds, 7.5e-4 m at CA-1M's, profiles/own_geometry_scene150_*.json)
OWN_GEOMETRY_FIRST_DIVERGENCE_SCENE150 = {"scannet": 20, "ca1m": 2}


@pytest.mark.parametrize("setup", ["scannet", "ca1m"])
def test_own_geometry_scene150_vs_oracle_chain(dev, setup):
    """Unfused boxes within north_star's 1e-4 m of the oracle chain at every keyframe before the
    first decision divergence, and that divergence no earlier than measured."""
    import os
    from boxfusion_amd.box_fusion import load_pst
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    from oracle.chain import OracleChain
    if setup == "ca1m":
        t = TU.load("fusion_trace_ca1m.npz")
        cfg, K, H, W = TU.trace_setup(t)
    else:
        cfg, K, H, W = dict(TU.SCANNET_CFG, data=dict(gap=1)), SCANNET_K, 480, 640
    scene = Scene(seed=5, n_objects=150)
    st = FusionStage(cfg, K, H=H, W=W, device=dev, native=True)
    ch = OracleChain(cfg, K, H=H, W=W, pst=load_pst(), legacy=True)
    rep = dict(setup=setup, keyframes=SCENE150_KEYFRAMES, first_divergence=None, max_unfused=0.0,
               max_fused=0.0, fused_boxes=0, global_boxes=0)
    for k in range(SCENE150_KEYFRAMES):
        f = 3 * k
        d = scene.detections(f, K=K, size=(W, H))
        ch.keyframe(f, scene.pose(f), d)
        st.keyframe(f, scene.pose(f), scene_instances(d, dev, H, W))
        bm = st.box_manager
        if bm.fusion_list != ch.fusion_list or bm.already_fusion != ch.already_fusion:
            rep["first_divergence"] = dict(keyframe=k, lists_equal=bm.fusion_list == ch.fusion_list,
                                           fused_equal=bm.already_fusion == ch.already_fusion)
            break
        got, want = st.boxes()[0], ch.g["tensor"]
        fused = np.array([fl in bm.already_fusion for fl in bm.fusion_list], bool)
        if (~fused).any():
            rep["max_unfused"] = max(rep["max_unfused"], float(np.abs(got[~fused] - want[~fused]).max()))
        if fused.any():
            rep["max_fused"] = max(rep["max_fused"], float(np.abs(got[fused] - want[fused]).max()))
        rep["fused_boxes"], rep["global_boxes"] = int(fused.sum()), int(len(fused))
    print("own geometry scene150", json.dumps(rep))
    if os.path.isdir("gpurun_out"):
        with open(f"gpurun_out/own_geometry_scene150_{setup}.json", "w") as fh:
            json.dump(rep, fh)
    assert rep["max_unfused"] < 1e-4, rep
    want_div = OWN_GEOMETRY_FIRST_DIVERGENCE_SCENE150[setup]
    got_div = rep["first_divergence"]["keyframe"] if rep["first_divergence"] else None
    if want_div != "unmeasured":
        assert got_div is None or (want_div is not None and got_div >= want_div), rep
    else:
        assert got_div is None or got_div >= 2, rep


@pytest.mark.parametrize("native", [True, False])
def test_fusion_stage_vs_oracle_chain_gap1(dev, native, monkeypatch):
    """40 consecutive keyframes (gap=1, the benchmark's regime, numpy<2 promotion) against
    oracle/chain.py, bit for bit given the chain's geometry."""
    from boxfusion_amd.box_fusion import load_pst
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    from oracle.chain import OracleChain
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
    scene = Scene(seed=0)
    st = FusionStage(cfg, SCANNET_K, device=dev, native=native)
    ch = OracleChain(cfg, SCANNET_K, pst=load_pst(), legacy=True)
    src = {}
    _inject_geometry(monkeypatch, dev, src)
    for f in range(40):
        d = scene.detections(f)
        ch.keyframe(f, scene.pose(f), d)
        src.update(tensor=ch.pf["tensor"], R=ch.pf["R"], proj=ch.pf["proj"])
        st.keyframe(f, scene.pose(f), scene_instances(d, dev))
        assert st.box_manager.fusion_list == ch.fusion_list, f"frame {f}"
        assert st.box_manager.already_fusion == ch.already_fusion, f"frame {f}"
        np.testing.assert_array_equal(st.boxes()[0], ch.g["tensor"], err_msg=f"frame {f}")
    assert len(ch.already_fusion) > 5


def test_fusion_stage_empty_last_keyframe_native_vs_python(dev):
    """The last keyframe has no detections and the stream's last frame is not a keyframe: the
    re-entry of demo.py:200 sees an empty pred_instances and only records num_record[last]
    (demo.py:206-212).  Native sequencer and Python-driven stage agree on every list and on
    num_record."""
    import copy
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    cfg = copy.deepcopy(TU.SCANNET_CFG)
    cfg["data"] = dict(gap=5)
    scene = Scene(seed=0)
    out = {}
    for native in (True, False):
        st = FusionStage(cfg, SCANNET_K, device=dev, native=native)
        for f in range(0, 30, 5):
            d = scene.detections(f)
            if f == 25:                      # empty last keyframe
                d = {k: v[:0] for k, v in d.items()}
            st.keyframe(f, scene.pose(f), scene_instances(d, dev))
        st.finish(28, scene.pose(28), False)
        bm = st.box_manager
        out[native] = (dict(bm.num_record), bm.fusion_list, bm.already_fusion, st.boxes()[0])
    assert out[True][0] == out[False][0]
    assert 28 in out[True][0] and out[True][0][28] == out[True][0][25] == out[True][0][20]
    assert out[True][1] == out[False][1] and out[True][2] == out[False][2]
    np.testing.assert_array_equal(out[True][3], out[False][3])


def test_detect_stage_filtered(dev):
    """reference mode: filters -> CLIP on every surviving box -> categories / score update."""
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.pipeline import DetectStage
    from boxfusion_amd.synthetic import SCANNET_K, Scene, frame_rgbd
    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(192, True).eval()
        vis = VisionTransformer(224, 14, 1280, 2, 16, 1024).eval()
    cfg = dict(TU.SCANNET_CFG)
    cfg["detection"] = dict(cfg["detection"], score_thresh=0.0, uv_bound=False, floor_mask=False,
                            class_sim_thres=-100.0)
    B = 2
    det = DetectStage(cutr, vis, cfg, B, 480, 640, SCANNET_K, clip_capacity=64, device=dev)
    rgb = torch.from_numpy(np.stack([frame_rgbd(f)[0] for f in range(B)])).to(dev)
    depth = torch.from_numpy(np.stack([frame_rgbd(f)[1] for f in range(B)])).to(dev)
    poses = np.stack([Scene().pose(f) for f in range(B)])
    out = det(rgb, depth, poses)
    assert len(out) == B
    for r in out:
        assert len(r) == 100                     # nothing filtered, every category non-empty
        assert r.features.shape == (100, 1024)
        assert torch.allclose(r.features.norm(dim=-1), torch.ones(100, device=dev), atol=1e-4)
        assert (r.categories != "").all()
    xyz, valid = det.last["xyz"][0]
    assert xyz.shape == (480, 640, 3) and valid.float().mean() > 0.9


def test_async_fusion_equals_sync(dev):
    """AsyncFusion (worker thread + side stream, native sequencer) produces exactly the
    synchronous Python-driven state."""
    from boxfusion_amd.fusion_stage import AsyncFusion, FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
    scene = Scene(seed=0)
    sync = FusionStage(cfg, SCANNET_K, device=dev, native=False)
    asyn = AsyncFusion(FusionStage(cfg, SCANNET_K, device=dev, native=True))
    for f in range(30):
        d = scene.detections(f)
        sync.keyframe(f, scene.pose(f), scene_instances(d, dev))
        ev = torch.cuda.Event()
        ev.record()
        asyn.submit(f, scene.pose(f), (lambda d=d: scene_instances(d, dev)), ev)
    st = asyn.join()
    assert st.box_manager.fusion_list == sync.box_manager.fusion_list
    assert st.box_manager.already_fusion == sync.box_manager.already_fusion
    np.testing.assert_array_equal(st.boxes()[0], sync.boxes()[0])
    assert st.stats == sync.stats


def test_detect_stage_graph_equals_eager(dev):
    """HIP-graph replay of the detect stage reproduces the eager run on new inputs."""
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.pipeline import DetectStage
    from boxfusion_amd.synthetic import SCANNET_K, Scene, frame_rgbd
    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(192, True).eval()
        vis = VisionTransformer(224, 14, 1280, 2, 16, 1024).eval()
    B = 2
    kw = dict(crop_source="top", crops_per_frame=4, clip_capacity=8, device=dev)
    eager = DetectStage(cutr, vis, TU.SCANNET_CFG, B, 480, 640, SCANNET_K, **kw)
    graph = DetectStage(cutr, vis, TU.SCANNET_CFG, B, 480, 640, SCANNET_K, graph=True, **kw)
    for start in (0, 5, 9):
        fr = range(start, start + B)
        rgb = torch.from_numpy(np.stack([frame_rgbd(f)[0] for f in fr])).to(dev)
        depth = torch.from_numpy(np.stack([frame_rgbd(f)[1] for f in fr])).to(dev)
        poses = np.stack([Scene().pose(f) for f in fr])
        eager(rgb, depth, poses, return_instances=False)
        graph(rgb, depth, poses, return_instances=False)
        torch.cuda.synchronize()
        # library kernels (rocBLAS / hipBLASLt) may pick other algorithms under capture: ulps
        for a, b in zip(eager.last["clip"][3:], graph.last["clip"][3:]):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
        for ra, rb in zip(eager.last["res"], graph.last["res"]):
            torch.testing.assert_close(ra.scores, rb.scores, rtol=1e-4, atol=1e-6)
            torch.testing.assert_close(ra.pred_boxes_3d.tensor, rb.pred_boxes_3d.tensor, rtol=1e-4, atol=1e-4)


def test_fusion_stage_batched_keyframes(dev):
    """FusionStage.keyframes (world transform / projection / ids batched over 8 keyframes, then
    the serial association in the native sequencer) == the Python-driven keyframe() one at a
    time, bit for bit, over 48 keyframes."""
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.instances import Instances3D
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
    scene = Scene(seed=0)
    one = FusionStage(cfg, SCANNET_K, device=dev, native=False)
    bat = FusionStage(cfg, SCANNET_K, device=dev, native=True)
    for s0 in range(0, 48, 8):
        fr = list(range(s0, s0 + 8))
        dets = [scene.detections(f) for f in fr]
        for f, d in zip(fr, dets):
            one.keyframe(f, scene.pose(f), scene_instances(d, dev))
        preds = Instances3D.cat([scene_instances(d, dev) for d in dets])
        bat.keyframes(fr, np.stack([scene.pose(f) for f in fr]), preds, [len(d["scores"]) for d in dets])
        assert bat.box_manager.fusion_list == one.box_manager.fusion_list, f"step at {s0}"
        assert bat.box_manager.already_fusion == one.box_manager.already_fusion, f"step at {s0}"
        assert bat.box_manager.fusion_flag == one.box_manager.fusion_flag, f"step at {s0}"
        for a, b in zip(bat.boxes(), one.boxes()):
            np.testing.assert_array_equal(a, b, err_msg=f"step at {s0}")
    assert bat.stats == one.stats and bat.stats["fused"] > 5


@pytest.mark.parametrize("n_objects,batch", [(30, 8), (150, 16)])
def test_native_sequencer_equals_python_path(dev, n_objects, batch):
    """The library's keyframe sequencer (bf_fseq: one call per batch of keyframes) == the
    Python-driven state machine, bit for bit after every batch: fusion lists, fusion flags,
    fused sets, global boxes, valid_num, init_ids, per-row poses and the statistics, at the
    benchmark's 30-object scene and a 150-object one (lists, NMS and fusion jobs several times
    larger); then the stale last-frame re-entry (demo.py:200) on both."""
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.instances import Instances3D
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
    scene = Scene(seed=2, n_objects=n_objects)
    py = FusionStage(cfg, SCANNET_K, device=dev, native=False)
    nat = FusionStage(cfg, SCANNET_K, device=dev, native=True)
    for s0 in range(0, 6 * batch, batch):
        fr = list(range(s0, s0 + batch))
        dets = [scene.detections(f) for f in fr]
        if s0 == batch:            # a keyframe without boxes inside a batch
            dets[3] = {k: v[:0] for k, v in dets[3].items()}
        for f, d in zip(fr, dets):
            py.keyframe(f, scene.pose(f), scene_instances(d, dev))
        preds = Instances3D.cat([scene_instances(d, dev) for d in dets])
        nat.keyframes(fr, np.stack([scene.pose(f) for f in fr]), preds, [len(d["scores"]) for d in dets])
        msg = f"batch at {s0}"
        assert nat._mode == "native" and py._mode == "python"
        assert nat.box_manager.fusion_list == py.box_manager.fusion_list, msg
        assert nat.box_manager.fusion_flag == py.box_manager.fusion_flag, msg
        assert nat.box_manager.already_fusion == py.box_manager.already_fusion, msg
        assert nat.box_manager.num_record == py.box_manager.num_record, msg
        assert len(nat.box_manager.last_fusion_frame) == len(py.box_manager.last_fusion_frame), msg
        for a, b in zip(nat.boxes(), py.boxes()):
            np.testing.assert_array_equal(a, b, err_msg=msg)
        na, pa = nat.all_pred_box, py.all_pred_box
        for k in ("valid_num", "init_id", "scores", "pred_boxes", "frame_id"):
            np.testing.assert_array_equal(na.get(k).cpu().numpy(), pa.get(k).cpu().numpy(), err_msg=f"{k} {msg}")
        np.testing.assert_array_equal(nat.all_poses, py.all_poses, err_msg=msg)
        assert nat.stats == py.stats, msg
        assert nat.fuser.fit_calls == py.fuser.fit_calls and nat.box_count == py.box_count
    assert py.stats["fused"] >= 3 and py.stats["suppressed"] > 50
    last = 6 * batch + 3
    nat.finish(last, scene.pose(last), False)
    py.finish(last, scene.pose(last), False)
    assert nat.box_manager.fusion_list == py.box_manager.fusion_list
    assert nat.box_manager.already_fusion == py.box_manager.already_fusion
    for a, b in zip(nat.boxes(), py.boxes()):
        np.testing.assert_array_equal(a, b)
    assert nat.stats == py.stats


def test_native_sequencer_single_keyframe_stale_reentry(dev):
    """demo.py:200's re-entry after ONE keyframe: the reference's all_pred_box / per_frame_ins
    alias that keyframe's pred and are transformed again through it; the native stage hands
    over to the Python path there and matches it"""
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=25))
    scene = Scene(seed=4)
    st = {}
    for native in (True, False):
        s = FusionStage(cfg, SCANNET_K, device=dev, native=native)
        s.keyframe(0, scene.pose(0), scene_instances(scene.detections(0), dev))
        s.finish(9, scene.pose(9), False)
        st[native] = s
    assert st[True].box_manager.fusion_list == st[False].box_manager.fusion_list
    for a, b in zip(st[True].boxes(), st[False].boxes()):
        np.testing.assert_array_equal(a, b)
    assert st[True].stats == st[False].stats


@pytest.mark.gpu
def test_fusion_stage_joint_association(dev):
    """nms + correspondence association chained on the device (bf_corr_assoc_chained, one read-back)
    == the reference's two separate calls, bit for bit, over 64 gap=1 keyframes."""
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
    scene = Scene(seed=3)
    jnt = FusionStage(cfg, SCANNET_K, device=dev)
    sep = FusionStage(cfg, SCANNET_K, device=dev)
    jnt.joint, sep.joint = True, False
    for f in range(64):
        d = scene.detections(f)
        jnt.keyframe(f, scene.pose(f), scene_instances(d, dev))
        sep.keyframe(f, scene.pose(f), scene_instances(d, dev))
        assert jnt.box_manager.fusion_list == sep.box_manager.fusion_list, f"keyframe {f}"
        assert jnt.box_manager.fusion_flag == sep.box_manager.fusion_flag, f"keyframe {f}"
        for a, b in zip(jnt.boxes(), sep.boxes()):
            np.testing.assert_array_equal(a, b, err_msg=f"keyframe {f}")
    assert jnt.box_manager.already_fusion == sep.box_manager.already_fusion
    assert jnt.stats == sep.stats and jnt.stats["suppressed"] > 50


@pytest.mark.gpu
def test_instances_rows_gather(dev):
    """Instances3D.cat / integer-array indexing through bf_rows_gather (one launch over every
    field) == torch.cat / torch indexing per field, including empty sets and 1-row sets."""
    from boxfusion_amd import _lib
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from boxfusion_amd.instances import Instances3D
    g = torch.Generator().manual_seed(5)

    def make(n):
        p = Instances3D((480, 640))
        p.scores = torch.rand(n, generator=g).to(dev)
        p.pred_boxes_3d = GeneralInstance3DBoxes(torch.rand(n, 6, generator=g).to(dev),
                                                 torch.rand(n, 3, 3, generator=g).to(dev))
        p.cam_pose = torch.rand(n, 4, 4, generator=g).to(dev)
        p.init_id = torch.randint(0, 1000, (n,), generator=g).to(dev)
        return p
    for na, nb in [(7, 5), (0, 4), (3, 0), (1, 1), (40, 17)]:
        a, b = make(na), make(nb)
        c = Instances3D.cat([a, b])
        for k in ("scores", "cam_pose", "init_id"):
            torch.testing.assert_close(c.get(k), torch.cat([a.get(k), b.get(k)]), rtol=0, atol=0)
        torch.testing.assert_close(c.pred_boxes_3d.tensor,
                                   torch.cat([a.pred_boxes_3d.tensor, b.pred_boxes_3d.tensor]), rtol=0, atol=0)
        torch.testing.assert_close(c.pred_boxes_3d.R,
                                   torch.cat([a.pred_boxes_3d.R, b.pred_boxes_3d.R]), rtol=0, atol=0)
        if na + nb:
            idx = np.random.default_rng(na).integers(0, na + nb, na + nb + 3)
            s = c[idx]
            it = torch.from_numpy(idx).to(dev)
            for k in ("scores", "cam_pose", "init_id"):
                torch.testing.assert_close(s.get(k), c.get(k)[it], rtol=0, atol=0)
            torch.testing.assert_close(s.pred_boxes_3d.R, c.pred_boxes_3d.R[it], rtol=0, atol=0)
            s32 = c._device_rows([], it.to(torch.int32))          # int32 device index
            torch.testing.assert_close(s32.cam_pose, c.cam_pose[it], rtol=0, atol=0)
    # an out-of-range row is reported, not written
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    x = torch.arange(4, dtype=torch.float32, device=dev)
    out = torch.full((2,), -1.0, device=dev)
    f = (_lib.RowsField * 1)()
    f[0].a, f[0].b, f[0].dst, f[0].n_a, f[0].n_b, f[0].row_bytes = x.data_ptr(), None, out.data_ptr(), 4, 0, 4
    idx = torch.tensor([2, 9], dtype=torch.int64, device=dev)
    assert _lib.lib().bf_rows_gather(f, 1, _lib._ptr(idx), 0, 2, _lib._ptr(st), _lib._stream()) == 0
    assert out.tolist() == [2.0, -1.0] and int(st.item()) == _lib.BF_DEV_INDEX_RANGE


class _DemoDetect:
    """demo.py:135-171 per keyframe on this package: the scene's detections (what the golden's
    stand-in model returned), bf_detection_filter (demo.py:138-148), tools_utils.scale_boxes +
    text_prompt with the golden's stand-in CLIP (seeded features, one draw per call), CLIP score
    bump and the "" category filter"""

    B = 1

    def __init__(self, scene, keyframes, names, text, cfg, dev, clip_seed):
        self.scene, self.keyframes, self.calls = scene, keyframes, 0
        self.names, self.text, self.cfg, self.dev = names, text, cfg, dev
        self.clip_seed, self.clip_calls = clip_seed, 0

    def get_batch_images_clip_features(self, images):
        # the golden generator's StubCLIP.features (make_golden_demo.py)
        rng = np.random.default_rng(self.clip_seed + self.clip_calls)
        self.clip_calls += 1
        t = self.text_rows
        f = rng.normal(0, 1, (len(images), t.shape[1])).astype(np.float32)
        pick = rng.integers(0, len(t), len(images))
        near = np.arange(len(images)) % 4 != 3
        f[near] = t[pick[near]] * 30.0 + f[near] * 0.4
        return torch.from_numpy(f), None

    def preprocess_frames(self, depth, poses):
        """demo.py:121-131 on non-keyframes: bf_depth_preprocess (standardise + unproject)"""
        from boxfusion_amd import _lib
        from boxfusion_amd.synthetic import SCANNET_K
        n = depth.shape[0]
        K = torch.from_numpy(np.stack([SCANNET_K] * n)).to(self.dev)
        RT = torch.from_numpy(np.asarray(poses, np.float32)).to(self.dev)
        self.frames_done = getattr(self, "frames_done", 0) + n
        return _lib.depth_preprocess(depth, K, RT, 10.0)

    def __call__(self, rgb, depth, poses):
        from boxfusion_amd import _lib
        from boxfusion_amd.pipeline import scene_instances
        from boxfusion_amd.tools_utils import scale_boxes, text_prompt
        f = self.keyframes[self.calls]
        self.calls += 1
        det = self.cfg["detection"]
        p = scene_instances(self.scene.detections(f), self.dev)
        keep = _lib.detection_filter(p.scores, p.pred_proj_xy, p.pred_boxes_3d.tensor,
                                     _lib.filter_cfg(det, 640, 480))
        p = p[keep]
        if len(p):
            boxes = scale_boxes(p.pred_boxes.cpu().numpy(), 480, 640, scale=det["scale_box"])
            cats, feats, sims = text_prompt(boxes, self.names, self.text, rgb[0], self, None,
                                            det["class_sim_thres"])
            p.categories = cats
            p.features = feats
            p.scores = p.scores + self.cfg["box_fusion"]["clip_sim_coeff"] * sims / 100.0
            p = p[p.categories != ""]
        return [p]


def _assert_rerun_records(got, want):
    """FrameLogger records (visualize.Recording) vs the reference's recorded rerun.log calls"""
    import zlib
    assert len(got) == len(want), (len(got), len(want))
    for i, ((path, t, kind, a), w) in enumerate(zip(got, want)):
        msg = f"record {i}: {w['path']} {w['kind']}"
        assert (path, kind) == (w["path"], w["kind"]), msg
        assert list(t) == w["time"], msg
        if kind == "Transform3D":
            np.testing.assert_allclose(a["translation"], w["translation"], rtol=0, atol=1e-6, err_msg=msg)
            np.testing.assert_allclose(a["quaternion_xyzw"], w["quaternion_xyzw"], rtol=0, atol=1e-9, err_msg=msg)
        elif kind == "Pinhole":
            np.testing.assert_array_equal(np.asarray(a["image_from_camera"], np.float64), w["image_from_camera"], err_msg=msg)
            np.testing.assert_array_equal(np.asarray(a["resolution"], np.float64), w["resolution"], err_msg=msg)
        elif kind in ("Image", "DepthImage"):
            img = np.ascontiguousarray(a["image"])
            assert [list(img.shape), str(img.dtype), zlib.adler32(img.tobytes())] == \
                [w["shape"], w["dtype"], w["adler32"]], msg
        elif kind == "LineStrips3D":
            strip = np.asarray(a["strips"][0], np.float64).reshape(-1, 3)
            assert len(strip) == w["n"], msg
            np.testing.assert_allclose(strip.sum(), w["sum"], rtol=1e-12, atol=1e-9, err_msg=msg)
            np.testing.assert_array_equal(np.asarray(a["colors"], np.float64), w["colors"], err_msg=msg)
        elif kind == "Boxes3D":
            np.testing.assert_allclose(a["centers"], w["centers"], rtol=0, atol=1e-5, err_msg=msg)
            np.testing.assert_allclose(a["sizes"], w["sizes"], rtol=0, atol=1e-6, err_msg=msg)
            np.testing.assert_allclose(a["quaternions_xyzw"], w["quaternions_xyzw"], rtol=0, atol=1e-6, err_msg=msg)
            np.testing.assert_allclose(np.asarray(a["colors"], np.float64).reshape(-1, 3),
                                       np.asarray(w["colors"]).reshape(-1, 3), rtol=0, atol=1e-12, err_msg=msg)
            assert a["labels"] == w["labels"] and a["show_labels"] == w["show_labels"], msg


@pytest.mark.parametrize("native", [True, False])
def test_pipeline_run_vs_reference_demo_gap25(dev, native, monkeypatch):
    """Pipeline.run + FusionStage (keyframes every 25 frames, stale re-fusion of the non-keyframe
    last frame, demo.py:200) against the REFERENCE's own demo.py run() on the same stream
    (tests/golden/make_golden_demo.py): final fusion lists, fused sets and num_record equal; the
    global boxes (demo.py:371-379) and the framewise boxes / class indices / CLIP features
    (demo.py:382-386) equal.  World-space geometry as the reference computed it is injected by
    init_id (the particle search amplifies the 1-ulp difference of the GPU transform).  The
    reference's fusion kernel overruns convex_inter[8] in this run (d["hull_over"]): the match
    is with its control flow and the exact hull there (test_gpu_fusion.py's face-on fixture is
    the overrun-free pin)."""
    import copy
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import Pipeline, load_class_features, load_class_names
    from boxfusion_amd.synthetic import SCANNET_K, Scene, frame_rgbd
    d = TU.load("demo_gap25.npz")
    _inject_geometry(monkeypatch, dev, dict(tensor=d["geom_tensor"], R=d["geom_R"], proj=d["geom_proj"]))
    cfg = copy.deepcopy(TU.SCANNET_CFG)
    cfg["data"] = dict(gap=int(d["gap"]))
    cfg["detection"] = dict(score_thresh=0.5, uv_bound=True, uv_bound_value=0.9, floor_mask=True,
                            floor_ratio=15, scale_box=1.5, class_sim_thres=25.0, size_max_thres=None)
    cfg["box_fusion"] = dict(cfg["box_fusion"], clip_sim_coeff=1.0)
    scene = Scene(seed=int(d["scene_seed"]), period=int(d["scene_period"]))
    n, gap = int(d["n_frames"]), int(d["gap"])
    names = np.asarray(load_class_names())
    text = load_class_features()
    det = _DemoDetect(scene, [f for f in range(n) if f % gap == 0], names, text.to(dev), cfg, dev,
                      int(d["clip_seed"]))
    det.text_rows = text.numpy()
    fusion = FusionStage(cfg, SCANNET_K, device=dev, legacy_promotion=False, native=native)

    def frames(ids):
        rgb = np.stack([frame_rgbd(i)[0] for i in ids])
        depth = np.stack([frame_rgbd(i)[1] for i in ids])
        return (torch.from_numpy(rgb).to(dev), torch.from_numpy(depth).to(dev),
                np.stack([scene.pose(i) for i in ids]))

    from boxfusion_amd.visualize import FrameLogger, Recording
    rec = Recording(forward=False)
    # the golden run's vis config (make_golden_demo.cfg_demo): trajectory on, no class / id labels
    # shown; timestamps = frame index (the synthetic stream's meta timestamp); a --device cpu run,
    # so the logged depth carries the preprocessor's in-place NaN fill
    viz = FrameLogger(rec, SCANNET_K, (640, 480), K_depth=SCANNET_K, depth_size=(640, 480), fps=1.0,
                      show_class=False, show_label=False, depth_invalid_nan=True)
    pipe = Pipeline(det, fusion, gap)
    pipe.run(frames, n, viz=viz)
    assert pipe.frames_preprocessed == det.frames_done == n - len(range(0, n, gap))
    # f4: the REFERENCE's own rerun.log calls (demo.py:93-197, 329-330, tools/utils.py:37-96,
    # recorded by make_golden_demo.py) call by call: entity path, time, archetype and its fields
    _assert_rerun_records(rec.records, json.loads(str(d["rerun_json"])))
    poses = [a for p_, _, k, a in rec.records if p_ == "/world/image" and k == "Transform3D"]
    assert len(poses) == n
    # frame order (demo.py:108): the pose records are frames 0..n-1 in turn, so the trajectory
    # strip of the last frame is the positions of every frame before it
    trans = np.array([a["translation"] for a in poses])
    np.testing.assert_allclose(trans, np.stack([scene.pose(i)[:3, 3] for i in range(n)]), rtol=0, atol=1e-6)
    traj = rec.last("/world/trajectory")["strips"][0]
    np.testing.assert_allclose(traj, trans[:n - 1], rtol=0, atol=1e-6)
    boxes_logged = [a for p_, _, k, a in rec.records if p_ == "/device/wide/pred_instances"]
    assert len(boxes_logged) == len(range(0, n, gap)) + 1
    fin = fusion.all_pred_box
    np.testing.assert_array_equal(boxes_logged[-1]["centers"], fin.pred_boxes_3d.tensor[:, :3].cpu().numpy())
    assert boxes_logged[-1]["labels"] == [str(i) for i in range(len(fin))]
    bm = fusion.box_manager
    ragged = lambda flat, off: [flat[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
    assert bm.fusion_list == ragged(d["fusion_list_flat"], d["fusion_list_off"])
    assert bm.already_fusion == ragged(d["already_fusion_flat"], d["already_fusion_off"])
    assert sorted(bm.num_record) == d["num_record_frames"].tolist()
    assert [bm.num_record[k] for k in sorted(bm.num_record)] == d["num_record"].tolist()
    assert n - 1 in bm.num_record and (n - 1) % gap != 0        # the stale re-fusion ran
    g = fusion.all_pred_box.pred_boxes_3d.corners.cpu().numpy()
    np.testing.assert_array_equal(g, d["global_corners"])
    pf = fusion.per_frame_ins
    cls = np.array([list(names).index(c) for c in pf.categories])
    np.testing.assert_array_equal(cls, d["fw_class"])
    np.testing.assert_array_equal(pf.pred_boxes_3d.corners.cpu().numpy(), d["fw_corners"])
    np.testing.assert_allclose(pf.features.cpu().numpy(), d["fw_features"], rtol=1e-6, atol=1e-7)
    # the run holds fitness evaluations past the reference kernel's convex_inter[8] (recorded by
    # the generator): there the reference is undefined and both sides use the exact hull
    assert (fusion.fuser.hull_overflow_calls > 0) == bool(d["hull_over"].any())


def test_detect_stage_ca1m_depth_ratio(dev):
    """CA-1M-shaped detect stage (BASELINE configs[1]): 384x512 portrait frames with the depth map
    at half resolution (RGB:depth 2) -- the CuTR depth tokens on their own grid, back-projection
    with the depth intrinsics -- equals CuTREngine called directly on the same standardised depth"""
    from boxfusion_amd import _lib
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.pipeline import DetectStage
    from boxfusion_amd.sensor import camera_to_gravity
    from boxfusion_amd.synthetic import Scene
    K = np.array([[360.0, 0.0, 191.5], [0.0, 360.0, 255.5], [0.0, 0.0, 1.0]], np.float32)
    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(192, True).eval()
        vis = VisionTransformer(224, 14, 1280, 2, 16, 1024).eval()
    B, H, W = 2, 512, 384
    det = DetectStage(cutr, vis, TU.SCANNET_CFG, B, H, W, K, crop_source="top", crops_per_frame=4,
                      clip_capacity=8, device=dev, depth_ratio=2)
    g = torch.Generator(device=dev).manual_seed(5)
    rgb = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    depth = torch.rand((B, H // 2, W // 2), device=dev, generator=g) * 4 + 0.5
    poses = np.stack([Scene().pose(f) for f in range(B)])
    det(rgb, depth, poses, return_instances=False)
    torch.cuda.synchronize()
    xyz, valid = det.last["xyz"][0]
    assert xyz.shape == (H // 2, W // 2, 3) and valid.all()
    got = [(r.scores.clone(), r.pred_boxes_3d.tensor.clone()) for r in det.last["res"]]
    dstd, params = _lib.depth_standardize(depth)
    Kd = torch.from_numpy(np.stack([K] * B)).to(dev)
    Tg = torch.from_numpy(np.stack([camera_to_gravity(p) for p in poses])).to(dev)
    ref = det.cutr(rgb, dstd, params, Kd, Tg, [(H, W)] * B, K_host=np.stack([K] * B))
    for (sa, ba), b in zip(got, ref):
        assert torch.isfinite(sa).all() and torch.isfinite(ba).all()
        assert torch.equal(sa, b.scores)
        assert torch.equal(ba, b.pred_boxes_3d.tensor)
    assert torch.isfinite(det.last["clip"][3]).all()
