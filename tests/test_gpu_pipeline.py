"""The demo.py keyframe state machine (FusionStage) and the per-frame DetectStage on the GPU.

FusionStage is compared with the reference's recorded traces: discrete state (fusion lists,
already-fused lists, global box count) exactly; boxes within 1e-4 where fusion did not touch them.
Fused boxes depend chaotically on ulp-level differences of the projected view hulls (GPU
projection vs the reference's torch-CPU projection), so the trace replay in test_gpu_fusion.py,
which feeds the recorded projections, is where fused boxes are pinned bit-exact."""
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


@pytest.mark.parametrize("name", ["fusion_trace.npz", "fusion_trace_small.npz"])
def test_fusion_stage_vs_trace(dev, name):
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K
    t = TU.load(name)
    st = FusionStage(TU.SCANNET_CFG, SCANNET_K, device=dev, legacy_promotion=False)
    nd = t["n_det"]
    worst = 0.0
    for k, frame in enumerate(t["frame"]):
        a, b = int(nd[:k].sum()), int(nd[:k + 1].sum())
        det = {key: t["det_" + key][a:b] for key in ["scores", "pred_boxes", "xyzlhw", "R", "proj_xy"]}
        st.keyframe(int(frame), t["pose"][k], scene_instances(det, dev))
        got, _ = st.boxes()
        post = TU._rows(t, "post_tensor", k)
        assert st.box_manager.fusion_list == TU._lists(t, "post_fl", k), f"kf {k}"
        assert st.box_manager.already_fusion == TU._lists(t, "fused", k), f"kf {k}"
        assert got.shape == post.shape
        fused = np.zeros(len(post), bool)
        for i, fl in enumerate(st.box_manager.fusion_list):
            fused[i] = fl in st.box_manager.already_fusion
        np.testing.assert_allclose(got[~fused], post[~fused], rtol=0, atol=1e-4, err_msg=f"kf {k}")
        if fused.any():
            worst = max(worst, float(np.abs(got[fused] - post[fused]).max()))
    print("max fused-box deviation", name, worst)
    assert worst < 5e-2


def test_fusion_stage_vs_oracle_chain_gap1(dev):
    """40 consecutive keyframes (gap=1, the benchmark's regime) against oracle/chain.py."""
    from boxfusion_amd.box_fusion import load_pst
    from boxfusion_amd.fusion_stage import FusionStage
    from boxfusion_amd.pipeline import scene_instances
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    from oracle.chain import OracleChain
    cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
    scene = Scene(seed=0)
    st = FusionStage(cfg, SCANNET_K, device=dev)
    ch = OracleChain(cfg, SCANNET_K, pst=load_pst(), legacy=True)
    for f in range(40):
        d = scene.detections(f)
        st.keyframe(f, scene.pose(f), scene_instances(d, dev))
        ch.keyframe(f, scene.pose(f), d)
        assert st.box_manager.fusion_list == ch.fusion_list, f"frame {f}"
        assert len(st.all_pred_box) == len(ch.g["tensor"])
    got, _ = st.boxes()
    print("gap1 fused", len(ch.already_fusion), "max dev", np.abs(got - ch.g["tensor"]).max())
    assert len(ch.already_fusion) > 5


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
