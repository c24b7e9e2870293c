"""HIP fusion path vs the reference (golden traces) and vs the CPU oracle (seeded inputs).
Runs only on a HIP device."""
import numpy as np
import pytest
import torch

from oracle import oracle as OR
from tests import trace_util as TU

pytestmark = pytest.mark.gpu

DEV = "cuda"
CAP = 64


def _t(a, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV, dtype)


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    return _lib


def nms_cfg(L, cap=CAP, cfg=TU.SCANNET_CFG):
    c = L.NmsCfg()
    c.iou_threshold = cfg["box_fusion"]["nms_threshold"]
    c.translation_gap = cfg["association"]["translation_gap"]
    c.rotation_gap = cfg["association"]["rotation_gap"]
    c.center_gap = 0.5
    c.max_list = 5
    c.list_capacity = cap
    return c


def corr_cfg(L, cap=CAP, cfg=TU.SCANNET_CFG, W=640, H=480):
    c = L.CorrCfg()
    c.small_size = cfg["box_fusion"]["small_size"]
    c.threshold = cfg["association"]["small_threshold"]
    c.translation_gap = cfg["association"]["translation_gap"]
    c.rotation_gap = cfg["association"]["rotation_gap"]
    c.W, c.H = float(W), float(H)
    c.max_list = 5
    c.list_capacity = cap
    return c


def fuse_cfg(L, legacy, cfg=TU.SCANNET_CFG, K=TU.SCANNET_K, H=480, W=640):
    o = OR.fuse_cfg(cfg, np.eye(4), H, W, legacy=legacy)
    c = L.FuseCfg()
    for name, _ in L.FuseCfg._fields_:
        if name == "K":
            K4 = np.eye(4, dtype=np.float32)
            K4[:3, :3] = K
            for i in range(16):
                c.K[i] = float(K4.reshape(-1)[i])
        else:
            setattr(c, name, getattr(o, name))
    return c


class HipBackend:
    def __init__(self, L, legacy=False, cfg=TU.SCANNET_CFG, K=TU.SCANNET_K, H=480, W=640):
        self.L = L
        self.pst = _t(np.load(TU.GOLDEN + "/../../boxfusion_amd/data/pst_1024_0.npy"))
        self.fcfg = fuse_cfg(L, legacy, cfg, K, H, W)
        self.ncfg, self.ccfg = nms_cfg(L, cfg=cfg), corr_cfg(L, cfg=cfg, W=W, H=H)

    def corners(self, tensor, R):
        return self.L.box_corners(_t(tensor), _t(R)).cpu().numpy()

    def iou_matrix(self, corners):
        return self.L.obb_iou_matrix(_t(corners)).cpu().numpy()

    def nms(self, iou, corners, scores, init_id, cam_poses, fusion_list, valid_num):
        items, lens = OR.pack_lists(fusion_list, CAP)
        it, ln, vn = _t(items, torch.int32), _t(lens, torch.int32), _t(valid_num)
        keep, succ, ev, cnt = self.L.nms_scan(_t(iou, torch.float64), _t(corners), _t(scores),
                                              _t(init_id, torch.int32), _t(cam_poses), it, ln, vn,
                                              self.ncfg)
        c = cnt.cpu().numpy()
        assert c[3] == 0
        return dict(keep=keep.cpu().numpy()[:c[0]], success=succ.cpu().numpy()[:c[1]],
                    events=ev.cpu().numpy()[:c[2]],
                    fusion_list=OR.unpack_lists(it.cpu().numpy(), ln.cpu().numpy(),
                                                len(fusion_list)),
                    valid_num=vn.cpu().numpy())

    def corr(self, corners, dims, scores, boxes2d, init_id, cam_poses, pose, K, n_glo, keep,
             success, fusion_list, valid_num):
        items, lens = OR.pack_lists(fusion_list, CAP)
        it, ln, vn = _t(items, torch.int32), _t(lens, torch.int32), _t(valid_num)
        k, ev, cnt = self.L.corr_assoc(_t(corners), _t(dims), _t(scores), _t(boxes2d),
                                       _t(init_id, torch.int32), _t(cam_poses), _t(pose), _t(K),
                                       n_glo, _t(keep, torch.int32), _t(success, torch.int32),
                                       it, ln, vn, self.ccfg)
        c = cnt.cpu().numpy()
        assert c[2] == 0
        return dict(keep=k.cpu().numpy()[:c[0]],
                    fusion_list=OR.unpack_lists(it.cpu().numpy(), ln.cpu().numpy(),
                                                len(fusion_list)),
                    valid_num=vn.cpu().numpy())

    def fuse(self, views):
        nv = [len(v[2]) for v in views]
        off = np.concatenate([[0], np.cumsum(nv)[:-1]]).astype(np.int32)
        cat = [np.concatenate([v[k] for v in views], 0) for k in range(5)]
        box, upd, it, st, _ = self.L.fusion_fit(_t(off, torch.int32), _t(nv, torch.int32),
                                                _t(cat[0]), _t(cat[1]), _t(cat[2]), _t(cat[3]),
                                                _t(cat[4]), self.pst, self.fcfg)
        b, u = box.cpu().numpy(), upd.cpu().numpy()
        self._over = getattr(self, "_over", False) | bool(int(st.item()) & self.L.BF_DEV_HULL_OVERFLOW)
        assert not int(st.item()) & self.L.BF_DEV_HULL_TRUNC
        return [(b[i], int(u[i])) for i in range(len(views))]

    def hull_overflow(self):
        o, self._over = getattr(self, "_over", False), False
        return o


@pytest.mark.parametrize("name", TU.TRACES)
def test_trace_replay_hip(L, name):
    """NMS keep/success, fusion lists, association and fused boxes bit-exact vs the reference
    (ScanNet scene traces, the CA-1M trace at ca1m.yaml thresholds on 384 x 512 portrait frames,
    and the overrun-free face-on trace, reference-pinned at every keyframe)."""
    t = TU.load(name)
    stats = TU.replay(t, HipBackend(L, False, *TU.trace_setup(t)))
    print(name, stats)
    assert stats["fused"] >= 10 and stats["reference_pinned"] >= 1
    if "faceon" in name:
        assert stats["reference_pinned"] == stats["keyframes"] and stats["hull_overflow_keyframes"] == 0


def test_faceon_fusion_reference_pinned(L):
    """BoxFusion.boxfusion (bf_fusion_fit + bf_fusion_writeback) against the reference's own
    boxfusion on the face-on jobs where no fitness evaluation overruns the reference kernel's
    buffers (tests/golden/make_golden.gen_faceon): fused boxes and already_fusion bit for bit,
    with strict_hull on (any BF_DEV_HULL_OVERFLOW would raise)"""
    import copy
    from boxfusion_amd.box_fusion import BoxFusion
    from boxfusion_amd.box_manager import BoxManager
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from boxfusion_amd.instances import Instances3D
    from tests.test_oracle_golden import faceon_jobs
    g = TU.load("fusion_faceon.npz")
    lists, _ = faceon_jobs(g)
    cfg = copy.deepcopy(TU.SCANNET_CFG)
    cfg["box_fusion"]["strict_hull"] = True
    pf = Instances3D((480, 640))
    pf.pred_boxes_3d = GeneralInstance3DBoxes(_t(g["pf_tensor"]), _t(g["pf_R"]))
    pf.scores = _t(g["pf_scores"])
    pf.cam_pose = _t(g["pf_pose"])
    pf.projected_boxes = _t(g["pf_proj"])
    rows = g["glob_rows"]
    allb = Instances3D((480, 640))
    allb.pred_boxes_3d = GeneralInstance3DBoxes(_t(g["pf_tensor"][rows]), _t(g["pf_R"][rows]))
    bm = BoxManager(cfg)
    bm.init_new_predictions(len(rows), 0)
    bm.fusion_list = [[int(i) for i in ls] for ls in lists]
    bf = BoxFusion(cfg, device=DEV, legacy_promotion=False)
    bf.update_intrinsics((640, 480), np.array(fuse_cfg(L, False).K).reshape(4, 4)[:3, :3])
    bf.boxfusion(allb, pf, bm)
    np.testing.assert_array_equal(g["before"], g["pf_tensor"][rows])
    np.testing.assert_array_equal(allb.pred_boxes_3d.tensor.cpu().numpy(), g["after"])
    want = [[int(v) for v in g["fused_flat"][g["fused_off"][k]:g["fused_off"][k + 1]]]
            for k in range(len(g["fused_off"]) - 1)]
    assert bm.already_fusion == want
    assert bf.hull_overflow_calls == 0 and bf.last_stats["updated"] == len(lists)


def test_obb_iou_pairs_hip(L):
    g = TU.load("obb_pairs.npz")
    c = g["corners"].reshape(-1, 8, 3)
    iou = L.obb_iou_matrix(_t(c)).cpu().numpy()
    got = np.array([iou[2 * k, 2 * k + 1] for k in range(len(g["iou"]))])
    np.testing.assert_array_equal(got, g["iou"])
    np.testing.assert_array_equal(iou, iou.T)


def test_obb_iou_matrix_vs_oracle_large(L):
    rng = np.random.default_rng(7)
    n = 160
    xyz = rng.uniform(-2, 2, (n, 3))
    xyz[n // 2:] = xyz[:n // 2] + rng.normal(0, 0.1, (n // 2, 3))
    b = np.concatenate([xyz, rng.uniform(0.1, 1.0, (n, 3))], 1).astype(np.float32)
    yaw = rng.uniform(-np.pi, np.pi, n)
    R = np.stack([[[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]]
                  for a in yaw]).astype(np.float32)
    corners = OR.box_corners(b, R)
    np.testing.assert_array_equal(L.box_corners(_t(b), _t(R)).cpu().numpy(), corners)
    ref = OR.obb_iou_matrix(corners)
    got = L.obb_iou_matrix(_t(corners)).cpu().numpy()
    assert (ref[np.triu_indices(n, 1)] > 0).sum() > 50
    np.testing.assert_array_equal(got, ref)


def test_obb_iou_matrix_vs_oracle_tilted(L):
    """Fully 3-D rotations (every facet plane has a z component, so the column form's binary
    searches run on prefixes and suffixes), plus axis-aligned boxes that share faces or are
    repeated (grid points exactly on a facet), flat boxes (a zero extent: zero z step) and
    tiny ones: bit-exact vs the oracle's point-by-point count."""
    rng = np.random.default_rng(11)
    n = 120
    xyz = rng.uniform(-1.5, 1.5, (n, 3))
    xyz[n // 2:] = xyz[:n // 2] + rng.normal(0, 0.15, (n // 2, 3))
    size = rng.uniform(0.1, 1.2, (n, 3))
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    R = np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
                  np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
                  np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], 1)
    # axis-aligned face-sharing neighbours, exact repeats, flat and tiny boxes
    R[:24] = np.eye(3)
    xyz[:8] = np.array([[0.25 * k, 0.0, 0.0] for k in range(8)])
    size[:8] = np.array([0.25, 0.5, 0.5])
    xyz[8:12], size[8:12] = xyz[:4], size[:4]
    size[12:16, 2] = 0.0
    size[16:20] *= 1e-3
    xyz[12:20] = xyz[:8] + 0.01
    b = np.concatenate([xyz, size], 1).astype(np.float32)
    R = R.astype(np.float32)
    corners = OR.box_corners(b, R)
    np.testing.assert_array_equal(L.box_corners(_t(b), _t(R)).cpu().numpy(), corners)
    ref = OR.obb_iou_matrix(corners)
    got = L.obb_iou_matrix(_t(corners)).cpu().numpy()
    assert (ref[np.triu_indices(n, 1)] > 0).sum() > 50
    np.testing.assert_array_equal(got, ref)


def test_fusion_legacy_promotion_vs_oracle(L):
    """numpy-1.26 (pinned) promotion mode: f64 host scalars, bit-exact vs the oracle."""
    t = TU.load("fusion_trace_small.npz")
    be = HipBackend(L, legacy=True)
    ocfg = OR.fuse_cfg(TU.SCANNET_CFG, np.array(be.fcfg.K).reshape(4, 4), 480, 640, legacy=True)
    pst = np.load(TU.GOLDEN + "/../../boxfusion_amd/data/pst_1024_0.npy")
    views = []
    for kf in TU.keyframes(t):
        for _, fl in kf.fusion_jobs():
            idx = np.asarray(fl)
            pf = kf.per_frame
            views.append((pf["tensor"][idx], pf["R"][idx], pf["scores"][idx], pf["pose"][idx],
                          pf["proj"][idx]))
    got = be.fuse(views)
    n_upd = 0
    for v, (box, upd) in zip(views, got):
        r = OR.fusion_fit(*v, pst, ocfg)
        assert upd == r["updated"]
        np.testing.assert_array_equal(box, r["box"])
        n_upd += upd
    assert n_upd > 10


def test_fitness_single_vs_oracle(L):
    t = TU.load("fusion_trace.npz")
    pf = dict(tensor=t["pf_tensor"], R=t["pf_R"], pose=t["pf_pose"], proj=t["pf_proj"])
    idx = np.arange(4)
    be = HipBackend(L)
    ss = np.array([0.1, 0.1, 0.1, 0.5, 0.5, 0.5], np.float32)
    box = pf["tensor"][0]
    got = L.fusion_fitness(_t(box), _t(pf["R"][0]), _t(pf["pose"][idx]), _t(pf["proj"][idx]),
                           be.pst, _t(ss), be.fcfg).cpu().numpy()
    ocfg = OR.fuse_cfg(TU.SCANNET_CFG, np.array(be.fcfg.K).reshape(4, 4), 480, 640)
    ref = OR.fitness(box, pf["R"][0], pf["pose"][idx], pf["proj"][idx], be.pst.cpu().numpy(), ss,
                     ocfg)
    np.testing.assert_array_equal(got, ref)


def test_geometry_vs_golden(L):
    g = TU.load("geometry.npz")
    np.testing.assert_array_equal(L.box_corners(_t(g["xyzlhw"]), _t(g["R"])).cpu().numpy(),
                                  g["corners_cam"])
    b, R = _t(g["xyzlhw"]), _t(g["R"])
    L.box_transform2world(b, R, _t(g["poses"]))
    np.testing.assert_allclose(b.cpu().numpy(), g["world_tensor"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(R.cpu().numpy(), g["world_R"], rtol=0, atol=2e-6)
    c = L.box_corners(b, R)
    K = _t(np.array([[574.540771, 0, 322.522827], [0, 577.583740, 238.558853], [0, 0, 1]]))
    uv = L.project_boxes(c, _t(g["poses"]), K, 640.0, 480.0).cpu().numpy()
    np.testing.assert_allclose(uv, g["projected"], rtol=0, atol=2e-3)


def test_depth_standardize_vs_golden_and_oracle(L):
    g = TU.load("depth.npz")
    out, params = L.depth_standardize(_t(g["depth"]))
    out, params = out.cpu().numpy(), params.cpu().numpy()
    np.testing.assert_allclose(params, g["params"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(out, g["out"], rtol=0, atol=3e-6)
    from boxfusion_amd.synthetic import frame_rgbd
    d = np.stack([frame_rgbd(f)[1] for f in range(3)])
    o2, p2 = L.depth_standardize(_t(d))
    for i in range(3):
        ro, rp = OR.depth_standardize(d[i])
        np.testing.assert_allclose(p2.cpu().numpy()[i], rp, rtol=1e-6)
        np.testing.assert_allclose(o2.cpu().numpy()[i], ro, rtol=0, atol=2e-6)


def test_backproject_vs_oracle(L):
    from boxfusion_amd.synthetic import frame_rgbd, Scene, SCANNET_K
    d = frame_rgbd(3)[1]
    RT = Scene().pose(3)
    xyz, valid = L.backproject(_t(d), _t(SCANNET_K), _t(RT), 10.0)
    rx, rv = OR.backproject(d, SCANNET_K, RT, 10.0)
    np.testing.assert_array_equal(valid.cpu().numpy(), rv)
    np.testing.assert_allclose(xyz.cpu().numpy(), rx, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("b,h,w", [(3, 480, 640), (2, 36, 64), (2, 37, 53), (5, 192, 256)])
def test_depth_preprocess_backprojection_equals_backproject(L, b, h, w):
    """bf_depth_preprocess's fused back-projection (xyz staged per wave in LDS, partial waves when
    h*w is not a multiple of 256, the scalar path when it is not a multiple of 4) == bf_backproject
    frame by frame, bit for bit; its standardisation == bf_depth_standardize"""
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    g = torch.Generator(device="cuda").manual_seed(h * w + b)
    d = torch.rand(b, h, w, device="cuda", generator=g) * 6.0
    d[:, ::7, ::5] = 0.0
    d[:, 1, :] = 11.0                                   # past max_depth
    K = torch.tensor(SCANNET_K, device="cuda").expand(b, 3, 3).contiguous()
    RT = torch.stack([torch.tensor(Scene().pose(f), device="cuda") for f in range(b)]).float()
    out, params, xyz, valid = L.depth_preprocess(d, K, RT, 10.0)
    o2, p2 = L.depth_standardize(d)
    assert torch.equal(out, o2) and torch.equal(params, p2)
    for f in range(b):
        x1, v1 = L.backproject(d[f], K[f], RT[f], 10.0)
        assert torch.equal(xyz[f], x1)
        assert torch.equal(valid[f].to(torch.uint8), v1.to(torch.uint8))


def _hexagon_views(n_views=3, twist_deg=14.0):
    """a box seen obliquely (projected hull = hexagon) in n views, each view's observed corners =
    the box's own projection twisted about its centroid: the intersection of the two hexagons has
    12 vertices, more than the reference kernel's convex_inter[8] (box_fusion.py:381-384)"""
    from boxfusion_amd.synthetic import SCANNET_K, look_at_pose
    box = np.array([0.0, 0.0, 0.5, 0.8, 0.6, 0.7], np.float32)
    R = np.eye(3, dtype=np.float32)
    poses, tcs = [], []
    K = SCANNET_K.astype(np.float64)
    c = OR.box_corners(box[None], R[None])[0].astype(np.float64)
    for v in range(n_views):
        a = 0.6 + 0.4 * v
        P = look_at_pose([2.5 * np.cos(a), 2.5 * np.sin(a), 1.8], [0.0, 0.0, 0.5]).astype(np.float64)
        cam = (np.linalg.inv(P) @ np.c_[c, np.ones(8)].T).T[:, :3]
        uv = np.stack([K[0, 0] * cam[:, 0] / cam[:, 2] + K[0, 2], K[1, 1] * cam[:, 1] / cam[:, 2] + K[1, 2]], 1)
        m = uv.mean(0)
        t = np.deg2rad(twist_deg)
        Rt = np.array([[np.cos(t), -np.sin(t)], [np.sin(t), np.cos(t)]])
        tcs.append(((uv - m) @ Rt.T + m).astype(np.float32))
        poses.append(P.astype(np.float32))
    n = n_views
    return (np.repeat(box[None], n, 0), np.repeat(R[None], n, 0), np.linspace(0.9, 0.7, n).astype(np.float32),
            np.stack(poses), np.stack(tcs))


@pytest.mark.parametrize("legacy", [True, False])
def test_fusion_hull_overflow_flag_and_exact_hull(L, legacy):
    """an input whose intersection hull exceeds the reference's 8-point buffer sets
    BF_DEV_HULL_OVERFLOW, and the kernel still matches the oracle (exact hull) bit for bit"""
    vb, vr, vs, vp, vt = _hexagon_views()
    be = HipBackend(L, legacy=legacy)
    nv = len(vs)
    off, cnt = _t(np.array([0], np.int32), torch.int32), _t(np.array([nv], np.int32), torch.int32)
    out, upd, it, status, _ = L.fusion_fit(off, cnt, _t(vb), _t(vr), _t(vs), _t(vp), _t(vt), be.pst,
                                           be.fcfg, max_views=nv)
    assert int(status.item()) & L.BF_DEV_HULL_OVERFLOW
    ocfg = OR.fuse_cfg(TU.SCANNET_CFG, np.array(be.fcfg.K).reshape(4, 4), 480, 640, legacy=legacy)
    r = OR.fusion_fit(vb, vr, vs, vp, vt, be.pst.cpu().numpy(), ocfg)
    assert int(upd.item()) == r["updated"]
    np.testing.assert_array_equal(out.cpu().numpy()[0], r["box"])


def test_boxfusion_hull_overflow_policy(L):
    """BoxFusion counts the overflow (warning once) by default and raises with strict_hull"""
    import copy
    import warnings
    from boxfusion_amd.box_fusion import BoxFusion
    from boxfusion_amd.box_manager import BoxManager
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from boxfusion_amd.instances import Instances3D
    vb, vr, vs, vp, vt = _hexagon_views()
    for strict in (False, True):
        cfg = copy.deepcopy(TU.SCANNET_CFG)
        cfg["box_fusion"]["strict_hull"] = strict
        pf = Instances3D((480, 640))
        pf.pred_boxes_3d = GeneralInstance3DBoxes(_t(vb), _t(vr))
        pf.scores = _t(vs)
        pf.cam_pose = _t(vp)
        pf.projected_boxes = _t(vt)
        allb = Instances3D((480, 640))
        allb.pred_boxes_3d = GeneralInstance3DBoxes(_t(vb[:1]), _t(vr[:1]))
        bm = BoxManager(cfg)
        bm.init_new_predictions(1, 0)
        bm.fusion_list = [[0, 1, 2]]
        bf = BoxFusion(cfg, device=DEV)
        bf.update_intrinsics((640, 480), np.array(fuse_cfg(L, True).K).reshape(4, 4)[:3, :3])
        if strict:
            with pytest.raises(L.HipError, match="HULL_OVERFLOW"):
                bf.boxfusion(allb, pf, bm)
        else:
            from boxfusion_amd import box_fusion as BFM
            BFM._HULL_WARNED[0] = False
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                bf.boxfusion(allb, pf, bm)
                bm.fusion_list = [[0, 1, 2]]
                bm.already_fusion = []
                bf.boxfusion(allb, pf, bm)        # counted again, not warned again
            assert bf.hull_overflow_calls == 2
            assert sum("convex_inter[8]" in str(x.message) for x in w) == 1


@pytest.mark.parametrize("n_glo,n_new", [(150, 25), (97, 0), (300, 40)])
def test_nms_scan_large_vs_oracle(L, n_glo, n_new):
    """the greedy scan + record() with more than 96 boxes (the 256-thread k_nms_scan of the
    default build; <= 96 runs the one-wave form): ~150 global boxes plus a keyframe's new ones,
    clustered so that suppressions, list merges (up to 5 views) and pose gates all occur;
    keep / success / events / fusion lists / valid_num bit-exact against the oracle"""
    from boxfusion_amd.synthetic import Scene
    rng = np.random.default_rng(n_glo + n_new)
    n = n_glo + n_new
    centres = rng.uniform(-2.5, 2.5, (n // 3 + 1, 3))
    xyz = centres[rng.integers(0, len(centres), n)] + rng.normal(0, 0.04, (n, 3))
    lhw = rng.uniform(0.2, 0.9, (n, 3))
    b = np.concatenate([xyz, lhw], 1).astype(np.float32)
    yaw = rng.uniform(-0.2, 0.2, n)
    R = np.stack([[[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]]
                  for a in yaw]).astype(np.float32)
    corners = OR.box_corners(b, R)
    scores = rng.permutation(np.linspace(0.3, 0.99, n)).astype(np.float32)
    init_id = np.arange(n, dtype=np.int32)
    scene = Scene(seed=1)
    cam_poses = np.stack([scene.pose(int(f)) for f in rng.integers(0, 1000, n)]).astype(np.float32)
    # global boxes carry earlier merges (lists of up to 4 views), the new ones their own id
    fusion_list = [sorted(set([i] + rng.integers(0, n_glo, rng.integers(0, 4)).tolist())) if i < n_glo
                   else [i] for i in range(n)]
    valid_num = rng.integers(0, 3, n).astype(np.float32)
    iou = L.obb_iou_matrix(_t(corners)).cpu().numpy()
    assert (iou[np.triu_indices(n, 1)] > 0.1).sum() > n // 4
    got = HipBackend(L).nms(iou, corners, scores, init_id, cam_poses, fusion_list, valid_num)
    ref = OR.nms_scan(iou, corners, scores, init_id, cam_poses, fusion_list, valid_num, nms_cfg(L))
    assert ref["status"] == 0
    for k in ("keep", "success", "events", "valid_num"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert got["fusion_list"] == ref["fusion_list"]
    assert len(ref["success"]) > 10 and len(ref["events"]) > 10


@pytest.mark.parametrize("n", [40, 130])
def test_nms_scan_input_list_longer_than_capacity(L, n):
    """an input fusion-list length above the row capacity (a caller error) raises the overflow status
    bit instead of reading / writing past the row, in the one-wave scan at n <= 96 and the bit-mask
    scan above it (bf_nms_scan_ws)"""
    rng = np.random.default_rng(n)
    b = np.concatenate([rng.uniform(-3, 3, (n, 3)), rng.uniform(0.2, 0.6, (n, 3))], 1).astype(np.float32)
    R = np.repeat(np.eye(3, dtype=np.float32)[None], n, 0)
    corners = _t(OR.box_corners(b, R))
    dev = corners.device
    cap = 8
    items = torch.full((n, cap), -1, dtype=torch.int32, device=dev)
    items[:, 0] = torch.arange(n, dtype=torch.int32, device=dev)
    lens = torch.ones(n, dtype=torch.int32, device=dev)
    lens[n // 2] = cap + 5                                   # longer than the row
    cfg = nms_cfg(L, cap=cap)
    iou = L.obb_iou_matrix(corners)
    scores = torch.from_numpy(rng.uniform(0.3, 0.9, n).astype(np.float32)).to(dev)
    init_id = torch.arange(n, dtype=torch.int32, device=dev)
    poses = torch.from_numpy(np.repeat(np.eye(4, dtype=np.float32)[None], n, 0)).to(dev)
    vn = torch.zeros(n, device=dev)
    keep, succ, events, counts = L.nms_scan(iou, corners, scores, init_id, poses, items, lens, vn, cfg)
    torch.cuda.synchronize()
    assert int(counts[3]) & L.BF_DEV_FUSION_LIST_OVERFLOW


@pytest.mark.parametrize("n_glo,n_new", [(1, 0), (0, 1), (1, 1), (2, 1), (94, 1), (95, 1), (96, 1), (90, 7)])
def test_nms_scan_small_and_boundary_vs_oracle(L, n_glo, n_new):
    """the IoU matrix + greedy scan at the smallest counts and around the 96-box switch between
    the one-wave scan and the block scan: bit-exact against the oracle"""
    from boxfusion_amd.synthetic import Scene
    rng = np.random.default_rng(1000 + 17 * n_glo + n_new)
    n = n_glo + n_new
    centres = rng.uniform(-2.0, 2.0, (max(1, n // 3), 3))
    xyz = centres[rng.integers(0, len(centres), n)] + rng.normal(0, 0.04, (n, 3))
    b = np.concatenate([xyz, rng.uniform(0.2, 0.9, (n, 3))], 1).astype(np.float32)
    yaw = rng.uniform(-0.2, 0.2, n)
    R = np.stack([[[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]]
                  for a in yaw]).astype(np.float32)
    corners = OR.box_corners(b, R)
    scores = rng.permutation(np.linspace(0.3, 0.99, n)).astype(np.float32)
    init_id = np.arange(n, dtype=np.int32)
    scene = Scene(seed=2)
    cam_poses = np.stack([scene.pose(int(f)) for f in rng.integers(0, 1000, n)]).astype(np.float32)
    fusion_list = [sorted(set([i] + rng.integers(0, max(1, n_glo), rng.integers(0, 3)).tolist()))
                   if i < n_glo else [i] for i in range(n)]
    valid_num = rng.integers(0, 3, n).astype(np.float32)
    iou = L.obb_iou_matrix(_t(corners)).cpu().numpy()
    np.testing.assert_array_equal(iou, OR.obb_iou_matrix(corners))
    got = HipBackend(L).nms(iou, corners, scores, init_id, cam_poses, fusion_list, valid_num)
    ref = OR.nms_scan(iou, corners, scores, init_id, cam_poses, fusion_list, valid_num, nms_cfg(L))
    assert ref["status"] == 0
    for k in ("keep", "success", "events", "valid_num"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert got["fusion_list"] == ref["fusion_list"]
