"""Pin the CPU oracle against the reference's own outputs (golden fixtures made by
tests/golden/make_golden.py, which runs the reference code).  CPU only."""
import numpy as np
import pytest

from oracle import oracle as OR
from tests import trace_util as TU


def test_obb_iou_pairs_exact():
    g = TU.load("obb_pairs.npz")
    got = np.array([OR.obb_iou(c[0], c[1]) for c in g["corners"]])
    assert (g["iou"] > 0).sum() > 100
    np.testing.assert_array_equal(got, g["iou"])


def test_corners_exact():
    g = TU.load("geometry.npz")
    np.testing.assert_array_equal(OR.box_corners(g["xyzlhw"], g["R"]), g["corners_cam"])
    np.testing.assert_array_equal(OR.box_corners(g["world_tensor"], g["world_R"]),
                                  g["corners_world"])


def test_depth_standardize():
    g = TU.load("depth.npz")
    for i in range(len(g["depth"])):
        out, params = OR.depth_standardize(g["depth"][i])
        np.testing.assert_allclose(params, g["params"][i], rtol=2e-6, atol=1e-6)
        np.testing.assert_allclose(out, g["out"][i], rtol=0, atol=2e-6)


def nms_cfg(cap=64, cfg=TU.SCANNET_CFG):
    c = OR.NmsCfg()
    c.iou_threshold = cfg["box_fusion"]["nms_threshold"]
    c.translation_gap = cfg["association"]["translation_gap"]
    c.rotation_gap = cfg["association"]["rotation_gap"]
    c.center_gap = 0.5
    c.max_list = 5
    c.list_capacity = cap
    return c


def corr_cfg(cap=64, cfg=TU.SCANNET_CFG, W=640, H=480):
    c = OR.CorrCfg()
    c.small_size = cfg["box_fusion"]["small_size"]
    c.threshold = cfg["association"]["small_threshold"]
    c.translation_gap = cfg["association"]["translation_gap"]
    c.rotation_gap = cfg["association"]["rotation_gap"]
    c.W, c.H = float(W), float(H)
    c.max_list = 5
    c.list_capacity = cap
    return c


class OracleBackend:
    def __init__(self, cfg=TU.SCANNET_CFG, K=TU.SCANNET_K, H=480, W=640):
        self.pst = np.load(TU.GOLDEN + "/../../boxfusion_amd/data/pst_1024_0.npy")
        K4 = np.eye(4, dtype=np.float32)
        K4[:3, :3] = K
        self.fcfg = OR.fuse_cfg(cfg, K4, H, W, legacy=False)
        self.ncfg, self.ccfg = nms_cfg(cfg=cfg), corr_cfg(cfg=cfg, W=W, H=H)

    corners = staticmethod(OR.box_corners)
    iou_matrix = staticmethod(OR.obb_iou_matrix)

    def nms(self, *a):
        return OR.nms_scan(*a, self.ncfg)

    def corr(self, *a):
        return OR.corr_assoc(*a, self.ccfg)

    def fuse(self, views):
        out = []
        for v in views:
            r = OR.fusion_fit(*v, self.pst, self.fcfg)
            out.append((r["box"], r["updated"]))
        return out

    def hull_overflow(self):
        return any(OR.hull_overflow(reset=True))


@pytest.mark.parametrize("name", TU.TRACES)
def test_trace_replay(name):
    t = TU.load(name)
    stats = TU.replay(t, OracleBackend(*TU.trace_setup(t)))
    print(name, stats)
    assert stats["fused"] >= 10
    if "faceon" in name:
        # overrun-free end to end: every keyframe pinned to the reference outright
        assert stats["hull_overflow_keyframes"] == 0
        assert stats["reference_pinned"] == stats["keyframes"] == len(t["frame"]) - 1
        assert stats["corr_changes"] >= 2 and stats["suppressions"] >= 16
    else:
        assert stats["reference_pinned"] >= 1 and stats["hull_overflow_keyframes"] > 0
        assert stats["suppressions"] > 100
    if "small" in name:
        assert stats["corr_changes"] > 5


def faceon_jobs(g):
    """the face-on fusion fixture's jobs: (views of job k, global row before, after)"""
    lists = [g["lists_flat"][g["lists_off"][k]:g["lists_off"][k + 1]] for k in range(len(g["lists_off"]) - 1)]
    views = [(g["pf_tensor"][i], g["pf_R"][i], g["pf_scores"][i], g["pf_pose"][i], g["pf_proj"][i])
             for i in lists]
    return lists, views


def test_faceon_fusion_reference_pinned():
    """box fusion against the reference with NO buffer overrun anywhere: the
    reference's BoxFusion.boxfusion on face-on views (make_golden.gen_faceon) -- every fitness
    evaluation of every iteration stays inside corners_i[36] / convex_inter[8] -- and the oracle
    reproduces its fused boxes bit for bit, again with zero overflow"""
    g = TU.load("fusion_faceon.npz")
    assert tuple(g["hull_over"]) == (0, 0) and int(g["launches"]) > 50
    be = OracleBackend()
    lists, views = faceon_jobs(g)
    OR.hull_overflow()
    n_upd = 0
    for k, v in enumerate(views):
        r = OR.fusion_fit(*v, be.pst, be.fcfg)
        want = g["after"][k]
        assert bool(r["updated"]) == bool((want != g["before"][k]).any())
        if r["updated"]:
            np.testing.assert_array_equal(r["box"], want)
            n_upd += 1
    assert OR.hull_overflow() == (0, 0)
    assert n_upd == len(views)


def test_backproject_vs_reference_unproject():
    """oracle.backproject (the a13 checker of test_gpu_fusion.py) against the reference's own
    tools/utils.unproject output on the same depth / K / RT (utils.npz, make_golden_utils.py):
    valid mask bit for bit, points to f32 rounding of the 4x4 inverse"""
    u = TU.load("utils.npz")
    xyz, valid = OR.backproject(u["depth"], u["K"], u["RT"], 10.0)
    np.testing.assert_array_equal(valid, u["valid"])
    assert valid.sum() > 1000 and (~valid).sum() > 100
    np.testing.assert_allclose(xyz, u["xyz"], rtol=1e-5, atol=2e-5)
