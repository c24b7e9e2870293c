"""Run visualisation (demo.py:93-197 / tools/utils.py:37-141) on the host:
the jet colours, the box mesh and its PLY, demo.py's per-frame log sequence, and the boxes the
Pipeline logs after each keyframe.  The real viewer (rerun) and open3d are absent from this image;
the records are compared with what the reference's calls would carry (parity of the geometry:
the box mesh against the corner formula of boxes.py:725-778 restated in oracle/bf_oracle.c)."""
import numpy as np
import pytest
import torch
from scipy.spatial.transform import Rotation

from boxfusion_amd import visualize as V
from boxfusion_amd.boxes import GeneralInstance3DBoxes


class _Inst:
    def __init__(self, boxes, categories):
        self.pred_boxes_3d = boxes
        self.categories = categories

    def __len__(self):
        return len(self.pred_boxes_3d.tensor)


def _boxes(n, seed=0):
    rng = np.random.default_rng(seed)
    xyz = rng.uniform(-2, 2, (n, 3))
    lhw = rng.uniform(0.2, 1.5, (n, 3))
    R = Rotation.from_euler("z", rng.uniform(-np.pi, np.pi, n)).as_matrix()
    return GeneralInstance3DBoxes(torch.tensor(np.hstack([xyz, lhw]), dtype=torch.float32),
                                  torch.tensor(R, dtype=torch.float32))


def test_random_color_v2_is_jet():
    assert np.allclose(V.random_color_v2(0.0), [0.0, 0.0, 0.5])
    assert np.allclose(V.random_color_v2(1.0), [0.5, 0.0, 0.0])
    c = np.array([V.random_color_v2(i / 10) for i in range(10)])
    assert c.shape == (10, 3) and (c >= 0).all() and (c <= 1).all()


def test_box_mesh_matches_corner_formula():
    from oracle.oracle import box_corners as or_corners
    b = _boxes(5, 1)
    q = V._quat_xyzw(b.R.numpy())
    verts, faces = V.box_mesh(b.dims.numpy(), b.gravity_center.numpy(), q)
    assert verts.shape == (40, 3) and faces.shape == (60, 3) and faces.max() == 39
    # the same eight points as the reference corners (any order): the box extent along R's axes
    ref = or_corners(b.tensor.numpy().astype(np.float32), b.R.numpy().astype(np.float32))
    for i in range(5):
        a = np.round(verts[8 * i:8 * i + 8], 4)
        r = np.round(ref[i].astype(np.float64), 4)
        assert sorted(map(tuple, a)) == pytest.approx(sorted(map(tuple, r)), abs=2e-4)


def test_ply_round_trip(tmp_path):
    b = _boxes(3, 2)
    q = V._quat_xyzw(b.R.numpy())
    cols = [V.random_color_v2(i / 3) for i in range(3)]
    fn = tmp_path / "box_7.ply"
    V.boxes3d_to_ply(b.dims.numpy(), b.gravity_center.numpy(), cols, q, str(fn))
    head = open(fn, "rb").read(300).decode("ascii", "ignore")
    assert head.startswith("ply\nformat binary_little_endian 1.0\nelement vertex 24\n")
    assert "element face 36" in head
    verts, rgb, faces = V.read_ply_mesh(str(fn))
    v0, f0 = V.box_mesh(b.dims.numpy(), b.gravity_center.numpy(), q)
    assert np.array_equal(verts, v0) and np.array_equal(faces, f0)
    assert np.array_equal(rgb[::8], np.rint(np.array(cols) * 255).astype(np.uint8))


def test_frame_logger_sequence_and_boxes(tmp_path):
    rec = V.Recording(forward=False)
    K = np.array([[577.9, 0, 319.5], [0, 577.9, 239.5], [0, 0, 1]])
    lg = V.FrameLogger(rec, K, (640, 480), K_depth=K, depth_size=(640, 480), save_ply=True,
                       out_dir=str(tmp_path), show_class=True)
    RT = np.eye(4)
    RT[:3, 3] = [1.0, 2.0, 3.0]
    img = np.zeros((480, 640, 3), np.uint8)
    dep = np.ones((480, 640), np.float32)
    lg.frame(0, RT, image=img, depth=dep)
    RT2 = RT.copy()
    RT2[:3, 3] = [1.5, 2.0, 3.0]
    lg.frame(1, RT2)
    seq = [(p, k) for p, _, k, _ in rec.records]
    # demo.py:86-108's order for a frame with image and depth
    assert seq[:8] == [("/world/image", "Transform3D"), ("/world/image", "Pinhole"),
                       ("/device/wide/image", "Transform3D"), ("/device/wide/image", "Image"),
                       ("/device/wide/image", "Pinhole"), ("/device/wide/depth", "DepthImage"),
                       ("/device/wide/depth", "Pinhole"), ("/world/trajectory", "LineStrips3D")]
    # the trajectory of frame 1 holds the positions before it (demo.py:108: traj[:count])
    tr = rec.last("/world/trajectory")
    assert np.allclose(tr["strips"][0], [[1.0, 2.0, 3.0]])
    assert rec.records[-1][1] == ("pts", 1 / 30.0)
    b = _boxes(4, 3)
    arch = lg.boxes(_Inst(b, np.array(["chair", "table", "sofa", "bed"])), 5)
    assert arch["labels"] == ["chair", "table", "sofa", "bed"]
    assert np.allclose(arch["centers"], b.tensor[:, :3].numpy())
    assert np.allclose(arch["sizes"], b.tensor[:, 3:6].numpy())
    # quaternions reproduce R
    assert np.allclose(Rotation.from_quat(arch["quaternions_xyzw"]).as_matrix(), b.R.numpy(), atol=1e-6)
    assert (tmp_path / "box_5.ply").exists()
    assert rec.entities()[0] == "/device/wide/depth" and "/device/wide/pred_instances" in rec.entities()
    out = tmp_path / "rec.jsonl"
    rec.save(str(out))
    lines = open(out).read().strip().split("\n")
    assert len(lines) == len(rec.records)
    assert '"kind": "Image"' in lines[3] and '"shape": [480, 640, 3]' in lines[3]


def test_pipeline_viz_frame_order():
    """Pipeline.run(viz=...) logs the frames in frame order for gap > 1 (demo.py:93-197 logs every
    frame as it arrives, the boxes after each keyframe's fusion): batch [0, g, ...] must not log
    its non-keyframes before its keyframes, so the trajectory strip of frame c is the poses of
    frames [0, c)."""
    import torch
    from boxfusion_amd.pipeline import Pipeline

    n, gap, B = 23, 4, 2
    poses_all = np.stack([np.eye(4) for _ in range(n)])
    poses_all[:, 0, 3] = np.arange(n)

    class Det:
        def __init__(self):
            self.B = B

        def preprocess_frames(self, depth, poses):
            pass

        def __call__(self, rgb, depth, poses):
            return [None] * len(poses)

    class Fus:
        all_pred_box = None

        def __init__(self):
            self.calls = []

        def keyframe(self, i, pose, pred):
            self.calls.append(("kf", i))

        def finish(self, last, pose, was_kf):
            self.calls.append(("finish", last))

    class Log:
        def __init__(self):
            self.seq = []
            self.lg = V.FrameLogger(V.Recording(forward=False), np.eye(3), (4, 4))

        def frame(self, i, pose, *images):
            self.seq.append(("frame", i))
            self.lg.frame(i, pose)

        def boxes(self, apb, i):
            self.seq.append(("boxes", i))

    def frames(ids):
        return (torch.zeros((len(ids), 4, 4, 3), dtype=torch.uint8), torch.zeros((len(ids), 4, 4)),
                poses_all[list(ids)])

    log, fus = Log(), Fus()
    Pipeline(Det(), fus, gap).run(frames, n, viz=log)
    assert [i for k, i in log.seq if k == "frame"] == list(range(n))
    kfs = list(range(0, n, gap))
    assert [i for k, i in log.seq if k == "boxes"] == kfs + [n - 1]
    # each keyframe's boxes come right after its own frame record
    for i in kfs:
        assert log.seq[log.seq.index(("frame", i)) + 1] == ("boxes", i)
    tr = log.lg.rec.last("/world/trajectory")
    assert np.array_equal(np.asarray(tr["strips"][0])[:, 0], np.arange(n - 1))
    assert fus.calls == [("kf", i) for i in kfs] + [("finish", n - 1)]
