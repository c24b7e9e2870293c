"""Result writers (demo.py:368-387, tools/utils.py:302-331): post_process against the reference's
own output (tests/golden/results.npz from make_golden_results.py), the save lists and the files
export() writes.  The GPU case takes its corners from bf_box_corners and checks them against the
oracle's corner restatement."""
import os
import pickle
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from boxfusion_amd import results as RS

HERE = os.path.dirname(os.path.abspath(__file__))
CLASSES = ["chair", "table", "sofa"]


def _golden():
    return np.load(os.path.join(HERE, "golden", "results.npz"))


def test_post_process_matches_reference():
    g = _golden()
    np.testing.assert_array_equal(RS.post_process(g["corners"]), g["post"])
    np.testing.assert_array_equal(RS.post_process(g["corners"], threshold=0.5), g["post_05"])


def test_post_process_empty():
    assert RS.post_process(np.zeros((0, 8, 3), np.float32)).shape == (0, 8, 3)


class _Inst:
    def __init__(self, corners, cats=None, feats=None):
        self.pred_boxes_3d = SimpleNamespace(corners=torch.from_numpy(corners))
        self.categories = cats
        self.features = feats

    def __len__(self):
        return self.pred_boxes_3d.corners.shape[0]


def _big_boxes(n, seed=0):
    rng = np.random.default_rng(seed)
    lo = rng.uniform(-2, 2, (n, 1, 3)).astype(np.float32)
    c = np.repeat(lo, 8, 1)
    c[:, 1:] += rng.uniform(0.5, 1.0, (n, 7, 3)).astype(np.float32)
    c[:, 7] = lo[:, 0] + 1.0
    return c


def test_save_lists_and_export(tmp_path):
    c = _big_boxes(5)
    glob = _Inst(c, cats=np.array(["chair", "sofa", "table", "chair", "sofa"]))
    feats = np.arange(5 * 4, dtype=np.float32).reshape(5, 4)
    frame = _Inst(c[:3], cats=np.array(["table", "chair", "sofa"]), feats=feats[:3])
    lst = RS.global_save_list(glob, CLASSES, "scannet")
    assert len(lst) == 1 and len(lst[0]) == 5
    assert all(t[0] == 0 and t[2] == 1.0 for t in lst[0])
    np.testing.assert_array_equal(np.stack([t[1] for t in lst[0]]), c)
    fl = RS.framewise_save_list(frame, CLASSES)
    assert [int(t[0]) for t in fl[0]] == [1, 0, 2]
    np.testing.assert_array_equal(fl[0][2][2], feats[2])
    cfg = {"dataset": "scannet", "eval": True, "data": {"output_dir": str(tmp_path)}}
    files = RS.export(glob, frame, CLASSES, cfg, "scene0000_00")
    assert [os.path.basename(f) for f in files] == ["scene0000_00_boxes.pkl", "framewise_boxes.pkl"]
    with open(files[0], "rb") as f:          # our own file
        back = pickle.load(f)
    np.testing.assert_array_equal(np.stack([t[1] for t in back[0]]), c)
    cfg["data"]["output_dir"] = None
    assert RS.export(glob, frame, CLASSES, cfg, "x") == []


def test_global_list_unknown_class_raises():
    glob = _Inst(_big_boxes(2), cats=np.array(["chair", "lamp"]))
    with pytest.raises(ValueError):
        RS.global_save_list(glob, CLASSES, "CA1M")


def test_global_list_post_process_drop_raises_like_reference():
    """demo.py:378 indexes the post-processed corners over len(all_pred_box): a dropped thin box
    makes the reference raise IndexError; the writer keeps that behaviour."""
    c = _big_boxes(3)
    c[1] = c[1, :1]                                  # degenerate: zero extent
    with pytest.raises(IndexError):
        RS.global_save_list(_Inst(c, cats=np.array(["chair"] * 3)), CLASSES, "scannet")
    assert len(RS.global_save_list(_Inst(c, cats=np.array(["chair"] * 3)), CLASSES, "CA1M")[0]) == 3


@pytest.mark.gpu
def test_export_corners_from_device(tmp_path):
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from oracle import oracle as OR
    rng = np.random.default_rng(3)
    n = 37
    t = np.concatenate([rng.uniform(-3, 3, (n, 3)), rng.uniform(0.4, 1.2, (n, 3))], 1).astype(np.float32)
    yaw = rng.uniform(-np.pi, np.pi, n)
    R = np.zeros((n, 3, 3), np.float32)
    R[:, 0, 0] = np.cos(yaw); R[:, 0, 2] = np.sin(yaw); R[:, 1, 1] = 1
    R[:, 2, 0] = -np.sin(yaw); R[:, 2, 2] = np.cos(yaw)
    dev = torch.device("cuda:0")
    inst = _Inst(np.zeros((n, 8, 3), np.float32), cats=np.array(["chair"] * n))
    inst.pred_boxes_3d = GeneralInstance3DBoxes(torch.from_numpy(t).to(dev), torch.from_numpy(R).to(dev))
    lst = RS.global_save_list(inst, CLASSES, "CA1M")
    got = np.stack([x[1] for x in lst[0]])
    np.testing.assert_allclose(got, OR.box_corners(t, R), rtol=0, atol=1e-6)
