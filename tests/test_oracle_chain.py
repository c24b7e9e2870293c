"""oracle/chain.py (the CPU restatement of demo.py:200-305 used as the bench CPU baseline and as
a checker) reproduces the reference's recorded fusion chain keyframe by keyframe.  CPU only."""
import numpy as np
import pytest

from oracle.chain import OracleChain
from tests import trace_util as TU


@pytest.mark.parametrize("name", TU.TRACES)
def test_chain_matches_trace(name):
    t = TU.load(name)
    pst = np.load(TU.GOLDEN + "/../../boxfusion_amd/data/pst_1024_0.npy")
    cfg, K, H, W = TU.trace_setup(t)
    ch = OracleChain(cfg, K, H=H, W=W, pst=pst, legacy=False)
    nd = t["n_det"]
    for k, frame in enumerate(t["frame"]):
        a, b = int(nd[:k].sum()), int(nd[:k + 1].sum())
        det = dict(scores=t["det_scores"][a:b], pred_boxes=t["det_pred_boxes"][a:b],
                   xyzlhw=t["det_xyzlhw"][a:b], R=t["det_R"][a:b])
        ch.keyframe(int(frame), t["pose"][k], det)
        post = TU._rows(t, "post_tensor", k)
        np.testing.assert_allclose(ch.g["tensor"], post, rtol=0, atol=2e-5, err_msg=f"kf {k}")
        assert ch.fusion_list == TU._lists(t, "post_fl", k), f"kf {k}"
        assert ch.already_fusion == TU._lists(t, "fused", k), f"kf {k}"
