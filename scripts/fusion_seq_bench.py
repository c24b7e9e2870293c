"""Host cost of the rank-0 fusion worker per keyframe: the Python-driven FusionStage against the
native keyframe sequencer (bf_fseq), on the batches rank 0 fuses at N=8 (64 keyframes of
records per step -> FusionStage.keyframes), 30- and 150-object scenes, GPU otherwise idle.
Checks that both end in the same state.  Usage: python scripts/fusion_seq_bench.py [steps]
BF_SEQ_CUS=32: the fusion runs on a stream confined to the CUs bench.py reserves for rank 0's
fusion at N>1 (the rest of the chip idle), to separate the CU budget from the detect load."""
import os
import sys
import time

import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from boxfusion_amd import _lib  # noqa: E402
from boxfusion_amd.fusion_stage import FusionStage  # noqa: E402
from boxfusion_amd.synthetic import SCANNET_K, Scene  # noqa: E402

dev = torch.device("cuda")
PER = 64
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6


def records(scene, s):
    fr = list(range(s * PER, (s + 1) * PER))
    return torch.from_numpy(bench.pack_records([scene.detections(f) for f in fr],
                                               [scene.pose(f) for f in fr])).to(dev)


def run(st, r, base):
    p, c = bench.record_meta(r)
    st.keyframes([base + j for j in range(r.shape[0])], p, bench.unpack_records(r, c, dev), c)


OBJS = [int(v) for v in os.environ.get("BF_SEQ_OBJECTS", "30,150").split(",")]
MODES = [m == "native" for m in os.environ.get("BF_SEQ_MODES", "python,native").split(",")]
CUS = int(os.environ.get("BF_SEQ_CUS", "0"))
if CUS:
    torch.cuda.set_stream(_lib.cu_masked_stream(_lib.partition_cus(CUS)[1]))
for n_obj in OBJS:
    scene = Scene(seed=0, n_objects=n_obj)
    recs = [records(scene, s) for s in range(steps)]
    out = {}
    for native in MODES:
        warm = FusionStage(bench.CFG, SCANNET_K, device=dev, native=native)
        run(warm, recs[0], 0)
        warm.boxes()
        torch.cuda.synchronize()
        st = FusionStage(bench.CFG, SCANNET_K, device=dev, native=native)
        per_step = []
        for s in range(steps):
            t0 = time.perf_counter()
            run(st, recs[s], s * PER)
            st.box_manager.flush() if not native else st._seq.sync()
            torch.cuda.synchronize()
            per_step.append(time.perf_counter() - t0)
        ms = 1e3 * np.asarray(per_step) / PER
        out[native] = st
        print(f"objects {n_obj:4d} {'native ' if native else 'python '}: {ms.mean():.3f} ms/keyframe "
              f"(steps {' '.join(f'{v:.3f}' for v in ms)}), global boxes {len(st.all_pred_box)}, "
              f"stats {st.stats}", flush=True)
    if len(out) < 2:
        continue
    a, b = out[True], out[False]
    same = (a.box_manager.fusion_list == b.box_manager.fusion_list and
            a.box_manager.already_fusion == b.box_manager.already_fusion and
            all(np.array_equal(x, y) for x, y in zip(a.boxes(), b.boxes())) and a.stats == b.stats)
    print(f"objects {n_obj}: native state == python state: {same}", flush=True)
