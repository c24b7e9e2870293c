"""Clean interpreter exit after a run's HIP resources (round 4: SIGSEGV in __cxa_finalize after the
--sim-ranks 8 bench printed its line).  Each case is a fresh child process (subprocess = spawn:
nothing GPU-side is inherited) that must exit with status 0."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# A fusion worker on a CU-masked stream, left running with keyframes queued (never joined), a
# native keyframe sequencer grown over 150-object keyframes (pinned staging buffers from the
# process-wide pool), and a second sequencer dropped by garbage collection.  _lib._shutdown must
# stop the worker, release the sequencers and destroy the masked streams while the HIP runtime is
# still up; the process then exits normally.
ABANDON = r"""
import sys, torch
sys.path.insert(0, {root!r})
from boxfusion_amd import _lib
from boxfusion_amd.fusion_stage import AsyncFusion, FusionStage
from boxfusion_amd.pipeline import scene_instances
from boxfusion_amd.synthetic import SCANNET_K, Scene
dev = torch.device("cuda")
det_s, fus_s = _lib.partition_streams(32, 0, masked=True)
from tests import trace_util as TU
cfg = dict(TU.SCANNET_CFG, data=dict(gap=1))
scene = Scene(seed=0, n_objects=150)
tmp = FusionStage(cfg, SCANNET_K, device=dev, native=True)
for f in range(4):
    tmp.keyframe(f, scene.pose(f), scene_instances(scene.detections(f), dev))
del tmp
asyn = AsyncFusion(FusionStage(cfg, SCANNET_K, device=dev, native=True), stream=fus_s)
with torch.cuda.stream(det_s):
    for f in range(40):
        d = scene.detections(f)
        ev = torch.cuda.Event()
        ev.record()
        asyn.submit(f, scene.pose(f), (lambda d=d: scene_instances(d, dev)), ev)
print("submitted", flush=True)
"""


def _run(args, timeout):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(args, cwd=ROOT, timeout=timeout, capture_output=True, text=True, env=env)
    return r


def test_exit_with_running_fusion_worker():
    r = _run([sys.executable, "-u", "-c", ABANDON.format(root=ROOT)], 110)
    assert r.returncode == 0, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert "submitted" in r.stdout


def test_bench_sim_ranks_exits_cleanly():
    """bench.py's own exit path: detect graphs on masked streams, the fusion worker fusing two
    ranks' keyframes through the native sequencer, CPU-side results, then a normal exit"""
    r = _run([sys.executable, "-u", "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
              "--sim-ranks", "2", "--fusion-cus", "32", "--mask-cus", "1", "--dim", "192",
              "--clip-layers", "2", "--crops", "2", "--roofline-steps", "1", "--roofline-keyframes", "4"], 115)
    assert r.returncode == 0, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert '"metric"' in r.stdout
