"""bench.py --gpus N as the driver runs it: the parent starts torch.distributed.run itself (no
GPU touched), every rank checks WORLD_SIZE == N, frames shard block-cyclically, the all-gather
(same all_gather_into_tensor sequence as the RCCL path) hands rank 0 every frame in global order,
and rank 0 prints one JSON line with n_gpus = N.  --cpu-rehearsal runs that control flow on CPU
with gloo (no kernels)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO,
                       capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_self_launch_rehearsal(n):
    r, lines = _bench("--gpus", str(n), "--cpu-rehearsal", "--no-cpu-baseline", "--steps", "3",
                      "--warmup", "1", "--batch", "4")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout           # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert line["config"]["parallelism"] == f"dp{n}"
    assert line["config"]["global_batch"] == 4 * n
    assert line["config"]["frames"] == 3 * 4 * n
    assert line["rehearsal"]["frame_order_ok"] is True
    assert line["rehearsal"]["frames_received"] == 4 * 4 * n     # warmup + timed steps


def test_bench_rank_count_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--cpu-rehearsal"], cwd=REPO, capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_fp8_workload_line():
    """--clip-fp8 --vocab 200 names BASELINE configs[4] as its workload and its compute dtype"""
    r, lines = _bench("--gpus", "2", "--cpu-rehearsal", "--no-cpu-baseline", "--steps", "2",
                      "--warmup", "1", "--batch", "2", "--clip-fp8", "--vocab", "200")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(lines[0])
    assert line["config"]["workload"].startswith("configs[4]")
    assert "200-class" in line["config"]["workload"]
    assert "fp8" in line["dtype"]
