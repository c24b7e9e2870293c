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


def test_bench_rank0_share_rehearsal():
    """rank 0 (the fusion owner) detecting fewer frames: its all-gather chunk is padded and the
    padding dropped, so rank 0 still receives every frame of the step in global order"""
    r, lines = _bench("--gpus", "3", "--cpu-rehearsal", "--no-cpu-baseline", "--steps", "3",
                      "--warmup", "1", "--batch", "4", "--rank0-batch", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(lines[0])
    assert line["config"]["rank0_batch"] == 2
    assert line["config"]["global_batch"] == 2 + 2 * 4
    assert line["config"]["frames"] == 3 * 10
    assert line["rehearsal"]["frame_order_ok"] is True
    assert line["rehearsal"]["frames_received"] == 4 * 10


def test_rank_frames_partition():
    import bench
    B, B0, N = 8, 6, 8
    per = B0 + (N - 1) * B
    for step in range(3):
        got = sorted(f for r in range(N) for f in bench.rank_frames(step, r, B, B0, per))
        assert got == list(range(step * per, (step + 1) * per))
    assert bench.rank_frames(1, 0, B, B0, per, G=25) == [(per + j) * 25 for j in range(B0)]
    assert bench.auto_rank0_batch(8, 1) == 8 and bench.auto_rank0_batch(8, 2) == 8
    assert bench.auto_rank0_batch(8, 4) == 8 and bench.auto_rank0_batch(8, 8) == 7
