"""bench.gather_step over gloo with world_size 2 (CPU): the fusion owner receives every rank's
per-frame records in global frame order."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from boxfusion_amd.synthetic import Scene
    scene = Scene(seed=0)
    B, step = 4, 3
    frames = [step * B * world + rank * B + j for j in range(B)]
    poses = np.stack([scene.pose(f) for f in frames])
    recs = torch.from_numpy(bench.pack_records([scene.detections(f) for f in frames], poses))
    feats = torch.full((B * 2, 8), float(rank))
    g_rec, g_feat = bench.gather_step(recs, feats, dist, world)
    if rank == 0:
        want = [step * B * world + j for j in range(B * world)]
        exp = bench.pack_records([scene.detections(f) for f in want], [scene.pose(f) for f in want])
        g_pose, g_cnt = bench.record_meta(g_rec)
        ok = (np.array_equal(g_rec.numpy(), exp)
              and np.array_equal(g_pose, np.stack([scene.pose(f) for f in want]).astype(np.float32))
              and np.array_equal(g_cnt, exp[:, 0].astype(np.int64))
              and g_feat[:B * 2].eq(0).all().item() and g_feat[B * 2:].eq(1).all().item())
        unpacked = bench.unpack_record(g_rec[1], "cpu")
        ok = ok and len(unpacked) == int(exp[1, 0])
        q.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_step_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert res
    assert all(p.exitcode == 0 for p in procs)


def _rccl_worker(port, q):
    """one rank on cuda:0 over RCCL (backend "nccl" = RCCL on ROCm): bench.gather_step's
    all_gather_into_tensor sequence on device tensors, forced at world size 1"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench
    from boxfusion_amd.synthetic import Scene
    scene = Scene(seed=0)
    frames = list(range(8))
    recs = torch.from_numpy(bench.pack_records([scene.detections(f) for f in frames],
                                               np.stack([scene.pose(f) for f in frames]))).to(dev)
    clip = torch.arange(8 * 16 * bench.CLIP_W, dtype=torch.float32, device=dev).view(8 * 16, -1)
    g_rec, g_clip = bench.gather_step(recs, clip, dist, 1, force=True)
    torch.cuda.synchronize()
    ok = bool(torch.equal(g_rec, recs) and torch.equal(g_clip, clip) and g_rec.data_ptr() != recs.data_ptr())
    g_rec, g_clip = bench.exchange_step(recs, clip, dist, 1, 8, 8, 16, 0)
    ok = ok and bool(torch.equal(g_rec, recs))
    dist.barrier()
    dist.destroy_process_group()
    q.put(ok)


import pytest  # noqa: E402


@pytest.mark.gpu
def test_gather_step_rccl_world1():
    """the RCCL branch of bench.gather_step on hardware (the 8-GPU run is the driver's)"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert res and p.exitcode == 0
