"""N-rank fusion output == 1-rank output (DESIGN.md §6 claims it).

Ranks run bench.py's own data path on CPU with gloo: each rank packs its block-cyclic frames into
the per-frame detection records (bench.pack_records) and CLIP rows, bench.exchange_step all-gathers
them with the same all_gather_into_tensor sequence the RCCL path uses (rank 0's smaller share
padded and dropped), and the fusion owner (rank 0) runs the reference-pinned oracle fusion chain
(oracle/chain.py: demo.py:200-305's keyframe sequence over the C restatement) on the gathered
records in global frame order -- CLIP similarities folded into the scores as unpack_records does
(demo.py:167-170).  The final global boxes, fusion_list, already_fusion and per-keyframe box counts
must be bit-equal to a 1-rank run over the same frames, at world sizes 2 and 8 and with rank 0
detecting fewer frames (--rank0-batch).  No kernels run; the device-side equality of the fusion
itself (HIP == oracle) is covered by the -m gpu fusion tests."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

GAP = 5          # keyframes every 5th frame: views far enough apart that lists grow and fuse
CROPS = 4
CLIP_COEFF = 1.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _clip_rows(frames, crops):
    """rank-independent CLIP rows of a batch of frames: feature[1024] (frame-coded), similarity,
    class index -- a function of (frame, crop) only"""
    import bench
    out = torch.zeros(len(frames) * crops, bench.CLIP_W)
    for j, f in enumerate(frames):
        for c in range(crops):
            r = j * crops + c
            out[r, 0] = float(f)
            out[r, 1024] = float((f * 31 + c * 7) % 97) / 97.0 * 30.0
            out[r, 1025] = float((f + c) % 11)
    return out


def _record_det(rec, clip, crops):
    """gathered record + its CLIP rows -> the detection dict the fusion chain takes (the numpy
    mirror of bench.unpack_records: detection r < crops gets crop r's similarity)"""
    import bench
    n = int(rec[0].item())
    rows = rec[bench.REC_HEAD:bench.REC_HEAD + n * bench.REC_W].view(n, bench.REC_W).numpy()
    scores = rows[:, 0].copy()
    sims = clip[:, 1024].numpy()
    m = min(n, crops)
    scores[:m] = (torch.from_numpy(scores[:m]) + CLIP_COEFF * torch.from_numpy(sims[:m]) / 100.0).numpy()
    return dict(scores=scores.astype(np.float32), pred_boxes=rows[:, 1:5].copy(), xyzlhw=rows[:, 5:11].copy(),
                R=rows[:, 11:20].reshape(n, 3, 3).copy())


def _digest(chain):
    h = hashlib.sha256()
    for k in ("tensor", "R", "scores", "init_id", "valid_num"):
        h.update(np.ascontiguousarray(chain.g[k]).tobytes())
    return dict(boxes=h.hexdigest(), n_global=int(len(chain.g["scores"])),
                fusion_list=[list(map(int, x)) for x in chain.fusion_list],
                already_fusion=[list(map(int, x)) for x in chain.already_fusion],
                num_record={int(k): int(v) for k, v in chain.num_record.items()})


def _run(rank, world, port, B, B0, total, q):
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        d = dist
    else:
        d = None
    try:
        import bench
        from boxfusion_amd.box_fusion import load_pst
        from boxfusion_amd.synthetic import SCANNET_K, Scene
        from oracle.chain import OracleChain
        scene = Scene(seed=0)
        per_step = B * world - (B - B0)
        assert total % per_step == 0
        chain = OracleChain(bench.CFG, SCANNET_K, pst=load_pst(), legacy=True) if rank == 0 else None
        order = []
        for s in range(total // per_step):
            frames = bench.rank_frames(s, rank, B, B0, per_step, GAP)
            recs = torch.from_numpy(bench.pack_records([scene.detections(f) for f in frames],
                                                       [scene.pose(f) for f in frames]))
            g_rec, g_clip = bench.exchange_step(recs, _clip_rows(frames, CROPS), d, world, B, B0, CROPS, rank)
            if rank == 0:
                poses, cnt = bench.record_meta(g_rec)
                for j in range(len(cnt)):
                    f = (s * per_step + j) * GAP
                    order.append(f)
                    assert g_clip[j * CROPS, 0].item() == float(f)      # the CLIP rows travel with the frame
                    chain.keyframe(f, poses[j].astype(np.float64), _record_det(g_rec[j], g_clip[j * CROPS:(j + 1) * CROPS], CROPS))
        if rank == 0:
            out = _digest(chain)
            out["order"] = order
            q.put(out)
    except BaseException as e:      # rank 0's failure reaches the parent instead of a queue timeout
        if rank == 0:
            q.put({"error": repr(e)})
        raise
    finally:
        if d is not None:
            dist.barrier()
            dist.destroy_process_group()


def _fuse(world, B, B0, total):
    if world == 1:
        import queue
        q = queue.Queue()
        _run(0, 1, 0, B, B0, total, q)
        return q.get()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, B, B0, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(120)
    assert "error" not in out, out.get("error")
    assert all(p.exitcode == 0 for p in procs)
    return out


_ONE = {}


def one_rank(total):
    """the 1-rank run over `total` frames (bench's path at world 1: exchange_step is the identity)"""
    if total not in _ONE:
        _ONE[total] = _fuse(1, total, total, total)
    return _ONE[total]


@pytest.mark.parametrize("world,B,B0,total", [(2, 5, 5, 60), (2, 4, 2, 60), (8, 2, 1, 60), (8, 8, 7, 63)])
def test_n_rank_fusion_equals_one_rank(world, B, B0, total):
    """world 2 (equal shares; rank 0 on half a share) and 8 (rank 0 on B - 1 frames: the
    auto_rank0_batch rule at 8 ranks, bench.py --rank0-batch 7 at the bench's B = 8): the fusion
    owner's result is bit-equal to the 1-rank run over the same frames"""
    ref = one_rank(total)
    got = _fuse(world, B, B0, total)
    assert got["order"] == [f * GAP for f in range(total)]
    assert ref["order"] == got["order"]
    assert ref["already_fusion"], "the scene must exercise BoxFusion for the test to mean anything"
    for k in ("boxes", "n_global", "fusion_list", "already_fusion", "num_record"):
        assert got[k] == ref[k], k
