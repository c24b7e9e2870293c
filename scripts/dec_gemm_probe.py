"""The CuTR decoder's f32 GEMMs (bf_gemm_f32) of one bench-shaped batch: every call's shape recorded
through the decoder engine, then each distinct shape timed alone (HIP events, 20 reps) with its
TF/s against the 155 TF/s f32 MFMA rate, and torch's f32 matmul beside it for reference."""
import collections
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from boxfusion_amd import _lib  # noqa: E402
from boxfusion_amd.clip import VisionTransformer  # noqa: E402
from boxfusion_amd.cubify_transformer import make_cubify_transformer  # noqa: E402
from boxfusion_amd.pipeline import DetectStage  # noqa: E402
from boxfusion_amd.synthetic import SCANNET_K, Scene  # noqa: E402


def tm(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(768, True).eval()
        vis = VisionTransformer(224, 14, 1280, 2, 16, 1024).eval()
    B, H, W = 8, 480, 640
    det = DetectStage(cutr, vis, bench.CFG, B, H, W, SCANNET_K, crops_per_frame=16,
                      crop_source="top", clip_capacity=B * 16, device=dev)
    rgb, depth = bench.gen_frames(list(range(B)), dev)
    poses = np.stack([Scene(seed=0).pose(f) for f in range(B)])
    calls = collections.Counter()
    orig = _lib.gemm_f32

    def rec(a, w, bias=None, act=None, resid=None, out=None, a_map=None, c_map=None, m=None):
        N, K = w.shape
        M = m if m is not None else (a_map.shape[0] if a_map is not None else a.shape[0])
        calls[(M, N, K, act or "", resid is not None, a_map is not None)] += 1
        return orig(a, w, bias, act, resid, out, a_map, c_map, m)
    _lib.gemm_f32 = rec
    det(rgb, depth, poses, return_instances=False)
    torch.cuda.synchronize()
    _lib.gemm_f32 = orig
    tot_us = tot_t = tot_fl = 0.0
    rows = []
    for (M, N, K, act, res, amap), n in sorted(calls.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1]):
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev) if res else None
        o = torch.empty(M, N, device=dev)
        us = tm(lambda: orig(a, w, b, act=act or None, resid=r, out=o))
        ut = tm(lambda: torch.addmm(b, a, w.T))
        fl = 2.0 * M * N * K
        tot_us += n * us
        tot_t += n * ut
        tot_fl += n * fl
        rows.append(dict(M=M, N=N, K=K, act=act, resid=res, a_map=amap, calls=n, us=round(us, 1),
                         tflops=round(fl / us / 1e6, 1), torch_us=round(ut, 1)))
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"calls": sum(calls.values()), "gemm_f32_us_per_batch": round(tot_us, 1),
                      "torch_f32_us_per_batch": round(tot_t, 1), "gflop": round(tot_fl / 1e9, 2)}))


if __name__ == "__main__":
    main()
