"""Colour-JPEG decode throughput: the GPU decode (bf_jpeg_decode_rgb, batches of F files resident
in HBM) against PIL (libjpeg-turbo) on host threads, on 1296 x 968 colour frames of the synthetic
scene written by PIL's encoder at quality 90, 4:2:0 (what a ScanNet-style exporter writes).
usage: python scripts/jpeg_bench.py [F] [reps] [host_threads] [quality]"""
import io
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

H, W = 968, 1296


def make_jpegs(n_distinct=8, quality=90, H=H, W=W):
    from boxfusion_amd.synthetic import frame_rgbd
    out = []
    for f in range(n_distinct):
        rgb = frame_rgbd(f * 5, H // 2, W // 2)[0]
        img = Image.fromarray(rgb).resize((W, H), Image.BILINEAR)
        b = io.BytesIO()
        img.save(b, format="JPEG", quality=quality)
        out.append(b.getvalue())
    return out


def host_rate(blobs, threads, seconds=3.0):
    def dec(b):
        return np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))
    n = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            k = max(1, threads // len(blobs) + 1)
            list(ex.map(dec, blobs * k))
            n += len(blobs) * k
    return n / (time.perf_counter() - t0)


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    quality = int(sys.argv[4]) if len(sys.argv) > 4 else 90
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    _lib.lib()
    pool = make_jpegs(quality=quality)
    blobs = [pool[i % len(pool)] for i in range(F)]
    print(f"{F} files {W}x{H} q{quality}, mean {np.mean([len(b) for b in blobs]) / 1e3:.0f} KB", flush=True)
    files, offs, _ = upload_files(blobs, "cuda")
    out = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
    work = torch.empty(_lib.jpeg_workspace_bytes(F, H, W), dtype=torch.uint8, device="cuda")
    _lib.jpeg_decode_rgb(files, offs, H, W, out=out, work=work)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.jpeg_decode_rgb(files, offs, H, W, out=out, work=work, check=False)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = min(ts)
    print(f"gpu decode {F} files: {ms:.2f} ms (min of {reps}; all {['%.2f' % t for t in ts]}) -> "
          f"{F / ms * 1e3:.0f} frames/s", flush=True)
    for th in sorted({1, threads}):
        print(f"host PIL decode, {th} threads: {host_rate(pool, th):.0f} frames/s", flush=True)


if __name__ == "__main__":
    main()
