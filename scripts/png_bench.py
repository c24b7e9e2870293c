"""Depth-PNG decode throughput: the GPU decode (bf_png_decode_depth, batches of F files resident in
HBM) against PIL on host threads, on 640 x 480 16-bit depth maps of the synthetic scene written by
PIL's encoder (adaptive filters, zlib level 6 -- what a ScanNet-style writer produces).
usage: python scripts/png_bench.py [F] [reps] [host_threads]"""
import io
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def make_pngs(n_distinct=16, H=480, W=640, level=6, smooth=False):
    """smooth=True: the same frames with the sensor noise box-filtered away (5 x 5) before the
    mm quantisation -- a more compressible file (longer matches), closer to a filtered depth map"""
    from boxfusion_amd.synthetic import frame_rgbd
    out = []
    for f in range(n_distinct):
        d = frame_rgbd(f * 5, H, W)[1].astype(np.float64)
        if smooth:
            from scipy.ndimage import uniform_filter
            d = np.where(d > 0, uniform_filter(d, 5), 0.0)
        d = np.clip(d * 1000.0, 0, 65535).astype(np.uint16)
        b = io.BytesIO()
        Image.fromarray(d).save(b, format="PNG", compress_level=level)
        out.append(b.getvalue())
    return out


def host_rate(blobs, threads, seconds=3.0):
    def dec(b):
        return np.asarray(Image.open(io.BytesIO(b)))
    n = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds:
            list(ex.map(dec, blobs * max(1, threads // len(blobs) + 1)))
            n += len(blobs) * max(1, threads // len(blobs) + 1)
    return n / (time.perf_counter() - t0)


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    _lib.lib()
    pool = make_pngs()
    blobs = [pool[i % len(pool)] for i in range(F)]
    print(f"{F} files, mean {np.mean([len(b) for b in blobs]) / 1e3:.0f} KB", flush=True)
    files, offs, offs_h = upload_files(blobs, "cuda")
    out = torch.empty((F, 480, 640), dtype=torch.float32, device="cuda")
    work = torch.empty(_lib.png_workspace_bytes(F, 480, 640, int(offs_h[-1])), dtype=torch.uint8, device="cuda")
    _lib.png_decode_u16(files, offs, 480, 640, out=out, offsets_host=offs_h, depth_scale=1000.0, work=work)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.png_decode_u16(files, offs, 480, 640, out=out, offsets_host=offs_h, depth_scale=1000.0, work=work,
                            check=False)
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
