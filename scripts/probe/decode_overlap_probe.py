"""Does a long colour-JPEG decode launch (one wave per file, ~130 ms) overlap with compute on another
stream?  Times a bf16 matmul loop on stream B alone, then with a 48-file decode launched on stream A
just before it.  usage: python scripts/probe/decode_overlap_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    from bench import jpeg_pool
    _lib.lib()
    pool = jpeg_pool(8)
    files, offs, _ = upload_files([pool[i % 8] for i in range(48)], "cuda")
    out = torch.empty((48, 968, 1296, 3), dtype=torch.uint8, device="cuda")
    work = torch.empty(_lib.jpeg_workspace_bytes(48, 968, 1296), dtype=torch.uint8, device="cuda")
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()

    def mm_loop(n=60):
        with torch.cuda.stream(sB):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                torch.mm(a, b)
            e1.record()
        return e0, e1

    def decode():
        with torch.cuda.stream(sA):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.jpeg_decode_rgb(files, offs, 968, 1296, out=out, work=work, check=False)
            e1.record()
        return e0, e1

    for _ in range(2):
        mm_loop(5)
        decode()
    torch.cuda.synchronize()
    m0, m1 = mm_loop()
    torch.cuda.synchronize()
    alone = m0.elapsed_time(m1)
    d0, d1 = decode()
    time.sleep(0.001)
    m0, m1 = mm_loop()
    torch.cuda.synchronize()
    print(f"matmul loop alone {alone:.1f} ms; with the decode running {m0.elapsed_time(m1):.1f} ms; "
          f"decode {d0.elapsed_time(d1):.1f} ms; matmul start - decode start {d0.elapsed_time(m0):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
