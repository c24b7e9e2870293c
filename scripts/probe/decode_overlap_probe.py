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
    # a spin kernel of the same residency (12 workgroups x 4 waves spinning) instead of the decode
    spin = torch.zeros(2 * 4096, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(sA):
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record()
        _lib.lib().bf_cu_probe(_lib._ptr(spin), 12, 200_000_000, _lib.c_void_p(sA.cuda_stream))
        s1.record()
    m0, m1 = mm_loop()
    torch.cuda.synchronize()
    print(f"matmul loop with a 12-workgroup spin kernel running {m0.elapsed_time(m1):.1f} ms "
          f"(spin {s0.elapsed_time(s1):.1f} ms)", flush=True)
    # CU-partitioned: the matmul stream masked off the decode's CUs
    det, res = _lib.partition_cus(16)
    sB = _lib.cu_masked_stream(det)
    sA = _lib.cu_masked_stream(res)
    mm_loop(5)
    torch.cuda.synchronize()
    m0, m1 = mm_loop()
    torch.cuda.synchronize()
    alone = m0.elapsed_time(m1)
    d0, d1 = decode()
    m0, m1 = mm_loop()
    torch.cuda.synchronize()
    print(f"masked (matmul on {len(det)} CUs, decode on {len(res)}): matmul alone {alone:.1f} ms, with the decode "
          f"{m0.elapsed_time(m1):.1f} ms; decode {d0.elapsed_time(d1):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
