"""Store throughput by row-segment shape (scripts/probe/store_shape.hip): a 32896 x 3840 bf16 output
(CLIP qkv's, 252 MB) written by 256 blocks of 128 rows x 7680 B, 16 B per lane, SEG contiguous bytes
per row in each wave-instruction."""
import ctypes
import os
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = ctypes.CDLL(os.path.join(ROOT, "boxfusion_amd/_build/probe/store_shape.so"))
M, NB = 32896, 3840 * 2
out = torch.empty(M * NB, dtype=torch.uint8, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
rows = 128
blocks = M // rows
for rnd in range(3):
    for seg in (512, 256, 128, 64, 32):
        f = lambda: P.store_launch(seg, ctypes.c_void_p(out.data_ptr()), ctypes.c_longlong(NB), blocks, rows, NB, st)
        assert f() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 10 * 1e3
        print(f"round {rnd} seg {seg:4d} B x {1024 // seg:2d} rows: {us:7.1f} us  {blocks * rows * NB / us / 1e6:6.2f} TB/s", flush=True)
