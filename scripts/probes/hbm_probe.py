"""HBM read-path probe (see hbm_probe.hip): GB/s of a 236 MB read with and without LDS atomics
and with a per-frame global histogram flush; the last rows time bf_depth's own hist kernels'
call (bf_depth_standardize) on the same data for reference."""
import ctypes, os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhbm_probe.so"))
n = 192 * 480 * 640
d = torch.rand(n, device="cuda") * 4 + 0.5
out = torch.zeros(1, device="cuda")
g = torch.zeros(2048 * 4096, dtype=torch.int32, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def timed(f, reps=20):
    for _ in range(3): f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for kv in (4, 16):
    for mode in (0, 1, 2, 3, 4):
        us = timed(lambda: lib.probe(mode, kv, ctypes.c_void_p(d.data_ptr()), ctypes.c_longlong(n),
                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(g.data_ptr()), st))
        print(f"kv {kv:2d} mode {mode}: {us:7.1f} us  {4 * n / us / 1e3:6.0f} GB/s", flush=True)
for kv in (4, 16):
    us = timed(lambda: lib.probe2(kv, ctypes.c_void_p(d.data_ptr()), 192, ctypes.c_longlong(307200),
                                  ctypes.c_void_p(g.data_ptr()), st))
    print(f"bf_depth layout kv {kv:2d}: {us:7.1f} us  {4 * n / us / 1e3:6.0f} GB/s", flush=True)
from boxfusion_amd import _lib
dd = d.view(192, 480, 640)
print(f"bf_depth_standardize (7 launches): {timed(lambda: _lib.depth_standardize(dd)):.1f} us")
