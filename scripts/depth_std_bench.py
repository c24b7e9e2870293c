"""bf_depth_standardize / bf_depth_preprocess timing on the path's shapes (8 and 192 frames of
480x640, 8 of 256x192) with HIP events, the algorithmic GB/s (read 4 B + write 4 B per pixel;
+13 B with the back-projection), and an A/B against an earlier build of bf_depth.hip when
scripts/_ab/libds_old.so exists (params and outputs bit for bit; round 4: the 7-launch form,
built from the previous commit's bf_depth.hip)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

OLD = os.path.join(ROOT, "scripts", "_ab", "libds_old.so")
old = ctypes.CDLL(OLD) if os.path.exists(OLD) else None


_OLD_WS = {}


def run_old(d):
    b, h, w = d.shape
    out = torch.empty_like(d)
    p = torch.empty((b, 2), device=d.device)
    st = torch.cuda.current_stream().cuda_stream
    ws = _OLD_WS.setdefault((b, h, w), _lib.new_depth_workspace(b, h, w, d.device))
    rc = old.bf_depth_standardize(ctypes.c_void_p(d.data_ptr()), b, h, w, ctypes.c_void_p(out.data_ptr()),
                                  ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                  ctypes.c_void_p(st))
    assert rc == 0
    return out, p


def run_old_bp(d, K, RT):
    b, h, w = d.shape
    out = torch.empty_like(d)
    p = torch.empty((b, 2), device=d.device)
    xyz = torch.empty((b, h, w, 3), device=d.device)
    valid = torch.empty((b, h, w), dtype=torch.uint8, device=d.device)
    st = torch.cuda.current_stream().cuda_stream
    ws = _OLD_WS.setdefault((b, h, w), _lib.new_depth_workspace(b, h, w, d.device))
    P = ctypes.c_void_p
    rc = old.bf_depth_preprocess(P(d.data_ptr()), b, h, w, P(out.data_ptr()), P(p.data_ptr()),
                                 P(K.data_ptr()), P(RT.data_ptr()), ctypes.c_float(10.0),
                                 P(xyz.data_ptr()), P(valid.data_ptr()), P(ws.data_ptr()), P(st))
    assert rc == 0
    return out, p, xyz, valid


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def frames(b, h, w, seed, kind="uniform"):
    g = torch.Generator(device="cuda").manual_seed(seed)
    if kind == "uniform":
        d = torch.rand((b, h, w), device="cuda", generator=g) * 4 + 0.5
    elif kind == "wall":      # most pixels within a few cm: one level-1 bin holds most values
        d = 2.0 + 0.01 * torch.rand((b, h, w), device="cuda", generator=g)
    elif kind == "ties":      # heavy ties (mm-quantised, as a u16 / 1000 depth map)
        d = torch.round((torch.rand((b, h, w), device="cuda", generator=g) * 4 + 0.5) * 1000) / 1000
    else:                     # wide range incl. tiny and huge values
        d = torch.exp(torch.randn((b, h, w), device="cuda", generator=g) * 4)
    d[torch.rand((b, h, w), device="cuda", generator=g) < 0.05] = 0
    d[torch.rand((b, h, w), device="cuda", generator=g) < 0.01] = float("nan")
    return d


print("shape            new_us   GB/s   frac   old_us  (bp: +back-projection, new / old)")
SHAPES = [(8, 480, 640), (192, 480, 640), (8, 256, 192)]
if os.environ.get("BF_DS_SHAPE"):     # one shape only (per-kernel profiles)
    SHAPES = [tuple(int(v) for v in os.environ["BF_DS_SHAPE"].split("x"))]
    old = None
for b, h, w in SHAPES:
    d = frames(b, h, w, 0)
    n = b * h * w
    t_new = timed(lambda: _lib.depth_standardize(d))
    K = torch.tensor([[574.5, 0, 322.5], [0, 577.6, 238.6], [0, 0, 1]], device="cuda").expand(b, 3, 3).contiguous()
    RT = torch.eye(4, device="cuda").expand(b, 4, 4).contiguous()
    t_bp = timed(lambda: _lib.depth_preprocess(d, K, RT, 10.0))
    t_old = timed(lambda: run_old(d)) if old else float("nan")
    t_bp_old = (timed(lambda: run_old_bp(d, K, RT)) if old is not None and hasattr(old, "bf_depth_preprocess")
                else float("nan"))
    gbs = 8.0 * n / (t_new * 1e-6) / 1e9
    gbs_bp = 21.0 * n / (t_bp * 1e-6) / 1e9
    print(f"{b:3d}x{h}x{w}  {t_new:8.1f} {gbs:6.0f} {gbs / 8000:6.3f} {t_old:8.1f}   bp {t_bp:7.1f} us "
          f"{gbs_bp:6.0f} GB/s {gbs_bp / 8000:.3f} / old {t_bp_old:7.1f} us", flush=True)

if old:
    bad = 0
    for kind in ("uniform", "wall", "ties", "wide"):
        for seed in range(4):
            d = frames(16, 480, 640, 100 + seed, kind)
            a, pa = _lib.depth_standardize(d)
            o, po = run_old(d)
            same_p = torch.equal(pa, po)
            same_o = torch.equal(a, o)
            if hasattr(old, "bf_depth_preprocess"):
                K = torch.tensor([[574.5, 0, 322.5], [0, 577.6, 238.6], [0, 0, 1]], device="cuda").expand(16, 3, 3).contiguous()
                RT = torch.eye(4, device="cuda").expand(16, 4, 4).contiguous()
                nb = _lib.depth_preprocess(d, K, RT, 10.0)
                ob = run_old_bp(d, K, RT)
                def bits(x):
                    return x.reshape(-1).view(torch.int32) if x.dtype == torch.float32 else x.reshape(-1).to(torch.uint8)
                same_o = same_o and all(torch.equal(bits(x), bits(y)) for x, y in zip(nb, ob))
            if not (same_p and same_o):
                bad += 1
                dp = (pa - po).abs().max().item()
                print(f"A/B {kind} seed {seed}: params equal {same_p} (max |d| {dp:.3g}), out equal {same_o}")
    print("A/B vs the round-2 kernel:", "all bit-identical" if bad == 0 else f"{bad} cases differ")
