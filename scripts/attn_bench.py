"""Attention microbenchmark on the path's shapes (TFLOP/s of 4*Sq*Sk*D per head), kernel variants
(_lib.set_knobs(attn_variant=...)) interleaved in one process, vs torch SDPA; max |err| vs SDPA in fp32."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

SHAPES = [("clip", 128, 16, 257, 80), ("cutr_win", 72, 12, 512, 64), ("cutr_glob", 8, 12, 1600, 64)]
variants = [int(v) for v in sys.argv[1:]] or [0, 1]
L = _lib.lib()
dev = torch.device("cuda")


def timeit(f, iters=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for name, B, H, S, D in SHAPES:
    qkv = torch.randn(B * S, 3 * H * D, device=dev).bfloat16()
    o = torch.empty(B * S, H * D, device=dev, dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    f = lambda: _lib.attention(q, k, v, o, B, H, S, S, D, D ** -0.5)
    qq = q.view(B, S, H, D).transpose(1, 2)
    kk = k.view(B, S, H, D).transpose(1, 2)
    vv = v.view(B, S, H, D).transpose(1, 2)
    ref = torch.nn.functional.scaled_dot_product_attention(qq[:4].float(), kk[:4].float(), vv[:4].float())
    ref = ref.transpose(1, 2).reshape(4 * S, H * D)
    fl = 4.0 * B * H * S * S * D
    msg = f"{name:10s} B={B} H={H} S={S} D={D}:"
    times = {vv_: [] for vv_ in variants}
    for rnd in range(3):
        for var in variants:
            _lib.set_knobs(attn_variant=var)
            times[var].append(timeit(f))
    first = None
    for var in variants:
        _lib.set_knobs(attn_variant=var)
        o.zero_()
        f()
        torch.cuda.synchronize()
        err = (o[:4 * S].float() - ref).abs().max().item()
        ms = sorted(times[var])[1]
        msg += f" | v{var} {ms*1e3:7.1f} us {fl/ms/1e9:6.1f} TF/s err {err:.1e}"
        if first is None:
            first = o.clone()
        else:
            # rows that differ from the first variant (bit for bit), max |diff|
            nd = (o != first).any(dim=1).sum().item()
            msg += f" neq_rows {nd} maxd {(o.float() - first.float()).abs().max().item():.1e}"
    mt = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv))
    msg += f" | sdpa {mt*1e3:7.1f} us {fl/mt/1e9:6.1f} TF/s"
    print(msg, flush=True)
