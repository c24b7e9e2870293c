"""Probe: k_attn4 variants (scripts/probe/attn4.hip builds) against the shipped attention on CLIP
ViT-H/14 heads (128 crops x 16 heads, 257 tokens, head_dim 80, token-major QKV): rows 0..255 must be
bit-identical to the shipped kernel, row 256 within bf16 rounding."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

B, H, S, D = 128, 16, 257, 80
W = H * D
VARIANTS = sys.argv[1:] or ["pin"]
PS = {v: ctypes.CDLL(os.path.join(ROOT, f"boxfusion_amd/_build/probe/attn4_{v}.so")) for v in VARIANTS}
L = _lib.lib()
vp = ctypes.c_void_p
torch.manual_seed(0)
qkv = (torch.randn(B * S, 3 * W, device="cuda") * 1.5).bfloat16()
o1 = torch.empty(B * S, W, device="cuda", dtype=torch.bfloat16)
o2 = torch.empty_like(o1)
st = vp(torch.cuda.current_stream().cuda_stream)
LL = ctypes.c_longlong
args = lambda o, hd=(): (vp(qkv.data_ptr()), vp(qkv.data_ptr() + 2 * W), vp(qkv.data_ptr() + 4 * W), vp(o.data_ptr()),
                         B, H, S, S, *hd, 3 * W, 3 * W, 3 * W, W, LL(S * 3 * W), LL(S * 3 * W), LL(S * 3 * W), LL(S * W),
                         ctypes.c_float(D ** -0.5), st)


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


fns = {"shipped": lambda: L.bf_attention_bf16(*args(o1, (D,)))}
assert fns["shipped"]() == 0
torch.cuda.synchronize()
for v, P in PS.items():
    fns[v] = (lambda P=P: P.attn4_launch(*args(o2)))
    o2.zero_()
    assert fns[v]() == 0, v
    torch.cuda.synchronize()
    a = o1.view(B, S, W)
    c = o2.view(B, S, W)
    eq = torch.equal(a[:, :256], c[:, :256])
    d256 = (a[:, 256].float() - c[:, 256].float()).abs().max().item()
    dall = (a.float() - c.float()).abs().max().item()
    print(f"{v}: rows0-255 bitequal {eq}, row256 maxdiff {d256:.3g}, all maxdiff {dall:.3g}", flush=True)
fl = 4.0 * B * H * S * S * D
res = {k: [] for k in fns}
for _ in range(3):
    for k, f in fns.items():
        res[k].append(bench(f))
for k, v in res.items():
    t = sorted(v)[1]
    print(f"{k:10s} {t:7.1f} us  {fl / t / 1e6:6.0f} TF  frac {fl / t / 1e6 / 2500:.3f}", flush=True)
