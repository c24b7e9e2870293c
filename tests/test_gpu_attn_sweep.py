"""Seeded random sweep of the attention entry points against torch SDPA in fp32: every dispatch
branch of bf_attention_bf16 (2-wave workgroups for <= 64 queries, 9-wave one-workgroup heads for
257..288 queries (4-wave tiles at head dim 80), 8-wave ones (4-wave tiles at head dims 64 and 80)
for 129..256, 8-wave 256-query tiles for 449..512 at head dim 64, 4-wave 128-query tiles
otherwise), head dims 32 / 64 / 80 / 128, sk != sq and ragged
lengths (the masked tail tile), an output row map, the fp8 output and the causal form; and the
bit-identity of the 4 / 8 / 9-wave forms of the 129..288-query range."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    yield _lib


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _qkv(B, H, sq, sk, D, g, mult=1.0):
    W = H * D
    q = (torch.randn(B * sq, W, device="cuda", generator=g) * mult).bfloat16()
    k = (torch.randn(B * sk, W, device="cuda", generator=g) * mult).bfloat16()
    v = torch.randn(B * sk, W, device="cuda", generator=g).bfloat16()
    return q, k, v


def _ref(q, k, v, B, H, sq, sk, D, causal=False):
    qq = q.float().view(B, sq, H, D).transpose(1, 2)
    kk = k.float().view(B, sk, H, D).transpose(1, 2)
    vv = v.float().view(B, sk, H, D).transpose(1, 2)
    o = F.scaled_dot_product_attention(qq, kk, vv, is_causal=causal)
    return o.transpose(1, 2).reshape(B * sq, H * D)


def _cases(n=24, seed=3):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        D = [32, 64, 80, 128][i % 4]
        sq = int(rng.choice([int(rng.integers(1, 65)), int(rng.integers(161, 289)), int(rng.integers(65, 700))]))
        sk = sq if rng.integers(0, 2) else int(rng.integers(1, 900))
        if D == 128:
            sq = int(rng.integers(65, 400))         # head_dim 128: the 4-wave kernel only
        B, H = int(rng.integers(1, 5)), int(rng.integers(1, 9))
        out.append((B, H, sq, sk, D, float(rng.choice([1.0, 3.0]))))
    return out


@pytest.mark.parametrize("B,H,sq,sk,D,mult", _cases())
def test_attention_dispatch_sweep(L, B, H, sq, sk, D, mult):
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + H * 100 + sq + sk + D)
    q, k, v = _qkv(B, H, sq, sk, D, g, mult)
    o = torch.zeros(B * sq, H * D, device="cuda", dtype=torch.bfloat16)
    L.attention(q, k, v, o, B, H, sq, sk, D, D ** -0.5)
    torch.cuda.synchronize()
    assert rel_err(o, _ref(q, k, v, B, H, sq, sk, D)) < 1e-2, (B, H, sq, sk, D, mult)


@pytest.mark.parametrize("sq", [2304, 3136, 4096])
def test_attention_large_global_blocks(L, sq):
    """CuTR global blocks at square pads 768 / 896 / 1024 (preprocessor.py:86, vit.py:482):
    (pad / 16)^2 tokens, 12 heads of 64; B = 2 frames"""
    B, H, D = 2, 12, 64
    g = torch.Generator(device="cuda").manual_seed(sq)
    q, k, v = _qkv(B, H, sq, sq, D, g, 3.0)
    o = torch.zeros(B * sq, H * D, device="cuda", dtype=torch.bfloat16)
    L.attention(q, k, v, o, B, H, sq, sq, D, D ** -0.5)
    torch.cuda.synchronize()
    assert rel_err(o, _ref(q, k, v, B, H, sq, sq, D)) < 1e-2, sq


@pytest.mark.parametrize("seed", range(4))
def test_attention_omap_sweep(L, seed):
    """output rows through o_map (the window attention's token-order write-back, pad queries
    dropped): mapped rows match, unmapped rows untouched"""
    rng = np.random.default_rng(50 + seed)
    B, H, D = int(rng.integers(1, 4)), int(rng.integers(1, 6)), [64, 80][seed % 2]
    sq = int(rng.integers(100, 600))
    g = torch.Generator(device="cuda").manual_seed(seed)
    q, k, v = _qkv(B, H, sq, sq, D, g)
    rows = B * sq + 13
    omap = torch.randperm(rows, device="cuda", generator=g)[:B * sq].int()
    omap[torch.rand(B * sq, device="cuda", generator=g) < 0.15] = -1
    o = torch.zeros(rows, H * D, device="cuda", dtype=torch.bfloat16)
    L.attention(q, k, v, o, B, H, sq, sq, D, D ** -0.5, o_bs=0, o_map=omap)
    torch.cuda.synchronize()
    ref = _ref(q, k, v, B, H, sq, sq, D)
    keep = omap >= 0
    assert rel_err(o[omap[keep].long()], ref[keep]) < 1e-2
    untouched = torch.ones(rows, dtype=torch.bool, device="cuda")
    untouched[omap[keep].long()] = False
    assert not o[untouched].float().abs().sum().item()


@pytest.mark.parametrize("seed", range(4))
def test_attention_fp8out_and_causal_sweep(L, seed):
    rng = np.random.default_rng(70 + seed)
    B, H, D = int(rng.integers(1, 4)), int(rng.integers(1, 9)), [64, 80][seed % 2]
    s = int(rng.choice([int(rng.integers(161, 289)), int(rng.integers(2, 160))]))
    g = torch.Generator(device="cuda").manual_seed(100 + seed)
    q, k, v = _qkv(B, H, s, s, D, g)
    ref = _ref(q, k, v, B, H, s, s, D)
    oqs = 16.0
    o8 = torch.zeros(B * s, H * D, device="cuda", dtype=L.FP8)
    L.attention_fp8out(q, k, v, o8, B, H, s, s, D, D ** -0.5, oqs)
    oc = torch.zeros(B * s, H * D, device="cuda", dtype=torch.bfloat16)
    L.attention_causal(q, k, v, oc, B, H, s, D, D ** -0.5)
    torch.cuda.synchronize()
    assert rel_err(o8.float() / oqs, ref) < 6e-2, ("fp8", B, H, s, D)
    assert rel_err(oc, _ref(q, k, v, B, H, s, s, D, causal=True)) < 1e-2, ("causal", B, H, s, D)


@pytest.mark.parametrize("D,sq,sk", [(64, 256, 256), (64, 256, 512), (80, 200, 333), (32, 129, 129),
                                     (64, 161, 70), (80, 257, 257), (64, 270, 300), (80, 288, 100),
                                     (64, 512, 512), (64, 470, 600)])
def test_attention_workgroup_forms_bit_identical(L, D, sq, sk):
    """129..288 queries (and 449..512 at head dim 64) run on 4-, 8- or 9-wave workgroups
    (bf_attention_bf16_ex variants 28 / 29 / 30 / 31 / 33; the default picks by head dim and query count; a 4-wave tile's empty waves skip the MFMA
    work): every query's key order and tile order is the same, so every form gives the same bits"""
    B, H = 3, 4
    g = torch.Generator(device="cuda").manual_seed(D * 7 + sq + sk)
    q, k, v = _qkv(B, H, sq, sk, D, g, 3.0)
    outs = []
    for var in (6, 28, 29, 30, 31, 33):
        o = torch.zeros(B * sq, H * D, device="cuda", dtype=torch.bfloat16)
        L.attention(q, k, v, o, B, H, sq, sk, D, D ** -0.5, variant=var)
        torch.cuda.synchronize()
        outs.append(o)
    assert rel_err(outs[0], _ref(q, k, v, B, H, sq, sk, D)) < 1e-2
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("D", [64, 80])
def test_attention_fp8out_forms_bit_identical(L, D):
    """the fp8-output attention at 257 queries: 4-wave tiles at D = 80 (the CLIP fp8 engine's
    shape), 9 waves under variant 28 -- the same bits"""
    B, H, s = 3, 4, 257
    g = torch.Generator(device="cuda").manual_seed(D)
    q, k, v = _qkv(B, H, s, s, D, g, 3.0)
    outs = []
    for var in (6, 28):
        o8 = torch.zeros(B * s, H * D, device="cuda", dtype=L.FP8)
        L.attention_fp8out(q, k, v, o8, B, H, s, s, D, D ** -0.5, 16.0, variant=var)
        torch.cuda.synchronize()
        outs.append(o8.view(torch.uint8))
    assert rel_err(outs[0].view(L.FP8).float() / 16.0, _ref(q, k, v, B, H, s, s, D)) < 6e-2
    assert torch.equal(outs[0], outs[1])
