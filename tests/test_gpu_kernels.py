"""MFMA / vision kernels vs plain PyTorch fp32 references of the same ops (GPU only).
Tolerances are for bf16 operands with f32 accumulation."""
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


@pytest.mark.parametrize("bm", [0, 160, 192, 224, 256])
@pytest.mark.parametrize("M,N,K,out_bf16,resid,bias", [
    (32896, 1280, 1280, False, "inplace", True),    # CLIP out_proj + residual
    (4112, 1280, 5120, False, "inplace", True),      # CLIP c_proj + residual (16 crops)
    (4112, 1280, 1280, False, "separate", True),
    (4112, 3840, 1280, True, None, True),            # qkv
    (12800, 768, 3072, False, "inplace", True),      # CuTR global fc2 + residual
    (1000, 768, 768, False, None, False),
    (257, 1280, 1280, True, None, False)])
def test_gemm_tile_rows_vs_torch(L, M, N, K, out_bf16, resid, bias, bm):
    """bf_gemm_bf16 at every tile height of k_gemm256q (0 = the per-shape model; 256 with an f32
    residual = k_gemm256p) against torch fp32 on the residual / plain linear forms; every height
    gives the same K-order MFMA chain, so the k_gemm256q heights agree bit for bit."""
    pl = dict(tile_rows=bm)
    if True:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
        b = torch.randn(N, device="cuda", generator=g) if bias else None
        r = torch.randn(M, N, device="cuda", generator=g)
        ref = a.float() @ w.float().T + (b if bias else 0)
        if resid:
            ref = ref + r
        if resid == "inplace":
            out = r.clone()
            L.gemm(a, w, b, resid=out, out=out, plan=pl)
        elif resid == "separate":
            out = torch.empty(M, N, device="cuda")
            L.gemm(a, w, b, resid=r, out=out, plan=pl)
        else:
            out = L.gemm(a, w, b, out_dtype=torch.bfloat16 if out_bf16 else torch.float32, plan=pl)
        torch.cuda.synchronize()
        assert rel_err(out, ref) < (8e-3 if out_bf16 else 2e-5 * math.sqrt(K / 64) + 1e-5), (M, N, K)
        if bm in (160, 224) and not (resid and bm == 256):
            p2 = dict(tile_rows=192)
            if resid == "inplace":
                out2 = r.clone()
                L.gemm(a, w, b, resid=out2, out=out2, plan=p2)
            elif resid == "separate":
                out2 = torch.empty(M, N, device="cuda")
                L.gemm(a, w, b, resid=r, out=out2, plan=p2)
            else:
                out2 = L.gemm(a, w, b, out_dtype=torch.bfloat16 if out_bf16 else torch.float32, plan=p2)
            torch.cuda.synchronize()
            assert torch.equal(out, out2), "tile height changed a value"


@pytest.mark.parametrize("M,N,K,act,out_bf16,resid,row_map", [
    (128, 1024, 1280, None, False, None, False),          # CLIP output projection (class tokens)
    (128, 5120, 1280, "gelu", True, None, False),         # cls-only last block fc1 + GELU
    (128, 1280, 5120, None, False, "inplace", True),      # cls-only last block fc2 + residual, row map
    (100, 1280, 1280, None, False, "separate", True),
    (200, 512, 768, "relu", True, None, False),
    (7, 64, 256, None, False, None, False)])
def test_gemm_skinny_vs_torch(L, M, N, K, act, out_bf16, resid, row_map):
    """few-row GEMMs (k_gemm_skinny: 8 waves split K, partial tiles summed in wave order)"""
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    ref = a.float() @ w.float().T + b
    if act == "gelu":
        ref = F.gelu(ref)
    elif act == "relu":
        ref = F.relu(ref)
    rows = M + 9 if row_map else M
    rm = (torch.randperm(rows, device="cuda", generator=g)[:M].int() if row_map else None)
    r = torch.randn(rows, N, device="cuda", generator=g)
    dt = torch.bfloat16 if out_bf16 else torch.float32
    if resid == "inplace":
        out = r.clone()
        L.gemm(a, w, b, act=act, resid=out, out=out, row_map=rm)
    elif resid == "separate":
        out = torch.zeros(rows, N, device="cuda")
        L.gemm(a, w, b, act=act, resid=r, out=out, row_map=rm)
    else:
        out = torch.zeros(rows, N, device="cuda", dtype=dt)
        L.gemm(a, w, b, act=act, out=out, row_map=rm)
    torch.cuda.synchronize()
    orow = rm.long() if rm is not None else torch.arange(M, device="cuda")
    want = ref + (r[orow] if resid else 0)
    assert rel_err(out[orow], want) < (8e-3 if out_bf16 else 2e-5 * math.sqrt(K / 64) + 1e-5)
    if row_map:      # rows outside the map untouched
        mask = torch.ones(rows, dtype=torch.bool, device="cuda")
        mask[orow] = False
        base = r if resid == "inplace" else torch.zeros_like(out)
        assert torch.equal(out[mask], base[mask])
    o1 = out.clone()
    if resid == "inplace":
        out = r.clone()
        L.gemm(a, w, b, act=act, resid=out, out=out, row_map=rm)
        torch.cuda.synchronize()
        assert torch.equal(out, o1), "not deterministic"


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(1600, 2304, 768), (257, 1280, 1280), (4112, 5120, 1280),
                                   (100, 4, 256), (130, 136, 64)])
def test_gemm_plain(L, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    ref = a.float() @ w.float().T + b
    out = L.gemm(a, w, b, out_dtype=torch.float32)
    assert rel_err(out, ref) < 1e-5
    outb = L.gemm(a, w, b)
    assert rel_err(outb, ref) < 5e-3


def test_gemm_gelu_resid_rowmap(L):
    g = torch.Generator(device="cuda").manual_seed(3)
    M, N, K = 300, 384, 192
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    resid = torch.randn(M + 10, N, device="cuda", generator=g)
    perm = torch.randperm(M + 10, device="cuda", generator=g)[:M].int()
    perm[::7] = -1
    out = resid.clone()
    L.gemm(a, w, b, act="gelu", resid=out, out=out, row_map=perm)
    ref = resid.clone()
    y = F.gelu(a.float() @ w.float().T + b)
    keep = perm >= 0
    ref[perm[keep].long()] += y[keep]
    assert rel_err(out, ref) < 1e-5
    # broadcast residual table (pos-embed style)
    tab = torch.randn(100, N, device="cuda", generator=g)
    o2 = L.gemm(a, w, b, resid=tab, resid_mod=100, out_dtype=torch.float32)
    r2 = a.float() @ w.float().T + b + tab[torch.arange(M, device="cuda") % 100]
    assert rel_err(o2, r2) < 1e-5


@pytest.mark.parametrize("small", [False, True])
@pytest.mark.parametrize("shape", [(3000, 2816, 320), (8292, 4352, 192), (8292, 4352, 64)])
@pytest.mark.parametrize("act,out_bf16,use_resid", [(None, True, False), ("gelu", True, False),
                                                   (None, False, True), ("relu", False, False)])
def test_gemm_large_tiles(L, small, shape, act, out_bf16, use_resid):
    """shapes that select the persistent 256x256 8-wave kernel (and, forced, the 128x128 one):
    fewer / more tiles than CUs (the K-tile ring crosses tiles), a single K-tile, partial M/N
    tiles, bias, activation, residual + row scatter."""
    from boxfusion_amd._lib import lib
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = shape
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    y = a.float() @ w.float().T + b
    if act == "gelu":
        y = F.gelu(y)
    elif act == "relu":
        y = F.relu(y)
    pl = dict(kernel=1 if small else 0)
    if use_resid:
        resid = torch.randn(M + 40, N, device="cuda", generator=g)
        perm = torch.randperm(M + 40, device="cuda", generator=g)[:M].int()
        perm[::5] = -1
        out = resid.clone()
        L.gemm(a, w, b, act=act, resid=out, out=out, row_map=perm, plan=pl)
        ref = resid.clone()
        keep = perm >= 0
        ref[perm[keep].long()] += y[keep]
        assert rel_err(out, ref) < 1e-5
    else:
        out = L.gemm(a, w, b, act=act, out_dtype=torch.bfloat16 if out_bf16 else torch.float32, plan=pl)
        assert rel_err(out, y) < (5e-3 if out_bf16 else 1e-5)


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("shape", [(3000, 2816, 320), (8292, 1280, 640), (600, 384, 64)])
@pytest.mark.parametrize("inplace,out_bf16", [(True, False), (False, False), (False, True)])
def test_gemm_resid_persistent(L, variant, shape, inplace, out_bf16):
    """residual without a row map (the accumulator-initialised path of k_gemm256p) and the
    schedule variants: in place (x += proj(h)) and out of place, partial tiles, f32 and bf16 out"""
    from boxfusion_amd._lib import lib
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = shape
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    resid = torch.randn(M, N, device="cuda", generator=g)
    ref = resid + a.float() @ w.float().T + b
    pl = dict(variant=variant)
    if inplace:
        out = resid.clone()
        L.gemm(a, w, b, resid=out, out=out, plan=pl)
    else:
        out = L.gemm(a, w, b, resid=resid, out_dtype=torch.bfloat16 if out_bf16 else torch.float32, plan=pl)
    assert rel_err(out, ref) < (5e-3 if out_bf16 else 1e-5)
    # a second call on the same output buffer (persistent walk state must not leak)
    if not inplace:
        out2 = L.gemm(a, w, b, resid=resid, out_dtype=out.dtype, plan=pl)
        assert torch.equal(out2, out)


@pytest.mark.parametrize("shape", [(3000, 2816, 320), (8292, 1280, 640), (600, 384, 192),
                                   (4112, 5120, 1280), (32896, 1280, 1280), (12800, 768, 3072)])
@pytest.mark.parametrize("kind", ["bf16", "gelu", "f32", "resid_inplace", "resid", "nobias"])
def test_gemm_overlapped_epilogue(L, shape, kind):
    """k_gemm256q (variant 6, every eligible shape; 5, the default, for bf16 outputs: the epilogue of every 64x32 quadrant spread over the phases around
    the tile boundary, transposed accumulators, permlane-widened bf16 stores) vs fp32 torch and vs
    the k_gemm256p default on the same operands: partial M / N tiles, 3..48 K-tiles, bias / no
    bias, GELU, f32 / bf16 out, residual in place and out of place"""
    from boxfusion_amd._lib import lib
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    M, N, K = shape
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = None if kind == "nobias" else torch.randn(N, device="cuda", generator=g)
    resid = torch.randn(M, N, device="cuda", generator=g) if kind.startswith("resid") else None
    y = a.float() @ w.float().T + (b if b is not None else 0.0)
    act = "gelu" if kind == "gelu" else None
    if act:
        y = F.gelu(y)
    if resid is not None:
        y = y + resid
    od = torch.bfloat16 if kind in ("bf16", "gelu", "nobias") else torch.float32

    def run(variant):
        pl = dict(variant=variant)
        if kind == "resid_inplace":
            out = resid.clone()
            L.gemm(a, w, b, resid=out, out=out, plan=pl)
        else:
            out = torch.full((M, N), float("nan"), device="cuda", dtype=od)
            L.gemm(a, w, b, act=act, resid=resid, out=out, plan=pl)
        torch.cuda.synchronize()
        return out
    out_q, out_p = run(6), run(1)
    assert torch.isfinite(out_q).all(), "rows / columns left unwritten"
    tol = 5e-3 if od == torch.bfloat16 else 1e-5
    assert rel_err(out_q, y) < tol
    assert rel_err(out_q, out_p) < (2e-3 if od == torch.bfloat16 else 1e-6)
    # out-of-range rows / columns untouched: a padded output view keeps its sentinels
    if kind == "bf16":
        big = torch.full((M + 3, N + 8), 7.0, device="cuda", dtype=od)
        L.gemm(a, w, b, out=big[:M, :N], plan=dict(variant=6))
        assert torch.equal(big[:M, :N], out_q)
        assert (big[M:] == 7.0).all() and (big[:, N:] == 7.0).all()


def _attn_ref(q, k, v, B, H, S, D, scale):
    qq = q.float().view(B, S, H, D).transpose(1, 2)
    kk = k.float().view(B, -1, H, D).transpose(1, 2)
    vv = v.float().view(B, -1, H, D).transpose(1, 2)
    p = torch.softmax((qq * scale) @ kk.transpose(-1, -2), dim=-1)
    return (p @ vv).transpose(1, 2).reshape(B * S, H * D)


@pytest.mark.parametrize("variant", [6, 27])
@pytest.mark.parametrize("B,H,S,D", [(9, 12, 512, 64), (2, 12, 1600, 64), (3, 16, 257, 80),
                                     (2, 8, 302, 32), (1, 4, 70, 128), (2, 4, 200, 64),
                                     (2, 4, 288, 80), (2, 2, 257, 128), (3, 12, 320, 64),
                                     (3, 12, 272, 64), (2, 16, 256, 80), (1, 3, 64, 64)])
def test_attention(L, B, H, S, D, variant):
    g = torch.Generator(device="cuda").manual_seed(B * S + D)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    scale = D ** -0.5
    L.attention(q, k, v, o, B, H, S, S, D, scale, variant=variant)
    ref = _attn_ref(q, k, v, B, H, S, D, scale)
    assert rel_err(o, ref) < 1e-2


@pytest.mark.parametrize("B,H,S,D", [(3, 16, 257, 80), (2, 4, 288, 80), (3, 12, 272, 64),
                                     (2, 16, 256, 80), (2, 4, 200, 64), (2, 3, 160, 80)])
def test_attention_short_heads_row_stores(L, B, H, S, D):
    """short heads (one 9-wave workgroup per (batch, head)): the default LDS-staged whole-row
    output stores (6) write exactly what the per-lane fragment stores (27) write"""
    g = torch.Generator(device="cuda").manual_seed(B * S + D + 12)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    outs = {}
    for var in (6, 27):
        o = torch.full((B * S, H * D), float("nan"), device="cuda", dtype=torch.bfloat16)
        L.attention(q, k, v, o, B, H, S, S, D, D ** -0.5, variant=var)
        outs[var] = o
    assert torch.equal(outs[27], outs[6])
    assert rel_err(outs[6], _attn_ref(q, k, v, B, H, S, D, D ** -0.5)) < 1e-2


@pytest.mark.parametrize("B,H,S,D,scatter", [(9, 12, 512, 64, True), (2, 12, 1600, 64, False),
                                               (2, 8, 302, 32, False), (3, 12, 320, 64, True),
                                               (2, 4, 600, 80, True)])
def test_attention_row_stores_equal_fragment_stores(L, B, H, S, D, scatter):
    """the default epilogue (rows staged in LDS, stored as whole head rows; 4-wave workgroups reuse
    the K ring after a barrier) writes exactly the rows of the per-lane fragment stores
    (variant 27), also through an o_map row scatter with dropped rows (the CuTR window layout)"""
    g = torch.Generator(device="cuda").manual_seed(B * S + D + 27)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    om = None
    if scatter:
        perm = torch.randperm(B * S, device="cuda", generator=g).to(torch.int32)
        om = torch.where(torch.arange(B * S, device="cuda") % 7 == 3, torch.full_like(perm, -1), perm)
    outs = []
    for var in (27, 6):
        o = torch.full((B * S, H * D), float("nan"), device="cuda", dtype=torch.bfloat16)
        L.attention(q, k, v, o, B, H, S, S, D, D ** -0.5, o_map=om, variant=var)
        outs.append(o)
    assert torch.equal(outs[1].nan_to_num(7.0), outs[0].nan_to_num(7.0))


@pytest.mark.parametrize("sq,D", [(1, 80), (1, 64), (40, 80), (64, 32)])
def test_attention_few_queries(L, sq, D):
    """<= 64 queries against 257 keys (CLIP's last block: the class token of every crop), the
    queries a strided subset of the token rows (q_bs = S rows), compact output rows"""
    B, H, S = 24, 16, 257
    g = torch.Generator(device="cuda").manual_seed(sq * D)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", generator=g).bfloat16()
    rs = qkv.stride(0)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * sq, H * D, device="cuda", dtype=torch.bfloat16)
    L.attention(q, k, v, o, B, H, sq, S, D, D ** -0.5, q_bs=S * rs, k_bs=S * rs, v_bs=S * rs,
                o_bs=sq * o.stride(0))
    qh = q.view(B, S, H, D)[:, :sq].float().transpose(1, 2)
    kh = k.reshape(B, S, H, D).float().transpose(1, 2)
    vh = v.reshape(B, S, H, D).float().transpose(1, 2)
    ref = torch.softmax(qh @ kh.transpose(-2, -1) * D ** -0.5, -1) @ vh
    assert rel_err(o, ref.transpose(1, 2).reshape(B * sq, H * D)) < 1e-2


@pytest.mark.parametrize("D", [64, 80])
@pytest.mark.parametrize("spike", [4.0, 1.6, 1.25])
def test_attention_forced_rescale(L, D, spike):
    """a spike key late in the sequence forces the online-softmax rescale branch (deferred-max
    kernel: a max growth beyond the threshold rescales, smaller growth is carried in P <= 2^8);
    each lane's query meets the spike in a different tile"""
    B, H, S = 1, 2, 300
    g = torch.Generator(device="cuda").manual_seed(11)
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", generator=g)
    qkv[250, H * D:2 * H * D] = qkv[0, :H * D] * spike
    qkv[130, H * D:2 * H * D] = qkv[1, :H * D] * spike * 0.8
    qkv = qkv.bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    L.attention(q, k, v, o, B, H, S, S, D, D ** -0.5)
    assert rel_err(o, _attn_ref(q, k, v, B, H, S, D, D ** -0.5)) < 1e-2


@pytest.mark.parametrize("C", [768, 1280, 256, 384])
def test_layernorm(L, C):
    g = torch.Generator(device="cuda").manual_seed(C)
    x = torch.randn(333, C, device="cuda", generator=g) * 3 + 1
    w = torch.randn(C, device="cuda", generator=g)
    b = torch.randn(C, device="cuda", generator=g)
    out = L.layernorm(x, w, b, 1e-6)
    ref = F.layer_norm(x, (C,), w, b, 1e-6)
    assert rel_err(out, ref) < 5e-3


def test_im2col_rgb8_and_f32(L):
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.randint(0, 256, (2, 480, 640, 3), device="cuda", dtype=torch.uint8, generator=g)
    mean, std = [123.675, 116.28, 103.53], [58.395, 57.12, 57.375]
    a = L.im2col_rgb8(img, 640, 16, mean, std)
    x = (img.permute(0, 3, 1, 2).float() - torch.tensor(mean, device="cuda").view(1, 3, 1, 1)) \
        / torch.tensor(std, device="cuda").view(1, 3, 1, 1)
    x = F.pad(x, (0, 0, 0, 160))
    ref = F.unfold(x, 16, stride=16).transpose(1, 2).reshape(-1, 768)
    assert torch.equal(a, ref.bfloat16())
    d = torch.rand(2, 480, 640, device="cuda", generator=g)
    ad = L.im2col_f32(d, 640, 16)
    refd = F.unfold(F.pad(d[:, None], (0, 0, 0, 160)), 16, stride=16).transpose(1, 2).reshape(-1, 256)
    assert torch.equal(ad, refd.bfloat16())


def test_crop_resize_im2col(L):
    g = torch.Generator(device="cuda").manual_seed(1)
    img = torch.randint(0, 256, (2, 480, 640, 3), device="cuda", dtype=torch.uint8, generator=g)
    boxes = torch.tensor([[10, 20, 200, 150], [0, 0, 640, 480], [300, 300, 301, 310],
                          [5, 5, 5, 40]], device="cuda", dtype=torch.int32)
    idx = torch.tensor([0, 1, 1, 0], device="cuda", dtype=torch.int32)
    mean = [0.48145466, 0.4578275, 0.40821073]
    std = [0.26862954, 0.26130258, 0.27577711]
    out = L.crop_resize_im2col(img, boxes, idx, 224, 14, mean, std, 640)
    assert out.shape == (4 * 256, 640)
    assert torch.all(out[:, 588:] == 0)
    # reference: torch bilinear (align_corners=False, no antialias) on the crop
    for n in range(3):
        x1, y1, x2, y2 = boxes[n].tolist()
        crop = img[idx[n], y1:y2, x1:x2].permute(2, 0, 1)[None].float()
        r = F.interpolate(crop, size=(224, 224), mode="bilinear", align_corners=False)
        r = (r / 255 - torch.tensor(mean, device="cuda").view(1, 3, 1, 1)) / \
            torch.tensor(std, device="cuda").view(1, 3, 1, 1)
        ref = F.unfold(r, 14, stride=14).transpose(1, 2).reshape(-1, 588)
        got = out[n * 256:(n + 1) * 256, :588].float()
        assert (got - ref).abs().max().item() < 0.05
    empty = ((0 - torch.tensor(mean, device="cuda")) / torch.tensor(std, device="cuda"))
    empty = empty.repeat_interleave(196).bfloat16().float()[None]
    assert torch.all(out[3 * 256:, :588].float() == empty)


@pytest.mark.parametrize("act,use_resid", [("gelu", False), (None, True)])
def test_gemm_balanced_grid(L, act, use_resid):
    """360 tiles of 256x256 (a last round 104/256 full) launch the balanced persistent grid
    (bf_gemm_plan.balanced): every tile is computed the same way whichever workgroup walks it, so
    the output is bit-identical to the one-block-per-CU grid, and matches the fp32 reference"""
    from boxfusion_amd._lib import lib
    g = torch.Generator(device="cuda").manual_seed(23)
    M, N, K = 10000, 2304, 128
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    resid = torch.randn(M, N, device="cuda", generator=g) if use_resid else None
    outs = []
    for bal in (0, 1):          # 0: the default balanced grid, 1: one workgroup per CU
        pl = dict(balanced=bal)
        if use_resid:
            o = resid.clone()
            L.gemm(a, w, b, resid=o, out=o, plan=pl)
        else:
            o = L.gemm(a, w, b, act=act, out_dtype=torch.bfloat16, plan=pl)
        torch.cuda.synchronize()
        outs.append(o)
    assert torch.equal(outs[0], outs[1])
    y = a.float() @ w.float().T + b
    if act == "gelu":
        y = F.gelu(y)
    if use_resid:
        y = y + resid
    assert rel_err(outs[0], y) < (5e-3 if not use_resid else 1e-5)


@pytest.mark.parametrize("force", [-1, 1])
def test_gemm_stem_rowmap_broadcast_resid(L, force):
    """the CLIP stem GEMM's combination on both tile kernels (forced):
    row map (patch row n*np + p -> token row n*S + 1 + p), broadcast residual table (pos-embed,
    resid_mod = np), no bias, f32 out -- against the old formulation P + pos scattered by torch"""
    from boxfusion_amd._lib import lib
    g = torch.Generator(device="cuda").manual_seed(29)
    crops, npch, S, W, K = 128, 256, 257, 1280, 640
    a = torch.randn(crops * npch, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(W, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    pos = torch.randn(npch, W, device="cuda", generator=g)
    row_map = (torch.arange(crops, device="cuda", dtype=torch.int32)[:, None] * S + 1
               + torch.arange(npch, device="cuda", dtype=torch.int32)[None]).reshape(-1)
    # kernel -1: the persistent 256x256 kernel (the default for this shape), 1: 128x128
    assert bool(lib().bf_gemm_large_tiles(crops * npch, W, K))
    X = torch.full((crops * S, W), 7.0, device="cuda")
    L.gemm(a, w, resid=pos, resid_mod=npch, out=X, row_map=row_map, plan=dict(kernel=force))
    ref = torch.full((crops * S, W), 7.0, device="cuda")
    P = a.float() @ w.float().T
    ref.view(crops, S, W)[:, 1:] = (P.view(crops, npch, W) + pos[None])
    assert rel_err(X, ref) < 1e-5
    assert torch.all(X.view(crops, S, W)[:, 0] == 7.0)      # class-token rows untouched


@pytest.mark.parametrize("shape", [(32896, 1280, 1280), (32896, 3840, 1280), (12800, 768, 3072), (128, 5120, 1280)])
def test_gemm_plan_budgets_two_streams(L, shape):
    """the GEMM ABI keeps no process-wide state: two streams launch the same problem concurrently
    with different CU budgets in their per-call plans (224: a rank-0 detect stream beside the
    fusion reservation; 0: every CU).  The kernel choice follows the device's CU count, only the
    persistent grid / tile height follow the budget, so both outputs are bit-identical -- and
    identical to the plan-less bf_gemm_bf16."""
    M, N, K = shape
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    torch.cuda.synchronize()
    for st, budget in ((s1, 224), (s2, 0), (s1, 96), (s2, 255)):
        o = r.clone()
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            L.gemm(a, w, b, resid=o, out=o, plan=L.GemmPlan(cu_budget=budget))
        outs.append(o)
    torch.cuda.synchronize()
    ref = r.clone()
    L.gemm(a, w, b, resid=ref, out=ref)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)
    assert rel_err(ref, a.float() @ w.float().T + b + r) < 2e-5 * math.sqrt(K / 64) + 1e-5
    # the thread-local budget of the Python wrapper goes into the plan, and is per thread
    L.set_cu_budget(160)
    try:
        o = r.clone()
        L.gemm(a, w, b, resid=o, out=o)
        torch.cuda.synchronize()
        assert torch.equal(o, ref)
        import threading
        seen = []
        th = threading.Thread(target=lambda: seen.append(L.cu_budget()))
        th.start()
        th.join()
        assert seen == [0] and L.cu_budget() == 160
    finally:
        L.set_cu_budget(0)


def test_gemm_operand_extent_capacity(L):
    """operands whose byte extent reaches 2^31 are refused (32-bit descriptors), not wrapped"""
    import ctypes
    from boxfusion_amd._lib import lib
    a = torch.empty(1, 64, device="cuda", dtype=torch.bfloat16)
    w = torch.empty(64, 64, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(1, 64, device="cuda", dtype=torch.bfloat16)
    # M = 2^24 rows at lda = 64: (M-1)*lda*2 + K*2 = 2^31 (only the extent is checked; nothing runs)
    rc = lib().bf_gemm_bf16(ctypes.c_void_p(a.data_ptr()), 64, ctypes.c_void_p(w.data_ptr()), 64,
                            None, None, 0, 0, ctypes.c_void_p(c.data_ptr()), 64, 1, None, 1 << 24, 64,
                            64, 0, None)
    assert rc == -3       # BF_ERR_CAPACITY


def test_cu_partition_placement(L):
    """the fusion reservation (first 32 mask bits) runs on 4 CUs of every XCD and the detect mask
    on the other 28 of each; a mask that leaves an XCD without CUs is not applied by the runtime
    (bench.py's old every-8th-CU set ran on every CU), so the layout is checked on the hardware"""
    from collections import Counter
    n = torch.cuda.get_device_properties(0).multi_processor_count
    if n % L.XCDS:
        pytest.skip("CU count not a multiple of the XCD count")
    det, fus = L.partition_cus(32)
    pf = L.cu_placement(L.cu_masked_stream(fus))
    pd = L.cu_placement(L.cu_masked_stream(det))
    assert len(pf) == 32 and len(pd) == n - 32
    assert not (pf & pd)
    assert set(Counter(k[0] for k in pf).values()) == {32 // L.XCDS}


@pytest.mark.parametrize("n_crops,n_cls", [(128, 473), (16, 200), (1, 1), (37, 33)])
def test_match_features_on_f32_gemm(L, n_crops, n_cls):
    """text_prompt's similarity (tools/utils.py:397-401, 486-493) on the device: (100 f) @ text^T on
    the f32 MFMA GEMM (bf_gemm_f32), then the threshold column and argmax -- against the same
    formula in float64; the class matches wherever the top two scores are apart, and the in-place
    text renormalisation still happens."""
    from boxfusion_amd.tools_utils import match_features
    g = torch.Generator(device="cuda").manual_seed(n_crops * 1000 + n_cls)
    img = torch.randn(n_crops, 1024, device="cuda", generator=g)
    text = torch.randn(n_cls, 1024, device="cuda", generator=g) * 3.0
    text_in = text.clone()
    thr = 0.0
    idx, f, mx = match_features(img, text_in, thr)
    torch.cuda.synchronize()
    fd = img.double() / img.double().norm(dim=-1, keepdim=True)
    td = text.double() / text.double().norm(dim=-1, keepdim=True)
    pd = 100.0 * fd @ td.T
    pd = torch.cat([pd, torch.full_like(pd, thr)[..., :1]], dim=-1)
    mxd, idxd = pd.max(dim=-1)
    assert torch.allclose(text_in.double(), td, atol=1e-6)      # renormalised in place
    assert torch.allclose(mx.double(), mxd, atol=2e-4)
    top2 = pd.topk(min(2, pd.shape[1]), dim=-1).values
    clear = (top2[:, 0] - top2[:, -1]) > 1e-3 if pd.shape[1] > 1 else torch.ones_like(mxd, dtype=torch.bool)
    assert torch.equal(idx[clear].cpu(), idxd[clear].cpu())


@pytest.mark.parametrize("seed", range(8))
def test_layernorm_forms_sweep(L, seed):
    """bf_layernorm's forms on the path: row map (the window partition's scatter, < 0 skipped),
    bf16 / f32 output, a strided input view, ragged M, and a large common offset (the variance
    must not cancel) -- against torch's layer_norm in float64"""
    rng = np.random.default_rng(200 + seed)
    C = int([192, 256, 384, 512, 640, 768, 1024, 1280][seed])
    M = int(rng.integers(1, 3000))
    g = torch.Generator(device="cuda").manual_seed(seed)
    base = torch.randn(M, C + 64, device="cuda", generator=g) * 2.0 + (500.0 if seed % 2 else 0.0)
    x = base[:, 32:32 + C]                          # row stride C + 64
    w = torch.randn(C, device="cuda", generator=g)
    b = torch.randn(C, device="cuda", generator=g)
    ref = F.layer_norm(x.double(), (C,), w.double(), b.double(), 1e-6)
    rows = M + 9
    rm = torch.randperm(rows, device="cuda", generator=g)[:M].int()
    rm[torch.rand(M, device="cuda", generator=g) < 0.1] = -1
    for dt, tol in ((torch.bfloat16, 5e-3), (torch.float32, 1e-5)):
        out = torch.zeros(rows, C, device="cuda", dtype=dt)
        L.layernorm(x, w, b, 1e-6, out=out, row_map=rm)
        torch.cuda.synchronize()
        keep = rm >= 0
        assert rel_err(out[rm[keep].long()], ref[keep]) < tol, (C, M, dt)
        untouched = torch.ones(rows, dtype=torch.bool, device="cuda")
        untouched[rm[keep].long()] = False
        assert not out[untouched].float().abs().sum().item()
