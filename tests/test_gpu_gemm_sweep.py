"""Seeded random sweep of bf_gemm_bf16's dispatch (skinny / 128x128 / persistent 256-wide at the
per-shape tile height) against torch fp32: ragged M and N, K multiples of 64, every epilogue form
(bf16 / f32 output, bias or none, GELU / ReLU, separate / in-place / broadcast residual, row map).
Catches a wrong result in a rarely taken path; the tolerances are those of test_gpu_kernels."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _cases(n=40, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        big = i % 3 == 0
        M = int(rng.integers(2048, 12000)) if big else int(rng.integers(1, 1500))
        N = int(rng.choice([32, 96, 256, 512, 768, 1000, 1280, 2304])) if i % 4 else int(rng.integers(1, 300)) * 8
        K = 64 * int(rng.integers(1, 48))
        act = [None, "gelu", "relu"][int(rng.integers(0, 3))]
        out_bf16 = bool(rng.integers(0, 2))
        resid = [None, "separate", "inplace", "mod"][int(rng.integers(0, 4))]
        if act is not None and resid is not None:
            resid = None
        if out_bf16 and resid is not None:
            out_bf16 = False
        row_map = bool(rng.integers(0, 4) == 0) and resid in (None, "separate")
        bias = bool(rng.integers(0, 2))
        out.append((M, N, K, act, out_bf16, resid, row_map, bias))
    return out


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    yield _lib


@pytest.mark.parametrize("M,N,K,act,out_bf16,resid,row_map,bias", _cases())
def test_gemm_dispatch_sweep(L, M, N, K, act, out_bf16, resid, row_map, bias):
    g = torch.Generator(device="cuda").manual_seed(M * 31 + N * 7 + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    ref = a.float() @ w.float().T + (b if bias else 0)
    if act == "gelu":
        ref = F.gelu(ref)
    elif act == "relu":
        ref = F.relu(ref)
    rows = M + 5 if row_map else M
    rm = torch.randperm(rows, device="cuda", generator=g)[:M].int() if row_map else None
    orow = rm.long() if rm is not None else torch.arange(M, device="cuda")
    dt = torch.bfloat16 if out_bf16 else torch.float32
    if resid == "mod":
        tab = torch.randn(17, N, device="cuda", generator=g)
        out = torch.zeros(rows, N, device="cuda", dtype=dt)
        L.gemm(a, w, b, act=act, resid=tab, resid_mod=17, out=out, row_map=rm)
        want = ref + tab[torch.arange(M, device="cuda") % 17]
    elif resid == "inplace":
        r = torch.randn(rows, N, device="cuda", generator=g)
        out = r.clone()
        L.gemm(a, w, b, act=act, resid=out, out=out, row_map=rm)
        want = ref + r[orow]
    elif resid == "separate":
        r = torch.randn(rows, N, device="cuda", generator=g)
        out = torch.zeros(rows, N, device="cuda", dtype=dt)
        L.gemm(a, w, b, act=act, resid=r, out=out, row_map=rm)
        want = ref + r[orow]
    else:
        out = torch.zeros(rows, N, device="cuda", dtype=dt)
        L.gemm(a, w, b, act=act, out=out, row_map=rm)
        want = ref
    torch.cuda.synchronize()
    tol = 8e-3 if out_bf16 else 2e-5 * math.sqrt(K / 64) + 1e-5
    assert rel_err(out[orow], want) < tol, (M, N, K, act, out_bf16, resid, row_map, bias)
    if row_map:
        mask = torch.ones(rows, dtype=torch.bool, device="cuda")
        mask[orow] = False
        assert not out[mask].any(), "rows outside the map were written"


def _fp8_cases(n=16, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        M = int(rng.integers(3000, 12000)) if i % 3 == 0 else int(rng.integers(1, 2000))
        N = 8 * int(rng.integers(1, 400))
        K = 128 * int(rng.integers(1, 24))
        kind = ["f32", "bf16", "fp8"][i % 3]
        act = "gelu" if (kind != "f32" and rng.integers(0, 2)) else None
        resid = kind == "f32" and bool(rng.integers(0, 2))
        out.append((M, N, K, kind, act, resid))
    return out


@pytest.mark.parametrize("M,N,K,kind,act,resid", _fp8_cases())
def test_gemm_fp8_dispatch_sweep(L, M, N, K, kind, act, resid):
    """bf_gemm_fp8 (k_gemm256q for bf16 outputs, k_gemm256p for f32 + residual and fp8 outputs)
    against torch on the dequantised operands"""
    g = torch.Generator(device="cuda").manual_seed(M * 13 + N + K)
    a8 = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(L.FP8)
    w8 = (torch.randn(N, K, device="cuda", generator=g) * 0.5).to(L.FP8)
    b = torch.randn(N, device="cuda", generator=g)
    sc = 1.0 / math.sqrt(K)
    ref = (a8.float() @ w8.float().T) * sc + b
    if act == "gelu":
        ref = F.gelu(ref)
    if kind == "f32":
        r = torch.randn(M, N, device="cuda", generator=g)
        out = r.clone() if resid else torch.empty(M, N, device="cuda")
        L.gemm_fp8(a8, w8, sc, bias=b, resid=out if resid else None, out=out)
        want, tol = ref + (r if resid else 0), 1e-4
    elif kind == "bf16":
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        L.gemm_fp8(a8, w8, sc, bias=b, act=act, out=out)
        want, tol = ref, 8e-3
    else:
        oqs = 4.0
        out = torch.empty(M, N, device="cuda", dtype=L.FP8)
        L.gemm_fp8(a8, w8, sc, bias=b, act=act, out=out, out_qscale=oqs)
        out = out.float() / oqs
        want, tol = ref.clamp(-448.0 / oqs, 448.0 / oqs), 6e-2      # e4m3: 3 mantissa bits
    torch.cuda.synchronize()
    assert rel_err(out, want) < tol, (M, N, K, kind, act, resid)


@pytest.mark.parametrize("seed", range(8))
def test_gemm_f32_row_maps_sweep(L, seed):
    """bf_gemm_f32 (the decoder's f32 MFMA GEMM) with gathered A rows and scattered / dropped C
    rows (negative map entries), ragged M / N / K, every activation and the in-place residual"""
    rng = np.random.default_rng(100 + seed)
    M, N, K = int(rng.integers(1, 3000)), int(rng.integers(1, 700)), 4 * int(rng.integers(1, 300))
    act = [None, "gelu", "relu"][seed % 3]
    g = torch.Generator(device="cuda").manual_seed(seed)
    src_rows = M + 11
    a = torch.randn(src_rows, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)
    b = torch.randn(N, device="cuda", generator=g)
    a_map = torch.randint(-1, src_rows, (M,), device="cuda", generator=g).int()     # -1: a zero row
    dst_rows = M + 7
    c_map = torch.randperm(dst_rows, device="cuda", generator=g)[:M].int()
    c_map[torch.rand(M, device="cuda", generator=g) < 0.1] = -1                    # dropped rows
    out = torch.randn(dst_rows, N, device="cuda", generator=g)
    before = out.clone()
    L.gemm_f32(a, w, bias=b, act=act, resid=out if seed % 2 else None, out=out, a_map=a_map, c_map=c_map)
    torch.cuda.synchronize()
    arows = torch.where(a_map[:, None] >= 0, a[a_map.clamp(min=0).long()], torch.zeros_like(a[:1]))
    ref = arows @ w.T + b
    if act == "gelu":
        ref = F.gelu(ref)
    elif act == "relu":
        ref = F.relu(ref)
    keep = c_map >= 0
    dst = c_map[keep].long()
    want = ref[keep] + (before[dst] if seed % 2 else 0)
    assert rel_err(out[dst], want) < 1e-5 * math.sqrt(K / 64) + 1e-6, (M, N, K, act)
    untouched = torch.ones(dst_rows, dtype=torch.bool, device="cuda")
    untouched[dst] = False
    assert torch.equal(out[untouched], before[untouched]), "rows outside the map were written"
