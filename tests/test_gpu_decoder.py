"""The CuTR decoder tail on the f32 HIP kernels (DecoderEngine, bf_dec_native.hip) on the GPU:
each kernel against the torch formula of the same op, then the whole engine against
  * the reference's own fp32 goldens (decoder fed the reference's backbone features; the same
    tolerances as the torch decoder's test in test_gpu_engine.py), and
  * the torch definition (CubifyTransformer.decode) on a ViT-B-sized batch of 8 frames.
f32 throughout; only the summation order differs from BLAS / torch (relative errors ~1e-6)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests.test_cutr_golden import CASES as CUTR_CASES  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    _lib.lib()
    return _lib


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,N,K,act,maps,res", [(2416, 256, 256, None, False, True),
                                                (2416, 2048, 256, "relu", False, False),
                                                (2416, 256, 2048, None, False, True),
                                                (12800, 1536, 256, None, False, False),
                                                (777, 100, 1000, "gelu", True, True),
                                                (5, 7, 36, None, True, False)])
def test_gemm_f32_vs_torch(L, M, N, K, act, maps, res):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M + 9, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g)
    a_map = c_map = None
    arows = torch.arange(M, device="cuda")
    crows = torch.arange(M, device="cuda")
    if maps:
        arows = torch.randperm(M + 9, device="cuda", generator=g)[:M]
        arows[::7] = -1
        crows = torch.randperm(M, device="cuda", generator=g)
        crows[::5] = -1
        a_map, c_map = arows.to(torch.int32), crows.to(torch.int32)
    A = torch.where(arows[:, None] >= 0, a[arows.clamp_min(0)], torch.zeros(1, device="cuda"))
    y = A @ w.T + b
    if act == "relu":
        y = F.relu(y)
    elif act == "gelu":
        y = F.gelu(y)
    out = torch.randn(M, N, device="cuda", generator=g)
    want = out.clone()
    keep = crows >= 0
    want[crows[keep]] = (want[crows[keep]] if res else 0) + y[keep]
    L.gemm_f32(a, w, b, act=act, resid=out if res else None, out=out, a_map=a_map, c_map=c_map, m=M)
    err = rel(out, want)
    print("gemm_f32", M, N, K, act, maps, res, err)
    assert err < 2e-6


def test_ln_rows_and_groupnorm_vs_torch(L):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(2416, 256, device="cuda", generator=g) * 3 + 1
    gam = torch.randn(256, device="cuda", generator=g)
    bet = torch.randn(256, device="cuda", generator=g)
    pos = torch.randn(2416, 256, device="cuda", generator=g)
    out2 = torch.empty_like(x)
    y = L.ln_rows(x, gam, bet, 1e-5, pos=pos, out2=out2)
    ref = F.layer_norm(x, (256,), gam, bet, 1e-5)
    assert rel(y, ref) < 1e-6 and rel(out2, ref + pos) < 1e-6
    yg = L.ln_rows(x, gam, bet, 1e-6, gelu=True)
    assert rel(yg, F.gelu(F.layer_norm(x, (256,), gam, bet, 1e-6))) < 1e-6
    # GroupNorm(32) of a channel-last [B, 1600, 256] map
    B, P = 3, 1600
    m = torch.randn(B * P, 256, device="cuda", generator=g) * 2 + 0.5
    out = torch.empty_like(m)
    pos = torch.randn(B * P, 256, device="cuda", generator=g)
    o2 = torch.empty_like(m)
    L.groupnorm_cl(m, B, 32, gam, bet, 1e-5, out, pos=pos, out2=o2)
    ref = F.group_norm(m.view(B, P, 256).permute(0, 2, 1), 32, gam, bet, 1e-5).permute(0, 2, 1).reshape(B * P, 256)
    assert rel(out, ref) < 1e-6 and rel(o2, ref + pos) < 1e-6


def test_s2d_conv_vs_torch(L):
    g = torch.Generator(device="cuda").manual_seed(2)
    B, H, W, C = 2, 40, 40, 256
    x = torch.randn(B, C, H, W, device="cuda", generator=g)
    conv = torch.nn.Conv2d(C, C, 2, 2).cuda()
    rows = x.permute(0, 2, 3, 1).reshape(-1, C).contiguous()
    p = L.s2d(rows, B, H, W)
    y = L.gemm_f32(p, conv.weight.detach().reshape(C, -1).contiguous(), conv.bias.detach())
    ref = conv(x).permute(0, 2, 3, 1).reshape(-1, C)
    assert rel(y, ref.detach()) < 2e-6


def test_self_attn_block_mask_vs_torch(L):
    g = torch.Generator(device="cuda").manual_seed(3)
    B, n, C, H, nm = 3, 302, 256, 8, 2
    mha = torch.nn.MultiheadAttention(C, H).cuda().eval()
    x = torch.randn(B, n, C, device="cuda", generator=g)
    pos = torch.randn(B, n, C, device="cuda", generator=g)
    mask = torch.ones((n, n), dtype=torch.bool, device="cuda")
    mask[:nm, :nm] = False
    mask[nm:, nm:] = False
    with torch.no_grad():
        q = x + pos
        ref = mha(q.transpose(0, 1), q.transpose(0, 1), x.transpose(0, 1), attn_mask=mask)[0].transpose(0, 1)
        wi, bi = mha.in_proj_weight, mha.in_proj_bias
        QK = q.reshape(B * n, C) @ wi[:2 * C].T + bi[:2 * C]
        V = x.reshape(B * n, C) @ wi[2 * C:].T + bi[2 * C:]
        att = torch.empty(B * n, C, device="cuda")
        L.self_attn(QK[:, :C], QK[:, C:], V, att, B, H, n, nm, (C // H) ** -0.5)
        got = att @ mha.out_proj.weight.T + mha.out_proj.bias
    err = rel(got, ref.reshape(B * n, C))
    print("self attention rel err", err)
    assert err < 2e-6


@pytest.mark.parametrize("n,k", [(2100, 300), (600, 100), (4096, 4096), (3, 1)])
def test_topk_rows_vs_torch(L, n, k):
    g = torch.Generator(device="cuda").manual_seed(n)
    B = 5
    v = torch.randn(B, n, 2, device="cuda", generator=g)
    idx = L.topk_rows(v, B, n, k, ldv=2)
    ref = torch.topk(v[..., 0], k, dim=1)[1]
    assert torch.equal(idx.long(), ref)
    # ties: equal values keep index order
    t = torch.zeros(1, 64, device="cuda")
    t[0, 10:20] = 1.0
    i2 = L.topk_rows(t, 1, 64, 12)
    assert i2[0].tolist() == list(range(10, 20)) + [0, 1]


def _rand_model(dim=768, seed=5):
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.weights import init_seeded
    torch.manual_seed(0)
    return init_seeded(make_cubify_transformer(dim, depth_model=True).eval(), seed).cuda()


def test_ray_positions_vs_torch(L):
    from boxfusion_amd.decoder_engine import DecoderEngine
    from boxfusion_amd.synthetic import SCANNET_K
    m = _rand_model(192)
    B, g = 2, 40
    eng = DecoderEngine(m, B, g, g)
    K = np.stack([np.asarray(SCANNET_K, np.float32)] * B)
    K[1, 0, 2] += 7.0
    sizes = [(640, 480), (600, 440)]
    pos = eng.positions(K, sizes)
    with torch.no_grad():
        ref = m.pos_embedding(torch.from_numpy(K).cuda(), sizes, g)
    ref = ref.flatten(2).transpose(1, 2).reshape(B * g * g, -1) + m.level_embed[0]
    err = rel(pos, ref)
    print("ray position rel err", err)
    assert err < 1e-5


def _assert_same(r, t, desc_tol=1e-4):
    """native vs torch decode on the same features: every instance field (well-separated scores)"""
    s = t.scores.cpu().numpy()
    np.testing.assert_allclose(r.scores.cpu().numpy(), s, rtol=1e-4, atol=1e-6)
    gap = np.minimum(np.abs(np.diff(s, prepend=np.inf)), np.abs(np.diff(s, append=-np.inf)))
    ok = gap > 1e-5
    assert ok.sum() > 50
    np.testing.assert_array_equal(r.pred_classes.cpu().numpy()[ok], t.pred_classes.cpu().numpy()[ok])
    for a, b, tol in ((r.pred_boxes, t.pred_boxes, 1e-3), (r.pred_proj_xy, t.pred_proj_xy, 1e-3),
                      (r.pred_boxes_3d.tensor, t.pred_boxes_3d.tensor, 1e-4),
                      (r.pred_boxes_3d.R, t.pred_boxes_3d.R, 1e-5), (r.object_desc, t.object_desc, desc_tol),
                      (r.pred_logits, t.pred_logits, 1e-4)):
        np.testing.assert_allclose(a.cpu().numpy()[ok], b.cpu().numpy()[ok], rtol=1e-4, atol=tol)


@pytest.mark.parametrize("case", CUTR_CASES)
def test_decoder_engine_vs_reference(L, case):
    """DecoderEngine on the reference's backbone features reproduces the reference's fp32 instances
    (tolerances of the torch decoder's test_demo_sequence_engine_vs_reference)"""
    from boxfusion_amd.cubify_transformer import sensor_inputs
    from boxfusion_amd.decoder_engine import DecoderEngine
    from tests import trace_util as TU
    from tests.test_cutr_golden import assert_instances
    from tests.test_gpu_engine import _demo_sequence
    g = TU.load(case)
    dev = torch.device("cuda")
    _, packaged = _demo_sequence(g, dev)
    from tests.test_cutr_golden import model_for
    m = model_for(g).to(dev)
    x = sensor_inputs(packaged)
    feat = torch.from_numpy(g["features"].astype(np.float32)).to(dev)
    B, C, h, w = feat.shape
    eng = DecoderEngine(m, B, h, w)
    pos = eng.positions(x["K"].cpu().numpy(), [(ww, hh) for hh, ww in x["image_sizes"]])
    rows = feat.permute(0, 2, 3, 1).reshape(B * h * w, C).contiguous()
    r = eng(rows, pos, x["depth_params"], torch.linalg.inv(x["K"]), x["T_gravity"], x["image_sizes"],
            (x["pad"], x["pad"]))[0]
    assert_instances(r, g, score_tol=(1e-4, 1e-5), box_tol=(1e-4, 2e-3), b3_tol=(2e-4, 2e-4),
                     R_tol=2e-5, desc_tol=5e-3)


def test_decoder_engine_vs_torch_decode_vitb_batch8(L):
    """ViT-B RGB-D, 8 frames of 640x480 (the bench's decode shape): native == torch decode"""
    from boxfusion_amd.cubify_transformer import FrameBatch
    from boxfusion_amd.decoder_engine import DecoderEngine
    from boxfusion_amd.synthetic import SCANNET_K
    m = _rand_model(768)
    B, g, C = 8, 40, 768
    gen = torch.Generator(device="cuda").manual_seed(9)
    feat = torch.randn(B, C, g, g, device="cuda", generator=gen)
    K = torch.from_numpy(np.stack([np.asarray(SCANNET_K, np.float32)] * B)).cuda()
    Tg = torch.linalg.qr(torch.randn(B, 3, 3, device="cuda", generator=gen))[0].contiguous()
    params = torch.rand(B, 2, device="cuda", generator=gen) + 0.5
    sizes = [(480, 640)] * B
    batch = FrameBatch(image=None, depth=torch.zeros(B, 640, 640, device="cuda"), depth_params=params, K=K,
                       T_gravity=Tg, image_sizes=sizes, pad=640, K_inv=torch.linalg.inv(K))
    eng = DecoderEngine(m, B, g, g)
    pos = eng.positions(K.cpu().numpy(), [(640, 480)] * B)
    with torch.no_grad():
        ref = m.decode(feat, batch, pos=pos.view(B, g, g, 256).permute(0, 3, 1, 2) - m.level_embed[0].view(1, -1, 1, 1))
    rows = feat.permute(0, 2, 3, 1).reshape(B * g * g, C).contiguous()
    got = eng(rows, pos, params, batch.K_inv, Tg, sizes, (640, 640))
    for r, t in zip(got, ref):
        _assert_same(r, t)
    # a second call on the same buffers gives the same result (no state carried between batches)
    got2 = eng(rows, pos, params, batch.K_inv, Tg, sizes, (640, 640))
    assert torch.equal(got2[3].scores, got[3].scores)


def test_decoder_engine_graph_capture(L):
    """the whole decode is capturable: a replay equals the eager call"""
    from boxfusion_amd.decoder_engine import DecoderEngine
    from boxfusion_amd.synthetic import SCANNET_K
    m = _rand_model(192, seed=6)
    B, g, C = 2, 40, 192
    gen = torch.Generator(device="cuda").manual_seed(10)
    feat = torch.randn(B * g * g, C, device="cuda", generator=gen)
    K = torch.from_numpy(np.stack([np.asarray(SCANNET_K, np.float32)] * B)).cuda()
    Ki = torch.linalg.inv(K)
    params = torch.rand(B, 2, device="cuda", generator=gen) + 0.5
    sizes = [(480, 640)] * B
    eng = DecoderEngine(m, B, g, g)
    pos = eng.positions(K.cpu().numpy(), [(640, 480)] * B)
    res = eng(feat, pos, params, Ki, None, sizes, (640, 640))
    eager = [r.scores.clone() for r in res]
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eng(feat, pos, params, Ki, None, sizes, (640, 640))
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(gr):
        res = eng(feat, pos, params, Ki, None, sizes, (640, 640))
    eng.out["scores"].zero_()
    gr.replay()
    torch.cuda.synchronize()
    for a, b in zip(res, eager):
        assert torch.equal(a.scores, b)
