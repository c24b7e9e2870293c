"""HIP engines vs the fp32 PyTorch definition of the same models on the same weights (GPU).
bf16 MFMA with f32 accumulation: tolerances are relative L2 errors."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests.test_cutr_golden import CASES as CUTR_CASES  # noqa: E402

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda")


@pytest.mark.parametrize("dim", [192, 768])
def test_cutr_backbone_engine_vs_fp32(dev, dim):
    from boxfusion_amd import _lib
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.engine import CuTREngine
    from boxfusion_amd.preprocessor import PIXEL_MEAN, PIXEL_STD
    from boxfusion_amd.synthetic import frame_rgbd
    from boxfusion_amd.weights import init_seeded
    torch.manual_seed(0)
    model = init_seeded(make_cubify_transformer(dim, True).eval()).to(dev)
    B = 2
    rgb = np.stack([frame_rgbd(f)[0] for f in range(B)])
    depth = np.stack([frame_rgbd(f)[1] for f in range(B)])
    img = torch.from_numpy(rgb).to(dev)
    dstd, params = _lib.depth_standardize(torch.from_numpy(depth).to(dev))
    eng = CuTREngine(model, B)
    feat = eng.backbone(img, dstd)
    mean = torch.tensor(PIXEL_MEAN, device=dev).view(1, 3, 1, 1)
    std = torch.tensor(PIXEL_STD, device=dev).view(1, 3, 1, 1)
    x = F.pad((img.permute(0, 3, 1, 2).float() - mean) / std, (0, 0, 0, 160))
    d = F.pad(dstd, (0, 0, 0, 160))
    with torch.no_grad():
        ref = model.backbone.backbone.forward_tensors(x, d)
    err = rel(feat, ref)
    print("backbone rel err", dim, err)
    assert err < 3e-2


def test_cutr_engine_end_to_end(dev):
    from boxfusion_amd import _lib
    from boxfusion_amd.cubify_transformer import FrameBatch, make_cubify_transformer
    from boxfusion_amd.engine import CuTREngine
    from boxfusion_amd.sensor import camera_to_gravity
    from boxfusion_amd.synthetic import Scene, SCANNET_K, frame_rgbd
    from boxfusion_amd.weights import init_seeded
    torch.manual_seed(0)
    model = init_seeded(make_cubify_transformer(384, True).eval()).to(dev)
    B = 2
    rgb = torch.from_numpy(np.stack([frame_rgbd(f)[0] for f in range(B)])).to(dev)
    depth = torch.from_numpy(np.stack([frame_rgbd(f)[1] for f in range(B)])).to(dev)
    dstd, params = _lib.depth_standardize(depth)
    K = torch.from_numpy(np.stack([SCANNET_K] * B)).to(dev)
    Tg = torch.from_numpy(np.stack([camera_to_gravity(Scene().pose(f)) for f in range(B)])).to(dev)
    eng = CuTREngine(model, B)
    res = eng(rgb, dstd, params, K, Tg, [(480, 640)] * B)
    assert len(res) == B and len(res[0]) == 100
    for r in res:
        assert torch.isfinite(r.scores).all() and torch.isfinite(r.pred_boxes_3d.tensor).all()
        assert (r.scores[:-1] >= r.scores[1:]).all()
    # the decoder's memory projections of all layers in one GEMM each == the per-layer linears
    orig = type(model)._memory_kv
    try:
        type(model)._memory_kv = lambda self, src, pos: None
        res2 = eng(rgb, dstd, params, K, Tg, [(480, 640)] * B)
    finally:
        type(model)._memory_kv = orig
    for r, r2 in zip(res, res2):
        torch.testing.assert_close(r.scores, r2.scores, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(r.pred_boxes_3d.tensor, r2.pred_boxes_3d.tensor, rtol=1e-3, atol=1e-3)


def test_clip_engine_vs_fp32(dev):
    from boxfusion_amd.clip import CLIP_MEAN, CLIP_STD, VisionTransformer
    from boxfusion_amd.engine import CLIPEngine
    from boxfusion_amd.weights import init_seeded
    torch.manual_seed(0)
    vis = init_seeded(VisionTransformer(224, 14, 1280, 4, 16, 1024).eval(), seed=3).to(dev)
    g = torch.Generator(device="cuda").manual_seed(5)
    frames = torch.randint(0, 256, (2, 480, 640, 3), device=dev, dtype=torch.uint8, generator=g)
    boxes = torch.tensor([[10, 20, 200, 150], [0, 0, 640, 480], [300, 100, 400, 310]],
                         device=dev, dtype=torch.int32)
    idx = torch.tensor([0, 1, 1], device=dev, dtype=torch.int32)
    eng = CLIPEngine(vis, 8)
    got = eng(frames, boxes, idx)
    crops = []
    for n in range(3):
        x1, y1, x2, y2 = boxes[n].tolist()
        c = frames[idx[n], y1:y2, x1:x2].permute(2, 0, 1)[None].float()
        c = F.interpolate(c, size=(224, 224), mode="bilinear", align_corners=False) / 255
        crops.append((c - torch.tensor(CLIP_MEAN, device=dev).view(1, 3, 1, 1)) /
                     torch.tensor(CLIP_STD, device=dev).view(1, 3, 1, 1))
    with torch.no_grad():
        ref = vis(torch.cat(crops))
    err = rel(got, ref)
    print("clip rel err", err)
    assert err < 3e-2


def test_clip_last_block_class_rows_only(dev):
    """the last block on the class tokens only (attention for the class query, proj / ln_2 / fc1 /
    fc2 on N rows) gives the features of the full last block, bf16 MFMA rounding apart"""
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.engine import CLIPEngine
    from boxfusion_amd.weights import init_seeded
    vis = init_seeded(VisionTransformer(224, 14, 1280, 3, 16, 1024).eval(), seed=6).to(dev)
    g = torch.Generator(device="cuda").manual_seed(9)
    frames = torch.randint(0, 256, (2, 480, 640, 3), device=dev, dtype=torch.uint8, generator=g)
    boxes = torch.tensor([[10, 20, 200, 150], [0, 0, 640, 480], [300, 100, 400, 310], [5, 5, 90, 470]],
                         device=dev, dtype=torch.int32)
    idx = torch.tensor([0, 1, 1, 0], device=dev, dtype=torch.int32)
    full = CLIPEngine(vis, 8, cls_only_last=False)(frames, boxes, idx).clone()
    cls = CLIPEngine(vis, 8)(frames, boxes, idx)
    err = rel(cls, full)
    print("class-rows-only last block vs full", err)
    assert err < 5e-3


def test_decoder_cross_attention_fused_vs_torch(dev):
    """GlobalCrossAttention with bf_cpb_mlp + bf_rpe_softmax == the torch ops (bias MLP, broadcast
    bias, index_put, clip, softmax), f32, on decoder-sized inputs (302 queries, 40x40 memory);
    the HIP sums run in a fixed order, so the bound is f32 rounding."""
    from boxfusion_amd.cubify_transformer import GlobalCrossAttention
    torch.manual_seed(3)
    xa = GlobalCrossAttention(256, 8, 512, 16).to(dev).eval()
    B, nq, h, w = 2, 300, 40, 40
    query = torch.randn(B, nq + 2, 256, device=dev)
    kv = torch.randn(B, h * w, 256, device=dev)
    cxcy = torch.rand(B, nq, 1, 2, device=dev) * 640
    wh = torch.rand(B, nq, 1, 2, device=dev) * 200 + 4
    ref = torch.cat([cxcy, wh], -1)
    with torch.no_grad():
        xa.fused = True
        got = xa(query, ref, kv, kv, (h, w), slice(2, None))
        xa.fused = False
        want = xa(query, ref, kv, kv, (h, w), slice(2, None))
    torch.testing.assert_close(got, want, rtol=1e-4, atol=2e-5)
    # the bias tables alone
    from boxfusion_amd import _lib
    px, _ = xa._positions(h, w, dev)
    rx = _lib.cpb_mlp(ref[:, :, 0].contiguous(), px, 0, xa.cpb_mlp1[0].weight, xa.cpb_mlp1[0].bias,
                      xa.cpb_mlp1[2].weight)
    r4 = torch.cat([ref[..., :2] - ref[..., 2:] / 2, ref[..., :2] + ref[..., 2:] / 2], -1)
    with torch.no_grad():
        rx_t = xa.cpb_mlp1(r4[..., 0::2] - px[None, None, :, None])
    torch.testing.assert_close(rx, rx_t, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("B,Nq,q0,h,w", [(2, 302, 2, 40, 40), (3, 37, 2, 30, 30), (1, 64, 0, 32, 32),
                                        (2, 33, 33, 7, 9), (1, 300, 2, 24, 32)])
def test_xattn_kernel_vs_torch(dev, B, Nq, q0, h, w):
    """bf_xattn_f32 against the torch formula: (scale q) k^T + rx + ry on rows >= q0, clip,
    softmax, @ v; k / v as one layer's column slice of the all-layer memory projections (row
    stride 6C), key counts off the 32-key block (900, 63), partial query blocks, no box queries"""
    from boxfusion_amd import _lib
    g = torch.Generator(device="cuda").manual_seed(B * Nq + h)
    C, H = 256, 8
    N = h * w
    q = torch.randn(B, Nq, C, device=dev, generator=g)
    kall = torch.randn(B, N, 6 * C, device=dev, generator=g)
    vall = torch.randn(B, N, 6 * C, device=dev, generator=g)
    k, v = kall[..., 2 * C:3 * C], vall[..., 2 * C:3 * C]
    rx = torch.randn(B, Nq - q0, w, H, device=dev, generator=g)
    ry = torch.randn(B, Nq - q0, h, H, device=dev, generator=g)
    scale = 32 ** -0.5
    got = _lib.xattn(q, k, v, rx, ry, h, w, q0, H, scale)
    qh = (q * scale).view(B, Nq, H, 32).permute(0, 2, 1, 3)
    kh = k.reshape(B, N, H, 32).permute(0, 2, 1, 3)
    vh = v.reshape(B, N, H, 32).permute(0, 2, 1, 3)
    a = qh @ kh.transpose(-2, -1)
    bias = (rx[:, :, None] + ry[:, :, :, None]).flatten(2, 3).permute(0, 3, 1, 2)
    a[:, :, q0:] += bias
    a = a.clip(torch.finfo(a.dtype).min, torch.finfo(a.dtype).max).softmax(-1)
    want = (a @ vh).transpose(1, 2).reshape(B, Nq, C)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("H,W,ratio,depth_model", [(480, 640, 2, True), (480, 640, 4, True),
                                                  (512, 384, 2, True), (512, 384, 1, True),
                                                  (480, 640, 1, False), (576, 768, 2, True),
                                                  (720, 896, 2, True), (768, 1024, 4, True)])
def test_cutr_backbone_shapes_vs_fp32(dev, H, W, ratio, depth_model):
    """depth at 1/2 and 1/4 of the image resolution (joint windows of 256 + 64 / 256 + 16 tokens),
    the CA-1M portrait frame (512 square, 2x2 windows) and the RGB-only model (windows without
    depth, layer scale folded into proj / fc2, encoder_norm)"""
    from boxfusion_amd import _lib
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.engine import CuTREngine
    from boxfusion_amd.preprocessor import PIXEL_MEAN, PIXEL_STD, square_pad_size
    from boxfusion_amd.synthetic import frame_rgbd
    from boxfusion_amd.weights import init_seeded
    torch.manual_seed(0)
    model = init_seeded(make_cubify_transformer(192, depth_model).eval(), seed=4).to(dev)
    if not depth_model:       # layer scales away from 1 so the folding is exercised
        with torch.no_grad():
            for blk in model.backbone.backbone.blocks:
                blk.ls1.gamma.uniform_(0.5, 1.5)
                blk.ls2.gamma.uniform_(0.5, 1.5)
    B = 2
    pad = square_pad_size(H, W)
    rgb = np.stack([frame_rgbd(f, H, W)[0] for f in range(B)])
    depth = np.stack([frame_rgbd(f, H, W)[1][::ratio, ::ratio] for f in range(B)])
    img = torch.from_numpy(rgb).to(dev)
    dstd, _ = _lib.depth_standardize(torch.from_numpy(np.ascontiguousarray(depth)).to(dev))
    eng = CuTREngine(model, B, H, W, pad=pad, depth_ratio=ratio)
    feat = eng.backbone(img, dstd if depth_model else None)
    mean = torch.tensor(PIXEL_MEAN, device=dev).view(1, 3, 1, 1)
    std = torch.tensor(PIXEL_STD, device=dev).view(1, 3, 1, 1)
    x = F.pad((img.permute(0, 3, 1, 2).float() - mean) / std, (0, pad - W, 0, pad - H))
    pd = pad // ratio
    d = F.pad(dstd, (0, pd - dstd.shape[2], 0, pd - dstd.shape[1])) if depth_model else None
    with torch.no_grad():
        ref = model.backbone.backbone.forward_tensors(x, d)
    err = rel(feat, ref)
    print("backbone rel err", H, W, ratio, depth_model, err)
    assert err < 3e-2


def _demo_sequence(g, dev, B=1, uniform_queries=False, model=None):
    """demo.py:129-136 on the GPU: package -> move to model.pixel_mean -> preprocess -> model"""
    from boxfusion_amd.preprocessor import Augmentor, Preprocessor, move_input_to_current_device
    from tests.test_cutr_golden import model_for
    from tests.test_demo_boundary import golden_sample
    if model is None:
        model = model_for(g, uniform_queries).to(dev)
    packaged = Augmentor(("wide/image", "wide/depth")).package(golden_sample(g))
    packaged = move_input_to_current_device(packaged, model.pixel_mean)
    packaged = Preprocessor().preprocess([packaged])
    with torch.no_grad():
        return model(packaged)[0], packaged


@pytest.mark.parametrize("case", CUTR_CASES)
def test_demo_sequence_engine_vs_reference(dev, case):
    """the HIP CuTR path through the reference's own call sequence (package -> move -> preprocess
    -> model(packaged)), against the REFERENCE's fp32 run on the same frame and seeded weights:
      * depth whitening parameters (bf_depth_standardize) within 1e-5 relative;
      * backbone features (bf16 MFMA backbone) within 3e-2 relative L2;
      * the top-100 score curve within 2.5e-2 per score and 3e-3 on average;
      * the decoder (f32 torch + bf_cpb_mlp / bf_rpe_softmax) on the reference's backbone features
        reproduces the reference's instances to f32 rounding (classes, 2-D / 3-D boxes, R, proj).
    End-to-end instances are not compared rank by rank: with random weights the encoder's top-300
    proposal logits sit ~1e-4 apart, so bf16 backbone rounding reorders which proposal a query
    slot gets."""
    from boxfusion_amd.cubify_transformer import FrameBatch, sensor_inputs
    from tests import trace_util as TU
    from tests.test_cutr_golden import assert_instances
    g = TU.load(case)
    r, packaged = _demo_sequence(g, dev)
    np.testing.assert_allclose(packaged["wide"]["depth"].info[0].parameters.reshape(-1).cpu().numpy(),
                               g["depth_params"], rtol=1e-5)
    from tests.test_cutr_golden import model_for
    m = model_for(g).to(dev)
    x = sensor_inputs(packaged)
    raw = x["image_raw"]
    from boxfusion_amd.engine import CuTREngine
    B, _, H, W = raw.shape
    eng = CuTREngine(m, B, H, W, pad=x["pad"], device=dev, depth_ratio=x["ratio"])
    feat = eng.backbone(raw.contiguous(), x["depth_std"], chw=True, pixel_mean=x["pixel_mean"],
                        pixel_std=x["pixel_std"])
    ref = torch.from_numpy(g["features"].astype(np.float32)).to(dev)
    err = rel(feat, ref)
    print(case, "backbone rel err vs reference", err)
    assert err < 3e-2
    # the score curve end to end: the bf16 backbone's 2.8e-3 relative error moves near-tied
    # proposals (random weights), so a few scores shift by up to ~1e-2 (measured 3e-3..1.3e-2 over
    # the three frames and two attention kernels); the curve as a whole stays within 3e-3
    s = r.scores.cpu().numpy()
    d = np.abs(s - g["scores"])
    print(case, "score curve |diff| max", d.max(), "mean", d.mean())
    assert d.max() < 2.5e-2 and d.mean() < 3e-3
    K_host = x["K"].cpu().numpy()
    batch = FrameBatch(image=None, depth=x["depth_std"], depth_params=x["depth_params"], K=x["K"],
                       T_gravity=x["T_gravity"], image_sizes=x["image_sizes"], pad=x["pad"])
    with torch.no_grad():
        r2 = m.decode(ref, batch, pos=eng.positions(K_host, x["image_sizes"]))[0]
    assert_instances(r2, g, score_tol=(1e-4, 1e-5), box_tol=(1e-4, 2e-3), b3_tol=(2e-4, 2e-4),
                     R_tol=2e-5, desc_tol=5e-3)


@pytest.mark.parametrize("case", CUTR_CASES)
def test_demo_sequence_instances_vs_reference(dev, case):
    """END TO END, instance by instance: model(packaged) on the HIP path (bf16 MFMA backbone, f32
    HIP decoder, top-300 / top-100 kernels, 3-D lift) through demo.py:129-136's call sequence,
    against the REFERENCE's fp32 run of the same frame with the uniform-query weights (dim 192 on
    four frame shapes, incl. CA-1M portrait at RGB:depth 1 and 2, and the bench's ViT-B width)
    (weights.uniform_queries: the decoder is then equivariant to the order of its proposal
    queries, so near-tied encoder logits do not swap content rows).  Every reference instance is
    paired with the HIP instance of the same class and 2-D box (<= 0.5 px); per pair: score,
    rank, 2-D box, logits, 3-D box, R, projected centre and object descriptor within the bf16
    backbone's tolerances below.  Unpaired instances may only sit at the top-100 cut (their
    score within 1e-3 of the 100th).  A second call on the same engine leaves the first call's
    instances untouched (the boundary returns fresh tensors)."""
    from tests import trace_util as TU
    from tests.test_cutr_golden import instance_arrays, match_instances, uniform_view
    from tests.test_cutr_golden import model_for
    g = uniform_view(TU.load(case))
    model = model_for(g, uniform_queries=True).to(dev)
    r, packaged = _demo_sequence(g, dev, model=model)
    got = instance_arrays(r)
    pairs, unpaired = match_instances(got, g)
    cut = g["scores"][-1]
    print(case, "paired", len(pairs), "unpaired golden ranks", unpaired)
    assert len(pairs) >= 97
    # an unpaired instance sits at one of the two cuts: the top-100 score cut, or the encoder's
    # top-300 proposal cut (its query slot's proposal logit within 1e-2 of the 300th logit, where
    # random-weight logits are spaced ~4e-4 apart; measured at ViT-B: slots 285 / 288, 6e-3 above)
    enc = g.get("uq_enc_logits_sorted")
    for i in unpaired:
        at_top100 = abs(g["scores"][i] - cut) < 1e-3
        at_top300 = enc is not None and abs(enc[g["uq_query"][i]] - enc[300]) < 1e-2
        assert at_top100 or at_top300, (i, g["scores"][i], cut)
    gi = np.array([p[0] for p in pairs])
    hi = np.array([p[1] for p in pairs])
    diffs = {}
    for k in ("scores", "pred_boxes", "pred_logits", "boxes3d", "R", "pred_proj_xy", "object_desc"):
        a, b = got[k][hi].astype(np.float64), g[k][gi].astype(np.float64)
        diffs[k] = float(np.abs(a - b).max())
    print(case, "max |HIP - reference| per field over the pairs", diffs,
          "max rank shift", int(np.abs(gi - hi).max()))
    # measured (MI355X, three frames): scores 1.5e-4, boxes 0.033 px, logits 6e-4, 3-D boxes
    # 1.4e-4, R 3.3e-5, proj 0.033 px, descriptors 5e-3, rank shift 3, 99-100 pairs
    tol = dict(scores=5e-4, pred_boxes=0.1, pred_logits=3e-3, boxes3d=1e-3, R=2e-4, pred_proj_xy=0.1,
               object_desc=2e-2)
    for k, t in tol.items():
        assert diffs[k] < t, (k, diffs[k], t)
    assert np.abs(gi - hi).max() <= 6
    # the boundary copies: a second frame through the same engine must not rewrite these
    first = {k: v.copy() for k, v in got.items()}
    _demo_sequence(g, dev, model=model)
    again = instance_arrays(r)
    for k in first:
        np.testing.assert_array_equal(again[k], first[k])


def test_detection_filter_kernel_vs_reference(dev):
    """bf_detection_filter == the reference's BoxManager filters + score threshold, bit for bit,
    per filter and combined, at the config thresholds and at thresholds splitting every mask"""
    from boxfusion_amd import _lib
    from tests import trace_util as TU
    for case in CUTR_CASES:
        g = TU.load(case)
        for suf in ("", "_med"):
            st, ub, fr, lg = g["thr" + suf]
            det = dict(score_thresh=float(st), uv_bound=True, uv_bound_value=float(ub), floor_mask=True,
                       floor_ratio=float(fr), size_max_thres=float(lg))
            cfg = _lib.filter_cfg(det, int(g["W"]), int(g["H"]))
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
            keep, bits = _lib.detection_filter(t(g["scores"]), t(g["pred_proj_xy"]), t(g["boxes3d"]), cfg,
                                               with_bits=True)
            b = bits.cpu().numpy()
            np.testing.assert_array_equal((b & 2) > 0, g["mask_score" + suf])
            np.testing.assert_array_equal((b & 4) > 0, g["mask_uv" + suf])
            np.testing.assert_array_equal((b & 8) > 0, g["mask_floor" + suf])
            np.testing.assert_array_equal((b & 16) > 0, g["mask_large" + suf])
            np.testing.assert_array_equal(np.nonzero(keep.cpu().numpy())[0], g["kept_sequential" + suf])


def test_unproject_vs_reference(dev):
    """tools_utils.unproject (bf_backproject) vs the reference's tools/utils.unproject output"""
    from boxfusion_amd.tools_utils import unproject
    from tests import trace_util as TU
    u = TU.load("utils.npz")
    xyz, valid = unproject(torch.from_numpy(u["depth"]).to(dev), torch.from_numpy(u["K"]).to(dev),
                           torch.from_numpy(u["RT"]).to(dev), max_depth=10.0)
    np.testing.assert_array_equal(valid.cpu().numpy(), u["valid"])
    np.testing.assert_allclose(xyz.cpu().numpy(), u["xyz"], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("B,nq,n,hidden,heads", [(3, 301, 39, 512, 8), (1, 7, 5, 512, 8), (2, 50, 30, 256, 8)])
def test_cpb_mlp_shapes_vs_torch(dev, B, nq, n, hidden, heads):
    """bf_cpb_mlp against Linear(2, hidden) + ReLU + Linear(hidden, heads) in f32: the register form
    (hidden 512, 8 heads) with a ragged last group of positions (B*nq*n % 4 != 0), and the LDS form
    for other widths"""
    from boxfusion_amd import _lib
    g = torch.Generator(device=dev).manual_seed(B * nq + n)
    ref = torch.rand(B, nq, 4, device=dev, generator=g) * 400
    pos = torch.linspace(0.5, n - 0.5, n, device=dev) * 16
    w1 = torch.randn(hidden, 2, device=dev, generator=g) * 0.05
    b1 = torch.randn(hidden, device=dev, generator=g)
    w2 = torch.randn(heads, hidden, device=dev, generator=g) * 0.05
    for axis in (0, 1):
        got = _lib.cpb_mlp(ref, pos, axis, w1, b1, w2)
        c, half = ref[..., axis], ref[..., 2 + axis] / 2
        x = torch.stack([(c - half)[..., None] - pos, (c + half)[..., None] - pos], -1)
        want = torch.relu(x @ w1.t() + b1) @ w2.t()
        assert got.shape == (B, nq, n, heads)
        torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)
