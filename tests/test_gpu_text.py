"""CLIP text tower on the GPU (the vocabulary builder, precompute_class_features.py:11-45):
bf_attention_causal vs torch's causal SDPA, bf_token_embed / bf_text_pool bit-exact vs torch
indexing, bf_l2_normalize_rows, and CLIPTextEngine vs the fp32 TextTransformer definition.

Tolerances: causal attention on bf16 operands vs the f32 SDPA of the same bf16 values: rel L2
< 1e-2 (bf16 P / output rounding); the engine (bf16 GEMM operands, f32 residual stream) vs the
fp32 definition: rel L2 < 3e-2 and min cosine > 0.999 per prompt.  Parity with open_clip is
UNPINNED (module and weights absent)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    _lib.lib()
    return _lib


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("B,H,S,D", [(3, 16, 77, 64), (2, 4, 200, 64), (2, 2, 130, 80), (1, 1, 5, 64)])
def test_attention_causal(L, B, H, S, D):
    g = torch.Generator(device="cuda").manual_seed(S + D)
    W = H * D
    qkv = (torch.randn(B * S, 3 * W, device="cuda", generator=g) * 1.5).bfloat16()
    o = torch.full((B * S, W), float("nan"), device="cuda", dtype=torch.bfloat16)
    L.attention_causal(qkv[:, :W], qkv[:, W:2 * W], qkv[:, 2 * W:], o, B, H, S, D, D ** -0.5)
    q, k, v = (qkv[:, i * W:(i + 1) * W].float().view(B, S, H, D).transpose(1, 2) for i in range(3))
    ref = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B * S, W)
    assert torch.isfinite(o.float()).all()
    assert rel(o, ref) < 1e-2
    # the first query sees only key 0: its output is v[0] exactly (to bf16)
    assert torch.equal(o.view(B, S, W)[:, 0], qkv.view(B, S, 3 * W)[:, 0, 2 * W:])


def test_token_embed_and_pool(L):
    g = torch.Generator(device="cuda").manual_seed(3)
    V, S, W, N = 1000, 77, 256, 5
    table = torch.randn(V, W, device="cuda", generator=g)
    pos = torch.randn(S, W, device="cuda", generator=g)
    ids = torch.randint(1, V - 1, (N, S), device="cuda", generator=g, dtype=torch.int32)
    ids[:, 40:] = 0
    ids[torch.arange(N), torch.tensor([3, 10, 39, 20, 5])] = V - 1       # EOT-like maximum
    ids[4, 30] = V - 1                                                   # a second maximum: first wins
    x = L.token_embed(ids, table, pos)
    ref = table[ids.long()] + pos
    assert torch.equal(x.view(N, S, W), ref)
    pooled = L.text_pool(ids, x)
    assert torch.equal(pooled, ref[torch.arange(N), ids.long().argmax(-1)])
    bad = ids.clone()
    bad[0, 0] = V
    with pytest.raises(L.HipError):
        L.token_embed(bad, table, pos)
    n = L.l2_normalize_rows(pooled)
    assert torch.allclose(n, pooled / pooled.norm(dim=1, keepdim=True), rtol=1e-6, atol=1e-7)


def _engine_vs_fp32(width, heads, layers, vocab, N, seed):
    from boxfusion_amd.clip import TextTransformer
    from boxfusion_amd.text_engine import CLIPTextEngine
    torch.manual_seed(seed)
    text = TextTransformer(77, vocab, width, heads, layers, 1024).cuda().eval()
    g = torch.Generator(device="cuda").manual_seed(seed)
    ids = torch.zeros(N, 77, dtype=torch.long, device="cuda")
    for i in range(N):
        n = 3 + 7 * i % 20
        ids[i, 0] = vocab - 2
        ids[i, 1:n] = torch.randint(1, vocab - 2, (n - 1,), device="cuda", generator=g)
        ids[i, n] = vocab - 1
    with torch.no_grad():
        ref = text(ids)
    eng = CLIPTextEngine(text, max_prompts=N)
    got = eng.encode_text(ids)
    cos = F.cosine_similarity(got, ref, dim=1)
    return rel(got, ref), cos.min().item(), eng, ids, ref


def test_text_engine_small(L):
    r, c, *_ = _engine_vs_fp32(256, 4, 3, 1000, 7, 0)
    assert r < 3e-2 and c > 0.999, (r, c)


def test_text_engine_vith_class_features(L):
    """ViT-H-14 text tower shape (24 x width 1024, 16 heads, vocab 49408) on 20 prompts, and the
    normalised class table of precompute_class_features.py:43 in two chunks"""
    r, c, eng, ids, ref = _engine_vs_fp32(1024, 16, 24, 49408, 20, 1)
    assert r < 3e-2 and c > 0.999, (r, c)
    tab = eng.class_features(ids.cpu(), chunk=8)
    assert tab.shape == (20, 1024)
    assert torch.allclose(tab.norm(dim=1), torch.ones(20, device="cuda"), atol=1e-5)
    assert F.cosine_similarity(tab, ref, dim=1).min().item() > 0.999


def test_vocabulary_builder_end_to_end(L):
    """precompute_class_features.build_class_features: class names -> BPE tokens -> HIP text tower
    -> L2-normalised table, against the fp32 TextTransformer on the same token ids"""
    from boxfusion_amd.clip import TextTransformer
    from boxfusion_amd.precompute_class_features import build_class_features
    from boxfusion_amd.tokenizer import SimpleTokenizer
    from tests.test_tokenizer import MERGES
    tok = SimpleTokenizer(MERGES)
    torch.manual_seed(3)
    text = TextTransformer(77, tok.vocab_size, 256, 4, 3, 1024).cuda().eval()
    names = ["chair", "table", "sofa", "kitchen cabinet", "tv stand", "a chair, and a table!"]
    tab = build_class_features(names, text, tok, max_prompts=4)
    ids = torch.from_numpy(tok(names)).cuda()
    with torch.no_grad():
        ref = F.normalize(text(ids), dim=-1)
    assert tab.shape == (len(names), 1024)
    assert F.cosine_similarity(tab, ref, dim=1).min().item() > 0.999
    assert torch.allclose(tab.norm(dim=1), torch.ones(len(names), device="cuda"), atol=1e-5)
