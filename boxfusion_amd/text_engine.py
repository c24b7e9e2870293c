"""CLIP text tower on the MFMA kernels: the vocabulary builder of precompute_class_features.py:11-45.

The reference builds its class-feature table once per vocabulary: class names (one per line of
`--class_txt`) -> tokenizer -> `encode_text` -> L2 normalise -> `torch.save` (lines 26-45; the
open_clip "ViT-H-14" path is the commented one, the live path calls the absent SAMCLIP wrapper).
`CLIPTextEngine` runs open_clip's TextTransformer (`clip.TextTransformer`, same parameter names)
as: bf_token_embed (token + positional embedding, f32 residual rows) -> 24 x [bf_layernorm ->
qkv bf_gemm_bf16 -> bf_attention_causal -> out_proj GEMM + f32 residual -> bf_layernorm -> c_fc
GEMM + GELU -> c_proj GEMM + residual] -> bf_text_pool (EOT row) -> ln_final -> text_projection
GEMM -> bf_l2_normalize_rows.  The output is the [V, 1024] table `tools/utils.py:383-403` matches
crop features against (`retriev` renormalises it in place, which is idempotent up to ulps).

Parity with open_clip is UNPINNED (module, tokenizer vocabulary and weights absent offline); the
engine is checked against the fp32 TextTransformer definition on the same weights.
"""
from __future__ import annotations

import torch

from boxfusion_amd import _lib


def _bf(t):
    return t.detach().to(torch.bfloat16).contiguous()


def _f(t):
    return t.detach().to(torch.float32).contiguous()


class CLIPTextEngine:
    def __init__(self, text, max_prompts, device="cuda"):
        dev = torch.device(device)
        self.text = text.to(dev).eval()
        t = text
        self.dev, self.N = dev, int(max_prompts)
        self.S, self.W, self.heads = t.context_length, t.width, t.heads
        self.D = self.W // self.heads
        self.tok = _f(t.token_embedding.weight)
        self.pos = _f(t.positional_embedding)
        self.blocks = []
        for blk in t.transformer.resblocks:
            self.blocks.append(dict(
                n1=(_f(blk.ln_1.weight), _f(blk.ln_1.bias), blk.ln_1.eps),
                n2=(_f(blk.ln_2.weight), _f(blk.ln_2.bias), blk.ln_2.eps),
                qkv=(_bf(blk.attn.in_proj_weight), _f(blk.attn.in_proj_bias)),
                proj=(_bf(blk.attn.out_proj.weight), _f(blk.attn.out_proj.bias)),
                fc1=(_bf(blk.mlp.c_fc.weight), _f(blk.mlp.c_fc.bias)),
                fc2=(_bf(blk.mlp.c_proj.weight), _f(blk.mlp.c_proj.bias))))
        self.ln_final = (_f(t.ln_final.weight), _f(t.ln_final.bias), t.ln_final.eps)
        self.proj_t = _bf(t.text_projection.t())           # [out, width]
        M = self.N * self.S
        bf16, f32 = dict(dtype=torch.bfloat16, device=dev), dict(dtype=torch.float32, device=dev)
        W = self.W
        self.X = torch.empty((M, W), **f32)
        self.LN = torch.empty((M, W), **bf16)
        self.QKV = torch.empty((M, 3 * W), **bf16)
        self.ATT = torch.empty((M, W), **bf16)
        self.H1 = torch.empty((M, 4 * W), **bf16)
        self.POOL = torch.empty((self.N, W), **f32)
        self.LNP = torch.empty((self.N, W), **bf16)
        self.FEAT = torch.empty((self.N, t.output_dim), **f32)

    @torch.no_grad()
    def encode_text(self, ids):
        """token ids [N, context_length] (int, on the device) -> features [N, out] f32, not
        normalised (open_clip encode_text(normalize=False))"""
        if ids.dim() != 2 or ids.shape[1] != self.S:
            raise _lib.HipError(f"token ids must be [N, {self.S}]")
        ids = ids.to(device=self.dev, dtype=torch.int32).contiguous()
        N = ids.shape[0]
        if N == 0:
            return torch.zeros((0, self.text.output_dim), device=self.dev)
        if N > self.N:
            raise _lib.HipError(f"{N} prompts > engine capacity {self.N}")
        W, S, M = self.W, self.S, N * self.S
        X = _lib.token_embed(ids, self.tok, self.pos, out=self.X[:M])
        LN, QKV, ATT, H1 = self.LN[:M], self.QKV[:M], self.ATT[:M], self.H1[:M]
        scale = self.D ** -0.5
        for blk in self.blocks:
            _lib.layernorm(X, *blk["n1"][:2], blk["n1"][2], out=LN)
            _lib.gemm(LN, *blk["qkv"], out=QKV)
            _lib.attention_causal(QKV[:, :W], QKV[:, W:2 * W], QKV[:, 2 * W:], ATT, N, self.heads, S,
                                  self.D, scale)
            _lib.gemm(ATT, *blk["proj"], resid=X, out=X)
            _lib.layernorm(X, *blk["n2"][:2], blk["n2"][2], out=LN)
            _lib.gemm(LN, *blk["fc1"], act="gelu", out=H1)
            _lib.gemm(H1, *blk["fc2"], resid=X, out=X)
        # ln_final is per row, so pooling the EOT row first gives the same rows
        pooled = _lib.text_pool(ids, X, out=self.POOL[:N])
        lnp = _lib.layernorm(pooled, *self.ln_final, out=self.LNP[:N])
        return _lib.gemm(lnp, self.proj_t, out=self.FEAT[:N], out_dtype=torch.float32)

    @torch.no_grad()
    def class_features(self, ids, chunk=None):
        """the normalised class-feature table (precompute_class_features.py:39-43), prompts in
        chunks of the engine capacity"""
        ids = torch.as_tensor(ids)
        out = []
        step = self.N if chunk is None else min(int(chunk), self.N)
        for i in range(0, ids.shape[0], step):
            f = self.encode_text(ids[i:i + step].to(self.dev))
            out.append(_lib.l2_normalize_rows(f))
        if not out:
            return torch.zeros((0, self.text.output_dim), device=self.dev)
        return torch.cat(out)
