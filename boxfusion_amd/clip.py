"""CLIP ViT-H/14 image tower used for open-vocabulary crop labelling
(reference: tools/utils.py:342-403 — open_clip "ViT-H-14" / the absent SAMCLIP wrapper).

Parameter names follow open_clip's VisionTransformer (`conv1`, `class_embedding`,
`positional_embedding`, `ln_pre`, `transformer.resblocks.{i}.{ln_1,attn,ln_2,mlp.c_fc,mlp.c_proj}`,
`ln_post`, `proj`) so an open_clip checkpoint's `visual.*` entries load unchanged.  The forward
here is the fp32 definition; `boxfusion_amd.engine.CLIPEngine` runs the same weights on the MFMA
kernels.  Parity with the real CLIP is UNPINNED (no weights / module offline); the output
contract (L2-normalised 1024-d features matched against data/class_features [473,1024]) is.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class ResidualAttentionBlock(nn.Module):
    def __init__(self, width, heads, mlp_ratio=4.0):
        super().__init__()
        self.ln_1 = nn.LayerNorm(width)
        self.attn = nn.MultiheadAttention(width, heads, batch_first=True)
        self.ln_2 = nn.LayerNorm(width)
        hidden = int(width * mlp_ratio)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(width, hidden)), ("gelu", nn.GELU()),
                                              ("c_proj", nn.Linear(hidden, width))]))

    def forward(self, x):
        y = self.ln_1(x)
        x = x + self.attn(y, y, y, need_weights=False)[0]
        return x + self.mlp(self.ln_2(x))


class Transformer(nn.Module):
    def __init__(self, width, layers, heads):
        super().__init__()
        self.resblocks = nn.ModuleList([ResidualAttentionBlock(width, heads) for _ in range(layers)])


class VisionTransformer(nn.Module):
    def __init__(self, image_size=224, patch_size=14, width=1280, layers=32, heads=16, output_dim=1024):
        super().__init__()
        self.image_size, self.patch_size = image_size, patch_size
        self.width, self.heads, self.layers = width, heads, layers
        self.output_dim = output_dim
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(scale * torch.randn((image_size // patch_size) ** 2 + 1, width))
        self.ln_pre = nn.LayerNorm(width)
        self.transformer = Transformer(width, layers, heads)
        self.ln_post = nn.LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))

    def forward(self, x):
        """x: [N,3,224,224] CLIP-normalised -> [N, output_dim] (not normalised)"""
        x = self.conv1(x).flatten(2).transpose(1, 2)
        cls = self.class_embedding.to(x.dtype)[None, None].expand(x.shape[0], 1, -1)
        x = torch.cat([cls, x], dim=1) + self.positional_embedding
        x = self.ln_pre(x)
        for blk in self.transformer.resblocks:
            x = blk(x)
        return self.ln_post(x[:, 0]) @ self.proj


def vit_h14(**kw):
    return VisionTransformer(224, 14, 1280, 32, 16, 1024, **kw)


class TextTransformer(nn.Module):
    """open_clip TextTransformer ("ViT-H-14" text tower: context 77, vocab 49408, width 1024,
    16 heads, 24 layers, output 1024), the encode_text of precompute_class_features.py:31-37's
    commented open_clip path.  Parameter names follow open_clip's CLIP (`token_embedding`,
    `positional_embedding`, `transformer.resblocks.{i}`, `ln_final`, `text_projection`) so a
    checkpoint's text entries load unchanged.  fp32 definition; `text_engine.CLIPTextEngine` runs
    the same weights on the MFMA kernels.  Parity with open_clip is UNPINNED (module and weights
    absent offline): the architecture is restated from open_clip's published model config."""

    def __init__(self, context_length=77, vocab_size=49408, width=1024, heads=16, layers=24,
                 output_dim=1024):
        super().__init__()
        self.context_length, self.vocab_size = context_length, vocab_size
        self.width, self.heads, self.layers, self.output_dim = width, heads, layers, output_dim
        self.token_embedding = nn.Embedding(vocab_size, width)
        self.positional_embedding = nn.Parameter(0.01 * torch.randn(context_length, width))
        self.transformer = Transformer(width, layers, heads)
        self.ln_final = nn.LayerNorm(width)
        self.text_projection = nn.Parameter(width ** -0.5 * torch.randn(width, output_dim))
        nn.init.normal_(self.token_embedding.weight, std=0.02)
        # causal mask (open_clip build_causal_mask: -inf above the diagonal)
        self.register_buffer("attn_mask", torch.full((context_length, context_length), float("-inf")).triu_(1),
                             persistent=False)

    def forward(self, text):
        """text: token ids [N, context_length] (int) -> [N, output_dim] (not normalised)"""
        x = self.token_embedding(text) + self.positional_embedding
        for blk in self.transformer.resblocks:
            y = blk.ln_1(x)
            x = x + blk.attn(y, y, y, need_weights=False, attn_mask=self.attn_mask)[0]
            x = x + blk.mlp(blk.ln_2(x))
        x = self.ln_final(x)
        x = x[torch.arange(x.shape[0], device=x.device), text.argmax(dim=-1)]
        return x @ self.text_projection


def text_h14(**kw):
    return TextTransformer(77, 49408, 1024, 16, 24, 1024, **kw)
