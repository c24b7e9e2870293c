"""RGB-D ViTDet backbone of CuTR (reference: boxfusion/vit.py).

Module tree and parameter names match the reference so its checkpoints load unchanged
(`backbone.0.patch_embed.proj.weight`, `backbone.0.blocks.{i}.attn.qkv.weight`, ...).  The
`forward` methods here are the fp32 definition of the maths (used to check the architecture
against the reference and as the numerical baseline of the HIP engine); the MI355X execution path
is `boxfusion_amd.engine.CuTREngine`, which runs the same parameters through the gfx950 kernels.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

DEPTH_WINDOW_SIZES = (4, 8, 16)


def window_partition(x, ws):
    """[B,H,W,C] -> [B*nW, ws, ws, C] with zero padding (vit.py:16-37)."""
    B, H, W, C = x.shape
    ph, pw = (ws - H % ws) % ws, (ws - W % ws) % ws
    x = F.pad(x, (0, 0, 0, pw, 0, ph))
    Hp, Wp = H + ph, W + pw
    x = x.view(B, Hp // ws, ws, Wp // ws, ws, C).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(-1, ws, ws, C), (Hp, Wp)


def window_unpartition(win, ws, pad_hw, hw):
    """inverse of window_partition, dropping the padding (vit.py:39-58)."""
    Hp, Wp = pad_hw
    H, W = hw
    B = win.shape[0] // (Hp * Wp // ws // ws)
    x = win.view(B, Hp // ws, Wp // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(B, Hp, Wp, -1)[:, :H, :W, :].contiguous()


def get_abs_pos(abs_pos, has_cls_token, hw):
    """bicubic resize of the pre-training position table to the token grid (vit.py:60-86)."""
    h, w = hw
    if has_cls_token:
        abs_pos = abs_pos[:, 1:]
    size = int(math.sqrt(abs_pos.shape[1]))
    assert size * size == abs_pos.shape[1]
    new = F.interpolate(abs_pos.reshape(1, size, size, -1).permute(0, 3, 1, 2), size=(h, w),
                        mode="bicubic", align_corners=False)
    return new.permute(0, 2, 3, 1)


class LayerScale(nn.Module):
    def __init__(self, dim, init_values=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))

    def forward(self, x):
        return x * self.gamma


class Mlp(nn.Module):
    """timm.layers.Mlp (fc1 -> GELU -> fc2), the pinned timm 1.0.19 layout used by vit.py:274."""

    def __init__(self, in_features, hidden_features, act_layer=nn.GELU, bias=True):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, in_features, bias=bias)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class PatchEmbed(nn.Module):
    def __init__(self, kernel_size=(16, 16), stride=(16, 16), in_chans=3, embed_dim=768, bias=True):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=kernel_size, stride=stride, bias=bias)

    def forward(self, x):
        return self.proj(x).permute(0, 2, 3, 1)


class Attention(nn.Module):
    """Window / global MHSA; with depth tokens the queries, keys and values of both modalities are
    concatenated per window and each row's softmax runs over all keys (vit.py:170-203)."""

    def __init__(self, dim, num_heads=8, qkv_bias=True, proj_bias=True, depth_modality=False):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)
        self.depth_modality = depth_modality

    def _qkv(self, x):
        B, H, W, _ = x.shape
        qkv = self.qkv(x).reshape(B, H * W, 3, self.num_heads, -1).permute(2, 0, 3, 1, 4)
        return qkv.reshape(3, B * self.num_heads, H * W, -1).unbind(0)

    def forward(self, x, depth=None):
        B, H, W, _ = x.shape
        q, k, v = self._qkv(x)
        n_rgb = H * W
        if self.depth_modality and depth is not None:
            _, Hd, Wd, _ = depth.shape
            qd, kd, vd = self._qkv(depth)
            q, k, v = torch.cat((q, qd), 1), torch.cat((k, kd), 1), torch.cat((v, vd), 1)
        attn = ((q * self.scale) @ k.transpose(-2, -1)).softmax(dim=-1)
        out = attn @ v
        x = out[:, :n_rgb].view(B, self.num_heads, H, W, -1).permute(0, 2, 3, 1, 4).reshape(B, H, W, -1)
        if self.depth_modality and depth is not None:
            depth = out[:, n_rgb:].view(B, self.num_heads, Hd, Wd, -1).permute(0, 2, 3, 1, 4)
            depth = self.proj(depth.reshape(B, Hd, Wd, -1))
        return self.proj(x), depth


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=True, norm_layer=nn.LayerNorm,
                 window_size=0, depth_modality=False, depth_window_size=0, layer_scale=False):
        super().__init__()
        if depth_modality and depth_window_size == 0:
            raise ValueError("unsupported")
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias,
                              depth_modality=depth_modality)
        self.ls1 = LayerScale(dim, 1.0) if layer_scale else None
        self.ls2 = LayerScale(dim, 1.0) if layer_scale else None
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.window_size = window_size
        self.depth_window_size = depth_window_size
        self.depth_modality = depth_modality

    def depth_window(self, H, Hd):
        ws = self.depth_window_size or int(self.window_size // (H / Hd))
        if ws not in DEPTH_WINDOW_SIZES:
            raise ValueError(f"Unexpected window size {ws}")
        return ws

    def forward(self, x, depth=None):
        shortcut = x
        x = self.norm1(x)
        H, W = x.shape[1], x.shape[2]
        if self.window_size > 0:
            x, pad_hw = window_partition(x, self.window_size)
        use_depth = self.depth_modality and depth is not None
        if use_depth:
            shortcut_d = depth
            depth = self.norm1(depth)
            Hd, Wd = depth.shape[1], depth.shape[2]
            dws = self.depth_window(H, Hd)
            depth, pad_d = window_partition(depth, dws)
        x, depth = self.attn(x, depth=depth if use_depth else None)
        if use_depth and self.window_size > 0:
            depth = window_unpartition(depth, dws, pad_d, (Hd, Wd))
        if self.window_size > 0:
            x = window_unpartition(x, self.window_size, pad_hw, (H, W))
        if self.ls1 is not None:
            x = self.ls1(x)
            if use_depth:
                depth = self.ls1(depth)
        x = shortcut + x
        y = self.mlp(self.norm2(x))
        if self.ls2 is not None:
            y = self.ls2(y)
        x = x + y
        if use_depth:
            depth = shortcut_d + depth
            yd = self.mlp(self.norm2(depth))
            if self.ls2 is not None:
                yd = self.ls2(yd)
            depth = depth + yd
        return x, depth


class ViT(nn.Module):
    """ViTDet backbone with a depth patch embedding; depth tokens join the window blocks only."""

    def __init__(self, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12,
                 mlp_ratio=4.0, qkv_bias=True, norm_layer=nn.LayerNorm, window_size=0,
                 window_block_indexes=(), pretrain_img_size=224, pretrain_use_cls_token=True,
                 depth_modality=False, depth_window_size=0, encoder_norm=False, layer_scale=False,
                 image_name="image", depth_name="depth"):
        super().__init__()
        self.pretrain_use_cls_token = pretrain_use_cls_token
        self.depth_modality = depth_modality
        self.image_name, self.depth_name = image_name, depth_name
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.patch_embed = PatchEmbed((patch_size, patch_size), (patch_size, patch_size), in_chans,
                                      embed_dim)
        n_pos = (pretrain_img_size // patch_size) ** 2 + (1 if pretrain_use_cls_token else 0)
        self.pos_embed = nn.Parameter(torch.zeros(1, n_pos, embed_dim))
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        self.pos_embed_depth = None
        if depth_modality:
            self.patch_embed_depth = PatchEmbed((16, 16), (16, 16), 1, embed_dim)
            self.pos_embed_depth = nn.Parameter(torch.zeros(1, n_pos, embed_dim))
        self.blocks = nn.ModuleList([
            Block(embed_dim, num_heads, mlp_ratio, qkv_bias, norm_layer,
                  window_size=window_size if i in window_block_indexes else 0,
                  depth_modality=depth_modality and (i in window_block_indexes),
                  depth_window_size=depth_window_size if i in window_block_indexes else 0,
                  layer_scale=layer_scale)
            for i in range(depth)])
        self.encoder_norm = norm_layer(embed_dim) if encoder_norm else nn.Identity()
        self.window_block_indexes = tuple(window_block_indexes)
        self.window_size = window_size
        self._square_pad = [256, 384, 512, 640, 768, 896, 1024, 1280]

    @property
    def num_channels(self):
        return [self.embed_dim]

    @property
    def size_divisibility(self):
        return self.patch_size

    def forward_tensors(self, image, depth=None):
        """image [B,3,P,P] normalised + padded, depth [B,P,P] standardised + padded -> [B,C,h,w]"""
        x = self.patch_embed(image)
        x = x + get_abs_pos(self.pos_embed, self.pretrain_use_cls_token, (x.shape[1], x.shape[2]))
        d = None
        if self.depth_modality and depth is not None:
            d = self.patch_embed_depth(depth[:, None])
            d = d + get_abs_pos(self.pos_embed_depth, self.pretrain_use_cls_token, (d.shape[1], d.shape[2]))
        for blk in self.blocks:
            if blk.depth_modality and d is not None:
                x, d = blk(x, depth=d)
            else:
                x, _ = blk(x)
        return self.encoder_norm(x).permute(0, 3, 1, 2)
