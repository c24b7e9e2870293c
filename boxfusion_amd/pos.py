"""Camera-ray Fourier embedding of the decoder memory (reference: boxfusion/pos.py:61-186).
Depends only on the intrinsics and image size, so the engine caches it per camera."""
from __future__ import annotations

from math import log2, pi

import torch
import torch.nn as nn
import torch.nn.functional as F


def generate_rays(K, width, height):
    """K f32[3,3] -> unit ray directions [H,W,3] at pixel centres (pos.py:61-108)."""
    device, dtype = K.device, K.dtype
    xs = torch.linspace(0, width - 1, width, device=device, dtype=dtype)
    ys = torch.linspace(0, height - 1, height, device=device, dtype=dtype)
    pix = torch.stack([xs.repeat(height, 1), ys.repeat(width, 1).t()], dim=2) + 0.5
    inv = torch.eye(3, device=device)
    inv[0, 0] = 1.0 / K[0, 0]
    inv[1, 1] = 1.0 / K[1, 1]
    inv[0, 2] = -K[0, 2] / K[0, 0]
    inv[1, 2] = -K[1, 2] / K[1, 1]
    homo = torch.cat([pix, torch.ones_like(pix[:, :, :1])], dim=2)
    dirs = torch.matmul(inv[None], homo.permute(2, 0, 1).flatten(-2)).view(3, height, width)
    return F.normalize(dirs.permute(1, 2, 0), dim=-1)


def fourier_features(x, dim, max_freq):
    """use_log=True, use_cos=False branch of generate_fourier_features (pos.py:110-149)."""
    num_bands = dim // x.shape[-1]
    scales = 2.0 ** torch.linspace(0.0, log2(max_freq), steps=num_bands, device=x.device,
                                   dtype=x.dtype)
    x = x.unsqueeze(-1) * scales[(None,) * (x.dim())] * pi
    return x.sin().flatten(3)


class CameraRayEmbedding(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.proj = nn.Linear(255, dim)

    def rays(self, K, size_wh, feat_size):
        """ray Fourier features for one camera: [feat, feat, 255]"""
        W, H = size_wh
        square_pad = feat_size * 16
        r = generate_rays(K, W, H)
        r = F.pad(r, (0, 0, 0, square_pad - r.shape[1], 0, square_pad - r.shape[0]))
        r = F.interpolate(r[None].permute(0, 3, 1, 2), (feat_size, feat_size), mode="nearest")
        r = F.normalize(r.permute(0, 2, 3, 1), dim=-1)
        return fourier_features(r, self.dim, feat_size // 2)[0]

    def forward(self, Ks, sizes_wh, feat_size):
        """Ks [B,3,3], sizes [(W,H)] -> [B, dim, feat, feat]"""
        f = torch.stack([self.rays(K, s, feat_size) for K, s in zip(Ks, sizes_wh)])
        return self.proj(f).permute(0, 3, 1, 2).contiguous()
