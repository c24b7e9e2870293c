"""CuTR (Cubify Transformer) RGB-D detector (reference: boxfusion/cubify_transformer.py).

`make_cubify_transformer(dimension, depth_model, embed_dim=256)` builds the same module tree and
parameter names as the reference (cubify_transformer.py:1232-1323) so `load_state_dict` accepts
its checkpoints.  The forward here is the fp32 definition of the maths; the MI355X path runs the
backbone through `boxfusion_amd.engine.CuTREngine` (gfx950 MFMA kernels) and the decoder tail
through `CubifyTransformer.decode`.

Inputs are a `FrameBatch`: normalised/padded image and standardised/padded depth tensors plus the
per-frame intrinsics, whitening parameters, T_gravity and original image sizes — exactly the
fields the reference reads from its BatchedSensors structure.
"""
from __future__ import annotations

import copy
import math
import os
from dataclasses import dataclass
from functools import partial
from typing import List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from boxfusion_amd.boxes import GeneralInstance3DBoxes
from boxfusion_amd.instances import Instances3D
from boxfusion_amd.pos import CameraRayEmbedding
from boxfusion_amd.transforms import euler_angles_to_matrix
from boxfusion_amd.vit import ViT


@dataclass
class FrameBatch:
    image: torch.Tensor            # [B,3,P,P] normalised, zero padded (Preprocessor.normalize/batch)
    depth: Optional[torch.Tensor]  # [B,P,P] standardised, zero padded
    depth_params: torch.Tensor     # [B,2] (trunc_mean, trunc_std) = WhitenedDepthMeasurementInfo
    K: torch.Tensor                # [B,3,3] image intrinsics
    T_gravity: Optional[torch.Tensor]  # [B,3,3]
    image_sizes: List[tuple]       # [(h, w)] before padding
    pad: int = 0                   # square pad size when `image` is not materialised (engine)
    K_inv: Optional[torch.Tensor] = None   # [B,3,3] precomputed inverse (keeps decode sync-free)

    @property
    def sizes_wh(self):
        return [(w, h) for h, w in self.image_sizes]


def conv_patch(conv, x):
    """Conv2d with kernel == stride and no padding (1x1 projections, 2x2/2 downsamplers) as one
    matmul over space-to-depth patches: the same contraction as the convolution, without the
    library's per-shape convolution search (which is unavailable inside a captured graph)."""
    k = conv.kernel_size[0]
    if conv.kernel_size != (k, k) or conv.stride != (k, k) or conv.padding != (0, 0) or conv.groups != 1:
        return conv(x)
    B, C, H, W = x.shape
    h, w = H // k, W // k
    p = x[:, :, :h * k, :w * k].reshape(B, C, h, k, w, k).permute(0, 2, 4, 1, 3, 5).reshape(B * h * w, C * k * k)
    y = F.linear(p, conv.weight.reshape(conv.out_channels, -1), conv.bias)
    return y.view(B, h, w, -1).permute(0, 3, 1, 2)


def run_seq(seq, x):
    """nn.Sequential forward with conv_patch for its patch convolutions"""
    if isinstance(seq, nn.Conv2d):
        return conv_patch(seq, x)
    if not isinstance(seq, nn.Sequential):
        return seq(x)
    for m in seq:
        x = conv_patch(m, x) if isinstance(m, nn.Conv2d) else m(x)
    return x


def clamp_xy(b, xmax, ymax):
    """clamp [..., 2k] x-columns to [0, xmax] and [..., 2k+1] y-columns to [0, ymax] with scalar
    bounds (same values as clamping against a [0..]/[W, H, ...] tensor; no host->device copy, so
    the decode stays graph-capturable)."""
    cols = [b[..., c].clamp(0, xmax if c % 2 == 0 else ymax) for c in range(b.shape[-1])]
    return torch.stack(cols, -1)


def box_cxcywh_to_xyxy(x):
    xc, yc, w, h = x.unbind(-1)
    return torch.stack([xc - 0.5 * w, yc - 0.5 * h, xc + 0.5 * w, yc + 0.5 * h], dim=-1)


def box_xyxy_to_cxcywh(x):
    x0, y0, x1, y1 = x.unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, x1 - x0, y1 - y0], dim=-1)


class LayerNorm2D(nn.Module):
    def __init__(self, normalized_shape):
        super().__init__()
        self.ln = nn.LayerNorm(normalized_shape)

    def forward(self, x):
        return self.ln(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)


class MLP(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))

    def forward(self, x):
        for i, layer in enumerate(self.layers):
            x = F.relu(layer(x)) if i < self.num_layers - 1 else layer(x)
        return x


# --------------------------------------------------------------------------------------------
# decoder (cubify_transformer.py:93-352)
# --------------------------------------------------------------------------------------------
class GlobalCrossAttention(nn.Module):
    def __init__(self, dim, num_heads, rpe_hidden_dim=512, feature_stride=16):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.feature_stride = feature_stride
        self.cpb_mlp1 = self._cpb(2, rpe_hidden_dim, num_heads)
        self.cpb_mlp2 = self._cpb(2, rpe_hidden_dim, num_heads)
        self.q = nn.Linear(dim, dim)
        self.k = nn.Linear(dim, dim)
        self.v = nn.Linear(dim, dim)
        self.proj = nn.Linear(dim, dim)

    # the HIP bias/softmax path on device tensors (BF_DECODER_TORCH=1: the torch ops below)
    fused = os.environ.get("BF_DECODER_TORCH", "0") != "1"

    def _positions(self, h, w, dev):
        """pos_x / pos_y of rpe() ([w], [h] f32), built by the same torch ops, cached"""
        key = (h, w, dev)
        cache = self.__dict__.setdefault("_pos_cache", {})
        if key not in cache:
            s = self.feature_stride
            cache[key] = (torch.linspace(0.5, w - 0.5, w, dtype=torch.float32, device=dev) * s,
                          torch.linspace(0.5, h - 0.5, h, dtype=torch.float32, device=dev) * s)
        return cache[key]

    @staticmethod
    def _cpb(i, h, o):
        return nn.Sequential(nn.Linear(i, h, bias=True), nn.ReLU(inplace=True), nn.Linear(h, o, bias=False))

    def rpe(self, reference_2d, h, w):
        """linear relative position bias [B, heads, nQ_box, h*w] (:146-167)"""
        s = self.feature_stride
        ref = torch.cat([reference_2d[..., :2] - reference_2d[..., 2:] / 2,
                         reference_2d[..., :2] + reference_2d[..., 2:] / 2], dim=-1)  # B,nQ,1,4
        dev = reference_2d.device
        pos_x = torch.linspace(0.5, w - 0.5, w, dtype=torch.float32, device=dev)[None, None, :, None] * s
        pos_y = torch.linspace(0.5, h - 0.5, h, dtype=torch.float32, device=dev)[None, None, :, None] * s
        rx = self.cpb_mlp1(ref[..., 0::2] - pos_x)
        ry = self.cpb_mlp2(ref[..., 1::2] - pos_y)
        return (rx[:, :, None] + ry[:, :, :, None]).flatten(2, 3).permute(0, 3, 1, 2)

    def forward(self, query, reference_2d, k_in, v_in, hw, box_mask, kv=None):
        """kv: this layer's (k(k_in), v(v_in)) when the caller computed every layer's projections
        of the (layer-invariant) memory in one GEMM each (CubifyTransformer.decode)"""
        h, w = hw
        B, N, C = k_in.shape
        kp, vp = kv if kv is not None else (self.k(k_in), self.v(v_in))
        if (self.fused and query.is_cuda and isinstance(box_mask, slice) and box_mask.step is None
                and box_mask.stop is None and C == 32 * self.num_heads and h <= 128 and w <= 128
                and w >= 4 and query.dtype == torch.float32):
            # bf_xattn_f32: logits, bias, clip, softmax and P.V in one kernel (the bias tables
            # from bf_cpb_mlp); the [B,heads,Nq,h*w] logits never reach HBM
            from boxfusion_amd import _lib
            pos_x, pos_y = self._positions(h, w, query.device)
            ref = reference_2d[:, :, 0].contiguous()
            m1, m2 = self.cpb_mlp1, self.cpb_mlp2
            rx = _lib.cpb_mlp(ref, pos_x, 0, m1[0].weight, m1[0].bias, m1[2].weight)
            ry = _lib.cpb_mlp(ref, pos_y, 1, m2[0].weight, m2[0].bias, m2[2].weight)
            x = _lib.xattn(self.q(query), kp, vp, rx, ry, h, w, box_mask.start or 0, self.num_heads,
                           self.scale)
            return self.proj(x)
        k = kp.reshape(B, N, self.num_heads, C // self.num_heads).permute(0, 2, 1, 3)
        v = vp.reshape(B, N, self.num_heads, C // self.num_heads).permute(0, 2, 1, 3)
        B, Nq, C = query.shape
        q = self.q(query).reshape(B, Nq, self.num_heads, C // self.num_heads).permute(0, 2, 1, 3)
        attn = (q * self.scale) @ k.transpose(-2, -1)
        if (attn.is_cuda and self.fused and isinstance(box_mask, slice) and box_mask.step is None
                and box_mask.stop is None and attn.dtype == torch.float32 and attn.is_contiguous()):
            # bf_cpb_mlp + bf_rpe_softmax: the bias tables, then bias + clip + softmax in one pass
            from boxfusion_amd import _lib
            pos_x, pos_y = self._positions(h, w, attn.device)
            ref = reference_2d[:, :, 0].contiguous()
            m1, m2 = self.cpb_mlp1, self.cpb_mlp2
            rx = _lib.cpb_mlp(ref, pos_x, 0, m1[0].weight, m1[0].bias, m1[2].weight)
            ry = _lib.cpb_mlp(ref, pos_y, 1, m2[0].weight, m2[0].bias, m2[2].weight)
            _lib.rpe_softmax(attn, rx, ry, h, w, box_mask.start or 0)
        else:
            attn[:, :, box_mask] += self.rpe(reference_2d, h, w)
            fmin, fmax = torch.finfo(attn.dtype).min, torch.finfo(attn.dtype).max
            attn = attn.clip(min=fmin, max=fmax).softmax(dim=-1)
        x = (attn @ v).transpose(1, 2).reshape(B, Nq, C)
        return self.proj(x)


class PreNormGlobalDecoderLayer(nn.Module):
    def __init__(self, xattn, d_model=256, d_ffn=1024, n_heads=8):
        super().__init__()
        self.xattn = xattn
        self.norm1 = nn.LayerNorm(d_model)
        self.self_attn = nn.MultiheadAttention(d_model, n_heads, dropout=0.0)
        self.norm2 = nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.norm3 = nn.LayerNorm(d_model)

    def forward(self, tgt, query_pos, reference_2d, src, src_pos, hw, self_attn_mask, box_mask, kv=None):
        t2 = self.norm2(tgt)
        q = k = t2 + query_pos
        t2 = self.self_attn(q.transpose(0, 1), k.transpose(0, 1), t2.transpose(0, 1),
                            attn_mask=self_attn_mask)[0].transpose(0, 1)
        tgt = tgt + t2
        t2 = self.norm1(tgt)
        k_in = src + src_pos if kv is None else src        # (only its shape is read with kv)
        t2 = self.xattn(t2 + query_pos, reference_2d, k_in, src, hw, box_mask, kv=kv)
        tgt = tgt + t2
        t2 = self.linear2(F.relu(self.linear1(self.norm3(tgt))))
        return tgt + t2


class ScalePredictor(nn.Module):
    def __init__(self, embed_dim):
        super().__init__()
        self.shift = nn.Linear(embed_dim, 1)
        self.scale = nn.Linear(embed_dim, 1)

    def forward(self, x, state):
        state["pred_parameters"] = torch.cat((torch.exp(self.shift(x[:, 0:1])),
                                              torch.exp(self.scale(x[:, 1:2]))), dim=-1)
        return x[:, 2:]


class ClassPredictor(nn.Module):
    def __init__(self, embed_dim, num_classes, prior_prob=0.01):
        super().__init__()
        self.num_classes = num_classes
        self.linear = nn.Linear(embed_dim, num_classes)
        self.linear.bias.data.fill_(-math.log((1 - prior_prob) / prior_prob))

    def forward(self, x, state):
        state["pred_logits"] = self.linear(x)
        return x


class DeltaBox2DTransform(nn.Module):
    def __init__(self, wh_ratio_clip=0.016):
        super().__init__()
        self._wh_ratio_clip = wh_ratio_clip
        self.register_buffer("means", torch.tensor((0.0, 0.0, 0.0, 0.0)), False)
        self.register_buffer("stds", torch.tensor((1.0, 1.0, 1.0, 1.0)), False)

    def apply_deltas(self, deltas, boxes, clamp_shape):
        """cubify_transformer.py:478-511 (no centre clamp, clamp to the padded image)"""
        dxy, dwh = deltas[..., :2], deltas[..., 2:]
        pxy, pwh = boxes[..., :2], boxes[..., 2:]
        max_ratio = np.abs(np.log(self._wh_ratio_clip))
        dwh = dwh.clamp(min=-max_ratio, max=max_ratio)
        gxy = pxy + pwh * dxy
        gwh = pwh * dwh.exp()
        b = torch.cat([gxy - gwh * 0.5, gxy + gwh * 0.5], dim=-1)
        return clamp_xy(b, clamp_shape[1], clamp_shape[0])


class DeltaBox2DPredictor(nn.Module):
    def __init__(self, embed_dim, num_layers=3):
        super().__init__()
        self.mlp = MLP(embed_dim, embed_dim, 4, num_layers)
        nn.init.constant_(self.mlp.layers[-1].weight.data, 0)
        nn.init.constant_(self.mlp.layers[-1].bias.data, 0)
        self.transform = DeltaBox2DTransform()

    def forward(self, x, state):
        deltas = self.mlp(x)
        state["pred_boxes_delta"] = deltas
        state["pred_boxes"] = box_xyxy_to_cxcywh(
            self.transform.apply_deltas(deltas, state["proposal_boxes"], state["clamp_shape"]))
        return x


class AbsoluteBox3DPredictor(nn.Module):
    def __init__(self, embed_dim, num_layers=3):
        super().__init__()
        self.mlp = MLP(embed_dim, embed_dim, 2 + 1 + 3 + 1, num_layers)
        nn.init.constant_(self.mlp.layers[-1].weight.data[:2], 0)
        nn.init.constant_(self.mlp.layers[-1].bias.data[:2], 0)

    def forward(self, x, state):
        """z: yaw-only pose, whitened-depth scale/shift (cubify_transformer.py:592-643)"""
        B = x.shape[0]
        d2, z, dims, yaw = torch.split(self.mlp(x), (2, 1, 3, 1), dim=-1)
        pose = torch.cat((yaw, torch.zeros_like(yaw), torch.zeros_like(yaw)), dim=-1)
        pose = euler_angles_to_matrix(pose.view(-1, 3), "YXZ").view(B, -1, 3, 3)
        params = state["depth_params"]                 # [B,2] -> shift, scale per frame
        if params is None:                             # RGB-only model: predicted scale tokens
            params = state["pred_parameters"][:, 0]
        shift, scale = params[:, None, 0:1], params[:, None, 1:2]
        z_scaled = scale * z + shift
        dims = torch.exp(dims.clip(max=5)) * scale
        cs = state["clamp_shape"]
        pxy = state["pred_boxes"][..., :2] + d2 * state["pred_boxes"][..., 2:]
        pxy = clamp_xy(pxy, cs[1], cs[0])
        state.update(pred_proj_xy=pxy, pred_z_unscaled=z, pred_z_scaled=z_scaled, pred_dims=dims,
                     pred_pose=pose)
        return x


class Box2DPromptEncoderLearned(nn.Module):
    def __init__(self, embed_dim, max_x=1280, max_y=1280, max_w=1280, max_h=1280):
        super().__init__()
        self.x = nn.Embedding(max_x, embed_dim // 4)
        self.y = nn.Embedding(max_y, embed_dim // 4)
        self.w = nn.Embedding(max_w, embed_dim // 4)
        self.h = nn.Embedding(max_h, embed_dim // 4)
        self.register_buffer("min_bounds", torch.tensor([0.0, 0.0, 0.0, 0.0]).float())
        self.register_buffer("max_bounds", torch.tensor([max_x - 1, max_y - 1, max_w - 1, max_h - 1]).float())

    def forward(self, boxes):
        idx = torch.clamp(boxes, min=self.min_bounds[None, None], max=self.max_bounds[None, None]).int()
        return torch.cat((self.x(idx[..., 0]), self.y(idx[..., 1]), self.w(idx[..., 2]),
                          self.h(idx[..., 3])), dim=-1)


class PromptEncoders(nn.Module):
    def __init__(self, **kwargs):
        super().__init__()
        for k, v in kwargs.items():
            setattr(self, k, v)


class MetricQueries(nn.Module):
    def __init__(self, input_channels, input_stride):
        super().__init__()
        self.embed_dim = input_channels
        self.query_embed = nn.Embedding(2, input_channels)


class EncoderProposals(nn.Module):
    def __init__(self, input_channels, input_stride, level_strides, predictors, min_size=50,
                 top_k_test=300):
        super().__init__()
        self.embed_dim = input_channels
        self.input_stride = input_stride
        self.level_strides = level_strides
        self.predictors = nn.ModuleList(predictors)
        self.min_proposal_size = min_size
        self.top_k_test = top_k_test
        self.query_embed = nn.Embedding(1200, input_channels)
        self.enc_output_proj = nn.ModuleList()
        for s in level_strides:
            if s == input_stride:
                self.enc_output_proj.append(nn.Identity())
            else:
                scale = int(math.log2(s / input_stride))
                layers = []
                for _ in range(scale - 1):
                    layers += [nn.Conv2d(self.embed_dim, self.embed_dim, 2, 2),
                               LayerNorm2D(self.embed_dim), nn.GELU()]
                layers.append(nn.Conv2d(self.embed_dim, self.embed_dim, 2, 2))
                self.enc_output_proj.append(nn.Sequential(*layers))
        self.enc_output = nn.Linear(self.embed_dim, self.embed_dim)
        self.enc_output_norm = nn.LayerNorm(self.embed_dim)

    def proposals(self, memory, hw):
        """gen_encoder_output_proposals (:864-916) for an unpadded (mask-free) memory"""
        B, _, C = memory.shape
        h, w = hw
        m = memory.view(B, h, w, C).permute(0, 3, 1, 2)
        mems = [run_seq(proj, m) for proj in self.enc_output_proj]
        out_mem = torch.cat([x.flatten(2).transpose(1, 2) for x in mems], dim=1)
        props = []
        for lvl, x in enumerate(mems):
            H_, W_ = x.shape[-2:]
            stride = self.level_strides[lvl]
            gy, gx = torch.meshgrid(torch.linspace(0, H_ - 1, H_, dtype=torch.float32, device=memory.device),
                                    torch.linspace(0, W_ - 1, W_, dtype=torch.float32, device=memory.device),
                                    indexing="ij")
            grid = (torch.cat([gx.unsqueeze(-1), gy.unsqueeze(-1)], -1)[None].expand(B, -1, -1, -1) + 0.5) * stride
            wh = torch.ones_like(grid) * self.min_proposal_size * (2.0 ** lvl)
            props.append(torch.cat((grid, wh), -1).view(B, -1, 4))
        props = torch.cat(props, 1)
        stride0 = self.level_strides[0]
        # (props > 0.01 * img) & (props < 0.99 * img) with img = [W, H, W, H] in f32, per column
        lim = [(float(np.float32(0.01) * np.float32(v)), float(np.float32(0.99) * np.float32(v)))
               for v in (w * stride0, h * stride0, w * stride0, h * stride0)]
        valid = torch.stack([(props[..., c] > lo) & (props[..., c] < hi) for c, (lo, hi) in enumerate(lim)],
                            -1).all(-1, keepdim=True)
        props = props.masked_fill(~valid, max(h, w) * stride0)
        out_mem = out_mem.masked_fill(~valid, 0.0)
        return self.enc_output_norm(self.enc_output(out_mem)), props


class PromptDecoder(nn.Module):
    def __init__(self, embed_dim, layer, num_layers, predictors, norm):
        super().__init__()
        self.embed_dim = embed_dim
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(num_layers)])
        self.num_layers = num_layers
        self.predictors = nn.ModuleList([nn.ModuleList([copy.deepcopy(p) for p in predictors])
                                         for _ in range(num_layers)])
        self.norm = norm


class CubifyAnythingPrompting(nn.Module):
    def __init__(self, embed_dim, prompters, encoders):
        super().__init__()
        self.embed_dim = embed_dim
        self.prompters = nn.ModuleList(prompters)
        self.encoders = encoders
        # the reference shares the encoders with every prompter (cubify_transformer.py:1013-1014),
        # so its state dict lists them under each prompter as well
        for p in self.prompters:
            p.encoders = encoders


class Joiner(nn.Sequential):
    def __init__(self, backbone):
        super().__init__(backbone)

    @property
    def backbone(self):
        return self[0]


class CubifyTransformer(nn.Module):
    def __init__(self, backbone, prompting, decoder, pixel_mean, pixel_std, pos_embedding,
                 topk_per_image=100):
        super().__init__()
        self.backbone = backbone
        self.prompting = prompting
        self.decoder = decoder
        self.pos_embedding = pos_embedding
        self.register_buffer("pixel_mean", torch.tensor(pixel_mean).view(-1, 1, 1), False)
        self.register_buffer("pixel_std", torch.tensor(pixel_std).view(-1, 1, 1), False)
        C = backbone.backbone.num_channels[0]
        self.input_proj = nn.ModuleList([nn.Sequential(nn.Conv2d(C, decoder.embed_dim, 1),
                                                       nn.GroupNorm(32, decoder.embed_dim))])
        self.level_embed = nn.Parameter(torch.zeros(1, decoder.embed_dim))
        self.topk_per_image = topk_per_image

    @property
    def device(self):
        return self.pixel_mean.device

    # ---- forward -----------------------------------------------------------------------------
    def forward(self, batch) -> List[Instances3D]:
        """`model(packaged)` (demo.py:135): the BatchedSensors dict of Preprocessor.preprocess runs
        on the MI355X engine (forward_sensors); a FrameBatch of materialised tensors runs the fp32
        definition of the maths (the parity reference of the tests)."""
        if isinstance(batch, dict):
            return self.forward_sensors(batch)
        feat = self.backbone.backbone.forward_tensors(batch.image, batch.depth)
        return self.decode(feat, batch)

    def forward_sensors(self, batched_sensors, sensor_name="wide"):
        """CubifyTransformer.inference (cubify_transformer.py:1172-1227) for the reference's input
        structure on the MI355X engine.  One CuTREngine is kept per (batch, frame size, pad,
        depth ratio, device).  Device tensors only: there is no CPU path."""
        from boxfusion_amd import _lib
        from boxfusion_amd.engine import CuTREngine
        x = sensor_inputs(batched_sensors, sensor_name)
        raw = x["image_raw"]
        if not raw.is_cuda:
            raise _lib.HipError("boxfusion_amd runs on the HIP device: move the inputs with "
                                "move_input_to_current_device(packaged, model.pixel_mean) first")
        if self.backbone.backbone.depth_modality and x["depth_std"] is None:
            raise _lib.HipError("depth model without a depth measurement")
        B, _, H, W = raw.shape
        key = (B, H, W, x["pad"], x["ratio"], raw.device)
        engines = self.__dict__.setdefault("_engines", {})
        if key not in engines:
            engines[key] = CuTREngine(self, B, H, W, pad=x["pad"], device=raw.device, depth_ratio=x["ratio"])
        res = engines[key](raw.contiguous(), x["depth_std"], x["depth_params"], x["K"], x["T_gravity"],
                           x["image_sizes"], chw=True, pixel_mean=x["pixel_mean"], pixel_std=x["pixel_std"])
        # the engine's instances are views of its persistent output buffers (the next call reuses
        # them); the reference's model(packaged) hands out fresh tensors, so the boundary copies
        # (100 rows per frame, one small device copy per field)
        return [r.clone() for r in res]

    def _memory_kv(self, src, pos):
        """Every decoder layer's cross-attention k(src + pos) and v(src) in one GEMM each (the
        memory is the same for all layers): [B, N, layers*C] pairs, layer l in columns
        [l*C, (l+1)*C).  Device only (the CPU path keeps the per-layer linears)."""
        if not src.is_cuda:
            return None
        cache = self.__dict__.setdefault("_kv_cache", {})
        key = src.device
        if key not in cache:
            xs = [layer.xattn for layer in self.decoder.layers]
            cache[key] = (torch.cat([x.k.weight for x in xs]).detach(), torch.cat([x.k.bias for x in xs]).detach(),
                          torch.cat([x.v.weight for x in xs]).detach(), torch.cat([x.v.bias for x in xs]).detach())
        wk, bk, wv, bv = cache[key]
        return F.linear(src + pos, wk, bk), F.linear(src, wv, bv)

    # ---- everything after the backbone (cubify_transformer.py:1172-1227) -------------------------
    def decode(self, feat, batch: FrameBatch, pos=None):
        B, _, h, w = feat.shape
        if pos is None:
            pos = self.pos_embedding(batch.K, batch.sizes_wh, w)
        src = run_seq(self.input_proj[0], feat).flatten(2).transpose(1, 2)
        pos = pos.flatten(2).transpose(1, 2) + self.level_embed[0].view(1, 1, -1)
        metric, enc = self.prompting.prompters
        clamp_shape = tuple(batch.image.shape[-2:]) if batch.image is not None else (batch.pad, batch.pad)
        # encoder proposals + top-k (:918-943)
        memory, props = enc.proposals(src, (h, w))
        st = dict(proposal_boxes=props, clamp_shape=clamp_shape)
        x = memory
        for p in enc.predictors:
            x = p(x, st)
        topk = torch.topk(st["pred_logits"][..., 0], min(enc.top_k_test, props.shape[1]), dim=1)[1]
        ref_boxes = torch.gather(st["pred_boxes"], 1, topk[..., None].expand(-1, -1, 4))
        box_pos = self.prompting.encoders.box_2d_encoder(ref_boxes.detach())
        nq = box_pos.shape[1]
        query = torch.cat([metric.query_embed.weight[None].expand(B, -1, -1),
                           enc.query_embed.weight[None, :nq].expand(B, -1, -1)], dim=1)
        qpos = torch.cat([torch.zeros(B, 2, self.decoder.embed_dim, device=feat.device), box_pos], 1)
        n = 2 + nq
        self_mask = torch.ones((n, n), dtype=torch.bool, device=feat.device)
        self_mask[:2, :2] = False
        self_mask[2:, 2:] = False
        box_mask = slice(2, None)      # the nq box queries follow the 2 metric queries
        out = query
        kv = self._memory_kv(src, pos)
        C = self.decoder.embed_dim
        for lid, layer in enumerate(self.decoder.layers):
            kv_l = None if kv is None else (kv[0][..., lid * C:(lid + 1) * C], kv[1][..., lid * C:(lid + 1) * C])
            out = layer(out, qpos, ref_boxes.detach()[:, :, None], src, pos, (h, w), self_mask, box_mask,
                        kv=kv_l)
            y = self.decoder.norm(out)
            st = dict(proposal_boxes=ref_boxes, clamp_shape=clamp_shape,
                      depth_params=batch.depth_params if batch.depth is not None else None)
            last = lid == len(self.decoder.layers) - 1
            for p in self.decoder.predictors[lid]:
                if not last and not isinstance(p, DeltaBox2DPredictor):
                    # before the last layer only the refined 2-D boxes are read (the next layer's
                    # reference boxes); the other heads' outputs are overwritten unread
                    if isinstance(p, ScalePredictor):
                        y = y[:, 2:]
                    continue
                y = p(y, st)
            st["object_desc"] = y
            ref_boxes = st["pred_boxes"]
        return self.inference(st, batch)

    def inference(self, st, batch: FrameBatch):
        """EncoderProposals.inference + inference_single_image (:945-996)"""
        results = []
        for i in range(len(batch.image_sizes)):
            K = batch.K[i][None].expand(st["pred_z_scaled"].shape[1], -1, -1)
            z = st["pred_z_scaled"][i]
            uvz = torch.cat((z * st["pred_proj_xy"][i], z), dim=-1)[..., None]
            Kinv = (torch.linalg.inv(K) if batch.K_inv is None
                    else batch.K_inv[i][None].expand(K.shape[0], -1, -1))
            xyz = torch.bmm(Kinv, uvz)[..., 0]
            pose = st["pred_pose"][i]
            if batch.T_gravity is not None:
                pose = batch.T_gravity[i][None] @ pose
            results.append(self.select_topk(st, i, xyz, pose, batch.image_sizes[i]))
        return results

    def select_topk(self, st, i, xyz, pose, image_size):
        prob = st["pred_logits"][i].sigmoid()
        vals, idx = torch.topk(prob.view(-1), self.topk_per_image)
        boxes_i = idx // prob.shape[-1]
        labels = idx % prob.shape[-1]
        r = Instances3D(image_size)
        r.scores = vals
        r.pred_classes = labels
        boxes = box_cxcywh_to_xyxy(st["pred_boxes"][i])[boxes_i]
        boxes = clamp_xy(boxes, image_size[1], image_size[0])
        r.pred_boxes = boxes
        r.pred_logits = st["pred_logits"][i][boxes_i]
        dims = st["pred_dims"][i][boxes_i]
        r.pred_boxes_3d = GeneralInstance3DBoxes(torch.cat((xyz[boxes_i], dims.flip(-1)), dim=-1),
                                                 pose[boxes_i])
        r.object_desc = st["object_desc"][i][boxes_i]
        r.pred_proj_xy = st["pred_proj_xy"][i][boxes_i]
        return r


def sensor_inputs(batched_sensors, sensor_name="wide"):
    """what the detector reads from Preprocessor.preprocess's BatchedSensors (device agnostic):
    the unpadded uint8 [B,3,H,W] frames (ImageList.raw) and their normalisation constants, the
    standardised depth [B,H/r,W/r] + whitening parameters (cubify_transformer.py:568-586), the
    image K (pos.py:64, :983-986), T_gravity (:991-992), image sizes, square pads and the
    rgb -> depth ratio"""
    sensor = batched_sensors[sensor_name]
    img = sensor["image"]
    raw = img.data.raw
    if raw is None or raw.dtype != torch.uint8 or raw.dim() != 4:
        raise ValueError("expected the uint8 [B,3,H,W] frames of Preprocessor.batch")
    consts = getattr(img, "normalize_consts", None)
    if consts is None:
        raise ValueError("the image measurement was not normalised by Preprocessor.normalize")
    dev = raw.device
    dep = sensor.get("depth")
    sens = img.sensor
    out = dict(image_raw=raw, image=img.data, pixel_mean=consts[0], pixel_std=consts[1],
               pad=int(img.data.padded_hw[0]),
               K=torch.stack([info.K[-1] for info in img.info]).to(dev, torch.float32),
               T_gravity=(torch.stack([s_.T_gravity[-1] for s_ in sens]).to(dev, torch.float32)
                          if all(s_.has("T_gravity") for s_ in sens) else None),
               image_sizes=[tuple(int(v) for v in s_) for s_ in img.data.image_sizes],
               ratio=int(getattr(dep, "rgb_to_depth_ratio", 1)) if dep is not None else 1,
               depth=dep.data if dep is not None else None, depth_std=None, depth_params=None)
    if dep is not None:
        out["depth_std"] = dep.data.raw.to(torch.float32).contiguous()
        out["depth_params"] = torch.stack([torch.as_tensor(i.parameters).reshape(-1)[:2]
                                           for i in dep.info]).to(dev, torch.float32)
    return out


def frame_batch(batched_sensors, sensor_name="wide"):
    """FrameBatch of the materialised (normalised, zero-padded) tensors -- the fp32 definition's
    input (tests: the same extraction as the engine path)"""
    x = sensor_inputs(batched_sensors, sensor_name)
    return FrameBatch(image=x["image"].tensor, depth=x["depth"].tensor if x["depth"] is not None else None,
                      depth_params=x["depth_params"], K=x["K"], T_gravity=x["T_gravity"],
                      image_sizes=x["image_sizes"])


def make_cubify_transformer(dimension, depth_model, embed_dim=256):
    """cubify_transformer.py:1232-1323: same module tree / parameter names."""
    heads = {768: 12, 384: 6, 192: 3}[dimension]
    backbone = Joiner(ViT(patch_size=16, embed_dim=dimension, depth=12, num_heads=heads,
                          window_size=16, mlp_ratio=4, qkv_bias=True,
                          norm_layer=partial(nn.LayerNorm, eps=1e-6),
                          window_block_indexes=[0, 1, 3, 4, 6, 7, 9, 10],
                          depth_modality=depth_model, depth_window_size=None,
                          layer_scale=not depth_model, encoder_norm=not depth_model,
                          pretrain_img_size=512 if not depth_model else 224))
    box_enc = Box2DPromptEncoderLearned(embed_dim)
    prompting = CubifyAnythingPrompting(
        embed_dim,
        [MetricQueries(embed_dim, 16),
         EncoderProposals(embed_dim, 16, [16, 32, 64],
                          [ClassPredictor(embed_dim, 2), DeltaBox2DPredictor(embed_dim, 3)],
                          top_k_test=300)],
        PromptEncoders(box_2d_encoder=box_enc))
    layer = PreNormGlobalDecoderLayer(GlobalCrossAttention(embed_dim, 8, 512, 16), d_model=embed_dim,
                                      d_ffn=2048, n_heads=8)
    decoder = PromptDecoder(embed_dim, layer, 6,
                            [ScalePredictor(embed_dim), ClassPredictor(embed_dim, 2),
                             DeltaBox2DPredictor(embed_dim, 3), AbsoluteBox3DPredictor(embed_dim, 3)],
                            nn.LayerNorm(embed_dim))
    return CubifyTransformer(backbone, prompting, decoder, [123.675, 116.28, 103.53],
                             [58.395, 57.12, 57.375], CameraRayEmbedding(embed_dim))
