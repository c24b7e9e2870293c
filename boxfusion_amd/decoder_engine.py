"""The CuTR decoder tail on the MI355X kernels, f32 end to end.

`DecoderEngine(model, B, h, w)` runs what `CubifyTransformer.decode` + `inference` run
(cubify_transformer.py:1172-1227 of the reference: input_proj, the camera-ray position embedding,
EncoderProposals :812-943, the PromptDecoder layers :93-352 and inference_single_image :945-996)
for a batch of B frames with an h x w feature grid, on bf_dec_native.hip / bf_decoder.hip:

  a6  input_proj (1x1 conv + GroupNorm)      bf_gemm_f32 + bf_groupnorm_cl_f32 (also src + pos)
      CameraRayEmbedding                     bf_ray_fourier_f32 + bf_gemm_f32 (cached per camera)
  a7  level convolutions (2x2/2)             bf_s2d_f32 + bf_gemm_f32 (+ LayerNorm2D/GELU rows)
      enc_output + LayerNorm                 bf_gemm_f32 (row map = the masked cat) + bf_ln_rows_f32
      class / box predictors, top-300        bf_gemm_f32 MLP + bf_row_heads_f32 + bf_topk_rows_f32
      box prompt embedding                   bf_prop_select_f32
  a8  every decoder layer                    bf_ln_rows_f32 (+ y + query_pos), bf_gemm_f32
                                             (in_proj / out_proj / q / proj / FFN, residual in
                                             the epilogue), bf_self_attn_f32 (block mask),
                                             bf_cpb_mlp + bf_xattn_f32 (RPE cross-attention)
      the predictors                         bf_gemm_f32 MLPs + bf_row_heads_f32
  a9  inference_single_image                 bf_infer_select_f32 (sigmoid, top-100, 3-D lift,
                                             T_gravity R, gathers)

About 140 launches per batch instead of ~1000 torch / hipBLASLt ones; every buffer is
preallocated, nothing synchronises the host, so the whole decode is HIP-graph capturable.
Numerics: f32; summation orders differ from BLAS, so results agree with the torch definition
(`CubifyTransformer.decode`, which the CPU tests pin to the reference's fp32 goldens) to f32
rounding.  No CPU path: the kernels need the HIP device.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from boxfusion_amd import _lib
from boxfusion_amd.boxes import GeneralInstance3DBoxes
from boxfusion_amd.cubify_transformer import (AbsoluteBox3DPredictor, ClassPredictor, DeltaBox2DPredictor,
                                              LayerNorm2D, ScalePredictor)
from boxfusion_amd.instances import Instances3D


def _f(t):
    return t.detach().to(torch.float32).contiguous()


def _linear(m):
    return _f(m.weight), _f(m.bias) if m.bias is not None else None


class DecoderEngine:
    def __init__(self, model, batch, h, w, device="cuda"):
        dev = torch.device(device)
        self.model, self.dev, self.B, self.h, self.w = model, dev, batch, h, w
        dec = model.decoder
        C = self.C = dec.embed_dim
        metric, enc = model.prompting.prompters
        self.enc = enc
        self.nm = metric.query_embed.num_embeddings                 # metric queries (2)
        self.nq = enc.top_k_test                                   # box queries (300)
        self.n = self.nm + self.nq
        self.topk = model.topk_per_image
        layer0 = dec.layers[0]
        self.heads = layer0.self_attn.num_heads
        if C != 32 * self.heads or layer0.xattn.num_heads != self.heads:
            raise _lib.HipError("DecoderEngine: head dim 32")
        B, P0 = batch, h * w
        self.P0 = P0
        # ---- a6: input projection + GroupNorm, ray position embedding ------------------------
        conv, gn = model.input_proj[0][0], model.input_proj[0][1]
        self.w_inproj = _f(conv.weight.reshape(C, -1))
        self.b_inproj = _f(conv.bias)
        self.gn = (gn.num_groups, _f(gn.weight), _f(gn.bias), gn.eps)
        pe = model.pos_embedding
        self.ray_nb = pe.dim // 3
        self.ray_scales = (2.0 ** torch.linspace(0.0, math.log2(w // 2), steps=self.ray_nb, device=dev,
                                                 dtype=torch.float32)).contiguous()
        wr = torch.zeros((pe.dim, 256 * math.ceil(pe.proj.in_features / 256)), device=dev)
        wr[:, : pe.proj.in_features] = pe.proj.weight.detach()
        self.w_ray, self.b_ray = wr.contiguous(), _f(pe.proj.bias)
        self.level_embed = _f(model.level_embed[0])
        self._pos_cache = {}
        # ---- a7: proposal levels -------------------------------------------------------------
        if list(enc.level_strides) != [enc.input_stride * 2 ** i for i in range(len(enc.level_strides))]:
            raise _lib.HipError("DecoderEngine: level strides must double from the input stride")
        self.levels = []                      # per level: list of ops on a channel-last map
        hs, ws, rows = [], [], []
        for lvl, proj in enumerate(enc.enc_output_proj):
            mods = [] if isinstance(proj, nn.Identity) else (list(proj) if isinstance(proj, nn.Sequential) else [proj])
            ops, i = [], 0
            while i < len(mods):
                m = mods[i]
                if isinstance(m, nn.Conv2d):
                    if m.kernel_size != (2, 2) or m.stride != (2, 2):
                        raise _lib.HipError("DecoderEngine: level convolutions are 2x2 / 2")
                    ops.append(("conv", _f(m.weight.reshape(m.out_channels, -1)), _f(m.bias)))
                    i += 1
                elif isinstance(m, LayerNorm2D):
                    gelu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.GELU)
                    ops.append(("ln", _f(m.ln.weight), _f(m.ln.bias), m.ln.eps, gelu))
                    i += 2 if gelu else 1
                else:
                    raise _lib.HipError(f"DecoderEngine: unsupported level module {type(m).__name__}")
            self.levels.append(ops)
            hs.append(h >> lvl)
            ws.append(w >> lvl)
            if (h >> lvl) << lvl != h or (w >> lvl) << lvl != w:
                raise _lib.HipError("DecoderEngine: the feature grid must halve evenly per level")
            rows.append((h >> lvl) * (w >> lvl))
        self.lvl_hw, self.lvl_rows = list(zip(hs, ws)), rows
        self.Pt = sum(rows)
        # row offsets of each level's block in LV ([level][frame][position])
        self.lvl_off = np.cumsum([0] + [B * r for r in rows]).tolist()
        self.w_encout, self.b_encout = _linear(enc.enc_output)
        n_eo = enc.enc_output_norm
        self.enc_norm = (_f(n_eo.weight), _f(n_eo.bias), n_eo.eps)
        cls_e, box_e = enc.predictors
        self.enc_cls = _linear(cls_e.linear)
        self.enc_box = [_linear(l) for l in box_e.mlp.layers]
        self.max_ratio = float(np.float32(np.abs(np.log(box_e.transform._wh_ratio_clip))))
        enc2 = model.prompting.encoders.box_2d_encoder
        self.box_emb = tuple(_f(e.weight) for e in (enc2.x, enc2.y, enc2.w, enc2.h))
        self.box_emb_max = float(enc2.max_bounds[0])
        if not bool((enc2.max_bounds == enc2.max_bounds[0]).all()):
            raise _lib.HipError("DecoderEngine: box prompt embeddings of one size")
        # constant proposals and validity (gen_encoder_output_proposals for a mask-free memory)
        props, valid = self._proposals()
        f32 = dict(dtype=torch.float32, device=dev)
        self.PROPS = props.reshape(B * self.Pt, 4).contiguous()
        # MEM row (f, i) <- LV row (level block + f * rows + position); invalid proposals -> zero row
        amap = np.empty((B, self.Pt), np.int64)
        off = 0
        for lvl, r in enumerate(rows):
            amap[:, off:off + r] = self.lvl_off[lvl] + np.arange(B)[:, None] * r + np.arange(r)[None]
            off += r
        amap[~valid.reshape(B, self.Pt).cpu().numpy()] = -1
        self.mem_map = torch.as_tensor(amap.reshape(-1).astype(np.int32), device=dev)
        # ---- a8: decoder layers --------------------------------------------------------------
        self.layers = []
        for L, P in zip(dec.layers, dec.predictors):
            sa = L.self_attn
            wi, bi = _f(sa.in_proj_weight), _f(sa.in_proj_bias)
            xa = L.xattn
            self.layers.append(dict(
                n1=(_f(L.norm1.weight), _f(L.norm1.bias), L.norm1.eps),
                n2=(_f(L.norm2.weight), _f(L.norm2.bias), L.norm2.eps),
                n3=(_f(L.norm3.weight), _f(L.norm3.bias), L.norm3.eps),
                qk=(wi[: 2 * C].contiguous(), bi[: 2 * C].contiguous()),
                v=(wi[2 * C:].contiguous(), bi[2 * C:].contiguous()),
                out=_linear(sa.out_proj), q=_linear(xa.q), proj=_linear(xa.proj),
                ff1=_linear(L.linear1), ff2=_linear(L.linear2),
                cpb1=(_f(xa.cpb_mlp1[0].weight), _f(xa.cpb_mlp1[0].bias), _f(xa.cpb_mlp1[2].weight)),
                cpb2=(_f(xa.cpb_mlp2[0].weight), _f(xa.cpb_mlp2[0].bias), _f(xa.cpb_mlp2[2].weight)),
                xscale=float(xa.scale), pos=xa._positions(h, w, dev), preds=list(P)))
        self.dnorm = (_f(dec.norm.weight), _f(dec.norm.bias), dec.norm.eps)
        self.kv_w = (torch.cat([_f(L.xattn.k.weight) for L in dec.layers]),
                     torch.cat([_f(L.xattn.k.bias) for L in dec.layers]),
                     torch.cat([_f(L.xattn.v.weight) for L in dec.layers]),
                     torch.cat([_f(L.xattn.v.bias) for L in dec.layers]))
        self.preds = []
        for P in dec.predictors:
            d = {}
            for p in P:
                if isinstance(p, ScalePredictor):
                    d["scale"] = (torch.cat([_f(p.shift.weight), _f(p.scale.weight)]).contiguous(),
                                  torch.cat([_f(p.shift.bias), _f(p.scale.bias)]).contiguous())
                elif isinstance(p, ClassPredictor):
                    d["class"] = _linear(p.linear)
                elif isinstance(p, DeltaBox2DPredictor):
                    d["box2d"] = [_linear(l) for l in p.mlp.layers]
                elif isinstance(p, AbsoluteBox3DPredictor):
                    d["box3d"] = [_linear(l) for l in p.mlp.layers]
                else:
                    raise _lib.HipError(f"DecoderEngine: unsupported predictor {type(p).__name__}")
            if "box2d" not in d:
                raise _lib.HipError("DecoderEngine: every layer refines the 2-D boxes")
            self.preds.append(d)
        last = self.preds[-1]
        if "class" not in last or "box3d" not in last:
            raise _lib.HipError("DecoderEngine: the last layer predicts classes and 3-D boxes")
        self.query0 = torch.cat([_f(metric.query_embed.weight), _f(enc.query_embed.weight[: self.nq])]) \
            .repeat(B, 1).contiguous()
        # ---- buffers ---------------------------------------------------------------------------
        n, nq, Pt = self.n, self.nq, self.Pt
        nL = len(self.layers)
        dffn = self.layers[0]["ff1"][0].shape[0]
        z = lambda *s: torch.zeros(s, **f32)
        self.PROJ = z(B * P0, C)
        self.LV = z(B * Pt, C)
        self.SRC = self.LV[: B * P0]
        self.SRCPOS = z(B * P0, C)
        self.S2D = z(B * rows[1] if len(rows) > 1 else 1, 4 * C)
        self.LT1 = z(B * rows[1] if len(rows) > 1 else 1, C)
        self.LT2 = z(B * rows[1] if len(rows) > 1 else 1, C)
        self.MEM = z(B * Pt, C)
        self.EH1, self.EH2 = z(B * Pt, C), z(B * Pt, C)
        self.ELOG = z(B * Pt, self.enc_cls[0].shape[0])
        self.EBOX = z(B * Pt, 4)
        self.TOPI = torch.zeros((B, nq), dtype=torch.int32, device=dev)
        self.REF = z(B * nq, 4)
        self.QPOS = z(B * n, C)            # metric rows stay zero
        self.TGT = z(B * n, C)
        self.T2, self.T2P = z(B * n, C), z(B * n, C)
        self.QK, self.V, self.ATT = z(B * n, 2 * C), z(B * n, C), z(B * n, C)
        self.Q, self.XO = z(B * n, C), z(B * n, C)
        self.FF = z(B * n, dffn)
        self.Y = z(B * n, C)
        self.MH1, self.MH2 = z(B * n, C), z(B * n, C)
        self.KALL, self.VALL = z(B * P0, nL * C), z(B * P0, nL * C)
        self.RX = z(B, nq, w, self.heads)
        self.RY = z(B, nq, h, self.heads)
        self.LOGITS = z(B * nq, last["class"][0].shape[0])
        self.B3 = z(B * nq, 16)
        self.PARAMS = z(B, 2)
        k = self.topk
        self.out = dict(scores=z(B, k), classes=torch.zeros((B, k), dtype=torch.int64, device=dev),
                        logits=z(B, k, self.LOGITS.shape[1]), boxes=z(B, k, 4), proj=z(B, k, 2), b3=z(B, k, 6),
                        R=z(B, k, 3, 3), desc=z(B, k, C))
        self._wh_cache = {}

    # ---- constants -----------------------------------------------------------------------------
    def _proposals(self):
        """gen_encoder_output_proposals (:864-916) for a mask-free memory, by the same torch ops as
        EncoderProposals.proposals (constant per grid size)"""
        enc, B, dev = self.enc, self.B, self.dev
        props = []
        for lvl, (H_, W_) in enumerate(self.lvl_hw):
            stride = enc.level_strides[lvl]
            gy, gx = torch.meshgrid(torch.linspace(0, H_ - 1, H_, dtype=torch.float32, device=dev),
                                    torch.linspace(0, W_ - 1, W_, dtype=torch.float32, device=dev), indexing="ij")
            grid = (torch.cat([gx.unsqueeze(-1), gy.unsqueeze(-1)], -1)[None].expand(B, -1, -1, -1) + 0.5) * stride
            wh = torch.ones_like(grid) * enc.min_proposal_size * (2.0 ** lvl)
            props.append(torch.cat((grid, wh), -1).view(B, -1, 4))
        props = torch.cat(props, 1)
        h, w, s0 = self.h, self.w, enc.level_strides[0]
        lim = [(float(np.float32(0.01) * np.float32(v)), float(np.float32(0.99) * np.float32(v)))
               for v in (w * s0, h * s0, w * s0, h * s0)]
        valid = torch.stack([(props[..., c] > lo) & (props[..., c] < hi) for c, (lo, hi) in enumerate(lim)],
                            -1).all(-1, keepdim=True)
        props = props.masked_fill(~valid, max(h, w) * s0)
        return props, valid

    def positions(self, K_host, sizes_wh):
        """CameraRayEmbedding(K, size) + level_embed as [B*h*w, C] rows (bf_ray_fourier_f32 + the
        projection GEMM), cached per (K, size) -- it depends on nothing else"""
        K_host = np.asarray(K_host, np.float32).reshape(self.B, 3, 3)
        key = (K_host.tobytes(), tuple(tuple(s) for s in sizes_wh))
        if key not in self._pos_cache:
            if self.h != self.w:
                raise _lib.HipError("DecoderEngine: square feature grid (the reference pads to a square)")
            feat, P0, C = self.h, self.P0, self.C
            out = torch.empty((self.B * P0, C), dtype=torch.float32, device=self.dev)
            fb = torch.empty((P0, self.w_ray.shape[1]), dtype=torch.float32, device=self.dev)
            for i in range(self.B):
                W, H = sizes_wh[i]
                _lib.ray_fourier(K_host[i], int(W), int(H), feat, 16, self.ray_scales, fb)
                _lib.gemm_f32(fb, self.w_ray, self.b_ray, out=out[i * P0:(i + 1) * P0])
            out += self.level_embed          # once per camera (the decode adds it per call)
            self._pos_cache[key] = out
        return self._pos_cache[key]

    def _img_wh(self, image_sizes):
        key = tuple(tuple(s) for s in image_sizes)
        if key not in self._wh_cache:
            self._wh_cache[key] = torch.tensor([[float(w), float(h)] for h, w in image_sizes],
                                               dtype=torch.float32, device=self.dev)
        return self._wh_cache[key]

    # ---- forward -------------------------------------------------------------------------------
    @torch.no_grad()
    def __call__(self, feat_rows, pos, depth_params, K_inv, T_gravity, image_sizes, clamp_shape):
        """feat_rows f32 [B*h*w, C_backbone] (channel-last backbone features), pos [B*h*w, C]
        (positions()), depth_params [B,2] or None (RGB-only: the predicted scale tokens),
        K_inv / T_gravity [B,3,3] (T_gravity may be None), image_sizes [(h, w)], clamp_shape
        (H, W) of clamp_xy -> list of B Instances3D (views of this engine's output buffers)"""
        L = _lib
        B, C, n, nq, P0 = self.B, self.C, self.n, self.nq, self.P0
        cw, ch = float(clamp_shape[1]), float(clamp_shape[0])
        # a6: input projection + GroupNorm -> src (LV level 0) and src + pos
        L.gemm_f32(feat_rows, self.w_inproj, self.b_inproj, out=self.PROJ)
        G, gw, gb, geps = self.gn
        L.groupnorm_cl(self.PROJ, B, G, gw, gb, geps, self.SRC, pos=pos, out2=self.SRCPOS)
        # a7: proposal levels (channel-last maps, 2x2/2 convolutions on space-to-depth rows)
        for lvl in range(1, len(self.levels)):
            cur, (H_, W_) = self.SRC, (self.h, self.w)
            ops = self.levels[lvl]
            for j, op in enumerate(ops):
                if op[0] == "conv":
                    x = L.s2d(cur, B, H_, W_, out=self.S2D[: B * (H_ // 2) * (W_ // 2)])
                    H_, W_ = H_ // 2, W_ // 2
                    last = j == len(ops) - 1
                    dst = (self.LV[self.lvl_off[lvl]: self.lvl_off[lvl + 1]] if last
                           else self.LT1[: B * H_ * W_])
                    L.gemm_f32(x, op[1], op[2], out=dst)
                    cur = dst
                else:
                    dst = self.LT2[: B * H_ * W_]
                    L.ln_rows(cur, op[1], op[2], op[3], out=dst, gelu=op[4])
                    cur = dst
        L.gemm_f32(self.LV, self.w_encout, self.b_encout, out=self.MEM, a_map=self.mem_map)
        en = self.enc_norm
        L.ln_rows(self.MEM, en[0], en[1], en[2], out=self.MEM)
        # encoder predictors: class logits, 2-D boxes from the constant proposals
        rows = B * self.Pt
        L.row_heads(self.MEM, self.Pt, 0, rows, self.Pt, *self.enc_cls, "class", out=self.ELOG)
        (w1, b1), (w2, b2), (w3, b3) = self.enc_box
        L.gemm_f32(self.MEM, w1, b1, act="relu", out=self.EH1)
        L.gemm_f32(self.EH1, w2, b2, act="relu", out=self.EH2)
        L.row_heads(self.EH2, self.Pt, 0, rows, self.Pt, w3, b3, "box2d", prop=self.PROPS, boxes=self.EBOX,
                    clamp_wh=(cw, ch), max_ratio=self.max_ratio)
        L.topk_rows(self.ELOG, B, self.Pt, nq, ldv=self.ELOG.shape[1], idx=self.TOPI)
        L.prop_select(self.EBOX, B, self.Pt, nq, self.TOPI, self.REF, self.box_emb, self.box_emb_max,
                      self.QPOS, n, self.nm)
        self.TGT.copy_(self.query0)
        # memory k / v projections of every layer: one GEMM each
        L.gemm_f32(self.SRCPOS, self.kv_w[0], self.kv_w[1], out=self.KALL)
        L.gemm_f32(self.SRC, self.kv_w[2], self.kv_w[3], out=self.VALL)
        # a8: decoder layers
        params = depth_params
        nL = len(self.layers)
        for lid, ly in enumerate(self.layers):
            # self-attention block
            L.ln_rows(self.TGT, *ly["n2"], out=self.T2, pos=self.QPOS, out2=self.T2P)
            L.gemm_f32(self.T2P, *ly["qk"], out=self.QK)
            L.gemm_f32(self.T2, *ly["v"], out=self.V)
            L.self_attn(self.QK[:, :C], self.QK[:, C:], self.V, self.ATT, B, self.heads, n, self.nm,
                        (C // self.heads) ** -0.5)
            L.gemm_f32(self.ATT, *ly["out"], resid=self.TGT, out=self.TGT)
            # global cross-attention with the relative position bias of the current boxes
            L.ln_rows(self.TGT, *ly["n1"], out=self.T2, pos=self.QPOS, out2=self.T2P)
            L.gemm_f32(self.T2P, *ly["q"], out=self.Q)
            ref = self.REF.view(B, nq, 4)
            px, py = ly["pos"]
            L.cpb_mlp_into(ref, px, 0, *ly["cpb1"], self.RX)
            L.cpb_mlp_into(ref, py, 1, *ly["cpb2"], self.RY)
            kl = self.KALL.view(B, P0, nL * C)[:, :, lid * C:(lid + 1) * C]
            vl = self.VALL.view(B, P0, nL * C)[:, :, lid * C:(lid + 1) * C]
            L.xattn(self.Q.view(B, n, C), kl, vl, self.RX, self.RY, self.h, self.w, self.nm, self.heads,
                    ly["xscale"], out=self.XO.view(B, n, C))
            L.gemm_f32(self.XO, *ly["proj"], resid=self.TGT, out=self.TGT)
            # FFN
            L.ln_rows(self.TGT, *ly["n3"], out=self.T2)
            L.gemm_f32(self.T2, *ly["ff1"], act="relu", out=self.FF)
            L.gemm_f32(self.FF, *ly["ff2"], resid=self.TGT, out=self.TGT)
            L.ln_rows(self.TGT, *self.dnorm, out=self.Y)
            # predictors (before the last layer only the refined 2-D boxes are read)
            pr = self.preds[lid]
            last = lid == nL - 1
            if last and "scale" in pr:
                L.row_heads(self.Y, n, 0, B * n, n, *pr["scale"], "scale", out=self.PARAMS)
            if last:
                L.row_heads(self.Y, n, self.nm, B * nq, nq, *pr["class"], "class", out=self.LOGITS)
            (w1, b1), (w2, b2), (w3, b3) = pr["box2d"]
            L.gemm_f32(self.Y, w1, b1, act="relu", out=self.MH1)
            L.gemm_f32(self.MH1, w2, b2, act="relu", out=self.MH2)
            L.row_heads(self.MH2, n, self.nm, B * nq, nq, w3, b3, "box2d", prop=self.REF, boxes=self.REF,
                        clamp_wh=(cw, ch), max_ratio=self.max_ratio)
            if last:
                if params is None:
                    params = self.PARAMS
                (w1, b1), (w2, b2), (w3, b3) = pr["box3d"]
                L.gemm_f32(self.Y, w1, b1, act="relu", out=self.MH1)
                L.gemm_f32(self.MH1, w2, b2, act="relu", out=self.MH2)
                L.row_heads(self.MH2, n, self.nm, B * nq, nq, w3, b3, "box3d", out=self.B3, prop=self.REF,
                            params=params.contiguous(), clamp_wh=(cw, ch))
        # a9: inference_single_image
        o = self.out
        L.infer_select(self.LOGITS, B, nq, self.LOGITS.shape[1], self.REF, self.B3, self.Y, n, self.nm,
                       K_inv.contiguous(), None if T_gravity is None else T_gravity.contiguous(),
                       self._img_wh(image_sizes), self.topk, o)
        res = []
        for i in range(B):
            r = Instances3D(tuple(image_sizes[i]))
            r.scores = o["scores"][i]
            r.pred_classes = o["classes"][i]
            r.pred_boxes = o["boxes"][i]
            r.pred_logits = o["logits"][i]
            r.pred_boxes_3d = GeneralInstance3DBoxes(o["b3"][i], o["R"][i])
            r.object_desc = o["desc"][i]
            r.pred_proj_xy = o["proj"][i]
            res.append(r)
        return res
