"""Seeded synthetic weights keyed by parameter name.

No CuTR / CLIP checkpoint is available offline, so parity and throughput runs use weights drawn
from PCG64(seed ^ crc32(name)) — the same rule the golden generator applies to the reference model,
so both sides hold identical parameters without shipping a weight file.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def canonical(name: str) -> str:
    # the reference registers the shared prompt encoders under every prompter as well
    if ".encoders." in name and name.startswith("prompting.prompters."):
        return "prompting.encoders." + name.split(".encoders.", 1)[1]
    return name


def value_for(name, shape, seed=0, std=0.02):
    key = canonical(name)
    rng = np.random.default_rng(np.random.PCG64(seed ^ zlib.crc32(key.encode())))
    leaf = key.rsplit(".", 1)[-1]
    if key.endswith("min_bounds") or key.endswith("max_bounds"):
        return None
    if leaf == "weight" and len(shape) == 1 and ("norm" in key or ".ln" in key or "input_proj.0.1" in key
                                                 or key.endswith("ln_pre.weight") or key.endswith("ln_post.weight")):
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    return (std * rng.standard_normal(shape)).astype(np.float32)


UNIFORM_QUERY_KEY = "prompting.prompters.1.query_embed.weight"


def seeded_state_dict(model: torch.nn.Module, seed=0, std=0.02, uniform_queries=False):
    """uniform_queries: every row of the encoder-proposal content embedding (EncoderProposals.
    query_embed, cubify_transformer.py:759,830) set to row 0.  The decoder is then equivariant to
    the order of its 300 proposal queries (self-attention without a mask, per-query cross-
    attention and heads), so near-tied encoder logits that bf16 rounding reorders no longer swap
    which content row a proposal gets: the end-to-end instances become comparable one by one."""
    sd = model.state_dict()
    out = {}
    for k, v in sd.items():
        val = value_for(k, tuple(v.shape), seed, std)
        out[k] = v.clone() if val is None else torch.from_numpy(val).to(v.dtype)
    if uniform_queries:
        q = out[UNIFORM_QUERY_KEY]
        out[UNIFORM_QUERY_KEY] = q[:1].expand_as(q).clone()
    return out


def init_seeded(model: torch.nn.Module, seed=0, std=0.02, uniform_queries=False):
    model.load_state_dict(seeded_state_dict(model, seed, std, uniform_queries))
    return model
