"""Vocabulary builder: class names -> normalised CLIP text features (the reference's
boxfusion/precompute_class_features.py:11-45, same arguments and output format).

    python -m boxfusion_amd.precompute_class_features --clip_path open_clip_pytorch_model.bin \
        --class_txt data/scannet200.txt --class_features data/scannet200_features.pt \
        --bpe bpe_simple_vocab_16e6.txt.gz

Reads one class name per line (`np.genfromtxt(..., delimiter='\\n', dtype=str)`, line 26),
tokenizes them (open_clip ViT-H-14 tokenizer, `tokenizer.SimpleTokenizer`), runs the text tower on
the GPU (`text_engine.CLIPTextEngine`), L2-normalises (line 43) and `torch.save`s the [V, 1024]
f32 table (line 45) — the `text_features` argument of `tools.utils.text_prompt`.  The checkpoint is
loaded with `torch.load(weights_only=True)`; its text-tower entries use open_clip's names.
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from boxfusion_amd.clip import text_h14
from boxfusion_amd.text_engine import CLIPTextEngine
from boxfusion_amd.tokenizer import SimpleTokenizer

TEXT_KEYS = ("token_embedding.", "positional_embedding", "transformer.", "ln_final.", "text_projection")


def load_text_tower(path, device="cuda", text=None):
    """the text-tower entries of an open_clip checkpoint (optionally under "state_dict" / with a
    "module." prefix; the visual.* entries are ignored) loaded into `text` (default ViT-H-14)"""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if "state_dict" in sd:
        sd = sd["state_dict"]
    sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    text = text_h14() if text is None else text
    missing, _ = text.load_state_dict({k: v for k, v in sd.items() if k.startswith(TEXT_KEYS)},
                                      strict=False)
    if missing:
        raise KeyError(f"checkpoint lacks text-tower entries: {missing[:5]} ...")
    return text.to(device)


def build_class_features(class_names, text, tokenizer, max_prompts=256, device="cuda"):
    ids = torch.from_numpy(tokenizer(list(class_names), context_length=text.context_length))
    eng = CLIPTextEngine(text, max_prompts=min(max_prompts, max(len(ids), 1)), device=device)
    return eng.class_features(ids)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clip_path", default="./models/open_clip_pytorch_model.bin", type=str)
    ap.add_argument("--class_txt", default="./data/cubicle_classes.txt", type=str)
    ap.add_argument("--class_features", default="./data/cubicle_class_features.pt", type=str)
    ap.add_argument("--bpe", default="./models/bpe_simple_vocab_16e6.txt.gz", type=str)
    args = ap.parse_args(argv)
    with torch.no_grad():
        text_class = np.atleast_1d(np.genfromtxt(args.class_txt, delimiter="\n", dtype=str))
        text = load_text_tower(args.clip_path)
        feats = build_class_features(text_class, text, SimpleTokenizer(args.bpe))
        torch.save(feats.cpu(), args.class_features)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
