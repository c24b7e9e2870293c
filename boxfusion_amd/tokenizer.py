"""CLIP byte-level BPE tokenizer (open_clip `SimpleTokenizer`, the `tokenizer(text_class)` of
precompute_class_features.py:24,31), restated from open_clip's published algorithm:

* byte -> printable-unicode table (`bytes_to_unicode`), words split by the CLIP regex
  (`<|startoftext|>`, `<|endoftext|>`, contractions, letter runs, single digits, punctuation runs),
  text lower-cased after HTML unescaping and whitespace collapsing;
* each word's bytes mapped through the table, the last symbol suffixed with `</w>`, then pairs
  merged greedily by merge rank;
* vocabulary = 256 byte symbols + their `</w>` forms + one entry per merge + the two specials;
  a prompt becomes [<start_of_text>] + tokens + [<end_of_text>], truncated to the context length
  (the last id forced to <end_of_text>) and zero padded.

The merges file (open_clip's `bpe_simple_vocab_16e6.txt.gz`) is not available offline, so it is a
constructor argument; `ftfy.fix_text` (also absent) is not applied — plain ASCII class names such
as the reference's category lists are unaffected.  Parity UNPINNED (no open_clip here).
"""
from __future__ import annotations

import gzip
import html
from functools import lru_cache

import numpy as np
import regex as re

SOT, EOT = "<start_of_text>", "<end_of_text>"


@lru_cache()
def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def _pairs(word):
    return set(zip(word[:-1], word[1:]))


def _clean(text):
    text = html.unescape(html.unescape(text)).strip()
    return re.sub(r"\s+", " ", text).strip()


class SimpleTokenizer:
    # open_clip builds the pattern from its own special tokens (SOT / EOT above), so a special
    # inside the text is one token
    PAT = re.compile("|".join(re.escape(t) for t in (SOT, EOT)) +
                     r"""|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""", re.IGNORECASE)

    def __init__(self, merges, n_merges=49152 - 256 - 2):
        """merges: path of a BPE merges file (.txt or .txt.gz; first line is a header), or a list
        of (a, b) pairs in rank order"""
        if isinstance(merges, str):
            opener = gzip.open if merges.endswith(".gz") else open
            with opener(merges, "rt", encoding="utf-8") as f:
                lines = f.read().split("\n")
            merges = [tuple(m.split()) for m in lines[1:n_merges + 1] if m.strip()]
        merges = [tuple(m) for m in merges]
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab]
        vocab += ["".join(m) for m in merges]
        vocab += [SOT, EOT]
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {SOT: SOT, EOT: EOT}
        self.sot_token_id, self.eot_token_id = self.encoder[SOT], self.encoder[EOT]
        self.vocab_size = len(self.encoder)

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        pairs = _pairs(word)
        if not pairs:
            return token + "</w>"
        while True:
            bigram = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if bigram not in self.bpe_ranks:
                break
            first, second = bigram
            new, i = [], 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    new.extend(word[i:])
                    break
                new.extend(word[i:j])
                i = j
                if word[i] == first and i < len(word) - 1 and word[i + 1] == second:
                    new.append(first + second)
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        out = " ".join(word)
        self.cache[token] = out
        return out

    def encode(self, text):
        ids = []
        for tok in re.findall(self.PAT, _clean(text).lower()):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(tok).split(" "))
        return ids

    def decode(self, ids):
        text = "".join(self.decoder[i] for i in ids)
        return bytearray([self.byte_decoder[c] for c in text]).decode("utf-8", errors="replace") \
            .replace("</w>", " ")

    def __call__(self, texts, context_length=77):
        """list of str (or one str) -> int64 [len, context_length] token ids"""
        if isinstance(texts, str):
            texts = [texts]
        out = np.zeros((len(texts), context_length), dtype=np.int64)
        for i, t in enumerate(texts):
            toks = [self.sot_token_id] + self.encode(t) + [self.eot_token_id]
            if len(toks) > context_length:
                toks = toks[:context_length]
                toks[-1] = self.eot_token_id
            out[i, :len(toks)] = toks
        return out
