"""CLIP BPE tokenizer (tokenizer.SimpleTokenizer, open_clip's algorithm restated) on a small merges
table: byte-level round trip, merge order, the <start_of_text> / <end_of_text> frame, truncation to
the context length, and the property the text tower's pooling relies on (the EOT id is the
largest id, so argmax(ids) is the EOT position).  Parity with open_clip UNPINNED (absent offline)."""
import numpy as np

from boxfusion_amd.tokenizer import SimpleTokenizer, bytes_to_unicode

MERGES = [("c", "h"), ("a", "i"), ("ai", "r</w>"), ("ch", "air</w>"), ("t", "a"), ("b", "l"), ("bl", "e</w>"),
          ("ta", "ble</w>"), ("s", "o"), ("so", "f"), ("sof", "a</w>")]


def test_bytes_to_unicode_is_a_bijection():
    m = bytes_to_unicode()
    assert len(m) == 256 and len(set(m.values())) == 256
    assert m[ord("a")] == "a" and m[ord(" ")] != " "


def test_bpe_merges_and_ids():
    tok = SimpleTokenizer(MERGES)
    assert tok.vocab_size == 512 + len(MERGES) + 2
    assert tok.bpe("chair") == "chair</w>"
    assert tok.bpe("table") == "table</w>"
    assert tok.bpe("tables") == "ta bl e s</w>"
    ids = tok.encode("Chair  table")
    assert [tok.decoder[i] for i in ids] == ["chair</w>", "table</w>"]
    assert tok.decode(ids) == "chair table "


def test_round_trip_unicode_and_punctuation():
    tok = SimpleTokenizer(MERGES)
    for text in ["sofa, chair & table!", "kitchen cabinet 2", "café  lamp", "it's a tv"]:
        ids = tok.encode(text)
        assert tok.decode(ids).split() == " ".join(text.lower().split()).replace(",", " ,") \
            .replace("!", " !").replace("&", "&").replace("2", "2").replace("'s", " 's").split()


def test_context_frame_truncation_and_eot_argmax():
    tok = SimpleTokenizer(MERGES)
    ids = tok(["chair", "table " * 100, ""], context_length=77)
    assert ids.shape == (3, 77) and ids.dtype == np.int64
    assert ids[0, 0] == tok.sot_token_id and ids[0, 2] == tok.eot_token_id and ids[0, 3:].sum() == 0
    assert ids[1, -1] == tok.eot_token_id and (ids[1] > 0).all()
    assert ids[2, 1] == tok.eot_token_id
    # the EOT id is the largest in the vocabulary: argmax pooling lands on it
    assert tok.eot_token_id == tok.vocab_size - 1
    for row in ids:
        assert row[row.argmax()] == tok.eot_token_id


def test_merges_file(tmp_path):
    import gzip
    p = tmp_path / "merges.txt.gz"
    with gzip.open(p, "wt", encoding="utf-8") as f:
        f.write("#version: 0.2\n" + "\n".join(" ".join(m) for m in MERGES) + "\n")
    a, b = SimpleTokenizer(str(p)), SimpleTokenizer(MERGES)
    assert a.encoder == b.encoder
    assert (a(["sofa chair"]) == b(["sofa chair"])).all()


def test_load_text_tower_from_open_clip_style_checkpoint(tmp_path):
    """precompute_class_features.load_text_tower: text entries of a checkpoint with a "module."
    prefix, a "state_dict" wrapper and unrelated visual.* entries load into the TextTransformer
    (open_clip parameter names); a checkpoint without them is rejected"""
    import torch
    from boxfusion_amd.clip import TextTransformer
    from boxfusion_amd.precompute_class_features import load_text_tower
    torch.manual_seed(0)
    src = TextTransformer(77, 300, 64, 2, 2, 32)
    sd = {"module." + k: v for k, v in src.state_dict().items()}
    sd["module.visual.proj"] = torch.zeros(3)
    torch.save({"state_dict": sd}, tmp_path / "ckpt.pt")
    dst = load_text_tower(str(tmp_path / "ckpt.pt"), device="cpu", text=TextTransformer(77, 300, 64, 2, 2, 32))
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v), k
    torch.save({"visual.proj": torch.zeros(3)}, tmp_path / "bad.pt")
    import pytest
    with pytest.raises(KeyError):
        load_text_tower(str(tmp_path / "bad.pt"), device="cpu", text=TextTransformer(77, 300, 64, 2, 2, 32))


def test_special_tokens_in_text_are_single_tokens():
    """the split pattern is built from the vocabulary's own SOT / EOT strings (as open_clip builds
    it from its special tokens), so a special inside the text encodes to its one id"""
    from boxfusion_amd.tokenizer import EOT, SOT, SimpleTokenizer
    t = SimpleTokenizer([("a", "b")])
    ids = t.encode(f"x {SOT} y {EOT}")
    assert t.encoder[SOT] in ids and t.encoder[EOT] in ids
    assert t.encode("<|startoftext|>") != [t.encoder[SOT]]
