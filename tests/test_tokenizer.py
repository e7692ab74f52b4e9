"""CPU tier: the CLIP byte-level BPE tokenizer (federated_multi_modal_amd/tokenizer.py) against the reference's
own SimpleTokenizer / clip.tokenize (clip/simple_tokenizer.py:62-127, clip/clip.py:185-221).

tests/golden/bpe_ids.json was written by tests/golden/make_golden.py (target `bpe`), which loads the
reference's simple_tokenizer.py and clip.py by file path (ftfy stubbed as identity: absent here) and
tokenizes 27 texts -- class names, captions with punctuation, digits, contractions, HTML entities, accented
Latin, CJK / Cyrillic / Greek, emoji, the special tokens inside text, repeated letters -- over
tests/golden/bpe_small_merges.txt.gz (a CLIP-format merges file learned by make_bpe_merges.py; CLIP's
own bpe_simple_vocab_16e6.txt.gz is not in this image).  Text that ftfy.fix_text would repair is "parity
unpinned" (no fixture holds ftfy's output).

Also: the CLIP checkpoint reader (clip_archive.py) that reads TorchScript archives without executing them."""
import gzip
import io
import json
import pickle
import zipfile
from pathlib import Path

import numpy as np
import pytest
import torch

from federated_multi_modal_amd import tokenizer as T

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def fx():
    return json.loads((GOLD / "bpe_ids.json").read_text())


@pytest.fixture(scope="module")
def tok(fx):
    return T.SimpleTokenizer(str(GOLD / fx["merges"]))


def test_vocabulary_layout_matches_reference(fx, tok):
    assert (tok.sot, tok.eot, tok.vocab_size) == (fx["sot"], fx["eot"], fx["vocab_size"])
    assert len(T.byte_alphabet()) == 256 and len(set(T.byte_alphabet().values())) == 256


def test_encode_ids_bit_exact(fx, tok):
    for text, ids in fx["encode"]:
        assert tok.encode(text) == ids, text


def test_tokenize_bit_exact(fx, tok):
    for text, ids in fx["tokenize"]:
        got = tok.tokenize(text)
        assert got.shape == (1, 77) and got.dtype == np.int64
        assert got[0].tolist() == ids, text
    text, ids = fx["context_16"]
    assert tok.tokenize(text, context_length=16)[0].tolist() == ids


def test_overflow_and_truncate(fx, tok):
    text, ids = fx["truncate"]
    assert fx["overflow_raises"]
    with pytest.raises(RuntimeError) as err:
        tok.tokenize(text)
    assert str(err.value) == fx["overflow_message"]
    assert tok.tokenize(text, truncate=True)[0].tolist() == ids
    assert tok.tokenize(text, truncate=True)[0, -1] == tok.eot


def test_merge_strings(fx, tok):
    for w, s in fx["bpe"].items():
        assert tok.bpe("".join(tok.byte_encoder[b] for b in w.encode("utf-8"))) == s, w


def test_decode_round_trip(fx, tok):
    for text, ids in fx["encode"]:
        dec = tok.decode(ids)
        assert dec.replace(" ", "") == T.clean(text).replace(" ", ""), text


def test_full_size_merges_file(tmp_path):
    """CLIP's file: only the first 49152 - 256 - 2 merges count (a longer file is cut), giving 49408 ids with
    <|startoftext|> = 49406 and <|endoftext|> = 49407 -- the ids the 49408-row token embedding expects."""
    syms = list(T.byte_alphabet().values())
    lines = ["#version: 0.2"] + [f"{a} {b}" for a in syms for b in syms][:T.N_MERGES + 500]
    p = tmp_path / T.BPE_FILE
    with gzip.open(p, "wb") as f:
        f.write(("\n".join(lines) + "\n").encode("utf-8"))
    t = T.SimpleTokenizer(str(p))
    assert t.vocab_size == 49408 and (t.sot, t.eot) == (49406, 49407)
    ids = t.tokenize(["a photo of a forest.", "zzz"])
    assert ids.max() == 49407 and (ids.argmax(-1) > 0).all()


def test_synthetic_fallback_and_resolution(tmp_path, monkeypatch):
    monkeypatch.delenv("MAPFED_BPE_PATH", raising=False)
    monkeypatch.setenv("HOME", str(tmp_path))
    assert T.resolve_bpe_path("", str(tmp_path / "ViT-B-16.pt")) == ""
    syn_tok = T.get_tokenizer("")
    assert syn_tok.kind == "synthetic" and "synthetic" in T.describe(syn_tok)
    (tmp_path / "ckpt").mkdir()
    beside = tmp_path / "ckpt" / T.BPE_FILE
    beside.write_bytes((GOLD / "bpe_small_merges.txt.gz").read_bytes())
    assert T.resolve_bpe_path("", str(tmp_path / "ckpt" / "ViT-B-16.pt")) == str(beside)
    cache = tmp_path / ".cache" / "clip"
    cache.mkdir(parents=True)
    (cache / T.BPE_FILE).write_bytes(beside.read_bytes())
    assert T.resolve_bpe_path("", "") == str(cache / T.BPE_FILE)
    monkeypatch.setenv("MAPFED_BPE_PATH", str(beside))
    assert T.resolve_bpe_path("", "") == str(beside)
    with pytest.raises(FileNotFoundError):
        T.resolve_bpe_path(str(tmp_path / "missing.gz"))
    assert T.get_tokenizer(str(beside)).kind == "bpe"


def test_prompt_prefix_and_class_prompts():
    """trainers/maple.py:96-106, 136-140: CTX_INIT ("_" -> " ") gives the prefix and the ctx token ids; no
    CTX_INIT (or n_ctx > 4) gives "X X" and no ids; class names "_" -> " " with a trailing "."."""
    from federated_multi_modal_amd.engine import EngineConfig, class_prompts, prompt_prefix
    bpe = str(GOLD / "bpe_small_merges.txt.gz")
    cfg = EngineConfig(batch=1, classnames=["dense_residential", "sea_or_lake"], ctx_init="a_photo of", bpe_path=bpe)
    prefix, ids = prompt_prefix(cfg)
    t = T.get_tokenizer(bpe)
    assert prefix == "a photo of" and ids.tolist() == t.encode("a photo")
    assert class_prompts(cfg) == ["a photo of dense residential.", "a photo of sea or lake."]
    cfg2 = EngineConfig(batch=1, classnames=["x"], ctx_init="")
    assert prompt_prefix(cfg2) == ("X X", None) and class_prompts(cfg2) == ["X X x."]


def test_caption_tokens_of_reference_case():
    """The BPE caption fixture's token ids (the reference's clip.tokenize) from captions.caption_tokens."""
    from federated_multi_modal_amd.captions import caption_tokens
    c = dict(np.load(GOLD / "case_cap_bpe_j3_b4.npz"))
    t = T.get_tokenizer(str(GOLD / str(c["bpe"])))
    assert np.array_equal(caption_tokens([str(x) for x in c["captions"]], tokenizer=t), c["caption_tokens"])


# --------------------------------------------------------------------------- CLIP checkpoint reader

class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(3, 2).half()
        self.ln = torch.nn.LayerNorm(2)
        self.seq = torch.nn.Sequential(torch.nn.Linear(2, 2), torch.nn.Linear(2, 4))
        self.register_buffer("buf", torch.arange(3.0))
        self.p = torch.nn.Parameter(torch.randn(2, 5)[:, 1:4])  # a non-contiguous storage view

    def forward(self, x):
        return self.seq(self.ln(self.lin(x.half()).float())).sum() + self.buf.sum() + self.p.sum()


def test_torchscript_archive_read_without_running_it(tmp_path):
    from federated_multi_modal_amd import clip_archive as A
    m = _Tiny()
    path = tmp_path / "ts.pt"
    torch.jit.save(torch.jit.trace(m, torch.randn(1, 3)), str(path))
    assert A.is_torchscript_archive(str(path))
    sd = A.load_clip_state_dict(str(path))
    ref = m.state_dict()
    assert sorted(sd) == sorted(ref)
    for k, v in ref.items():
        assert sd[k].dtype == v.dtype and torch.equal(sd[k], v), k
    plain = tmp_path / "plain.pt"
    torch.save({"state_dict": ref}, str(plain))
    assert not A.is_torchscript_archive(str(plain))
    assert sorted(A.load_clip_state_dict(str(plain))) == sorted(ref)


def test_torchscript_archive_refuses_other_globals(tmp_path):
    """Only the constructs a module tree uses are allowed: any other global in data.pkl is refused."""
    from federated_multi_modal_amd import clip_archive as A

    class Evil:
        def __reduce__(self):
            return (print, ("should not run",))
    path = tmp_path / "evil.pt"
    with zipfile.ZipFile(path, "w") as zf:
        zf.writestr("arch/data.pkl", pickle.dumps({"x": Evil()}, protocol=2))
        zf.writestr("arch/code/__torch__.py", "")
    with pytest.raises(pickle.UnpicklingError):
        A.load_clip_state_dict(str(path))
    corrupt = tmp_path / "corrupt.pt"
    corrupt.write_bytes(b"not a checkpoint")
    with pytest.raises(Exception) as err:
        A.load_clip_state_dict(str(corrupt))
    assert not isinstance(err.value, pickle.UnpicklingError) or "weights" in str(err.value).lower()
