"""CLIP's byte-level BPE tokenizer and clip.tokenize, for the prompt and caption token ids.

Reference: clip/simple_tokenizer.py:15-127 (bytes_to_unicode, get_pairs, basic_clean,
whitespace_clean, SimpleTokenizer.bpe/encode/decode) and clip/clip.py:185-221 (tokenize: SOT + ids +
EOT, zero padding to the context length, RuntimeError on overflow unless truncate).  Call sites on
the path: the ctx init and class prompts (trainers/maple.py:96-103, 136-143), the class-name lengths
(:137) and the batch captions (:309).

The merges file is the one CLIP ships beside its tokenizer, `bpe_simple_vocab_16e6.txt.gz`.  It is
not in this image (no network); `resolve_bpe_path` looks for it where a user of the reference keeps
it, and `get_tokenizer("")` falls back to the seeded synthetic word-id tokenizer (synthetic.py) when
there is none -- the trainer logs which one is active.

Text cleaning: the reference runs ftfy.fix_text, then html.unescape twice, then collapses white space
and lower-cases.  ftfy is used when importable; it is absent here, and the fallback applies the
subset of its default fixes that changes well-formed text (NFC normalisation, curly quotes to ASCII,
Latin ligatures and full-width forms unfolded, line-break normalisation).  The ids are pinned bit for
bit to the reference's own SimpleTokenizer on ASCII and on Unicode inputs that none of those fixes
touch (tests/golden/bpe_ids.json); text that ftfy would repair (mojibake, control characters) is
"parity unpinned".
"""
from __future__ import annotations

import gzip
import html
import os
import os.path as osp
import unicodedata
from functools import lru_cache
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

try:
    import regex as _re
except ImportError as exc:  # pragma: no cover - regex is in the image
    raise ImportError("the BPE tokenizer needs the `regex` module (\\p{L} / \\p{N} classes)") from exc

BPE_FILE = "bpe_simple_vocab_16e6.txt.gz"
SOT, EOT = "<|startoftext|>", "<|endoftext|>"
# CLIP keeps the first 49152 - 256 - 2 merges (the vocab is 256 bytes x 2 + merges + 2 specials = 49408)
N_MERGES = 49152 - 256 - 2

# pre-split: the special tokens, English contractions, letter runs, single digits, other symbol runs
_SPLIT = _re.compile(r"<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+",
                     _re.IGNORECASE)
_WS = _re.compile(r"\s+")


@lru_cache()
def byte_alphabet() -> Dict[int, str]:
    """bytes_to_unicode (clip/simple_tokenizer.py:15-35): the 188 printable Latin-1 bytes map to
    themselves, the other 68 to the code points 256, 257, ... in byte order."""
    keep = [b for b in range(256) if 0x21 <= b <= 0x7E or 0xA1 <= b <= 0xAC or 0xAE <= b <= 0xFF]
    moved = [b for b in range(256) if b not in set(keep)]
    # insertion order = vocabulary order: the kept bytes ascending, then the remapped ones
    table = {b: chr(b) for b in keep}
    table.update({b: chr(256 + n) for n, b in enumerate(moved)})
    return table


# ftfy's uncurl_quotes (U+02BC and U+2018..U+201B -> ', U+201C..U+201F -> ") and fix_latin_ligatures
_FOLD = {"\u02bc": "'", **{chr(c): "'" for c in range(0x2018, 0x201C)},
         **{chr(c): '"' for c in range(0x201C, 0x2020)},
         "\ufb00": "ff", "\ufb01": "fi", "\ufb02": "fl", "\ufb03": "ffi", "\ufb04": "ffl", "\ufb05": "st",
         "\ufb06": "st", "\u0132": "IJ", "\u0133": "ij", "\u01c7": "LJ", "\u01c8": "Lj", "\u01c9": "lj",
         "\u01ca": "NJ", "\u01cb": "Nj", "\u01cc": "nj"}


def _fix_text_fallback(text: str) -> str:
    """The part of ftfy.fix_text's default pipeline that rewrites well-formed Unicode (see module doc):
    quotes and ligatures folded, full-width forms and the ideographic space NFKC-unfolded
    (fix_character_width), then NFC.  Line-break fixes are left out: whitespace_clean collapses every
    white-space run afterwards anyway."""
    text = "".join(_FOLD.get(ch, ch) for ch in text)
    text = "".join(unicodedata.normalize("NFKC", ch) if 0xFF01 <= ord(ch) <= 0xFF5E or ch == "\u3000" else ch
                   for ch in text)
    return unicodedata.normalize("NFC", text)


try:  # pragma: no cover - not installed in this image
    import ftfy as _ftfy
    _fix_text = _ftfy.fix_text
    _HAVE_FTFY = True
except ImportError:
    _fix_text = _fix_text_fallback
    _HAVE_FTFY = False


def clean(text: str) -> str:
    """basic_clean + whitespace_clean + lower() (clip/simple_tokenizer.py:50-59, 123)."""
    text = html.unescape(html.unescape(_fix_text(text))).strip()
    return _WS.sub(" ", text).strip().lower()


def read_merges(path: str) -> List[Tuple[str, ...]]:
    """The ranked merge list: lines 1 .. N_MERGES of the gzip'd file (line 0 is a version header),
    each split on white space, exactly as the reference slices and splits them."""
    with gzip.open(path, "rb") as f:
        lines = f.read().decode("utf-8").split("\n")
    return [tuple(line.split()) for line in lines[1:N_MERGES + 1]]


class SimpleTokenizer:
    """CLIP's byte-level BPE over a ranked merge list.

    Vocabulary order (the ids): the 256 byte symbols, the same with the end-of-word marker `</w>`, one
    entry per merge in rank order, then <|startoftext|> and <|endoftext|> -- 49408 ids for CLIP's file."""

    kind = "bpe"

    def __init__(self, bpe_path: str):
        if not osp.isfile(bpe_path):
            raise FileNotFoundError(f"BPE merges file {bpe_path} not found")
        self.path = bpe_path
        self.byte_encoder = byte_alphabet()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        merges = read_merges(bpe_path)
        symbols = list(self.byte_encoder.values())
        vocab = symbols + [s + "</w>" for s in symbols] + ["".join(m) for m in merges] + [SOT, EOT]
        self.encoder: Dict[str, int] = {}
        for i, v in enumerate(vocab):  # a repeated string keeps its last id, as dict(zip(...)) does
            self.encoder[v] = i
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.ranks: Dict[Tuple[str, ...], int] = {}
        for r, m in enumerate(merges):
            self.ranks[m] = r
        self.sot, self.eot = self.encoder[SOT], self.encoder[EOT]
        self.vocab_size = len(vocab)
        self._cache: Dict[str, Tuple[str, ...]] = {SOT: (SOT,), EOT: (EOT,)}

    def bpe_symbols(self, token: str) -> Tuple[str, ...]:
        """Merge the characters of one pre-split token (its last one carrying `</w>`): repeatedly take
        the adjacent pair of lowest rank present and join every left-to-right, non-overlapping
        occurrence of it, until no ranked pair is left (clip/simple_tokenizer.py:80-119)."""
        hit = self._cache.get(token)
        if hit is not None:
            return hit
        syms = list(token[:-1]) + [token[-1] + "</w>"]
        ranks = self.ranks
        while len(syms) > 1:
            best, best_rank = None, None
            for a, b in zip(syms, syms[1:]):
                r = ranks.get((a, b))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = (a, b), r
            if best is None:
                break
            a, b = best
            out, i, n = [], 0, len(syms)
            while i < n:
                if i + 1 < n and syms[i] == a and syms[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(syms[i])
                    i += 1
            syms = out
        res = tuple(syms)
        self._cache[token] = res
        return res

    def bpe(self, token: str) -> str:
        """The reference's string form: merged symbols joined by spaces."""
        return " ".join(self.bpe_symbols(token))

    def encode(self, text: str) -> List[int]:
        """clip/simple_tokenizer.py:121-127."""
        ids: List[int] = []
        enc = self.byte_encoder
        for piece in _SPLIT.findall(clean(text)):
            mapped = "".join(enc[b] for b in piece.encode("utf-8"))
            ids.extend(self.encoder[s] for s in self.bpe_symbols(mapped))
        return ids

    def decode(self, ids: Sequence[int]) -> str:
        """clip/simple_tokenizer.py:129-132."""
        text = "".join(self.decoder[int(i)] for i in ids)
        return bytearray(self.byte_decoder[c] for c in text).decode("utf-8", errors="replace").replace("</w>", " ")

    def tokenize(self, texts: Union[str, Sequence[str]], context_length: int = 77, truncate: bool = False) -> np.ndarray:
        return _tokenize(self, texts, context_length, truncate)


class SyntheticTokenizer:
    """The seeded word-id stand-in (synthetic.py) behind the same interface: used when no merges file
    exists.  Its ids are NOT CLIP's; the golden fixtures that pin the model path were made with it."""

    kind = "synthetic"
    path = ""

    def __init__(self):
        from . import synthetic as syn
        self._syn = syn
        self.sot, self.eot = syn.SOT_TOKEN, syn.EOT_TOKEN
        self.vocab_size = syn.VOCAB_SIZE

    def encode(self, text: str) -> List[int]:
        return self._syn.encode(text)

    def tokenize(self, texts: Union[str, Sequence[str]], context_length: int = 77, truncate: bool = False) -> np.ndarray:
        return _tokenize(self, texts, context_length, truncate)


def _tokenize(tok, texts, context_length: int, truncate: bool) -> np.ndarray:
    """clip.tokenize (clip/clip.py:185-221): [SOT] + encode(text) + [EOT] per text, zero padded to
    context_length; longer -> RuntimeError, or with truncate the first context_length ids with the last
    one replaced by EOT.  int64 [n, context_length]."""
    if isinstance(texts, str):
        texts = [texts]
    out = np.zeros((len(texts), context_length), dtype=np.int64)
    for i, t in enumerate(texts):
        ids = [tok.sot] + tok.encode(t) + [tok.eot]
        if len(ids) > context_length:
            if not truncate:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            ids = ids[:context_length]
            ids[-1] = tok.eot
        out[i, :len(ids)] = ids
    return out


def resolve_bpe_path(explicit: str = "", backbone: str = "") -> str:
    """Where a user of the reference keeps CLIP's merges file, first hit wins: an explicit path
    (MODEL.BACKBONE.BPE_PATH or $MAPFED_BPE_PATH), beside the CLIP checkpoint, the clip package's own
    directory layout (clip/simple_tokenizer.py:10-12: next to the tokenizer module, i.e. this package),
    ~/.cache/clip.  "" when there is none."""
    explicit = explicit or os.environ.get("MAPFED_BPE_PATH", "")
    if explicit:
        if not osp.isfile(explicit):
            raise FileNotFoundError(f"BPE merges file {explicit} not found")
        return explicit
    cands = []
    if backbone:
        cands.append(osp.join(osp.dirname(osp.abspath(backbone)), BPE_FILE))
    cands.append(osp.join(osp.dirname(osp.abspath(__file__)), BPE_FILE))
    cands.append(osp.join(osp.expanduser("~/.cache/clip"), BPE_FILE))
    for c in cands:
        if osp.isfile(c):
            return c
    return ""


@lru_cache(maxsize=8)
def get_tokenizer(bpe_path: str = "") -> Union[SimpleTokenizer, SyntheticTokenizer]:
    """The BPE tokenizer over `bpe_path`, or the synthetic one for ""."""
    return SimpleTokenizer(bpe_path) if bpe_path else SyntheticTokenizer()


def describe(tok) -> str:
    if tok.kind == "bpe":
        fix = "ftfy" if _HAVE_FTFY else ("ftfy absent: its quote / ligature / width folds and NFC are applied; its "
                                         "repairs of broken text (mojibake, control characters, HTML entities "
                                         "beyond html.unescape) are not, so such captions may tokenize differently")
        return f"CLIP byte-level BPE ({tok.path}, {tok.vocab_size} ids; {fix})"
    return ("synthetic word ids (no bpe_simple_vocab_16e6.txt.gz found: text features differ from CLIP's "
            "tokenizer on real prompts)")
