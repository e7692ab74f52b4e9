"""Portable, counter-based synthetic data for the federated MaPLe hot path.

The reference trains on pretrained CLIP ViT-B/16 weights that are downloaded at
run time (``clip/clip.py:29-68``, called from ``trainers/maple.py:21-40``) and on
disk datasets (``datasets/*.py``).  Neither exists offline, so every weight,
image, label and token id used by this build (and by the golden fixtures that
pin it to the reference) comes from this module.

The generator is a pure function of (seed, tensor name, element index):

    z_i = splitmix64(seed_of(name) + (i + 1) * 0x9E3779B97F4A7C15)
    u_i = (z_i >> 11) * 2**-53                              in [0, 1)
    n_j = sqrt(-2 ln(1 - u_{2j})) * cos(2 pi u_{2j+1})      Box-Muller, float64

so the container that writes the fixtures and the GPU box that checks against
them regenerate bit-identical tensors without shipping 150 M weights.  Values
are rounded to fp16 (also for parameters the reference keeps in fp32), like the
fp16 CLIP checkpoint the reference loads and like every tensor after its first
FedAvg round (``trainers/maple_fed.py:314``).
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Sequence

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

SOT_TOKEN = 49406  # clip/clip.py:207 encoder["<|startoftext|>"]
EOT_TOKEN = 49407  # clip/clip.py:208 encoder["<|endoftext|>"], the row max -> argmax gather
DOT_TOKEN = 269    # id of "." in the CLIP BPE vocab
CONTEXT_LENGTH = 77
VOCAB_SIZE = 49408


def _name_seed(seed: int, name: str) -> np.uint64:
    h = zlib.crc32(name.encode()) | (zlib.adler32(name.encode()) << 32)
    return np.uint64((h ^ (seed * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF)


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.copy()
        z ^= z >> np.uint64(30)
        z *= _M1
        z ^= z >> np.uint64(27)
        z *= _M2
        z ^= z >> np.uint64(31)
    return z


def uniform(seed: int, name: str, n: int, start: int = 0) -> np.ndarray:
    """n uniforms in [0,1) for counters start..start+n-1 of stream (seed, name)."""
    base = _name_seed(seed, name)
    idx = np.arange(start + 1, start + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _splitmix(base + idx * _GOLDEN)
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def normal(seed: int, name: str, n: int, start: int = 0) -> np.ndarray:
    """n standard normals (float64) for elements start..start+n-1 of stream (seed, name)."""
    u = uniform(seed, name, 2 * n, 2 * start)
    u1, u2 = u[0::2], u[1::2]
    return np.sqrt(-2.0 * np.log1p(-u1)) * np.cos(2.0 * math.pi * u2)


def fp16_round(a: np.ndarray) -> np.ndarray:
    return a.astype(np.float16).astype(np.float32)


def randn16(seed: int, name: str, shape: Sequence[int], std: float, mean: float = 0.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    v = mean + std * normal(seed, name, n)
    return fp16_round(v).reshape(shape)


def randint(seed: int, name: str, n: int, low: int, high: int) -> np.ndarray:
    u = uniform(seed, name, n)
    return (low + np.floor(u * (high - low))).astype(np.int64)


# --------------------------------------------------------------------------
# Synthetic tokenizer (the BPE vocab file is absent: clip/simple_tokenizer.py:10-13)
# --------------------------------------------------------------------------

def word_token(word: str) -> int:
    """Deterministic id in [300, 40300) for a lower-cased word; '.' -> DOT_TOKEN."""
    w = word.lower()
    if w == ".":
        return DOT_TOKEN
    return 300 + (zlib.crc32(w.encode()) % 40000)


def encode(text: str) -> List[int]:
    """Whitespace/period split, one token per word (stands in for SimpleTokenizer.encode)."""
    out: List[int] = []
    for raw in text.replace("_", " ").split():
        w = raw
        trail = []
        while w.endswith("."):
            trail.append(".")
            w = w[:-1]
        if w:
            out.append(word_token(w))
        out.extend(word_token(t) for t in trail)
    return out


def tokenize(texts, context_length: int = CONTEXT_LENGTH) -> np.ndarray:
    """clip.tokenize semantics (clip/clip.py:185-221): [SOT] + ids + [EOT], zero pad."""
    if isinstance(texts, str):
        texts = [texts]
    res = np.zeros((len(texts), context_length), dtype=np.int64)
    for i, t in enumerate(texts):
        toks = [SOT_TOKEN] + encode(t) + [EOT_TOKEN]
        if len(toks) > context_length:
            raise RuntimeError(f"Input {t} is too long for context length {context_length}")
        res[i, : len(toks)] = toks
    return res


_SYLL = ["ar", "ba", "co", "de", "el", "fo", "gu", "hi", "in", "jo", "ka", "lu", "mo", "ne",
         "or", "pa", "qu", "ri", "su", "ta", "ur", "vi", "wa", "xe", "yo", "za"]


def synthetic_classnames(n_cls: int, seed: int = 0) -> List[str]:
    """n_cls distinct class names of 1-3 words (ragged EOT positions, like real names)."""
    names = []
    for k in range(n_cls):
        u = uniform(seed, f"classname/{k}", 7)
        nw = 1 + int(u[0] * 3)
        words = []
        for w in range(nw):
            a = _SYLL[int(u[1 + 2 * w] * len(_SYLL))]
            b = _SYLL[int(u[2 + 2 * w] * len(_SYLL))]
            words.append(a + b)
        words[-1] = words[-1] + str(k)
        names.append("_".join(words))
    return names


# --------------------------------------------------------------------------
# CLIP ViT-B/16 + MaPLe synthetic parameters
# --------------------------------------------------------------------------

@dataclass(frozen=True)
class ClipDims:
    """ViT-B/16 geometry (clip/model.py:750-781 infers these from the state dict)."""
    embed_dim: int = 512
    image_resolution: int = 224
    vision_layers: int = 12
    vision_width: int = 768
    vision_patch: int = 16
    context_length: int = 77
    vocab_size: int = VOCAB_SIZE
    text_width: int = 512
    text_heads: int = 8
    text_layers: int = 12

    @property
    def vision_heads(self) -> int:
        return self.vision_width // 64

    @property
    def grid(self) -> int:
        return self.image_resolution // self.vision_patch


def _block_params(seed: int, prefix: str, d: int, n_layers: int) -> Dict[str, np.ndarray]:
    """Init stds follow CLIP.initialize_parameters (clip/model.py:667-674)."""
    out: Dict[str, np.ndarray] = {}
    attn_std = d ** -0.5
    proj_std = d ** -0.5 * (2 * n_layers) ** -0.5
    fc_std = (2 * d) ** -0.5
    for i in range(n_layers):
        p = f"{prefix}.resblocks.{i}."
        out[p + "attn.in_proj_weight"] = randn16(seed, p + "attn.in_proj_weight", (3 * d, d), attn_std)
        out[p + "attn.in_proj_bias"] = randn16(seed, p + "attn.in_proj_bias", (3 * d,), 0.02)
        out[p + "attn.out_proj.weight"] = randn16(seed, p + "attn.out_proj.weight", (d, d), proj_std)
        out[p + "attn.out_proj.bias"] = randn16(seed, p + "attn.out_proj.bias", (d,), 0.02)
        out[p + "ln_1.weight"] = randn16(seed, p + "ln_1.weight", (d,), 0.05, 1.0)
        out[p + "ln_1.bias"] = randn16(seed, p + "ln_1.bias", (d,), 0.02)
        out[p + "mlp.c_fc.weight"] = randn16(seed, p + "mlp.c_fc.weight", (4 * d, d), fc_std)
        out[p + "mlp.c_fc.bias"] = randn16(seed, p + "mlp.c_fc.bias", (4 * d,), 0.02)
        out[p + "mlp.c_proj.weight"] = randn16(seed, p + "mlp.c_proj.weight", (d, 4 * d), proj_std)
        out[p + "mlp.c_proj.bias"] = randn16(seed, p + "mlp.c_proj.bias", (d,), 0.02)
        out[p + "ln_2.weight"] = randn16(seed, p + "ln_2.weight", (d,), 0.05, 1.0)
        out[p + "ln_2.bias"] = randn16(seed, p + "ln_2.bias", (d,), 0.02)
    return out


def token_embedding_rows(seed: int, rows: np.ndarray, width: int = 512) -> np.ndarray:
    """Rows of the [49408, width] token-embedding table (std 0.02, clip/model.py:651),
    generated by random access into the counter stream."""
    rows = np.asarray(rows, dtype=np.int64).reshape(-1)
    out = np.empty((rows.size, width), dtype=np.float32)
    for k, r in enumerate(rows):
        out[k] = fp16_round(0.02 * normal(seed, "token_embedding.weight", width, int(r) * width))
    return out


def clip_state_dict(seed: int = 0, dims: ClipDims = ClipDims(), full_token_table: bool = False,
                    vision_layers: int | None = None, text_layers: int | None = None) -> Dict[str, np.ndarray]:
    """A CLIP ViT-B/16 state dict with the checkpoint's key set (fp32 arrays, fp16-representable)."""
    vl = dims.vision_layers if vision_layers is None else vision_layers
    tl = dims.text_layers if text_layers is None else text_layers
    dv, dt = dims.vision_width, dims.text_width
    sd: Dict[str, np.ndarray] = {}
    g = dims.grid
    sd["visual.class_embedding"] = randn16(seed, "visual.class_embedding", (dv,), dv ** -0.5)
    sd["visual.positional_embedding"] = randn16(seed, "visual.positional_embedding", (g * g + 1, dv), dv ** -0.5)
    sd["visual.conv1.weight"] = randn16(seed, "visual.conv1.weight", (dv, 3, dims.vision_patch, dims.vision_patch),
                                        (3 * dims.vision_patch ** 2) ** -0.5)
    sd["visual.ln_pre.weight"] = randn16(seed, "visual.ln_pre.weight", (dv,), 0.05, 1.0)
    sd["visual.ln_pre.bias"] = randn16(seed, "visual.ln_pre.bias", (dv,), 0.02)
    sd.update(_block_params(seed, "visual.transformer", dv, vl))
    sd["visual.ln_post.weight"] = randn16(seed, "visual.ln_post.weight", (dv,), 0.05, 1.0)
    sd["visual.ln_post.bias"] = randn16(seed, "visual.ln_post.bias", (dv,), 0.02)
    sd["visual.proj"] = randn16(seed, "visual.proj", (dv, dims.embed_dim), dv ** -0.5)
    sd["positional_embedding"] = randn16(seed, "positional_embedding", (dims.context_length, dt), 0.01)
    if full_token_table:
        sd["token_embedding.weight"] = fp16_round(
            0.02 * normal(seed, "token_embedding.weight", dims.vocab_size * dt)).reshape(dims.vocab_size, dt)
    sd.update(_block_params(seed, "transformer", dt, tl))
    sd["ln_final.weight"] = randn16(seed, "ln_final.weight", (dt,), 0.05, 1.0)
    sd["ln_final.bias"] = randn16(seed, "ln_final.bias", (dt,), 0.02)
    sd["text_projection"] = randn16(seed, "text_projection", (dt, dims.embed_dim), dt ** -0.5)
    sd["logit_scale"] = np.array(math.log(1 / 0.07), dtype=np.float32)
    return sd


def prompt_learner_params(seed: int, prompt_depth: int, n_ctx: int = 2, text_width: int = 512,
                          vision_width: int = 768) -> Dict[str, np.ndarray]:
    """Learnable MaPLe tensors except `ctx` (which is the token embedding of the init words),
    names as in MultiModalPromptLearner (trainers/maple.py:111-131)."""
    p: Dict[str, np.ndarray] = {}
    d_t, d_v = text_width, vision_width
    p["proj_lang_to_vis.weight"] = randn16(seed, "pl.proj_lang_to_vis.weight", (d_v, d_t), (3 * d_t) ** -0.5)
    p["proj_lang_to_vis.bias"] = randn16(seed, "pl.proj_lang_to_vis.bias", (d_v,), (3 * d_t) ** -0.5)
    p["proj_vis_to_lang.weight"] = randn16(seed, "pl.proj_vis_to_lang.weight", (d_t, d_v), (3 * d_v) ** -0.5)
    p["proj_vis_to_lang.bias"] = randn16(seed, "pl.proj_vis_to_lang.bias", (d_t,), (3 * d_v) ** -0.5)
    nt = nv = 0
    for i in range(prompt_depth - 1):
        if i % 2 == 0:
            p[f"compound_prompts_text_parameters.{nt}"] = randn16(seed, f"pl.cpt.{nt}", (n_ctx, d_t), 0.02)
            nt += 1
        else:
            p[f"visual_deep_prompts_parameters.{nv}"] = randn16(seed, f"pl.vdp.{nv}", (n_ctx, d_v), 0.02)
            nv += 1
    for i in range(prompt_depth - 1):
        fin, fout = (d_t, d_v) if i % 2 == 0 else (d_v, d_t)
        p[f"compound_prompt_projections.{i}.weight"] = randn16(seed, f"pl.cpp.{i}.w", (fout, fin), (3 * fin) ** -0.5)
        p[f"compound_prompt_projections.{i}.bias"] = randn16(seed, f"pl.cpp.{i}.b", (fout,), (3 * fin) ** -0.5)
    return p


_CAP_WORDS = ["dense", "sparse", "green", "river", "road", "field", "roof", "forest", "harbor", "runway",
              "parking", "lot", "bridge", "lake", "farmland", "residential", "industrial", "beach", "desert",
              "meadow", "highway", "airplane", "cars", "trees", "buildings", "with", "near", "many", "a", "the"]


def synthetic_captions(seed: int, client_id: int, step: int, batch: int) -> List[str]:
    """BLIP-style caption strings for a batch (the reference's datasets carry one per image,
    datasets/patternnet.py Datum.caption); the first is empty, as a missing caption arrives."""
    out = []
    for b in range(batch):
        u = uniform(seed, f"caption/c{client_id}/s{step}/{b}", 12)
        n = 0 if b == 0 else 3 + int(u[0] * 8)
        out.append(" ".join(["a", "satellite", "image", "of"] + [_CAP_WORDS[int(x * len(_CAP_WORDS))] for x in u[1:1 + n]])
                   if n else "")
    return out


@dataclass
class ClientBatch:
    images: np.ndarray   # [B,3,224,224] float32 (already "normalized")
    labels: np.ndarray   # [B] int64


def client_batch(seed: int, client_id: int, step: int, batch: int, n_cls: int,
                 image_resolution: int = 224) -> ClientBatch:
    """Synthetic batch: images ~ N(0,1) rounded to fp16 (the reference casts the image to
    fp16 at trainers/maple.py:336), labels uniform in [0, n_cls)."""
    tag = f"batch/c{client_id}/s{step}"
    n = batch * 3 * image_resolution * image_resolution
    img = fp16_round(normal(seed, tag + "/img", n)).reshape(batch, 3, image_resolution, image_resolution)
    lab = randint(seed, tag + "/label", batch, 0, n_cls)
    return ClientBatch(img, lab)
