"""MaPLe client engine: explicit forward + backward + optimizer step of one federated client on one
MI355X, every op a libmapfed.so kernel over preallocated HBM buffers.

What it computes is CustomCLIP.forward + loss.backward + clip_grad_norm_ + SGD.step of the reference
(trainers/maple.py:304-381, 586-598) for the MaPLe towers of clip/model.py:269-572, with the freeze
policy of trainers/maple.py:447-479.  Because the graph is static, the backward is written out by
hand instead of recorded by autograd:

* dX flows through all 12 blocks of both towers (LN params and prompts are trainable everywhere);
* weight gradients are produced only for block 11 of each tower, every LayerNorm, and the prompt
  learner (nothing else is trainable);
* injected prompt rows are reduced over the batch into the prompt gradient and zeroed in dX, which
  is exactly autograd's result for the `torch.cat([prefix, prompt])` replacement.

Data layout in HBM: activations are [N*L, D] row-major, batch-major (row n*L + l);
the reference's LND permutes are layout-only and vanish.  Per layer the forward saves exactly what
its backward reads (X, QKV, O, LSE, X1, pre-GELU F, LN statistics); block 11 also keeps the LN
outputs and GELU output for its weight gradients.  Trainable parameters live in two flat buffers
(fp16 / fp32) with matching gradient and momentum buffers, so clip-norm, SGD and FedAvg are single
streaming kernels and FedAvg is one RCCL all-reduce of one contiguous bucket.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import ops
from . import synthetic as syn
from .tokenizer import get_tokenizer

F16, F32 = torch.float16, torch.float32
N_CTX = 2


@dataclass
class EngineConfig:
    batch: int                  # B images per client step
    classnames: List[str]       # K classes (text prompts)
    prompt_depth: int = 9       # J (cfg.TRAINER.MAPLE.PROMPT_DEPTH, train.py:113)
    seed: int = 0
    n_ctx: int = N_CTX
    ctx_init: str = "a photo of a"
    dims: syn.ClipDims = field(default_factory=syn.ClipDims)
    momentum: float = 0.9       # Dassl SGD defaults (cfg.OPTIM.MOMENTUM / WEIGHT_DECAY)
    weight_decay: float = 5e-4
    max_grad_norm: float = 1.0
    # Run the text tower on the first max(EOT)+1 tokens instead of all 77 (SURVEY.md §8(d) optional
    # mode, reported separately).  Under the causal mask a token only sees earlier ones, and the tower's
    # output is gathered at the EOT row, so the dropped tokens cannot reach the loss and their gradients are
    # exactly zero.  The truncated tower runs its backward's row reductions (LayerNorm dgamma / dbeta, block
    # 11's dW and db) over the 77-row layout with zero rows in the dropped places (_Tower.live), so logits,
    # loss, every gradient and the updated weights are bit-identical to the full tower's.  Off by default: the
    # reference computes all 77, and the headline bench keeps its work.
    eot_truncate: bool = False
    # The caption-conditioned visual prompts (captions.py, clip/model.py:550-561): the vision tower's
    # prompted blocks each append the batch's B projected caption rows, so block i runs 199 + i*B rows.
    # Buffers are sized for it at construction; a batch then needs set_captions().
    captions: bool = False
    # CLIP's BPE merges file (bpe_simple_vocab_16e6.txt.gz) for the prompt / caption token ids
    # (tokenizer.py); "" -> the seeded synthetic word-id tokenizer
    bpe_path: str = ""
    # towers whose in-projection + attention forward run as one launch (mf_qkv_attention_fwd, bit-identical to the
    # unfused pair): "side" (default) fuses the tower that runs beside the other one on its throughput tiles (tile
    # -1, >= 2 048 rows: the text tower at c4, the vision tower at C5; same-box A/Bs in DESIGN.md §4), "none",
    # "both", "vision" or "text" one tower
    fused_qkv_attn: str = "side"
    # enqueue (and capture) order of the two towers after each fork: the vision tower (the step's critical path)
    # first, so its launches are dispatched ahead of the text tower's (False: text first, the measured baseline)
    vision_first: bool = True
    # forward-only engine (test(): trainers/maple.py:660-681): the towers keep one set of per-block buffers
    # (the forward's intermediates are not saved for a backward) and allocate no gradient buffers, so the eval
    # engine can run large batches; the kernels and their results are those of the training engine's forward
    inference: bool = False


def prompt_prefix(cfg: EngineConfig) -> Tuple[str, Optional[np.ndarray]]:
    """MultiModalPromptLearner.__init__'s context (trainers/maple.py:96-106): with CTX_INIT and n_ctx <= 4 the
    prefix is CTX_INIT ("_" -> " ") and ctx starts from the token embedding of its first n_ctx tokens (ids
    returned); otherwise the prefix is "X X .." and ctx is drawn N(0, 0.02) (ids None)."""
    if cfg.ctx_init and cfg.n_ctx <= 4:
        init = cfg.ctx_init.replace("_", " ")
        ids = get_tokenizer(cfg.bpe_path).tokenize(init, cfg.dims.context_length)[0, 1:1 + cfg.n_ctx]
        return init, ids
    return " ".join(["X"] * cfg.n_ctx), None


def class_prompts(cfg: EngineConfig) -> List[str]:
    """trainers/maple.py:136-138: prefix + " " + classname ("_" -> " ") + "."."""
    prefix, _ = prompt_prefix(cfg)
    return [prefix + " " + c.replace("_", " ") + "." for c in cfg.classnames]


def _is_trainable(name: str) -> bool:
    """trainers/maple.py:447-479."""
    if name.startswith("prompt_learner.") and not name.startswith("prompt_learner.token_"):
        return True
    if "ln_" in name:
        return True
    return "transformer.resblocks.11." in name


_FP16_SUFFIX = ("conv1.weight", "in_proj_weight", "in_proj_bias", "out_proj.weight", "out_proj.bias",
                "c_fc.weight", "c_fc.bias", "c_proj.weight", "c_proj.bias")


def reference_param_specs(cfg: EngineConfig) -> List[Tuple[str, Tuple[int, ...], torch.dtype]]:
    """(name, shape, dtype) of every CustomCLIP parameter the path uses, in named_parameters order."""
    d = cfg.dims
    dv, dt = d.vision_width, d.text_width
    specs: List[Tuple[str, Tuple[int, ...], torch.dtype]] = []
    pl = "prompt_learner."
    specs += [(pl + "ctx", (cfg.n_ctx, dt), F16),
              (pl + "proj_lang_to_vis.weight", (dv, dt), F16), (pl + "proj_lang_to_vis.bias", (dv,), F16),
              (pl + "proj_vis_to_lang.weight", (dt, dv), F16), (pl + "proj_vis_to_lang.bias", (dt,), F16)]
    J = cfg.prompt_depth
    for k in range((J - 1 + 1) // 2):
        specs.append((pl + f"compound_prompts_text_parameters.{k}", (cfg.n_ctx, dt), F32))
    for k in range((J - 1) // 2):
        specs.append((pl + f"visual_deep_prompts_parameters.{k}", (cfg.n_ctx, dv), F32))
    for i in range(J - 1):
        fin, fout = (dt, dv) if i % 2 == 0 else (dv, dt)
        specs += [(pl + f"compound_prompt_projections.{i}.weight", (fout, fin), F32),
                  (pl + f"compound_prompt_projections.{i}.bias", (fout,), F32)]
    ie = "image_encoder."
    g = d.grid
    specs += [(ie + "class_embedding", (dv,), F32), (ie + "positional_embedding", (g * g + 1, dv), F32),
              (ie + "proj", (dv, d.embed_dim), F16), (ie + "conv1.weight", (dv, 3, d.vision_patch, d.vision_patch), F16),
              (ie + "ln_pre.weight", (dv,), F32), (ie + "ln_pre.bias", (dv,), F32)]

    def blocks(prefix, D, n):
        out = []
        for i in range(n):
            p = f"{prefix}.resblocks.{i}."
            out += [(p + "attn.in_proj_weight", (3 * D, D), F16), (p + "attn.in_proj_bias", (3 * D,), F16),
                    (p + "attn.out_proj.weight", (D, D), F16), (p + "attn.out_proj.bias", (D,), F16),
                    (p + "ln_1.weight", (D,), F32), (p + "ln_1.bias", (D,), F32),
                    (p + "mlp.c_fc.weight", (4 * D, D), F16), (p + "mlp.c_fc.bias", (4 * D,), F16),
                    (p + "mlp.c_proj.weight", (D, 4 * D), F16), (p + "mlp.c_proj.bias", (D,), F16),
                    (p + "ln_2.weight", (D,), F32), (p + "ln_2.bias", (D,), F32)]
        return out

    specs += blocks(ie + "transformer", dv, d.vision_layers)
    specs += [(ie + "ln_post.weight", (dv,), F32), (ie + "ln_post.bias", (dv,), F32)]
    te = "text_encoder."
    specs += blocks(te + "transformer", dt, d.text_layers)
    specs += [(te + "positional_embedding", (d.context_length, dt), F32), (te + "ln_final.weight", (dt,), F32),
              (te + "ln_final.bias", (dt,), F32), (te + "text_projection", (dt, d.embed_dim), F16),
              ("logit_scale", (), F32)]
    return specs


def clip_dims_from_state_dict(sd) -> syn.ClipDims:
    """CLIP geometry from a checkpoint's tensors, as clip/model.py:750-777 (build_model) infers it.  The
    MaPLe path is the ViT one (VisionTransformer_MaPLe); MultiModalPromptLearner hard-codes the 768-wide
    vision and 512-wide text prompts (trainers/maple.py:111-124), i.e. ViT-B/16 and ViT-B/32."""
    shape = lambda k: tuple(np.shape(sd[k]))
    if "visual.proj" not in sd:
        raise NotImplementedError("a ResNet CLIP checkpoint: MaPLe's image encoder is the ViT (clip/model.py:478)")
    vw = shape("visual.conv1.weight")[0]
    vl = len([k for k in sd if k.startswith("visual.") and k.endswith(".attn.in_proj_weight")])
    patch = shape("visual.conv1.weight")[-1]
    grid = round((shape("visual.positional_embedding")[0] - 1) ** 0.5)
    tw = shape("ln_final.weight")[0]
    return syn.ClipDims(embed_dim=shape("text_projection")[1], image_resolution=patch * grid, vision_layers=vl,
                        vision_width=vw, vision_patch=patch, context_length=shape("positional_embedding")[0],
                        vocab_size=shape("token_embedding.weight")[0] if "token_embedding.weight" in sd
                        else syn.VOCAB_SIZE, text_width=tw, text_heads=tw // 64,
                        text_layers=len({k.split(".")[2] for k in sd if k.startswith("transformer.resblocks")}))


def check_dims(d: syn.ClipDims):
    """The geometry the kernels take: head dim 64, sequence lengths <= 256 (attention), GEMM K a multiple of
    64 (patch embedding 3*patch^2, widths), the prompt learner's 768 / 512 widths."""
    Lv = d.grid * d.grid + 1 + N_CTX
    bad = []
    if d.vision_width != 768 or d.text_width != 512:
        bad.append("vision / text width 768 / 512 (trainers/maple.py:111-124 hard-codes them)")
    if Lv > 256 or d.context_length > 256:
        bad.append(f"sequence lengths <= 256 (vision {Lv}, text {d.context_length})")
    if (3 * d.vision_patch ** 2) % 64:
        bad.append(f"3*patch^2 a multiple of 64 (patch {d.vision_patch})")
    if bad:
        raise NotImplementedError("CLIP geometry outside the MI355X path: " + "; ".join(bad))


def synthetic_state(cfg: EngineConfig) -> Dict[str, np.ndarray]:
    """Synthetic values for every spec, keyed by CustomCLIP parameter name (numpy fp32)."""
    d = cfg.dims
    sd = syn.clip_state_dict(cfg.seed, d, vision_layers=d.vision_layers, text_layers=d.text_layers)
    return engine_state_from_clip(sd, cfg)


def engine_state_from_clip(clip_sd: Dict[str, np.ndarray], cfg: EngineConfig,
                           prompt_learner: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
    """Map a CLIP checkpoint state dict (keys of clip/model.py CLIP: visual.*, transformer.*,
    positional_embedding, ln_final.*, text_projection, token_embedding.weight, logit_scale) onto the
    engine's CustomCLIP parameter names (trainers/maple.py:44-58,221-229), the way build_model +
    CustomCLIP wire it (clip/model.py:750-793).  ctx is initialised from the token embedding of
    CTX_INIT (trainers/maple.py:96-103); the other prompt-learner tensors come from
    `prompt_learner` (names without the prefix) or the synthetic generator.  logit_scale is MaPLe's
    own ln(1/0.07) (trainers/maple.py:227), not the checkpoint's."""
    out: Dict[str, np.ndarray] = {}
    for k, v in clip_sd.items():
        v = np.asarray(v, dtype=np.float32)
        if k.startswith("visual."):
            out["image_encoder." + k[7:]] = v
        elif k in ("positional_embedding", "ln_final.weight", "ln_final.bias", "text_projection") or \
                k.startswith("transformer."):
            out["text_encoder." + k] = v
    _, init = prompt_prefix(cfg)
    if init is None:  # no CTX_INIT: nn.init.normal_(ctx, std=0.02) (trainers/maple.py:104-105)
        out["prompt_learner.ctx"] = syn.randn16(cfg.seed, "pl.ctx", (cfg.n_ctx, cfg.dims.text_width), 0.02)
    elif "token_embedding.weight" in clip_sd:
        table = np.asarray(clip_sd["token_embedding.weight"], dtype=np.float32)
        _check_ids(init, table.shape[0])
        out["prompt_learner.ctx"] = table[init]
    else:
        _check_ids(init, cfg.dims.vocab_size)
        out["prompt_learner.ctx"] = syn.token_embedding_rows(cfg.seed, init)
    pl = prompt_learner if prompt_learner is not None else syn.prompt_learner_params(cfg.seed, cfg.prompt_depth,
                                                                                     cfg.n_ctx)
    for k, v in pl.items():
        out["prompt_learner." + k] = np.asarray(v, dtype=np.float32)
    out["logit_scale"] = np.array(math.log(1 / 0.07), dtype=np.float32)
    # CLIP's own tensors the towers do not read but CustomCLIP.state_dict() carries as clip_model2.*
    # aliases (trainers/maple.py:229): its logit_scale and the token-embedding table
    if "logit_scale" in clip_sd:
        out["clip_model2.logit_scale"] = np.asarray(clip_sd["logit_scale"], dtype=np.float32)
    if "token_embedding.weight" in clip_sd:
        out["clip_model2.token_embedding.weight"] = np.asarray(clip_sd["token_embedding.weight"], dtype=np.float32)
    return out


def _check_ids(ids: np.ndarray, vocab: int):
    """Token ids index CLIP's [vocab, 512] embedding table (on the host here, on the device for captions)."""
    ids = np.asarray(ids)
    if ids.size and (int(ids.min()) < 0 or int(ids.max()) >= vocab):
        raise ValueError(f"token ids in [{int(ids.min())}, {int(ids.max())}] outside the {vocab}-row token embedding "
                         "(a BPE merges file larger than the checkpoint's vocabulary?)")


class _Tower:
    """Buffers + forward/backward schedule of one 12-block transformer tower.

    Ls (optional): the input sequence length of every block.  Without it every block runs L rows per
    sequence and the deep prompt of a prompted block overwrites rows inject_row0.. of its input in place
    (fused into ln_1).  With it (the vision tower under the caption path, captions.py) a prompted block's
    input is built from the previous block's output by mf_seq_grow: all but its last n_ctx rows, the ncap
    caption rows, the block's deep prompt -- Ls[i] = Ls[i-1] + ncap -- and the backward undoes it
    (mf_seq_grow_bwd, the prompt's gradient reduced over the sequences)."""

    def __init__(self, eng: "MapleEngine", name: str, N: int, L: int, D: int, H: int, layers: int,
                 causal: bool, inject_row0: int, Ls: Optional[List[int]] = None, ncap: int = 0,
                 L_full: Optional[int] = None):
        self.e, self.name, self.N, self.L, self.D, self.H = eng, name, N, L, D, H
        # L_full (the EOT-truncated text tower): the tower computes only the first L of every L_full-row sequence;
        # the row reductions of its backward (LayerNorm dgamma / dbeta, block 11's dW and db) run over the
        # L_full-row layout with zero rows in the other places, so every result is bit for bit the full tower's
        self.live = (L, L_full) if L_full is not None and L_full != L else None
        self.layers, self.causal, self.row0 = layers, causal, inject_row0
        self.Ls = list(Ls) if Ls is not None else [L] * layers
        assert len(self.Ls) == layers and self.Ls[0] == L
        self.ncap = ncap
        self.grow = [i > 0 and self.Ls[i] != self.Ls[i - 1] for i in range(layers)]
        assert not any(self.grow) or all(self.Ls[i] - self.Ls[i - 1] in (0, ncap) for i in range(1, layers))
        self.L_out = self.Ls[-1]
        dev = eng.device
        Rs = [N * l for l in self.Ls]
        self.Rs = Rs
        R = max(Rs)
        self.R = R
        e = lambda *s, dt=F16: torch.empty(*s, device=dev, dtype=dt)
        self.inference = bool(eng.cfg.inference)
        # cls_only (set by MapleEngine for a forward-only vision tower): the last block computes only what row 0 of
        # each sequence of its output needs (the class token that ln_post reads, clip/model.py:567) -- K / V of every
        # row, query 0's attention, and out-proj / ln_2 / MLP on the N class rows; each row's arithmetic is the full
        # block's (GEMM rows and attention queries are independent), so the class rows are bit-identical
        self.cls_only = False
        if self.inference:
            if any(self.grow):
                raise NotImplementedError("EngineConfig.inference with growing (caption) sequences")
            self._alloc_forward_only(e, R, N, H, D, layers)
            return
        # X[i]: input of block i (X[layers]: the tower's output); Y[i]: block i's output buffer -- X[i+1] itself
        # unless block i+1 grows the sequence
        self.X = [e(Rs[0], D)]
        self.Y = []
        for i in range(layers):
            if i + 1 < layers and self.grow[i + 1]:
                self.Y.append(e(Rs[i], D))
                self.X.append(e(Rs[i + 1], D))
            else:
                self.X.append(e(Rs[i], D))
                self.Y.append(self.X[i + 1])
        self.QKV = [e(Rs[i], 3 * D) for i in range(layers)]
        self.O = [e(Rs[i], D) for i in range(layers)]
        self.X1 = [e(Rs[i], D) for i in range(layers)]
        self.Fp = [e(Rs[i], 4 * D) for i in range(layers)]
        self.LSE = [e(N * H * self.Ls[i], dt=F32) for i in range(layers)]
        self.mean1 = [e(Rs[i], dt=F32) for i in range(layers)]
        self.rstd1 = [e(Rs[i], dt=F32) for i in range(layers)]
        self.mean2 = [e(Rs[i], dt=F32) for i in range(layers)]
        self.rstd2 = [e(Rs[i], dt=F32) for i in range(layers)]
        self.H1 = e(R, D)
        self.H2 = e(R, D)
        self.G = e(R, 4 * D)
        # backward
        self.dX = e(R, D)
        self.dX2 = e(R, D) if any(self.grow) else None  # the shrunk gradient of a growing block's input
        self.dX1 = e(R, D)
        self.dO = e(R, D)
        self.dH = e(R, D)
        self.dQKV = e(R, 3 * D)
        self.dF = e(R, 4 * D)
        self.attn_ws = e(N * H * max(self.Ls), dt=F32)
        # the in-projection + attention forward as one launch (mf_qkv_attention_fwd) where its shapes allow
        # (EngineConfig.fused_qkv_attn; "side" is resolved by MapleEngine once both towers exist)
        sel = eng.cfg.fused_qkv_attn
        if sel not in ("side", "none", "both", "vision", "text"):
            raise ValueError(f"EngineConfig.fused_qkv_attn: {sel!r}")
        self.fused_qkv_attn = sel == "both" or sel == ("vision" if name == "image_encoder" else "text")
        # GEMM tile rule of this tower's projections: 0 = latency picks (the tower that sets the step), -1 =
        # work-per-CU-second picks (the tower beside it; MapleEngine.__init__ decides, csrc/gemm.hip text_tile)
        self.tile = 0
        # this tower's LayerNorm dgamma/dbeta partials, reduced in one launch at the end of its backward
        self.lnb = ops.LNGradBatch(dev)
        self.cs_ws = e(ops.colsum_ws_floats(R if self.live is None else N * self.live[1], 4 * D), dt=F32)
        # split-K weight gradients of the trainable block (few output tiles, K = R tokens): fp32 partial
        # planes, summed in a fixed order (only where the automatic split count exceeds 1: few 128x128 output tiles)
        shapes = ((3 * D, D), (D, D), (4 * D, D), (D, 4 * D))
        Rl = Rs[-1] if self.live is None else N * self.live[1]
        ws = {s: ops.gemm_splitk_ws_floats(s[0], s[1], Rl) for s in shapes}
        self.dw_split = {s for s in shapes if ws[s] > s[0] * s[1]}
        self.dw_ws = e(max(ws[s] for s in self.dw_split), dt=F32) if self.dw_split else None
        # the live tower's block-11 dW / db operands in the full row layout (rows past L stay zero: written once)
        self.full_dy = self.full_x = None
        if self.live is not None:
            z = lambda: torch.zeros(Rl, 4 * D, device=dev, dtype=F16)
            self.full_dy, self.full_x = z(), z()

    def _alloc_forward_only(self, e, R, N, H, D, layers):
        """Inference buffers: block i reads X[i] and writes X[i + 1], so two alternating activation buffers
        serve every block; each per-block intermediate list aliases one buffer (nothing is kept for a
        backward)."""
        xb = (e(R, D), e(R, D))
        self.X = [xb[i % 2] for i in range(layers + 1)]
        self.Y = self.X[1:]
        one = lambda *s, dt=F16: [e(*s, dt=dt)] * layers
        self.QKV, self.O, self.X1, self.Fp = one(R, 3 * D), one(R, D), one(R, D), one(R, 4 * D)
        self.LSE = one(N * H * self.L, dt=F32)
        self.mean1, self.rstd1, self.mean2, self.rstd2 = (one(R, dt=F32) for _ in range(4))
        self.H1, self.H2, self.G = e(R, D), e(R, D), e(R, 4 * D)
        self.dX = self.dX2 = self.dX1 = self.dO = self.dH = self.dQKV = self.dF = self.attn_ws = None
        self.fused_qkv_attn = self.e.cfg.fused_qkv_attn in ("both", "vision" if self.name == "image_encoder"
                                                             else "text")
        self.tile = 0
        self.lnb = self.cs_ws = self.dw_ws = None
        self.dw_split = set()

    # -- parameters of block i
    def p(self, i: int, key: str) -> torch.Tensor:
        return self.e.P[f"{self.name}.transformer.resblocks.{i}.{key}"]

    def wt(self, i: int, key: str) -> torch.Tensor:
        return self.e.WT[f"{self.name}.transformer.resblocks.{i}.{key}"]

    def g(self, i: int, key: str) -> torch.Tensor:
        return self.e.G[f"{self.name}.transformer.resblocks.{i}.{key}"]

    # ------------------------------------------------------------------------------------------
    def forward(self, deep_prompts: List[torch.Tensor], cap: Optional[torch.Tensor] = None):
        """X[0] must be filled.  deep_prompts[j] (fp32 [n_ctx, D]) is injected before layer j+1; cap [ncap, D]
        (fp16): the caption rows a growing block appends before its prompt."""
        N, D, H = self.N, self.D, self.H
        for i in range(self.layers):
            L, R = self.Ls[i], self.Rs[i]
            x = self.X[i]
            h1 = self.H1[:R]
            if 1 <= i <= len(deep_prompts) and not self.grow[i]:  # prompt injected into x and ln_1 in one pass
                ops.layernorm_fwd_inject(x, self.p(i, "ln_1.weight"), self.p(i, "ln_1.bias"), h1, self.mean1[i],
                                         self.rstd1[i], deep_prompts[i - 1], L, self.row0, N_CTX)
            else:
                ops.layernorm_fwd(x, self.p(i, "ln_1.weight"), self.p(i, "ln_1.bias"), h1, self.mean1[i],
                                  self.rstd1[i])
            if self.cls_only and i == self.layers - 1:
                self._last_block_cls_rows(i, x, h1, L)
                continue
            if self.fused_qkv_attn and ops.qkv_attention_supported(N, L, H, self.causal):
                # in-projection + attention in one launch (bit-identical to the pair below)
                ops.qkv_attention_fwd(h1, self.p(i, "attn.in_proj_weight"), self.p(i, "attn.in_proj_bias"),
                                      self.QKV[i], self.O[i], self.LSE[i], N, L, H, self.causal)
            else:
                ops.gemm_nt(h1, self.p(i, "attn.in_proj_weight"), self.QKV[i], bias=self.p(i, "attn.in_proj_bias"),
                            epilogue=ops.EPI_BIAS, tile=self.tile)
                ops.attention_fwd(self.QKV[i], N, L, H, self.causal, out=self.O[i], lse=self.LSE[i])
            h2 = self.H2[:R]
            ops.gemm_nt(self.O[i], self.p(i, "attn.out_proj.weight"), self.X1[i],
                        bias=self.p(i, "attn.out_proj.bias"), aux_in=x, epilogue=ops.EPI_BIAS_RESID, tile=self.tile)
            ops.layernorm_fwd(self.X1[i], self.p(i, "ln_2.weight"), self.p(i, "ln_2.bias"), h2, self.mean2[i],
                              self.rstd2[i])
            g = self.G[:R]
            # the pre-activation is kept for the backward (QuickGELU'); a forward-only engine skips its store
            ops.gemm_nt(h2, self.p(i, "mlp.c_fc.weight"), g, bias=self.p(i, "mlp.c_fc.bias"),
                        aux_out=None if self.inference else self.Fp[i], epilogue=ops.EPI_BIAS_GELU, tile=self.tile)
            ops.gemm_nt(g, self.p(i, "mlp.c_proj.weight"), self.Y[i], bias=self.p(i, "mlp.c_proj.bias"),
                        aux_in=self.X1[i], epilogue=ops.EPI_BIAS_RESID, tile=self.tile)
            if i + 1 < self.layers and self.grow[i + 1]:
                ops.seq_grow(self.Y[i], self.X[i + 1], cap, deep_prompts[i], N, L, self.ncap, N_CTX, D)
        # self.H1 / H2 / G now hold the last layer's (block 11) tensors, kept for its dW

    def _last_block_cls_rows(self, i: int, x: torch.Tensor, h1: torch.Tensor, L: int):
        """Block i (the last) of a forward-only tower for the rows n * L only (cls_only): the key / value part of the
        in-projection for every row and its query part for the class rows, the attention of query row 0
        (mf_attention_fwd_rows; the other queries of its 16-row tile read stale q rows and are not used), then
        out-proj + residual, ln_2 and the MLP on the N class rows through strided views (row n * L of O, X1, Y)."""
        N, H, D = self.N, self.H, self.D
        w, b = self.p(i, "attn.in_proj_weight"), self.p(i, "attn.in_proj_bias")
        ops.gemm_nt(h1, w[D:], self.QKV[i][:, D:], bias=b[D:], epilogue=ops.EPI_BIAS, tile=self.tile)
        ops.gemm_nt(h1[::L], w[:D], self.QKV[i][::L, :D], bias=b[:D], epilogue=ops.EPI_BIAS, tile=self.tile)
        ops.attention_fwd_rows(self.QKV[i], N, L, H, self.causal, 1, out=self.O[i], lse=self.LSE[i])
        x1 = self.X1[i][::L]
        ops.gemm_nt(self.O[i][::L], self.p(i, "attn.out_proj.weight"), x1, bias=self.p(i, "attn.out_proj.bias"),
                    aux_in=x[::L], epilogue=ops.EPI_BIAS_RESID, tile=self.tile)
        h2 = self.H2[:N]
        ops.layernorm_fwd(x1, self.p(i, "ln_2.weight"), self.p(i, "ln_2.bias"), h2, self.mean2[i][:N],
                          self.rstd2[i][:N])
        g = self.G[:N]
        ops.gemm_nt(h2, self.p(i, "mlp.c_fc.weight"), g, bias=self.p(i, "mlp.c_fc.bias"), epilogue=ops.EPI_BIAS_GELU,
                    tile=self.tile)
        ops.gemm_nt(g, self.p(i, "mlp.c_proj.weight"), self.Y[i][::L], bias=self.p(i, "mlp.c_proj.bias"), aux_in=x1,
                    epilogue=ops.EPI_BIAS_RESID, tile=self.tile)

    def _dw(self, dY: torch.Tensor, Xin: torch.Tensor, dW: torch.Tensor, db: torch.Tensor):
        """dW[out,in] = dY^T . Xin (fp16 out; both operands read K-major in place, K = rows), db = colsum(dY).
        A live (EOT-truncated) tower first scatters both operands into the full row layout, so K and the
        summation order are the full tower's (its extra rows contribute exact zeros)."""
        if self.live is not None:
            Ll, Lf = self.live
            # exactness rests on full_dy / full_x rows t >= Ll staying zero: they are zeroed at allocation and the
            # only writer is this scatter, which writes rows t < Ll of column views that start at the buffers'
            # own first element (checked here, so no caller can hand it an offset view)
            for src, full in ((dY, self.full_dy), (Xin, self.full_x)):
                assert src.shape[0] == self.N * Ll and src.shape[1] <= full.shape[1] and full.shape[0] == self.N * Lf
            dY = ops.seq_scatter(dY, self.full_dy[:, :dY.shape[1]], self.N, Ll, Lf)[:self.N * Lf]
            Xin = ops.seq_scatter(Xin, self.full_x[:, :Xin.shape[1]], self.N, Ll, Lf)[:self.N * Lf]
        if tuple(dW.shape) in self.dw_split:
            ops.gemm_splitk(dY, Xin, dW, self.dw_ws, a_kmajor=True, b_kmajor=True)
        else:
            ops.gemm(dY, Xin, dW, epilogue=ops.EPI_NONE, a_kmajor=True, b_kmajor=True)
        ops.colsum(dY, db, self.cs_ws)

    def backward(self, n_prompted: int, prompt_grads: List[torch.Tensor]):
        """self.dX[:Rs[-1]] holds d(loss)/d(X[layers]).  On return self.dX[:Rs[0]] = d(loss)/d(X[0]) (the
        injected rows of prompted layers reduced into prompt_grads[j] for the prompt injected before layer
        j+1)."""
        if self.inference:
            raise RuntimeError("backward on a forward-only (EngineConfig.inference) engine")
        N, D, H = self.N, self.D, self.H
        last = self.layers - 1
        for i in reversed(range(self.layers)):
            L, R = self.Ls[i], self.Rs[i]
            dX = self.dX[:R]
            dF, dH, dO, dQKV = self.dF[:R], self.dH[:R], self.dO[:R], self.dQKV[:R]
            trainable_w = i == last
            # ---- MLP: X[i+1] = X1 + c_proj(gelu(c_fc(ln_2(X1))))
            ops.gemm_nt(dX, self.wt(i, "mlp.c_proj.weight"), dF, aux_in=self.Fp[i], epilogue=ops.EPI_DGELU,
                        tile=self.tile)
            if trainable_w:
                self._dw(dX, self.G[:R], self.g(i, "mlp.c_proj.weight"), self.g(i, "mlp.c_proj.bias"))
            ops.gemm_nt(dF, self.wt(i, "mlp.c_fc.weight"), dH, epilogue=ops.EPI_NONE, tile=self.tile)
            if trainable_w:
                self._dw(dF, self.H2[:R], self.g(i, "mlp.c_fc.weight"), self.g(i, "mlp.c_fc.bias"))
            self.lnb.bwd(dH, self.X1[i], self.p(i, "ln_2.weight"), self.mean2[i], self.rstd2[i], dX,
                         self.g(i, "ln_2.weight"), self.g(i, "ln_2.bias"), dres=dX, live=self.live)
            # ---- attention: X1 = X + out_proj(attn(ln_1(X)))
            ops.gemm_nt(dX, self.wt(i, "attn.out_proj.weight"), dO, epilogue=ops.EPI_NONE, tile=self.tile)
            if trainable_w:
                self._dw(dX, self.O[i], self.g(i, "attn.out_proj.weight"), self.g(i, "attn.out_proj.bias"))
            ops.attention_bwd(self.QKV[i], self.O[i], dO, self.LSE[i], N, L, H, self.causal, dqkv=dQKV,
                              ws=self.attn_ws)
            ops.gemm_nt(dQKV, self.wt(i, "attn.in_proj_weight"), dH, epilogue=ops.EPI_NONE, tile=self.tile)
            if trainable_w:
                self._dw(dQKV, self.H1[:R], self.g(i, "attn.in_proj_weight"), self.g(i, "attn.in_proj_bias"))
            if 1 <= i <= n_prompted and not self.grow[i]:
                # ln_1 backward + the deep prompt's gradient (its rows of dX) in one pass
                self.lnb.bwd_inject(dH, self.X[i], self.p(i, "ln_1.weight"), self.mean1[i], self.rstd1[i], dX,
                                    self.g(i, "ln_1.weight"), self.g(i, "ln_1.bias"), dX, prompt_grads[i - 1], L,
                                    self.row0, N_CTX, live=self.live)
            else:
                self.lnb.bwd(dH, self.X[i], self.p(i, "ln_1.weight"), self.mean1[i], self.rstd1[i], dX,
                             self.g(i, "ln_1.weight"), self.g(i, "ln_1.bias"), dres=dX, live=self.live)
            if self.grow[i]:
                # the block's input was [previous output minus its last n_ctx rows | captions | prompt]: the
                # prompt's gradient is its rows summed over the sequences; the previous output gets the rest
                ops.prompt_inject_bwd(dX, N, L, L - N_CTX, N_CTX, D, prompt_grads[i - 1], accumulate=False,
                                      zero_rows=False)
                Lp = self.Ls[i - 1]
                ops.seq_grow_bwd(dX, self.dX2[:N * Lp], N, Lp, self.ncap, N_CTX, D)
                self.dX, self.dX2 = self.dX2, self.dX


class MapleEngine:
    """One federated client on one GPU."""

    def __init__(self, cfg: EngineConfig, device="cuda", state: Optional[Dict[str, np.ndarray]] = None,
                 shared: Optional["MapleEngine"] = None):
        """state: parameter values by CustomCLIP name (default: the synthetic generator).
        shared: another engine whose parameters (and gradients, optimizer state, text constants)
        this one uses -- e.g. the test-batch engine next to a training engine (different batch
        size, same model), as trainers/maple.py:660-681 evaluates the model being trained."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.tokenizer = get_tokenizer(cfg.bpe_path)  # prompts and captions (CLIP BPE or the synthetic ids)
        d = cfg.dims
        self.B, self.K, self.J = cfg.batch, len(cfg.classnames), cfg.prompt_depth
        assert 1 <= self.J <= 12, "PROMPT_DEPTH must be in [1, 12]"
        check_dims(d)
        self.specs = reference_param_specs(cfg)
        if shared is None:
            vals = state if state is not None else synthetic_state(cfg)
            self._build_params(vals)
            # clip_model2.logit_scale (CLIP's, not MaPLe's) and clip_model2.token_embedding.weight: host
            # copies for the reference's state-dict key set; the table is generated on first use when the
            # weights are the seeded synthetic CLIP
            ls = vals.get("clip_model2.logit_scale", math.log(1 / 0.07))
            self.clip_logit_scale = torch.tensor(float(torch.as_tensor(ls).reshape(-1)[0].item()),
                                                 dtype=F32, device=self.device)
            tok = vals.get("clip_model2.token_embedding.weight")
            self._token_table = None if tok is None else torch.as_tensor(np.asarray(tok, dtype=np.float32))
            self._table_owner = self
            self._build_text_constants()
            # {lr, momentum, weight_decay, first_step, halt}: read by the SGD kernels from device memory
            self.hyper = torch.tensor([0.0, cfg.momentum, cfg.weight_decay, 1.0, 0.0], device=self.device, dtype=F32)
        else:
            assert shared.K == self.K and shared.J == self.J and shared.device == self.device
            assert shared.cfg.eot_truncate == cfg.eot_truncate
            for a in ("n16", "n32", "flat16", "flat32", "gflat16", "gflat32", "mom16", "mom32", "P", "G",
                      "trainable_names", "conv_w", "chunks", "nchunks", "norm_part", "clip_out", "WT", "tokenized",
                      "token_prefix", "token_suffix", "token_suffix_run", "text_len", "eot_rows", "hyper",
                      "clip_logit_scale", "_table_owner"):
                setattr(self, a, getattr(shared, a))
        G2 = d.grid * d.grid
        self.Lv = G2 + 1 + cfg.n_ctx
        self.G2 = G2
        Ls = None
        if cfg.captions:
            from .captions import vision_lengths
            Ls = vision_lengths(G2, cfg.n_ctx, d.vision_layers, self.J - 1, self.B)
            if max(Ls) > 512:
                raise NotImplementedError(f"caption path: vision sequence of {max(Ls)} rows (> 512) at B={self.B}, "
                                          f"J={self.J}")
        self.vis = _Tower(self, "image_encoder", self.B, self.Lv, d.vision_width, d.vision_heads, d.vision_layers,
                          False, G2 + 1, Ls=Ls, ncap=self.B if cfg.captions else 0)
        self.txt = _Tower(self, "text_encoder", self.K, self.text_len, d.text_width, d.text_heads, d.text_layers,
                          True, 1, L_full=d.context_length)
        self._build_io()
        # the tower with less projection work per step runs beside the other one (the text tower at c4, the
        # vision tower at C5): its GEMMs take the work-per-CU-second tiles (csrc/gemm.hip, tile -1)
        vis_work = self.vis.N * self.vis.L * self.vis.D ** 2
        txt_work = self.txt.N * self.txt.L * self.txt.D ** 2
        (self.txt if txt_work <= vis_work else self.vis).tile = -1
        if cfg.fused_qkv_attn == "side":
            # the side tower's in-projection + attention as one launch (the text tower at c4, the vision tower at
            # C5; r04 same-box A/Bs)
            for t in (self.vis, self.txt):
                t.fused_qkv_attn = t.tile == -1 and t.Rs[0] >= 2048
        # a forward-only engine's vision tower: ln_post reads the last block's output at the class rows only
        self.vis.cls_only = bool(cfg.inference) and not cfg.captions
        self.side = torch.cuda.Stream(device=self.device)
        self.overlap_towers = True  # False: both towers on the current stream (isolated kernel timing)
        self.vision_first = cfg.vision_first  # tower enqueue order after each fork (EngineConfig)
        self.step_count = 0
        self.momentum_initialised = False

    # ------------------------------------------------------------------ parameters
    def _build_params(self, vals: Dict[str, np.ndarray]):
        dev = self.device
        tr16 = [(n, s) for n, s, dt in self.specs if _is_trainable(n) and dt == F16 and "proj_vis_to_lang" not in n]
        tr32 = [(n, s) for n, s, dt in self.specs if _is_trainable(n) and dt == F32]
        n16 = sum(int(np.prod(s)) for _, s in tr16)
        n32 = sum(int(np.prod(s)) for _, s in tr32)
        self.n16, self.n32 = n16, n32
        self.flat16 = torch.empty(n16, device=dev, dtype=F16)
        self.flat32 = torch.empty(n32, device=dev, dtype=F32)
        self.gflat16 = torch.zeros(n16, device=dev, dtype=F16)
        self.gflat32 = torch.zeros(n32, device=dev, dtype=F32)
        self.mom16 = torch.zeros(n16, device=dev, dtype=F16)
        self.mom32 = torch.zeros(n32, device=dev, dtype=F32)
        self.P: Dict[str, torch.Tensor] = {}
        self.G: Dict[str, torch.Tensor] = {}
        self.trainable_names: List[str] = []
        segs = []  # (offset, numel, is16) per trainable tensor, in order
        off = 0
        for n, s in tr16:
            k = int(np.prod(s))
            self.P[n] = self.flat16[off:off + k].view(s)
            self.G[n] = self.gflat16[off:off + k].view(s)
            segs.append((off, k, 1))
            self.trainable_names.append(n)
            off += k
        off = 0
        for n, s in tr32:
            k = int(np.prod(s))
            self.P[n] = self.flat32[off:off + k].view(s)
            self.G[n] = self.gflat32[off:off + k].view(s)
            segs.append((off, k, 0))
            self.trainable_names.append(n)
            off += k
        for n, s, dt in self.specs:
            if n in self.P:
                continue
            self.P[n] = torch.empty(s, device=dev, dtype=dt)
        for n, s, dt in self.specs:
            v = vals[n]
            assert tuple(v.shape) == tuple(s), (n, v.shape, s)
            self.P[n].copy_(torch.from_numpy(np.ascontiguousarray(v).reshape(s)).to(dt))
        # conv1 as a [768, 3*16*16] GEMM operand (im2col K order c, kh, kw)
        cw = self.P["image_encoder.conv1.weight"]
        self.conv_w = cw.view(cw.shape[0], -1)
        # chunk table for clip_grad_norm (segments in trainable order; fp16 first then fp32)
        ce = ops.optim_chunk_elems()
        rows = []
        for sid, (o, k, is16) in enumerate(segs):
            for s0 in range(o, o + k, ce):
                rows.append((sid, is16, s0, min(o + k, s0 + ce)))
        arr = np.zeros(len(rows), dtype=np.dtype([("seg", np.int32), ("is16", np.int32), ("s", np.int64),
                                                  ("e", np.int64)]))
        for i, r in enumerate(rows):
            arr[i] = r
        self.chunks = torch.from_numpy(arr.view(np.uint8)).to(dev)
        self.nchunks = len(rows)
        self.norm_part = torch.empty(self.nchunks, device=dev, dtype=F32)
        self.clip_out = torch.zeros(3, device=dev, dtype=F32)
        # W^T copies for the dX products (a row-major B operand keeps them on the fast ds_read_b128
        # fragment path; measured 15-18 % faster than reading W K-major).  Frozen blocks are transposed
        # once; block 11 after every optimizer step.  The weight gradients and the head projections
        # read their operands in place (K-major GEMM operands, mf_gemm).
        self.WT: Dict[str, torch.Tensor] = {}
        for n, s, dt in self.specs:
            if ".resblocks." in n and n.endswith(("in_proj_weight", "out_proj.weight", "c_fc.weight", "c_proj.weight")):
                self.WT[n] = torch.empty(s[1], s[0], device=dev, dtype=F16)
        self.refresh_transposes(all_layers=True)

    def refresh_transposes(self, all_layers: bool = False):
        """W^T copies of the dX products: every block once, block 11 (trainable) after each update."""
        for n, t in self.WT.items():
            if all_layers or ".resblocks.11." in n:
                ops.transpose(self.P[n], t)

    def _build_text_constants(self):
        """token prefix / suffix buffers and the EOT gather index (trainers/maple.py:136-149)."""
        cfg = self.cfg
        d = cfg.dims
        texts = class_prompts(cfg)
        tok = self.tokenizer.tokenize(texts, d.context_length)
        self.tokenized = torch.from_numpy(tok)
        if self._token_table is not None:  # the checkpoint's token embedding (trainers/maple.py:140-143)
            _check_ids(tok, self._token_table.shape[0])
            emb = self._token_table.cpu()[torch.from_numpy(tok.reshape(-1))].numpy()
        else:
            _check_ids(tok, d.vocab_size)
            emb = syn.token_embedding_rows(cfg.seed, tok.reshape(-1), d.text_width)
        emb = emb.reshape(len(texts), d.context_length, d.text_width)
        dev = self.device
        self.token_prefix = torch.from_numpy(emb[:, :1]).to(dev, F16).contiguous()
        self.token_suffix = torch.from_numpy(emb[:, 1 + cfg.n_ctx:]).to(dev, F16).contiguous()
        eot = tok.argmax(axis=-1)
        L = cfg.dims.context_length
        self.text_len = max(int(eot.max()) + 1, 1 + cfg.n_ctx) if cfg.eot_truncate else L
        self.eot_rows = torch.empty(len(texts), device=dev, dtype=torch.int32)
        self.token_suffix_run = self.token_suffix
        self._refresh_text_run(eot)

    def _refresh_text_run(self, eot: np.ndarray):
        """EOT gather rows and the suffix rows the text tower runs on (all 77 tokens, or the first
        text_len under eot_truncate; the assemble kernel reads a contiguous [K, text_len-1-n_ctx, D])."""
        Lt, n_ctx = self.text_len, self.cfg.n_ctx
        if int(eot.max()) >= Lt:
            raise ValueError(f"EOT at token {int(eot.max())} beyond the {Lt} tokens the text tower runs on")
        self.eot_rows.copy_(torch.from_numpy((np.arange(len(eot)) * Lt + eot).astype(np.int32)))
        if Lt != self.cfg.dims.context_length:
            run = self.token_suffix[:, :Lt - 1 - n_ctx].contiguous()
            if self.token_suffix_run is self.token_suffix or self.token_suffix_run.shape != run.shape:
                self.token_suffix_run = run
            else:
                self.token_suffix_run.copy_(run)

    def set_text_prompts(self, token_prefix: torch.Tensor, token_suffix: torch.Tensor, tokenized: torch.Tensor):
        """Use real tokenizer output (prefix/suffix embeddings as the reference registers them)."""
        self.token_prefix.copy_(token_prefix)
        self.token_suffix.copy_(token_suffix)
        self._refresh_text_run(tokenized.argmax(dim=-1).cpu().numpy())

    # ------------------------------------------------------------------ activations / io
    def _build_io(self):
        dev, B, K = self.device, self.B, self.K
        d = self.cfg.dims
        dv, dt, E = d.vision_width, d.text_width, d.embed_dim
        J = self.J
        e = lambda *s, dt_=F16: torch.empty(*s, device=dev, dtype=dt_)
        self.img_in = e(B, 3, d.image_resolution, d.image_resolution, dt_=F32)
        self.label_in = torch.zeros(B, device=dev, dtype=torch.int64)
        # soft (float) labels [B, K] select the KL branch of the loss (trainers/maple.py:356-360)
        self.soft_label_in = torch.zeros(B, K, device=dev, dtype=F32)
        self.soft_labels = False
        self.input_flag = torch.zeros(1, device=dev, dtype=torch.int32)
        self.im2col = e(B * self.G2, 3 * d.vision_patch ** 2)
        self.patch = e(B * self.G2, dv)
        self.Xpre = e(B * self.Lv, dv)
        self.pre_mean, self.pre_rstd = e(B * self.Lv, dt_=F32), e(B * self.Lv, dt_=F32)
        self.shared_ctx = e(N_CTX, dv)
        # deep prompts (trainers/maple.py:194-215): the tower that owns a prompt parameter reads (and
        # writes the gradient of) the parameter tensor itself; the other tower gets its projection
        self.vis_deep, self.txt_deep, self.g_vis_deep, self.g_txt_deep = [], [], [], []
        pl = "prompt_learner."
        for i in range(J - 1):
            if i % 2 == 0:
                name = pl + f"compound_prompts_text_parameters.{i // 2}"
                self.txt_deep.append(self.P[name])
                self.g_txt_deep.append(self.G[name])
                self.vis_deep.append(e(N_CTX, dv, dt_=F32))
                self.g_vis_deep.append(e(N_CTX, dv, dt_=F32))
            else:
                name = pl + f"visual_deep_prompts_parameters.{(i - 1) // 2}"
                self.vis_deep.append(self.P[name])
                self.g_vis_deep.append(self.G[name])
                self.txt_deep.append(e(N_CTX, dt, dt_=F32))
                self.g_txt_deep.append(e(N_CTX, dt, dt_=F32))
        self.g_shared_ctx = e(N_CTX, dv)
        self.vis_post = e(B, dv)
        self.post_mean, self.post_rstd = e(B, dt_=F32), e(B, dt_=F32)
        Lo = self.vis.L_out
        self.cls_rows = torch.arange(0, B * Lo, Lo, dtype=torch.int32, device=dev)
        if self.cfg.captions:  # caption path inputs (set_captions) and its projected rows
            self.cap_tokens = torch.zeros(B, d.context_length, device=dev, dtype=torch.int32)
            self.cap_w = torch.zeros(dt, device=dev, dtype=F16)
            self.cap_W = torch.zeros(dv, dt, device=dev, dtype=F16)
            self.cap_b = torch.zeros(dv, device=dev, dtype=F16)
            self.cap_pooled = e(B, dt)
            self.cap_rows = e(B, dv)
        self.img_feat = e(B, E)
        self.txt_final = e(K, dt)
        self.fin_mean, self.fin_rstd = e(K, dt_=F32), e(K, dt_=F32)
        self.txt_feat = e(K, E)
        self.img_n, self.txt_n = e(B, E), e(K, E)
        self.norms = e(B + K, dt_=F32)
        self.mm, self.logits, self.dmm = e(B, K), e(B, K), e(B, K)
        self.cos_ws = e(2 * B, dt_=F32)
        self.soft_ws = e(2 * B * E)
        self.loss_out = torch.zeros(4, device=dev, dtype=F32)
        self.dimg_n, self.dtxt_n = e(B, E), e(K, E)
        self.dimg, self.dtxt = e(B, E), e(K, E)
        self.d_vis_post, self.d_txt_final = e(B, dv), e(K, dt)
        self.dXpre = e(B * self.Lv, dv)
        # the prompt learner's Linears (proj_lang_to_vis on ctx + the J-1 compound projections), one
        # launch per direction (trainers/maple.py:111-131, 194-215)
        P, G = self.P, self.G
        ents = [dict(X=P[pl + "ctx"], W=P[pl + "proj_lang_to_vis.weight"], b=P[pl + "proj_lang_to_vis.bias"],
                     Y=self.shared_ctx, dY=self.g_shared_ctx, dX=G[pl + "ctx"], acc_dx=True,
                     dW=G[pl + "proj_lang_to_vis.weight"], db=G[pl + "proj_lang_to_vis.bias"])]
        for i in range(J - 1):
            name = (pl + f"compound_prompts_text_parameters.{i // 2}" if i % 2 == 0
                    else pl + f"visual_deep_prompts_parameters.{(i - 1) // 2}")
            y, dy = (self.vis_deep[i], self.g_vis_deep[i]) if i % 2 == 0 else (self.txt_deep[i], self.g_txt_deep[i])
            ents.append(dict(X=P[name], W=P[pl + f"compound_prompt_projections.{i}.weight"],
                             b=P[pl + f"compound_prompt_projections.{i}.bias"], Y=y, dY=dy, dX=G[name], acc_dx=True,
                             dW=G[pl + f"compound_prompt_projections.{i}.weight"],
                             db=G[pl + f"compound_prompt_projections.{i}.bias"]))
        self.pl_linears = ops.SmallLinearBatch(dev, ents)


    def set_captions(self, tokens, weights):
        """The caption path's per-batch inputs: tokens [B, T] (clip.tokenize of the batch's captions) and the
        random (w [512], W [768, 512], b [768]) fp16 the reference draws in that forward
        (captions.draw_caption_weights).  Copied into static buffers (graph-capturable)."""
        if not self.cfg.captions:
            raise RuntimeError("engine built without the caption path (EngineConfig.captions)")
        tok = torch.as_tensor(tokens)
        if tuple(tok.shape) != tuple(self.cap_tokens.shape):
            raise ValueError(f"caption tokens {tuple(tok.shape)}; expected {tuple(self.cap_tokens.shape)}")
        # mf_caption_pool gathers table rows by id on the device: range-check on the host first (token tensors
        # passed directly, trainers/maple.py:310-311, bypass the tokenizer)
        _check_ids(tok.cpu().numpy(), self.cfg.dims.vocab_size)
        self.cap_tokens.copy_(tok.to(torch.int32), non_blocking=True)
        w, W, b = weights
        self.cap_w.copy_(w, non_blocking=True)
        self.cap_W.copy_(W, non_blocking=True)
        self.cap_b.copy_(b, non_blocking=True)

    def load_batch(self, images: torch.Tensor, labels: Optional[torch.Tensor] = None):
        """Copy a batch into the static input buffers (H2D when given host tensors)."""
        self.img_in.copy_(images, non_blocking=True)
        if labels is not None:
            self.set_labels(labels)

    def set_labels(self, labels: torch.Tensor):
        """Integer labels [B] -> cross-entropy; float labels [B, K] (soft targets) -> the KL-divergence
        branch (trainers/maple.py:356-363: `label.dtype == torch.float`).  Switching branch changes the
        launched kernels, so a captured step is per branch (trainers.MapleTrainer keeps one per branch)."""
        if labels.is_floating_point():
            if labels.dtype != F32:
                raise TypeError(f"soft labels must be float32 (the reference tests label.dtype == torch.float), "
                                f"got {labels.dtype}")
            if tuple(labels.shape) != (self.B, self.K):
                raise ValueError(f"soft labels of shape {tuple(labels.shape)}; expected ({self.B}, {self.K})")
            self.soft_label_in.copy_(labels, non_blocking=True)
            self.soft_labels = True
        else:
            self.label_in.copy_(labels, non_blocking=True)
            self.soft_labels = False

    # ------------------------------------------------------------------ prompt learner
    def _prompt_learner_fwd(self):
        """MultiModalPromptLearner.forward (trainers/maple.py:177-218): shared_ctx = proj_lang_to_vis(ctx)
        and the J-1 compound projections, in one batched launch."""
        self.pl_linears.fwd()

    def _prompt_learner_bwd(self):
        """Their backward in one dX launch + one dW/db launch.  Each parameter's gradient already holds
        the tower's gradient of its direct use (text ctx / deep prompts); the projection path adds to
        it, as autograd accumulates the two uses (fp16 ctx: the new term rounded once, then added)."""
        self.pl_linears.bwd()

    # ------------------------------------------------------------------ forward
    def _text_forward(self):
        with ops.probe_tag("text"):
            self._text_forward_ops()

    def _text_forward_ops(self):
        P = self.P
        t = self.txt
        ops.text_assemble(self.token_prefix, P["prompt_learner.ctx"], self.token_suffix_run,
                          P["text_encoder.positional_embedding"], t.X[0], self.K, t.L, N_CTX, t.D)
        t.forward(self.txt_deep)
        ops.layernorm_fwd(t.X[-1], P["text_encoder.ln_final.weight"], P["text_encoder.ln_final.bias"], self.txt_final,
                          self.fin_mean, self.fin_rstd, row_index=self.eot_rows)
        ops.gemm(self.txt_final, P["text_encoder.text_projection"], self.txt_feat, epilogue=ops.EPI_NONE,
                 b_kmajor=True)

    def _vision_forward(self):
        with ops.probe_tag("vision"):
            self._vision_forward_ops()

    def _vision_forward_ops(self):
        P = self.P
        v = self.vis
        ops.im2col_patch(self.img_in, self.im2col, self.cfg.dims.vision_patch)
        ops.gemm_nt(self.im2col, self.conv_w, self.patch, epilogue=ops.EPI_NONE)
        ops.vision_assemble(self.patch, P["image_encoder.class_embedding"], P["image_encoder.positional_embedding"],
                            self.shared_ctx, self.Xpre, self.B, self.G2, N_CTX, v.D)
        ops.layernorm_fwd(self.Xpre, P["image_encoder.ln_pre.weight"], P["image_encoder.ln_pre.bias"], v.X[0],
                          self.pre_mean, self.pre_rstd)
        cap = None
        if self.cfg.captions:  # AttentionPooling + Linear(512, 768) of the batch's captions (clip/model.py:550-557)
            ops.caption_pool(self.cap_tokens, self.token_embedding_table(), self.cap_w, self.cap_pooled)
            ops.gemm_nt(self.cap_pooled, self.cap_W, self.cap_rows, bias=self.cap_b, epilogue=ops.EPI_BIAS)
            cap = self.cap_rows
        v.forward(self.vis_deep, cap)
        ops.layernorm_fwd(v.X[-1], P["image_encoder.ln_post.weight"], P["image_encoder.ln_post.bias"], self.vis_post,
                          self.post_mean, self.post_rstd, row_index=self.cls_rows)
        ops.gemm(self.vis_post, P["image_encoder.proj"], self.img_feat, epilogue=ops.EPI_NONE, b_kmajor=True)

    def eval_batch(self, labels: Optional[torch.Tensor], acc: torch.Tensor, pred: Optional[torch.Tensor] = None,
                   reuse_text: bool = False):
        """One test batch (trainers/maple.py:671-677): logits, argmax, correct count accumulated in
        acc (device float[2]: correct, total).  Images must already be in img_in.  reuse_text: see
        forward()."""
        logits = self.forward(reuse_text=reuse_text)
        ops.argmax_correct(logits, labels, pred, acc)
        return logits

    def forward(self, reuse_text: bool = False):
        """CustomCLIP.forward up to the logits (eval path, trainers/maple.py:304-346).  The text and
        vision towers are independent until the head: the text tower runs on a side stream, forked
        from and joined back into the current stream (also inside a captured hipGraph), so its
        smaller kernels fill the CUs the vision GEMMs leave idle.

        reuse_text=True keeps the text features of the previous forward: the
        reference re-encodes every class prompt for every test batch (trainers/maple.py:329 under
        test(), :660-681), although they depend on the weights only.  Within a test pass the weights
        are fixed and the text tower is deterministic, so the cached features are bit-identical to
        recomputed ones; the caller must not set it after a weight change."""
        self._prompt_learner_fwd()
        main = torch.cuda.current_stream(self.device)
        side = self.side if (self.overlap_towers and not reuse_text) else main
        if not reuse_text:
            side.wait_stream(main)
        if self.vision_first:
            self._vision_forward()
        if not reuse_text:
            with torch.cuda.stream(side):
                self._text_forward()
        if not self.vision_first:
            self._vision_forward()
        if not reuse_text:
            main.wait_stream(side)
        ops.clip_head_fwd(self.img_feat, self.txt_feat, self.P["logit_scale"], self.img_n, self.txt_n, self.norms,
                          self.mm, self.logits)
        return self.logits

    # ------------------------------------------------------------------ backward
    def _text_backward(self):
        with ops.probe_tag("text"):
            self._text_backward_ops()

    def _text_backward_ops(self):
        P, G = self.P, self.G
        t = self.txt
        ops.gemm_nt(self.dtxt, P["text_encoder.text_projection"], self.d_txt_final, epilogue=ops.EPI_NONE)
        t.dX.zero_()
        t.lnb.bwd(self.d_txt_final, t.X[-1], P["text_encoder.ln_final.weight"], self.fin_mean, self.fin_rstd,
                     t.dX, G["text_encoder.ln_final.weight"], G["text_encoder.ln_final.bias"],
                          row_index=self.eot_rows)
        t.backward(self.J - 1, self.g_txt_deep)
        # d ctx (text path): sum over classes of the rows 1..n_ctx of d prompts (fp16 result)
        ops.prompt_inject_bwd(t.dX, self.K, t.L, 1, N_CTX, t.D, self.G["prompt_learner.ctx"], accumulate=False,
                              zero_rows=False)
        t.lnb.finish()  # the text LayerNorms' dgamma/dbeta, on the text stream (overlaps the vision backward)

    def _vision_backward(self):
        with ops.probe_tag("vision"):
            self._vision_backward_ops()

    def _vision_backward_ops(self):
        P, G = self.P, self.G
        v = self.vis
        ops.gemm_nt(self.dimg, P["image_encoder.proj"], self.d_vis_post, epilogue=ops.EPI_NONE)
        v.dX.zero_()
        v.lnb.bwd(self.d_vis_post, v.X[-1], P["image_encoder.ln_post.weight"], self.post_mean,
                          self.post_rstd, v.dX, G["image_encoder.ln_post.weight"], G["image_encoder.ln_post.bias"],
                     row_index=self.cls_rows)
        v.backward(self.J - 1, self.g_vis_deep)
        v.lnb.bwd(v.dX[:v.Rs[0]], self.Xpre, P["image_encoder.ln_pre.weight"], self.pre_mean, self.pre_rstd,
                  self.dXpre, G["image_encoder.ln_pre.weight"], G["image_encoder.ln_pre.bias"])
        ops.prompt_inject_bwd(self.dXpre, self.B, self.Lv, self.G2 + 1, N_CTX, v.D, self.g_shared_ctx,
                              accumulate=False, zero_rows=False)
        v.lnb.finish()

    def forward_loss(self):
        """loss = CustomCLIP(image, label) (trainers/maple.py:304-381): the forward, the loss, and d loss /
        d features (the fused loss kernel).  The trainable block's W^T copies (read by its dX products in
        backward()) are refreshed from the current weights first, on the side stream, where they overlap
        the vision forward."""
        # check_tensor_validity of the inputs (trainers/maple.py:556-557) on the device: a NaN/Inf image (or
        # soft label) sets input_flag and halts the update like a non-finite loss; the trainer raises
        # ValueError for it at the end of the epoch
        self.input_flag.zero_()
        ops.nonfinite_flag(self.img_in, self.input_flag)
        if self.soft_labels:
            ops.nonfinite_flag(self.soft_label_in, self.input_flag)
        # (mf_optimizer_step latches the input flag into hyper[4] at the step's end)
        main = torch.cuda.current_stream(self.device)
        side = self.side if self.overlap_towers else main
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.refresh_transposes(all_layers=False)
        self.forward()  # joins the side stream before returning
        if self.soft_labels:
            ops.clip_loss_soft_fwd_bwd(self.img_feat, self.txt_feat, self.img_n, self.txt_n, self.norms,
                                       self.logits, self.soft_label_in, self.P["logit_scale"], self.dmm, self.cos_ws,
                                       self.soft_ws, self.loss_out, self.dimg_n, self.dtxt_n, self.dimg, self.dtxt)
        else:
            ops.clip_loss_fwd_bwd(self.img_feat, self.txt_feat, self.img_n, self.txt_n, self.norms, self.logits,
                                  self.label_in, self.P["logit_scale"], self.dmm, self.cos_ws, self.loss_out,
                                  self.dimg_n, self.dtxt_n, self.dimg, self.dtxt)

    def backward(self):
        """loss.backward() after forward_loss(): every trainable gradient lands in gflat16 / gflat32."""
        main = torch.cuda.current_stream(self.device)
        side = self.side if self.overlap_towers else main
        side.wait_stream(main)
        if self.vision_first:
            self._vision_backward()
        with torch.cuda.stream(side):
            self._text_backward()
        if not self.vision_first:
            self._vision_backward()
        main.wait_stream(side)
        self._prompt_learner_bwd()

    def forward_backward(self):
        """loss = CustomCLIP(image, label); loss.backward()  — grads land in gflat16/gflat32."""
        self.forward_loss()
        self.backward()

    # ------------------------------------------------------------------ optimizer
    def set_lr(self, lr: float):
        self.hyper[0] = lr

    def reset_momentum(self):
        """broadcast_weights deletes the SGD state (trainers/maple_fed.py:331-335)."""
        self.hyper[3] = 1.0

    def optimizer_step(self):
        """clip_grad_norm_(1.0) + SGD.step (trainers/maple.py:592-598), all on device.

        A non-finite loss latches hyper[4] (halt): the reference raises RuntimeError("NaN/Inf in total
        loss") at that step before its backward (trainers/maple.py:375-376), so neither that step nor any
        later one of the epoch updates the weights; the SGD kernels skip while halt is set.  The trainer
        clears it at the start of an epoch and reports the failure (MaPLe.run_epoch)."""
        # the halt latch, clip coefficient and both flat buffers' SGD in three launches (mf_optimizer_step)
        ops.optimizer_step(self.flat16, self.gflat16, self.mom16, self.flat32, self.gflat32, self.mom32, self.chunks,
                           self.nchunks, self.cfg.max_grad_norm, self.norm_part, self.clip_out, self.hyper,
                           self.loss_out[3:4], self.input_flag)
        # the momentum buffers now exist (first_step -> 0) unless the update was skipped
        self.hyper[3:4].mul_(self.hyper[4:5])  # device ops, legal inside graph capture

    def clear_halt(self):
        self.hyper[4:5].zero_()

    def train_step(self):
        self.forward_backward()
        self.optimizer_step()
        self.step_count += 1

    def after_weights_loaded(self):
        """broadcast_weights (trainers/maple_fed.py:327-339): new weights, SGD momentum dropped."""
        self.refresh_transposes(all_layers=False)
        self.reset_momentum()

    def capture_train_step(self, pool=None) -> "torch.cuda.CUDAGraph":
        """Capture forward + backward + clip + SGD as one hipGraph (static buffers, no host syncs).
        Replaying it is exactly train_step(); the LR / first-step flag are read from device memory."""
        first = self.hyper[3].item()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            self.forward_backward()
            self.optimizer_step()
        self.hyper[3] = first  # capture does not execute the step
        return g

    # ------------------------------------------------------------------ state
    def loss(self) -> float:
        v = self.loss_out.cpu()
        if v[3].item() != 0.0:
            raise RuntimeError("NaN/Inf in total loss")
        return float(v[0])

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """CustomCLIP parameter names -> device tensors (the reference's model.state_dict() minus the
        clip_model2.* aliases and buffers, see reference_state_dict)."""
        return {n: t for n, t in self.P.items()}

    def token_embedding_table(self) -> torch.Tensor:
        """CLIP's token-embedding table [vocab, 512] fp32 on the device (clip/model.py:642; frozen): the
        checkpoint's, or the seeded synthetic one (the values the prompt rows were taken from)."""
        o = self._table_owner
        if o._token_table is None:
            d = o.cfg.dims
            tab = syn.fp16_round(0.02 * syn.normal(o.cfg.seed, "token_embedding.weight", d.vocab_size * d.text_width))
            o._token_table = torch.from_numpy(tab.reshape(d.vocab_size, d.text_width))
        if o._token_table.device != o.device:
            o._token_table = o._token_table.to(o.device)
        return o._token_table

    @staticmethod
    def alias_of(name: str) -> Optional[str]:
        """The clip_model2.* alias of a tower parameter (CustomCLIP keeps clip_model as clip_model2 and
        its visual / text modules as image_encoder / text_encoder, trainers/maple.py:221-229)."""
        if name.startswith("image_encoder."):
            return "clip_model2.visual." + name[len("image_encoder."):]
        if name.startswith("text_encoder."):
            return "clip_model2." + name[len("text_encoder."):]
        return None

    def reference_state_dict(self) -> Dict[str, torch.Tensor]:
        """The reference's full CustomCLIP state-dict key set (trainers/maple.py:221-229): parameters,
        the prompt learner's token_prefix/suffix buffers and the clip_model2.* aliases of the CLIP
        modules (616 keys at J=3, 634 at J=9; tests/golden/state_dict_keys.json)."""
        out = dict(self.state_dict())
        out["prompt_learner.token_prefix"] = self.token_prefix
        out["prompt_learner.token_suffix"] = self.token_suffix
        for n, t in self.P.items():
            a = self.alias_of(n)
            if a is not None:
                out[a] = t
        out["clip_model2.logit_scale"] = self.clip_logit_scale
        out["clip_model2.token_embedding.weight"] = self.token_embedding_table()
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        """load_state_dict of the reference model (trainers/maple_fed.py:329): with strict, every key of
        reference_state_dict() must be present and no other; values are cast to each tensor's dtype.  A
        tower parameter absent under its own name is taken from its clip_model2.* alias."""
        own = set(self.reference_state_dict()) if strict else None
        if strict:
            missing = sorted(own - set(sd))
            unexpected = sorted(set(sd) - own)
            if missing or unexpected:
                raise RuntimeError(f"Error(s) in loading state_dict: missing keys {missing[:5]} "
                                   f"({len(missing)}), unexpected keys {unexpected[:5]} ({len(unexpected)})")
        frozen_changed = False
        with torch.no_grad():
            for n, t in self.P.items():
                src = sd.get(n)
                if src is None and self.alias_of(n) is not None:
                    src = sd.get(self.alias_of(n))
                if src is not None:
                    t.copy_(torch.as_tensor(src).reshape(t.shape).to(device=t.device, dtype=t.dtype))
                    frozen_changed |= n not in self.trainable_names
            if "clip_model2.logit_scale" in sd:
                self.clip_logit_scale.copy_(torch.as_tensor(sd["clip_model2.logit_scale"]).float())
            if "clip_model2.token_embedding.weight" in sd:
                self.token_embedding_table().copy_(torch.as_tensor(sd["clip_model2.token_embedding.weight"]).float())
            if "prompt_learner.token_prefix" in sd:
                self.token_prefix.copy_(sd["prompt_learner.token_prefix"])
                self.token_suffix.copy_(sd["prompt_learner.token_suffix"])
                self._refresh_text_run(self.tokenized.argmax(dim=-1).numpy())
        self.refresh_transposes(all_layers=frozen_changed)

    def trainable_state(self) -> Dict[str, torch.Tensor]:
        return {n: self.P[n] for n in self.trainable_names}

    def grads(self) -> Dict[str, torch.Tensor]:
        return {n: self.G[n] for n in self.trainable_names}
