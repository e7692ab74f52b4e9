"""The reference's module API over the MI355X kernels.

    model = CustomCLIP(engine)                      # trainers/maple.py:220-381
    loss = model(image, label)                      # train mode: 0-dim fp16 loss with a grad_fn
    optim.zero_grad(); loss.backward()              # the engine's explicit backward (libmapfed.so)
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0); optim.step()
    logits = model.eval()(image)                    # [B, K] fp16
    model.image_encoder(x, shared_ctx, deep_vis)    # clip/model.py:509-572
    model.text_encoder(prompts, tokenized, deep_txt)  # trainers/maple.py:52-79
    model.image_encoder.transformer.resblocks[i]([x, deep, counter])  # clip/model.py:307-352
    model.prompt_learner()                          # trainers/maple.py:177-218

Every parameter is an nn.Parameter that shares the engine's device memory, registered under the
reference's names and in the reference's order (state_dict() equals CustomCLIP.state_dict(): 616 keys
at J=3, 634 at J=9, clip_model2.* aliases included; named_parameters() in the reference's order, so a
torch optimizer / clip_grad_norm_ over model.parameters() sees the reference's parameter list).
Updating them in place (torch.optim.SGD) updates the engine.

CustomCLIP.forward in train mode is a torch.autograd.Function over the whole client step: its forward
is MapleEngine.forward_loss (both towers + the fused loss kernel), its backward MapleEngine.backward
(the hand-written backward) -- the gradient of every trainable parameter is returned to
autograd, which stores it in p.grad.  Eval mode returns the logits of MapleEngine.forward.

The tower / block / prompt-learner callables compose the same kernels (ops.*) on buffers they allocate,
for any batch / class count; with the engine's shapes they give the engine's values bit for bit.
Gradients flow through CustomCLIP.forward only (the towers are frozen except LayerNorms and block 11,
and the reference trains through CustomCLIP.forward as well, trainers/maple.py:588-590)."""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import ops
from .captions import caption_tokens, draw_caption_weights, has_captions
from .engine import MapleEngine, N_CTX, _is_trainable

F16, F32 = torch.float16, torch.float32


class _Holder(nn.Module):
    """A parameter container (nn.Linear / LayerNorm / Conv2d / Embedding stand-in: weight [, bias])."""


def _param(engine: MapleEngine, name: str, cache: Dict[int, nn.Parameter]) -> nn.Parameter:
    t = engine.P[name]
    key = id(t)
    if key not in cache:
        cache[key] = nn.Parameter(t, requires_grad=_is_trainable(name))
    return cache[key]


class ResidualAttentionBlock(nn.Module):
    """ResidualAttentionBlock_MaPLe (clip/model.py:269-352) on the HIP kernels.  forward([x, deep, counter])
    with x [L, N, D] fp16 (LND) returns [x', deep, counter'] like the reference, including the deep-prompt
    replacement at layers > 0 (vision: the last n_ctx rows; text: rows 1..n_ctx)."""

    def __init__(self, engine: MapleEngine, tower: str, index: int, D: int, H: int, causal: bool, cache):
        super().__init__()
        self.tower, self.i, self.D, self.H, self.causal = tower, index, D, H, causal
        self.text_layer = tower == "text_encoder"
        pre = f"{tower}.transformer.resblocks.{index}."
        self.attn = _Holder()
        self.attn.in_proj_weight = _param(engine, pre + "attn.in_proj_weight", cache)
        self.attn.in_proj_bias = _param(engine, pre + "attn.in_proj_bias", cache)
        self.attn.out_proj = _Holder()
        self.attn.out_proj.weight = _param(engine, pre + "attn.out_proj.weight", cache)
        self.attn.out_proj.bias = _param(engine, pre + "attn.out_proj.bias", cache)
        self.ln_1 = _Holder()
        self.ln_1.weight = _param(engine, pre + "ln_1.weight", cache)
        self.ln_1.bias = _param(engine, pre + "ln_1.bias", cache)
        self.mlp = _Holder()
        self.mlp.c_fc = _Holder()
        self.mlp.c_fc.weight = _param(engine, pre + "mlp.c_fc.weight", cache)
        self.mlp.c_fc.bias = _param(engine, pre + "mlp.c_fc.bias", cache)
        self.mlp.c_proj = _Holder()
        self.mlp.c_proj.weight = _param(engine, pre + "mlp.c_proj.weight", cache)
        self.mlp.c_proj.bias = _param(engine, pre + "mlp.c_proj.bias", cache)
        self.ln_2 = _Holder()
        self.ln_2.weight = _param(engine, pre + "ln_2.weight", cache)
        self.ln_2.bias = _param(engine, pre + "ln_2.bias", cache)

    @torch.no_grad()
    def rows(self, x: torch.Tensor, N: int, L: int, prompt: Optional[torch.Tensor]) -> torch.Tensor:
        """The block on NLD rows x [N*L, D] (modified in place by the prompt replacement); returns the
        output rows.  Same kernel sequence as the engine's _Tower.forward."""
        if prompt is not None:
            row0 = 1 if self.text_layer else L - N_CTX
            ops.prompt_inject_fwd(x, prompt.float().contiguous(), N, L, row0, N_CTX, self.D)
        h1, _, _ = ops.layernorm_fwd(x, self.ln_1.weight, self.ln_1.bias)
        qkv = ops.gemm_nt(h1, self.attn.in_proj_weight, bias=self.attn.in_proj_bias, epilogue=ops.EPI_BIAS)
        o, _ = ops.attention_fwd(qkv, N, L, self.H, self.causal)
        x1 = ops.gemm_nt(o, self.attn.out_proj.weight, bias=self.attn.out_proj.bias, aux_in=x,
                         epilogue=ops.EPI_BIAS_RESID)
        h2, _, _ = ops.layernorm_fwd(x1, self.ln_2.weight, self.ln_2.bias)
        pre = torch.empty(x.shape[0], 4 * self.D, device=x.device, dtype=F16)
        g = ops.gemm_nt(h2, self.mlp.c_fc.weight, bias=self.mlp.c_fc.bias, aux_out=pre, epilogue=ops.EPI_BIAS_GELU)
        return ops.gemm_nt(g, self.mlp.c_proj.weight, bias=self.mlp.c_proj.bias, aux_in=x1,
                           epilogue=ops.EPI_BIAS_RESID)

    def forward(self, inputs):
        x, deep, counter = inputs[0], inputs[1], inputs[2]
        L, N, D = x.shape
        rows = x.detach().to(F16).permute(1, 0, 2).contiguous().view(N * L, D)
        prompt = None
        if self.i > 0 and len(deep) > 0 and not counter > len(deep) - 1:
            prompt = deep[counter]
            counter += 1
        out = self.rows(rows, N, L, prompt)
        return [out.view(N, L, D).permute(1, 0, 2).contiguous(), deep, counter]


class Transformer(nn.Module):
    """clip/model.py:355-380: resblocks (nn.Sequential over [x, deep, counter])."""

    def __init__(self, engine: MapleEngine, tower: str, D: int, H: int, layers: int, causal: bool, cache):
        super().__init__()
        self.width, self.layers = D, layers
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(engine, tower, i, D, H, causal, cache)
                                         for i in range(layers)])

    def forward(self, inputs):
        return self.resblocks(inputs)

    def rows(self, x: torch.Tensor, N: int, L: int, deep: List[torch.Tensor],
             cap: Optional[torch.Tensor] = None):
        """The blocks on NLD rows; returns (rows, final sequence length).  cap [ncap, D] fp16 (the caption
        path's projected rows, clip/model.py:550-561): each prompted block's input keeps all but the last
        n_ctx rows of the previous output and appends cap + the deep prompt, so the sequence grows by ncap."""
        counter = 0
        for i, blk in enumerate(self.resblocks):
            prompt = None
            if i > 0 and len(deep) > 0 and not counter > len(deep) - 1:
                prompt = deep[counter]
                counter += 1
            if prompt is not None and cap is not None:
                grown = torch.empty(N * (L + cap.shape[0]), x.shape[1], device=x.device, dtype=F16)
                ops.seq_grow(x, grown, cap, prompt.float().contiguous(), N, L, cap.shape[0], N_CTX, x.shape[1])
                x, L, prompt = grown, L + cap.shape[0], None
            x = blk.rows(x, N, L, prompt)
        return x, L


class VisionTransformer(nn.Module):
    """VisionTransformer_MaPLe (clip/model.py:478-572)."""

    def __init__(self, engine: MapleEngine, cache):
        super().__init__()
        d = engine.cfg.dims
        self.e = [engine]  # not a submodule
        self.input_resolution, self.output_dim = d.image_resolution, d.embed_dim
        self.patch, self.grid, self.width = d.vision_patch, d.grid, d.vision_width
        ie = "image_encoder."
        self.class_embedding = _param(engine, ie + "class_embedding", cache)
        self.positional_embedding = _param(engine, ie + "positional_embedding", cache)
        self.proj = _param(engine, ie + "proj", cache)
        self.conv1 = _Holder()
        self.conv1.weight = _param(engine, ie + "conv1.weight", cache)
        self.ln_pre = _Holder()
        self.ln_pre.weight = _param(engine, ie + "ln_pre.weight", cache)
        self.ln_pre.bias = _param(engine, ie + "ln_pre.bias", cache)
        self.transformer = Transformer(engine, "image_encoder", d.vision_width, d.vision_heads, d.vision_layers, False,
                                       cache)
        self.ln_post = _Holder()
        self.ln_post.weight = _param(engine, ie + "ln_post.weight", cache)
        self.ln_post.bias = _param(engine, ie + "ln_post.bias", cache)
        self.caption_generator: Optional[torch.Generator] = None  # None: torch's global generator

    def caption_rows(self, clip_embeddings: torch.Tensor) -> torch.Tensor:
        """clip/model.py:550-558: AttentionPooling with a fresh random vector, then a fresh random
        Linear(512, 768), both fp16 and drawn (in the reference's order) from the generator CustomCLIP names
        (torch's global one by default): [ncap, 77, 512] token embeddings -> [ncap, 768]."""
        emb = clip_embeddings.to(device=self.conv1.weight.device, dtype=F16).contiguous()
        ncap, T, Dt = emb.shape
        gen = self.caption_generator if self.caption_generator is not None else torch.default_generator
        w, W, b = draw_caption_weights(gen, Dt, self.width)
        dev = emb.device
        pooled = torch.empty(ncap, Dt, device=dev, dtype=F16)
        # the pooling kernel gathers rows by token id: here every caption's own rows, in order
        ids = torch.arange(ncap * T, device=dev, dtype=torch.int32).view(ncap, T)
        ops.caption_pool(ids, emb.view(ncap * T, Dt).float(), w.to(dev), pooled)
        return ops.gemm_nt(pooled, W.to(dev), bias=b.to(dev), epilogue=ops.EPI_BIAS)

    @torch.no_grad()
    def forward(self, x: torch.Tensor, shared_ctx: torch.Tensor, compound_deeper_prompts, clip_embeddings=None):
        """clip/model.py:509-572.  clip_embeddings [ncap, 77, 512] (the caption tokens' embedding): the
        caption-conditioned visual prompts, each prompted block's sequence growing by ncap rows."""
        cap = self.caption_rows(clip_embeddings) if clip_embeddings is not None else None
        B = x.shape[0]
        G2, D, p = self.grid * self.grid, self.width, self.patch
        L = G2 + 1 + N_CTX
        img = x.contiguous()
        if img.dtype not in (F16, F32):
            img = img.float()
        cols = torch.empty(B * G2, 3 * p * p, device=img.device, dtype=F16)
        ops.im2col_patch(img, cols, p)
        patch = ops.gemm_nt(cols, self.conv1.weight.view(D, -1), epilogue=ops.EPI_NONE)
        xpre = torch.empty(B * L, D, device=img.device, dtype=F16)
        ops.vision_assemble(patch, self.class_embedding, self.positional_embedding, shared_ctx.to(F16).contiguous(),
                            xpre, B, G2, N_CTX, D)
        h, _, _ = ops.layernorm_fwd(xpre, self.ln_pre.weight, self.ln_pre.bias)
        h, L = self.transformer.rows(h, B, L, list(compound_deeper_prompts), cap)
        cls_rows = torch.arange(0, B * L, L, dtype=torch.int32, device=img.device)
        post, _, _ = ops.layernorm_fwd(h, self.ln_post.weight, self.ln_post.bias, row_index=cls_rows)
        return ops.gemm(post, self.proj, epilogue=ops.EPI_NONE, b_kmajor=True)


class TextEncoder(nn.Module):
    """TextEncoder (trainers/maple.py:43-79)."""

    def __init__(self, engine: MapleEngine, cache):
        super().__init__()
        d = engine.cfg.dims
        te = "text_encoder."
        self.transformer = Transformer(engine, "text_encoder", d.text_width, d.text_heads, d.text_layers, True, cache)
        self.positional_embedding = _param(engine, te + "positional_embedding", cache)
        self.ln_final = _Holder()
        self.ln_final.weight = _param(engine, te + "ln_final.weight", cache)
        self.ln_final.bias = _param(engine, te + "ln_final.bias", cache)
        self.text_projection = _param(engine, te + "text_projection", cache)
        self.dtype = F16

    @torch.no_grad()
    def forward(self, prompts: torch.Tensor, tokenized_prompts: torch.Tensor, compound_prompts_deeper_text):
        K, L, D = prompts.shape
        x = (prompts.to(F16) + self.positional_embedding.to(F16)).contiguous().view(K * L, D)
        x, _ = self.transformer.rows(x, K, L, list(compound_prompts_deeper_text))
        eot = tokenized_prompts.to(x.device).argmax(dim=-1).to(torch.int64)
        rows = (torch.arange(K, device=x.device, dtype=torch.int64) * L + eot).to(torch.int32)
        fin, _, _ = ops.layernorm_fwd(x, self.ln_final.weight, self.ln_final.bias, row_index=rows)
        return ops.gemm(fin, self.text_projection, epilogue=ops.EPI_NONE, b_kmajor=True)


class MultiModalPromptLearner(nn.Module):
    """MultiModalPromptLearner (trainers/maple.py:82-218)."""

    def __init__(self, engine: MapleEngine, cache):
        super().__init__()
        pl = "prompt_learner."
        J = engine.J
        self.e = [engine]
        self.n_cls, self.n_ctx, self.compound_prompts_depth = engine.K, N_CTX, J
        self.ctx = _param(engine, pl + "ctx", cache)
        self.register_buffer("token_prefix", engine.token_prefix)
        self.register_buffer("token_suffix", engine.token_suffix)
        self.proj_lang_to_vis = _Holder()
        self.proj_lang_to_vis.weight = _param(engine, pl + "proj_lang_to_vis.weight", cache)
        self.proj_lang_to_vis.bias = _param(engine, pl + "proj_lang_to_vis.bias", cache)
        self.proj_vis_to_lang = _Holder()
        self.proj_vis_to_lang.weight = _param(engine, pl + "proj_vis_to_lang.weight", cache)
        self.proj_vis_to_lang.bias = _param(engine, pl + "proj_vis_to_lang.bias", cache)
        self.compound_prompts_text_parameters = nn.ParameterList(
            [_param(engine, pl + f"compound_prompts_text_parameters.{k}", cache) for k in range((J - 1 + 1) // 2)])
        self.visual_deep_prompts_parameters = nn.ParameterList(
            [_param(engine, pl + f"visual_deep_prompts_parameters.{k}", cache) for k in range((J - 1) // 2)])
        projs = []
        for i in range(J - 1):
            h = _Holder()
            h.weight = _param(engine, pl + f"compound_prompt_projections.{i}.weight", cache)
            h.bias = _param(engine, pl + f"compound_prompt_projections.{i}.bias", cache)
            projs.append(h)
        self.compound_prompt_projections = nn.ModuleList(projs)
        self.tokenized_prompts = engine.tokenized

    @staticmethod
    def _linear(x, holder):
        y = torch.empty(x.shape[0], holder.weight.shape[0], device=x.device, dtype=x.dtype)
        return ops.small_linear_fwd(x.contiguous(), holder.weight, holder.bias, y)

    @torch.no_grad()
    def forward(self):
        K = self.token_prefix.shape[0]
        ctx = self.ctx.unsqueeze(0).expand(K, -1, -1)
        prompts = torch.cat([self.token_prefix, ctx, self.token_suffix], dim=1)
        text, vis = [], []
        for i, layer in enumerate(self.compound_prompt_projections):
            if i % 2 == 0:
                t = self.compound_prompts_text_parameters[i // 2]
                vis.append(self._linear(t, layer))
                text.append(t)
            else:
                v = self.visual_deep_prompts_parameters[(i - 1) // 2]
                text.append(self._linear(v, layer))
                vis.append(v)
        shared_ctx = self._linear(self.ctx, self.proj_lang_to_vis)
        return prompts, shared_ctx, text, vis


class _CLIP(nn.Module):
    """clip_model2 (trainers/maple.py:229): the CLIP module whose submodules the towers share."""


class _ClientStep(torch.autograd.Function):
    """loss = CustomCLIP(image, label) with the engine's backward as d loss / d trainables."""

    @staticmethod
    def forward(ctx, engine: MapleEngine, *params):
        engine.forward_loss()
        ctx.engine = engine
        return engine.loss_out[0].to(F16)

    @staticmethod
    def backward(ctx, grad_out):
        e = ctx.engine
        if float(grad_out) != 1.0:
            raise NotImplementedError("the engine's backward is d(loss)/d(params) for loss.backward() "
                                      "(gradient 1.0); scale the gradients instead")
        e.backward()
        return (None,) + tuple(e.G[n] for n in e.trainable_names)


class CustomCLIP(nn.Module):
    """CustomCLIP (trainers/maple.py:220-381) over a MapleEngine (which owns every buffer)."""

    def __init__(self, engine: MapleEngine):
        super().__init__()
        cache: Dict[int, nn.Parameter] = {}
        self.engine = [engine]  # plain list: not a submodule
        self.logit_scale = _param(engine, "logit_scale", cache)
        self.prompt_learner = MultiModalPromptLearner(engine, cache)
        self.tokenized_prompts = engine.tokenized
        self.image_encoder = VisionTransformer(engine, cache)
        self.text_encoder = TextEncoder(engine, cache)
        self.dtype = F16
        c = _CLIP()
        c.positional_embedding = self.text_encoder.positional_embedding
        c.text_projection = self.text_encoder.text_projection
        c.logit_scale = nn.Parameter(engine.clip_logit_scale, requires_grad=False)
        c.visual = self.image_encoder
        c.transformer = self.text_encoder.transformer
        c.token_embedding = _Holder()
        c.token_embedding.weight = nn.Parameter(engine.token_embedding_table(), requires_grad=False)
        c.ln_final = self.text_encoder.ln_final
        self.clip_model2 = c
        self._by_name = {n: cache[id(engine.P[n])] for n in engine.trainable_names}
        self._eval: Dict[object, MapleEngine] = {}
        # where the caption path's random AttentionPooling / Linear weights come from: torch's global CPU
        # generator, as in the reference (clip/model.py:461, 557); the federated trainer assigns each client
        # its own seeded generator here, and its training step draws from the same attribute
        self.caption_generator = torch.default_generator

    @property
    def caption_generator(self) -> torch.Generator:
        return self.__dict__["_caption_generator"]

    @caption_generator.setter
    def caption_generator(self, gen: torch.Generator):
        self.__dict__["_caption_generator"] = gen
        if "image_encoder" in self._modules:
            self.image_encoder.caption_generator = gen

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """nn.Module.load_state_dict semantics on the engine (MapleEngine.load_state_dict: strict key check
        against the reference's key set, values cast to each tensor's dtype, aliases accepted), which also
        refreshes what depends on the weights (the W^T copies, the text-token run)."""
        if assign:
            raise NotImplementedError("assign=True: the parameters are views of the engine's buffers")
        e = self.engine[0]
        own = set(self.state_dict())
        missing = sorted(own - set(state_dict)) if strict else []
        unexpected = sorted(set(state_dict) - own) if strict else []
        e.load_state_dict(state_dict, strict=strict)
        from torch.nn.modules.module import _IncompatibleKeys
        return _IncompatibleKeys(missing, unexpected)

    def _engine_for(self, batch: int) -> MapleEngine:
        e = self.engine[0]
        if batch == e.B:
            return e
        if batch not in self._eval:
            self._eval[batch] = MapleEngine(dataclasses.replace(e.cfg, batch=batch), device=e.device, shared=e)
        return self._eval[batch]

    def _caption_engine(self, batch: int, caption) -> MapleEngine:
        """The caption path (trainers/maple.py:307-322 -> clip/model.py:550-561) for a batch: an engine with
        the growing vision sequence (shared parameters), this batch's caption tokens, and the random
        AttentionPooling vector / Linear(512, 768) drawn from self.caption_generator (torch's global CPU
        generator unless the trainer set a per-client one), as the reference draws them in every such forward
        (captions.draw_caption_weights reproduces its draws)."""
        e = self.engine[0]
        key = ("captions", batch)
        if key not in self._eval:
            self._eval[key] = MapleEngine(dataclasses.replace(e.cfg, batch=batch, captions=True), device=e.device,
                                          shared=e)
        ce = self._eval[key]
        if all(isinstance(c, str) for c in caption):
            tok = caption_tokens(list(caption), ce.cfg.dims.context_length, ce.tokenizer)
        else:
            tok = torch.stack([torch.as_tensor(c) for c in caption]).cpu()
        ce.set_captions(tok, draw_caption_weights(self.caption_generator))
        return ce

    def forward(self, image, label=None, caption=None, return_feature=False):
        """trainers/maple.py:304-381: the loss in train mode (label required), the logits [B, K] in eval
        mode.  caption: a list of strings (or token tensors) turns on the caption-conditioned visual prompts
        (clip/model.py:550-561) exactly as in the reference, random weights included (drawn from torch's
        global generator)."""
        if has_captions(caption):
            e = self._caption_engine(image.shape[0], caption)
        else:
            e = self._engine_for(image.shape[0])
        e.img_in.copy_(image)
        if self.training:
            if label is None:
                raise ValueError("train mode needs labels (trainers/maple.py:349-378)")
            if not label.is_floating_point():
                lo, hi = torch.stack([label.min(), label.max()]).tolist()
                assert lo >= 0 and hi < e.K, "Label index out of bounds"
            e.set_labels(label.to(e.device))
            params = [self._by_name[n] for n in e.trainable_names]
            loss = _ClientStep.apply(e, *params)
            if float(e.loss_out[3]) != 0.0:
                raise RuntimeError("NaN/Inf in total loss")
            return loss
        return e.forward().clone()
