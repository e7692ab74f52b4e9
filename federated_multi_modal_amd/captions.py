"""Caption-conditioned visual prompts (§8(f) rank 4).

Reference (clip/model.py:457-476, 550-561; trainers/maple.py:307-322): when a batch carries captions (a list
of strings -- the Dassl caption fork's loaders always do, empty strings included), CustomCLIP tokenizes
them, embeds the tokens with CLIP's token embedding (fp16), and the image encoder
  1. builds an AttentionPooling whose weight vector is a FRESH torch.randn(512) (fp16): scores = emb . w,
     p = softmax over the 77 tokens, pooled = sum_t emb_t * p_t                              [B, 512];
  2. builds a FRESH nn.Linear(512, 768) (default init, fp16) and projects the pooled captions  [B, 768];
  3. prepends those B rows to every visual deep prompt: combined_i = cat(projected, deep_vis_i) [B+2, 768].
The block at each prompted layer keeps all but the last n_ctx = 2 rows of its input and appends combined_i
(expanded over the batch), so the vision sequence grows by B rows per prompted layer:
L_i = 199 + i*B for i = 1 .. J-1 (455 at J = 9, B = 32).  No gradient reaches the random weights (they
are not parameters); the caption rows act as extra keys / values for every image of the batch.

Here the random tensors are drawn by `draw_caption_weights` from a torch.Generator in exactly the
reference's order and with its init formulas, so seeding the generator the way the reference's global
generator is seeded reproduces the reference's weights bit for bit; the trainer gives each client its own
seeded generator (the reference's draws depend on every earlier use of the global generator)."""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np
import torch

from . import synthetic as syn


def draw_caption_weights(gen: torch.Generator, text_width: int = 512,
                         vision_width: int = 768) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(w [512], W [768, 512], b [768]) fp16 on the host: AttentionPooling's torch.randn(512) (clip/model.py:461),
    then nn.Linear(512, 768).reset_parameters (kaiming_uniform_(a=sqrt(5)) weight, uniform(+-1/sqrt(512))
    bias; clip/model.py:557), in that order from `gen`."""
    w = torch.randn(text_width, generator=gen)
    W = torch.empty(vision_width, text_width)
    torch.nn.init.kaiming_uniform_(W, a=math.sqrt(5), generator=gen)
    b = torch.empty(vision_width)
    bound = 1.0 / math.sqrt(text_width)
    torch.nn.init.uniform_(b, -bound, bound, generator=gen)
    return w.half(), W.half(), b.half()


def caption_tokens(captions: List[str], context_length: int = syn.CONTEXT_LENGTH, tokenizer=None) -> np.ndarray:
    """clip.tokenize(caption) (trainers/maple.py:309-311): int64 [B, context_length] with the given tokenizer
    (tokenizer.get_tokenizer: CLIP's BPE, or the synthetic stand-in when None); a caption longer than the
    context raises RuntimeError as clip.tokenize does (no truncation)."""
    from .tokenizer import get_tokenizer
    tok = tokenizer if tokenizer is not None else get_tokenizer("")
    return tok.tokenize(list(captions), context_length)


def has_captions(caption) -> bool:
    """trainers/maple.py:307-322: a list of strings (or of token tensors) turns the caption path on."""
    if caption is None or not isinstance(caption, (list, tuple)) or len(caption) == 0:
        return False
    return all(isinstance(c, str) for c in caption) or all(isinstance(c, torch.Tensor) for c in caption)


def vision_lengths(grid2: int, n_ctx: int, layers: int, n_prompted: int, ncap: int) -> List[int]:
    """Sequence length of every vision block's input: 197 + n_ctx at layer 0, + ncap per prompted layer."""
    L0 = grid2 + 1 + n_ctx
    return [L0 + min(i, n_prompted) * ncap for i in range(layers)]
