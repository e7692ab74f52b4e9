"""Generate the golden fixtures that pin this build to the reference (run in the build container).

    python tests/golden/make_golden.py

Imports the reference's own clip/model.py + trainers/maple.py + trainers/maple_fed.py (read-only,
/root/reference; see ref_harness.py) and runs it on synthetic weights/inputs from
federated_multi_modal_amd.synthetic, which the GPU box regenerates bit-identically.  Writes small
.npz files next to this script:

  c1_maple.npz   config C1 (J=3, K=10, B=4, ViT-B/16, 12+12 layers):
                 eval logits (fp16) + the float64 restatement's logits (the fp16 noise floor),
                 train loss, every trainable gradient (full for small tensors, norm + a fixed
                 sample of 4096 entries for large ones), the same for the float64 restatement,
                 and the parameter deltas of one clip_grad_norm_(1.0) + SGD step (lr 0.0026).
  fedavg.npz     MaPLeFederated.safe_average_weights on 3 synthetic client state dicts
                 (fp16 and fp32 keys, logit_scale), inputs and outputs.

Only data is written (inputs and expected outputs); no reference source is copied.
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parents[1]))

sys.path.insert(0, str(HERE.parent))
import ref_harness as h  # noqa: E402
from _cases import trace_idx  # noqa: E402  (the GPU tests regenerate the same sample positions)
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from oracle import maple_oracle as O  # noqa: E402

SAMPLE = 4096
FULL_MAX = 100_000


def sample_idx(name: str, n: int) -> np.ndarray:
    u = syn.uniform(1234, "sample/" + name, SAMPLE)
    return np.unique((u * n).astype(np.int64))


def pack_tensors(prefix: str, tensors: dict, out: dict):
    for k, t in tensors.items():
        a = t.detach().double().reshape(-1).numpy()
        out[f"{prefix}norm/{k}"] = np.array(np.linalg.norm(a))
        if a.size <= FULL_MAX:
            out[f"{prefix}full/{k}"] = a.astype(np.float32)
        else:
            idx = sample_idx(k, a.size)
            out[f"{prefix}idx/{k}"] = idx
            out[f"{prefix}val/{k}"] = a[idx].astype(np.float32)


def make_c1(seed=0, J=3, K=10, B=4, lr=0.0026):
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, 0, 0, B, K)
    img = torch.from_numpy(batch.images)
    lab = torch.from_numpy(batch.labels)
    t0 = time.time()
    ref = h.build_reference_model(seed, J, names)
    out = {"seed": np.array(seed), "J": np.array(J), "K": np.array(K), "B": np.array(B), "lr": np.array(lr),
           "labels": batch.labels}
    ref.eval()
    with torch.no_grad():
        out["logits"] = ref(img).numpy()
    ref.train()
    loss = ref(img, lab)
    loss.backward()
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    tr = {n: p for n, p in ref.named_parameters() if p.requires_grad}
    grads = {n: p.grad for n, p in tr.items() if p.grad is not None}
    pack_tensors("grad/", grads, out)
    # clip + SGD (torch.optim.SGD is what Dassl's build_optimizer returns; defaults momentum .9 wd 5e-4)
    before = {n: p.detach().clone() for n, p in tr.items()}
    total = torch.nn.utils.clip_grad_norm_([p for p in tr.values()], max_norm=1.0, error_if_nonfinite=False)
    out["total_norm"] = np.array(float(total))
    opt = torch.optim.SGD([p for p in ref.parameters() if p.requires_grad], lr=lr, momentum=0.9,
                          weight_decay=5e-4, dampening=0, nesterov=False)
    opt.step()
    deltas = {n: (p.detach().double() - before[n].double()) for n, p in tr.items() if p.grad is not None}
    pack_tensors("delta/", deltas, out)
    print(f"reference fp16 pass {time.time() - t0:.1f}s  loss {loss.item():.5f}  |g| {float(total):.4f}")

    # float64 restatement (same graph, no fp16 rounding) -> the noise floor
    M64 = O.build_model(seed, J, names, compute_dtype=torch.float64)
    with torch.no_grad():
        out["logits64"] = O.forward(M64, img.double(), train=False).numpy()
    loss64 = O.forward(M64, img.double(), lab, train=True)
    loss64.backward()
    out["loss64"] = np.array(loss64.item())
    g64 = {n: p.grad for n, p in M64.trainable().items() if p.grad is not None}
    pack_tensors("grad64/", g64, out)
    np.savez_compressed(HERE / "c1_maple.npz", **out)
    d = np.abs(out["logits"].astype(np.float64) - out["logits64"]).max()
    print(f"wrote c1_maple.npz: {len(out)} arrays; fp16-vs-fp64 logit gap {d:.2e}")


def make_fedavg(seed=0):
    _, _, maple_fed = h.load_reference()
    rng = lambda n, s, sd: torch.from_numpy(syn.normal(seed, f"fedavg/{n}/{sd}", int(np.prod(s))).reshape(s))
    keys = {"prompt_learner.ctx": ((2, 512), torch.float16), "prompt_learner.compound_prompts_text_parameters.0":
            ((2, 512), torch.float32), "image_encoder.ln_pre.weight": ((768,), torch.float32),
            "image_encoder.transformer.resblocks.11.attn.in_proj_bias": ((2304,), torch.float16),
            "logit_scale": ((), torch.float32)}
    dicts = []
    out = {}
    for c in range(3):
        sd = {}
        for k, (s, dt) in keys.items():
            v = rng(k, s, c) if k != "logit_scale" else torch.tensor(np.log(1 / 0.07))
            sd[k] = v.to(dt)
            out[f"in{c}/{k}"] = sd[k].float().numpy()
        dicts.append(sd)
    avg = maple_fed.MaPLeFederated.safe_average_weights(None, dicts, 3)
    for k, v in avg.items():
        assert v.dtype == torch.float16
        out[f"out/{k}"] = v.float().numpy()
    out["keys"] = np.array(list(keys))
    np.savez_compressed(HERE / "fedavg.npz", **out)
    print("wrote fedavg.npz")


# (name, seed, client, step, J, K, B, grads+deltas, per-layer trace) -- SURVEY.md §8(c) items 1-5
CASES = [
    ("c1_s0_b0", 0, 0, 0, 3, 10, 4, False, True),
    ("c1_s0_b1", 0, 0, 1, 3, 10, 4, False, False),
    ("c1_s1_b0", 1, 0, 0, 3, 10, 4, False, False),
    ("c1_s1_b1", 1, 0, 1, 3, 10, 4, True, False),
    ("c1_s2_b0", 2, 0, 0, 3, 10, 4, False, False),
    ("c1_s2_b1", 2, 0, 1, 3, 10, 4, False, False),
    # C3 per-client shape (BASELINE configs[2]: EuroSAT 10 classes, J=9 train.py:113, batch 4)
    ("c3_j9_k10_b4", 0, 1, 0, 9, 10, 4, True, True),
    ("j9_k38_b4", 5, 1, 0, 9, 38, 4, False, False),
    # the bench's own workload (BASELINE configs[3] per client: PatternNet 38 classes, B=32, J=9)
    ("c4_j9_k38_b32", 4, 2, 0, 9, 38, 32, True, True),
    # more rows at the bench's shape (eval logits, features, loss): 4 x 32 images on other seeds / clients
    ("c4e_s6_b32", 6, 0, 1, 9, 38, 32, False, False),
    ("c4e_s7_b32", 7, 1, 2, 9, 38, 32, False, False),
    ("c4e_s8_b32", 8, 3, 0, 9, 38, 32, False, False),
    ("c4e_s9_b32", 9, 2, 3, 9, 38, 32, False, False),
    # CLIP byte-level BPE ids (the reference's own SimpleTokenizer over bpe_small_merges.txt.gz) for the
    # ctx init and the class prompts of real PatternNet class names
    ("bpe_j3_k10_b4", 3, 0, 0, 3, 10, 4, True, False, True),
]

BPE_CLASSNAMES = ["airplane", "baseball_field", "christmas_tree_farm", "dense_residential", "ferry_terminal",
                  "mobile_home_park", "oil_gas_field", "runway_marking", "wastewater_treatment_plant", "sea_or_lake"]


def _hook_reference(ref, trace: dict):
    """Forward hooks on every residual block of both towers (clip/model.py:307-352): block i's output
    x (LND) is recorded as NLD, the layout the engine keeps in HBM."""
    hooks = []
    towers = (("vision", ref.image_encoder.transformer.resblocks), ("text", ref.text_encoder.transformer.resblocks))
    for tower, blocks in towers:
        for i, blk in enumerate(blocks):
            def hook(mod, inp, out, key=f"{tower}/{i}"):
                trace[key] = out[0].detach().permute(1, 0, 2).contiguous()
            hooks.append(blk.register_forward_hook(hook))
    return hooks


def _bpe_tokenizer():
    from federated_multi_modal_amd.tokenizer import SimpleTokenizer
    return SimpleTokenizer(str(BPE_MERGES))


def make_case(name, seed, client, step, J, K, B, grads, traced, bpe=False, lr=0.0026):
    names = BPE_CLASSNAMES[:K] if bpe else syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, client, step, B, K)
    img = torch.from_numpy(batch.images)
    lab = torch.from_numpy(batch.labels)
    t0 = time.time()
    if bpe:
        with h.reference_bpe(str(BPE_MERGES)):
            ref = h.build_reference_model(seed, J, names)
    else:
        ref = h.build_reference_model(seed, J, names)
    out = {"seed": np.array(seed), "client": np.array(client), "step": np.array(step), "J": np.array(J),
           "K": np.array(K), "B": np.array(B), "lr": np.array(lr), "labels": batch.labels}
    if bpe:
        out["bpe"] = np.array(BPE_MERGES.name)
        out["classnames"] = np.array(names)
        out["tokenized"] = ref.tokenized_prompts.numpy()
    trace: dict = {}
    hooks = _hook_reference(ref, trace) if traced else []
    feats = {}
    fh = [ref.image_encoder.register_forward_hook(lambda m, i, o: feats.__setitem__("img", o.detach())),
          ref.text_encoder.register_forward_hook(lambda m, i, o: feats.__setitem__("txt", o.detach()))]
    ref.eval()
    with torch.no_grad():
        out["logits"] = ref(img).numpy()
    for hk in hooks + fh:
        hk.remove()
    out["img_feat"] = feats["img"].float().numpy()
    out["txt_feat"] = feats["txt"].float().numpy()
    ref.train()
    if grads:
        loss = ref(img, lab)
        loss.backward()
        tr = {n: p for n, p in ref.named_parameters() if p.requires_grad}
        pack_tensors("grad/", {n: p.grad for n, p in tr.items() if p.grad is not None}, out)
        before = {n: p.detach().clone() for n, p in tr.items()}
        total = torch.nn.utils.clip_grad_norm_(list(tr.values()), max_norm=1.0, error_if_nonfinite=False)
        out["total_norm"] = np.array(float(total))
        opt = torch.optim.SGD([p for p in ref.parameters() if p.requires_grad], lr=lr, momentum=0.9,
                              weight_decay=5e-4, dampening=0, nesterov=False)
        opt.step()
        pack_tensors("delta/", {n: (p.detach().double() - before[n].double()) for n, p in tr.items()
                                if p.grad is not None}, out)
    else:
        with torch.no_grad():
            loss = ref(img, lab)
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    t_ref = time.time() - t0

    # float64 restatement: the noise floor per fixture (and per layer when traced)
    M64 = O.build_model(seed, J, names, compute_dtype=torch.float64, tokenizer=_bpe_tokenizer() if bpe else None)
    tr64: dict = {}
    with torch.no_grad():
        out["logits64"] = O.forward(M64, img.double(), train=False, trace=tr64).numpy()
    out["img_feat64"] = tr64["img_feat"].numpy()
    out["txt_feat64"] = tr64["txt_feat"].numpy()
    if grads:
        loss64 = O.forward(M64, img.double(), lab, train=True)
        loss64.backward()
        pack_tensors("grad64/", {n: p.grad for n, p in M64.trainable().items() if p.grad is not None}, out)
    else:
        with torch.no_grad():
            loss64 = O.forward(M64, img.double(), lab, train=True)
    out["loss64"] = np.array(loss64.item())
    if traced:
        for key, x in trace.items():
            flat = x.double().reshape(-1).numpy()
            f64 = tr64[key].reshape(-1).numpy()
            idx = trace_idx(name, key, flat.size)
            out[f"trace/{key}/shape"] = np.array(x.shape)
            out[f"trace/{key}/norm"] = np.array(np.linalg.norm(flat))
            out[f"trace/{key}/norm64"] = np.array(np.linalg.norm(f64))
            out[f"trace/{key}/err64"] = np.array(np.linalg.norm(flat - f64))  # the reference's own fp16 error
            out[f"trace/{key}/val"] = flat[idx].astype(np.float32)
            out[f"trace/{key}/val64"] = f64[idx]
    np.savez_compressed(HERE / f"case_{name}.npz", **out)
    d = np.abs(out["logits"].astype(np.float64) - out["logits64"]).max()
    print(f"case {name}: J={J} K={K} B={B} ref {t_ref:.1f}s total {time.time() - t0:.1f}s loss {out['loss']:.5f} "
          f"fp16-vs-fp64 logits {d:.2e}")


def make_c5_text(seed=0, J=9, K=1000, B=2, name="c5_text_k1000", client=0):
    """BASELINE configs[4] text side: all 1000 class prompts (77 tokens each) through the reference's
    TextEncoder (trainers/maple.py:52-79) and CustomCLIP's eval logits on B images."""
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, client, 0, B, K)
    img = torch.from_numpy(batch.images)
    t0 = time.time()
    ref = h.build_reference_model(seed, J, names)
    feats = {}
    fh = ref.text_encoder.register_forward_hook(lambda m, i, o: feats.__setitem__("txt", o.detach()))
    ref.eval()
    with torch.no_grad():
        logits = ref(img).numpy()
    fh.remove()
    t_ref = time.time() - t0
    M64 = O.build_model(seed, J, names, compute_dtype=torch.float64)
    with torch.no_grad():
        logits64 = O.forward(M64, img.double(), train=False).numpy()
    np.savez_compressed(HERE / f"case_{name}.npz", seed=np.array(seed), client=np.array(client), step=np.array(0),
                        J=np.array(J), K=np.array(K), B=np.array(B), labels=batch.labels, logits=logits,
                        logits64=logits64, txt_feat=feats["txt"].numpy())
    d = np.abs(logits.astype(np.float64) - logits64).max()
    print(f"case {name}: ref {t_ref:.1f}s total {time.time() - t0:.1f}s fp16-vs-fp64 logits {d:.2e}")


CAPTION_CASES = [
    # (name, seed, client, step, J, K, B, caption seed): the caption-conditioned visual prompts (K19)
    ("cap_c1_j3_b4", 0, 0, 0, 3, 10, 4, 1234),
    ("cap_j9_k10_b4", 0, 1, 0, 9, 10, 4, 99),
    # the caption tokens (and the class prompts) through the reference's own BPE tokenizer
    ("cap_bpe_j3_b4", 3, 0, 0, 3, 10, 4, 321, True),
]


def make_caption_case(name, seed, client, step, J, K, B, cap_seed, bpe=False, lr=0.0026):
    """The reference's training forward + backward with a caption list (trainers/maple.py:307-322 ->
    clip/model.py:550-561), its global generator seeded with cap_seed right before the call, so the
    AttentionPooling vector and the Linear(512, 768) it draws are the ones captions.draw_caption_weights
    draws from a generator seeded the same way.  Stores the loss, every gradient, the image features and
    every vision block's output (the sequence grows by B rows per prompted layer)."""
    names = BPE_CLASSNAMES[:K] if bpe else syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, client, step, B, K)
    caps = syn.synthetic_captions(seed, client, step, B)
    if bpe:  # punctuation, digits and a contraction through the BPE pre-split
        caps = [c if not c else c + (", it's 2 km wide." if i % 2 else "!") for i, c in enumerate(caps)]
    img, lab = torch.from_numpy(batch.images), torch.from_numpy(batch.labels)
    t0 = time.time()
    bpe_ctx = h.reference_bpe(str(BPE_MERGES)) if bpe else None
    if bpe_ctx:
        bpe_ctx.__enter__()
    ref = h.build_reference_model(seed, J, names)
    out = {"seed": np.array(seed), "client": np.array(client), "step": np.array(step), "J": np.array(J),
           "K": np.array(K), "B": np.array(B), "lr": np.array(lr), "labels": batch.labels,
           "cap_seed": np.array(cap_seed), "captions": np.array(caps)}
    if bpe:
        out["bpe"] = np.array(BPE_MERGES.name)
        out["classnames"] = np.array(names)
        out["tokenized"] = ref.tokenized_prompts.numpy()
        _, tokenize, _ = h.load_reference_tokenizer(str(BPE_MERGES))
        out["caption_tokens"] = tokenize(caps).numpy()
    # the random tensors the forward below draws, drawn the same way beforehand by the reference's own
    # classes (AttentionPooling, clip/model.py:457-462; nn.Linear(512, 768).half(), :557)
    model_mod, _, _ = h.load_reference()
    with h.cuda_as_cpu():
        torch.manual_seed(cap_seed)
        ap = model_mod.AttentionPooling(512)
        lin = torch.nn.Linear(512, 768).half().to("cuda")
    out["cap_w"] = ap.attention_weights.detach().float().numpy()
    out["cap_b"] = lin.bias.detach().float().numpy()
    wl = lin.weight.detach().double().reshape(-1).numpy()
    out["cap_W_norm"] = np.array(np.linalg.norm(wl))
    out["cap_W_idx"] = sample_idx("cap_W", wl.size)
    out["cap_W_val"] = wl[out["cap_W_idx"]].astype(np.float32)
    trace: dict = {}
    hooks = _hook_reference(ref, trace)
    feats = {}
    hooks.append(ref.image_encoder.register_forward_hook(lambda m, i, o: feats.__setitem__("img", o.detach())))
    ref.train()
    with h.cuda_as_cpu():
        torch.manual_seed(cap_seed)
        loss = ref(img, lab, caps)
    for hk in hooks:
        hk.remove()
    if bpe_ctx:
        bpe_ctx.__exit__(None, None, None)
    loss.backward()
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    out["img_feat"] = feats["img"].float().numpy()
    tr = {n: p for n, p in ref.named_parameters() if p.requires_grad}
    pack_tensors("grad/", {n: p.grad for n, p in tr.items() if p.grad is not None}, out)
    for key, x in trace.items():
        if not key.startswith("vision/"):
            continue
        flat = x.double().reshape(-1).numpy()
        idx = trace_idx(name, key, flat.size)
        out[f"trace/{key}/shape"] = np.array(x.shape)
        out[f"trace/{key}/norm"] = np.array(np.linalg.norm(flat))
        out[f"trace/{key}/val"] = flat[idx].astype(np.float32)
    np.savez_compressed(HERE / f"case_{name}.npz", **out)
    print(f"caption case {name}: J={J} K={K} B={B} {time.time() - t0:.1f}s loss {out['loss']:.5f} "
          f"vision lengths {[int(out[f'trace/vision/{i}/shape'][1]) for i in range(12)]}")


BPE_MERGES = HERE / "bpe_small_merges.txt.gz"   # tests/golden/make_bpe_merges.py

BPE_TEXTS = [
    "a photo of a", "a photo of a dense residential.", "a photo of a baseball field.", "X X",
    "a photo of a wastewater treatment plant.", "a photo of a sea or lake.", "a photo of a highway or road.",
    "Annual Crop Land", "Herbaceous Vegetation Land", "mobilehomepark", "storagetanks",
    "there's a harbor with boats docked along the pier, and the water is calm.",
    "the airport's runway has two airplanes waiting; it's a busy day.",
    "they'll build a new bridge by 2025; I'm sure they'd like to finish early.",
    "we've  seen   solar\tpanels\non the roof!!", "UPPER case Words And MiXeD", "",
    "numbers 0 1 23 456 7890 3.14 50% #1 @home $5 a-b a_b a/b...", "html &amp; entities &lt;b&gt; &amp;amp;",
    "café résumé naïve façade jalapeño über", "東京 北京 ソウル 서울 москва αθήνα", "emoji 🙂🛰️ © ® ™ ° ± × ÷",
    "unseen words: quixotic zephyr xylophone juxtaposition bureaucracy", "<|startoftext|> inside <|endoftext|> text",
    "aaaaaaaaaaaa abababababab mississippi bookkeeper", "'s 't 're 've 'm 'll 'd", "   leading and trailing   ",
]


def make_bpe():
    """The reference's own SimpleTokenizer.encode / clip.tokenize (clip/simple_tokenizer.py:121-127,
    clip/clip.py:185-221) over the committed small merges file: ids of every text, tokenize at context
    77 (incl. the overflow RuntimeError and truncate=True), and the vocabulary's special ids."""
    import json
    tok, tokenize, _ = h.load_reference_tokenizer(str(BPE_MERGES))
    out = {"merges": BPE_MERGES.name, "sot": tok.encoder["<|startoftext|>"], "eot": tok.encoder["<|endoftext|>"],
           "vocab_size": len(tok.encoder), "encode": [], "tokenize": [], "bpe": {}}
    for t in BPE_TEXTS:
        out["encode"].append([t, tok.encode(t)])
    out["tokenize"] = [[t, tokenize(t).tolist()[0]] for t in BPE_TEXTS]
    long_text = " ".join(["quixotic zephyr"] * 30)
    try:
        tokenize(long_text)
        out["overflow_raises"] = False
    except RuntimeError as err:
        out["overflow_raises"] = True
        out["overflow_message"] = str(err)
    out["truncate"] = [long_text, tokenize(long_text, truncate=True).tolist()[0]]
    out["context_16"] = [BPE_TEXTS[1], tokenize(BPE_TEXTS[1], context_length=16).tolist()[0]]
    for w in ("residential", "mississippi", "quixotic", "a", "12"):
        enc = "".join(tok.byte_encoder[b] for b in w.encode("utf-8"))
        out["bpe"][w] = tok.bpe(enc)
    (HERE / "bpe_ids.json").write_text(json.dumps(out, ensure_ascii=False, indent=0))
    print(f"wrote bpe_ids.json: {len(BPE_TEXTS)} texts, vocab {out['vocab_size']}")


def make_state_dict_keys():
    """The reference CustomCLIP.state_dict() key set, shapes and dtypes (trainers/maple.py:221-229) at
    J=3 and J=9, and the dtypes FedAvg leaves in the aggregator checkpoint (every key .half(),
    trainers/maple_fed.py:314, 367-386)."""
    import json
    out = {}
    for J in (3, 9):
        ref = h.build_reference_model(0, J, syn.synthetic_classnames(10, 0))
        sd = ref.state_dict()
        out[f"J{J}"] = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()]
    (HERE / "state_dict_keys.json").write_text(json.dumps(out, indent=0))
    print("wrote state_dict_keys.json:", {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    import sys as _sys
    what = _sys.argv[1:] or ["fedavg", "c1", "cases", "c5", "keys"]
    if "fedavg" in what:
        make_fedavg()
    if "c1" in what:
        make_c1()
    if "cases" in what:
        for c in CASES:
            make_case(*c)
    for c in CASES + CAPTION_CASES:  # one case by name: python make_golden.py case:<name>
        if f"case:{c[0]}" in what:
            (make_caption_case if c in CAPTION_CASES else make_case)(*c)
    if "c5" in what:
        make_c5_text()
    if "c5b8" in what:
        make_c5_text(seed=1, B=8, name="c5_k1000_b8", client=3)
    if "keys" in what:
        make_state_dict_keys()
    if "captions" in what:
        for c in CAPTION_CASES:
            make_caption_case(*c)
    if "bpe" in what:
        make_bpe()
