"""CPU tier: pin the oracle (oracle/maple_oracle.py) against the golden fixtures generated from the
reference itself (tests/golden/make_golden.py imports /root/reference's clip/model.py,
trainers/maple.py and trainers/maple_fed.py), plus the host logic of the product package that
needs no GPU (synthetic generator, tokenizer, parameter inventory, C-ABI exports)."""
import ctypes
import math
import re
from pathlib import Path

import numpy as np
import pytest
import torch

import _cases as C
from federated_multi_modal_amd import synthetic as syn
from oracle import maple_oracle as O

GOLD = Path(__file__).resolve().parent / "golden"
ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def c1():
    return dict(np.load(GOLD / "c1_maple.npz"))


@pytest.fixture(scope="module")
def c1_oracle(c1):
    """The oracle's fp16 forward/backward on C1 (J=3, K=10, B=4): ~2 s on 8 CPU cores."""
    J, K, B, seed = int(c1["J"]), int(c1["K"]), int(c1["B"]), int(c1["seed"])
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, 0, 0, B, K)
    M = O.build_model(seed, J, names)
    img = torch.from_numpy(batch.images)
    lab = torch.from_numpy(batch.labels)
    with torch.no_grad():
        logits = O.forward(M, img, train=False)
    opt = O.SGDState(lr=float(c1["lr"]))
    before = {k: v.detach().clone() for k, v in M.trainable().items()}
    loss, grads, total = O.train_step(M, img, lab, opt)
    deltas = {k: (v.detach().double() - before[k].double()) for k, v in M.trainable().items()}
    return dict(M=M, logits=logits, loss=loss, grads=grads, total=total, deltas=deltas, labels=batch.labels)


def _golden_tensor(g, prefix, name):
    if f"{prefix}full/{name}" in g:
        return None, g[f"{prefix}full/{name}"]
    return g[f"{prefix}idx/{name}"], g[f"{prefix}val/{name}"]


def test_golden_inputs_regenerate(c1):
    """The portable PRNG regenerates the fixture's labels bit-exactly (inputs are not shipped)."""
    b = syn.client_batch(int(c1["seed"]), 0, 0, int(c1["B"]), int(c1["K"]))
    assert np.array_equal(b.labels, c1["labels"])


def test_oracle_logits_match_reference(c1, c1_oracle):
    """Oracle eval logits == the reference's (trainers/maple.py:304-346) on the same inputs, bit for bit."""
    ours = c1_oracle["logits"].numpy()
    assert ours.dtype == np.float16
    assert np.array_equal(ours, c1["logits"])
    # the fp16 noise floor the 1e-3 gate sits on: fp16-vs-fp64 gap of the reference
    assert np.abs(c1["logits"].astype(np.float64) - c1["logits64"]).max() < 5e-3


def test_oracle_loss_and_grads_match_reference(c1, c1_oracle):
    assert abs(float(c1_oracle["loss"]) - float(c1["loss"])) <= 2e-3
    assert abs(float(c1_oracle["total"]) - float(c1["total_norm"])) <= 1e-3 * float(c1["total_norm"])
    grads = c1_oracle["grads"]
    names = sorted(k[len("grad/norm/"):] for k in c1 if k.startswith("grad/norm/"))
    assert set(names) == set(grads), set(names) ^ set(grads)
    for n in names:
        g = grads[n].double().reshape(-1).numpy()
        ref_norm = float(c1[f"grad/norm/{n}"])
        assert abs(np.linalg.norm(g) - ref_norm) <= 1e-2 * ref_norm + 1e-6, n
        idx, val = _golden_tensor(c1, "grad/", n)
        got = g if idx is None else g[idx]
        scale = np.abs(val).max() + 1e-12
        assert np.abs(got - val).max() <= 2e-2 * scale, n


def test_oracle_sgd_deltas_match_reference(c1, c1_oracle):
    """clip_grad_norm_(1.0) + SGD(momentum .9, wd 5e-4) first step (trainers/maple.py:590-598)."""
    for k, d in c1_oracle["deltas"].items():
        if f"delta/norm/{k}" not in c1:
            continue
        idx, val = _golden_tensor(c1, "delta/", k)
        got = d.reshape(-1).numpy()
        got = got if idx is None else got[idx]
        scale = np.abs(val).max() + 1e-12
        assert np.abs(got - val).max() <= 2e-2 * scale + 1e-6, k


@pytest.mark.parametrize("name", C.case_names())
def test_oracle_matches_reference_case(name):
    """Every reference-generated fixture (tests/golden/case_*.npz: C1 at 3 seeds x 2 batches, the C3
    per-client shape J=9 K=10 B=4, J=9 K=38 B=4, the C5 text side K=1000): the oracle's fp16 eval
    logits, tower features and train loss equal the reference's bit for bit; on traced cases every
    block output of both towers (clip/model.py:307-352) too."""
    c = C.load_case(name)
    J, K, B, seed, names, batch = C.case_inputs(c)
    M = O.build_model(seed, J, names, tokenizer=C.case_tokenizer(c))
    if "tokenized" in c:
        assert np.array_equal(M.tokenized.numpy(), c["tokenized"])
    img = torch.from_numpy(batch.images)
    tr: dict = {}
    with torch.no_grad():
        logits = O.forward(M, img, train=False, trace=tr).numpy()
    assert np.array_equal(logits, c["logits"])
    assert np.array_equal(tr["txt_feat"].float().numpy(), c["txt_feat"].astype(np.float32))
    if "img_feat" in c:
        assert np.array_equal(tr["img_feat"].float().numpy(), c["img_feat"])
    for key in C.trace_keys(c):
        flat = tr[key].double().reshape(-1).numpy()
        assert tuple(tr[key].shape) == tuple(c[f"trace/{key}/shape"]), key
        idx = C.trace_idx(name, key, flat.size)
        assert np.array_equal(flat[idx].astype(np.float32), c[f"trace/{key}/val"]), key
        assert np.isclose(np.linalg.norm(flat), float(c[f"trace/{key}/norm"]), rtol=1e-12), key
    if "loss" in c:
        with torch.no_grad():
            loss = O.forward(M, img, torch.from_numpy(batch.labels), train=True)
        assert float(loss) == float(c["loss"])


def test_oracle_fedavg_matches_reference():
    g = np.load(GOLD / "fedavg.npz")
    keys = [str(k) for k in g["keys"]]
    dicts = []
    for c in range(3):
        sd = {}
        for k in keys:
            dt = torch.float16 if k in ("prompt_learner.ctx",
                                         "image_encoder.transformer.resblocks.11.attn.in_proj_bias") else torch.float32
            sd[k] = torch.from_numpy(g[f"in{c}/{k}"]).to(dt)
        dicts.append(sd)
    avg = O.safe_average_weights(dicts)
    for k in keys:
        assert avg[k].dtype == torch.float16
        assert np.array_equal(avg[k].float().numpy(), g[f"out/{k}"]), k
    assert O.check_weights_valid(avg)
    bad = dict(avg)
    bad[keys[0]] = bad[keys[0]].clone()
    bad[keys[0]].view(-1)[0] = float("nan")
    assert not O.check_weights_valid(bad)


# --------------------------------------------------------------------------- host logic (no GPU)

def test_synthetic_generator_is_counter_based():
    a = syn.normal(7, "x", 100)
    b = syn.normal(7, "x", 60, start=40)
    assert np.array_equal(a[40:], b)
    assert not np.array_equal(syn.normal(8, "x", 10), a[:10])
    u = syn.uniform(0, "u", 100000)
    assert 0 <= u.min() and u.max() < 1 and abs(u.mean() - 0.5) < 0.01


def test_synthetic_tokenizer_semantics():
    t = syn.tokenize(["a photo of a forest.", "a photo of a dense residential."])
    assert t.shape == (2, 77) and t[0, 0] == syn.SOT_TOKEN
    eot = t.argmax(-1)
    assert (t[np.arange(2), eot] == syn.EOT_TOKEN).all()
    assert eot[1] == eot[0] + 1
    with pytest.raises(RuntimeError):
        syn.tokenize(" ".join(["w"] * 80))


def test_param_specs_and_trainable_inventory():
    """The engine's parameter inventory == the reference's CustomCLIP parameters used on the path
    and the freeze policy of trainers/maple.py:447-479 (counts measured in SURVEY.md §8 a16)."""
    from federated_multi_modal_amd.engine import EngineConfig, reference_param_specs, _is_trainable
    for J, n_tr, n_tensors in ((3, 11_879_680, 129), (9, 14_250_496, 147), (11, 15_040_768, 153)):
        cfg = EngineConfig(batch=4, classnames=["a", "b"], prompt_depth=J)
        specs = reference_param_specs(cfg)
        tr = [(n, s) for n, s, _ in specs if _is_trainable(n)]
        assert len(tr) == n_tensors, (J, len(tr))
        assert sum(int(np.prod(s)) for _, s in tr) == n_tr, J


def test_abi_header_matches_binding():
    """Every entry point include/mapfed.h declares is bound by _lib.SIGNATURES with the same arity."""
    from federated_multi_modal_amd import _lib
    hdr = (ROOT / "include" / "mapfed.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    decls = re.findall(r"\b(?:int|int64_t|const char\*)\s+(mf_\w+)\s*\(([^)]*)\)\s*;", hdr)
    assert len(decls) >= 25
    for name, args in decls:
        assert name in _lib.exported_symbols(), name
        if name == "mf_last_error":
            continue
        n = 0 if args.strip() in ("", "void") else len(args.split(","))
        assert len(_lib.SIGNATURES[name]) == n, (name, n, len(_lib.SIGNATURES[name]))


def test_library_loads_and_exports_every_symbol():
    """libmapfed.so (built by __graft_entry__.build()) loads without a GPU and exports the ABI."""
    from federated_multi_modal_amd import _lib
    if not _lib.LIB_PATH.exists():
        import __graft_entry__
        __graft_entry__.build()
    h = ctypes.CDLL(str(_lib.LIB_PATH))
    for name in _lib.exported_symbols():
        assert hasattr(h, name), name
    h.mf_abi_version.restype = ctypes.c_int
    assert h.mf_abi_version() == 1
    assert _lib.call("mf_optim_chunk_elems") > 0
    # argument validation runs on the host, before any launch
    rc = h.mf_gemm_nt(None, 64, None, 64, None, 64, 8, 8, 63, None, None, None, 0, 0, 0, None)
    assert rc != 0
    h.mf_last_error.restype = ctypes.c_char_p
    assert b"multiple of 64" in h.mf_last_error()


def test_fused_qkv_attention_shape_rule():
    """Host side of mf_qkv_attention_fwd: the shapes it covers (the vision blocks, D = 768 at 193..208 tokens;
    the text blocks, D = 512 causal at 65..80 tokens) and the argument checks that run before any launch."""
    from federated_multi_modal_amd import _lib, ops
    assert ops.qkv_attention_supported(32, 199, 12, False) and ops.qkv_attention_supported(38, 77, 8, True)
    assert not ops.qkv_attention_supported(32, 199, 12, True) and not ops.qkv_attention_supported(38, 10, 8, True)
    assert not ops.qkv_attention_supported(32, 455, 12, False)  # the caption path's grown sequences
    h = _lib.lib()
    assert h.mf_qkv_attention_fwd(None, 768, 10, None, None, None, 2304, None, 768, None, 199, 1, 199, 12, 0,
                                  None) != 0  # x_rows < N*L: refused on the host
    assert b"fewer than" in h.mf_last_error()


def test_product_library_has_one_gemm_path():
    """The product library links no vendor GEMM and exports no route to one: every product of
    the step runs on csrc/gemm.hip's kernels; torch.mm (hipBLASLt) stays a yardstick in tests/diagnostics only."""
    import subprocess
    from federated_multi_modal_amd import _lib
    so = str(_lib.LIB_PATH)
    dyn = subprocess.run(["readelf", "-d", so], capture_output=True, text=True, check=True).stdout
    assert "NEEDED" in dyn and "hipblaslt" not in dyn.lower() and "rocblas" not in dyn.lower()
    syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    assert "mf_gemm_lib" not in syms and "mf_gemm_nt" in syms


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from federated_multi_modal_amd import _lib
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setenv("MAPFED_LIB", str(tmp_path / "missing.so"))
    with pytest.raises(_lib.MapfedError):
        _lib.lib()
    monkeypatch.setattr(_lib, "_LIB", None)


def test_clip_dims_inferred_from_state_dict():
    """clip/model.py:750-777: the geometry comes from the checkpoint's tensor shapes (ViT-B/16 and -B/32
    load; ResNet and other widths are refused with the reason)."""
    from federated_multi_modal_amd.engine import check_dims, clip_dims_from_state_dict
    d = clip_dims_from_state_dict(syn.clip_state_dict(0, vision_layers=2, text_layers=3))
    assert (d.vision_width, d.vision_patch, d.grid, d.image_resolution, d.vision_layers) == (768, 16, 14, 224, 2)
    assert (d.text_width, d.text_heads, d.text_layers, d.context_length, d.embed_dim) == (512, 8, 3, 77, 512)
    check_dims(d)
    b32 = {"visual.proj": np.empty((768, 512)), "visual.conv1.weight": np.empty((768, 3, 32, 32)),
           "visual.positional_embedding": np.empty((50, 768)), "text_projection": np.empty((512, 512)),
           "positional_embedding": np.empty((77, 512)), "token_embedding.weight": np.empty((49408, 512)),
           "ln_final.weight": np.empty(512)}
    for i in range(12):
        b32[f"visual.transformer.resblocks.{i}.attn.in_proj_weight"] = np.empty((2304, 768))
        b32[f"transformer.resblocks.{i}.attn.in_proj_weight"] = np.empty((1536, 512))
    d32 = clip_dims_from_state_dict(b32)
    assert (d32.vision_patch, d32.grid, d32.image_resolution, d32.vision_layers, d32.text_layers) == (32, 7, 224, 12, 12)
    check_dims(d32)
    with pytest.raises(NotImplementedError):
        clip_dims_from_state_dict({"visual.layer1.0.conv1.weight": np.empty((64, 3, 3, 3))})
    l14 = dict(b32, **{"visual.conv1.weight": np.empty((1024, 3, 14, 14)),
                       "visual.positional_embedding": np.empty((257, 1024))})
    with pytest.raises(NotImplementedError):
        check_dims(clip_dims_from_state_dict(l14))


@pytest.mark.parametrize("name", C.caption_case_names())
def test_oracle_caption_path_matches_reference(name):
    """K19 (clip/model.py:457-476, 550-561): the random AttentionPooling vector and Linear(512, 768) drawn by
    captions.draw_caption_weights from a generator seeded like the reference's global one equal the
    reference's draws bit for bit; the oracle's training forward with those captions and weights then gives
    the reference's loss, image features and every (growing) vision block output bit for bit, and its
    gradients within the tolerance of the C1 pin."""
    from federated_multi_modal_amd.captions import draw_caption_weights
    c = C.load_case(name)
    J, K, B, seed, names, batch = C.case_inputs(c)
    w, W, b = draw_caption_weights(torch.Generator().manual_seed(int(c["cap_seed"])))
    assert np.array_equal(w.float().numpy(), c["cap_w"]) and np.array_equal(b.float().numpy(), c["cap_b"])
    assert np.array_equal(W.double().reshape(-1).numpy()[c["cap_W_idx"]].astype(np.float32), c["cap_W_val"])
    M = O.build_model(seed, J, names, tokenizer=C.case_tokenizer(c))
    tr: dict = {}
    caps = [str(x) for x in c["captions"]]
    loss = O.forward(M, torch.from_numpy(batch.images), torch.from_numpy(batch.labels), train=True, trace=tr,
                     captions=caps, cap_weights=(w, W, b))
    assert float(loss) == float(c["loss"])
    assert np.array_equal(tr["img_feat"].float().numpy(), c["img_feat"])
    for key in C.trace_keys(c):
        flat = tr[key].double().reshape(-1).numpy()
        assert tuple(tr[key].shape) == tuple(c[f"trace/{key}/shape"]), key
        assert np.array_equal(flat[C.trace_idx(name, key, flat.size)].astype(np.float32), c[f"trace/{key}/val"]), key
    loss.backward()
    for n, p in M.trainable().items():
        if f"grad/norm/{n}" not in c:
            assert p.grad is None, n
            continue
        g = p.grad.double().reshape(-1).numpy()
        ours, ref = C.sel(c, "grad/", n, g)
        assert np.abs(ours - ref).max() <= 2e-2 * (np.abs(ref).max() + 1e-12), n
