"""Import the reference's own MaPLe code (read-only, /root/reference) for golden fixtures.

Runs ONLY in the build container (the reference never travels to the GPU box).
How:
  * clip/model.py is loaded by file path (its package __init__ needs torchvision);
  * trainers/maple.py and trainers/maple_fed.py are loaded after stub modules for the
    absent third-party pieces: Dassl (registry/TrainerX/optim/utils), the `clip`
    package (tokenize -> the build's synthetic tokenizer) and SimpleTokenizer (the
    BPE vocab file is absent).
Nothing from the reference is copied; this module only wires imports.
"""
from __future__ import annotations

import importlib.util
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
REPO = Path(__file__).resolve().parents[2]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

from federated_multi_modal_amd import synthetic as syn  # noqa: E402


def _load(name: str, path: Path):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


_CACHE = {}


def load_reference():
    if "maple" in _CACHE:
        return _CACHE["model"], _CACHE["maple"], _CACHE["maple_fed"]
    if not REF.exists():
        raise RuntimeError("/root/reference is not present (golden generation runs in the build container only)")

    # ---- Dassl stubs (un-vendored third party) ----
    dassl = types.ModuleType("dassl")
    engine = types.ModuleType("dassl.engine")

    class _Registry:
        def register(self):
            return lambda cls: cls

    class TrainerX:  # minimal base; the harness never calls TrainerX.__init__
        def __init__(self, *a, **k):
            pass

    engine.TRAINER_REGISTRY = _Registry()
    engine.TrainerX = TrainerX
    metrics = types.ModuleType("dassl.metrics")
    metrics.compute_accuracy = lambda *a, **k: None
    utils = types.ModuleType("dassl.utils")
    utils.load_pretrained_weights = lambda *a, **k: None
    utils.load_checkpoint = lambda *a, **k: None
    utils.mkdir_if_missing = lambda *a, **k: None
    utils.save_checkpoint = lambda *a, **k: None
    optim = types.ModuleType("dassl.optim")
    optim.build_optimizer = lambda *a, **k: None
    optim.build_lr_scheduler = lambda *a, **k: None
    data = types.ModuleType("dassl.data")
    data.DataManager = object
    datasets = types.ModuleType("dassl.data.datasets")
    datasets.Datum = object
    dm = types.ModuleType("dassl.data.data_manager")
    dm.build_transform = lambda *a, **k: None
    dm.build_data_loader = lambda *a, **k: None
    for m, n in [(dassl, "dassl"), (engine, "dassl.engine"), (metrics, "dassl.metrics"), (utils, "dassl.utils"),
                 (optim, "dassl.optim"), (data, "dassl.data"), (datasets, "dassl.data.datasets"),
                 (dm, "dassl.data.data_manager")]:
        sys.modules[n] = m
    dassl.engine, dassl.metrics, dassl.utils, dassl.optim, dassl.data = engine, metrics, utils, optim, data
    data.datasets = datasets

    # ---- clip package stub: reference model.py + synthetic tokenizer ----
    model = _load("ref_clip_model", REF / "clip" / "model.py")
    clip_pkg = types.ModuleType("clip")
    clip_pkg.__path__ = []
    clip_mod = types.ModuleType("clip.clip")
    clip_mod.tokenize = lambda texts, context_length=77, truncate=False: torch.from_numpy(
        syn.tokenize(texts, context_length))
    clip_mod.build_model = model.build_model
    clip_mod._MODELS = {}
    st = types.ModuleType("clip.simple_tokenizer")

    class SimpleTokenizer:
        def encode(self, text):
            return syn.encode(text)

    st.SimpleTokenizer = SimpleTokenizer
    clip_pkg.clip = clip_mod
    clip_pkg.model = model
    clip_pkg.simple_tokenizer = st
    sys.modules["clip"] = clip_pkg
    sys.modules["clip.clip"] = clip_mod
    sys.modules["clip.model"] = model
    sys.modules["clip.simple_tokenizer"] = st

    # tqdm / PIL used by maple_fed at import time
    for opt in ("tqdm", "PIL"):
        try:
            __import__(opt)
        except Exception:  # pragma: no cover
            stub = types.ModuleType(opt)
            if opt == "tqdm":
                stub.trange = range
            else:
                stub.Image = None
            sys.modules[opt] = stub

    maple = _load("ref_trainers_maple", REF / "trainers" / "maple.py")
    trainers_pkg = types.ModuleType("trainers")
    trainers_pkg.__path__ = []
    trainers_pkg.maple = maple
    sys.modules["trainers"] = trainers_pkg
    sys.modules["trainers.maple"] = maple
    cdm = types.ModuleType("trainers.client_datamanager")
    cdm.ClientDataManager = object
    sys.modules["trainers.client_datamanager"] = cdm
    # maple_fed does `from .client_datamanager import ...`: give it a package context
    spec = importlib.util.spec_from_file_location("trainers.maple_fed", str(REF / "trainers" / "maple_fed.py"))
    maple_fed = importlib.util.module_from_spec(spec)
    maple_fed.__package__ = "trainers"
    sys.modules["trainers.maple_fed"] = maple_fed
    spec.loader.exec_module(maple_fed)

    _CACHE.update(model=model, maple=maple, maple_fed=maple_fed)
    return model, maple, maple_fed


def load_reference_tokenizer(bpe_path: str):
    """The reference's own tokenizer over a merges file: clip/simple_tokenizer.py (SimpleTokenizer) and
    clip/clip.py (tokenize), loaded by file path as the package `refclip_bpe`.  Wiring only:
      * ftfy is absent: a stub module whose fix_text returns its input (the fixtures hold only text
        ftfy leaves unchanged; see federated_multi_modal_amd/tokenizer.py);
      * torchvision is absent: clip.py imports its transforms at module level for `_transform`, which
        tokenize never touches -- stub classes stand in;
      * clip.py builds its module-level `_tokenizer = _Tokenizer()` with the default merges path (absent):
        the default argument is pointed at `bpe_path` before clip.py is executed.
    Returns (SimpleTokenizer instance, clip.tokenize function, the clip module)."""
    key = ("bpe", str(bpe_path))
    if key in _CACHE:
        return _CACHE[key]
    load_reference()  # the model module (clip.py does `from .model import build_model`)
    if "ftfy" not in sys.modules:
        ftfy = types.ModuleType("ftfy")
        ftfy.fix_text = lambda text, *a, **k: text
        sys.modules["ftfy"] = ftfy
    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tr = types.ModuleType("torchvision.transforms")
        for n in ("Compose", "Resize", "CenterCrop", "ToTensor", "Normalize"):
            setattr(tr, n, type(n, (), {"__init__": lambda self, *a, **k: None}))
        tr.InterpolationMode = types.SimpleNamespace(BICUBIC="bicubic")
        tv.transforms = tr
        sys.modules["torchvision"], sys.modules["torchvision.transforms"] = tv, tr
    pkg_name = f"refclip_bpe{len([k for k in _CACHE if isinstance(k, tuple)])}"
    pkg = types.ModuleType(pkg_name)
    pkg.__path__ = []
    sys.modules[pkg_name] = pkg
    sys.modules[pkg_name + ".model"] = _CACHE["model"]
    st = _load(pkg_name + ".simple_tokenizer", REF / "clip" / "simple_tokenizer.py")
    st.SimpleTokenizer.__init__.__defaults__ = (str(bpe_path),)
    spec = importlib.util.spec_from_file_location(pkg_name + ".clip", str(REF / "clip" / "clip.py"))
    clip_mod = importlib.util.module_from_spec(spec)
    clip_mod.__package__ = pkg_name
    sys.modules[pkg_name + ".clip"] = clip_mod
    spec.loader.exec_module(clip_mod)
    res = (st.SimpleTokenizer(str(bpe_path)), clip_mod.tokenize, clip_mod)
    _CACHE[key] = res
    return res


class reference_bpe:
    """`with reference_bpe(path):` the reference's trainers/maple.py tokenizes with its own BPE tokenizer
    over `path` (its module globals `clip` -> the loaded clip/clip.py, `_tokenizer` -> SimpleTokenizer)
    instead of the synthetic stand-in the other fixtures use."""

    def __init__(self, bpe_path):
        self.bpe_path = bpe_path

    def __enter__(self):
        _, maple, _ = load_reference()
        tok, _, clip_mod = load_reference_tokenizer(self.bpe_path)
        self.saved = (maple.clip, maple._tokenizer)
        maple.clip, maple._tokenizer = clip_mod, tok
        return self

    def __exit__(self, *exc):
        _, maple, _ = load_reference()
        maple.clip, maple._tokenizer = self.saved


class cuda_as_cpu:
    """The reference's caption path hard-codes `.to("cuda")` (clip/model.py:461, 554, 557); on this CPU-only
    host `with cuda_as_cpu():` maps a "cuda" device argument of Tensor.to / Module.to to "cpu" for the
    duration of the call (test wiring, like the Dassl stubs; the arithmetic is the reference's)."""

    @staticmethod
    def _fix(args, kwargs):
        hit = []

        def f(a):
            if isinstance(a, str) and a.startswith("cuda"):
                hit.append(1)
                return "cpu"
            if isinstance(a, torch.device) and a.type == "cuda":
                hit.append(1)
                return torch.device("cpu")
            return a
        return tuple(f(a) for a in args), {k: f(v) for k, v in kwargs.items()}, bool(hit)

    def __enter__(self):
        self.t_to, self.m_to = torch.Tensor.to, torch.nn.Module.to
        t_to, m_to, fix = self.t_to, self.m_to, self._fix

        def tensor_to(x, *a, **k):
            a, k, moved = fix(a, k)
            if moved:  # a device transfer returns a new plain tensor (a Parameter's .to("cuda") is no Parameter)
                k["copy"] = True
            return t_to(x, *a, **k)

        def module_to(m, *a, **k):
            a, k, _ = fix(a, k)
            return m_to(m, *a, **k)
        torch.Tensor.to, torch.nn.Module.to = tensor_to, module_to
        return self

    def __exit__(self, *exc):
        torch.Tensor.to, torch.nn.Module.to = self.t_to, self.m_to


class _NS:
    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, _NS(**v) if isinstance(v, dict) else v)


def make_cfg(prompt_depth: int, n_ctx: int = 2, ctx_init: str = "a photo of a"):
    return _NS(TRAINER={"MAPLE": {"N_CTX": n_ctx, "CTX_INIT": ctx_init, "PREC": "fp16",
                                  "PROMPT_DEPTH": prompt_depth}},
               INPUT={"SIZE": (224, 224)})


def build_reference_model(seed: int, prompt_depth: int, classnames, vision_layers: int = 12,
                          text_layers: int = 12):
    """CustomCLIP exactly as MaPLe.build_model builds it (trainers/maple.py:421-479), with
    synthetic weights in place of the downloaded checkpoint."""
    model_mod, maple, _ = load_reference()
    dims = syn.ClipDims()
    sd = syn.clip_state_dict(seed, dims, full_token_table=True, vision_layers=vision_layers,
                             text_layers=text_layers)
    design = {"trainer": "MaPLe", "vision_depth": 0, "language_depth": 0, "vision_ctx": 0,
              "language_ctx": 0, "maple_length": 2}
    clip_model = model_mod.CLIP(dims.embed_dim, dims.image_resolution, vision_layers, dims.vision_width,
                                dims.vision_patch, dims.context_length, dims.vocab_size, dims.text_width,
                                dims.text_heads, text_layers, design)
    model_mod.convert_weights(clip_model)
    tsd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
    clip_model.load_state_dict(tsd, strict=True)  # load_state_dict keeps each param's dtype
    clip_model.eval()
    cfg = make_cfg(prompt_depth)
    torch.manual_seed(seed)
    model = maple.CustomCLIP(cfg, list(classnames), clip_model)
    pl = syn.prompt_learner_params(seed, prompt_depth)
    with torch.no_grad():
        for k, v in pl.items():
            p = dict(model.prompt_learner.named_parameters())[k]
            p.copy_(torch.from_numpy(v).to(p.dtype))
    # freeze policy, restated from trainers/maple.py:447-479
    for p in model.parameters():
        p.requires_grad_(False)
    for _, mod in model.named_modules():
        if isinstance(mod, (torch.nn.LayerNorm, torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            for p in mod.parameters():
                p.requires_grad_(True)
    for n, p in model.named_parameters():
        if "prompt_learner" in n:
            p.requires_grad_(True)
    for n, p in model.named_parameters():
        if "visual.transformer.resblocks.11" in n or "transformer.resblocks.11" in n:
            p.requires_grad_(True)
    return model
