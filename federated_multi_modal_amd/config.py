"""Config surface of the reference's train.py: a yacs-compatible CfgNode, the Dassl defaults the
MaPLe federated path reads, and train.py's extend_cfg / setup_cfg.

yacs and Dassl are not installed here or on the GPU box, so this module restates
the small part of them the path uses:
  * CfgNode: attribute access, merge_from_file (YAML, safe loader), merge_from_list (key/value
    pairs with literal parsing and the type check yacs applies), clone / freeze / defrost / dump;
  * get_cfg_default(): the Dassl defaults touched by train.py, trainers/maple.py,
    trainers/maple_fed.py and configs/trainers/MaPLeFederated/*.yaml (Dassl itself is un-vendored
    and unpinned: values restated from its published defaults);
  * extend_cfg: train.py:83-138 (TRAINER.COOP/COCOOP/MAPLE/IVLP/VPT, DATASET.SUBSAMPLE_CLASSES, FED);
  * reset_cfg / setup_cfg: train.py:51-80, 140-160.
"""
from __future__ import annotations

import ast
import copy
from typing import Any, Iterable

import yaml


class CfgNode(dict):
    """Minimal yacs.config.CfgNode: nested dict with attribute access and immutability."""

    _FROZEN = "__frozen__"

    def __init__(self, init: dict | None = None):
        super().__init__()
        object.__setattr__(self, CfgNode._FROZEN, False)
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, name: str) -> Any:
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setattr__(self, name: str, value: Any):
        if getattr(self, CfgNode._FROZEN):
            raise AttributeError(f"Attempted to set {name} to {value}, but CfgNode is immutable")
        self[name] = value

    # -- yacs API
    def freeze(self):
        self._set_frozen(True)

    def defrost(self):
        self._set_frozen(False)

    def is_frozen(self) -> bool:
        return getattr(self, CfgNode._FROZEN)

    def _set_frozen(self, flag: bool):
        object.__setattr__(self, CfgNode._FROZEN, flag)
        for v in self.values():
            if isinstance(v, CfgNode):
                v._set_frozen(flag)

    def clone(self) -> "CfgNode":
        c = copy.deepcopy(self)
        return c

    def __deepcopy__(self, memo):
        c = CfgNode()
        for k, v in self.items():
            dict.__setitem__(c, k, copy.deepcopy(v, memo))
        object.__setattr__(c, CfgNode._FROZEN, self.is_frozen())
        return c

    def merge_from_file(self, path: str):
        with open(path) as f:
            data = yaml.safe_load(f) or {}
        self._merge(data, [])

    def merge_from_other_cfg(self, other: "CfgNode"):
        self._merge(other, [])

    def merge_from_list(self, opts: Iterable[Any]):
        opts = list(opts or [])
        if len(opts) % 2:
            raise ValueError(f"Override list has odd length: {opts}; it must be a list of pairs")
        for key, v in zip(opts[0::2], opts[1::2]):
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                if p not in node:
                    raise KeyError(f"Non-existent config key: {key}")
                node = node[p]
            last = parts[-1]
            if last not in node:
                raise KeyError(f"Non-existent config key: {key}")
            node[last] = _check_type(_decode(v), node[last], key)

    def _merge(self, data: dict, path):
        if self.is_frozen():
            raise AttributeError("CfgNode is immutable")
        for k, v in data.items():
            full = ".".join(path + [k])
            if k not in self:
                raise KeyError(f"Non-existent config key: {full}")
            if isinstance(self[k], CfgNode) and isinstance(v, dict):
                self[k]._merge(v, path + [k])
            else:
                self[k] = _check_type(_decode(v), self[k], full)

    def dump(self) -> str:
        def plain(n):
            return {k: plain(v) for k, v in n.items()} if isinstance(n, dict) else (
                list(n) if isinstance(n, tuple) else n)
        return yaml.safe_dump(plain(self), sort_keys=True)

    def __str__(self):
        return self.dump()


def _decode(v: Any) -> Any:
    """yacs' _decode_cfg_value: strings are parsed as Python literals when possible."""
    if isinstance(v, dict):
        return CfgNode(v)
    if not isinstance(v, str):
        return v
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def _check_type(new: Any, old: Any, key: str) -> Any:
    """yacs' _check_and_coerce_cfg_value_type (tuple<->list, int->float and None are allowed)."""
    if old is None or new is None or type(new) is type(old):
        return new
    if isinstance(old, tuple) and isinstance(new, list):
        return tuple(new)
    if isinstance(old, list) and isinstance(new, tuple):
        return list(new)
    if isinstance(old, float) and isinstance(new, int):
        return float(new)
    if isinstance(old, str) and isinstance(new, str):
        return new
    raise ValueError(f"Type mismatch ({type(old)} vs. {type(new)}) with values ({old} vs. {new}) for config key: {key}")


def get_cfg_default() -> CfgNode:
    """The Dassl defaults the federated MaPLe path reads (Dassl.pytorch dassl/config/defaults.py)."""
    C = CfgNode()
    C.OUTPUT_DIR = "./output"
    C.RESUME = ""
    C.SEED = -1
    C.USE_CUDA = True
    C.VERBOSE = True
    C.INPUT = CfgNode(dict(SIZE=(224, 224), INTERPOLATION="bilinear", TRANSFORMS=(), NO_TRANSFORM=False,
                           PIXEL_MEAN=[0.485, 0.456, 0.406], PIXEL_STD=[0.229, 0.224, 0.225],
                           CROP_PADDING=4, RRCROP_SCALE=(0.08, 1.0)))
    C.DATASET = CfgNode(dict(ROOT="", NAME="", SOURCE_DOMAINS=(), TARGET_DOMAINS=(), NUM_LABELED=-1,
                             NUM_SHOTS=-1, VAL_PERCENT=0.1, STL10_FOLD=-1, CIFAR_C_TYPE="", CIFAR_C_LEVEL=1,
                             ALL_AS_UNLABELED=False))
    C.DATALOADER = CfgNode(dict(NUM_WORKERS=4, K_TRANSFORMS=1, RETURN_IMG0=False,
                                TRAIN_X=CfgNode(dict(SAMPLER="RandomSampler", BATCH_SIZE=32, N_DOMAIN=0, N_INS=16)),
                                TRAIN_U=CfgNode(dict(SAME_AS_X=True, SAMPLER="RandomSampler", BATCH_SIZE=32,
                                                     N_DOMAIN=0, N_INS=16)),
                                TEST=CfgNode(dict(SAMPLER="SequentialSampler", BATCH_SIZE=32))))
    C.MODEL = CfgNode(dict(INIT_WEIGHTS="", NUM_CLASSES=0,
                           # PATH (MI355X addition): the local CLIP checkpoint clip._download would fetch for
                           # NAME (trainers/maple.py:21-40); empty -> clip's download cache, else synthetic.
                           # BPE_PATH (MI355X addition): CLIP's bpe_simple_vocab_16e6.txt.gz; empty -> looked
                           # up beside the checkpoint / in ~/.cache/clip (tokenizer.resolve_bpe_path)
                           BACKBONE=CfgNode(dict(NAME="", PRETRAINED=True, PATH="", BPE_PATH="")),
                           HEAD=CfgNode(dict(NAME="", HIDDEN_LAYERS=(), ACTIVATION="relu", BN=True, DROPOUT=0.0))))
    C.OPTIM = CfgNode(dict(NAME="adam", LR=0.0003, WEIGHT_DECAY=5e-4, MOMENTUM=0.9, SGD_DAMPNING=0,
                           SGD_NESTEROV=False, RMSPROP_ALPHA=0.99, ADAM_BETA1=0.9, ADAM_BETA2=0.999,
                           STAGED_LR=False, NEW_LAYERS=(), BASE_LR_MULT=0.1, LR_SCHEDULER="single_step",
                           STEPSIZE=(-1,), GAMMA=0.1, MAX_EPOCH=10, WARMUP_EPOCH=-1, WARMUP_TYPE="linear",
                           WARMUP_CONS_LR=1e-5, WARMUP_MIN_LR=1e-5, WARMUP_RECOUNT=True))
    C.TRAIN = CfgNode(dict(CHECKPOINT_FREQ=0, PRINT_FREQ=10, COUNT_ITER="train_x"))
    C.TEST = CfgNode(dict(EVALUATOR="Classification", PER_CLASS_RESULT=False, COMPUTE_CMAT=False,
                          NO_TEST=False, SPLIT="test", FINAL_MODEL="last_step"))
    C.TRAINER = CfgNode(dict(NAME=""))
    return C


def extend_cfg(cfg: CfgNode) -> None:
    """train.py:83-138."""
    cfg.TRAINER.COOP = CfgNode(dict(N_CTX=16, CSC=False, CTX_INIT="", PREC="fp16", CLASS_TOKEN_POSITION="end"))
    cfg.TRAINER.COCOOP = CfgNode(dict(N_CTX=16, CTX_INIT="", PREC="fp16"))
    # EOT_TRUNCATE (MI355X addition, off by default): run the text tower on the first max(EOT) + 1 tokens
    # only.  The causal mask makes every later position dead for the EOT features and gives it an exactly zero
    # gradient; the truncated tower runs its backward's row reductions over the 77-row layout, so logits, loss,
    # every gradient and the updated weights are bit-identical to the full tower's
    # (tests/test_engine_gpu.py::test_eot_truncated_text_tower_matches_full).
    # EVAL_GROUP (MI355X addition): test() feeds this many TEST.BATCH_SIZE loader batches to one forward of a
    # forward-only engine.  Every product accumulates each output in the same k order whatever the tile, and
    # every other kernel is per row / per head, so a row's logits do not depend on the batch it is in
    # (tests/test_trainers_gpu.py::test_eval_group_counts_bit_identical): larger launches, the same counts.
    cfg.TRAINER.MAPLE = CfgNode(dict(N_CTX=2, CTX_INIT="a photo of a", PREC="fp16", PROMPT_DEPTH=9,
                                     EOT_TRUNCATE=False, EVAL_GROUP=4))
    cfg.DATASET.SUBSAMPLE_CLASSES = "all"
    cfg.TRAINER.IVLP = CfgNode(dict(N_CTX_VISION=2, N_CTX_TEXT=2, CTX_INIT="a photo of a", PREC="fp16",
                                    PROMPT_DEPTH_VISION=9, PROMPT_DEPTH_TEXT=9))
    cfg.TRAINER.VPT = CfgNode(dict(N_CTX_VISION=2, CTX_INIT="a photo of a", PREC="fp16", PROMPT_DEPTH_VISION=1))
    cfg.FED = CfgNode(dict(NUM_CLIENTS=2, NUM_ROUNDS=30, LOCAL_EPOCHS=10,
                           # MI355X additions (federated.py): the bucket exchange -- "ordered" (all_gather +
                           # client-order sum, bit-identical to safe_average_weights) or "allreduce"
                           AGGREGATION="ordered",
                           # size of each client's synthetic test split (no DATASET.ROOT); 0: one test batch
                           SYNTHETIC_TEST_IMAGES=0,
                           # > 0: the synthetic splits repeat that many generated images (bench timing runs)
                           SYNTHETIC_UNIQUE_IMAGES=0))


def reset_cfg(cfg: CfgNode, args) -> None:
    """train.py:51-80."""
    if getattr(args, "root", ""):
        cfg.DATASET.ROOT = args.root
    if getattr(args, "output_dir", ""):
        cfg.OUTPUT_DIR = args.output_dir
    if getattr(args, "resume", ""):
        cfg.RESUME = args.resume
    if getattr(args, "seed", None):
        cfg.SEED = args.seed
    if getattr(args, "source_domains", None):
        cfg.DATASET.SOURCE_DOMAINS = args.source_domains
    if getattr(args, "target_domains", None):
        cfg.DATASET.TARGET_DOMAINS = args.target_domains
    if getattr(args, "transforms", None):
        cfg.INPUT.TRANSFORMS = args.transforms
    if getattr(args, "trainer", ""):
        cfg.TRAINER.NAME = args.trainer
    if getattr(args, "backbone", ""):
        cfg.MODEL.BACKBONE.NAME = args.backbone
    if getattr(args, "head", ""):
        cfg.MODEL.HEAD.NAME = args.head


def setup_cfg(args) -> CfgNode:
    """train.py:140-160: defaults -> extend -> dataset yaml -> method yaml -> CLI args -> opts -> freeze."""
    cfg = get_cfg_default()
    extend_cfg(cfg)
    if getattr(args, "dataset_config_file", ""):
        cfg.merge_from_file(args.dataset_config_file)
    if getattr(args, "config_file", ""):
        cfg.merge_from_file(args.config_file)
    reset_cfg(cfg, args)
    cfg.merge_from_list(getattr(args, "opts", []) or [])
    cfg.freeze()
    return cfg
