"""The reference's trainer plugin API for the federated MaPLe path, on the MI355X engine.

Mirrors (same class names, registry, method names, return dicts and error behaviour):
  * Dassl's TRAINER_REGISTRY / build_trainer / TrainerX subset used by train.py:177-185
  * MaPLe(TrainerX)            trainers/maple.py:384-716   (one federated client)
  * MaPLeFederated(TrainerX)   trainers/maple_fed.py:24-500 (round loop, FedAvg, checkpoints)

What runs where:
  * every forward/backward/optimizer step is MapleEngine (libmapfed.so kernels), replayed as one
    hipGraph per step; the loss, NaN flags and accuracy counters stay on the device and are read
    once per epoch instead of ~150 host syncs per step (trainers/maple.py:601-615);
  * the LR schedule is Dassl's, evaluated on the host (schedule.py) and handed to the SGD kernel;
  * FedAvg is FedAvgExchange over the clients' FedAvgBuckets: launched with torch.distributed, the
    FED.NUM_CLIENTS clients are split over the ranks in contiguous blocks (one client per GPU when
    WORLD_SIZE == FED.NUM_CLIENTS, several trained one after another per rank otherwise) and exchanged
    over RCCL; launched as one process, the reference's sequential clients (buckets summed in client order).

Error behaviour kept: NaN/Inf loss -> RuntimeError("NaN/Inf in total loss") from run_epoch
(caught per client by the round loop, trainers/maple_fed.py:262-265); non-finite inputs ->
ValueError (trainers/maple.py:526-535, not caught); kernel failures -> RuntimeError (MapfedError).
"""
from __future__ import annotations

import dataclasses
import os
import os.path as osp
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import ops
from .data import DATASET_CLASSES, SyntheticClientDataManager, unified_classnames
from .engine import EngineConfig, MapleEngine
from .federated import FedAvgBucket, FedAvgExchange, FederatedAbort
from .captions import caption_tokens, draw_caption_weights, has_captions
from .modules import CustomCLIP
from .schedule import HostLR
from .tokenizer import BPE_FILE, describe as describe_tokenizer, get_tokenizer, resolve_bpe_path


class Registry:
    """Dassl's Registry: name -> class, `@TRAINER_REGISTRY.register()`."""

    def __init__(self, name: str):
        self.name, self._map = name, {}

    def register(self, obj=None):
        def deco(o):
            if o.__name__ in self._map:
                raise KeyError(f'An object named "{o.__name__}" was already registered in "{self.name}" registry')
            self._map[o.__name__] = o
            return o
        return deco(obj) if obj is not None else deco

    def get(self, name: str):
        if name not in self._map:
            raise KeyError(f'Object name "{name}" does not exist in "{self.name}" registry')
        return self._map[name]

    def registered_names(self):
        return list(self._map)


TRAINER_REGISTRY = Registry("TRAINER")


def build_trainer(cfg):
    """dassl.engine.build_trainer (train.py:177)."""
    return TRAINER_REGISTRY.get(cfg.TRAINER.NAME)(cfg)


def _device(cfg) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("the MI355X trainers need a GPU (libmapfed.so kernels); none is visible")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MAPFED_DIST_BACKEND", "nccl") != "nccl":
        local %= torch.cuda.device_count()  # the gloo rehearsal: several ranks share the box's GPU(s)
    return torch.device("cuda", local)


class TrainerX:
    """The part of Dassl's SimpleTrainer/TrainerX the MaPLe trainers rely on."""

    def __init__(self, cfg):
        self.cfg = cfg
        self._models: Dict[str, object] = {}
        self._optims: Dict[str, object] = {}
        self._scheds: Dict[str, object] = {}
        self.start_epoch = self.epoch = 0
        self.max_epoch = cfg.OPTIM.MAX_EPOCH
        self.output_dir = cfg.OUTPUT_DIR
        if not hasattr(self, "device"):
            self.device = _device(cfg)
        self.build_data_loader()
        self.build_model()

    def build_data_loader(self):
        pass

    def build_model(self):
        raise NotImplementedError

    def register_model(self, name="model", model=None, optim=None, sched=None):
        self._models[name] = model
        self._optims[name] = optim
        self._scheds[name] = sched

    def get_model_names(self, names=None):
        names_real = list(self._models.keys())
        if names is not None:
            names = [names] if isinstance(names, str) else names
            for n in names:
                assert n in names_real
            return names
        return names_real


@TRAINER_REGISTRY.register()
class MaPLe(TrainerX):
    """One federated client (trainers/maple.py:384-716) on one GPU."""

    def __init__(self, cfg, client_id=None, classnames=None, dm=None, device=None):
        self.client_id = client_id
        self.nan_count = 0
        self.total_batches = 0
        self.classnames = classnames
        self.dm = dm
        if device is not None:
            self.device = torch.device(device)
        self.lr_history: List[float] = []
        self.grad_norms: List[float] = []
        # wall seconds by phase (host clock read at the host syncs run_epoch / test() make anyway): local
        # training steps, test() passes, and the FedAvg launch hook run between them (MaPLeFederated.round_times)
        self.timing = {"train_s": 0.0, "test_s": 0.0, "fedavg_launch_s": 0.0, "steps": 0, "epochs": 0}
        self.batch_idx = 0
        self._built = False
        self.check_cfg(cfg)
        super().__init__(cfg)

    def check_cfg(self, cfg):
        assert cfg.TRAINER.MAPLE.PREC in ["fp16", "fp32", "amp"], f"Invalid precision setting: {cfg.TRAINER.MAPLE.PREC}"
        if cfg.TRAINER.MAPLE.PREC != "fp16":
            # the reference crashes for fp32/amp on its own path (hard-coded .half())
            raise NotImplementedError("the MaPLe hot path runs the reference's fp16 precision (PREC=fp16)")

    def build_data_loader(self):
        if self.dm is None:  # standalone client: one synthetic split over the configured classes
            K = self.cfg.MODEL.NUM_CLASSES or len(self.classnames or []) or DATASET_CLASSES["EuroSAT"]
            if self.classnames is None:
                self.classnames = unified_classnames(["EuroSAT"])[:K]
            self.dm = SyntheticClientDataManager(self.client_id or 0, self.classnames, n_train=16 * len(
                self.classnames), n_test=len(self.classnames) * 4, train_batch=self.cfg.DATALOADER.TRAIN_X.BATCH_SIZE,
                test_batch=self.cfg.DATALOADER.TEST.BATCH_SIZE, device=self.device, seed=max(self.cfg.SEED, 0))

    def build_model(self):
        """trainers/maple.py:421-524: CLIP ViT-B/16 + CustomCLIP, freeze policy (:447-479), SGD + LR
        schedule (:498-499).  Backbone: load_clip_to_cpu (:21-40) reads the checkpoint clip._download
        caches for MODEL.BACKBONE.NAME; it is taken from MODEL.BACKBONE.PATH or that cache
        (~/.cache/clip/<file>), else the seeded synthetic CLIP (there is no network).  MODEL.INIT_WEIGHTS
        is then applied on top as Dassl's load_pretrained_weights does (:489-490): a CustomCLIP / MaPLe
        checkpoint loaded by key match (see load_pretrained_weights below)."""
        if self._built:
            return
        cfg = self.cfg
        mcfg = cfg.TRAINER.MAPLE
        classnames = self.classnames
        state, dims = None, None
        backbone = _backbone_file(cfg)
        bpe = resolve_bpe_path(cfg.MODEL.BACKBONE.get("BPE_PATH", "") if hasattr(cfg.MODEL.BACKBONE, "get") else "",
                               backbone)
        tok = get_tokenizer(bpe)
        if self.client_id in (None, 0):
            print(f"[INFO] tokenizer: {describe_tokenizer(tok)}")
            if backbone and tok.kind != "bpe":
                print(f"[WARN] CLIP checkpoint {backbone} with the synthetic tokenizer: put {BPE_FILE} beside it "
                      "or set MODEL.BACKBONE.BPE_PATH, or the prompts do not match CLIP's")
        if backbone:
            state, dims = _load_clip_weights(backbone, cfg, classnames, mcfg, bpe)
        ecfg = EngineConfig(batch=cfg.DATALOADER.TRAIN_X.BATCH_SIZE, classnames=list(classnames),
                            prompt_depth=mcfg.PROMPT_DEPTH, seed=max(cfg.SEED, 0), n_ctx=mcfg.N_CTX,
                            ctx_init=mcfg.CTX_INIT, momentum=cfg.OPTIM.MOMENTUM,
                            weight_decay=cfg.OPTIM.WEIGHT_DECAY, bpe_path=bpe,
                            eot_truncate=bool(mcfg.get("EOT_TRUNCATE", False)))
        if dims is not None:
            ecfg.dims = dims
        if cfg.OPTIM.NAME != "sgd":
            raise NotImplementedError(f"optimizer {cfg.OPTIM.NAME}: the MaPLe configs use sgd")
        self.engine = MapleEngine(ecfg, device=self.device, state=state)
        self._eval_engine: Optional[MapleEngine] = None
        self.model = CustomCLIP(self.engine)  # the reference's module API over the engine (modules.py)
        if cfg.MODEL.INIT_WEIGHTS:
            load_pretrained_weights(self.model, cfg.MODEL.INIT_WEIGHTS)
        self.optim = HostLR(cfg.OPTIM)          # param_groups[0]['lr'] and the scheduler
        self.sched = self.optim.sched
        self.scaler = None
        self.register_model(f"MultiModalPromptLearner_{self.client_id}", self.model, self.optim, self.sched)
        self._graphs = {}
        self._cap_engine: Optional[MapleEngine] = None
        # the caption path's random AttentionPooling / Linear draws (captions.py): a per-client generator in
        # place of the reference's global one, shared by the training step and model(image, label, caption)
        self._cap_gen = torch.Generator().manual_seed(max(cfg.SEED, 0) * 1000 + (self.client_id or 0))
        self.model.caption_generator = self._cap_gen
        self._loss_sum = torch.zeros(1, device=self.device)
        self._bad = torch.zeros(1, device=self.device)
        self._ok = torch.zeros(1, device=self.device)   # steps of the epoch before its first non-finite loss
        self._bad_in = torch.zeros(1, device=self.device)  # the same for non-finite inputs (ValueError)
        self._ok_in = torch.zeros(1, device=self.device)
        self._acc = torch.zeros(2, device=self.device)
        self.lr_history = [self.optim.lr]
        self._built = True

    # ---------------------------------------------------------------- training
    def check_tensor_validity(self, tensor, name):
        """trainers/maple.py:526-535."""
        if tensor is None:
            raise ValueError(f"Null tensor: {name}")
        if not isinstance(tensor, torch.Tensor):
            raise TypeError(f"Invalid tensor type: {name}")
        if tensor.is_floating_point() and not torch.isfinite(tensor).all():
            raise ValueError(f"NaN/Inf values in {name}")

    def parse_batch_train(self, batch):
        return batch["img"], batch["label"], batch.get("caption")

    def _engine_for(self, caption) -> MapleEngine:
        """The training engine for a batch: captions (a list of str, trainers/maple.py:307-322) take the
        caption-conditioned engine (vision sequence growing by B rows per prompted layer; parameters,
        gradients and optimizer state shared with the main engine), with this batch's token ids and a
        fresh draw of the random pooling / projection weights."""
        if not has_captions(caption):
            return self.engine
        if self._cap_engine is None:
            self._cap_engine = MapleEngine(dataclasses.replace(self.engine.cfg, captions=True), device=self.device,
                                           shared=self.engine)
        ce = self._cap_engine
        if all(isinstance(c, str) for c in caption):
            tok = caption_tokens(caption, ce.cfg.dims.context_length, ce.tokenizer)
        else:
            tok = torch.stack([torch.as_tensor(c) for c in caption]).cpu()
        ce.set_captions(tok, draw_caption_weights(self.model.caption_generator))
        return ce

    def _load(self, image, label, e=None):
        e = self.engine if e is None else e
        if image.shape[0] != e.B:
            raise ValueError(f"batch of {image.shape[0]} images; the client engine is built for {e.B}")
        if not label.is_floating_point() and label.device.type == "cpu" and label.numel():
            # trainers/maple.py:352-353 (label sanity); device labels are range-checked by the loss kernels,
            # which flag the step as non-finite instead of indexing out of bounds
            if int(label.min()) < 0 or int(label.max()) >= e.K:
                raise AssertionError("Label index out of bounds")
        e.img_in.copy_(image, non_blocking=True)
        e.set_labels(label)  # float labels -> KL branch (trainers/maple.py:356-360)

    def _step_async(self, batch) -> MapleEngine:
        """One forward_backward without host synchronisation; the loss accumulates on the device.  Returns
        the engine that ran (captioned batches run on the caption engine)."""
        image, label, caption = self.parse_batch_train(batch)
        self.total_batches += 1
        e = self._engine_for(caption)
        self._load(image, label, e)
        e.set_lr(self.optim.lr)
        key = (e.cfg.captions, e.soft_labels)  # one captured step per (caption path, loss branch)
        g = self._graphs.get(key)
        if g is None:
            e.train_step()          # first step of a branch eager (the first one creates the momentum buffers)
            self._graphs[key] = e.capture_train_step()
        else:
            g.replay()
        self._loss_sum.add_(e.loss_out[0:1])
        self._bad.add_(e.loss_out[3:4])
        self._ok.add_((self._bad == 0).float())
        self._bad_in.add_(e.input_flag)
        self._ok_in.add_((self._bad_in == 0).float())
        return e

    def forward_backward(self, batch):
        """trainers/maple.py:547-627: returns {"loss": float} (one host sync, like loss.item()).  A
        non-finite loss raises RuntimeError("NaN/Inf in total loss") with the weights untouched by that
        step (the reference raises before its backward, :375-376)."""
        image, label, _ = self.parse_batch_train(batch)
        self.check_tensor_validity(image, "input image")
        self.check_tensor_validity(label, "input label")
        if not label.is_floating_point() and label.numel():  # trainers/maple.py:352-353
            lo_hi = torch.stack([label.min(), label.max()]).tolist()
            if lo_hi[0] < 0 or lo_hi[1] >= self.engine.K:
                raise AssertionError("Label index out of bounds")
        self.engine.clear_halt()
        e = self._step_async(batch)
        out = e.loss_out.tolist()
        loss = out[0]
        if out[3] != 0.0:
            raise RuntimeError("NaN/Inf in total loss")
        # the grad-norm log of trainers/maple.py:605-612 (norm of the clipped gradients): total * coef
        total, coef = self.engine.clip_out[:2].tolist()
        self.grad_norms.append(total * coef)
        return {"loss": loss}

    def run_epoch(self, epoch, before_test=None):
        """trainers/maple.py:629-653: one pass over the train loader, update_lr, test().

        No host synchronisation per step: the losses and the non-finite flag accumulate on the device
        and are read once after the pass.  A non-finite loss halts the weight updates from that step on
        (MapleEngine.optimizer_step) and raises RuntimeError("NaN/Inf in total loss") here, as the
        reference raises at that step (:375-376, re-raised at :627); total_batches / batch_idx then count
        up to the failing batch.  before_test: called after update_lr, before test() (the federated loop
        starts the FedAvg exchange there so it overlaps the local test)."""
        self.model.train()
        self._loss_sum.zero_()
        for t in (self._bad, self._ok, self._bad_in, self._ok_in):
            t.zero_()
        self.engine.clear_halt()
        steps = 0
        start = self.total_batches
        t0 = time.perf_counter()
        for batch_idx, batch in enumerate(self.dm.train_loader):
            self.batch_idx = batch_idx
            self._step_async(batch)
            steps += 1
        bad, ok, bad_in, ok_in = torch.cat([self._bad, self._ok, self._bad_in, self._ok_in]).tolist()
        t1 = time.perf_counter()  # .tolist() waited for the epoch's last step
        self.timing["train_s"] += t1 - t0
        self.timing["steps"] += steps
        self.timing["epochs"] += 1
        if bad_in != 0.0 and ok_in <= ok:  # check_tensor_validity (trainers/maple.py:556-557): not caught upstream
            self.total_batches = start + int(ok_in) + 1
            self.batch_idx = int(ok_in)
            raise ValueError("NaN/Inf values in input image")
        if bad != 0.0:  # NaN/Inf loss in this epoch (trainers/maple.py:375-376)
            self.total_batches = start + int(ok) + 1
            self.batch_idx = int(ok)
            raise RuntimeError("NaN/Inf in total loss")
        self.update_lr()
        if before_test is not None:
            before_test()
        t2 = time.perf_counter()
        self.timing["fedavg_launch_s"] += t2 - t1
        local = self.test()
        self.timing["test_s"] += time.perf_counter() - t2  # test() ends in a host read of its counters
        avg_loss = float(self._loss_sum.item()) / max(1, steps)
        print(f"[Client {self.client_id}] Epoch {epoch} done. Loss={avg_loss:.4f}, Acc={local['accuracy']:.2f}%")
        return {"avg_loss": avg_loss}

    def update_lr(self):
        if self.sched is not None:
            self.optim.step()
            self.sched = self.optim.sched
            lr = self.optim.lr
            if lr != self.lr_history[-1]:
                self.lr_history.append(lr)

    # ---------------------------------------------------------------- evaluation
    def _evaluator(self, batch_size: int) -> MapleEngine:
        if self._eval_engine is None or self._eval_engine.B != batch_size:
            self._eval_engine = None  # free the old buffers first
            # forward-only: one set of per-block buffers, no gradients (EngineConfig.inference)
            ecfg = dataclasses.replace(self.engine.cfg, batch=batch_size, inference=not self.engine.cfg.captions)
            self._eval_engine = MapleEngine(ecfg, device=self.device, shared=self.engine)
        return self._eval_engine

    def test(self, evaluate_train: bool = False):
        """trainers/maple.py:660-681: accuracy (%) over the test loader; one host sync at the end.

        TRAINER.MAPLE.EVAL_GROUP loader batches go to one forward of the forward-only eval engine (a row's logits
        do not depend on the batch it is in, so the counts are those of batch-by-batch evaluation)."""
        self.model.eval()
        loader = self.dm.test_loader
        group = max(1, int(self.cfg.TRAINER.MAPLE.get("EVAL_GROUP", 1)))
        group = min(group, max(1, len(loader)))
        ev = self._evaluator(loader.batch * group)
        self._acc.zero_()
        # the class-prompt text features depend on the weights only: encoded by the first launch and
        # reused by the rest of the pass (bit-identical)
        reuse = False
        filled, labels = 0, []

        def launch(n):
            nonlocal reuse
            y = labels[0] if len(labels) == 1 else torch.cat(labels)
            if n == ev.B:
                ev.eval_batch(y, self._acc, reuse_text=reuse)
            else:  # ragged last launch: pad the static buffer, count only the real rows
                ev.img_in[n:].zero_()
                logits = ev.forward(reuse_text=reuse)
                ops.argmax_correct(logits[:n], y, None, self._acc)
            reuse = True

        for batch in loader:
            x, y, _ = self.parse_batch_train(batch)
            n = y.numel()
            if filled + n > ev.B:  # (a loader batch never exceeds loader.batch; defensive)
                launch(filled)
                filled, labels = 0, []
            ev.img_in[filled:filled + n].copy_(x)
            labels.append(y)
            filled += n
            if filled == ev.B:
                launch(filled)
                filled, labels = 0, []
        if filled:
            launch(filled)
        correct, total = self._acc.tolist()
        acc = 100.0 * correct / total if total > 0 else 0.0
        print(f"[Client {self.client_id}] Test Accuracy: {acc:.2f}%")
        self.model.train()
        return {"accuracy": acc}

    def load_model(self, directory, epoch=None):
        """trainers/maple.py:685-716."""
        if not directory:
            print("Note that load_model() is skipped as no pretrained model is given")
            return
        model_file = "model-best.pth.tar" if epoch is None else f"model.pth.tar-{epoch}"
        for name in self.get_model_names():
            path = osp.join(directory, name, model_file)
            if not osp.exists(path):
                raise FileNotFoundError(f"Model not found at '{path}'")
            ckpt = torch.load(path, map_location="cpu", weights_only=True)
            sd = ckpt["state_dict"]
            sd.pop("prompt_learner.token_prefix", None)
            sd.pop("prompt_learner.token_suffix", None)
            self._models[name].load_state_dict(sd, strict=False)


_CLIP_FILES = {"ViT-B/16": "ViT-B-16.pt", "ViT-B/32": "ViT-B-32.pt", "ViT-L/14": "ViT-L-14.pt"}


def _backbone_file(cfg) -> str:
    """The CLIP checkpoint load_clip_to_cpu would read (trainers/maple.py:21-40 -> clip._download, whose
    cache is ~/.cache/clip/<basename of the URL>, clip/clip.py:39-44): MODEL.BACKBONE.PATH, else that
    cache file when present, else "" (seeded synthetic CLIP)."""
    path = cfg.MODEL.BACKBONE.get("PATH", "") if hasattr(cfg.MODEL.BACKBONE, "get") else ""
    if path:
        if not osp.isfile(path):
            raise FileNotFoundError(f"MODEL.BACKBONE.PATH {path} not found")
        return path
    name = _CLIP_FILES.get(cfg.MODEL.BACKBONE.NAME)
    if name:
        cached = osp.join(osp.expanduser("~/.cache/clip"), name)
        if osp.isfile(cached):
            return cached
    return ""


def load_pretrained_weights(model, weight_path):
    """Dassl's load_pretrained_weights (called at trainers/maple.py:489-490): read a checkpoint (a dict
    with "state_dict", or a state dict), drop a "module." prefix, keep the keys the model has with the
    same shape, load them; report what was discarded.  Loaded with weights_only=True (no code runs)."""
    ckpt = torch.load(weight_path, map_location="cpu", weights_only=True)
    sd = ckpt["state_dict"] if isinstance(ckpt, dict) and "state_dict" in ckpt else ckpt
    own = model.state_dict()
    matched, discarded = {}, []
    for k, v in sd.items():
        k = k[7:] if k.startswith("module.") else k
        if k in own and tuple(own[k].shape) == tuple(v.shape):
            matched[k] = v
        else:
            discarded.append(k)
    if not matched:
        print(f"Cannot load {weight_path} (check the key names manually)")
        return
    model.load_state_dict(matched, strict=False)
    print(f"Successfully loaded pretrained weights from {weight_path}")
    if discarded:
        print(f"** The following layers are discarded due to unmatched keys or layer size: {discarded[:10]}")


def _load_clip_weights(path, cfg, classnames, mcfg, bpe_path=""):
    """A CLIP checkpoint (load_clip_to_cpu, trainers/maple.py:21-40): the TorchScript archive clip._download
    fetches, or a state dict saved with torch.save -- read by clip_archive.load_clip_state_dict, which
    executes nothing from the file (an allow-listed unpickler over the archive's tensors, or torch.load
    with weights_only=True)."""
    from .clip_archive import load_clip_state_dict
    from .engine import check_dims, clip_dims_from_state_dict, engine_state_from_clip
    sd = load_clip_state_dict(path)
    sd = {k: v.float().numpy() for k, v in sd.items() if k not in ("input_resolution", "context_length", "vocab_size")}
    dims = clip_dims_from_state_dict(sd)  # clip/model.py:750-777
    check_dims(dims)
    ecfg = EngineConfig(batch=1, classnames=list(classnames), prompt_depth=mcfg.PROMPT_DEPTH, seed=max(cfg.SEED, 0),
                        n_ctx=mcfg.N_CTX, ctx_init=mcfg.CTX_INIT, dims=dims, bpe_path=bpe_path)
    return engine_state_from_clip(sd, ecfg), dims


class _ExchangeLaunchError(BaseException):
    """The FedAvg collective failed to launch inside a client's epoch hook.  A BaseException, so the per-client
    handlers of the round loop (which exclude a failed client and exchange again) never see it: the launch is
    not retried on this rank alone, which would leave its peers in mismatched collectives; train() re-raises
    the cause."""


@TRAINER_REGISTRY.register()
class MaPLeFederated(TrainerX):
    """The federated aggregator (trainers/maple_fed.py:24-500).

    Process layout: launched with torch.distributed (backend nccl = RCCL), FED.NUM_CLIENTS must be a
    multiple of WORLD_SIZE: rank r trains clients r*C .. r*C + C - 1 (C = NUM_CLIENTS / WORLD_SIZE) one
    after another on its GPU, as the reference trains all of them on one (trainers/maple_fed.py:247), and
    FedAvg exchanges every rank's C buckets; launched as one process, every client trains on one GPU."""

    CLIENT_DATASETS = ("PatternNet", "Ucmerced", "EuroSAT")

    def __init__(self, cfg):
        self.lab2cname = {}
        self.cfg = cfg
        self.num_clients = cfg.FED.NUM_CLIENTS
        self.num_rounds = cfg.FED.NUM_ROUNDS
        self.local_epochs = cfg.FED.LOCAL_EPOCHS
        self.clients: List[MaPLe] = []
        self.global_weights = None
        self.nan_stats = {"total_updates": 0, "failed_clients": [], "skipped_rounds": 0}
        self.round_times: List[dict] = []  # per round: wall seconds split by phase (train())
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.rank = dist.get_rank() if self.distributed else 0
        if self.distributed and self.num_clients % dist.get_world_size():
            raise ValueError(f"FED.NUM_CLIENTS {self.num_clients} is not a multiple of WORLD_SIZE "
                             f"{dist.get_world_size()}: each rank trains the same number of clients")
        super().__init__(cfg)

    def _local_client_ids(self) -> List[int]:
        """This process's clients: a contiguous block, so [rank][local index] is the global client order the
        ordered FedAvg sums in."""
        if not self.distributed:
            return list(range(self.num_clients))
        per = self.num_clients // dist.get_world_size()
        return list(range(self.rank * per, (self.rank + 1) * per))

    def _disk_datasets(self) -> bool:
        root = self.cfg.DATASET.ROOT
        return bool(root) and all(osp.isdir(osp.join(osp.expanduser(root), d)) for d in ("PatternNet", "Ucmerced",
                                                                                          "eurosat"))

    def build_data_loader(self):
        """trainers/maple_fed.py:48-159: the unified class list over the client datasets, then one data
        manager per client.  With PatternNet / Ucmerced / eurosat under DATASET.ROOT: the disk datasets
        (datasets.py; client 0 = PatternNet, client 1 = UcMerced, as the reference hard-codes), images decoded
        on the host and transformed on the device; otherwise seeded synthetic splits of the same shapes
        (data.py)."""
        if self._disk_datasets():
            from . import datasets as dsets
            if self.num_clients != 2:
                raise ValueError("the disk datasets give the reference's two clients (PatternNet, UcMerced); "
                                 f"FED.NUM_CLIENTS is {self.num_clients}")
            seed = max(self.cfg.SEED, 0)
            loaded = {n: dsets.load_dataset(n, self.cfg.DATASET.ROOT, self.cfg.DATASET.NUM_SHOTS, seed)
                      for n in self.CLIENT_DATASETS}
            names, loaded = dsets.union_and_remap(loaded)
            print(f"[INFO] Unified #classes = {len(names)}")
            self.lab2cname = {i: c for i, c in enumerate(names)}
            self.client_data_managers = {
                i: dsets.client_data_manager(i, names, loaded[("PatternNet", "Ucmerced")[i]], self.cfg, self.device,
                                             seed) for i in self._local_client_ids()}
            self.train_loader_x = self.val_loader = self.test_loader = self.dm = None
            return
        K = self.cfg.MODEL.NUM_CLASSES
        names = unified_classnames(self.CLIENT_DATASETS, max(self.cfg.SEED, 0))
        if K:
            names = names[:K]
        print(f"[INFO] Unified #classes = {len(names)}")
        self.lab2cname = {i: c for i, c in enumerate(names)}
        shots = self.cfg.DATASET.NUM_SHOTS if self.cfg.DATASET.NUM_SHOTS > 0 else 16
        bs = self.cfg.DATALOADER.TRAIN_X.BATCH_SIZE
        get = self.cfg.FED.get if hasattr(self.cfg.FED, "get") else (lambda k, d: d)
        n_test, n_unique = get("SYNTHETIC_TEST_IMAGES", 0), get("SYNTHETIC_UNIQUE_IMAGES", 0)
        self.client_data_managers = {}
        for i in self._local_client_ids():
            self.client_data_managers[i] = SyntheticClientDataManager(
                i, names, n_train=max(bs, min(shots * len(names), 64 * bs)),
                n_test=n_test if n_test > 0 else self.cfg.DATALOADER.TEST.BATCH_SIZE,
                train_batch=bs, test_batch=self.cfg.DATALOADER.TEST.BATCH_SIZE, device=self.device,
                seed=max(self.cfg.SEED, 0), unique_images=n_unique)
        self.train_loader_x = self.val_loader = self.test_loader = self.dm = None

    def build_model(self):
        """trainers/maple_fed.py:164-176."""
        global_classnames = list(self.lab2cname.values())
        self.clients = []
        for i in self._local_client_ids():
            self.clients.append(MaPLe(self.cfg, client_id=i, classnames=global_classnames,
                                      dm=self.client_data_managers[i], device=self.device))
        c0 = self.clients[0]
        self.register_model("MultiModalPromptLearner_Aggregator", c0.model, None, None)
        mode = self.cfg.FED.get("AGGREGATION", "ordered") if hasattr(self.cfg.FED, "get") else "ordered"
        self.fed = [FedAvgBucket(c.engine, mode=mode) for c in self.clients]
        self.exchange = FedAvgExchange(self.fed, mode=mode)
        self.global_weights = self.clients[0].model.state_dict()

    # ---------------------------------------------------------------- round loop
    def train(self):
        """trainers/maple_fed.py:228-303.

        FedAvg overlap: each client's bucket is packed right after its last local epoch's SGD steps and LR
        update, before that epoch's test() (trainers/maple.py:646), which only reads the weights; after the
        rank's last client packs, the exchange (federated.FedAvgExchange) is launched there, flies while the
        test batches run, and is waited for after the client loop.  The result equals the reference's
        FedAvg-after-training order: the test reads the same local weights and the bucket holds them.  A
        client whose test() then raises is still excluded (finish re-exchanges with its vote withdrawn).

        Each round appends its wall time, split by phase, to self.round_times (the FedAvg round wall-time of
        SURVEY.md §8(d): local epochs + tests + exchange); bench.py reports it."""
        try:
            self._train_rounds()
        except _ExchangeLaunchError as err:  # a collective that failed to launch is not a client failure
            raise err.__cause__
        self.finalize_training()

    def _train_rounds(self):
        for round_idx in range(self.num_rounds):
            print(f"\n--- Federated Round {round_idx + 1}/{self.num_rounds} ---")
            t_round = time.perf_counter()
            before = [dict(getattr(c, "timing", {})) for c in self.clients]
            self.broadcast_weights()
            round_losses, late_failed, abort = [], [], None
            n_local = len(self.clients)
            for j, (trainer, fed) in enumerate(zip(self.clients, self.fed)):
                if abort is not None:  # this rank is stopping: its remaining clients only vote "failed"
                    fed.pack(failed=True)
                    if j == n_local - 1:
                        self.exchange.start()
                    continue
                print(f"[Client {trainer.client_id}] local training ...")
                trainer.epoch = round_idx * self.local_epochs
                trainer.max_epoch = (round_idx + 1) * self.local_epochs
                last = 0.0
                started, failed = [], False

                def start_fedavg(fed=fed, started=started, last_local=j == n_local - 1):
                    fed.pack()
                    started.append(True)  # the bucket is out: from here on a failure is a late one
                    if last_local:
                        try:
                            self.exchange.start()
                        except Exception as err:  # never retried as a client failure (peers would mismatch)
                            raise _ExchangeLaunchError() from err
                try:
                    for ep in range(trainer.epoch, trainer.max_epoch):
                        hook = start_fedavg if ep == trainer.max_epoch - 1 else None
                        last = trainer.run_epoch(ep, before_test=hook).get("avg_loss", 0.0)
                    round_losses.append(last)
                except RuntimeError as err:
                    print(f"Client {trainer.client_id} failed training: {err}")
                    self.nan_stats["failed_clients"].append(trainer.client_id)
                    failed = True
                    if started:  # failed in its last test(), after its bucket went out
                        late_failed.append(j)
                except Exception as err:  # not caught by the reference (its process dies): with peers, make
                    if not self.distributed:  # every rank stop at this round's exchange instead of hanging
                        raise
                    abort, failed = err, True
                    if started:
                        late_failed.append(j)
                if not started:  # failed, or no local epochs: pack (excluded when failed) and exchange now
                    fed.pack(failed=failed)
                    if j == n_local - 1:
                        self.exchange.start()
            if round_losses:
                print(f"[Round {round_idx + 1}] Avg local training loss = {sum(round_losses) / len(round_losses):.4f}")
            t_fin = time.perf_counter()
            try:
                n_valid = self._fedavg_finish(late_failed, abort=abort is not None)
            except FederatedAbort:
                if abort is not None:
                    raise abort
                raise
            dev = getattr(self, "device", None)
            if isinstance(dev, torch.device) and dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t_avg = time.perf_counter()
            if n_valid > 0:
                self.nan_stats["total_updates"] += 1
            else:
                print("All clients failed! Reverting to previous global model.")
                self.nan_stats["skipped_rounds"] += 1
            self.global_weights = self.clients[0].model.state_dict()
            t_gt = time.perf_counter()
            if self.rank == 0:
                res = self.clients[0].test()
                print(f"[Round {round_idx + 1}] Test accuracy (client 0) = {res['accuracy']:.2f}%")
            t_end = time.perf_counter()
            d = {k: sum(getattr(c, "timing", {}).get(k, 0) - b.get(k, 0) for c, b in zip(self.clients, before))
                 for k in ("train_s", "test_s", "fedavg_launch_s", "steps", "epochs")}
            rec = {"round": round_idx + 1, "wall_s": t_end - t_round, "local_train_s": d["train_s"],
                   "local_test_s": d["test_s"], "fedavg_launch_s": d["fedavg_launch_s"],
                   # the exchange's wait + unpack after the client loop: what the overlap with the last test() left
                   "fedavg_exposed_s": t_avg - t_fin,
                   "global_state_s": t_gt - t_avg, "global_test_s": t_end - t_gt,
                   "steps": d["steps"], "epochs": d["epochs"], "clients": len(self.clients), "valid": n_valid}
            # broadcast, LR schedule, prints, loader iteration: the round's host time outside the timed phases
            rec["other_s"] = rec["wall_s"] - sum(rec[k] for k in ("local_train_s", "local_test_s", "fedavg_launch_s",
                                                                  "fedavg_exposed_s", "global_state_s",
                                                                  "global_test_s"))
            if not hasattr(self, "round_times"):
                self.round_times = []
            self.round_times.append(rec)

    def _fedavg(self, failed_local) -> int:
        """check_weights_valid + safe_average_weights + broadcast, on the device (federated.py), for
        clients that finished training: pack every local client, exchange, unpack."""
        for c, fed in zip(self.clients, self.fed):
            fed.pack(failed=c.client_id in failed_local)
        self.exchange.start()
        return self._fedavg_finish([])

    def _fedavg_finish(self, late_failed=(), abort: bool = False) -> int:
        """Wait for the exchange the rank's last client started (FedAvgExchange: every client's bucket then
        holds the sum over all clients), unpack into every local client."""
        self.exchange.finish(late_failed, abort=abort)
        for fed in self.fed:
            fed.unpack()
        return self.fed[0].n_valid()

    # ---------------------------------------------------------------- reference utilities
    def safe_average_weights(self, local_dicts, valid_clients=None):
        """trainers/maple_fed.py:309-315 on state dicts (host API; the round loop averages on device)."""
        avg = {}
        for key in local_dicts[0].keys():
            stacked = torch.stack([sd[key].float() for sd in local_dicts])
            stacked = torch.nan_to_num(stacked, nan=0.0, posinf=1e4, neginf=-1e4)
            avg[key] = torch.mean(stacked, dim=0).half()
        return avg

    def check_weights_valid(self, state_dict):
        """trainers/maple_fed.py:317-325."""
        for name, p in state_dict.items():
            if torch.isnan(p).any():
                print(f"NaN in {name}")
                return False
            if torch.isinf(p).any():
                print(f"Inf in {name}")
                return False
        return True

    def broadcast_weights(self, global_sd=None):
        """trainers/maple_fed.py:327-339: load the global weights (already resident on every client after
        the on-device FedAvg unless a state dict is given), drop SGD momentum, rebuild the scheduler
        with last_epoch = epoch - 1."""
        for c in self.clients:
            if global_sd is not None:
                c.model.load_state_dict(global_sd, strict=True)
            c.engine.reset_momentum()
            c.optim.rebuild(getattr(c, "epoch", None))
            c.sched = c.optim.sched

    def finalize_training(self):
        print("\nTraining Summary:")
        print(f"Completed Rounds: {self.nan_stats['total_updates']}")
        print(f"Skipped Rounds: {self.nan_stats['skipped_rounds']}")
        fail_rate = len(self.nan_stats["failed_clients"]) / max(1, self.num_clients)
        print(f"Client Failure Rate: {fail_rate:.1%}")
        if self.rank == 0:
            result = self.clients[0].test()
            print("Final test result:", result)
            self.save_model()

    def save_model(self, epoch=None, directory="", is_best=False, val_result=None):
        """trainers/maple_fed.py:367-386: OUTPUT_DIR/MultiModalPromptLearner_Aggregator/model.pth.tar-<MAX_EPOCH>
        with the fp16 global state dict (Dassl save_checkpoint format)."""
        directory = directory or self.cfg.OUTPUT_DIR
        target = osp.join(directory, "MultiModalPromptLearner_Aggregator")
        os.makedirs(target, exist_ok=True)
        sd = {k: v.detach().half().cpu() for k, v in self.clients[0].model.state_dict().items()}
        ckpt = {"epoch": self.cfg.OPTIM.MAX_EPOCH, "state_dict": sd, "optimizer": None, "scheduler": None,
                "val_result": val_result, "cfg": self.cfg.dump()}
        fpath = osp.join(target, f"model.pth.tar-{self.cfg.OPTIM.MAX_EPOCH}")
        torch.save(ckpt, fpath)
        with open(osp.join(target, "checkpoint"), "w") as f:
            f.write(osp.basename(fpath) + "\n")
        if self.cfg.VERBOSE:
            print(f"Model saved to {target}")
        return fpath

    def load_model(self, directory, epoch=None):
        """trainers/maple_fed.py:388-411."""
        if not directory:
            print("Skipping load_model, no pretrained path given")
            return
        model_file = f"model.pth.tar-{epoch}" if epoch is not None else "model.pth.tar"
        path = osp.join(directory, "MultiModalPromptLearner_Aggregator", model_file)
        if not osp.exists(path):
            raise FileNotFoundError(f"Model not found at {path}")
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        self.global_weights = ckpt["state_dict"]
        print(f"Loaded aggregator weights from '{path}' (epoch={ckpt.get('epoch')}).")
        if self.check_weights_valid(self.global_weights):
            self.broadcast_weights(self.global_weights)
            for fed in getattr(self, "fed", []):
                fed.snapshot()  # an all-failed round now reverts to the loaded weights
            print("Broadcasted loaded global weights.")
        else:
            print("Warning: loaded global weights invalid! Skipping broadcast.")

    def test(self):
        """trainers/maple_fed.py:493-498: evaluate the global model on client 0."""
        if self.rank != 0:
            return {}
        return self.clients[0].test(evaluate_train=True)
