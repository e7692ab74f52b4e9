"""GPU tier: the reference's trainer API (train.py -> build_trainer -> MaPLeFederated / MaPLe) running
on the MI355X engine: a 2-client, 1-round federated run, FedAvg against the reference's
safe_average_weights, the checkpoint format and the eval-only path (train.py:179-182)."""
import json
import os
from pathlib import Path

import numpy as np
import pytest
import torch

from federated_multi_modal_amd import synthetic as syn
from federated_multi_modal_amd.config import get_cfg_default, extend_cfg
from federated_multi_modal_amd.trainers import build_trainer
from oracle import maple_oracle as O

GOLD = Path(__file__).resolve().parent / "golden"

pytestmark = pytest.mark.gpu


def small_cfg(out, clients=2, rounds=1, epochs=2, extra=()):
    cfg = get_cfg_default()
    extend_cfg(cfg)
    cfg.merge_from_file("configs/trainers/MaPLeFederated/vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml")
    cfg.merge_from_list(["TRAINER.NAME", "MaPLeFederated", "SEED", 1, "OUTPUT_DIR", str(out),
                         "FED.NUM_CLIENTS", clients, "FED.NUM_ROUNDS", rounds, "FED.LOCAL_EPOCHS", epochs,
                         "MODEL.NUM_CLASSES", 10, "DATASET.NUM_SHOTS", 1, "DATALOADER.TEST.BATCH_SIZE", 12,
                         "TRAINER.MAPLE.PROMPT_DEPTH", 3] + list(extra))
    cfg.freeze()
    return cfg


def test_c3_four_client_round(dev, tmp_path):
    """BASELINE configs[2] (C3: 4 federated clients, EuroSAT-shape 10 classes, J = 9, batch 4) with the four
    clients in one process: a local epoch each, then FedAvg equal to the reference's safe_average_weights (the
    oracle) on the 4 clients' trainables, bit for bit, and every client holding the same global weights.
    The one-client-per-GPU RCCL exchange of the same buckets is covered by tests/test_fedavg_rccl_gpu.py and
    the gloo tests (tests/test_fedavg_dist.py)."""
    cfg = small_cfg(tmp_path, clients=4, epochs=1, extra=["TRAINER.MAPLE.PROMPT_DEPTH", 9])
    tr = build_trainer(cfg)
    assert len(tr.clients) == 4 and tr.clients[0].engine.K == 10 and tr.clients[0].engine.J == 9
    for c in tr.clients:
        c.run_epoch(0)
    names = tr.clients[0].engine.trainable_names
    snaps = [{n: c.engine.P[n].detach().clone().cpu() for n in names} for c in tr.clients]
    assert not all(torch.equal(snaps[0][n], snaps[i][n]) for n in names for i in range(1, 4))  # clients differ
    assert tr._fedavg([]) == 4
    ref = O.safe_average_weights(snaps)
    for n in names:
        for c in tr.clients:
            assert torch.equal(c.engine.P[n].detach().cpu().float(), ref[n].float()), n


def test_federated_round_checkpoint_and_eval_only(dev, tmp_path):
    cfg = small_cfg(tmp_path)
    tr = build_trainer(cfg)
    assert len(tr.clients) == 2 and tr.clients[0].engine.K == 10
    res = tr.clients[0].forward_backward(next(iter(tr.clients[0].dm.train_loader)))
    assert isinstance(res["loss"], float) and res["loss"] == res["loss"]
    assert len(tr.clients[0].grad_norms) == 1 and 0.0 < tr.clients[0].grad_norms[0] <= 1.0 + 1e-3
    # FedAvg of two clients == the reference's safe_average_weights (the oracle, pinned to the reference by
    # tests/golden/fedavg.npz) on their trainables, bit-exact
    for c in tr.clients:
        c.run_epoch(0)
    names = tr.clients[0].engine.trainable_names
    snaps = [{n: c.engine.P[n].detach().clone().cpu() for n in names} for c in tr.clients]
    assert not all(torch.equal(snaps[0][n], snaps[1][n]) for n in names)
    n_valid = tr._fedavg([])
    assert n_valid == 2
    ref = O.safe_average_weights(snaps)
    for n in names:
        for c in tr.clients:
            got = c.engine.P[n].detach().cpu()
            assert torch.equal(got.float(), ref[n].float()), n
    # a full round through train(): checkpoint written in the reference's layout
    tr.train()
    assert tr.nan_stats["total_updates"] == 1 and tr.nan_stats["skipped_rounds"] == 0
    ck = os.path.join(str(tmp_path), "MultiModalPromptLearner_Aggregator", f"model.pth.tar-{cfg.OPTIM.MAX_EPOCH}")
    assert os.path.exists(ck)
    sd = torch.load(ck, map_location="cpu", weights_only=True)
    assert sd["epoch"] == cfg.OPTIM.MAX_EPOCH and sd["optimizer"] is None
    assert all(v.dtype == torch.float16 for v in sd["state_dict"].values())
    # exactly the reference CustomCLIP.state_dict() key set and shapes at J=3 (616 keys incl. the
    # clip_model2.* aliases and clip_model2.token_embedding.weight; tests/golden/state_dict_keys.json,
    # generated from the reference), all fp16 as FedAvg leaves them (trainers/maple_fed.py:314)
    gold = {k: tuple(shape) for k, shape, _ in json.loads((GOLD / "state_dict_keys.json").read_text())["J3"]}
    assert {k: tuple(v.shape) for k, v in sd["state_dict"].items()} == {
        k: (shape if not k.startswith("prompt_learner.token_") else (10,) + shape[1:]) for k, shape in gold.items()}
    tok = sd["state_dict"]["clip_model2.token_embedding.weight"].float().numpy()
    rows = [7, 49406, 12345]
    assert np.array_equal(tok[rows], syn.token_embedding_rows(1, np.array(rows)))
    acc0 = tr.clients[0].test()["accuracy"]
    # eval-only: a fresh aggregator loads the checkpoint and reproduces the accuracy
    tr2 = build_trainer(cfg)
    tr2.load_model(str(tmp_path), epoch=cfg.OPTIM.MAX_EPOCH)
    acc = tr2.test()["accuracy"]
    assert 0.0 <= acc <= 100.0 and acc == acc0


def test_failed_client_is_excluded(dev, tmp_path):
    cfg = small_cfg(tmp_path, epochs=1)
    tr = build_trainer(cfg)
    good = {n: tr.clients[0].engine.P[n].detach().clone() for n in tr.clients[0].engine.trainable_names}
    tr.clients[1].engine.flat32[0] = float("nan")   # client 1 produces invalid weights
    assert tr._fedavg([]) == 1
    for n, v in good.items():  # average of the single valid client = its own weights, fp16-rounded
        assert torch.equal(tr.clients[1].engine.P[n].float(), v.half().float()), n


def test_soft_label_batches_through_the_trainer(dev, tmp_path):
    """A batch with float labels [B, K] (mixup-style soft targets) takes the KL branch of the loss
    (trainers/maple.py:356-360) through the client's forward_backward; each branch gets its own captured
    step, and alternating branches keeps training finite."""
    cfg = small_cfg(tmp_path, clients=1)
    tr = build_trainer(cfg)
    c = tr.clients[0]
    batch = next(iter(c.dm.train_loader))
    B, K = batch["label"].shape[0], c.engine.K
    g = torch.Generator().manual_seed(3)
    soft = torch.rand(B, K, generator=g)
    soft = soft / soft.sum(1, keepdim=True)
    sbatch = dict(batch, label=soft)
    losses = [c.forward_backward(sbatch)["loss"], c.forward_backward(batch)["loss"],
              c.forward_backward(sbatch)["loss"], c.forward_backward(batch)["loss"]]
    assert set(c._graphs) == {(False, False), (False, True)}
    assert all(l == l and abs(l) < 1e3 for l in losses)
    assert c.engine.soft_labels is False
    with pytest.raises(ValueError):
        c.forward_backward(dict(batch, label=soft[:, :-1].contiguous()))


def test_reference_format_checkpoint_strict_load_and_init_weights(dev, tmp_path):
    """A checkpoint with the reference's key set (the aggregator file written by save_model, equal to
    tests/golden/state_dict_keys.json) loads with strict=True (trainers/maple_fed.py:330), and through
    MODEL.INIT_WEIGHTS (Dassl load_pretrained_weights, trainers/maple.py:489-490) into a fresh client:
    every trainable then holds the checkpoint's values."""
    cfg = small_cfg(tmp_path, clients=1, epochs=1)
    tr = build_trainer(cfg)
    tr.train()
    ck = os.path.join(str(tmp_path), "MultiModalPromptLearner_Aggregator", f"model.pth.tar-{cfg.OPTIM.MAX_EPOCH}")
    sd = torch.load(ck, map_location="cpu", weights_only=True)["state_dict"]
    c = tr.clients[0]
    c.model.load_state_dict(sd, strict=True)
    bad = dict(sd)
    bad.pop("clip_model2.token_embedding.weight")
    with pytest.raises(RuntimeError):
        c.model.load_state_dict(bad, strict=True)
    cfg2 = small_cfg(tmp_path / "b", clients=1, epochs=1, extra=["MODEL.INIT_WEIGHTS", ck, "SEED", 2])
    tr2 = build_trainer(cfg2)
    e2 = tr2.clients[0].engine
    for n in e2.trainable_names:
        assert torch.equal(e2.P[n].detach().cpu().float(), sd[n].float()), n
    assert torch.equal(e2.P["image_encoder.conv1.weight"].cpu(), sd["image_encoder.conv1.weight"])


def test_nonfinite_loss_stops_the_epoch_at_its_step(dev, tmp_path):
    """trainers/maple.py:375-376 + :617-627: the first non-finite loss raises RuntimeError out of the epoch
    with the weights as they were before that step; total_batches counts up to the failing batch.  Here
    image 1 of step 2 (of 4) is finite but saturates fp16 (the patch embedding overflows), inside the
    graph-replayed epoch with no per-step host sync.  A NaN input instead raises ValueError
    (check_tensor_validity, :526-535, :556-557), also at its step."""
    cfg = small_cfg(tmp_path, clients=1)
    K = 10
    batches = []
    for s in range(4):
        b = syn.client_batch(1, 0, s, 4, K)
        batches.append({"img": torch.from_numpy(b.images).to(dev), "label": torch.from_numpy(b.labels).to(dev),
                        "caption": [""] * 4})
    overflow = dict(batches[2], img=batches[2]["img"].clone())
    overflow["img"][1] = 60000.0
    nan_in = dict(batches[2], img=batches[2]["img"].clone())
    nan_in["img"][1, 0, 5, 5] = float("nan")

    class DM:
        def __init__(self, base, train):
            self.train_loader, self.test_loader = train, base.test_loader

    tr = build_trainer(cfg)
    c = tr.clients[0]
    base = c.dm
    c.dm = DM(base, batches[:2] + [overflow] + batches[3:])
    with pytest.raises(RuntimeError, match="NaN/Inf in total loss"):
        c.run_epoch(0)
    assert c.total_batches == 3 and c.batch_idx == 2
    got = {n: v.detach().clone() for n, v in c.engine.trainable_state().items()}
    ref_tr = build_trainer(cfg)
    r = ref_tr.clients[0]
    for b in batches[:2]:
        r.forward_backward(b)
    for n, v in r.engine.trainable_state().items():
        assert torch.equal(got[n], v), n
    # the per-batch API raises at the bad batch itself, and the next good batch trains again
    with pytest.raises(RuntimeError, match="NaN/Inf in total loss"):
        r.forward_backward(overflow)
    assert torch.equal(r.engine.flat16, c.engine.flat16) and torch.equal(r.engine.flat32, c.engine.flat32)
    with pytest.raises(ValueError):
        r.forward_backward(nan_in)
    r.forward_backward(batches[3])
    assert not torch.equal(r.engine.flat16, c.engine.flat16)
    with pytest.raises(AssertionError, match="Label index out of bounds"):
        r.forward_backward(dict(batches[3], label=batches[3]["label"].clone().fill_(K)))
    # a NaN image inside an epoch: ValueError at its step, no update from it on
    tr3 = build_trainer(cfg)
    c3 = tr3.clients[0]
    c3.dm = DM(base, batches[:1] + [nan_in] + batches[2:])
    with pytest.raises(ValueError, match="NaN/Inf values in input image"):
        c3.run_epoch(0)
    assert c3.total_batches == 2 and c3.batch_idx == 1


def test_backbone_checkpoint_file(dev, tmp_path):
    """load_clip_to_cpu + build_model (trainers/maple.py:21-40, clip/model.py:750-793) from a CLIP state-dict
    file (MODEL.BACKBONE.PATH; the download is offline): geometry inferred from the tensors, every tower
    parameter equal to the file's tensor in the reference's fp16 / fp32 policy (convert_weights), the
    prompt prefix / suffix rows and ctx taken from the file's token embedding (trainers/maple.py:96-103,
    140-143), CLIP's own logit_scale kept as clip_model2.logit_scale, MaPLe's as ln(1/0.07)."""
    sd = syn.clip_state_dict(7, full_token_table=True)
    sd["logit_scale"] = np.array(4.6052, dtype=np.float32)  # a trained CLIP's value (ln 100)
    half = ("conv1.weight", "in_proj_weight", "in_proj_bias", "out_proj.weight", "out_proj.bias", "c_fc.weight",
            "c_fc.bias", "c_proj.weight", "c_proj.bias", "visual.proj", "text_projection")
    tsd = {k: torch.from_numpy(np.ascontiguousarray(v)).to(torch.float16 if k.endswith(half) else torch.float32)
           for k, v in sd.items()}
    path = tmp_path / "ViT-B-16-state.pt"
    torch.save(tsd, path)
    cfg = small_cfg(tmp_path, clients=1, epochs=1, extra=["MODEL.BACKBONE.PATH", str(path)])
    tr = build_trainer(cfg)
    e = tr.clients[0].engine
    for k, v in tsd.items():
        if k.startswith("visual."):
            name = "image_encoder." + k[7:]
        elif k.startswith("transformer.") or k in ("positional_embedding", "ln_final.weight", "ln_final.bias",
                                                    "text_projection"):
            name = "text_encoder." + k
        else:
            continue
        assert torch.equal(e.P[name].cpu(), v.to(e.P[name].dtype)), name
    tok = e.tokenized
    table = tsd["token_embedding.weight"]
    assert torch.equal(e.token_prefix.cpu(), table[tok[:, :1]].half())
    assert torch.equal(e.token_suffix.cpu(), table[tok[:, 3:]].half())
    init = syn.tokenize(cfg.TRAINER.MAPLE.CTX_INIT)[0, 1:3]
    assert torch.equal(e.P["prompt_learner.ctx"].cpu(), table[torch.from_numpy(init)].half())
    assert abs(float(e.clip_logit_scale) - 4.6052) < 1e-6 and abs(float(e.P["logit_scale"]) - np.log(1 / 0.07)) < 1e-6
    res = tr.clients[0].forward_backward(next(iter(tr.clients[0].dm.train_loader)))
    assert np.isfinite(res["loss"])


def test_captioned_batches_through_the_trainer(dev, tmp_path):
    """Batches with captions (list of str, trainers/maple.py:307-322) take the caption-conditioned path in
    the client's forward_backward and run_epoch (its own captured step); batches without captions the plain
    one; both update the same parameters, and the per-batch loss of a captioned batch equals an engine run
    with the same captions and the same generator draws."""
    from federated_multi_modal_amd.captions import caption_tokens, draw_caption_weights
    from federated_multi_modal_amd.data import SyntheticClientDataManager
    from federated_multi_modal_amd.engine import EngineConfig, MapleEngine
    cfg = small_cfg(tmp_path, clients=1)
    tr = build_trainer(cfg)
    c = tr.clients[0]
    names = c.engine.cfg.classnames
    c.dm = SyntheticClientDataManager(0, names, n_train=8, n_test=4, train_batch=4, test_batch=4, device=dev, seed=1,
                                      captions=True)
    batch = next(iter(c.dm.train_loader))
    assert isinstance(batch["caption"], list) and all(isinstance(x, str) for x in batch["caption"])
    ref = MapleEngine(EngineConfig(batch=4, classnames=names, prompt_depth=3, seed=1, captions=True), device=dev)
    ref.set_captions(caption_tokens(batch["caption"]),
                     draw_caption_weights(torch.Generator().manual_seed(1 * 1000 + 0)))
    ref.load_batch(batch["img"], batch["label"])
    ref.forward_backward()
    loss = c.forward_backward(batch)["loss"]
    assert loss == ref.loss()
    c.run_epoch(0)
    assert (True, False) in c._graphs
    plain = dict(batch, caption=None)
    c.forward_backward(plain)
    assert (False, False) in c._graphs
    assert c._cap_engine.flat16.data_ptr() == c.engine.flat16.data_ptr()


def test_disk_datasets_round(dev, tmp_path):
    """DATASET.ROOT with PatternNet / Ucmerced / eurosat trees (tests/test_datasets.py writes the same
    layout): the aggregator builds the class union (trainers/maple_fed.py:48-159), client 0 trains on
    PatternNet and client 1 on UcMerced images decoded on the host and transformed on the device, their
    captions turn on the caption-conditioned path, and a round completes."""
    import test_datasets as TD
    root = str(tmp_path / "data")
    TD._write_tree(root, "PatternNet/images", ["forest", "parking_lot"], 10, "PatternNet/Captions", size=(64, 80))
    TD._write_tree(root, "Ucmerced/Images", ["forest", "parkinglot", "beach"], 10, "Ucmerced/Captions", size=(72, 64))
    TD._write_tree(root, "eurosat/2750", ["AnnualCrop"], 10, "eurosat/captions", size=(64, 64))
    for k in range(10):
        with open(os.path.join(root, "eurosat/captions/AnnualCrop", f"img_{k:03d}.txt"), "w") as f:
            f.write("field")
    cfg = small_cfg(tmp_path, epochs=1, extra=["DATASET.ROOT", root, "DATASET.NUM_SHOTS", 2,
                                                "DATALOADER.TRAIN_X.BATCH_SIZE", 2, "DATALOADER.TEST.BATCH_SIZE", 4,
                                                "MODEL.NUM_CLASSES", 0])
    tr = build_trainer(cfg)
    assert [c for _, c in sorted(tr.lab2cname.items())] == ["Annual Crop Land", "beach", "forest", "parking_lot"]
    b = next(iter(tr.clients[1].dm.train_loader))
    assert b["img"].shape == (2, 3, 224, 224) and isinstance(b["caption"], list)
    tr.train()
    assert tr.nan_stats["total_updates"] == 1
    assert tr.clients[0]._cap_engine is not None  # captioned batches took the caption path


class _Node(torch.nn.Module):
    def forward(self, x):
        return x


def _torchscript_clip(tsd, path):
    """A TorchScript archive with CLIP's parameter names (what clip._download fetches: a traced module
    tree), written with torch.jit.save from tensors of our own."""
    root = _Node()
    for k, v in tsd.items():
        parts, m = k.split("."), root
        for p in parts[:-1]:
            if p not in m._modules:
                m.add_module(p, _Node())
            m = m._modules[p]
        m.register_parameter(parts[-1], torch.nn.Parameter(v.clone(), requires_grad=False))
    torch.jit.save(torch.jit.trace(root, torch.zeros(1)), str(path))


def test_torchscript_backbone_with_bpe_vocab(dev, tmp_path):
    """MODEL.BACKBONE.PATH pointing at a TorchScript CLIP archive (the official file format; read by
    clip_archive without running it) with CLIP's merges file beside it: the tower weights are the archive's,
    and the class prompts / ctx init are tokenized with the byte-level BPE (trainers/maple.py:96-103,
    136-143): the token ids equal the tokenizer's (pinned to the reference's SimpleTokenizer by
    tests/test_tokenizer.py), the prefix / suffix rows and ctx are those ids' embedding rows."""
    from federated_multi_modal_amd.tokenizer import BPE_FILE, get_tokenizer
    sd = syn.clip_state_dict(11, full_token_table=True)
    half = ("conv1.weight", "in_proj_weight", "in_proj_bias", "out_proj.weight", "out_proj.bias", "c_fc.weight",
            "c_fc.bias", "c_proj.weight", "c_proj.bias", "visual.proj", "text_projection")
    tsd = {k: torch.from_numpy(np.ascontiguousarray(v)).to(torch.float16 if k.endswith(half) else torch.float32)
           for k, v in sd.items()}
    (tmp_path / "ckpt").mkdir()
    path = tmp_path / "ckpt" / "ViT-B-16.pt"
    _torchscript_clip(tsd, path)
    (tmp_path / "ckpt" / BPE_FILE).write_bytes((GOLD / "bpe_small_merges.txt.gz").read_bytes())
    cfg = small_cfg(tmp_path, clients=1, epochs=1, extra=["MODEL.BACKBONE.PATH", str(path)])
    tr = build_trainer(cfg)
    e = tr.clients[0].engine
    assert e.tokenizer.kind == "bpe"
    assert torch.equal(e.P["image_encoder.transformer.resblocks.3.mlp.c_fc.weight"].cpu(),
                       tsd["visual.transformer.resblocks.3.mlp.c_fc.weight"])
    bpe = get_tokenizer(str(tmp_path / "ckpt" / BPE_FILE))
    prompts = [f"a photo of a {c.replace('_', ' ')}." for c in e.cfg.classnames]
    tok = torch.from_numpy(bpe.tokenize(prompts))
    assert torch.equal(e.tokenized, tok)
    table = tsd["token_embedding.weight"]
    assert torch.equal(e.token_prefix.cpu(), table[tok[:, :1]].half())
    assert torch.equal(e.token_suffix.cpu(), table[tok[:, 3:]].half())
    init = torch.from_numpy(bpe.tokenize("a photo of a")[0, 1:3])
    assert torch.equal(e.P["prompt_learner.ctx"].cpu(), table[init].half())
    res = tr.clients[0].forward_backward(next(iter(tr.clients[0].dm.train_loader)))
    assert np.isfinite(res["loss"])


def test_caption_generator_shared_by_trainer_and_module(dev, tmp_path):
    """One source for the caption path's random weights per client: the trainer's training step and
    model(image, label, caption) both draw from model.caption_generator (the client's seeded generator), so
    for the same seed the two entry points compute the same caption weights -- the same loss."""
    from federated_multi_modal_amd.data import SyntheticClientDataManager
    cfg = small_cfg(tmp_path, clients=1)
    tr = build_trainer(cfg)
    c = tr.clients[0]
    assert c.model.caption_generator is c._cap_gen
    c.dm = SyntheticClientDataManager(0, c.engine.cfg.classnames, n_train=4, n_test=4, train_batch=4, test_batch=4,
                                      device=dev, seed=1, captions=True)
    batch = next(iter(c.dm.train_loader))
    state = c._cap_gen.get_state()
    c.engine.clear_halt()
    e = c._engine_for(batch["caption"])
    c._load(batch["img"], batch["label"], e)
    e.forward_backward()
    loss_trainer = e.loss()
    c._cap_gen.set_state(state)
    c.model.train()
    loss_module = float(c.model(batch["img"], batch["label"], batch["caption"]))
    assert abs(loss_module - loss_trainer) <= 1e-6 * max(1.0, abs(loss_trainer))


def test_eot_truncate_config_key(dev, tmp_path):
    """TRAINER.MAPLE.EOT_TRUNCATE (MI355X addition, default off): the client engines run the text tower on
    the first max(EOT) + 1 tokens, and a training step's logits, loss and gradients equal the full 77-token
    tower's bit for bit (the causal mask makes every later position dead for the EOT features; the backward's row
    reductions run over the 77-row layout)."""
    full = build_trainer(small_cfg(tmp_path / "a", clients=1))
    trunc = build_trainer(small_cfg(tmp_path / "b", clients=1, extra=["TRAINER.MAPLE.EOT_TRUNCATE", True]))
    ef, et = full.clients[0].engine, trunc.clients[0].engine
    assert ef.text_len == 77 and et.text_len < 77
    batch = next(iter(full.clients[0].dm.train_loader))
    out = []
    for c in (full.clients[0], trunc.clients[0]):
        c.engine.clear_halt()
        c._load(batch["img"], batch["label"], c.engine)
        c.engine.forward_backward()
        out.append((c.engine.logits.detach().cpu().clone(), c.engine.loss(),
                    {k: v.detach().clone() for k, v in c.engine.grads().items()}))
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
    assert all(torch.equal(out[0][2][k], out[1][2][k]) for k in out[0][2])


def test_eval_group_counts_bit_identical(dev, tmp_path):
    """test() with TRAINER.MAPLE.EVAL_GROUP loader batches per forward of the forward-only eval engine
    (EngineConfig.inference): every row's logits equal those of the training engine's forward at the loader's
    batch size, bit for bit (a ragged last batch included), so the accuracy counts of a test pass are those of
    batch-by-batch evaluation (trainers/maple.py:660-681)."""
    import dataclasses
    from federated_multi_modal_amd.engine import MapleEngine
    cfg = small_cfg(tmp_path, extra=["FED.SYNTHETIC_TEST_IMAGES", 30])
    tr = build_trainer(cfg)
    c = tr.clients[0]
    for _ in range(2):  # weights away from the initial state
        c.forward_backward(next(iter(c.dm.train_loader)))
    X, Y = c.dm.test.images, c.dm.test.labels
    n, b = Y.numel(), c.dm.test_loader.batch
    assert n == 30 and b == 12
    big = MapleEngine(dataclasses.replace(c.engine.cfg, batch=n, inference=True), device=dev, shared=c.engine)
    big.img_in.copy_(X)
    Lb = big.forward().clone()
    small = MapleEngine(dataclasses.replace(c.engine.cfg, batch=b), device=dev, shared=c.engine)
    rows = []
    for s in range(0, n, b):
        small.img_in.zero_()
        small.img_in[:min(b, n - s)].copy_(X[s:s + b])
        rows.append(small.forward().clone()[:min(b, n - s)])
    Ls = torch.cat(rows)
    assert torch.equal(Lb, Ls), (Lb.float() - Ls.float()).abs().max().item()
    accs = []
    for group in (1, 2, 4):
        c.cfg.defrost()
        c.cfg.TRAINER.MAPLE.EVAL_GROUP = group
        c.cfg.freeze()
        res = c.test()
        accs.append((res["accuracy"], c._acc.tolist()))
        assert c._eval_engine.B == b * min(group, 3) and c._eval_engine.cfg.inference
    assert accs[0] == accs[1] == accs[2], accs
    pred = Ls.float().argmax(1)
    assert accs[0][1] == [float((pred == Y).sum().item()), float(n)]
