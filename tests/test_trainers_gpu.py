"""GPU tier: the reference's trainer API (train.py -> build_trainer -> MaPLeFederated / MaPLe) running
on the MI355X engine: a 2-client, 1-round federated run, FedAvg against the reference's
safe_average_weights, the checkpoint format and the eval-only path (train.py:179-182)."""
import os

import pytest
import torch

from federated_multi_modal_amd.config import get_cfg_default, extend_cfg
from federated_multi_modal_amd.trainers import build_trainer

pytestmark = pytest.mark.gpu


def small_cfg(out, clients=2, rounds=1, epochs=2):
    cfg = get_cfg_default()
    extend_cfg(cfg)
    cfg.merge_from_file("configs/trainers/MaPLeFederated/vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml")
    cfg.merge_from_list(["TRAINER.NAME", "MaPLeFederated", "SEED", 1, "OUTPUT_DIR", str(out),
                         "FED.NUM_CLIENTS", clients, "FED.NUM_ROUNDS", rounds, "FED.LOCAL_EPOCHS", epochs,
                         "MODEL.NUM_CLASSES", 10, "DATASET.NUM_SHOTS", 1, "DATALOADER.TEST.BATCH_SIZE", 12,
                         "TRAINER.MAPLE.PROMPT_DEPTH", 3])
    cfg.freeze()
    return cfg


def test_federated_round_checkpoint_and_eval_only(dev, tmp_path):
    cfg = small_cfg(tmp_path)
    tr = build_trainer(cfg)
    assert len(tr.clients) == 2 and tr.clients[0].engine.K == 10
    res = tr.clients[0].forward_backward(next(iter(tr.clients[0].dm.train_loader)))
    assert isinstance(res["loss"], float) and res["loss"] == res["loss"]
    assert len(tr.clients[0].grad_norms) == 1 and 0.0 < tr.clients[0].grad_norms[0] <= 1.0 + 1e-3
    # FedAvg of two clients == the reference's safe_average_weights on their trainables (bit-exact)
    for c in tr.clients:
        c.run_epoch(0)
    names = tr.clients[0].engine.trainable_names
    snaps = [{n: c.engine.P[n].detach().clone().cpu() for n in names} for c in tr.clients]
    assert not all(torch.equal(snaps[0][n], snaps[1][n]) for n in names)
    n_valid = tr._fedavg([])
    assert n_valid == 2
    ref = tr.safe_average_weights(snaps, 2)
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
    assert "prompt_learner.ctx" in sd["state_dict"] and any(k.startswith("clip_model2.") for k in sd["state_dict"])
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
    assert set(c._graphs) == {False, True}
    assert all(l == l and abs(l) < 1e3 for l in losses)
    assert c.engine.soft_labels is False
    with pytest.raises(ValueError):
        c.forward_backward(dict(batch, label=soft[:, :-1].contiguous()))
