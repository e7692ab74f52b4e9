"""CPU tier: the host-side mirror of the reference's config surface (train.py:83-160) and Dassl LR
schedule semantics across federated broadcasts (trainers/maple_fed.py:327-339)."""
import warnings

import pytest

from federated_multi_modal_amd.config import CfgNode, get_cfg_default, extend_cfg, setup_cfg
from federated_multi_modal_amd.schedule import HostLR

FED_YAML = "configs/trainers/MaPLeFederated/vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml"


class Args:
    root = output_dir = resume = trainer = backbone = head = ""
    seed = -1
    source_domains = target_domains = transforms = None
    config_file = FED_YAML
    dataset_config_file = "configs/datasets/PatternNet.yaml"
    eval_only = no_train = False
    opts = []


def test_setup_cfg_defaults_and_overrides():
    a = Args()
    a.trainer = "MaPLeFederated"
    a.seed = 3
    a.opts = ["DATASET.NUM_SHOTS", "16", "FED.NUM_CLIENTS", "8", "TRAINER.MAPLE.PROMPT_DEPTH", "3"]
    cfg = setup_cfg(a)
    assert cfg.TRAINER.NAME == "MaPLeFederated" and cfg.SEED == 3
    assert cfg.DATASET.NAME == "PatternNet" and cfg.DATASET.NUM_SHOTS == 16
    assert cfg.FED.NUM_CLIENTS == 8 and cfg.FED.NUM_ROUNDS == 30 and cfg.FED.LOCAL_EPOCHS == 10
    assert cfg.TRAINER.MAPLE.PROMPT_DEPTH == 3 and cfg.TRAINER.MAPLE.N_CTX == 2
    assert cfg.TRAINER.MAPLE.CTX_INIT == "a photo of a" and cfg.TRAINER.MAPLE.PREC == "fp16"
    assert cfg.OPTIM.LR == 0.0026 and cfg.OPTIM.WARMUP_CONS_LR == 1e-4 and cfg.INPUT.SIZE == (224, 224)
    assert cfg.DATALOADER.TRAIN_X.BATCH_SIZE == 4 and cfg.DATALOADER.TEST.BATCH_SIZE == 100
    with pytest.raises(AttributeError):
        cfg.SEED = 5  # frozen
    c2 = cfg.clone()
    c2.defrost()
    c2.SEED = 5
    assert cfg.SEED == 3 and c2.SEED == 5
    assert "MAPLE" in cfg.dump()


def test_cfg_rejects_unknown_keys_and_bad_types():
    cfg = get_cfg_default()
    extend_cfg(cfg)
    with pytest.raises(KeyError):
        cfg.merge_from_list(["FED.NOT_A_KEY", "1"])
    with pytest.raises(ValueError):
        cfg.merge_from_list(["FED.NUM_CLIENTS", "'two'"])
    with pytest.raises(ValueError):
        cfg.merge_from_list(["FED.NUM_CLIENTS"])


def test_lr_schedule_across_broadcasts():
    """per-epoch LR of the reference's clients with the federated yaml (cosine,
    T_max=MAX_EPOCH=2, 1 constant warm-up epoch at 1e-4, 10 local epochs, scheduler rebuilt with
    last_epoch = epoch-1 at every broadcast)."""
    warnings.filterwarnings("ignore")
    cfg = setup_cfg(Args())
    h = HostLR(cfg.OPTIM)
    epoch, got = 0, []
    for r in range(3):
        h.rebuild(epoch)
        epoch = r * 10
        lrs = []
        for _ in range(10):
            lrs.append(round(h.lr, 7))
            h.step()
        got.append(lrs)
        h.rebuild(epoch)
    r01 = [1e-4, 1e-4, 1e-4, 5e-5, 0.0, 1.3e-3, 2.6e-3, 1.3e-3, 0.0, 1.3e-3]
    r2 = [1e-4, 5e-5, 0.0, 1.3e-3, 2.6e-3, 1.3e-3, 0.0, 1.3e-3, 2.6e-3, 1.3e-3]
    assert got[0] == r01 and got[1] == r01 and got[2] == r2


def test_trainer_registry():
    from federated_multi_modal_amd.trainers import TRAINER_REGISTRY, Registry
    assert {"MaPLe", "MaPLeFederated"} <= set(TRAINER_REGISTRY.registered_names())
    r = Registry("X")

    @r.register()
    class A:
        pass
    with pytest.raises(KeyError):
        r.register()(A)
    with pytest.raises(KeyError):
        r.get("B")
