"""Drop-in for the reference's train.py (train.py:163-242): same flags, same config assembly, the
MI355X trainers (federated_multi_modal_amd.trainers) behind the same registry names.

    python train.py --trainer MaPLeFederated --config-file configs/trainers/MaPLeFederated/\\
        vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml --dataset-config-file configs/datasets/PatternNet.yaml \\
        --output-dir out/ [KEY VALUE ...]
    # one federated client per GPU (RCCL FedAvg):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ... FED.NUM_CLIENTS 8
"""
import argparse
import os
import random
import sys

import numpy as np
import torch

from federated_multi_modal_amd.config import setup_cfg
from federated_multi_modal_amd.trainers import build_trainer


def set_random_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


class _Tee:
    """Dassl setup_logger: stdout also goes to OUTPUT_DIR/log.txt."""

    def __init__(self, path):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self.f = open(path, "a")
        self.out = sys.stdout

    def write(self, s):
        self.out.write(s)
        self.f.write(s)

    def flush(self):
        self.out.flush()
        self.f.flush()


def main(args):
    cfg = setup_cfg(args)
    if cfg.SEED >= 0:
        print("Setting fixed seed: {}".format(cfg.SEED))
        set_random_seed(cfg.SEED)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not torch.distributed.is_initialized():
        # one rank per GPU over RCCL; MAPFED_DIST_BACKEND=gloo rehearses several ranks on one GPU
        backend = os.environ.get("MAPFED_DIST_BACKEND", "nccl")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if backend != "nccl":
            local %= max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    if int(os.environ.get("RANK", "0")) == 0:
        sys.stdout = _Tee(os.path.join(cfg.OUTPUT_DIR, "log.txt"))
    print(cfg)
    trainer = build_trainer(cfg)
    if args.eval_only:
        trainer.load_model(args.model_dir, epoch=args.load_epoch)
        trainer.test()
        return
    if not args.no_train:
        trainer.train()


def get_parser():
    p = argparse.ArgumentParser()
    p.add_argument("--root", type=str, default="", help="path to dataset")
    p.add_argument("--output-dir", type=str, default="", help="output directory")
    p.add_argument("--resume", type=str, default="", help="checkpoint directory (from which the training resumes)")
    p.add_argument("--seed", type=int, default=-1, help="only positive value enables a fixed seed")
    p.add_argument("--source-domains", type=str, nargs="+", help="source domains for DA/DG")
    p.add_argument("--target-domains", type=str, nargs="+", help="target domains for DA/DG")
    p.add_argument("--transforms", type=str, nargs="+", help="data augmentation methods")
    p.add_argument("--config-file", type=str, default="", help="path to config file")
    p.add_argument("--dataset-config-file", type=str, default="", help="path to config file for dataset setup")
    p.add_argument("--trainer", type=str, default="", help="name of trainer")
    p.add_argument("--backbone", type=str, default="", help="name of CNN backbone")
    p.add_argument("--head", type=str, default="", help="name of head")
    p.add_argument("--eval-only", action="store_true", help="evaluation only")
    p.add_argument("--model-dir", type=str, default="", help="load model from this directory for eval-only mode")
    p.add_argument("--load-epoch", type=int, help="load model weights at this epoch for evaluation")
    p.add_argument("--no-train", action="store_true", help="do not call trainer.train()")
    p.add_argument("opts", default=None, nargs=argparse.REMAINDER, help="modify config options using the command-line")
    return p


if __name__ == "__main__":
    main(get_parser().parse_args())
