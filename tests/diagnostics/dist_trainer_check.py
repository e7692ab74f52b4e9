"""The trainer's distributed branch with the real HIP kernels, checked against the reference's FedAvg.

    MAPFED_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29611 tests/diagnostics/dist_trainer_check.py --clients 2 --out gpurun_out/dist_check.json

Every rank builds MaPLeFederated exactly as train.py does (registry, yacs config, synthetic client data),
on the box's one GPU (gloo: RCCL refuses two ranks on one device), and runs one federated round of
MaPLeFederated.train() (trainers/maple_fed.py:228-303) with real engines: J=3, K=10, B=4, one local
epoch.  --clients 4 on 2 ranks trains two clients one after another per rank.  Each client's trainables
are captured at the moment its bucket is packed (its local weights after its last SGD step); afterwards
the ranks gather those snapshots and every rank checks that every one of its clients now holds
oracle.safe_average_weights (the reference's trainers/maple_fed.py:309-315, pinned by
tests/golden/fedavg.npz) of all clients, bit for bit.  Rank 0 writes the verdict as JSON.

Test infrastructure: imports the oracle as the checker only."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    backend = os.environ.get("MAPFED_DIST_BACKEND", "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()

    from federated_multi_modal_amd.config import extend_cfg, get_cfg_default
    from federated_multi_modal_amd.federated import FedAvgBucket
    from federated_multi_modal_amd.trainers import build_trainer
    from oracle import maple_oracle as O

    out_dir = tempfile.mkdtemp(prefix=f"mapfed_dist_{rank}_")
    cfg = get_cfg_default()
    extend_cfg(cfg)
    cfg.merge_from_file(str(ROOT / "configs/trainers/MaPLeFederated/vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml"))
    cfg.merge_from_list(["TRAINER.NAME", "MaPLeFederated", "SEED", 1, "OUTPUT_DIR", out_dir,
                         "FED.NUM_CLIENTS", args.clients, "FED.NUM_ROUNDS", 1, "FED.LOCAL_EPOCHS", 1,
                         "MODEL.NUM_CLASSES", 10, "DATASET.NUM_SHOTS", 1, "DATALOADER.TEST.BATCH_SIZE", 12,
                         "TRAINER.MAPLE.PROMPT_DEPTH", args.depth])
    cfg.freeze()

    captured = {}
    pack = FedAvgBucket.pack

    def capture(self, failed=False):
        captured[id(self)] = None if failed else {n: self.e.P[n].detach().cpu().clone() for n in self.e.trainable_names}
        return pack(self, failed)
    FedAvgBucket.pack = capture

    tr = build_trainer(cfg)
    ids = [c.client_id for c in tr.clients]
    tr.train()
    FedAvgBucket.pack = pack
    torch.cuda.synchronize()

    mine = [(c.client_id, captured[id(f)]) for c, f in zip(tr.clients, tr.fed)]
    every = [None] * world
    dist.all_gather_object(every, mine)
    snaps = dict(kv for part in every for kv in part)
    valid = [snaps[c] for c in sorted(snaps) if snaps[c] is not None]
    ref = O.safe_average_weights(valid)
    bad = []
    for c in tr.clients:
        for n in c.engine.trainable_names:
            got = c.engine.P[n].detach().cpu().float()
            if not torch.equal(got, ref[n].float()):
                bad.append((c.client_id, n, float((got - ref[n].float()).abs().max())))
    # the clients trained on different data: the average is not any one client's weights
    differ = any(not torch.equal(valid[0][n], v[n]) for v in valid[1:] for n in valid[0])
    res = {"rank": rank, "world": world, "clients": ids, "valid_clients": len(valid), "mismatches": bad[:10],
           "n_mismatch": len(bad), "tensors": len(ref), "clients_differ": differ, "ok": not bad and differ,
           "nan_stats": tr.nan_stats}
    allres = [None] * world
    dist.all_gather_object(allres, res)
    if rank == 0:
        verdict = {"check": "MaPLeFederated.train() distributed branch, real HIP kernels, FedAvg vs "
                            "oracle.safe_average_weights (bit-exact)", "backend": backend,
                   "num_clients": args.clients, "prompt_depth": args.depth, "ranks": allres,
                   "ok": all(r["ok"] for r in allres)}
        text = json.dumps(verdict, indent=1)
        print(text)
        if args.out:
            Path(args.out).parent.mkdir(parents=True, exist_ok=True)
            Path(args.out).write_text(text)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if all(r["ok"] for r in allres) else 1)


if __name__ == "__main__":
    main()
