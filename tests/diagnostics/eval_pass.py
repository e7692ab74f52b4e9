"""Diagnostic (GPU box): test() passes of one c4 client over PatternNet's test-split size (9 120 images,
TEST.BATCH_SIZE 100), at TRAINER.MAPLE.EVAL_GROUP values given on the command line; prints img/s per pass.
Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split of an eval pass.

    python tests/diagnostics/eval_pass.py [groups, e.g. 1,4,8] [passes]
"""
import sys
import tempfile
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from federated_multi_modal_amd.config import extend_cfg, get_cfg_default  # noqa: E402
from federated_multi_modal_amd.trainers import build_trainer  # noqa: E402

groups = [int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "1,4").split(",")]
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = get_cfg_default()
extend_cfg(cfg)
cfg.merge_from_file(str(ROOT / "configs/trainers/MaPLeFederated/vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml"))
cfg.merge_from_list(["TRAINER.NAME", "MaPLeFederated", "SEED", 1, "OUTPUT_DIR", tempfile.mkdtemp(), "VERBOSE", False,
                     "FED.NUM_CLIENTS", 1, "FED.NUM_ROUNDS", 1, "FED.LOCAL_EPOCHS", 1, "MODEL.NUM_CLASSES", 38,
                     "DATASET.NUM_SHOTS", 16, "DATALOADER.TRAIN_X.BATCH_SIZE", 32, "FED.SYNTHETIC_TEST_IMAGES", 9120,
                     "FED.SYNTHETIC_UNIQUE_IMAGES", 64, "TRAINER.MAPLE.PROMPT_DEPTH", 9])
cfg.freeze()
tr = build_trainer(cfg)
c = tr.clients[0]
for g in groups:
    c.cfg.defrost()
    c.cfg.TRAINER.MAPLE.EVAL_GROUP = g
    c.cfg.freeze()
    c.test()  # builds the eval engine
    torch.cuda.synchronize()
    for _ in range(passes):
        a = time.perf_counter()
        c.test()
        torch.cuda.synchronize()
        dt = time.perf_counter() - a
        print(f"EVAL_GROUP {g}: {9120 / dt:8.0f} img/s ({dt * 1e3:.1f} ms per pass)", flush=True)
