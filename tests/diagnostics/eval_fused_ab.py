"""Diagnostic (GPU box): test() over PatternNet's test-split size (9 120 images) with the forward-only eval
engine's in-projection + attention fused (EngineConfig.fused_qkv_attn "both") or not ("none" / the default
"side"), interleaved in one process; prints img/s per pass and checks the accuracy counts agree.

    python tests/diagnostics/eval_fused_ab.py [rounds]
"""
import dataclasses
import sys
import tempfile
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from federated_multi_modal_amd.config import extend_cfg, get_cfg_default  # noqa: E402
from federated_multi_modal_amd.engine import MapleEngine  # noqa: E402
from federated_multi_modal_amd.trainers import build_trainer  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
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
c.test()
B = c._eval_engine.B
engines = {}
for sel in ("side", "both"):
    ecfg = dataclasses.replace(c.engine.cfg, batch=B, inference=True, fused_qkv_attn=sel)
    engines[sel] = MapleEngine(ecfg, device=c.device, shared=c.engine)
print("vision fused:", {k: e.vis.fused_qkv_attn for k, e in engines.items()}, flush=True)
counts = {}
for r in range(rounds):
    for sel, e in engines.items():
        c._eval_engine = e
        torch.cuda.synchronize()
        a = time.perf_counter()
        c.test()
        torch.cuda.synchronize()
        dt = time.perf_counter() - a
        counts.setdefault(sel, c._acc.tolist())
        assert c._acc.tolist() == counts[sel]
        print(f"{sel:5s} {9120 / dt:8.0f} img/s", flush=True)
assert counts["side"] == counts["both"], counts
print("counts identical:", counts["side"])
