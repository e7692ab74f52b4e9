"""Diagnostic (GPU box): sha256 digests of one client step's results, for bit-identity A/B of two trees
(scripts/ab_digest.sh runs this in the repo and in a copy of an earlier commit under _ab/).

Per config (c4: J=9, K=38, B=32; c5: J=9, K=1000, B=32 -- the K = 1 000 head and text tower) one eager
train step from the same synthetic weights and batch, then digests of: the loss, every trainable gradient
(gflat16 / gflat32) and the updated weights (flat16 / flat32).  Equal digests = bit-identical results.
    python tests/diagnostics/step_digest.py [c4] [c5]"""
import hashlib
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

CFG = {"c4": (9, 38, 32), "c5": (9, 1000, 32), "c2": (3, 10, 4)}


def digest(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes()).hexdigest()[:16]


def main():
    dev = torch.device("cuda:0")
    for name in sys.argv[1:] or ["c4", "c5"]:
        J, K, B = CFG[name]
        e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, 0), prompt_depth=J, seed=0),
                        device=dev)
        e.set_lr(0.0026)
        b = syn.client_batch(0, 0, 0, B, K)
        e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
        e.forward_backward()
        torch.cuda.synchronize()
        out = {"loss": digest(e.loss_out[:1]), "gflat16": digest(e.gflat16), "gflat32": digest(e.gflat32)}
        e.optimizer_step()
        torch.cuda.synchronize()
        out.update(flat16=digest(e.flat16), flat32=digest(e.flat32))
        print(name, f"loss={e.loss():.6f}", " ".join(f"{k}={v}" for k, v in out.items()), flush=True)
        del e
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
