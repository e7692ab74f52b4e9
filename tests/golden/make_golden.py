"""Generate the golden fixtures that pin this build to the reference (run in the build container).

    python tests/golden/make_golden.py

Imports the reference's own clip/model.py + trainers/maple.py + trainers/maple_fed.py (read-only,
/root/reference; see ref_harness.py) and runs it on synthetic weights/inputs from
federated_multi_modal_amd.synthetic, which the GPU box regenerates bit-identically.  Writes small
.npz files next to this script:

  c1_maple.npz   config C1 (J=3, K=10, B=4, ViT-B/16, 12+12 layers):
                 eval logits (fp16) + the float64 restatement's logits (the fp16 noise floor),
                 train loss, every trainable gradient (full for small tensors, norm + a fixed
                 sample of 4096 entries for large ones), the same for the float64 restatement,
                 and the parameter deltas of one clip_grad_norm_(1.0) + SGD step (lr 0.0026).
  fedavg.npz     MaPLeFederated.safe_average_weights on 3 synthetic client state dicts
                 (fp16 and fp32 keys, logit_scale), inputs and outputs.

Only data is written (inputs and expected outputs); no reference source is copied.
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parents[1]))

import ref_harness as h  # noqa: E402
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from oracle import maple_oracle as O  # noqa: E402

SAMPLE = 4096
FULL_MAX = 100_000


def sample_idx(name: str, n: int) -> np.ndarray:
    u = syn.uniform(1234, "sample/" + name, SAMPLE)
    return np.unique((u * n).astype(np.int64))


def pack_tensors(prefix: str, tensors: dict, out: dict):
    for k, t in tensors.items():
        a = t.detach().double().reshape(-1).numpy()
        out[f"{prefix}norm/{k}"] = np.array(np.linalg.norm(a))
        if a.size <= FULL_MAX:
            out[f"{prefix}full/{k}"] = a.astype(np.float32)
        else:
            idx = sample_idx(k, a.size)
            out[f"{prefix}idx/{k}"] = idx
            out[f"{prefix}val/{k}"] = a[idx].astype(np.float32)


def make_c1(seed=0, J=3, K=10, B=4, lr=0.0026):
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, 0, 0, B, K)
    img = torch.from_numpy(batch.images)
    lab = torch.from_numpy(batch.labels)
    t0 = time.time()
    ref = h.build_reference_model(seed, J, names)
    out = {"seed": np.array(seed), "J": np.array(J), "K": np.array(K), "B": np.array(B), "lr": np.array(lr),
           "labels": batch.labels}
    ref.eval()
    with torch.no_grad():
        out["logits"] = ref(img).numpy()
    ref.train()
    loss = ref(img, lab)
    loss.backward()
    out["loss"] = np.array(loss.item(), dtype=np.float32)
    tr = {n: p for n, p in ref.named_parameters() if p.requires_grad}
    grads = {n: p.grad for n, p in tr.items() if p.grad is not None}
    pack_tensors("grad/", grads, out)
    # clip + SGD (torch.optim.SGD is what Dassl's build_optimizer returns; defaults momentum .9 wd 5e-4)
    before = {n: p.detach().clone() for n, p in tr.items()}
    total = torch.nn.utils.clip_grad_norm_([p for p in tr.values()], max_norm=1.0, error_if_nonfinite=False)
    out["total_norm"] = np.array(float(total))
    opt = torch.optim.SGD([p for p in ref.parameters() if p.requires_grad], lr=lr, momentum=0.9,
                          weight_decay=5e-4, dampening=0, nesterov=False)
    opt.step()
    deltas = {n: (p.detach().double() - before[n].double()) for n, p in tr.items() if p.grad is not None}
    pack_tensors("delta/", deltas, out)
    print(f"reference fp16 pass {time.time() - t0:.1f}s  loss {loss.item():.5f}  |g| {float(total):.4f}")

    # float64 restatement (same graph, no fp16 rounding) -> the noise floor
    M64 = O.build_model(seed, J, names, compute_dtype=torch.float64)
    with torch.no_grad():
        out["logits64"] = O.forward(M64, img.double(), train=False).numpy()
    loss64 = O.forward(M64, img.double(), lab, train=True)
    loss64.backward()
    out["loss64"] = np.array(loss64.item())
    g64 = {n: p.grad for n, p in M64.trainable().items() if p.grad is not None}
    pack_tensors("grad64/", g64, out)
    np.savez_compressed(HERE / "c1_maple.npz", **out)
    d = np.abs(out["logits"].astype(np.float64) - out["logits64"]).max()
    print(f"wrote c1_maple.npz: {len(out)} arrays; fp16-vs-fp64 logit gap {d:.2e}")


def make_fedavg(seed=0):
    _, _, maple_fed = h.load_reference()
    rng = lambda n, s, sd: torch.from_numpy(syn.normal(seed, f"fedavg/{n}/{sd}", int(np.prod(s))).reshape(s))
    keys = {"prompt_learner.ctx": ((2, 512), torch.float16), "prompt_learner.compound_prompts_text_parameters.0":
            ((2, 512), torch.float32), "image_encoder.ln_pre.weight": ((768,), torch.float32),
            "image_encoder.transformer.resblocks.11.attn.in_proj_bias": ((2304,), torch.float16),
            "logit_scale": ((), torch.float32)}
    dicts = []
    out = {}
    for c in range(3):
        sd = {}
        for k, (s, dt) in keys.items():
            v = rng(k, s, c) if k != "logit_scale" else torch.tensor(np.log(1 / 0.07))
            sd[k] = v.to(dt)
            out[f"in{c}/{k}"] = sd[k].float().numpy()
        dicts.append(sd)
    avg = maple_fed.MaPLeFederated.safe_average_weights(None, dicts, 3)
    for k, v in avg.items():
        assert v.dtype == torch.float16
        out[f"out/{k}"] = v.float().numpy()
    out["keys"] = np.array(list(keys))
    np.savez_compressed(HERE / "fedavg.npz", **out)
    print("wrote fedavg.npz")


if __name__ == "__main__":
    make_fedavg()
    make_c1()
