"""The reference-generated parity fixtures (tests/golden/case_*.npz, made by tests/golden/make_golden.py
in the build container by importing the reference's own clip/model.py + trainers/maple.py).

Each case holds the inputs' regeneration keys (seed, client, step, J, K, B; the portable PRNG of
federated_multi_modal_amd/synthetic.py rebuilds weights and images bit-identically on any host) and
the reference's outputs: eval logits, train loss, tower features, and per case optionally every
trainable gradient + the clip/SGD parameter deltas and per-block activation samples of both towers,
each next to the float64 restatement's value (the noise floor)."""
from __future__ import annotations

from pathlib import Path
from typing import Dict, List

import numpy as np

from federated_multi_modal_amd import synthetic as syn

GOLD = Path(__file__).resolve().parent / "golden"
TRACE_SAMPLE = 2048


def case_names() -> List[str]:
    """Caption-free fixtures (eval logits + train loss, optionally gradients and block traces)."""
    return sorted(p.stem[len("case_"):] for p in GOLD.glob("case_*.npz") if not p.stem.startswith("case_cap_"))


def caption_case_names() -> List[str]:
    """Fixtures of the caption-conditioned path (K19): train loss, gradients, growing vision block traces."""
    return sorted(p.stem[len("case_"):] for p in GOLD.glob("case_cap_*.npz"))


def load_case(name: str) -> Dict[str, np.ndarray]:
    return dict(np.load(GOLD / f"case_{name}.npz"))


def case_inputs(c: Dict[str, np.ndarray]):
    """(J, K, B, seed, classnames, ClientBatch) of a case (class names stored in BPE cases, else synthetic)."""
    J, K, B, seed = int(c["J"]), int(c["K"]), int(c["B"]), int(c["seed"])
    names = [str(n) for n in c["classnames"]] if "classnames" in c else syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, int(c["client"]), int(c["step"]), B, K)
    return J, K, B, seed, names, batch


def case_bpe_path(c: Dict[str, np.ndarray]) -> str:
    """The merges file a case was tokenized with ("" = the synthetic word ids)."""
    return str(GOLD / str(c["bpe"])) if "bpe" in c else ""


def case_tokenizer(c: Dict[str, np.ndarray]):
    from federated_multi_modal_amd.tokenizer import get_tokenizer
    return get_tokenizer(case_bpe_path(c))


def trace_idx(case: str, key: str, n: int) -> np.ndarray:
    """Sample positions (flat NLD index) of one traced activation."""
    u = syn.uniform(4321, f"trace/{case}/{key}", TRACE_SAMPLE)
    return np.unique((u * n).astype(np.int64))


def trace_keys(c: Dict[str, np.ndarray]) -> List[str]:
    keys = {k[len("trace/"):-len("/val")] for k in c if k.startswith("trace/") and k.endswith("/val")}
    return sorted(keys, key=lambda k: (k.split("/")[0], int(k.split("/")[1])))


def sel(g, prefix, name, full):
    """(ours, reference) for a packed tensor: full when small, else the fixture's sampled entries."""
    if f"{prefix}full/{name}" in g:
        return full, g[f"{prefix}full/{name}"].astype(np.float64)
    idx = g[f"{prefix}idx/{name}"]
    return full[idx], g[f"{prefix}val/{name}"].astype(np.float64)


def case_floor(name: str) -> Dict[str, float]:
    """The fixture's fp16 reproducibility floor (tests/golden/floors.json, make_floors.py): how far the
    reference's logits move when only its GEMMs are computed exactly, and that variant's distance to float64."""
    import json
    path = GOLD / "floors.json"
    return json.loads(path.read_text()).get(name, {}) if path.exists() else {}


def fp16_ulp(x: np.ndarray) -> np.ndarray:
    """The spacing of fp16 values at |x| (subnormal spacing 2^-24 below 2^-14)."""
    a = np.maximum(np.abs(np.asarray(x, dtype=np.float64)), 2.0 ** -14)
    return np.exp2(np.floor(np.log2(a)) - 10)


def logit_gate(ours: np.ndarray, ref: np.ndarray, ref64: np.ndarray, floor: Dict[str, float] = None):
    """The GPU logit gate.  Two correct fp16 implementations of the model bound it: the
    reference itself and the reference with exactly rounded GEMMs (`floor`, per fixture):
      * max |ours - ref| <= max(4e-3, 1.25 x the exact-GEMM variant's max distance to the reference),
        mean likewise against max(1.5e-3, 1.25 x its mean);
      * max and mean |ours - fp64| <= 1.25 x the larger of the two implementations' own;
      * argmax identical on EVERY row (north_star: class predictions bit-exact; r05: all rows, not only those
        whose top-2 margin exceeds the max gate -- the margin-cleared count is still reported);
      * reported beside the gate: the share of logits within north_star's 1e-3 of the reference
        (`within_1e3`), so the distance to the stated target stays visible next to the floor-relative pass, and
        the error in fp16 ulps of the reference logit (`max_ulps`, `mean_ulps` over |logit| >= 1/4, `within_1ulp`; r06): the
        reference's logits are fp16, and wherever |logit| >= 2 one fp16 ulp (2^-9) already exceeds 1e-3
        (`share_ulp_gt_1e3` = the share of logits where it does).
    Without a floor: 4e-3 / 1.5e-3 and the reference's own fp64 distance.  Returns (ok, report dict)."""
    floor = floor or {}
    ours = ours.astype(np.float64)
    ref = ref.astype(np.float64)
    err = np.abs(ours - ref)
    d64_ours, d64_ref = np.abs(ours - ref64), np.abs(ref - ref64)
    max_gate = max(4e-3, 1.25 * floor.get("exact_vs_ref_max", 0.0))
    mean_gate = max(1.5e-3, 1.25 * floor.get("exact_vs_ref_mean", 0.0))
    e64_max_gate = 1.25 * max(float(d64_ref.max()), floor.get("exact_vs64_max", 0.0))
    e64_mean_gate = 1.25 * max(float(d64_ref.mean()), floor.get("exact_vs64_mean", 0.0))
    top2 = np.sort(ref, 1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > max_gate
    argmax_ok = bool(np.array_equal(ours.argmax(1), ref.argmax(1)))
    rep = dict(max=float(err.max()), mean=float(err.mean()), max_gate=max_gate, mean_gate=mean_gate,
               e64_ours=float(d64_ours.max()), e64_ref=float(d64_ref.max()), e64_max_gate=e64_max_gate,
               e64_mean_ours=float(d64_ours.mean()), e64_mean_ref=float(d64_ref.mean()), e64_mean_gate=e64_mean_gate,
               floor=floor, rows=int(ref.shape[0]), rows_compared=int(clear.sum()), argmax_ok=argmax_ok,
               argmax_all_equal=bool(np.array_equal(ours.argmax(1), ref.argmax(1))),
               argmax_rows_equal=int((ours.argmax(1) == ref.argmax(1)).sum()),
               within_1e3=float((err <= 1e-3).mean()), ref_within_1e3_of64=float((d64_ref <= 1e-3).mean()))
    ulp = fp16_ulp(ref)
    big = np.abs(ref) >= 0.25  # ulps of tiny logits are tiny: there the absolute gate speaks (max_ulps over |ref| >= 1/4)
    ue = err / ulp
    rep.update(max_ulps=float(ue[big].max()) if big.any() else 0.0, mean_ulps=float(ue[big].mean()) if big.any() else 0.0,
               within_1ulp=float((err <= ulp).mean()), share_ulp_gt_1e3=float((ulp > 1e-3).mean()),
               ulp_at_max=float(ulp.flat[int(err.argmax())]))
    ok = (err.max() <= max_gate and err.mean() <= mean_gate and d64_ours.max() <= e64_max_gate
          and d64_ours.mean() <= e64_mean_gate and argmax_ok)
    return ok, rep
