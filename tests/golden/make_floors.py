"""The fp16 reproducibility floor of every logit fixture (run in the build container; CPU only).

    python tests/golden/make_floors.py

For each caption-free fixture (tests/golden/case_*.npz) the oracle -- bit-identical to the reference on
this host (tests/test_oracle_golden.py) -- is re-run with ONLY its projection GEMMs computed exactly
(float64 accumulate, one fp16 rounding; tests/test_noise_floor.py): a strictly more accurate
implementation of the same model.  How far its logits move from the reference's, and how far they sit
from the float64 restatement's, is the spread that any correct fp16 implementation with a different
summation order shows on that fixture.  The GPU logit gate (tests/_cases.py logit_gate) is expressed
against it.  Writes tests/golden/floors.json (data)."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parents[1]))

import _cases as C  # noqa: E402
from oracle import maple_oracle as O  # noqa: E402
from test_noise_floor import _block_exact_gemm  # noqa: E402


def floor_of(name: str) -> dict:
    c = C.load_case(name)
    J, K, B, seed, names, batch = C.case_inputs(c)
    M = O.build_model(seed, J, names, tokenizer=C.case_tokenizer(c))
    img = torch.from_numpy(batch.images)
    saved = O._block
    O._block = _block_exact_gemm
    try:
        with torch.no_grad():
            lg = O.forward(M, img, train=False).float().numpy().astype(np.float64)
    finally:
        O._block = saved
    ref, ref64 = c["logits"].astype(np.float64), c["logits64"].astype(np.float64)
    d, e = np.abs(lg - ref), np.abs(lg - ref64)
    return {"exact_vs_ref_max": float(d.max()), "exact_vs_ref_mean": float(d.mean()),
            "exact_vs64_max": float(e.max()), "exact_vs64_mean": float(e.mean()),
            "ref_vs64_max": float(np.abs(ref - ref64).max()), "ref_vs64_mean": float(np.abs(ref - ref64).mean()),
            "rows": int(ref.shape[0]), "classes": int(ref.shape[1])}


def main():
    out = {}
    path = HERE / "floors.json"
    if path.exists():
        out = json.loads(path.read_text())
    for name in C.case_names():
        if name in out and "--all" not in sys.argv:
            continue
        t0 = time.time()
        out[name] = floor_of(name)
        print(f"{name}: {out[name]} ({time.time() - t0:.0f}s)", flush=True)
        path.write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
