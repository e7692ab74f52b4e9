"""Diagnostic (GPU box): dump attention forward outputs of the current MAPFED_ATTN_FWD variant for a few
shapes into gpurun_out/attn_dump_v<variant>.npz, and with --compare A B report where two dumps differ."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
SHAPES = [(10, 77, 8, True), (38, 77, 8, True), (32, 199, 12, False)]

if len(sys.argv) > 1 and sys.argv[1] == "--compare":
    a = np.load(ROOT / f"gpurun_out/attn_dump_v{sys.argv[2]}.npz")
    b = np.load(ROOT / f"gpurun_out/attn_dump_v{sys.argv[3]}.npz")
    for (N, L, H, causal) in SHAPES:
        k = f"{N}_{L}_{H}_{int(causal)}"
        oa, ob = a["out_" + k].reshape(N, L, H, 64), b["out_" + k].reshape(N, L, H, 64)
        la, lb = a["lse_" + k].reshape(N, H, L), b["lse_" + k].reshape(N, H, L)
        bad = np.argwhere((oa != ob).any(-1))  # (n, l, h)
        badl = np.argwhere(la != lb)            # (n, h, l)
        print(k, "out rows differing:", len(bad), "lse differing:", len(badl))
        if len(bad):
            ls = sorted(set(int(x) for x in bad[:, 1]))
            print("  query positions:", ls[:40], "..." if len(ls) > 40 else "")
            hs = sorted(set((int(n), int(h)) for n, _, h in bad))
            print("  (seq, head) pairs:", hs[:20], len(hs))
            n, l, h = bad[0]
            print("  first:", (n, l, h), oa[n, l, h, :8], ob[n, l, h, :8])
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, str(ROOT))
from federated_multi_modal_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
res = {}
for (N, L, H, causal) in SHAPES:
    torch.manual_seed(L + N)
    qkv = torch.randn(N * L, 3 * H * 64).half().to(dev)
    out, lse = ops.attention_fwd(qkv, N, L, H, causal)
    torch.cuda.synchronize()
    k = f"{N}_{L}_{H}_{int(causal)}"
    res["out_" + k] = out.cpu().numpy()
    res["lse_" + k] = lse.cpu().numpy()
np.savez(ROOT / f"gpurun_out/attn_dump_v{os.environ.get('MAPFED_ATTN_FWD', 'default')}.npz", **res)
print("dumped")
