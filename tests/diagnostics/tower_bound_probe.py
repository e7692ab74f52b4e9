"""Diagnostic (GPU box): how much of the c4 step the two-stream tower overlap leaves on the table.

Captures the c4 train step as a hipGraph several ways in one process, interleaved over 5 rounds of 20 replays:
  full      -- the product step (text tower on the side stream);
  serial    -- both towers on one stream (overlap_towers = False);
  -text     -- the text tower's forward and backward left out (the vision tower's own critical path);
  -vision   -- the vision tower's forward and backward left out (the text tower alone).
The -text / -vision variants compute wrong numbers (the head reads stale features); they only time the step
without those launches.  full - (-text) is what the text tower costs the step through contention."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

J, K, B, seed = 9, 38, 32, 0
dev = torch.device("cuda:0")
e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, seed), prompt_depth=J, seed=seed),
                device=dev)
e.set_lr(0.0026)
b = syn.client_batch(seed, 0, 0, B, K)
e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
e.train_step()

real = {n: getattr(e, n) for n in ("_text_forward", "_text_backward", "_vision_forward", "_vision_backward")}


def noop(*a, **k):
    return None


def capture(skip=(), overlap=True):
    for n, f in real.items():
        setattr(e, n, noop if n in skip else f)
    e.overlap_towers = overlap
    g = e.capture_train_step()
    for n, f in real.items():
        setattr(e, n, f)
    e.overlap_towers = True
    return g


graphs = {"full": capture(), "serial": capture(overlap=False),
          "-text": capture(("_text_forward", "_text_backward")),
          "-vision": capture(("_vision_forward", "_vision_backward"))}


def cu_masked_stream(every):
    """A HIP stream limited to every `every`-th CU (hipExtStreamCreateWithCUMask), as a torch ExternalStream."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(0, n, every):
        mask[c // 32] |= 1 << (c % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
    return torch.cuda.ExternalStream(st.value, device=dev)


# the text tower on a side stream limited to a quarter / half of the CUs (does the mask survive capture?)
for every in (4, 2):
    try:
        keep = e.side
        e.side = cu_masked_stream(every)
        graphs[f"cumask1/{every}"] = capture()
        e.side = keep
    except Exception as ex:  # noqa: BLE001 -- diagnostic: report and go on
        print(f"cumask 1/{every}: {ex}", flush=True)
        e.side = keep
for g in graphs.values():
    g.replay()
torch.cuda.synchronize()
res = {k: [] for k in graphs}
for rnd in range(5):
    for k, g in graphs.items():
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        res[k].append(1e3 * (time.perf_counter() - a) / 20)
for k in graphs:
    v = sorted(res[k])
    print(f"{k:8s}: median {v[2]:.3f} ms/step, rounds {', '.join(f'{x:.3f}' for x in res[k])}", flush=True)
