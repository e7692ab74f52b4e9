"""Benchmark: federated MaPLe client step (ViT-B/16 + text transformer, deep coupled V-L prompts,
fwd + bwd + clip_grad_norm_ + SGD) on N MI355X, one client per GPU, FedAvg over RCCL at round end.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One timed "round" = K local steps on every client (one hipGraph replay each, inputs resident in HBM)
followed by one FedAvg (validity scan + pack + all-reduce + fp16 unpack).  value = images all
clients processed / max-over-ranks wall time.  Prints ONE JSON line on rank 0.

Workload (BASELINE.json configs): default c4 = per client B=32, K=38 classes (PatternNet shape),
J=9 prompt depth, the configuration the metric's 1/2/4/8-client scaling is quoted on (configs[3]);
c2 = configs[1] (J=3, K=10, B=4) is the numerics-gate config, selectable with --config c2.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from federated_multi_modal_amd import ops  # noqa: E402
from federated_multi_modal_amd import synthetic as syn  # noqa: E402
from federated_multi_modal_amd.captions import caption_tokens, draw_caption_weights  # noqa: E402
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402
from federated_multi_modal_amd.federated import FedAvgBucket  # noqa: E402

CONFIGS = {
    # name: (J, K, B, description)
    "c2": (3, 10, 4, "MaPLe ViT-B/16, 2 prompt tokens, J=3, 10-class synthetic 224x224, batch=4 (configs[1])"),
    "c3": (9, 10, 4, "EuroSAT-shape 10-class synthetic, J=9, batch=4 per client (configs[2])"),
    "c4": (9, 38, 32, "PatternNet-shape 38-class synthetic, J=9, batch=32 per client (configs[3])"),
    "c5": (9, 1000, 32, "ImageNet-shape 1000-class text side, 77-token prompts, J=9, batch=32 (configs[4])"),
}
FLOP_PER_IMAGE = 75.04e9   # vision fwd 35.50 + bwd 39.54 GFLOP
FLOP_PER_CLASS = 12.55e9   # text fwd 5.96 + bwd 6.59 GFLOP
MFMA_PEAK_F16 = 2.5e15     # MI355X dense fp16 (MI355X_MICROARCH.md: 1024 flop/clk/SIMD x 1024 SIMD x 2.4 GHz)
HBM_PEAK = 8.0e12


def text_flop_per_class(L, D=512, layers=12):
    """Executed text-tower FLOP per class at L tokens (SURVEY.md §8(d) formulas; L = 77 gives 12.55 G)."""
    fwd = layers * (24 * L * D * D + 4 * L * L * D) + 2 * D * D
    bwd = layers * (24 * L * D * D + 8 * L * L * D) + 24 * L * D * D
    return fwd + bwd


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(J, K, B, budget_s=30.0, seed=0):
    """The oracle (CPU restatement of the reference, oracle/maple_oracle.py; bit-identical to the
    reference on the same host) timed on the host cores: forward + backward + clip + SGD of one
    client step.  Bounded sample: ONE image and ONE class prompt per step (B=1, K=1, same J) --
    87.6 GFLOP per image against the workload's (B*75.04 + K*12.55)/B GFLOP per image (89.9 at c4),
    so images/s transfers to the workload's unit; steps are repeated until `budget_s` of CPU time or
    3 steps.  (The reference's fp16 backward GEMMs run at < 1 GFLOP/s on AMD EPYC hosts: one full
    c4 step would take many minutes there.)"""
    from oracle import maple_oracle as O
    Bs, Ks = 1, 1
    names = syn.synthetic_classnames(Ks, seed)
    M = O.build_model(seed, J, names)
    opt = O.SGDState(lr=0.0026)
    b = syn.client_batch(seed, 0, 0, Bs, Ks)
    img, lab = torch.from_numpy(b.images), torch.from_numpy(b.labels)
    ts = []
    t_all = time.perf_counter()
    # one warm-up step, then at least 3 timed steps, more while the budget lasts
    while len(ts) < 4 or (time.perf_counter() - t_all) < budget_s:
        t0 = time.perf_counter()
        O.train_step(M, img, lab, opt)
        ts.append(time.perf_counter() - t0)
        log(f"[bench] cpu step {len(ts)}: {ts[-1]:.1f}s")
        if len(ts) >= 8:
            break
    sec = float(np.median(ts[1:]))
    return {"value": Bs / sec, "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": cpu_model(),
            "steps_timed": len(ts) - 1,
            "sample": f"{len(ts)} steps of one client at J={J}, B=1 image, K=1 class prompt "
                      f"({sec:.2f} s/step, median of the {len(ts) - 1} after the first), torch-CPU fp16 "
                      f"oracle, {torch.get_num_threads()} threads of {cpu_model()}; workload per-image work 87.6 vs "
                      f"{(B * FLOP_PER_IMAGE + K * FLOP_PER_CLASS) / B / 1e9:.1f} GFLOP"}


def side_config(name, dev, world, rank, steps=5, warmup=2, seed=0, eot_truncate=False, probe_gemm=True):
    """Another BASELINE config on the same ranks, reported beside `value` (never as it): the graph-replayed
    client step (fwd + bwd + clip + SGD) timed over `steps` steps (max over ranks), and the GEMM family
    split by tower from one probed eager step (HIP events around every launch, towers serialised).
    eot_truncate: the text tower on the first max(EOT)+1 tokens (the optional mode, never the value)."""
    J, K, B, desc = CONFIGS[name]
    names = syn.synthetic_classnames(K, seed)
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=eot_truncate),
                    device=dev)
    e.set_lr(0.0026)
    cb = syn.client_batch(seed, rank, 0, B, K)
    e.img_in.copy_(torch.from_numpy(cb.images))
    e.label_in.copy_(torch.from_numpy(cb.labels))
    e.train_step()
    g = e.capture_train_step()
    for _ in range(warmup):
        g.replay()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - a
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    loss = e.loss()
    fam = {}
    if probe_gemm:
        probe = ops.KernelProbe("gemm")
        e.overlap_towers = False
        ops.set_probe(probe)
        e.train_step()
        ops.set_probe(None)
        for tower in ("text", "vision"):
            p = probe.summary(f"gemm/{tower}")
            fam[tower] = {"launches": p["launches"], "avg_launch_us": p["avg_us"], "tflops": p["tflops"],
                          "mfma_frac": p["tflops"] * 1e12 / MFMA_PEAK_F16, "flop_per_launch": p["flops_per_launch"]}
    step_flop = B * FLOP_PER_IMAGE + K * FLOP_PER_CLASS
    # FLOP the step executes: the algorithmic count, except with the EOT-truncated text tower, whose rate and
    # MFMA fraction are priced on what it runs (no fraction counts FLOP that did not execute)
    exec_flop = B * FLOP_PER_IMAGE + K * text_flop_per_class(e.text_len)
    out = {"workload": f"{name}: {desc}", "value": world * B * steps / el, "unit": "images/s",
           "ms_per_step": 1e3 * el / steps, "steps": steps, "loss": loss,
           "model_tflops": world * exec_flop * steps / el / 1e12,
           "model_mfma_frac": exec_flop * steps / el / MFMA_PEAK_F16, "gemm_by_tower": fam or None}
    if eot_truncate:
        Lt = e.text_len
        out.update(text_tokens=Lt, executed_gflop_per_step=exec_flop / 1e9,
                   algorithmic_gflop_per_step=step_flop / 1e9,
                   flop_basis="model_tflops / model_mfma_frac: executed FLOP (text tower on text_tokens rows)",
                   parity="bit-identical to the 77-token tower: logits, loss, every gradient and the updated "
                          "weights (tests/test_engine_gpu.py::test_eot_truncated_text_tower_matches_full)")
    del g, e
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


# PatternNet's test split: 30 % of its 38 x 800 images (datasets/patternnet.py:33, 66-72 of the reference: 50 % train,
# 20 % val, the rest test, unshuffled), which the reference's client evaluates after every local epoch
PATTERNNET_TEST_IMAGES = 38 * 800 - int(0.5 * 38 * 800) - int(0.2 * 38 * 800)


def fed_round_wall(name, world, rank, epochs=10, test_images=1000, shots=16, seed=1, eval_group=None):
    """The metric's second half, the FedAvg round wall-time (local epochs + tests +
    exchange), through the reference's trainer API: MaPLeFederated.train() (trainers/maple_fed.py:228-303)
    with one client per rank, FED.LOCAL_EPOCHS local epochs per round, each epoch a pass over the client's
    `shots`-shot train split followed by test() over `test_images` images (trainers/maple.py:629-681), then
    the FedAvg exchange (started before the last test()), the global-state read and client 0's round test.
    Two rounds run; round 2 is reported (round 1 also captures the step graphs and builds the eval engine).
    Synthetic splits repeat 64 generated images (the host PRNG stays out of the run; the device work per
    batch is the same).  Times are host wall seconds, max over ranks; the trainer reads them at the host
    syncs it makes anyway (MaPLeFederated.round_times)."""
    import contextlib
    import io
    import tempfile
    from federated_multi_modal_amd.config import extend_cfg, get_cfg_default
    from federated_multi_modal_amd.trainers import build_trainer
    J, K, B, desc = CONFIGS[name]
    cfg = get_cfg_default()
    extend_cfg(cfg)
    cfg.merge_from_file(str(ROOT / "configs/trainers/MaPLeFederated/vit_b16_c2_ep5_batch4_2ctx_cross_datasets.yaml"))
    out_dir = tempfile.mkdtemp(prefix="mapfed_round_")
    cfg.merge_from_list(["TRAINER.NAME", "MaPLeFederated", "SEED", seed, "OUTPUT_DIR", out_dir, "VERBOSE", False,
                         "FED.NUM_CLIENTS", world, "FED.NUM_ROUNDS", 2, "FED.LOCAL_EPOCHS", epochs,
                         "MODEL.NUM_CLASSES", K, "DATASET.NUM_SHOTS", shots, "DATALOADER.TRAIN_X.BATCH_SIZE", B,
                         "FED.SYNTHETIC_TEST_IMAGES", test_images, "FED.SYNTHETIC_UNIQUE_IMAGES", 64,
                         "TRAINER.MAPLE.PROMPT_DEPTH", J]
                        + (["TRAINER.MAPLE.EVAL_GROUP", eval_group] if eval_group is not None else []))
    cfg.freeze()
    with contextlib.redirect_stdout(io.StringIO()):  # the trainer's per-epoch prints (stdout carries the JSON line)
        tr = build_trainer(cfg)
        tr.train()
    rec = dict(tr.round_times[-1])
    keys = [k for k, v in rec.items() if k.endswith("_s")]
    if world > 1:
        t = torch.tensor([rec[k] for k in keys], device=tr.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rec.update(zip(keys, t.tolist()))
    c0 = tr.clients[0]
    n_train = len(c0.dm.train_loader) * B
    out = {"workload": f"{name}: {desc}; {shots}-shot train split ({n_train} images, {len(c0.dm.train_loader)} "
                       f"steps per epoch), {test_images}-image test split in batches of "
                       f"{cfg.DATALOADER.TEST.BATCH_SIZE} ({cfg.TRAINER.MAPLE.EVAL_GROUP} per forward-only eval launch), "
                       f"{epochs} local epochs, {world} client(s), one per rank",
           "round_wall_s": rec["wall_s"],
           "split_s": {k: rec[k] for k in keys if k != "wall_s"},
           "steps": rec["steps"], "train_ms_per_step": 1e3 * rec["local_train_s"] / max(rec["steps"], 1),
           "test_images_per_s": epochs * test_images * len(tr.clients) / max(rec["local_test_s"], 1e-9),
           "valid_clients": rec["valid"], "round": rec["round"],
           "note": "max over ranks per phase; local_train_s = the graph-replayed client steps of all local epochs "
                   "(one host sync per epoch), local_test_s = the per-epoch test() passes (text features encoded once "
                   "per pass), fedavg_exposed_s = the exchange's wait + unpack after the client loop"}
    del tr
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a hipGraph")
    ap.add_argument("--cpu-budget", type=float, default=30.0, help="seconds of CPU-baseline sampling")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-kernel", default="gemm", choices=["gemm", "attention_fwd"])
    ap.add_argument("--no-eot-mode", action="store_true", help="skip the separately reported EOT-truncated run")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (K=1000 text side) side metric")
    ap.add_argument("--no-caption-mode", action="store_true", help="skip the caption-batch (K19) side metric")
    ap.add_argument("--no-round", action="store_true", help="skip the FedAvg round wall-time (trainer) runs")
    ap.add_argument("--no-eval", action="store_true",
                    help="skip the eval-rate side metrics (keeps a kernel profile of the run to the training step's mix)")
    # engine options (EngineConfig; results bit-identical, for same-box A/B: scripts/bench_ab.sh)
    ap.add_argument("--fused-qkv-attn", default="side", choices=["side", "none", "both", "vision", "text"])
    ap.add_argument("--text-first", action="store_true", help="enqueue the text tower first after each fork")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MAPFED_DIST_BACKEND", "nccl") != "nccl":
        local %= max(torch.cuda.device_count(), 1)  # rehearsal: ranks share the box's GPU(s)
    if world > 1:
        torch.cuda.set_device(local)
        # MAPFED_DIST_BACKEND=gloo: rehearse the multi-rank path with several ranks on one GPU (RCCL refuses
        # two ranks on one device); the driver's runs use RCCL, one rank per GPU
        backend = os.environ.get("MAPFED_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    J, K, B, desc = CONFIGS[args.config]
    seed = 0

    t0 = time.time()
    names = syn.synthetic_classnames(K, seed)
    eng = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed,
                                   fused_qkv_attn=args.fused_qkv_attn, vision_first=not args.text_first), device=dev)
    eng.set_lr(0.0026)
    # two resident synthetic batches per client (client id = rank), alternated step to step
    batches = []
    for s in range(2):
        cb = syn.client_batch(seed, rank, s, B, K)
        batches.append((torch.from_numpy(cb.images).to(dev), torch.from_numpy(cb.labels).to(dev)))
    fed = FedAvgBucket(eng)
    log(f"[bench] engine built in {time.time() - t0:.1f}s (config {args.config}, J={J} K={K} B={B}, world {world})")

    def load(i):
        img, lab = batches[i % 2]
        eng.img_in.copy_(img)
        eng.label_in.copy_(lab)

    if args.no_graph:
        def step():
            eng.train_step()
    else:
        load(0)
        eng.train_step()  # first step eager (creates the momentum buffers: first_step flag)
        graph = eng.capture_train_step()

        def step():
            graph.replay()

    for i in range(args.warmup):
        load(i)
        step()
    torch.cuda.synchronize()
    loss_w = eng.loss()  # also the NaN/Inf check of trainers/maple.py:375-376

    # ---------------- timed region: K local steps + one FedAvg round end
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        load(i)
        step()
    fed.start()
    fed.finish()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = eng.loss()

    # ---------------- optional mode, reported separately: the text tower on the first
    # max(EOT)+1 tokens (bit-identical logits; engine.EngineConfig.eot_truncate).  Same protocol: K graph
    # steps + one FedAvg, max over ranks; the headline `value` above stays the reference's 77 tokens.
    eot_mode = None
    if not args.no_eot_mode:
        eng_t = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=True),
                            device=dev)
        eng_t.set_lr(0.0026)
        fed_t = FedAvgBucket(eng_t)

        def load_t(i):
            img, lab = batches[i % 2]
            eng_t.img_in.copy_(img)
            eng_t.label_in.copy_(lab)

        load_t(0)
        eng_t.train_step()
        graph_t = eng_t.capture_train_step()
        for i in range(args.warmup):
            load_t(i)
            graph_t.replay()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        a = time.perf_counter()
        for i in range(args.steps):
            load_t(i)
            graph_t.replay()
        fed_t.start()
        fed_t.finish()
        torch.cuda.synchronize()
        el_t = time.perf_counter() - a
        if world > 1:
            t = torch.tensor([el_t], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_t = float(t.item())
        Lt = eng_t.text_len
        exec_flop_t = B * FLOP_PER_IMAGE + K * text_flop_per_class(Lt)
        eot_mode = {"value": world * B * args.steps / el_t, "unit": "images/s", "ms_per_step": 1e3 * el_t / args.steps,
                    "text_tokens": Lt, "loss": eng_t.loss(),
                    "model_tflops": world * exec_flop_t * args.steps / el_t / 1e12,
                    "model_mfma_frac": exec_flop_t * args.steps / el_t / MFMA_PEAK_F16,
                    "flop_basis": "model_tflops / model_mfma_frac: executed FLOP (text tower on text_tokens rows)",
                    "executed_gflop_per_step": exec_flop_t / 1e9,
                    "algorithmic_gflop_per_step": (B * FLOP_PER_IMAGE + K * FLOP_PER_CLASS) / 1e9,
                    "parity": "bit-identical to the 77-token tower: logits, loss, every gradient and the updated "
                              "weights (tests/test_engine_gpu.py::test_eot_truncated_text_tower_matches_full); the "
                              "backward's row reductions run over the 77-row layout (mf_layernorm_bwd_live, "
                              "mf_seq_scatter)",
                    # live check: this run and the `value` run took the same steps from the same seed and batches
                    "weights_equal_value_run": bool(torch.equal(eng.flat16, eng_t.flat16)
                                                    and torch.equal(eng.flat32, eng_t.flat32)
                                                    and eng.loss() == eng_t.loss())}
        del graph_t, eng_t, fed_t
        torch.cuda.synchronize()

    # ---------------- caption-conditioned batches (K19), reported beside `value`:
    # the caption fork's loaders attach captions to every batch, and the reference then grows the vision
    # sequence by B rows per prompted layer (199 -> 455 at B = 32, J = 9).  Same protocol as the EOT mode;
    # one draw of the random pooling / projection weights for the whole run (the reference draws them per
    # forward on the host side; the device work per step is the same).
    cap_mode = None
    if not args.no_caption_mode:
        eng_c = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, captions=True),
                            device=dev)
        eng_c.set_lr(0.0026)
        eng_c.set_captions(caption_tokens(syn.synthetic_captions(seed, rank, 0, B)),
                           draw_caption_weights(torch.Generator().manual_seed(1000 * seed + rank)))

        def load_c(i):
            img, lab = batches[i % 2]
            eng_c.img_in.copy_(img)
            eng_c.label_in.copy_(lab)

        load_c(0)
        eng_c.train_step()
        graph_c = eng_c.capture_train_step()
        for i in range(args.warmup):
            load_c(i)
            graph_c.replay()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        a = time.perf_counter()
        for i in range(args.steps):
            load_c(i)
            graph_c.replay()
        torch.cuda.synchronize()
        el_c = time.perf_counter() - a
        if world > 1:
            t = torch.tensor([el_c], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_c = float(t.item())
        cap_mode = {"value": world * B * args.steps / el_c, "unit": "images/s",
                    "ms_per_step": 1e3 * el_c / args.steps, "vision_rows_per_layer": list(eng_c.vis.Ls),
                    "loss": eng_c.loss(),
                    "parity": "tests/test_captions_gpu.py (reference caption fixtures: loss bit-identical, "
                              "growing block outputs within the fp16 floor)"}
        del graph_c, eng_c
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    # ---------------- FedAvg alone (round-end cost), median of 5
    fts = []
    for _ in range(5):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        a = time.perf_counter()
        fed.run()
        torch.cuda.synchronize()
        fts.append(time.perf_counter() - a)
    fedavg_ms = 1e3 * float(np.median(fts))

    # ---------------- eval (test() path, trainers/maple.py:660-681): logits + argmax per batch, with
    # the class-prompt text features re-encoded per batch as the reference does, and cached across
    # the pass (bit-identical logits)
    acc = torch.zeros(2, device=dev)

    def eval_rate(reuse, n=10):
        load(0)
        eng.eval_batch(batches[0][1], acc)  # encodes the text features once
        torch.cuda.synchronize()
        a = time.perf_counter()
        for i in range(n):
            load(i)
            eng.eval_batch(batches[i % 2][1], acc, reuse_text=reuse)
        torch.cuda.synchronize()
        return B * n / (time.perf_counter() - a)

    eval_full, eval_cached = (None, None) if args.no_eval else (eval_rate(False), eval_rate(True))

    # the engine test() itself runs (trainers.MaPLe.test): forward-only (EngineConfig.inference), TRAINER.MAPLE.
    # EVAL_GROUP (4) x TEST.BATCH_SIZE (100) images per launch, the text features encoded by the first launch of
    # the pass; each launch copies its 400 images into the engine's input buffer as test() does
    def eval_rate_test_engine(images=400, n=6):
        import dataclasses
        ev = MapleEngine(dataclasses.replace(eng.cfg, batch=images, inference=True), device=dev, shared=eng)
        reps = -(-images // B)
        imgs = torch.cat([batches[i % 2][0] for i in range(reps)])[:images].contiguous()
        labs = torch.cat([batches[i % 2][1] for i in range(reps)])[:images].contiguous()
        ev.img_in.copy_(imgs)
        ev.eval_batch(labs, acc)
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(n):
            ev.img_in.copy_(imgs)
            ev.eval_batch(labs, acc, reuse_text=True)
        torch.cuda.synchronize()
        rate = images * n / (time.perf_counter() - a)
        del ev
        torch.cuda.empty_cache()
        return rate

    eval_test_engine = None if args.no_eval else eval_rate_test_engine()

    # ---------------- FedAvg overlapped with the client's last local test() (trainers/maple.py:646; the
    # trainer starts the exchange there, MaPLeFederated.train): exposed = (pack + exchange started, test
    # pass, wait + unpack) - (test pass alone), max over ranks, median of 3
    def test_pass(n=4):
        for i in range(n):
            load(i)
            eng.eval_batch(batches[i % 2][1], acc, reuse_text=i > 0)

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - a
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    def overlapped():
        fed.start()
        test_pass()
        fed.finish()

    test_pass()
    exposed = []
    for _ in range(3):
        exposed.append(timed(overlapped) - timed(test_pass))
    fedavg_exposed_ms = 1e3 * float(np.median(exposed))
    fed_ar = FedAvgBucket(eng, mode="allreduce")
    fedavg_allreduce_ms = 1e3 * float(np.median([timed(fed_ar.run) for _ in range(5)]))
    del fed_ar

    # ---------------- the data step in front of the path: the train transform
    # (RandomResizedCrop + flip + Normalize -> fp16, Pillow-exact bicubic) on B decoded PatternNet-size
    # 256x256 RGB images resident in HBM; reported beside `value`, never in it
    from federated_multi_modal_amd import transforms as dtf
    rng = np.random.default_rng(seed)
    packed = dtf.pack_images([rng.integers(0, 256, (256, 256, 3), dtype=np.uint8) for _ in range(B)], dev)
    tfm = dtf.DeviceTransform(True, generator=torch.Generator().manual_seed(seed))
    tf_out = torch.empty(B, 3, 224, 224, device=dev, dtype=torch.float16)
    geoms = [tfm.geometry(packed.shapes) for _ in range(20)]
    tfm(packed, geoms[0], out=tf_out)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for g in geoms:
        tfm(packed, g, out=tf_out)
    ev1.record()
    torch.cuda.synchronize()
    tf_us = ev0.elapsed_time(ev1) * 1e3 / len(geoms)
    tf_bytes = float(np.mean([(g[:, 4] * g[:, 5] * 3).sum() for g in geoms])) + B * 3 * 224 * 224 * 2
    a0 = time.perf_counter()
    for _ in range(5):
        tfm(packed, out=tf_out)  # host draws the crop parameters per batch, as the reference's workers do
    torch.cuda.synchronize()
    input_transform = {"images_per_s_device": B / (tf_us * 1e-6), "us_per_batch_device": tf_us,
                       "images_per_s_with_host_sampling": 5 * B / (time.perf_counter() - a0),
                       "algorithmic_bytes_per_batch": tf_bytes, "gbs": tf_bytes / (tf_us * 1e-6) / 1e9,
                       "hbm_frac": tf_bytes / (tf_us * 1e-6) / HBM_PEAK,
                       "workload": f"train transform, {B} decoded 256x256 RGB images -> fp16 [{B},3,224,224]",
                       "parity": "bit-exact vs Pillow resize + torchvision ToTensor/Normalize "
                                 "(tests/test_transforms.py)"}

    # ---------------- per-launch roofline of the dominant kernel (eager pass, HIP events on the
    # launching stream around every launch of that kernel during 2 full steps)
    # (towers serialised on one stream here so that no other kernel runs inside a probed launch)
    probe = ops.KernelProbe({"gemm": "gemm", "attention_fwd": "attention"}[args.roofline_kernel])
    aprobe = ops.KernelProbe("attention") if args.roofline_kernel == "gemm" else probe
    hprobe = ops.KernelProbe("hbm")  # the streaming kernels (LayerNorm, clip-grad-norm, SGD) against 8 TB/s
    eng.overlap_towers = False
    for pr in dict.fromkeys((probe, aprobe, hprobe)):  # one probe at a time, each over its own two steps
        ops.set_probe(pr)
        for i in range(2):
            load(i)
            eng.train_step()
        ops.set_probe(None)
    eng.overlap_towers = True
    ps = probe.summary("gemm" if args.roofline_kernel == "gemm" else "attention_fwd")
    # the attention kernels (north star: their MFMA-roofline fraction) against both roofs, per direction and
    # tower; at these lengths they sit below the 312 flop/B ridge, so the HBM roof binds
    attn_roof = {}
    for key in aprobe.keys():
        a = aprobe.summary(key)
        attn_roof[key] = {"launches_per_step": a["launches"] // 2, "avg_launch_us": a["avg_us"],
                          "flop_per_launch": a["flops_per_launch"], "bytes_per_launch": a["bytes_per_launch"],
                          "tflops": a["tflops"], "mfma_frac": a["tflops"] * 1e12 / MFMA_PEAK_F16,
                          "gbs": a["gbs"], "hbm_frac": a["gbs"] * 1e9 / HBM_PEAK,
                          "flop_per_byte": a["flops_per_launch"] / max(a["bytes_per_launch"], 1.0)}
        # the attention kernel against min(MFMA peak, AI x 8 TB/s)
        roof_t = min(MFMA_PEAK_F16, attn_roof[key]["flop_per_byte"] * HBM_PEAK)
        attn_roof[key]["roof_tflops"] = roof_t / 1e12
        attn_roof[key]["roof_frac"] = a["tflops"] * 1e12 / roof_t

    # the HBM-bound kernels against 8 TB/s (algorithmic bytes per launch: ops._hbm call sites)
    hbm_roof = {}
    for key in hprobe.keys():
        a = hprobe.summary(key)
        hbm_roof[key] = {"launches_per_step": a["launches"] // 2, "avg_launch_us": a["avg_us"],
                         "bytes_per_launch": a["bytes_per_launch"], "gbs": a["gbs"], "hbm_frac": a["gbs"] * 1e9 / HBM_PEAK}

    # HBM traffic of the dominant kernel family, per launch, from rocprofv3 PMC passes over exactly the launches
    # this probe times (tests/diagnostics/gemm_traffic.py: the same two eager steps, FETCH_SIZE x 2 + WRITE_SIZE
    # per MI355X_MICROARCH.md §HBM, memory-side counters) -> profiles/r<round>_v<n>_<config>_gemm_traffic.json,
    # which also holds the algorithmic bytes of those same launches; None when no such file exists
    traffic = traffic_alg = traffic_src = None

    def _ver(path):  # r<round>_v<n>_... -> (round, n)
        m = re.match(r"r(\d+)_v(\d+)_", path.name)
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)

    pmc = sorted((ROOT / "profiles").glob(f"*_{args.config}_gemm_traffic.json"), key=_ver)
    traffic_note = "no traffic file for this config under profiles/"
    if pmc and args.roofline_kernel == "gemm":
        try:
            tj = json.loads(pmc[-1].read_text())
            t_launches, t_alg = tj["launches"], tj["algorithmic_bytes_per_launch"]
            # the file must describe THIS probe's launch set: the same launch count over the two probed steps and
            # the same algorithmic bytes per launch (within 1 %); otherwise its traffic is another kernel set's
            if t_launches == ps["launches"] and abs(t_alg / ps["bytes_per_launch"] - 1.0) <= 0.01:
                traffic, traffic_alg = tj["traffic_bytes_per_launch"], t_alg
                traffic_note = "PMC passes over exactly the launches this probe times"
            else:
                traffic_note = (f"{pmc[-1].name} covers {t_launches} launches at {t_alg / 1e6:.2f} MB algorithmic per "
                                f"launch, this probe {ps['launches']} at {ps['bytes_per_launch'] / 1e6:.2f} MB: stale, "
                                f"not used")
            traffic_src = str(pmc[-1].relative_to(ROOT))
        except (OSError, ValueError, KeyError):
            traffic = traffic_alg = None

    step_flop = B * FLOP_PER_IMAGE + K * FLOP_PER_CLASS
    value = world * B * args.steps / elapsed
    if args.roofline_kernel == "gemm":
        roof = {"bound": "mfma", "achieved": ps["tflops"], "peak": MFMA_PEAK_F16 / 1e12, "unit": "TFLOP/s",
                "frac": ps["tflops"] * 1e12 / MFMA_PEAK_F16, "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": traffic_src, "traffic_note": traffic_note,
                "algorithmic_bytes_per_launch": ps["bytes_per_launch"],
                "traffic_source_algorithmic_bytes_per_launch": traffic_alg,
                "traffic_over_algorithmic": traffic / traffic_alg if traffic and traffic_alg else None,
                "kernel": "GEMM family: the hand-written gemm_nt_kernel / gemm8(s)_kernel launches (csrc/gemm.hip) -- "
                          "every projection GEMM of both towers, fwd + bwd",
                "launches_per_step": ps["launches"] // 2,
                "avg_launch_us": ps["avg_us"], "flop_per_launch": ps["flops_per_launch"]}
        by_tower = {}
        for tower in ("vision", "text"):
            try:
                pt = probe.summary(f"gemm/{tower}")
            except (KeyError, ZeroDivisionError):
                continue
            by_tower[tower] = {"launches_per_step": pt["launches"] // 2, "avg_launch_us": pt["avg_us"],
                               "tflops": pt["tflops"], "frac": pt["tflops"] * 1e12 / MFMA_PEAK_F16,
                               "flop_per_launch": pt["flops_per_launch"]}
        roof["by_tower"] = by_tower or None
        roof["by_tower_note"] = ("the text tower's products run on 160x128 tiles chosen for work per CU-second beside "
                                 "the vision tower, not for their own latency (DESIGN.md §4): isolated here (towers "
                                 "serialised) they take longer than the latency picks while the step gets faster")
    else:
        roof = {"bound": "mfma", "achieved": ps["tflops"], "peak": MFMA_PEAK_F16 / 1e12, "unit": "TFLOP/s",
                "frac": ps["tflops"] * 1e12 / MFMA_PEAK_F16, "traffic": None, "kernel": "attention_fwd_kernel",
                "avg_launch_us": ps["avg_us"], "flop_per_launch": ps["flops_per_launch"]}

    # ---------------- FedAvg round wall-time through MaPLeFederated.train() at the reference's cadence, at the
    # C3 client shape (configs[2]) and at this workload's (the metric's second half; beside `value`)
    fed_round = None
    if not args.no_round:
        fed_round = {}
        for cname in dict.fromkeys(("c3", args.config)):
            log(f"[bench] FedAvg round wall-time ({cname}) ...")
            fed_round[cname] = fed_round_wall(cname, world, rank)
        if args.config == "c4":  # the reference's own test cadence: PatternNet's whole test split after every epoch
            for grp in (1, None):
                key = "c4_patternnet_test_split" + ("_eval_group1" if grp == 1 else "")
                log(f"[bench] FedAvg round wall-time ({key}: {PATTERNNET_TEST_IMAGES} test images per epoch) ...")
                fed_round[key] = fed_round_wall("c4", world, rank, test_images=PATTERNNET_TEST_IMAGES, eval_group=grp)

    c5 = None
    if args.config == "c4" and not args.no_c5:
        c5 = side_config("c5", dev, world, rank)
        if not args.no_eot_mode:  # where the optional mode matters: 1000 prompts of <= 10 tokens out of 77
            c5["eot_truncated_mode"] = side_config("c5", dev, world, rank, eot_truncate=True, probe_gemm=False)

    out = {
        "metric": "images/sec/node (ViT-B/16 MaPLe fwd+bwd)",
        "value": value,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16",
        "data": "synthetic (portable counter-based PRNG images/labels/token ids; random-init CLIP ViT-B/16 weights)",
        "config": {"workload": f"{args.config}: {desc}", "clients": world, "batch_per_client": B,
                   "global_batch": world * B, "classes": K, "prompt_depth": J, "n_ctx": 2,
                   "parallelism": f"one federated client per GPU x{world}, FedAvg all-reduce per round",
                   "round": f"{args.steps} local steps + 1 FedAvg", "hipgraph": not args.no_graph},
        "fedavg_ms": fedavg_ms,
        "fedavg_mode": fed.mode,
        "fedavg_exposed_ms": fedavg_exposed_ms,
        "fedavg_exposed_note": ("world 1: no collective (validity scan + pack + unpack only), nothing to hide"
                                if world == 1 else f"{fed.mode} exchange over {world} ranks beside the last test()"),
        "fedavg_allreduce_ms": fedavg_allreduce_ms,
        "fedavg_bucket_mb": 4.0 * (eng.n16 + eng.n32 + 1) / 1e6,
        "fedavg_valid_clients": fed.n_valid(),
        "fedavg_round_wall": fed_round,
        "eot_truncated_mode": eot_mode,
        "caption_mode": cap_mode,
        "c5_side": c5,
        "eval_images_per_s": {"text_reencoded_per_batch": eval_full, "text_cached_per_pass": eval_cached,
                              "test_engine_group4_per_pass": eval_test_engine, "per_gpu": True,
                              "note": "text_* fields: the training engine's forward at its B-image batch; "
                                      "test_engine_group4_per_pass: the forward-only engine test() runs, 400 "
                                      "images (EVAL_GROUP 4 x TEST.BATCH_SIZE 100) per launch, text cached"},
        "input_transform": input_transform,
        "model_tflops": world * step_flop * args.steps / elapsed / 1e12,
        "model_mfma_frac": world * step_flop * args.steps / elapsed / MFMA_PEAK_F16 / world,
        "loss": loss,
        "roofline": roof,
        "attention_roofline": attn_roof,
        "hbm_kernels": hbm_roof,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log(f"[bench] timing the CPU baseline (oracle, {torch.get_num_threads()} threads) ...")
        out["cpu_baseline"] = cpu_baseline(J, K, B, args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
