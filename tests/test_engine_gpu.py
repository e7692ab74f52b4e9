"""End-to-end parity of the MI355X MaPLe client engine (every op a libmapfed.so kernel) against the
golden fixtures generated from the reference's own CPU path (tests/golden/make_golden.py) and
against the oracle on other shapes.

Tolerances (north_star: logits within 1e-3 of the reference in fp16, class predictions bit-exact):
  * logits: max |diff| <= 4e-3 (4 fp16 ulps at |logit| < 2), mean |diff| <= 1.5e-3, argmax identical,
    and the error against the float64 restatement at most 1.25x the reference's own.  The max-1e-3
    form is below the reference's reproducibility floor: re-running the reference with only its
    GEMMs correctly rounded (no other change) moves its logits by 3.4e-3
    (tests/test_noise_floor.py), so no implementation with a different summation order than
    oneDNN's CPU kernels can meet it; DESIGN.md §5.
  * loss: |diff| <= 2e-3 (fp16 scalar, 1 ulp at 2.7 is 2e-3);
  * gradients (fp16 activations through 24 transformer blocks, where the reference's own
    fp16-vs-fp64 gap is several % on small tensors): per tensor, relative L2 error vs the
    reference <= 5 %, and norm within 3 %; the global clip norm within 1 %;
  * SGD deltas: relative L2 error <= 5 % per tensor.
"""
import numpy as np
import pytest
import torch

from federated_multi_modal_amd import synthetic as syn
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine

pytestmark = pytest.mark.gpu
from pathlib import Path

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def c1():
    return dict(np.load(GOLD / "c1_maple.npz"))


@pytest.fixture(scope="module")
def c1_engine(c1, dev):
    J, K, B, seed = int(c1["J"]), int(c1["K"]), int(c1["B"]), int(c1["seed"])
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, 0, 0, B, K)
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    e.load_batch(torch.from_numpy(batch.images), torch.from_numpy(batch.labels))
    logits = e.forward().float().cpu().numpy()
    e.forward_backward()
    loss = e.loss()
    grads = {k: v.detach().double().cpu().reshape(-1).numpy() for k, v in e.grads().items()}
    before = {k: v.detach().double().cpu() for k, v in e.trainable_state().items()}
    total = None
    e.set_lr(float(c1["lr"]))
    e.optimizer_step()
    torch.cuda.synchronize()
    total = float(e.clip_out[0].item())
    deltas = {k: (v.detach().double().cpu() - before[k]).reshape(-1).numpy() for k, v in e.trainable_state().items()}
    before = {k: v.reshape(-1).numpy() for k, v in before.items()}
    dtypes = {k: v.dtype for k, v in e.trainable_state().items()}
    return dict(e=e, logits=logits, loss=loss, grads=grads, total=total, deltas=deltas, before=before,
                dtypes=dtypes)


def _sel(g, prefix, name, full):
    if f"{prefix}full/{name}" in g:
        return full, g[f"{prefix}full/{name}"].astype(np.float64)
    idx = g[f"{prefix}idx/{name}"]
    return full[idx], g[f"{prefix}val/{name}"].astype(np.float64)


def test_c1_logits(c1, c1_engine):
    ours, ref = c1_engine["logits"], c1["logits"].astype(np.float64)
    err = np.abs(ours - ref)
    e64_ours = np.abs(ours - c1["logits64"]).max()
    e64_ref = np.abs(ref - c1["logits64"]).max()
    print(f"C1 logits max|err| {err.max():.3e} mean {err.mean():.3e}; vs fp64: ours {e64_ours:.3e} "
          f"reference {e64_ref:.3e}")
    assert err.mean() <= 1.5e-3 and err.max() <= 4e-3
    assert e64_ours <= 1.25 * e64_ref
    assert np.array_equal(ours.argmax(1), ref.argmax(1))


def test_c1_loss(c1, c1_engine):
    assert abs(c1_engine["loss"] - float(c1["loss"])) <= 2e-3


def test_c1_grads(c1, c1_engine):
    grads = c1_engine["grads"]
    names = sorted(k[len("grad/norm/"):] for k in c1 if k.startswith("grad/norm/"))
    assert set(names) <= set(grads)
    worst = []
    for n in names:
        ours, ref = _sel(c1, "grad/", n, grads[n])
        rel = np.linalg.norm(ours - ref) / (np.linalg.norm(ref) + 1e-30)
        nrm = abs(np.linalg.norm(grads[n]) - float(c1[f"grad/norm/{n}"])) / (float(c1[f"grad/norm/{n}"]) + 1e-30)
        worst.append((rel, nrm, n))
    worst.sort(reverse=True)
    print("worst grads (rel L2, rel norm):", [(f"{a:.2e}", f"{b:.2e}", n) for a, b, n in worst[:6]])
    for rel, nrm, n in worst:
        assert rel <= 5e-2 and nrm <= 3e-2, (n, rel, nrm)
    assert abs(c1_engine["total"] - float(c1["total_norm"])) <= 1e-2 * float(c1["total_norm"])


def test_c1_sgd_deltas(c1, c1_engine):
    """fp32 params: relative L2 error of the update <= 5 %.  fp16 params store p - lr*buf rounded to
    fp16, so their update is quantised to ulps of p: per element the difference may be one fp16 ulp
    of p (a rounding flip) plus 10 % of the update (the gradient's own error), and over the tensor
    ||diff|| <= 5 % ||update|| + half the rms ulp."""
    worst = 0.0
    for n, d in c1_engine["deltas"].items():
        if f"delta/norm/{n}" not in c1:
            continue
        ours, ref = _sel(c1, "delta/", n, d)
        diff = np.abs(ours - ref)
        if c1_engine["dtypes"][n] == torch.float16:
            p0, _ = _sel(c1, "delta/", n, c1_engine["before"][n])
            u = np.exp2(np.floor(np.log2(np.maximum(np.abs(p0), 2.0 ** -14))) - 10)
            assert (diff <= u + 0.1 * np.abs(ref) + 1e-12).all(), (n, (diff / u).max())
            assert np.linalg.norm(diff) <= 0.05 * np.linalg.norm(ref) + 0.5 * np.linalg.norm(u), n
            continue
        if np.linalg.norm(ref) == 0:
            continue
        rel = np.linalg.norm(ours - ref) / np.linalg.norm(ref)
        worst = max(worst, rel)
        assert rel <= 5e-2, (n, rel)
    print(f"worst fp32 SGD delta rel err {worst:.2e}")


def test_engine_vs_oracle_other_shape(dev):
    """J=9 (depth default, train.py:113), K=38 ragged class names, B=3: logits vs the oracle."""
    from oracle import maple_oracle as O
    J, K, B, seed = 9, 38, 3, 5
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, 1, 0, B, K)
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    e.load_batch(torch.from_numpy(batch.images), torch.from_numpy(batch.labels))
    logits = e.forward().float().cpu().numpy()
    M = O.build_model(seed, J, names)
    with torch.no_grad():
        ref = O.forward(M, torch.from_numpy(batch.images), train=False).float().numpy()
    err = np.abs(logits - ref)
    print(f"J=9 K=38 B=3 logits max|err| {err.max():.3e} mean {err.mean():.3e}")
    assert err.mean() <= 1.5e-3 and err.max() <= 4e-3
    top2 = np.sort(ref, 1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 4e-3  # argmax is only defined past the tolerance
    assert np.array_equal(logits.argmax(1)[clear], ref.argmax(1)[clear])


def test_training_is_deterministic_and_finite(dev):
    """Two engines from the same seed give bit-identical losses over 3 steps; no NaN/Inf."""
    names = syn.synthetic_classnames(10, 0)
    losses = []
    for _ in range(2):
        e = MapleEngine(EngineConfig(batch=4, classnames=names, prompt_depth=3, seed=0), device=dev)
        e.set_lr(0.0026)
        ls = []
        for s in range(3):
            b = syn.client_batch(0, 0, s, 4, 10)
            e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
            e.train_step()
            ls.append(e.loss())
        losses.append(ls)
    assert losses[0] == losses[1]
    assert all(np.isfinite(losses[0]))


def test_engine_soft_labels_vs_oracle(dev):
    """Soft (float) labels take the KL branch (trainers/maple.py:356-360): engine loss and gradients
    against the oracle run in fp32 on the same inputs (B=4, K=10, depth 3), same tolerances as C1."""
    from oracle import maple_oracle as O
    J, K, B, seed = 3, 10, 4, 11
    names = syn.synthetic_classnames(K, seed)
    batch = syn.client_batch(seed, 0, 0, B, K)
    g = torch.Generator().manual_seed(seed)
    q = torch.rand(B, K, generator=g) ** 3
    q[1] = torch.nn.functional.one_hot(torch.tensor(3), K).float()   # a hard row inside a soft batch
    q = q / q.sum(1, keepdim=True)
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    e.load_batch(torch.from_numpy(batch.images), q)
    assert e.soft_labels
    e.forward_backward()
    loss = e.loss()
    grads = {k: v.detach().double().cpu().reshape(-1) for k, v in e.grads().items()}
    M = O.build_model(seed, J, names, compute_dtype=torch.float32)
    ref_loss, ref_grads, _ = O.train_step(M, torch.from_numpy(batch.images), q, O.SGDState(lr=0.0))
    print(f"soft-label loss ours {loss:.5f} oracle(fp32) {ref_loss.item():.5f}")
    assert abs(loss - ref_loss.item()) <= 5e-3
    worst = []
    for n, r in ref_grads.items():
        r = r.double().reshape(-1)
        if r.norm() == 0:
            continue
        worst.append(((grads[n] - r).norm().item() / r.norm().item(), n))
    worst.sort(reverse=True)
    print("worst soft-label grads (rel L2):", [(f"{a:.2e}", n) for a, n in worst[:5]])
    assert worst[0][0] <= 5e-2, worst[0]
    # switching back to integer labels returns to the cross-entropy branch
    e.load_batch(torch.from_numpy(batch.images), torch.from_numpy(batch.labels))
    assert not e.soft_labels


def test_eval_reuses_text_features_bit_exactly(dev):
    """Eval with the class-prompt text features cached across test batches:
    the logits of a second batch equal a full forward (text re-encoded) bit for bit."""
    J, K, B, seed = 3, 10, 4, 2
    names = syn.synthetic_classnames(K, seed)
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    b0, b1 = syn.client_batch(seed, 0, 0, B, K), syn.client_batch(seed, 0, 1, B, K)
    e.load_batch(torch.from_numpy(b0.images))
    e.forward()
    e.load_batch(torch.from_numpy(b1.images))
    cached = e.forward(reuse_text=True).clone()
    full = e.forward().clone()
    assert torch.equal(cached, full)
    acc = torch.zeros(2, device=dev)
    e.eval_batch(torch.from_numpy(b1.labels).to(dev), acc, reuse_text=True)
    assert acc[1].item() == B


def test_eval_launch_size_does_not_change_logits(dev):
    """The precondition of TRAINER.MAPLE.EVAL_GROUP > 1 at the reference's cadence (PatternNet, TEST.BATCH_SIZE 100):
    one 400-image forward of the forward-only eval engine -- other GEMM tiles, and at 4 800 heads the persistent
    attention forward -- gives the rows of four 100-image forwards (1 200 heads: attn_fwd4) bit for bit, so the
    accuracy counts of a grouped test pass are those of batch-by-batch evaluation (trainers/maple.py:660-681)."""
    J, K, seed = 9, 38, 3
    names = syn.synthetic_classnames(K, seed)
    big = MapleEngine(EngineConfig(batch=400, classnames=names, prompt_depth=J, seed=seed, inference=True),
                      device=dev)
    small = MapleEngine(EngineConfig(batch=100, classnames=names, prompt_depth=J, seed=seed, inference=True),
                        device=dev, shared=big)
    imgs = torch.cat([torch.from_numpy(syn.client_batch(seed, 0, s, 100, K).images) for s in range(4)])
    big.load_batch(imgs)
    lb = big.forward().clone()
    rows = []
    for s in range(4):
        small.load_batch(imgs[100 * s:100 * (s + 1)])
        rows.append(small.forward().clone())
    ls = torch.cat(rows)
    assert torch.isfinite(lb.float()).all()
    assert torch.equal(lb, ls), (lb.float() - ls.float()).abs().max().item()
    # the forward-only engine computes its last vision block for the class rows only (cls_only, r06): the full
    # block gives the same logits bit for bit
    assert big.vis.cls_only and small.vis.cls_only
    big.vis.cls_only = False
    big.load_batch(imgs)
    assert torch.equal(big.forward(), lb)


@pytest.mark.parametrize("J,K,B,seed", [(3, 10, 4, 4), (9, 38, 8, 1)])
def test_eot_truncated_text_tower_matches_full(dev, J, K, B, seed):
    """EngineConfig.eot_truncate: the text tower on the first max(EOT)+1 tokens of each class prompt.  Under the
    causal mask the later tokens never reach an EOT row and their gradients are exactly zero, and the truncated
    tower runs every row reduction of its backward (LayerNorm dgamma / dbeta, block 11's dW and db) over the
    77-row layout (mf_layernorm_bwd_live, mf_seq_scatter): logits, loss, every gradient and the weights after an
    SGD step (eager, then a replayed graph) are bit-identical to the 77-token tower's."""
    names = syn.synthetic_classnames(K, seed)
    b = syn.client_batch(seed, 0, 0, B, K)
    out = []
    for trunc in (False, True):
        e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=trunc),
                        device=dev)
        e.set_lr(0.0026)
        e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
        logits = e.forward().clone()
        e.forward_backward()
        grads = {k: v.detach().clone() for k, v in e.grads().items()}
        e.train_step()
        g = e.capture_train_step()
        g.replay()
        torch.cuda.synchronize()
        out.append((e.text_len, logits, e.loss(), grads, e.flat16.detach().clone(), e.flat32.detach().clone()))
    (l77, lg0, loss0, g0, a0, b0), (lt, lg1, loss1, g1, a1, b1) = out
    assert l77 == 77 and lt < 77
    assert torch.equal(lg0, lg1)
    assert loss0 == loss1
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, f"gradients differ: {bad[:5]}"
    assert torch.equal(a0, a1) and torch.equal(b0, b1)


def test_concurrent_towers_are_reproducible_and_eot_exact(dev):
    """Three c4-shape engines stepped in lockstep with the towers on two streams (eager steps, client 1's two
    batches): two EOT-truncated ones and the 77-token one agree bit for bit in every gradient and weight after every
    step.  r05 regression: a LayerNorm-backward build whose loads sat behind a branch gave run-to-run different
    dgamma partials only when the towers overlapped (tests/diagnostics/eot_exact_steps.py)."""
    J, K, B, seed = 9, 38, 32, 0
    names = syn.synthetic_classnames(K, seed)
    cb = [syn.client_batch(seed, 1, s, B, K) for s in range(2)]
    es = [MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=t), device=dev)
          for t in (False, True, True)]
    for e in es:
        e.set_lr(0.0026)
    for s in range(4):
        for e in es:
            e.img_in.copy_(torch.from_numpy(cb[s % 2].images).to(dev))
            e.label_in.copy_(torch.from_numpy(cb[s % 2].labels).to(dev))
            e.train_step()
        torch.cuda.synchronize()
        g = [e.grads() for e in es]
        for other in (1, 2):
            bad = [n for n in g[0] if not torch.equal(g[0][n], g[other][n])]
            assert not bad, f"step {s}, engine {other}: {bad[:4]}"
            assert torch.equal(es[0].flat16, es[other].flat16) and torch.equal(es[0].flat32, es[other].flat32)


def test_tower_order_does_not_change_results(dev):
    """The towers' enqueue order after each fork (EngineConfig.vision_first: vision first by default, text first
    as the A/B baseline) only changes which stream's launches reach the GPU first: every reduction is
    deterministic, so logits, loss and every gradient are bit-identical, eagerly and in a replayed graph."""
    J, K, B, seed = 3, 10, 4, 6
    names = syn.synthetic_classnames(K, seed)
    b = syn.client_batch(seed, 0, 0, B, K)
    out = []
    for order in ("vision", "text"):
        e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed,
                                     vision_first=order == "vision"), device=dev)
        assert e.vision_first == (order == "vision")
        e.set_lr(0.0026)
        e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
        logits = e.forward().clone()
        e.train_step()  # eager step (creates the momentum buffers)
        g = e.capture_train_step()
        g.replay()
        torch.cuda.synchronize()
        out.append((logits, e.loss(), {k: v.detach().clone() for k, v in e.grads().items()},
                    e.flat16.detach().clone(), e.flat32.detach().clone()))
    (l0, s0, g0, a0, b0), (l1, s1, g1, a1, b1) = out
    assert torch.equal(l0, l1) and s0 == s1
    assert all(torch.equal(g0[n], g1[n]) for n in g0)
    assert torch.equal(a0, a1) and torch.equal(b0, b1)


def test_c4_full_size_properties(dev):
    """BASELINE configs[3] size (B=32, K=38, J=9), where the oracle is too slow to run: size-independent
    properties.  Two engines from one seed agree bit for bit (logits, loss, every gradient, the updated
    weights); the EOT-truncated text tower gives bit-identical logits and loss; cached-text eval equals a
    full forward; everything finite."""
    J, K, B, seed = 9, 38, 32, 0
    names = syn.synthetic_classnames(K, seed)
    b = syn.client_batch(seed, 0, 0, B, K)
    runs = []
    for trunc in (False, False, True):
        e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=trunc),
                        device=dev)
        e.set_lr(0.0026)
        e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
        logits = e.forward().clone()
        e.forward_backward()
        loss = e.loss()
        grads = {k: v.detach().clone() for k, v in e.grads().items()}
        e.optimizer_step()
        params = {k: v.detach().clone() for k, v in e.trainable_state().items()}
        runs.append((logits, loss, grads, params, e))
    (l0, s0, g0, p0, e0), (l1, s1, g1, p1, _), (l2, s2, _, _, _) = runs
    assert torch.isfinite(l0.float()).all() and np.isfinite(s0)
    assert torch.equal(l0, l1) and s0 == s1
    assert all(torch.equal(g0[k], g1[k]) for k in g0) and all(torch.equal(p0[k], p1[k]) for k in p0)
    assert all(torch.isfinite(v.float()).all() for v in g0.values())
    assert torch.equal(l0, l2) and s0 == s2
    # eval with the text features of the previous forward (weights updated since: re-encode once first)
    full = e0.forward().clone()
    e0.load_batch(torch.from_numpy(syn.client_batch(seed, 0, 1, B, K).images))
    full2 = e0.forward().clone()
    cached2 = e0.forward(reuse_text=True).clone()
    assert torch.equal(full2, cached2) and not torch.equal(full, full2)


def test_c5_full_size_properties(dev):
    """BASELINE configs[4] size (B=32, K=1000 class prompts of 77 tokens, J=9): the text tower runs
    77 000 rows (M of every text GEMM) and 8 000 causal attention heads.  The reference's own outputs on
    all 1000 prompts are pinned at B=2 (tests/golden/case_c5_text_k1000.npz, test_parity_cases_gpu.py);
    here, size-independent properties at the full size: two engines from one seed agree bit for bit
    (logits, loss, every gradient, updated weights), so does the EOT-truncated tower (its LayerNorm partials
    over 4 813 full-layout row blocks, block 11's dW over all 77 000 rows), cached-text eval equals a full
    forward, everything finite."""
    J, K, B, seed = 9, 1000, 32, 0
    names = syn.synthetic_classnames(K, seed)
    b = syn.client_batch(seed, 0, 0, B, K)
    runs = []
    for trunc in (False, False, True):
        e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, eot_truncate=trunc),
                        device=dev)
        e.set_lr(0.0026)
        e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
        logits = e.forward().clone()
        e.forward_backward()
        loss = e.loss()
        if trunc:
            assert e.text_len < 77
            grads = {k: v.detach().clone() for k, v in e.grads().items()}
            e.optimizer_step()
            params = {k: v.detach().clone() for k, v in e.trainable_state().items()}
            runs.append((logits, loss, grads, params))
            del e
            break
        grads = {k: v.detach().clone() for k, v in e.grads().items()}
        e.optimizer_step()
        params = {k: v.detach().clone() for k, v in e.trainable_state().items()}
        runs.append((logits, loss, grads, params))
        if len(runs) == 2:
            full = e.forward().clone()
            cached = e.forward(reuse_text=True).clone()
            assert torch.equal(full, cached)
        del e
        torch.cuda.empty_cache()
    (l0, s0, g0, p0), (l1, s1, g1, p1), (l2, s2, g2, p2) = runs
    assert torch.isfinite(l0.float()).all() and np.isfinite(s0)
    assert torch.equal(l0, l1) and s0 == s1
    assert all(torch.equal(g0[k], g1[k]) for k in g0) and all(torch.equal(p0[k], p1[k]) for k in p0)
    assert all(torch.isfinite(v.float()).all() for v in g0.values())
    assert torch.equal(l0, l2) and s0 == s2
    assert all(torch.equal(g0[k], g2[k]) for k in g0) and all(torch.equal(p0[k], p2[k]) for k in p0)


@pytest.mark.parametrize("K,variants", [(38, ("none", "both", "side")), (1000, ("none", "side"))], ids=["c4", "c5"])
def test_fused_qkv_attention_does_not_change_results(dev, K, variants):
    """The in-projection + attention forward as one launch against the unfused pair (EngineConfig.fused_qkv_attn):
    at the c4 client shape (J = 9, K = 38, B = 32) both towers fused and the default ("side": the text tower, which
    runs beside the vision tower), and at C5 (K = 1 000) the default, which fuses the VISION tower there (the side
    tower: less projection work than the 77 000-row text tower) -- logits, loss and every gradient bit-identical
    to the unfused step."""
    J, B, seed = 9, 32, 2
    names = syn.synthetic_classnames(K, seed)
    b = syn.client_batch(seed, 0, 0, B, K)
    out = []
    for fused in variants:
        e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, fused_qkv_attn=fused),
                        device=dev)
        side_vis = K > 100  # c4: the text tower is the side tower; C5: the vision tower
        want_vis = fused == "both" or (fused == "side" and side_vis)
        want_txt = fused == "both" or (fused == "side" and not side_vis)
        assert e.vis.fused_qkv_attn == want_vis and e.txt.fused_qkv_attn == want_txt, fused
        e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
        logits = e.forward().clone()
        e.forward_backward()
        out.append((logits, e.loss(), {k: v.detach().clone() for k, v in e.grads().items()},
                    e.vis.QKV[3].clone(), e.vis.O[3].clone(), e.txt.O[5].clone()))
        del e
        torch.cuda.empty_cache()
    (lg0, l0, g0, q0, vo0, o0) = out[0]
    for lg1, l1, g1, q1, vo1, o1 in out[1:]:
        assert torch.equal(lg0, lg1) and l0 == l1
        assert torch.equal(q0, q1) and torch.equal(vo0, vo1) and torch.equal(o0, o1)
        for n in g0:
            assert torch.equal(g0[n], g1[n]), n


@pytest.mark.parametrize("J,K,B", [(9, 38, 32), (9, 1000, 32)], ids=["c4", "c5"])
def test_graph_replay_equals_eager_step(dev, J, K, B):
    """The captured step (one hipGraph: the text tower forked onto the side stream and joined back, the
    optimizer's halt latch, the LR read from device memory) computes exactly what the same step launched
    eagerly computes, at the bench's C4 shape and at C5 (K = 1 000): two engines built identically take the
    same eager first step (momentum buffers created), then engine A runs step 2 eagerly and engine B replays
    its captured graph on the same batch -- loss, every trainable gradient, the updated weights and the
    momentum, bit for bit.  A missing or misplaced cross-stream edge in the captured graph (r03: forking the
    text tower ahead of the prompt learner it reads) shows here as a mismatch."""
    names = syn.synthetic_classnames(K, 0)
    b0, b1 = syn.client_batch(0, 0, 0, B, K), syn.client_batch(0, 0, 1, B, K)
    out = []
    for graph in (False, True):
        e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=0), device=dev)
        e.set_lr(0.0026)
        e.load_batch(torch.from_numpy(b0.images), torch.from_numpy(b0.labels))
        e.train_step()
        if graph:
            g = e.capture_train_step()
            e.load_batch(torch.from_numpy(b1.images), torch.from_numpy(b1.labels))
            g.replay()
        else:
            e.load_batch(torch.from_numpy(b1.images), torch.from_numpy(b1.labels))
            e.train_step()
        torch.cuda.synchronize()
        out.append({"loss": e.loss_out.detach().clone().cpu(), "gflat16": e.gflat16.detach().clone().cpu(),
                    "gflat32": e.gflat32.detach().clone().cpu(), "flat16": e.flat16.detach().clone().cpu(),
                    "flat32": e.flat32.detach().clone().cpu(),
                    "mom": [e.mom16.detach().clone().cpu(), e.mom32.detach().clone().cpu()]})
        del e
        torch.cuda.empty_cache()
    a, g = out
    assert torch.isfinite(a["loss"][:1]).all()
    for k in ("loss", "gflat16", "gflat32", "flat16", "flat32"):
        assert torch.equal(a[k], g[k]), k
    assert len(a["mom"]) == len(g["mom"]) > 0 and all(torch.equal(x, y) for x, y in zip(a["mom"], g["mom"]))
