"""GPU tier: the reference's module API (federated_multi_modal_amd/modules.py) driven the
way the reference drives it, against the engine path and the reference-generated fixtures.

  * CustomCLIP.state_dict(): the reference's keys, order, shapes and dtypes (tests/golden/state_dict_keys.json,
    generated from the reference's CustomCLIP.state_dict() at J=3 and J=9);
  * eval: model(x) (trainers/maple.py:674) == the engine's logits bit for bit, and within the logit gate
    of the reference's own logits (tests/golden/case_c1_s0_b0.npz);
  * image_encoder / text_encoder / prompt_learner / resblocks[i]([x, deep, counter]) with the reference's
    signatures == the engine's tower outputs bit for bit;
  * train: the reference's step restated (trainers/maple.py:588-598: loss = model(image, label);
    optim.zero_grad(); loss.backward(); clip_grad_norm_(model.parameters(), 1.0); optim.step() with
    torch.optim.SGD(momentum .9, wd 5e-4)) -- loss and every gradient equal the engine's bit for bit; the
    updated weights equal the engine's fused clip+SGD kernels' within one rounding step (torch's clip
    norm reduces in a different order and its fp32 foreach update may fuse multiply-add)."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

import _cases as C
from federated_multi_modal_amd import synthetic as syn
from federated_multi_modal_amd.engine import EngineConfig, MapleEngine
from federated_multi_modal_amd.modules import CustomCLIP

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def _engine(dev, J=3, K=10, B=4, seed=0):
    names = syn.synthetic_classnames(K, seed)
    return MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)


@pytest.mark.parametrize("J", [3, 9])
def test_state_dict_is_the_references(dev, J):
    gold = json.loads((GOLD / "state_dict_keys.json").read_text())[f"J{J}"]
    model = CustomCLIP(_engine(dev, J=J))
    sd = model.state_dict()
    assert list(sd) == [k for k, _, _ in gold]
    for k, shape, dtype in gold:
        assert tuple(sd[k].shape) == tuple(shape) and str(sd[k].dtype) == "torch." + dtype, k
    # aliases share storage, as clip_model2 shares the towers' modules in the reference
    assert sd["clip_model2.visual.proj"].data_ptr() == sd["image_encoder.proj"].data_ptr()
    names = [n for n, _ in model.named_parameters()]
    assert names[0] == "logit_scale" and names[-1] == "clip_model2.token_embedding.weight"
    trainable = [n for n, p in model.named_parameters() if p.requires_grad]
    # the freeze policy's 129 / 147 tensors (trainers/maple.py:447-479), incl. proj_vis_to_lang, which the
    # reference creates trainable but never uses (its grad stays None)
    assert len(trainable) == {3: 129, 9: 147}[J]
    assert "prompt_learner.proj_vis_to_lang.weight" in trainable


def test_eval_and_tower_callables(dev):
    c = C.load_case("c1_s0_b0")
    J, K, B, seed, names, batch = C.case_inputs(c)
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    model = CustomCLIP(e).eval()
    img = torch.from_numpy(batch.images).to(dev)
    with torch.no_grad():
        logits = model(img)                                  # trainers/maple.py:674
    e.img_in.copy_(img)
    ref_logits = e.forward().clone()
    assert torch.equal(logits, ref_logits)
    ok, rep = C.logit_gate(logits.float().cpu().numpy(), c["logits"], c["logits64"])
    assert ok, rep
    # the components with the reference's signatures
    prompts, shared_ctx, deep_text, deep_vis = model.prompt_learner()
    assert torch.equal(shared_ctx, e.shared_ctx)
    assert all(torch.equal(a, b) for a, b in zip(deep_vis, e.vis_deep))
    assert all(torch.equal(a, b) for a, b in zip(deep_text, e.txt_deep))
    txt = model.text_encoder(prompts, model.tokenized_prompts, deep_text)
    assert torch.equal(txt, e.txt_feat)
    imf = model.image_encoder(img.half(), shared_ctx, deep_vis)
    assert torch.equal(imf, e.img_feat)
    # one residual block on [x, deep, counter] (LND): block 2 replaces the last n_ctx rows with the second
    # visual deep prompt (clip/model.py:320-333); its output is the engine's X[3] (no prompt follows at J=3)
    blk = model.image_encoder.transformer.resblocks[2]
    L, D = e.Lv, 768
    x2 = e.vis.X[2].view(B, L, D).permute(1, 0, 2).contiguous()
    out, deep, counter = blk([x2, deep_vis, 1])
    assert counter == 2 and deep is deep_vis
    assert torch.equal(out.permute(1, 0, 2).reshape(B * L, D), e.vis.X[3])
    # a batch size other than the engine's (the test loader's 100, trainers/maple.py:671): same logits per row
    with torch.no_grad():
        two = model(img[:2])
    d = float((two.float() - logits[:2].float()).abs().max())
    print(f"rows 0-1 at batch 2 vs batch {B}: max |d| = {d:.3e}, bit-identical {torch.equal(two, logits[:2])}")
    assert torch.equal(two, logits[:2]) or d <= 2e-3


def test_reference_training_step_through_the_module(dev):
    """trainers/maple.py:588-598 restated over the module API vs the engine's fused step."""
    J, K, B, seed = 3, 10, 4, 0
    e_mod, e_ref = _engine(dev, J, K, B, seed), _engine(dev, J, K, B, seed)
    model = CustomCLIP(e_mod).train()
    optim = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.0026, momentum=0.9,
                            weight_decay=5e-4, dampening=0, nesterov=False)
    e_ref.set_lr(0.0026)
    for step in range(2):
        b = syn.client_batch(seed, 0, step, B, K)
        image, label = torch.from_numpy(b.images).to(dev), torch.from_numpy(b.labels).to(dev)
        loss = model(image, label)                     # trainers/maple.py:588
        optim.zero_grad()
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0, error_if_nonfinite=False)
        optim.step()
        # the engine path on the same weights (identical before step 0; after it, within one rounding step)
        if step == 0:
            e_ref.load_batch(image, label)
            e_ref.forward_backward()
            assert loss.dtype == torch.float16 and loss.item() == e_ref.loss()
            assert set(grads) == set(e_ref.trainable_names)
            for n in e_ref.trainable_names:
                assert torch.equal(grads[n], e_ref.G[n]), n
            e_ref.optimizer_step()
            torch.cuda.synchronize()
            coef = float(e_ref.clip_out[1])
            for n in e_ref.trainable_names:
                ours, ref = e_mod.P[n].float(), e_ref.P[n].float()
                if e_ref.P[n].dtype == torch.float16:
                    ulp = torch.exp2(torch.floor(torch.log2(ref.abs().clamp_min(2.0 ** -14))) - 10)
                    assert ((ours - ref).abs() <= ulp).all(), n
                else:
                    torch.testing.assert_close(ours, ref, rtol=2e-6, atol=1e-8, msg=n)
            assert 0.0 < coef <= 1.0
    assert torch.isfinite(loss.float())


def test_module_caption_forward_like_the_reference(dev):
    """CustomCLIP.forward(image, label, caption) with torch's global generator seeded as the reference's was
    when it produced tests/golden/case_cap_c1_j3_b4.npz: the same random AttentionPooling / Linear draws, so
    the loss matches the reference's (2 fp16 ulps) and the engine's caption path bit for bit; loss.backward()
    fills p.grad for the trainables."""
    from federated_multi_modal_amd.captions import caption_tokens, draw_caption_weights
    c = C.load_case("cap_c1_j3_b4")
    J, K, B, seed, names, batch = C.case_inputs(c)
    caps = [str(x) for x in c["captions"]]
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    model = CustomCLIP(e).train()
    img, lab = torch.from_numpy(batch.images).to(dev), torch.from_numpy(batch.labels).to(dev)
    torch.manual_seed(int(c["cap_seed"]))
    loss = model(img, lab, caps)
    ulp = 2.0 ** (np.floor(np.log2(abs(float(c["loss"])))) - 10)
    assert abs(loss.item() - float(c["loss"])) <= 2 * ulp
    loss.backward()
    assert model.prompt_learner.ctx.grad is not None and torch.isfinite(model.prompt_learner.ctx.grad.float()).all()
    ref = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, captions=True), device=dev)
    ref.set_captions(caption_tokens(caps), draw_caption_weights(torch.Generator().manual_seed(int(c["cap_seed"]))))
    ref.load_batch(img, lab)
    ref.forward_backward()
    assert loss.item() == ref.loss()
    for n in ref.trainable_names:
        assert torch.equal(dict(model.named_parameters())[n].grad, ref.G[n]), n


def test_image_encoder_with_caption_embeddings(dev):
    """image_encoder(x, shared_ctx, deep_vis, clip_embeddings) (clip/model.py:509, 550-561): the caption tokens'
    embedding pooled with a fresh random vector, projected by a fresh random Linear(512, 768), prepended to
    every deep prompt -- the growing sequence of the engine's caption path, bit for bit with the same draws,
    and the reference's image features (tests/golden/case_cap_c1_j3_b4.npz) within the fp16 floor."""
    from federated_multi_modal_amd.captions import caption_tokens, draw_caption_weights
    c = C.load_case("cap_c1_j3_b4")
    J, K, B, seed, names, batch = C.case_inputs(c)
    caps = [str(x) for x in c["captions"]]
    e = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed), device=dev)
    model = CustomCLIP(e).eval()
    img = torch.from_numpy(batch.images).to(dev)
    prompts, shared_ctx, deep_text, deep_vis = model.prompt_learner()
    tok = torch.from_numpy(caption_tokens(caps)).to(dev)
    emb = model.clip_model2.token_embedding.weight[tok].half()        # trainers/maple.py:319
    model.caption_generator = torch.Generator().manual_seed(int(c["cap_seed"]))
    imf = model.image_encoder(img.half(), shared_ctx, deep_vis, emb)
    ref = MapleEngine(EngineConfig(batch=B, classnames=names, prompt_depth=J, seed=seed, captions=True), device=dev)
    ref.set_captions(tok.cpu(), draw_caption_weights(torch.Generator().manual_seed(int(c["cap_seed"]))))
    ref.load_batch(img)
    ref.forward()
    assert torch.equal(imf, ref.img_feat)
    a, b = imf.double().cpu().numpy(), c["img_feat"].astype(np.float64)
    assert np.linalg.norm(a - b) / np.linalg.norm(b) <= 3e-3
