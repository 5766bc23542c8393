"""Phi-3-vision (``models/phi3v.py``) on CPU.  transformers has no Phi-3-V class, so the reference
is assembled from transformers' own ``Phi3ForCausalLM`` and ``CLIPVisionModel`` (tiny, random,
fp32) plus an independent re-statement of Phi-3-V's HD feature transform (2x2 merge, crop
stitching, ``sub_GN`` row separators, ``glb_GN``, sub-then-global order, GELU projector).  Checks
the image features, the placeholder expansion count and greedy generation with two images of
different crop grids through the engine; the image processor's resize / pad geometry is checked
against the formula of the Phi-3-V processor (pixel parity unpinned)."""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.phi3v import hd_size, num_image_tokens, preprocess_phi3v  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

CROP = 56


def _image(seed, h, w):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _build(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = T.Phi3Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=1024,
                      original_max_position_embeddings=1024, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    lm = T.Phi3ForCausalLM(tc)
    vc = T.CLIPVisionConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3, num_attention_heads=2,
                            image_size=CROP, patch_size=14)
    vis = T.CLIPVisionModel(vc)
    for m in (lm, vis):
        with torch.no_grad():
            for n, p in m.named_parameters():
                if "norm" in n:
                    p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
                else:
                    p.normal_(0.0, 0.08)
        m.float().eval()
        m.config._attn_implementation = "eager"
    H, C4 = 256, 4 * 128
    g = torch.Generator().manual_seed(1)
    proj = {"img_projection.0.weight": torch.randn(H, C4, generator=g) * 0.05,
            "img_projection.0.bias": torch.randn(H, generator=g) * 0.02,
            "img_projection.2.weight": torch.randn(H, H, generator=g) * 0.05,
            "img_projection.2.bias": torch.randn(H, generator=g) * 0.02,
            "glb_GN": torch.randn(1, 1, C4, generator=g) * 0.5, "sub_GN": torch.randn(1, 1, 1, C4, generator=g) * 0.5}
    sd = {k: v.detach().clone().contiguous() for k, v in lm.state_dict().items() if "rotary" not in k}
    for k, v in vis.state_dict().items():
        k = k[len("vision_model."):] if k.startswith("vision_model.") else k   # transformers 4 / 5 spellings
        sd["model.vision_embed_tokens.img_processor.vision_model." + k] = v.detach().clone().contiguous()
    for k, v in proj.items():
        sd["model.vision_embed_tokens." + k] = v.contiguous()
    sd["model.vision_embed_tokens.wte.weight"] = sd["model.embed_tokens.weight"].clone()
    save_file(sd, tmp_path / "model.safetensors")
    cfg = {k: v for k, v in tc.to_dict().items() if k not in ("architectures", "model_type", "transformers_version")}
    cfg.update(architectures=["Phi3VForCausalLM"], model_type="phi3_v", num_crops=4,
               embd_layer={"embedding_cls": "image", "hd_transform_order": "sub_glb", "projection_cls": "mlp",
                           "use_hd_transform": True, "with_learnable_separator": True},
               img_processor={"image_dim_out": 128, "layer_idx": -2, "type_feature": "patch",
                              "vision_config": {k: vc.to_dict()[k] for k in ("hidden_size", "intermediate_size",
                                                                             "num_hidden_layers",
                                                                             "num_attention_heads", "image_size",
                                                                             "patch_size", "hidden_act")}})
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    return lm, vis, proj


def _ref_features(vis, proj, px, grids):
    """Phi-3-V HD transform, restated from the published model code."""
    with torch.no_grad():
        f = vis(px, output_hidden_states=True).hidden_states[-2][:, 1:]
    N, L, C = f.shape
    S = int(L ** 0.5)
    out, off = [], 0
    sub_gn, glb_gn = proj["sub_GN"], proj["glb_GN"]
    for _, h, w in grids:
        x = f[off:off + 1 + h * w]
        off += 1 + h * w

        def merge(t, hc, wc):
            n = t.shape[0]
            return (t.reshape(n, S, S, C).reshape(n, S // 2, 2, S // 2, 2, C).permute(0, 1, 3, 2, 4, 5)
                    .reshape(n, -1, 4 * C).reshape(n // (hc * wc), hc, wc, S // 2, S // 2, -1)
                    .permute(0, 1, 3, 2, 4, 5).reshape(n // (hc * wc), hc * S // 2, wc * S // 2, 4 * C))

        def newline(t):
            n, hh = t.shape[0], t.shape[1]
            return torch.cat([t, sub_gn.expand(n, hh, -1, -1)], 2).reshape(n, -1, t.shape[-1])

        glb = newline(merge(x[:1], 1, 1))
        sub = newline(merge(x[1:], h, w))
        out += [sub[0], glb_gn[0], glb[0]]
    e = torch.cat(out, 0)
    e = F.gelu(e @ proj["img_projection.0.weight"].T + proj["img_projection.0.bias"])
    return e @ proj["img_projection.2.weight"].T + proj["img_projection.2.bias"]


def test_hd_geometry():
    # portrait: transposed, width 2 * 336, height padded to a multiple of 336, transposed back
    assert hd_size(600, 800, 16) == (int(4 * 336 / (800 / 600)), 4 * 336, 1008, 4 * 336)
    # 5:1 landscape: 8 * ceil(8 / 5) = 16 crops fit, 9 * ceil(9 / 5) = 18 do not
    assert hd_size(1000, 200, 16) == (8 * 336, int(8 * 336 / 5), 8 * 336, 2 * 336)
    px, g = preprocess_phi3v(_image(0, 200, 1000), 16)
    assert g == (1, 2, 8) and px.shape == (17, 3, 336, 336)
    assert num_image_tokens(2, 8) == (2 * 8 + 1) * 144 + 1 + (2 + 1) * 12   # the processor's count formula


def test_phi3v_matches_reference(tmp_path):
    lm, vis, proj = _build(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 40, 150)]
    pre = [preprocess_phi3v(im, 4, CROP) for im in imgs]
    assert [g for _, g in pre] == [(1, 2, 2), (1, 1, 3)]
    px = torch.cat([p for p, _ in pre])
    grids = [g for _, g in pre]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "Phi3VForCausalLM"
    want = _ref_features(vis, proj, px, grids)
    got = m.encode_images(px, grids)
    assert got.shape == want.shape == (27 + 21, 256)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, 17, -1, 33, 41, -2, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    assert [n for _, n in req.mm.spans] == [27, 21]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = torch.tensor(req.prompt_ids)
    rows = torch.cat([torch.arange(s, s + n) for s, n in req.mm.spans])
    with torch.no_grad():
        emb = lm.model.embed_tokens(ids.clamp(max=511))
        emb[rows] = want
        out = lm.generate(inputs_embeds=emb[None], attention_mask=torch.ones(1, len(ids), dtype=torch.long),
                          max_new_tokens=6, do_sample=False, output_scores=True, return_dict_in_generate=True,
                          eos_token_id=None)
    ref = out.sequences[0, -6:].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
