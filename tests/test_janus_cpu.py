"""Janus / Janus-Pro image understanding (``models/janus.py``) against transformers (tiny random
JanusForConditionalGeneration, fp32, CPU reference ops): preprocessing vs the PIL processor,
SigLIP tower + aligner features and greedy generation with log-probs through the engine -- in the
transformers layout and re-laid into the original ``MultiModalityCausalLM`` layout (timm tower
names, ``aligner.layers.*``, ``language_config``)."""
import json

import numpy as np
import pytest
import torch
from safetensors.torch import load_file, save_file

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
if not hasattr(transformers, "JanusConfig"):
    pytest.skip("transformers without Janus", allow_module_level=True)

from ome_amd.models.janus import preprocess_janus  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, BOI, EOI = 500, 501, 502


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = T.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024)
    vc = T.JanusVisionConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, image_size=64, patch_size=16,
                             projection_dim=256, depth=2, num_image_tokens=16)
    vq = T.JanusVQVAEConfig(embed_dim=8, num_embeddings=64, latent_channels=32, base_channels=32,
                            channel_multiplier=[1, 1], num_res_blocks=1, num_patches=4, projection_dim=256,
                            image_token_embed_dim=256)
    m = T.JanusForConditionalGeneration(T.JanusConfig(text_config=tc, vision_config=vc, vq_config=vq,
                                                      image_token_id=IMG, tie_word_embeddings=False))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config, m.config.text_config):
        c._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def _to_original_layout(src, out):
    sd = {}
    for f in src.glob("*.safetensors"):
        sd.update(load_file(str(f)))
    ren, qkv = {}, {}
    for k, v in sd.items():
        k = k[len("model."):] if k.startswith("model.") else k
        if k.startswith("vision_model."):
            r = k[len("vision_model."):]
            if r.startswith("embeddings.patch_embedding."):
                r = "patch_embed.proj." + r.split(".")[-1]
            elif r == "embeddings.position_embedding.weight":
                r, v = "pos_embed", v[None]
            elif r.startswith("post_layernorm."):
                r = "norm." + r.split(".")[-1]
            elif r.startswith("encoder.layers."):
                p = r.split(".")
                b, mod, kind = p[2], ".".join(p[3:-1]), p[-1]
                if mod in ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"):
                    qkv.setdefault((b, kind), {})[mod[-6]] = v
                    continue
                mod = {"self_attn.projection_layer": "attn.proj", "layer_norm1": "norm1",
                       "layer_norm2": "norm2"}.get(mod, mod)
                r = f"blocks.{b}.{mod}.{kind}"
            ren["vision_model.vision_tower." + r] = v
        elif k.startswith("aligner."):
            p = k.split(".")
            idx = 0 if p[1] == "fc1" else 2 * (int(p[2]) + 1)
            ren[f"aligner.layers.{idx}.{p[-1]}"] = v
        elif k.startswith("language_model."):
            ren[k] = v
        elif k == "lm_head.weight":
            ren["language_model.lm_head.weight"] = v
    for (b, kind), d in qkv.items():
        ren[f"vision_model.vision_tower.blocks.{b}.attn.qkv.{kind}"] = torch.cat([d["q"], d["k"], d["v"]])
    out.mkdir()
    save_file({k: v.contiguous() for k, v in ren.items()}, str(out / "model.safetensors"))
    c = json.loads((src / "config.json").read_text())
    cfg = {"architectures": ["MultiModalityCausalLM"], "model_type": "multi_modality",
           "language_config": {**c["text_config"], "architectures": ["LlamaForCausalLM"]},
           "vision_config": {"cls": "CLIPVisionTower", "params": {"image_size": 64, "model_name":
                                                                 "siglip_large_patch16_384", "select_layer": -1}},
           "aligner_config": {"cls": "MlpProjector", "params": {"depth": 2, "input_dim": 64, "n_embed": 256,
                                                                "projector_type": "mlp_gelu"}},
           "image_token_id": IMG, "boi_token_id": BOI, "eoi_token_id": EOI, "tie_word_embeddings": False}
    (out / "config.json").write_text(json.dumps(cfg))


def test_janus_preprocessing_matches_hf():
    from transformers.models.janus.image_processing_pil_janus import JanusImageProcessorPil

    proc = JanusImageProcessorPil(size={"height": 64, "width": 64}, image_mean=[0.5] * 3, image_std=[0.5] * 3)
    for im in (_image(0, 80, 60), _image(1, 50, 200), _image(2, 64, 64)):
        want = proc(images=[im], return_tensors="pt")["pixel_values"]
        got = preprocess_janus(im, 64)
        assert got.shape == want.shape and (got - want).abs().max().item() < 1e-4


@pytest.mark.parametrize("layout", ["hf", "original"])
def test_janus_matches_hf(tmp_path, layout, monkeypatch):
    import ome_amd.models.janus as J

    src = tmp_path / "hf"
    src.mkdir()
    hf = _hf_model(src)
    path = src
    if layout == "original":
        # the original config only names the timm tower; the tiny test tower stands in for SigLIP-L
        monkeypatch.setattr(J, "SIGLIP_L16_384", dict(hidden_size=64, intermediate_size=256, num_hidden_layers=2,
                                                      num_attention_heads=4, image_size=64, patch_size=16,
                                                      hidden_act="gelu", layer_norm_eps=1e-6))
        path = tmp_path / "orig"
        _to_original_layout(src, path)
    imgs = [_image(0), _image(1, 50, 90)]
    px = torch.cat([preprocess_janus(im, 64) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512))
    m = eng.runner.model
    assert m.orig == (layout == "original") and m.n_tokens == 16
    with torch.no_grad():
        want = torch.cat(list(hf.model.get_image_features(pixel_values=px).pooler_output))
    got = m.encode_images(px)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    if layout == "hf":
        m.boi, m.eoi = BOI, EOI
    prompt = [1, 9, BOI, IMG, EOI, 33, 41, BOI, IMG, EOI, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == 32
    eng.add_request(req)
    while not req.finished:
        eng.step()
    with torch.no_grad():
        out = hf.generate(torch.tensor([ex]), pixel_values=px, max_new_tokens=6, do_sample=False, output_scores=True,
                          return_dict_in_generate=True, generation_mode="text")
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
