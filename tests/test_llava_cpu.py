"""LLaVA-1.5 (``models/llava.py``) against transformers (tiny random LlavaForConditionalGeneration
with a CLIP tower, fp32, CPU reference ops): vision features from layer -2 without the class
token, projector, and greedy generation with two images through the engine -- in the llava-hf
layout and re-laid into the original LLaVA repository layout (``LlavaLlamaForCausalLM``,
``mm_projector.*``, ``vision_tower.vision_tower.*``, image token -200)."""
import json

import numpy as np
import pytest
import torch
from safetensors.torch import load_file, save_file

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.models.llava import ORIG_IMAGE_TOKEN, preprocess_clip  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG = 500


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = T.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024)
    vc = T.CLIPVisionConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3, num_attention_heads=2,
                            image_size=56, patch_size=14, projection_dim=64)
    m = T.LlavaForConditionalGeneration(T.LlavaConfig(text_config=tc, vision_config=vc, image_token_index=IMG))
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


def _to_original_layout(tmp_path, out):
    """llava-hf checkpoint -> the original LLaVA repository's names and config."""
    sd = {}
    for f in tmp_path.glob("*.safetensors"):
        sd.update(load_file(str(f)))
    ren = {}
    for k, v in sd.items():
        if k.startswith("model.vision_tower."):
            k = "model.vision_tower.vision_tower.vision_model." + k[len("model.vision_tower."):]
        elif k.startswith("model.multi_modal_projector.linear_1."):
            k = "model.mm_projector.0." + k.split(".")[-1]
        elif k.startswith("model.multi_modal_projector.linear_2."):
            k = "model.mm_projector.2." + k.split(".")[-1]
        elif k.startswith("model.language_model."):
            k = "model." + k[len("model.language_model."):]
        ren[k] = v.contiguous()
    out.mkdir()
    save_file(ren, str(out / "model.safetensors"))
    c = json.loads((tmp_path / "config.json").read_text())
    tc = c["text_config"]
    cfg = {**{k: v for k, v in tc.items() if k != "architectures"}, "architectures": ["LlavaLlamaForCausalLM"],
           "model_type": "llava_llama", "mm_vision_tower": "openai/clip-vit-large-patch14-336",
           "mm_projector_type": "mlp2x_gelu", "mm_vision_select_layer": -2, "mm_vision_select_feature": "patch",
           "mm_hidden_size": 128, "image_aspect_ratio": "square", "vision_config": c["vision_config"]}
    (out / "config.json").write_text(json.dumps(cfg))


@pytest.mark.parametrize("layout", ["hf", "original"])
def test_llava_matches_hf(tmp_path, layout):
    src = tmp_path / "hf"
    src.mkdir()
    hf = _hf_model(src)
    path, tok = src, IMG
    if layout == "original":
        path, tok = tmp_path / "orig", ORIG_IMAGE_TOKEN
        _to_original_layout(src, path)
    imgs = [_image(0), _image(1, 50, 90)]
    px = torch.cat([preprocess_clip(im, 56) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "LlavaForConditionalGeneration" and m.orig == (layout == "original")
    with torch.no_grad():
        want = torch.cat(list(hf.get_image_features(pixel_values=px, return_dict=True).pooler_output))
    got = m.encode_images(px)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, 17, tok, 33, 41, tok, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == 32
    eng.add_request(req)
    while not req.finished:
        eng.step()
    t = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(t, pixel_values=px, max_new_tokens=6, do_sample=False, output_scores=True,
                          return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
