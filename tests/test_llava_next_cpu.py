"""LLaVA-NeXT / LLaVA-1.6 (``models/llava_next.py``) against transformers (tiny random
LlavaNextForConditionalGeneration with a CLIP tower and Llama LM, fp32, CPU reference ops): anyres
preprocessing vs the PIL processor, packed features (unpad, image_newline, every image anyres) and
greedy generation with log-probs through the engine, in the transformers layout and re-laid into
the original ``LlavaLlamaForCausalLM`` layout with ``image_aspect_ratio: anyres``."""
import json

import numpy as np
import pytest
import torch
from safetensors.torch import load_file, save_file

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
if not hasattr(transformers, "LlavaNextConfig"):
    pytest.skip("transformers without LLaVA-NeXT", allow_module_level=True)

from ome_amd.models.llava import ORIG_IMAGE_TOKEN  # noqa: E402
from ome_amd.models.llava_onevision import preprocess_onevision  # noqa: E402
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG = 500
PINS = [[56, 112], [112, 56], [112, 112], [168, 56], [56, 168]]


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = T.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=4096)
    vc = T.CLIPVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=3, num_attention_heads=4,
                            image_size=56, patch_size=14, projection_dim=64)
    m = T.LlavaNextForConditionalGeneration(T.LlavaNextConfig(
        text_config=tc, vision_config=vc, image_token_index=IMG, image_grid_pinpoints=PINS,
        vision_feature_layer=-2, vision_feature_select_strategy="default", tie_word_embeddings=False))
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
    ren = {}
    for k, v in sd.items():
        k = k[len("model."):] if k.startswith("model.") else k
        if k.startswith("vision_tower."):
            r = k[len("vision_tower."):]
            r = r[len("vision_model."):] if r.startswith("vision_model.") else r
            ren["model.vision_tower.vision_tower.vision_model." + r] = v
        elif k.startswith("multi_modal_projector.linear_1."):
            ren["model.mm_projector.0." + k.split(".")[-1]] = v
        elif k.startswith("multi_modal_projector.linear_2."):
            ren["model.mm_projector.2." + k.split(".")[-1]] = v
        elif k == "image_newline":
            ren["model.image_newline"] = v
        elif k.startswith("language_model."):
            r = k[len("language_model."):]
            ren[r if r.startswith(("model.", "lm_head")) else "model." + r] = v
        elif k == "lm_head.weight":
            ren[k] = v
    out.mkdir()
    save_file({k: v.contiguous() for k, v in ren.items()}, str(out / "model.safetensors"))
    c = json.loads((src / "config.json").read_text())
    vc = c["vision_config"]
    cfg = {**{k: v for k, v in c["text_config"].items() if k != "architectures"},
           "architectures": ["LlavaLlamaForCausalLM"], "model_type": "llava",
           "mm_vision_tower": "openai/clip-vit-large-patch14-336", "mm_projector_type": "mlp2x_gelu",
           "mm_vision_select_layer": -2, "mm_vision_select_feature": "patch", "mm_patch_merge_type": "spatial_unpad",
           "image_aspect_ratio": "anyres", "image_grid_pinpoints": PINS, "mm_hidden_size": 64,
           "vision_config": {k: vc[k] for k in ("hidden_size", "intermediate_size", "num_hidden_layers",
                                                 "num_attention_heads", "image_size", "patch_size")},
           "tie_word_embeddings": False}
    (out / "config.json").write_text(json.dumps(cfg))


def _hf_pixels(imgs):
    from transformers.models.llava_next.image_processing_pil_llava_next import LlavaNextImageProcessorPil

    proc = LlavaNextImageProcessorPil(image_grid_pinpoints=PINS, size={"shortest_edge": 56},
                                      crop_size={"height": 56, "width": 56}, image_mean=list(CLIP_MEAN),
                                      image_std=list(CLIP_STD))
    out = proc(images=imgs, return_tensors="pt")
    return out["pixel_values"], out["image_sizes"]


def test_llava_next_preprocessing_matches_hf():
    for im in (_image(0, 80, 60), _image(1, 40, 150), _image(2, 120, 110)):
        want, sizes = _hf_pixels([im])
        got, h, w = preprocess_onevision(im, [tuple(p) for p in PINS], 56, True, mean=CLIP_MEAN, std=CLIP_STD)
        assert (h, w) == tuple(sizes[0].tolist())
        assert (got - want[0, :got.shape[0]]).abs().max().item() < 1e-4


@pytest.mark.parametrize("layout,n_img", [("hf", 1), ("original", 1), ("hf", 2)])
def test_llava_next_matches_hf(tmp_path, layout, n_img):
    src = tmp_path / "hf"
    src.mkdir()
    hf = _hf_model(src)
    path, tok = src, IMG
    if layout == "original":
        path, tok = tmp_path / "orig", ORIG_IMAGE_TOKEN
        _to_original_layout(src, path)
    imgs = [_image(0, 80, 60), _image(1, 40, 150)][:n_img]
    eng = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=2048))
    m = eng.runner.model
    assert type(m).__name__ == "LlavaNextForConditionalGeneration" and m.orig == (layout == "original")
    pv, sizes = _hf_pixels(imgs)
    prompt = [1, 9, 17, tok, 33, 41] + ([tok, 12] if n_img == 2 else []) + [7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    with torch.no_grad():
        want = hf.model.get_image_features(pixel_values=pv, image_sizes=sizes)
        want = getattr(want, "pooler_output", want)
        want = torch.cat(list(want))
    got = m.encode_images(req.mm.pixel_values, req.mm.grid_thw)
    assert got.shape == want.shape and (got - want).abs().max().item() < 1e-3, (got.shape, want.shape)
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == want.shape[0]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    with torch.no_grad():
        out = hf.generate(torch.tensor([ex]), pixel_values=pv, image_sizes=sizes, max_new_tokens=6, do_sample=False,
                          output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
