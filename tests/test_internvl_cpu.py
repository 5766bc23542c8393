"""InternVL (``models/internvl.py``) against transformers (tiny random
InternVLForConditionalGeneration with a Qwen2 LM, fp32, CPU reference ops): dynamic-tiling
preprocessing vs the transformers PIL processor, vision features (InternViT + pixel shuffle +
projector) and greedy generation with log-probs through the engine -- in the transformers layout
and re-laid into the original ``InternVLChatModel`` layout (``vision_model.*``, ``mlp1.*``,
``language_model.*``, ``llm_config``)."""
import json

import numpy as np
import pytest
import torch
from safetensors.torch import load_file, save_file

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
if not hasattr(transformers, "InternVLConfig"):
    pytest.skip("transformers without InternVL", allow_module_level=True)

from ome_amd.models.internvl import IMAGENET_MEAN, IMAGENET_STD, preprocess_internvl  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, START, END = 500, 501, 502


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = T.Qwen2Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=2048)
    vc = T.InternVLVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=3, num_attention_heads=4,
                                image_size=[112, 112], patch_size=[14, 14], attention_bias=True)
    cfg = T.InternVLConfig(text_config=tc, vision_config=vc, image_token_id=IMG, image_seq_length=16,
                           downsample_ratio=0.5, img_start_token_id=START, img_end_token_id=END,
                           max_dynamic_patch=6, tie_word_embeddings=False)
    m = T.InternVLForConditionalGeneration(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            elif "lambda" in n:
                p.normal_(0.5, 0.1)
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
        if k.startswith("vision_tower."):
            r = k[len("vision_tower."):]
            r = (r.replace("embeddings.cls_token", "embeddings.class_embedding")
                 .replace("embeddings.patch_embeddings.projection", "embeddings.patch_embedding")
                 .replace("embeddings.position_embeddings", "embeddings.position_embedding")
                 .replace("encoder.layer.", "encoder.layers.").replace("attention.projection_layer", "attn.proj")
                 .replace("layernorm_before", "norm1").replace("layernorm_after", "norm2")
                 .replace("lambda_1", "ls1").replace("lambda_2", "ls2"))
            if ".attention." in r:   # q / k / v -> fused attn.qkv
                pre, proj, kind = r.split(".attention.")[0], r.split(".")[-2], r.split(".")[-1]
                qkv.setdefault((pre, kind), {})[proj[0]] = v
                continue
            ren["vision_model." + r] = v
        elif k.startswith("multi_modal_projector."):
            r = k[len("multi_modal_projector."):]
            r = r.replace("layer_norm", "mlp1.0").replace("linear_1", "mlp1.1").replace("linear_2", "mlp1.3")
            ren[r] = v
        elif k.startswith("language_model."):
            ren[k] = v
    for (pre, kind), d in qkv.items():
        ren[f"vision_model.{pre}.attn.qkv.{kind}"] = torch.cat([d["q"], d["k"], d["v"]])
    out.mkdir()
    save_file({k: v.contiguous() for k, v in ren.items()}, str(out / "model.safetensors"))
    c = json.loads((src / "config.json").read_text())
    vc = c["vision_config"]
    cfg = {"architectures": ["InternVLChatModel"], "model_type": "internvl_chat",
           "llm_config": {**c["text_config"], "architectures": ["Qwen2ForCausalLM"]},
           "vision_config": {"hidden_size": vc["hidden_size"], "intermediate_size": vc["intermediate_size"],
                             "num_attention_heads": vc["num_attention_heads"],
                             "num_hidden_layers": vc["num_hidden_layers"], "image_size": 112, "patch_size": 14,
                             "qkv_bias": True, "qk_normalization": False, "norm_type": "layer_norm",
                             "layer_norm_eps": vc["layer_norm_eps"], "hidden_act": "gelu"},
           "downsample_ratio": 0.5, "select_layer": -1, "ps_version": "v2", "dynamic_image_size": True,
           "max_dynamic_patch": 6, "use_thumbnail": True, "img_context_token_id": IMG, "img_start_token_id": START,
           "img_end_token_id": END, "tie_word_embeddings": False}
    (out / "config.json").write_text(json.dumps(cfg))


def test_internvl_tiling_matches_hf():
    from transformers.models.got_ocr2.image_processing_pil_got_ocr2 import GotOcr2ImageProcessorPil

    proc = GotOcr2ImageProcessorPil(crop_to_patches=True, max_patches=6, size={"height": 112, "width": 112},
                                    image_mean=list(IMAGENET_MEAN), image_std=list(IMAGENET_STD))
    for im in (_image(0, 80, 60), _image(1, 100, 330), _image(2, 300, 300), _image(3, 50, 200)):
        want = proc(images=[im], return_tensors="pt")["pixel_values"]
        got = preprocess_internvl(im, 112, 6)
        assert got.shape == want.shape and (got - want).abs().max().item() < 1e-4


@pytest.mark.parametrize("layout", ["hf", "original"])
def test_internvl_matches_hf(tmp_path, layout):
    src = tmp_path / "hf"
    src.mkdir()
    hf = _hf_model(src)
    path = src
    if layout == "original":
        path = tmp_path / "orig"
        _to_original_layout(src, path)
    imgs = [_image(0, 80, 60), _image(1, 100, 330)]
    px = torch.cat([preprocess_internvl(im, 112, 6) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=1024))
    m = eng.runner.model
    assert m.orig_layout == (layout == "original") and m.tokens_per_tile == 16
    with torch.no_grad():
        want = torch.cat(list(hf.get_image_features(pixel_values=px, return_dict=True).pooler_output))
    got = m.encode_images(px)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, START, IMG, END, 33, 41, START, IMG, END, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == px.shape[0] * 16
    eng.add_request(req)
    while not req.finished:
        eng.step()
    with torch.no_grad():
        out = hf.generate(torch.tensor([ex]), pixel_values=px, max_new_tokens=6, do_sample=False, output_scores=True,
                          return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
