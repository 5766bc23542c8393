"""Phi-4-multimodal (``models/phi4mm.py``) on CPU reference ops against transformers (tiny random
``Phi4MultimodalForCausalLM``, fp32): dynamic-HD image features (NaViT bucketed positions over each
crop's valid patches, padded-patch queries, layer -2 features, 2 x 2 pooling cropped to the useful
extent, sub / global separators, projector) and greedy generation with log-probs through the
engine on the Phi-3 decoder path (partial rotary 0.75).  The original checkpoint layout
(``base_layer`` + LoRA names, ``img_projection.0/2``, ``glb_GN`` / ``sub_GN``) is checked with the
vision LoRA folded in.  The HD preprocessing rule is transcribed from the transformers processor,
which needs torchvision (absent here): the crop / padding / token-count arithmetic is checked,
pixel parity is unpinned."""
import json

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
if not hasattr(transformers, "Phi4MultimodalConfig"):
    pytest.skip("transformers without Phi-4-multimodal", allow_module_level=True)

from safetensors.torch import load_file, save_file  # noqa: E402

from ome_amd.models.phi4mm import crop_masks, hd_layout, num_image_tokens, preprocess_phi4mm  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG = 500


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    vc = dict(hidden_size=64, intermediate_size=96, num_hidden_layers=3, num_attention_heads=4, image_size=56,
              patch_size=14, crop_size=56, image_token_id=IMG)
    ac = dict(hidden_size=64, intermediate_size=64, num_blocks=1, num_attention_heads=4, nemo_conv_channels=32,
              ext_pw_out_channel=64, depthwise_separable_out_channel=64, audio_token_id=501)
    cfg = T.Phi4MultimodalConfig(vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2,
                                 num_attention_heads=4, num_key_value_heads=2, vision_config=vc, audio_config=ac,
                                 partial_rotary_factor=0.75, max_position_embeddings=2048,
                                 original_max_position_embeddings=2048, pad_token_id=0, bos_token_id=1,
                                 eos_token_id=2)
    m = T.Phi4MultimodalForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config):
        c._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def _hf_inputs(imgs):
    pre = [preprocess_phi4mm(im, 56, 14) for im in imgs]
    n = max(p.shape[0] for p, _ in pre)
    pv = torch.zeros(len(pre), n, 3, 56, 56)
    am = torch.ones(len(pre), n, 4, 4)
    sizes = []
    for i, (p, g) in enumerate(pre):
        pv[i, :p.shape[0]] = p
        am[i, :p.shape[0]] = crop_masks(g, 4).float()
        sizes.append([g[0] * 56, g[1] * 56])
    return pre, pv, am, torch.tensor(sizes)


def _to_original(src, dst, lora_r=4):
    """transformers names -> the original checkpoint's (``base_layer`` weights with a vision LoRA
    pair whose product is subtracted, so that folding it back restores the transformers weights)."""
    import shutil

    dst.mkdir()
    w = load_file(str(src / "model.safetensors"))
    g = torch.Generator().manual_seed(3)
    out = {}
    for n, t in w.items():
        n = n.replace("image_embed.img_projection_up", "image_embed.img_projection.0")
        n = n.replace("image_embed.img_projection_down", "image_embed.img_projection.2")
        n = n.replace("image_embed.global_img_feature_extensor", "image_embed.glb_GN")
        n = n.replace("image_embed.sub_img_feature_extensor", "image_embed.sub_GN")
        if n.startswith("model.layers.") and n.endswith(("qkv_proj.weight", "o_proj.weight", "gate_up_proj.weight",
                                                            "down_proj.weight")):
            base = n[:-len(".weight")]
            A = torch.randn(lora_r, t.shape[1], generator=g) * 0.1
            B = torch.randn(t.shape[0], lora_r, generator=g) * 0.1
            out[base + ".base_layer.weight"] = t - 2.0 * B @ A          # lora_alpha / r = 8 / 4
            out[base + ".lora_A.vision.weight"], out[base + ".lora_B.vision.weight"] = A, B
            out[base + ".lora_A.speech.weight"] = torch.randn(lora_r, t.shape[1], generator=g)
            out[base + ".lora_B.speech.weight"] = torch.randn(t.shape[0], lora_r, generator=g)
            continue
        out[n] = t
    save_file({k: v.contiguous() for k, v in out.items()}, str(dst / "model.safetensors"))
    cfg = json.loads((src / "config.json").read_text())
    cfg.update(architectures=["Phi4MMForCausalLM"], vision_lora={"r": lora_r, "lora_alpha": 2 * lora_r,
                                                                  "layer": "all-linear"})
    (dst / "config.json").write_text(json.dumps(cfg))
    shutil.copy(src / "generation_config.json", dst / "generation_config.json")


def test_hd_layout_rule():
    assert hd_layout(80, 60, 56) == ((2, 2), (84, 112), (28, 0))
    assert hd_layout(60, 110, 56) == ((2, 2), (112, 61), (0, 51))
    (wc, hc), (nw, nh), (pw, ph) = hd_layout(300, 9000, 448, max_num=36)   # closest-ratio branch
    assert wc * hc <= 36 and wc >= hc and (pw == 0 or ph == 0)
    _, g = preprocess_phi4mm(_image(1, 60, 110), 56, 14)
    assert g == (2, 2, 3, 0) and num_image_tokens(g, 4) == 3 * (4 + 1) + 1 + 6
    g448 = (1, 2, 0, 5)
    assert num_image_tokens(g448, 32) == 256 + 1 + 16 * 30 + 16 + 16   # the reference processor's formula


@pytest.mark.parametrize("layout", ["transformers", "original"])
def test_phi4mm_matches_hf(tmp_path, layout, monkeypatch):
    hf = _hf_model(tmp_path / "hf")
    path = tmp_path / "hf"
    if layout == "original":
        path = tmp_path / "orig"
        _to_original(tmp_path / "hf", path)
        monkeypatch.setenv("OME_PHI4MM_VISION_LORA", "1")
    imgs = [_image(0, 80, 60), _image(1, 60, 110)]
    eng = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=1024))
    m = eng.runner.model
    assert type(m).__name__ == "Phi4MMForCausalLM"
    m.crop = 56
    pre, pv, am, sizes = _hf_inputs(imgs)
    prompt = [1, 9, IMG, 33, 41, IMG, 12, 7]
    req = eng.make_mm_request(prompt, [(p, g) for p, g in pre],
                              SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    ids = torch.tensor([ex])
    with torch.no_grad():
        emb = hf.model.embed_tokens(ids)
        want = hf.model.embed_tokens_extend(ids, emb, image_pixel_values=pv, image_sizes=sizes,
                                            image_attention_mask=am)[0][ids[0] == IMG]
    got = m.encode_images(req.mm.pixel_values, req.mm.grid_thw)
    assert got.shape == want.shape and (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    eng.add_request(req)
    while not req.finished:
        eng.step()
    with torch.no_grad():
        out = hf.generate(ids, image_pixel_values=pv, image_sizes=sizes, image_attention_mask=am, max_new_tokens=6,
                          do_sample=False, output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
