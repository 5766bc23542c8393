"""Mistral 3 / Pixtral (``models/mistral3.py``) against transformers (tiny random
Mistral3ForConditionalGeneration, fp32, CPU reference ops): Pixtral preprocessing vs the PIL
image processor, tower + projector features for two differently-sized images, and greedy
generation with log-probs through the engine ([IMG] rows spliced between [IMG_BREAK] /
[IMG_END] tokens)."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
if not hasattr(transformers, "Mistral3Config"):
    pytest.skip("transformers without Mistral3", allow_module_level=True)

from ome_amd.models.mistral3 import preprocess_pixtral  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, BRK, END = 10, 12, 13


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = T.MistralConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=2, head_dim=64, max_position_embeddings=1024,
                         sliding_window=None)
    vc = T.PixtralVisionConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3, num_attention_heads=4,
                               head_dim=32, image_size=112, patch_size=14, hidden_act="silu")
    m = T.Mistral3ForConditionalGeneration(T.Mistral3Config(text_config=tc, vision_config=vc, image_token_index=IMG,
                                                            spatial_merge_size=2, tie_word_embeddings=False))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config, m.config.text_config):
        c._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def _hf_pixels(im, longest=112):
    from transformers.models.pixtral.image_processing_pil_pixtral import PixtralImageProcessorPil

    proc = PixtralImageProcessorPil(size={"longest_edge": longest}, patch_size={"height": 28, "width": 28})
    out = proc(images=[im], return_tensors="pt")
    return out["pixel_values"][0], tuple(int(x) for x in out["image_sizes"][0])


def test_pixtral_preprocessing_matches_hf():
    for im in (_image(0, 80, 60), _image(1, 300, 170), _image(2, 20, 33)):
        want, (H, W) = _hf_pixels(im)
        rows, h, w = preprocess_pixtral(im, 112, 28, 14)
        assert (h * 14, w * 14) == (H, W)
        got = rows.view(h, w, 3, 14, 14).permute(2, 0, 3, 1, 4).reshape(3, H, W)
        assert (got - want[:, :H, :W]).abs().max().item() < 1e-4


def test_mistral3_matches_hf(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 50, 110)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "Mistral3ForConditionalGeneration"
    pix = [_hf_pixels(im) for im in imgs]
    Hm, Wm = max(p[1][0] for p in pix), max(p[1][1] for p in pix)
    pv = torch.zeros(2, 3, Hm, Wm)
    for i, (p, (H, W)) in enumerate(pix):
        pv[i, :, :H, :W] = p[:, :H, :W]
    sizes = torch.tensor([p[1] for p in pix])
    with torch.no_grad():
        want = torch.cat(list(hf.get_image_features(pixel_values=pv, image_sizes=sizes, return_dict=True).pooler_output))
    pre = [preprocess_pixtral(im, 112, 28, 14) for im in imgs]
    got = m.encode_images(torch.cat([r for r, _, _ in pre]), [(1, h, w) for _, h, w in pre])
    assert got.shape == want.shape and (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, 17, IMG, 33, 41, IMG, 22, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == want.shape[0] and ex.count(END) == 2 and BRK in ex
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
