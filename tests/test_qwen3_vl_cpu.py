"""Qwen3-VL dense and MoE against transformers (tiny random models, fp32, CPU reference ops):
the vision tower (interpolated learned positions, deepstack mergers), the Qwen2-VL image
processor contract at patch 16 / mean = std = 0.5, and greedy generation with log-probs through
the engine (interleaved M-RoPE table on the image chunk, deepstack features added after the
first decoder layers, one-shot and chunked prefill)."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.multimodal.inputs import expand_image_tokens, preprocess_image  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, VS, VE = 500, 502, 503


def _image(h=150, w=97, seed=0):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path, moe: bool):
    T = transformers
    torch.manual_seed(0)
    tc = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=3, num_attention_heads=4,
              num_key_value_heads=2, head_dim=64, max_position_embeddings=2048, rms_norm_eps=1e-6,
              rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "mrope_section": [12, 10, 10],
                               "mrope_interleaved": True})
    if moe:
        tc.update(num_experts=4, num_experts_per_tok=2, moe_intermediate_size=128, decoder_sparse_step=1,
                  norm_topk_prob=True)
    vc = dict(depth=3, hidden_size=64, intermediate_size=128, num_heads=2, patch_size=16, spatial_merge_size=2,
              temporal_patch_size=2, in_channels=3, out_hidden_size=256, num_position_embeddings=64,
              deepstack_visual_indexes=[0, 1])
    Cfg, Mdl = (T.Qwen3VLMoeConfig, T.Qwen3VLMoeForConditionalGeneration) if moe else \
        (T.Qwen3VLConfig, T.Qwen3VLForConditionalGeneration)
    m = Mdl(Cfg(text_config=tc, vision_config=vc, image_token_id=IMG, video_token_id=501,
                vision_start_token_id=VS, vision_end_token_id=VE))
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


def test_preprocess_matches_hf_processor():
    from transformers.models.qwen2_vl.image_processing_pil_qwen2_vl import Qwen2VLImageProcessorPil

    img = _image(150, 97)
    proc = Qwen2VLImageProcessorPil(patch_size=16, image_mean=[0.5] * 3, image_std=[0.5] * 3,
                                    size={"shortest_edge": 65536, "longest_edge": 16777216})
    want = proc(images=[img], return_tensors="np")
    pv, grid = preprocess_image(img, patch=16, min_pixels=65536, max_pixels=16777216, mean=(0.5,) * 3, std=(0.5,) * 3)
    assert tuple(want["image_grid_thw"][0]) == grid
    assert np.abs(want["pixel_values"] - pv).max() < 2e-2


@pytest.mark.parametrize("moe,chunk", [(False, 8192), (False, 50), (True, 8192)])
def test_qwen3_vl_matches_hf(tmp_path, moe, chunk):
    hf = _hf_model(tmp_path, moe)
    img = _image(120, 90)
    pv, grid = preprocess_image(img, patch=16, min_pixels=65536, max_pixels=16777216, mean=(0.5,) * 3,
                                std=(0.5,) * 3)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=1024, chunked_prefill_size=chunk))
    m = eng.runner.model
    assert type(m).__name__ == ("Qwen3VLMoeForConditionalGeneration" if moe else "Qwen3VLForConditionalGeneration")
    with torch.no_grad():
        out = hf.model.visual(torch.from_numpy(pv), grid_thw=torch.tensor([grid]))
    main, deep = m.encode_images(torch.from_numpy(pv), [grid])
    assert (main - out.pooler_output).abs().max().item() < 1e-3
    assert len(deep) == 2 and all((a - b).abs().max().item() < 1e-3 for a, b in zip(deep, out.deepstack_features))
    prompt = [5, 9, 17, VS, IMG, VE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex, _ = expand_image_tokens(prompt, IMG, [grid], 2)
    t = torch.tensor([ex])
    with torch.no_grad():
        o = hf.generate(t, pixel_values=torch.from_numpy(pv), image_grid_thw=torch.tensor([grid]),
                        mm_token_type_ids=(t == IMG).int(), max_new_tokens=6, do_sample=False,
                        output_scores=True, return_dict_in_generate=True)
    ref = o.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tok].item() for s, tok in zip(o.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
