"""Qwen2.5-VL against transformers (tiny random model, fp32, CPU reference ops): the windowed
vision tower (window-major patch permutation, window / full-attention layers, RMSNorm, biased
SwiGLU with a non-multiple-of-8 intermediate size) and greedy generation with an image through
the engine (the Qwen2-VL M-RoPE / placeholder path)."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.multimodal.inputs import expand_image_tokens, preprocess_image  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from tests.test_qwen2_vl_cpu import IMG, VE, VS, _image  # noqa: E402


def _hf_model(tmp_path):
    torch.manual_seed(0)
    # head dim 64: the LM also runs on the gfx950 kernels (tests/test_qwen2_5_vl_gpu.py)
    tc = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=1024, rms_norm_eps=1e-6, bos_token_id=1,
              eos_token_id=2, rope_parameters={"rope_type": "default", "rope_theta": 10000.0,
                                               "mrope_section": [8, 12, 12]})
    vc = dict(depth=3, hidden_size=64, intermediate_size=108, num_heads=4, patch_size=14, spatial_merge_size=2,
              temporal_patch_size=2, in_channels=3, window_size=84, fullatt_block_indexes=[1], out_hidden_size=256,
              hidden_act="silu")
    cfg = transformers.Qwen2_5_VLConfig(text_config=tc, vision_config=vc, image_token_id=IMG, video_token_id=501,
                                        vision_start_token_id=VS, vision_end_token_id=VE)
    m = transformers.Qwen2_5_VLForConditionalGeneration(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n or "ln_q" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config, m.config.text_config):
        c._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def test_qwen2_5_vl_tower_and_generate_match_hf(tmp_path):
    hf = _hf_model(tmp_path)
    img = _image(170, 230)   # 6 x 8 merge blocks, 3 x 3-block windows: partial windows on the w axis
    pv, grid = preprocess_image(img)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=1024))
    m = eng.runner.model
    assert type(m).__name__ == "Qwen2_5_VLForConditionalGeneration"
    with torch.no_grad():
        want_feat = hf.model.visual(torch.from_numpy(pv), grid_thw=torch.tensor([grid])).pooler_output
    got_feat = m.encode_images(torch.from_numpy(pv), [grid])
    assert (got_feat - want_feat).abs().max().item() < 1e-3
    # two images in one call (per-image window offsets and full-attention segments)
    pv2, grid2 = preprocess_image(_image(84, 112, seed=3))
    both = torch.cat([torch.from_numpy(pv), torch.from_numpy(pv2)])
    with torch.no_grad():
        want2 = hf.model.visual(both, grid_thw=torch.tensor([grid, grid2])).pooler_output
    assert (m.encode_images(both, [grid, grid2]) - want2).abs().max().item() < 1e-3

    prompt = [5, 9, 17, VS, IMG, VE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=5, ignore_eos=True, logprobs=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex, _ = expand_image_tokens(prompt, IMG, [grid], 2)
    t = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(t, pixel_values=torch.from_numpy(pv), image_grid_thw=torch.tensor([grid]),
                          mm_token_type_ids=(t == IMG).int(), max_new_tokens=5, do_sample=False,
                          output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tok].item() for s, tok in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
