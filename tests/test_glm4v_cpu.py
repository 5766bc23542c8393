"""GLM-4.5V (``models/glm4v.py``) against transformers (tiny random Glm4vMoeForConditionalGeneration,
fp32, CPU reference ops): GLM-4V preprocessing vs the PIL processor, vision features
(grid-sampled positions, SwiGLU blocks, down-sampling conv, merger) and greedy generation with
log-probs through the engine (M-RoPE over the partial rotary half, sigmoid grouped MoE routing
with correction bias, shared expert, dense first layer)."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
if not hasattr(transformers, "Glm4vMoeConfig"):
    pytest.skip("transformers without GLM-4.5V", allow_module_level=True)

from ome_amd.models.glm4v import preprocess_glm4v  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, BOI, EOI = 500, 501, 502


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = dict(vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, head_dim=64, attention_bias=True, moe_intermediate_size=64, n_routed_experts=8,
              num_experts_per_tok=2, n_shared_experts=1, first_k_dense_replace=1, n_group=2, topk_group=1,
              routed_scaling_factor=2.0, norm_topk_prob=True, max_position_embeddings=2048,
              rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "partial_rotary_factor": 0.5,
                               "mrope_section": [4, 6, 6]})
    vc = dict(hidden_size=64, depth=2, num_heads=4, out_hidden_size=256, intermediate_size=128, image_size=56,
              patch_size=14, spatial_merge_size=2, temporal_patch_size=2)
    cfg = T.Glm4vMoeConfig(text_config=tc, vision_config=vc, image_token_id=IMG, image_start_token_id=BOI,
                           image_end_token_id=EOI, tie_word_embeddings=False)
    m = T.Glm4vMoeForConditionalGeneration(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            else:
                p.normal_(0.0, 0.08)
        for n, b in m.named_buffers():
            if n.endswith("e_score_correction_bias"):
                b.normal_(0.0, 0.05)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config, m.config.text_config):
        c._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def _hf_pixels(imgs):
    from transformers.models.glm4v.image_processing_pil_glm4v import Glm4vImageProcessorPil

    proc = Glm4vImageProcessorPil()
    out = proc(images=imgs, return_tensors="pt")
    return out["pixel_values"], out["image_grid_thw"]


def test_glm4v_preprocessing_matches_hf():
    for im in (_image(0, 80, 60), _image(1, 20, 90), _image(2, 300, 170)):
        want, grid = _hf_pixels([im])
        got, g = preprocess_glm4v(im)
        assert tuple(grid[0].tolist()) == g
        assert np.abs(got - want.numpy()).max() < 1e-4


def test_glm4v_matches_hf(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 60, 110)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=1024))
    m = eng.runner.model
    assert type(m).__name__ == "Glm4vMoeForConditionalGeneration" and m.cfg.rot_dim == 32
    pv, grid = _hf_pixels(imgs)
    with torch.no_grad():
        want = torch.cat(list(hf.model.get_image_features(pixel_values=pv, image_grid_thw=grid).pooler_output))
    got = m.encode_images(pv, [tuple(g.tolist()) for g in grid])
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, BOI, IMG, EOI, 33, 41, BOI, IMG, EOI, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == want.shape[0]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(ids, pixel_values=pv, image_grid_thw=grid, mm_token_type_ids=(ids == IMG).int(),
                          max_new_tokens=6, do_sample=False, output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
