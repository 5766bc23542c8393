"""Llama 4 with images against transformers (tiny random Llama4ForConditionalGeneration, fp32,
CPU reference ops): tile canvas selection, the vision tower + pixel-shuffle adapter + projector
on the same tiles, and greedy generation through the engine with the ``<|image|>`` placeholder
expanded into the tile-token layout (multi-tile image: separators + thumbnail).  Pixel-level
preprocessing parity is unpinned (the reference processor needs torchvision, absent here)."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.models.llama4_vision import best_canvas, preprocess_llama4, supported_canvases  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

PATCH, BOI, EOI, IMAGE, TX, TY = 500, 501, 502, 503, 504, 505


def _image(h, w, seed=0):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = dict(vocab_size=512, hidden_size=256, intermediate_size=256, intermediate_size_mlp=384, num_hidden_layers=2,
              num_attention_heads=4, num_key_value_heads=2, head_dim=64, num_local_experts=2, num_experts_per_tok=1,
              max_position_embeddings=1024, no_rope_layers=[1, 0], attention_chunk_size=64,
              interleave_moe_layer_step=1, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    vc = dict(hidden_size=176, num_attention_heads=2, intermediate_size=704, num_hidden_layers=2, image_size=56,
              patch_size=14, pixel_shuffle_ratio=0.5, projector_input_dim=256, projector_output_dim=256,
              vision_output_dim=256, rope_theta=10000)
    cfg = T.Llama4Config(text_config=tc, vision_config=vc, image_token_index=PATCH, boi_token_index=BOI,
                         eoi_token_index=EOI, image_placeholder_token_id=IMAGE, tile_x_separator_token_id=TX,
                         tile_y_separator_token_id=TY)
    m = T.Llama4ForConditionalGeneration(cfg)
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


def test_canvas_candidates_and_best_fit():
    # the reference processor's documented example: max_num_chunks=5, patch 224
    assert sorted(supported_canvases(5)) == sorted([(1, 4), (2, 2), (1, 1), (4, 1), (1, 3), (3, 1), (1, 2), (2, 1),
                                                    (1, 5), (5, 1)])
    assert best_canvas(200, 300, 5, 224) == (224, 448)   # documented: smallest up-scale, least area
    assert best_canvas(2000, 300, 16, 336) == (336 * 7, 336 * 2) or best_canvas(2000, 300, 16, 336)[0] > 336


def test_llama4_vision_tower_and_generate_match_hf(tmp_path):
    hf = _hf_model(tmp_path)
    img = _image(70, 120)        # least up-scale 1.4: 2 x 3 tiles of 56 px + thumbnail
    tiles, ratio = preprocess_llama4(img, 56, 16)
    assert ratio == (2, 3) and tiles.shape == (7, 3, 56, 56)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "Llama4ForConditionalGeneration"
    with torch.no_grad():
        feats = hf.get_image_features(pixel_values=tiles, vision_feature_select_strategy="default",
                                            return_dict=True).last_hidden_state
        want = hf.multi_modal_projector(feats.reshape(-1, feats.shape[-1]))
    got = m.encode_images(tiles, None)
    assert got.shape == want.shape and (got - want).abs().max().item() < 1e-3, (got - want).abs().max()

    prompt = [1, 9, 17, IMAGE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s0, k in req.mm.spans:   # content-hash ids on the patch rows -> the reference's <|patch|>
        assert len(set(ex[s0:s0 + k])) == 1
        ex[s0:s0 + k] = [PATCH] * k
    n = m.visual.tokens_per_tile
    row = [PATCH] * n + [TX] + [PATCH] * n + [TX] + [PATCH] * n + [TY]
    assert ex[3:4 + 2 * len(row)] == [BOI] + row + row and ex.count(PATCH) == 7 * n
    assert ex[4 + 2 * len(row):][:n + 2] == [IMAGE] + [PATCH] * n + [EOI]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    t = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(t, pixel_values=tiles, max_new_tokens=6, do_sample=False, output_scores=True,
                          return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tok].item() for s, tok in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
