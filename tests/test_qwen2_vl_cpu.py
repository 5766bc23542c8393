"""Qwen2-VL against Hugging Face transformers (tiny random model, fp32, CPU reference ops):

* preprocessing: ``preprocess_image`` == ``Qwen2VLImageProcessor`` pixel_values / grid;
* vision tower: merged features == HF ``model.visual(...).pooler_output``;
* M-RoPE positions == HF ``get_rope_index``;
* end to end through the engine (image placeholder expansion, vision features spliced into the
  prefill rows, per-row M-RoPE table, ``rope_delta`` on decode rows, chunked prefill that splits
  an image span): greedy tokens and their log-probs == HF ``generate``."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.multimodal.inputs import expand_image_tokens, mrope_positions, preprocess_image  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, VS, VE = 500, 502, 503


def _image(h=112, w=84, seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    return Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    torch.manual_seed(0)
    tc = dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=1024, rms_norm_eps=1e-6, bos_token_id=1,
              eos_token_id=2, rope_parameters={"rope_type": "default", "rope_theta": 10000.0,
                                               "mrope_section": [4, 6, 6]})
    vc = dict(depth=2, embed_dim=64, hidden_size=128, num_heads=4, mlp_ratio=2, patch_size=14,
              spatial_merge_size=2, temporal_patch_size=2, in_channels=3)
    cfg = transformers.Qwen2VLConfig(text_config=tc, vision_config=vc, image_token_id=IMG, video_token_id=501,
                                     vision_start_token_id=VS, vision_end_token_id=VE)
    m = transformers.Qwen2VLForConditionalGeneration(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n or "ln_q" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.config.vision_config._attn_implementation = "eager"
    m.config.text_config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None  # compare fixed-length continuations (ignore_eos)
    return m


def test_preprocess_matches_hf_processor():
    from transformers.models.qwen2_vl.image_processing_pil_qwen2_vl import Qwen2VLImageProcessorPil

    img = _image(150, 97)
    proc = Qwen2VLImageProcessorPil()
    want = proc(images=[img], return_tensors="np")
    pv, grid = preprocess_image(img)
    assert tuple(want["image_grid_thw"][0]) == grid
    assert np.abs(want["pixel_values"] - pv).max() < 2e-2  # resampler rounding only


def test_mrope_positions_match_hf(tmp_path):
    hf = _hf_model(tmp_path)
    grids = [(1, 8, 6), (1, 4, 4)]
    ids = [5, 6, VS, IMG, VE, 7, VS, IMG, VE, 8, 9]
    ex, spans = expand_image_tokens(ids, IMG, grids, 2)
    pos, delta = mrope_positions(len(ex), spans, grids, 2)
    t = torch.tensor([ex])
    tt = (t == IMG).int()
    want, wd = hf.model.get_rope_index(t, tt, image_grid_thw=torch.tensor(grids))
    assert np.array_equal(want[:, 0].numpy(), pos) and int(wd) == delta


@pytest.mark.parametrize("chunk", [8192, 10])  # 10: the image span straddles two chunks
def test_qwen2_vl_generate_matches_hf(tmp_path, chunk):
    hf = _hf_model(tmp_path)
    img = _image()
    pv, grid = preprocess_image(img)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512, chunked_prefill_size=chunk))
    m = eng.runner.model
    assert type(m).__name__ == "Qwen2VLForConditionalGeneration"
    # vision tower alone
    with torch.no_grad():
        want_feat = hf.model.visual(torch.from_numpy(pv), grid_thw=torch.tensor([grid])).pooler_output
    got_feat = m.encode_images(torch.from_numpy(pv), [grid])
    assert (got_feat - want_feat).abs().max().item() < 1e-3
    prompt = [5, 9, 17, VS, IMG, VE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex, _ = expand_image_tokens(prompt, IMG, [grid], 2)
    t = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(t, pixel_values=torch.from_numpy(pv), image_grid_thw=torch.tensor([grid]),
                          mm_token_type_ids=(t == IMG).int(), max_new_tokens=6, do_sample=False,
                          output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tok].item() for s, tok in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)


def test_text_only_prompt_on_vl_model(tmp_path):
    hf = _hf_model(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    ids = [(7 * i + 3) % 490 + 3 for i in range(30)]
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=5, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=5, ignore_eos=True))[0].output_ids == ref


def test_gme_style_image_text_embedding_matches_hf(tmp_path):
    """GME-Qwen2-VL (reference ``config/models/Alibaba-NLP/gme-Qwen2-VL-2B-Instruct.yaml``): a
    Qwen2-VL checkpoint served with --is-embedding; an image + text prompt is embedded as the
    L2-normalised final hidden state of its last token (GME's pooling)."""
    hf = _hf_model(tmp_path)
    img = _image()
    pv, grid = preprocess_image(img)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512, is_embedding=True))
    prompt = [5, 9, VS, IMG, VE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=0))
    req.is_embedding = True
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex, _ = expand_image_tokens(prompt, IMG, [grid], 2)
    t = torch.tensor([ex])
    with torch.no_grad():
        h = hf.model(input_ids=t, pixel_values=torch.from_numpy(pv), image_grid_thw=torch.tensor([grid]),
                     mm_token_type_ids=(t == IMG).int()).last_hidden_state[0, -1]
    want = torch.nn.functional.normalize(h.float(), dim=-1)
    got = torch.tensor(req.embedding)
    assert (got - want).abs().max().item() < 1e-3
