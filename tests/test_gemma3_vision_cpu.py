"""Gemma 3 with images against transformers (tiny random Gemma3ForConditionalGeneration, fp32,
CPU reference ops): the SigLIP tower + pooled projector, and greedy generation through the engine
with bidirectional attention inside each image block (the per-row visible-key limit of the
prefill attention) on sliding-window and global layers, including a chunked prefill that the
scheduler must not split inside an image block."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.models.gemma3_vision import preprocess_gemma3  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

SOFT, BOI, EOI, NL2 = 500, 501, 502, 108


def _image(seed=0, h=90, w=130):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, head_dim=64, max_position_embeddings=1024, sliding_window=8,
              layer_types=["sliding_attention", "full_attention"], pad_token_id=0, bos_token_id=2, eos_token_id=1)
    vc = dict(hidden_size=144, intermediate_size=288, num_hidden_layers=2, num_attention_heads=2, image_size=112,
              patch_size=14)
    cfg = T.Gemma3Config(text_config=tc, vision_config=vc, mm_tokens_per_image=16, image_token_index=SOFT,
                         boi_token_index=BOI, eoi_token_index=EOI, image_newline_token_id=NL2)
    m = T.Gemma3ForConditionalGeneration(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(0.0, 0.1) if "language_model" in n or "soft_emb" in n else (
                    p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05))
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config, m.config.text_config):
        c._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def _hf_ids(req):
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [SOFT] * k
    return ex


@pytest.mark.parametrize("chunk", [8192, 12])   # 12: chunk boundaries fall inside the image blocks
def test_gemma3_vision_matches_hf(tmp_path, chunk):
    hf = _hf_model(tmp_path)
    imgs = [_image(0), _image(1, 120, 60)]
    px = torch.cat([preprocess_gemma3(im, 112) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512, chunked_prefill_size=chunk))
    m = eng.runner.model
    assert type(m).__name__ == "Gemma3ForConditionalGeneration"
    with torch.no_grad():
        want = hf.get_image_features(pixel_values=px, return_dict=True).pooler_output.reshape(-1, 256)
    got = m.encode_images(px)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()

    prompt = [2, 9, 17, BOI, 33, 41, BOI, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = _hf_ids(req)
    assert ex[:4] == [2, 9, 17, NL2] and ex[4:6] == [BOI, SOFT] and ex.count(SOFT) == 32
    eng.add_request(req)
    while not req.finished:
        eng.step()
    t = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(t, pixel_values=px, token_type_ids=(t == SOFT).long(), max_new_tokens=6,
                          do_sample=False, output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tok].item() for s, tok in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)


def test_bidirectional_block_changes_the_result(tmp_path):
    """The image block really is bidirectional: HF without token_type_ids (pure causal) differs."""
    hf = _hf_model(tmp_path)
    px = preprocess_gemma3(_image(0), 112)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=512))
    req = eng.make_mm_request([2, 9, BOI, 7], [_image(0)], SamplingParams(max_new_tokens=1, ignore_eos=True,
                                                                         logprobs=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    t = torch.tensor([_hf_ids(req)])
    with torch.no_grad():
        bi = hf(t, pixel_values=px, token_type_ids=(t == SOFT).long()).logits[0, -1].log_softmax(-1)
        causal = hf(t, pixel_values=px).logits[0, -1].log_softmax(-1)
    assert abs(req.output_logprobs[0] - bi[req.output_ids[0]].item()) < 2e-3
    assert (bi - causal).abs().max().item() > 1e-3
