"""Llama 3.2 Vision (``MllamaForConditionalGeneration``) against Hugging Face transformers on CPU:
a tiny random Mllama (2 cross-attention layers, 4-tile vision tower with a global encoder and
intermediate-layer features) is served by the engine; prefill logits and greedy generations must
match HF's for a text-only prompt, a one-image prompt (image after some text, so rows before the
image take the "attend everything, no MLP" path) with a 3-tile aspect ratio (padding tile), and a
prompt with two consecutive images.  The image preprocessing (tiling, canvas choice, aspect
ratio ids) is checked against transformers' Mllama image processor."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd.multimodal.mllama import CLIP_MEAN, CLIP_STD, preprocess_image  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG = 512  # image token id (inside the text vocab of this tiny config)


def _hf(tmp_path):
    T = transformers
    tc = dict(vocab_size=520, hidden_size=128, intermediate_size=256, num_hidden_layers=5, num_attention_heads=2,
              num_key_value_heads=1, cross_attention_layers=[1, 3], rope_theta=10000.0, max_position_embeddings=512,
              rms_norm_eps=1e-5, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    vc = dict(hidden_size=64, intermediate_size=128, num_hidden_layers=3, num_global_layers=2, attention_heads=2,
              image_size=28, patch_size=14, max_num_tiles=4, intermediate_layers_indices=[0, 2],
              vision_output_dim=64 * 3, norm_eps=1e-5)
    torch.manual_seed(0)
    m = T.MllamaForConditionalGeneration(T.MllamaConfig(text_config=tc, vision_config=vc, image_token_index=IMG))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "gate" in n:
                p.fill_(0.7)
            elif ("norm" in n or "layernorm" in n) and n.endswith("weight"):
                p.normal_(1.0, 0.2)
            elif p.dim() >= 2:
                p.normal_(0.0, 0.08)
            else:
                p.normal_(0.0, 0.05)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.config.text_config._attn_implementation = "eager"
    m.config.vision_config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


def _images():
    from PIL import Image

    rng = np.random.default_rng(3)
    return [Image.fromarray(rng.integers(0, 255, (50, 140, 3), dtype=np.uint8)),   # 1x3 tiles (+1 padding)
            Image.fromarray(rng.integers(0, 255, (60, 60, 3), dtype=np.uint8))]


def _hf_inputs(ids, imgs):
    import transformers as T

    if not imgs:
        return {"input_ids": torch.tensor([ids])}
    p = T.MllamaImageProcessorPil(size={"height": 28, "width": 28}, max_image_tiles=4, image_mean=list(CLIP_MEAN),
                                  image_std=list(CLIP_STD))
    o = p(images=[imgs], return_tensors="pt")
    locs = [k for k, t in enumerate(ids) if t == IMG]
    # processor.get_cross_attention_token_mask semantics for this prompt
    from transformers.models.mllama.processing_mllama import (convert_sparse_cross_attention_mask_to_dense,
                                                              get_cross_attention_token_mask)
    sparse = [get_cross_attention_token_mask(ids, IMG)]
    dense = convert_sparse_cross_attention_mask_to_dense(sparse, o["num_tiles"], 4, len(ids))
    assert len(locs) == len(imgs)
    return {"input_ids": torch.tensor([ids]), "pixel_values": o["pixel_values"], "aspect_ratio_ids": o["aspect_ratio_ids"],
            "aspect_ratio_mask": o["aspect_ratio_mask"], "cross_attention_mask": torch.tensor(dense)}


CASES = {
    "text": ([1, 7, 9, 40, 11, 13, 99, 100, 3, 5], 0),
    "one_image": ([1, 7, 9, 40, IMG, 11, 13, 99, 100, 3, 5, 6, 77, 88], 1),
    "two_images": ([1, 7, IMG, IMG, 40, 11, 13, 99, 100, 3, 5], 2),
}


@pytest.mark.parametrize("case", list(CASES))
def test_mllama_matches_hf(tmp_path, case):
    hf = _hf(tmp_path)
    ids, n_img = CASES[case]
    imgs = _images()[:n_img] if n_img == 1 else [_images()[0], _images()[1]][:n_img]
    inputs = _hf_inputs(ids, imgs)
    with torch.no_grad():
        want = hf(**inputs).logits[0].float()
        gen = hf.generate(**inputs, max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "MllamaForConditionalGeneration"
    p = SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True) if hasattr(SamplingParams, "logprobs") \
        else SamplingParams(max_new_tokens=6, ignore_eos=True)
    req = eng.make_mm_request(ids, imgs, p) if imgs else eng.make_request(ids, p)
    eng.add_request(req)
    while not req.finished:
        eng.step()
    assert req.output_ids == gen, (req.output_ids, gen)
    got = _prefill_logits(eng, ids, req.mm)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err


def _prefill_logits(eng, ids, mm):
    """Every position's logits of one eager prefill through the model (vision-token cache included)."""
    from types import SimpleNamespace

    from ome_amd import ops
    from ome_amd.models.common import AttnMeta

    run, m = eng.runner, eng.runner.model
    slot = run.slots.alloc()
    pages = run.pages.alloc(-(-len(ids) // run.P))
    run.slots.set_pages(slot, 0, pages)
    run.slots.flush()
    T = len(ids)
    t = lambda a: torch.tensor(a, dtype=torch.int32, device=run.device)  # noqa: E731
    m.prepare_chunks([SimpleNamespace(req=SimpleNamespace(req_slot=slot, mm=mm), start=0)])
    meta = AttnMeta("prefill", t(list(range(T))), t([pages[p // run.P] * run.P + p % run.P for p in range(T)]),
                    run.slots.table.index_select(0, t([slot])), cu_q=t([0, T]), kv_lens=t([T]),
                    items=t(ops.prefill_work_items([T], [T])).view(-1, 2))
    meta.extra["ssm"] = (t([0, T]), t([slot]), t([1]))
    out = m.compute_logits(m.forward(t(ids), meta, run.kv)).float()
    m._free_slot(slot)
    run.pages.free(pages)
    run.slots.free(slot)
    return out


def test_mllama_image_preprocessing_matches_hf():
    from PIL import Image

    rng = np.random.default_rng(0)
    for w, h in [(640, 480), (300, 900), (1200, 200), (560, 560), (100, 80)]:
        img = Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8))
        p = transformers.MllamaImageProcessorPil(size={"height": 224, "width": 224}, max_image_tiles=4,
                                                 image_mean=list(CLIP_MEAN), image_std=list(CLIP_STD))
        o = p(images=[[img]], return_tensors="pt")
        pv, ar, nt = preprocess_image(img, tile=224, max_tiles=4)
        assert ar == int(o["aspect_ratio_ids"][0, 0]) and nt == o["num_tiles"][0][0]
        assert torch.equal(pv, o["pixel_values"][0, 0])


def test_cross_segments():
    from ome_amd.multimodal.mllama import CrossMMInput

    mm = CrossMMInput(torch.zeros(3, 4, 3, 28, 28), [1, 2, 3], [1, 3, 2], [4, 5, 20])
    # real tiles first: image0 [0,5) image1 [5,20) image2 [20,30); padding after -> 60 total
    assert mm.segments(5, 4) == [(0, 0, 60, 0), (4, 0, 5, 1), (5, 0, 20, 1), (20, 20, 30, 1)]
