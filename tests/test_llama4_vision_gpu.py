"""Llama 4 with images on gfx950: the vision tower (head dim 88 on the varlen MFMA attention
kernel, LayerNorm / GELU kernels, hipBLASLt GEMMs) in bf16 against transformers fp32, and an image
request served end to end (multi-tile prompt layout, features spliced into the prefill rows)."""
import pytest
import torch

from ome_amd.models.llama4_vision import preprocess_llama4
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_llama4_vision_cpu import IMAGE, PATCH, _hf_model, _image

pytestmark = pytest.mark.gpu


def test_llama4_vision_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    img = _image(70, 120)
    tiles, _ = preprocess_llama4(img, 56, 16)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=512))
    m = eng.runner.model
    with torch.no_grad():
        feats = hf.get_image_features(pixel_values=tiles, vision_feature_select_strategy="default",
                                      return_dict=True).last_hidden_state
        want = hf.multi_modal_projector(feats.reshape(-1, feats.shape[-1])).float()
    got = m.encode_images(tiles, None).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    prompt = [1, 9, 17, IMAGE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=8, ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex = list(req.prompt_ids)
    for s0, k in req.mm.spans:
        ex[s0:s0 + k] = [PATCH] * k
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ex]), pixel_values=tiles, max_new_tokens=8,
                          do_sample=False)[0, len(ex):].tolist()
    assert sum(int(a == b) for a, b in zip(req.output_ids, ref)) >= 6, (req.output_ids, ref)
